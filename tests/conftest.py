import pathlib
import sys

import pytest

REPO = pathlib.Path(__file__).resolve().parents[1]
for p in (REPO, REPO / "gpr.jl_amd"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the gfx950 library)")


@pytest.fixture(scope="session")
def golden_dir():
    return REPO / "tests" / "golden"
