"""Regenerates theta_config.json from the reference's tuned hyper-parameters
(/root/reference/examples/config/config.json -- a data file: 84 vectors '<ID>_<MAX|MIN><N>' ->
[σ_f, ℓ_1..ℓ_d]).  Run in the build container only; the GPU box reads the vendored JSON."""
import json
import pathlib
import sys

src = pathlib.Path(sys.argv[1] if len(sys.argv) > 1 else "/root/reference/examples/config/config.json")
dst = pathlib.Path(__file__).resolve().parent / "theta_config.json"
json.dump(json.loads(src.read_text()), open(dst, "w"), indent=0, sort_keys=True)
