#!/usr/bin/env python3
"""The hyperparameter.jl random-restart search on MI355X: 8 experiments x N in {2..2048} x trials,
trial-sharded over one rank per GPU.  See gpr.jl_amd/gprx/search.py.

    python search.py [--trials 100 --max-evals 30 ...]                      # one GPU
    python search.py --gpus 8                                               # 8 GPUs: starts its ranks
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \\
        --master-addr 127.0.0.1 --master-port 29500 search.py              # 8 GPUs (RCCL)
"""
import pathlib
import sys

REPO = pathlib.Path(__file__).resolve().parent
sys.path[:0] = [str(REPO), str(REPO / "gpr.jl_amd")]

from gprx.search import main  # noqa: E402

if __name__ == "__main__":
    main()
