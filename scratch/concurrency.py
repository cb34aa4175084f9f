"""Are evaluations reproducible while another process uses the same GPU?

  python scratch/concurrency.py probe [--reps R] [--trials T]   alternating theta_a / theta_b
      evaluations, every result compared bit for bit with the first; statuses and NaN counts kept
  python scratch/concurrency.py load-torch --seconds S           fp64 torch matmuls on the card
  python scratch/concurrency.py load-gprx --seconds S            this library's own evaluations

Run two at once on the box (probe & load-*), then the probe alone.
"""
from __future__ import annotations

import argparse
import json
import pathlib
import sys
import time

import numpy as np

REPO = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "gpr.jl_amd"))


def setup(trials):
    import bench
    import gprx
    from gprx import shard

    ctx = gprx.Context(0)
    trs, X, Y, T, XT = bench.make_workload(trials, 0, 1)
    rb = shard.RankBatch(trs, ctx=ctx)
    return ctx, rb.batch, T


def probe(args):
    ctx, batch, T = setup(args.trials)
    rng = np.random.default_rng(7)
    th = {"a": T, "b": T + 0.02 * rng.standard_normal(T.shape)}
    ref = {k: batch.run(v, grad=True, predict=True) for k, v in th.items()}
    for k in ref:
        assert np.all(ref[k]["status"] == 0), (k, ref[k]["status"])
    bad = []
    t0 = time.time()
    n = 0
    while n < 2 * args.reps and time.time() - t0 < args.seconds:
        k = "ab"[n % 2]
        r = batch.run(th[k], grad=True, predict=True)
        n += 1
        rec = {}
        st = np.nonzero(r["status"] != 0)[0]
        if st.size:
            rec["status"] = {int(s): [int(r["status"][s]), int(r["info"][s])] for s in st[:8]}
            rec["n_status"] = int(st.size)
        for q in ("mll", "grad", "mu", "var"):
            a = np.ascontiguousarray(ref[k][q]).view(np.uint64).reshape(T.shape[0], -1)
            b = np.ascontiguousarray(r[q]).view(np.uint64).reshape(T.shape[0], -1)
            sl = np.nonzero(np.any(a != b, axis=1))[0]
            if sl.size:
                fa = ref[k][q].reshape(T.shape[0], -1)[sl]
                fb = r[q].reshape(T.shape[0], -1)[sl]
                fin = np.isfinite(fb)
                rec[q] = dict(n=int(sl.size), slots=sl[:10].tolist(), nan=int(np.sum(~fin)),
                              max_abs_finite=float(np.max(np.abs(fa - fb)[fin])) if fin.any() else None)
        if rec:
            rec["eval"] = n
            bad.append(rec)
    out = dict(evaluations=n, mismatches=len(bad), first=bad[:6], seconds=round(time.time() - t0, 1))
    print(json.dumps(out))


def dump_probe(args):
    """probe with the debug-dump library (scratch/var/libgprx_dump.so): the diagonal wave's tile
    image at the start of every diagonal tile and its block-3 lane state are dumped per (slot,
    tile); an evaluation that differs from the first is compared dump against dump."""
    import ctypes as C

    import torch

    from gprx import _lib as L

    ctx, batch, T = setup(args.trials)
    B = T.shape[0]
    W = 4096 + 64 * 17
    buf = torch.zeros(B * 32 * W, dtype=torch.float64, device="cuda")
    L.lib.gprx_debug_set_dump.argtypes = [C.c_void_p]
    assert L.lib.gprx_debug_set_dump(C.c_void_p(buf.data_ptr())) == 0
    ref_r = batch.run(T, grad=True, predict=False)
    torch.cuda.synchronize()
    ref = buf.clone().view(B, 32, W)
    assert np.all(ref_r["status"] == 0)
    out = []
    t0 = time.time()
    n = 0
    while time.time() - t0 < args.seconds:
        r = batch.run(T, grad=True, predict=False)
        n += 1
        torch.cuda.synchronize()
        cur = buf.view(B, 32, W)
        neq = (cur != ref).any(dim=2)  # (B, 32)
        bad = np.nonzero(r["status"] != 0)[0]
        if neq.any().item() or bad.size:
            rec = dict(eval=n, status={int(s): [int(r["status"][s]), int(r["info"][s])] for s in bad[:4]},
                       dump_diff_slots_tiles=torch.nonzero(neq)[:8].tolist())
            for s, jt in torch.nonzero(neq)[:3].tolist():
                a = ref[s, jt].cpu().numpy()
                b = cur[s, jt].cpu().numpy()
                img = np.nonzero(a[:4096] != b[:4096])[0]
                lane = np.nonzero(a[4096:] != b[4096:])[0]
                rec[f"s{s}_t{jt}"] = dict(
                    img_diff=[[int(i % 64), int(i // 64), float(a[i]), float(b[i])] for i in img[:8]],  # row, col
                    n_img=int(img.size),
                    lane_diff=[[int(i // 17), int(i % 17), float(a[4096 + i]), float(b[4096 + i])] for i in lane[:8]],
                    n_lane=int(lane.size))
            out.append(rec)
            if len(out) >= 6:
                break
    L.lib.gprx_debug_set_dump(None)
    print(json.dumps(dict(evaluations=n, events=out)))


def load_torch(args):
    import torch

    a = torch.randn(4096, 4096, dtype=torch.float64, device="cuda")
    t0 = time.time()
    k = 0
    while time.time() - t0 < args.seconds:
        a = torch.tanh(a @ a * 1e-3)
        k += 1
        if k % 16 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    print(json.dumps(dict(load="torch", iterations=k)))


def load_gprx(args):
    ctx, batch, T = setup(args.trials)
    t0 = time.time()
    k = 0
    while time.time() - t0 < args.seconds:
        batch.run(T, grad=True, predict=True)
        k += 1
    print(json.dumps(dict(load="gprx", evaluations=k)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["probe", "dump", "load-torch", "load-gprx"])
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--seconds", type=float, default=20.0)
    ap.add_argument("--trials", type=int, default=40)
    args = ap.parse_args()
    {"probe": probe, "dump": dump_probe, "load-torch": load_torch, "load-gprx": load_gprx}[args.mode](args)


if __name__ == "__main__":
    main()
