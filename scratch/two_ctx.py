"""Concurrency probe: the bench's P2 workload as one 240-slot batch on one context, against two
120-slot batches on two contexts (two HIP streams) evaluated by two host threads at once."""
import sys, threading, time
import numpy as np
sys.path.insert(0, ".")
import bench
import gprx
from gprx import shard

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
G = bench.G


def setup(trials, ctx):
    trs, X, Y, T, XT = bench.make_workload(trials, 0, 1)
    rb = shard.RankBatch(trs, ctx=ctx)
    return rb, T.reshape(rb.n, G, -1)


c1 = gprx.Context(0)
rb, TH = setup(40, c1)
for _ in range(2):
    rb.evaluate(TH)
t0 = time.perf_counter()
for _ in range(steps):
    rb.evaluate(TH)
t1 = time.perf_counter() - t0
print(f"one ctx 240 slots: {1e3 * t1 / steps:.2f} ms/step, {240 * steps / t1:.0f} fits/s", flush=True)
rb.close()

c2 = gprx.Context(0)
ra, TA = setup(20, c1)
rc, TC = setup(20, c2)
for _ in range(2):
    ra.evaluate(TA)
    rc.evaluate(TC)


def run(r, T, n, out, i):
    s = time.perf_counter()
    for _ in range(n):
        r.evaluate(T)
    out[i] = time.perf_counter() - s


out = [0.0, 0.0]
th = [threading.Thread(target=run, args=(ra, TA, steps, out, 0)), threading.Thread(target=run, args=(rc, TC, steps, out, 1))]
t0 = time.perf_counter()
for t in th:
    t.start()
for t in th:
    t.join()
t2 = time.perf_counter() - t0
print(f"two ctx x 120 slots: {1e3 * t2 / steps:.2f} ms per 240 fits, {240 * steps / t2:.0f} fits/s (threads {out})", flush=True)
t0 = time.perf_counter()
for _ in range(steps):
    ra.evaluate(TA)
t3 = time.perf_counter() - t0
print(f"one ctx 120 slots alone: {1e3 * t3 / steps:.2f} ms/step", flush=True)
