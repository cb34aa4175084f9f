"""Raw fp64 CState dataset files.

The reference stores its datasets with Julia `Serialization` (`.jls`, examples/utils/datasets.jl:
90-108), which nothing outside Julia can read.  This format carries one trial's training set in the
exact memory layout the GP path consumes, so a Julia dump is a plain `write` and the reader is a
memory map:

    offset  size        field
    0       8           magic b"GPRXCST1"
    8       4 (u32 LE)  d   state dimension (13 per body)
    12      4 (u32 LE)  G   number of output rows that follow X (0: inputs only)
    16      8 (u64 LE)  N   number of states
    24      8           reserved (0)
    32      8 d N       X: float64 LE, column t = one CState (d x N column-major, the layout of
                        reduce(hcat, CState.(df.sold)), CPnoise.jl:26)
    32+8dN  8 G N       Y: float64 LE, row g = output g over the N states (the N x G column-major
                        matrix reduce(hcat, ytrain), CPnoise.jl:28-29)

Julia writer (a maintainer's one-off conversion of the .jls sets):
    open(path, "w") do io
        write(io, b"GPRXCST1", UInt32(size(X, 1)), UInt32(length(ytrain)), UInt64(size(X, 2)), UInt64(0))
        write(io, X); foreach(y -> write(io, y), ytrain)
    end
"""
from __future__ import annotations

import os
import struct

import numpy as np

MAGIC = b"GPRXCST1"
HEADER = struct.Struct("<8sIIQQ")  # 32 bytes


def write_cstates(path, X, Y=None) -> None:
    """X: (d, N) states (column = one CState); Y: (G, N) targets or None."""
    X = np.ascontiguousarray(np.asarray(X, dtype="<f8"))
    if X.ndim != 2:
        raise ValueError("X must be (d, N)")
    d, N = X.shape
    Yc = None
    G = 0
    if Y is not None:
        Yc = np.ascontiguousarray(np.asarray(Y, dtype="<f8"))
        if Yc.ndim == 1:
            Yc = Yc[None, :]
        if Yc.shape[1] != N:
            raise ValueError("Y must be (G, N) with the same N as X")
        G = Yc.shape[0]
    with open(path, "wb") as f:
        f.write(HEADER.pack(MAGIC, d, G, N, 0))
        f.write(np.ascontiguousarray(X.T).tobytes())  # column t contiguous
        if Yc is not None:
            f.write(Yc.tobytes())


def read_cstates(path, mmap: bool = True) -> dict:
    """Returns dict(X=(d, N), Y=(G, N) or None, d, N, G).  With mmap the arrays are read-only views
    of the file (no copy until the library stages them to HBM)."""
    size = os.path.getsize(path)
    if size < HEADER.size:
        raise ValueError(f"{path}: too short for a GPRXCST1 header")
    with open(path, "rb") as f:
        magic, d, G, N, _ = HEADER.unpack(f.read(HEADER.size))
    if magic != MAGIC:
        raise ValueError(f"{path}: not a GPRXCST1 file")
    need = HEADER.size + 8 * (d * N + G * N)
    if d < 1 or size != need:
        raise ValueError(f"{path}: size {size} != {need} for d={d}, N={N}, G={G}")
    if mmap:
        raw = np.memmap(path, dtype="<f8", mode="r", offset=HEADER.size, shape=(d * N + G * N,))
    else:
        with open(path, "rb") as f:
            f.seek(HEADER.size)
            raw = np.frombuffer(f.read(), dtype="<f8")
    X = raw[: d * N].reshape(N, d).T  # (d, N) view of the column-major dump
    Y = raw[d * N:].reshape(G, N) if G else None
    return dict(X=X, Y=Y, d=d, N=N, G=G)
