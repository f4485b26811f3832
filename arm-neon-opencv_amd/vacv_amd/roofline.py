"""Algorithmic byte counts for the roofline.

B_alg(image) = bytes of every source row that carries a non-zero vertical
weight for some output row (each counted once) + bytes written.  For the
elementwise operators it is simply input + output bytes.  The row weights are
recomputed here with the reference's arithmetic (numpy float32/float64 in the
same order as vacv_semantics.hpp), so the count matches what the resize
kernel actually stages.
"""
from __future__ import annotations

import numpy as np

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def _sat_short_away(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.float32)
    r = x + np.where(x >= 0, np.float32(0.5), np.float32(-0.5)).astype(np.float32)
    return np.clip(np.trunc(r), -32768, 32767).astype(np.int32)


def linear_row_weights(n_in: int, n_out: int, mode: int = 0):
    d = np.arange(n_out, dtype=np.float64)
    if mode == 0:
        s = np.float64(np.float32(n_in) / np.float32(n_out))
    else:
        s = np.float64(n_in) / np.float64(n_out)
    f = ((d + 0.5) * s - 0.5).astype(np.float32)
    i = np.floor(f).astype(np.int64)
    f = (f - i.astype(np.float32)).astype(np.float32)
    lo = i < 0
    i[lo], f[lo] = 0, np.float32(0)
    hi = i >= n_in - 1
    i[hi], f[hi] = n_in - 2, np.float32(1)
    a = ((np.float32(1) - f) * np.float32(2048)).astype(np.float32)
    b = (f * np.float32(2048)).astype(np.float32)
    if mode == 2:
        w0, w1 = np.rint(a).astype(np.int32), np.rint(b).astype(np.int32)
    else:
        w0, w1 = _sat_short_away(a), _sat_short_away(b)
    return i, w0, w1


def weighted_rows_linear(n_in: int, n_out: int, mode: int = 0) -> int:
    i, w0, w1 = linear_row_weights(n_in, n_out, mode)
    rows = set(i[w0 != 0].tolist()) | set((i[w1 != 0] + 1).tolist())
    return len(rows)


def weighted_rows_cubic(n_in: int, n_out: int) -> int:
    A = np.float32(-0.75)
    rows = set()
    s = np.float64(n_in) / np.float64(n_out)
    for d in range(n_out):
        f = np.float32((d + 0.5) * s - 0.5)
        i = int(np.floor(f))
        f = np.float32(f - np.float32(i))
        t0, t1, t2 = np.float32(f + 1), f, np.float32(1 - f)
        c0 = A * t0 * t0 * t0 - np.float32(5) * A * t0 * t0 + np.float32(8) * A * t0 - np.float32(4) * A
        c1 = (A + 2) * t1 * t1 * t1 - (A + 3) * t1 * t1 + np.float32(1)
        c2 = (A + 2) * t2 * t2 * t2 - (A + 3) * t2 * t2 + np.float32(1)
        c3 = np.float32(1) - c0 - c1 - c2
        c = [c0, c1, c2, c3]
        if i <= -1:
            i, c = 1, [1 - c[3], c[3], 0, 0]
        if i == 0:
            i, c = 1, [c[0] + c[1], c[2], c[3], 0]
        if i == n_in - 2:
            i, c = n_in - 3, [0, c[0], c[1], c[2] + c[3]]
        if i >= n_in - 1:
            i, c = n_in - 3, [0, 0, c[0], 1 - c[0]]
        for j in range(4):
            if c[j] != 0:
                rows.add(i - 1 + j)
    return len(rows)


def resize_bytes(w_in: int, h_in: int, c: int, w_out: int, h_out: int, in_esize: int = 1, out_esize: int = 1,
                 cubic: bool = False, mode: int = 0) -> int:
    rows = weighted_rows_cubic(h_in, h_out) if cubic else weighted_rows_linear(h_in, h_out, mode)
    return rows * w_in * c * in_esize + w_out * h_out * c * out_esize


def yuv_resize_bytes(w_in: int, h_in: int, w_out: int, h_out: int, out_esize: int = 4, mode: int = 0) -> int:
    """B_alg of the fused YUV420sp -> BGR -> resize kernel: every weighted Y row,
    every chroma row (one per Y row pair) that a weighted Y row needs, and the
    3-channel output."""
    i, w0, w1 = linear_row_weights(h_in, h_out, mode)
    rows = set(i[w0 != 0].tolist()) | set((i[w1 != 0] + 1).tolist())
    chroma = {r >> 1 for r in rows}
    return (len(rows) + len(chroma)) * w_in + w_out * h_out * 3 * out_esize
