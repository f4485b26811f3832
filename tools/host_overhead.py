#!/usr/bin/env python3
"""Host time per call of the bench workloads' ops (no synchronisation inside
the loop): if it exceeds the kernel time, back-to-back launches leave the GPU
idle between kernels."""
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "arm-neon-opencv_amd")]
import torch  # noqa: E402
import bench  # noqa: E402
from vacv_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
for wl in ("resize_normalize", "warp", "cvt_normalize", "cubic_stats", "yuv_resize"):
    w = bench.make_workload(wl, 0, dev, 0, 1, ops)
    f = w["main"]
    for _ in range(5):
        f()
    torch.cuda.synchronize(dev)
    n = 50
    t0 = time.perf_counter()
    for _ in range(n):
        f()
    t1 = time.perf_counter()
    torch.cuda.synchronize(dev)
    t2 = time.perf_counter()
    print(f"{wl:18s} host {1e6 * (t1 - t0) / n:8.1f} us/call   wall {1e6 * (t2 - t0) / n:8.1f} us/call", flush=True)
    del w, f
    torch.cuda.empty_cache()
