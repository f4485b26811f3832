"""bench.py's host side on the CPU: every workload's CPU baseline case (the
reference's own loops from oracle/_ref, or the C restatement) runs and sizes
its sample as the GPU line reports it.  No GPU needed."""
from __future__ import annotations

import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent
if str(REPO) not in sys.path:
    sys.path.insert(0, str(REPO))

WORKLOADS = {"resize_normalize": 1920 * 1080, "warp": 1280 * 720, "cvt_normalize": 1920 * 1080,
             "cubic_stats": 2560 * 1440, "yuv_resize": 1920 * 1080}


@pytest.mark.parametrize("workload", sorted(WORKLOADS))
def test_cpu_case_runs(workload):
    import bench
    one, imgs, px, kind, what = bench.cpu_case(workload)
    assert px == WORKLOADS[workload]
    assert kind in ("reference", "port") and what
    out = one(imgs[0])
    assert out is not None


def test_workload_choices_match_parser(monkeypatch):
    import bench
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    a = bench.parse()
    assert a.workload == "resize_normalize" and a.gpus == 1 and a.batch == 0
    for w in WORKLOADS:
        monkeypatch.setattr(sys, "argv", ["bench.py", "--workload", w])
        assert bench.parse().workload == w
