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

WORKLOADS = {"resize_normalize": 1920 * 1080, "resize_normalize_720p": 1920 * 1080, "warp": 1280 * 720, "cvt_normalize": 1920 * 1080,
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


def _run_bench(args, env_extra=None, timeout=240):
    import json
    import os
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK",
                                                                "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, str(REPO / "bench.py")] + args, env=env, capture_output=True,
                       text=True, timeout=timeout)
    lines = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]
    return p.returncode, lines, p.stderr


@pytest.mark.parametrize("workload", ["resize_normalize", "cubic_stats"])
def test_gpus_flag_spawns_ranks(workload):
    """bench.py --gpus 2 with no torchrun environment starts two rank processes
    itself (gloo here, via --dry-run); rank 0 alone prints the line, and the
    rank count comes from the process group, not from the flag."""
    rc, lines, err = _run_bench(["--gpus", "2", "--dry-run", "--steps", "3", "--warmup", "1",
                                 "--workload", workload])
    assert rc == 0, err
    assert len(lines) == 1, lines
    out = lines[0]
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2" and out["dry_run"] is True
    assert out["steps"] == 3 and out["warmup"] == 1


def test_gpus_flag_must_match_world_size():
    """Under torchrun the flag and WORLD_SIZE must agree: a mismatch fails
    instead of reporting a 1-GPU number under an N-GPU label."""
    rc, lines, err = _run_bench(["--gpus", "4", "--dry-run", "--steps", "1", "--warmup", "0"],
                                {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert rc != 0 and not lines and "WORLD_SIZE" in err


@pytest.mark.gpu
@pytest.mark.parametrize("workload", ["cubic_stats", "warp"])
def test_bench_main_two_ranks_on_one_gpu(workload):
    """bench.py's real world > 1 path -- main() with the kernels, the barriers,
    the shard-size check, cfg5's all-reduce and the MAX-over-ranks merge --
    with two ranks on the box's one GPU: VACV_BENCH_BACKEND=gloo replaces RCCL
    (which needs a GPU per rank).  The parent spawns the ranks before anything
    touches the GPU.  One JSON line, n_gpus 2, dp2, a roofline and a finite
    step time; cfg5's statistics are global (the count covers both shards)."""
    import math
    rc, lines, err = _run_bench(["--gpus", "2", "--workload", workload, "--steps", "3", "--warmup", "1",
                                 "--no-cpu-baseline"], {"VACV_BENCH_BACKEND": "gloo"}, timeout=300)
    assert rc == 0, err[-3000:]
    assert len(lines) == 1, lines
    out = lines[0]
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2"
    assert out["config"]["backend"] == "gloo" and out["config"]["global_batch"] == 2 * out["config"]["batch_per_gpu"]
    assert math.isfinite(out["ms_per_step"]) and out["ms_per_step"] > 0
    r = out["roofline"]
    assert r["bound"] == "hbm" and r["kernel_ms"] > 0 and 0 < r["frac"] < 1.2
    assert out["value"] > 0 and out["cpu_baseline"] is None
    if workload == "cubic_stats":
        assert out["global_stats_check"]["ok"], out["global_stats_check"]


def test_gpus_8_dry_run_single_line():
    """The driver's 8-GPU scaling run, rehearsed on the CPU: `--gpus 8` spawns
    eight ranks (gloo, --dry-run), cfg5's step all-reduces its sums across all
    eight, and rank 0 alone prints one dp8 line."""
    rc, lines, err = _run_bench(["--gpus", "8", "--dry-run", "--steps", "2", "--warmup", "1",
                                 "--workload", "cubic_stats"], timeout=400)
    assert rc == 0, err[-3000:]
    assert len(lines) == 1, lines
    out = lines[0]
    assert out["n_gpus"] == 8 and out["config"]["parallelism"] == "dp8" and out["dry_run"] is True


def test_only_rank0_builds(monkeypatch, tmp_path):
    """A rank other than 0 never runs the build: with the library missing it
    exits non-zero instead of racing rank 0's make into the same lib/."""
    import bench
    sys.path.insert(0, str(REPO / "arm-neon-opencv_amd"))
    import vacv_amd
    calls = []
    monkeypatch.setattr(vacv_amd._lib, "HIP_LIB", tmp_path / "libvacv_hip.so")
    monkeypatch.setattr(vacv_amd._lib, "build", lambda: calls.append("build"))
    with pytest.raises(SystemExit) as e:
        bench.ensure_built(rank=1, world=1)
    assert e.value.code == 2 and calls == []
    with pytest.raises(SystemExit):
        bench.ensure_built(rank=0, world=1)  # rank 0 builds (stubbed: still missing -> exit)
    assert calls == ["build"]
