#!/usr/bin/env python3
"""vacv MI355X benchmark -- the driver's contract (one JSON line on rank 0).

Workload (BASELINE.json north_star target, configs[1] geometry): fused
resize_normalize, 1920x1080x3 u8 NHWC -> 640x360x3 fp32, INTER_LINEAR with
the reference's arithmetic, mean (103.94,116.78,123.68) / std
(57.375,57.12,58.395), a batch of --batch images per GPU resident in HBM.
One step = one vacv_resize_normalize call over the whole per-GPU batch (one
kernel launch: resize_cols_kernel, k_resize_direct.hip).  Metric = input-frame Mpixels/s over all GPUs ("at 1080p").

Other BASELINE configs (--workload; the default is the headline above):
  resize_normalize_720p  the headline op at 1080p -> 1280x720 fp32: every output
                row weights two source rows (SURVEY 8(d)'s "honest roofline
                case"; resize_strip_kernel), 256 per GPU
  warp          cfg4: warp_affine INTER_LINEAR 1280x720x3 u8, scale 0.9, rot 15,
                aux (640,360,640,360), 128 frames per GPU (1024 over 8 GPUs)
  cvt_normalize cfg3: NV21 1920x1620 -> BGR 1920x1080x3 fp32 normalised, 256 per GPU
  cubic_stats   cfg5: INTER_CUBIC 2560x1440x3 u8 -> 224x224x3 fp32 (128 per GPU),
                then the GLOBAL per-channel mean/stddev of the whole sharded
                batch: exact sums per rank + one RCCL all-reduce per step
  yuv_resize    SURVEY 8(f)2: NV21 1080p -> 640x360 planar (NCHW) fp32 normalised,
                decode + resize + normalize + layout in one kernel, 256 per GPU
The roofline covers the step's dominant kernel (HIP events around it alone).

Multi-GPU: one process per GPU; images are independent, so each rank owns its
own batch (weak scaling) and there is no data-path collective (cfg5's
statistics are the one RCCL all-reduce).  Either torchrun starts the ranks
(WORLD_SIZE in the environment must then equal --gpus), or `bench.py --gpus N`
with no WORLD_SIZE spawns the N rank processes itself before anything touches
the GPU (127.0.0.1 rendezvous) and exits with the first failing rank's status.
--dry-run exercises that launcher and the rank protocol on CPU (gloo, a CPU
stand-in step, no measurement): the multi-rank CPU test uses it.
Timing: barrier + synchronize around exactly --steps steps, max over ranks.

Also reported: the roofline of the kernel (algorithmic bytes per launch /
average launch time from HIP events on the launch stream, vs 8 TB/s) and the
reference's own CPU path (oracle/_ref, compiled from the reference sources;
the C restatement when that is absent) timed on a bounded sample on rank 0,
on 1 thread and batch-parallel on up to 16 threads.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO / "arm-neon-opencv_amd"))

W_IN, H_IN, C = 1920, 1080, 3
W_OUT, H_OUT = 640, 360
MEAN = [103.94, 116.78, 123.68]
STD = [57.375, 57.12, 58.395]
PROFILES = REPO / "profiles"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    # 50 warmup launches (~12 ms): measured 0.2225 ms/launch after 50 or 200
    # warmups vs 0.2285 after 10 (the GPU's clocks settle under the load)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--workload", default="resize_normalize",
                    choices=["resize_normalize", "resize_normalize_720p", "warp", "cvt_normalize", "cubic_stats",
                             "yuv_resize"])
    ap.add_argument("--batch", type=int, default=0, help="images per GPU (0: the workload's default)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget of the CPU baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--graph", action="store_true",
                    help="replay the step from a captured HIP graph (measured no faster than eager launches)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher / rank-protocol check on CPU: gloo, a CPU stand-in step, no GPU, no measurement")
    return ap.parse_args()


def spawn_ranks(n: int) -> int:
    """`bench.py --gpus N` outside torchrun: start N rank processes (RANK /
    LOCAL_RANK / WORLD_SIZE / MASTER_* as torchrun sets them), wait for all,
    return the first non-zero exit status.  The parent never touches the GPU
    (no torch import), so each child owns its device from a clean process."""
    import signal
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(Path(__file__).resolve())] + sys.argv[1:], env=env))
    rc = 0
    pending = list(procs)
    while pending:
        for p in list(pending):
            code = p.poll()
            if code is None:
                continue
            pending.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                for q in pending:  # one rank failed: the others would wait at a barrier forever
                    q.send_signal(signal.SIGTERM)
        time.sleep(0.05)
    return rc


def ensure_built(rank: int, world: int):
    """Only rank 0 may build libvacv_hip.so (N ranks running make into one
    lib/ at once would race); the other ranks wait at a barrier until it is
    done, then load it or exit non-zero.  The driver's runs find it prebuilt."""
    import vacv_amd
    lib = vacv_amd._lib.HIP_LIB
    if rank == 0 and not lib.exists():
        vacv_amd._lib.build()
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    if not lib.exists():
        print(f"bench: rank {rank}: {lib} is missing after rank 0's build step", file=sys.stderr)
        sys.exit(2)
    vacv_amd._lib.load()


def cpu_case(workload: str):
    """(one(img), inputs, input pixels per image, kind, what) of the reference's
    own CPU path for a workload: oracle/_ref (the reference's loops compiled
    from its sources) where present, else the C restatement (oracle/)."""
    import numpy as np
    sys.path.insert(0, str(REPO / "oracle"))
    from oracle import Oracle, Reference, synthetic_image
    mean = np.array(MEAN, np.float32)
    std = np.array(STD, np.float32)
    O = Oracle()
    R = Reference() if Reference.available() else None
    kind = "reference" if R else "port"
    if workload == "warp":
        imgs = [synthetic_image(1000 + k, 720, 1280, 3) for k in range(4)]
        m = O.rotation_matrix(0.9, 15.0, (640, 360, 640, 360))
        inv = O.invert_affine(m)
        if R:
            def one(img):  # warp_affine.cpp:121-133 inverse, warp_affine_naive.cpp:9-62
                return R.warp_affine_inv(img, inv, 1280, 720)
        else:
            def one(img):
                return O.warp_affine(img, m, 1280, 720)
        return one, imgs, 1280 * 720, kind, "warp_affine_naive 1280x720 rot15 scale0.9"
    if workload in ("cvt_normalize", "yuv_resize"):
        imgs = [O.bgr2nv21(synthetic_image(1000 + k, 1080, 1920, 3)) for k in range(4)]
        to_bgr = R.nv21_to_bgr if R else O.yuv420sp_to_bgr
        rs = R.resize_linear if R else O.resize_linear
        norm = R.normalize if R else O.normalize
        if workload == "cvt_normalize":
            def one(yuv):  # cvt_color.cpp:39-135, tensor.cpp:477-481, normalize_naive.cpp:74-90
                return norm(to_bgr(yuv).astype(np.float32), mean, std)
            return one, imgs, 1920 * 1080, kind, "nv_to_bgr_naive 1080p + u8->fp32 + normalize"

        def one(yuv):  # + resize_naive.cpp:10-68 and the HWC->CHW of tensor.cpp:160-182
            return O.hwc_to_chw(norm(rs(to_bgr(yuv), 640, 360).astype(np.float32), mean, std))
        return one, imgs, 1920 * 1080, kind, "nv_to_bgr_naive 1080p + resize_naive 640x360 + normalize + hwc_to_chw"
    if workload == "cubic_stats":
        imgs = [synthetic_image(1000 + k, 1440, 2560, 3) for k in range(2)]
        cubic = R.resize_cubic if R else O.resize_cubic
        stats = R.mean_stddev if R else O.mean_stddev_ref

        def one(img):  # tensor.cpp:477-481, resize_naive.cpp:130-569, normalize_naive.cpp:7-48
            return stats(cubic(img.astype(np.float32), 224, 224))
        return one, imgs, 2560 * 1440, kind, "u8->fp32 2560x1440 + cubic 224x224 + mean_stddev"
    imgs = [synthetic_image(1000 + k, H_IN, W_IN, C) for k in range(4)]
    wo, ho = (1280, 720) if workload == "resize_normalize_720p" else (W_OUT, H_OUT)
    if R:
        def one(img):
            r = R.resize_linear(img, wo, ho)           # resize_naive.cpp:10-68
            return R.normalize(r.astype(np.float32), mean, std)  # tensor.cpp:477-481 + normalize_naive.cpp:74-90
    else:
        def one(img):
            return O.normalize(O.u8_to_f32(O.resize_linear(img, wo, ho)), mean, std)
    return one, imgs, W_IN * H_IN, kind, f"1920x1080x3 u8 frames, resize_naive {wo}x{ho} + u8->fp32 + normalize"


def host_cpus():
    """(threads to use, description): the CPUs this process may actually run
    on -- its affinity mask, capped by a cgroup-v2 `cpu.max` quota when one is
    set (the GPU box's container shows the whole machine in nproc but grants a
    CPU share) -- and the CPU model from /proc/cpuinfo."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        q, period = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        if q != "max":
            quota = int(q) / int(period)
    except (OSError, ValueError):
        pass
    threads = max(1, min(aff, int(quota + 0.999)) if quota else aff)
    model = "unknown"
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    desc = f"{model}; affinity {aff} CPUs" + (f", cgroup cpu.max quota {quota:g} CPUs" if quota else ", no cgroup quota")
    return threads, model, desc


def cpu_baseline(budget_s: float, workload: str = "resize_normalize"):
    """The reference's own CPU path of the workload on the host, on a bounded
    sample: first on 1 thread, then batch-parallel with one image per thread
    on every CPU the process may use (host_cpus: affinity capped by the cgroup
    quota; ctypes releases the GIL, so the reference's loops run concurrently).
    SURVEY.md 8(d) asks for both; the multi-core figure is the reported
    baseline.  oracle/_ref is the reference's sources built at -O3."""
    from concurrent.futures import ThreadPoolExecutor
    one, imgs, px, kind, what = cpu_case(workload)

    def run(threads, seconds):
        def worker(t):
            n, t0 = 0, time.perf_counter()
            while True:
                one(imgs[(t + n) % len(imgs)])
                n += 1
                if time.perf_counter() - t0 >= seconds and n >= 2:
                    return n
        one(imgs[0])  # warm
        t0 = time.perf_counter()
        with ThreadPoolExecutor(threads) as ex:
            n = sum(ex.map(worker, range(threads)))
        el = time.perf_counter() - t0
        return n, el

    n1, el1 = run(1, budget_s * 0.4)
    threads, model, desc = host_cpus()
    nt, elt = run(threads, budget_s * 0.6)
    v1 = n1 * px / el1 / 1e6
    vt = nt * px / elt / 1e6
    return {"value": round(vt, 3), "unit": "Mpixels/s", "cores": threads, "kind": kind,
            "value_1_core": round(v1, 3), "cpu_model": model,
            "sample": f"synthetic {what}: {nt} frames on {threads} threads (one frame per thread) in {elt:.1f} s; "
                      f"{n1} frames on 1 thread in {el1:.1f} s; host: {desc}"}


def pmc_traffic(workload: str = "resize_normalize"):
    """Corrected HBM bytes per launch from the committed rocprofv3 PMC passes
    (profiles/pmc_<workload>.json, written by tools/pmc_summary.py)."""
    p = PROFILES / f"pmc_{workload}.json"
    if not p.exists():
        return None
    try:
        return json.loads(p.read_text()).get("hbm_bytes_per_launch")
    except Exception:
        return None


def global_sums(sums):
    """All-reduce (SUM) of a rank's (groups, c, 2) fp64 channel sums over the
    default process group: in place on the device under RCCL ("nccl"); gloo
    reduces host tensors, so a device tensor goes through a host copy there."""
    import torch.distributed as dist
    if dist.get_backend() == "gloo" and sums.is_cuda:
        host = sums.cpu()
        dist.all_reduce(host, op=dist.ReduceOp.SUM)
        sums.copy_(host)
    else:
        dist.all_reduce(sums, op=dist.ReduceOp.SUM)
    return sums


def make_workload(name: str, batch: int, dev, rank: int, world: int, ops) -> dict:
    """Inputs resident in HBM, the step's launches and the roofline terms of
    one BASELINE config.  b_alg = algorithmic bytes of the dominant kernel per
    launch; px = input-frame pixels per image."""
    import torch
    from vacv_amd.roofline import resize_bytes, yuv_resize_bytes
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)

    def u8(*shape):
        return torch.randint(0, 256, shape, dtype=torch.uint8, device=dev, generator=g)

    if name == "warp":
        B = batch or 128
        src = u8(B, 720, 1280, 3)
        dst = torch.empty_like(src)
        m = ops.rotation_matrix(0.9, 15.0, (640, 360, 640, 360))
        return {"batch": B, "px": 1280 * 720, "b_alg": B * 2 * 1280 * 720 * 3, "kernel": "warp_exp_kernel",
                "frame": "1280x720x3", "output": "1280x720x3 u8",
                "desc": "warp_affine INTER_LINEAR BORDER_CONSTANT 1280x720x3 u8, scale 0.9 rot 15 aux (640,360,640,360)",
                "main": lambda stream=None: ops.warp_affine(src, m, 1280, 720, out=dst, stream=stream)}
    if name == "cvt_normalize":
        B = batch or 256
        yuv = u8(B, 1620, 1920)
        dst = torch.empty((B, 1080, 1920, 3), dtype=torch.float32, device=dev)
        return {"batch": B, "px": 1920 * 1080, "b_alg": B * (1920 * 1620 + 1920 * 1080 * 12), "kernel": "color_kernel",
                "frame": "NV21 1920x1620", "output": "1920x1080x3 fp32",
                "desc": "cvt_color YUV2BGR_NV21 1080p + normalize(mean/std) -> 1920x1080x3 fp32, one pass",
                "main": lambda stream=None: ops.cvt_color_normalize(yuv, mean=MEAN, std=STD, out=dst, stream=stream)}
    if name == "yuv_resize":
        B = batch or 256
        yuv = u8(B, 1620, 1920)
        dst = torch.empty((B, 3, 360, 640), dtype=torch.float32, device=dev)
        return {"batch": B, "px": 1920 * 1080, "b_alg": B * yuv_resize_bytes(1920, 1080, 640, 360),
                "kernel": "yuv_cols_kernel", "frame": "NV21 1920x1620", "output": "3x360x640 fp32 (NCHW)",
                "desc": "cvt_color NV21 -> resize INTER_LINEAR 640x360 -> normalize -> NCHW, one kernel",
                "main": lambda stream=None: ops.cvt_color_resize_normalize(yuv, 640, 360, MEAN, STD, out=dst,
                                                                           stream=stream)}
    if name == "cubic_stats":
        from vacv_amd import INTER_CUBIC
        B = batch or 128
        src = u8(B, 1440, 2560, 3)
        dst = torch.empty((B, 224, 224, 3), dtype=torch.float32, device=dev)
        stats = {}
        count = float(B) * world * 224 * 224

        if world == 1:
            def main(stream=None):
                # one GPU: the resize with the batch's (Sum x, Sum x^2) fused
                # into the cubic kernel and one fixed-order reduction launch
                # that also derives mean / stddev (vacv_resize_mean_stddev)
                _, stats["sums"], stats["mean"], stats["std"] = ops.resize_mean_stddev(
                    src, 224, 224, INTER_CUBIC, per_image=False, out=dst, stream=stream)
            extra = None
        else:
            def main(stream=None):
                # the per-rank sums (vacv_resize_channel_sums) ...
                stats["sums"] = ops.resize_channel_sums(src, 224, 224, INTER_CUBIC, per_image=False, out=dst,
                                                        stream=stream)[1]

            def extra(stream=None):
                # ... then the global mean/stddev of the whole sharded batch:
                # ONE all-reduce of the (c, 2) fp64 sums, vacv_stats_from_sums --
                # identical on every rank
                stats["sums"] = global_sums(stats["sums"])
                stats["mean"], stats["std"] = ops.stats_from_sums(stats["sums"], count, stream=stream)
        return {"batch": B, "px": 2560 * 1440, "b_alg": B * resize_bytes(2560, 1440, 3, 224, 224, 1, 4, cubic=True),
                "kernel": "cubic_cols_kernel", "frame": "2560x1440x3", "output": "224x224x3 fp32 + global mean/std",
                "desc": "resize INTER_CUBIC 2560x1440x3 u8 -> 224x224x3 fp32 + global mean_stddev (RCCL all-reduce)",
                "main": main, "extra": extra, "stats": stats, "inputs": src}
    if name == "resize_normalize_720p":
        B = batch or 256
        src = u8(B, H_IN, W_IN, C)
        dst = torch.empty((B, 720, 1280, C), dtype=torch.float32, device=dev)
        return {"batch": B, "px": W_IN * H_IN, "b_alg": resize_bytes(W_IN, H_IN, C, 1280, 720, 1, 4) * B,
                "kernel": "resize_strip_kernel", "frame": "1920x1080x3", "output": "1280x720x3 fp32",
                "desc": "resize_normalize INTER_LINEAR 1920x1080x3 u8 NHWC -> 1280x720x3 fp32 "
                        "(reference arithmetic, two weighted source rows per output row) + per-channel normalize",
                "main": lambda stream=None: ops.resize_normalize(src, 1280, 720, MEAN, STD, out=dst, stream=stream)}
    B = batch or 256
    src = u8(B, H_IN, W_IN, C)
    dst = torch.empty((B, H_OUT, W_OUT, C), dtype=torch.float32, device=dev)
    return {"batch": B, "px": W_IN * H_IN, "b_alg": resize_bytes(W_IN, H_IN, C, W_OUT, H_OUT, 1, 4) * B,
            "kernel": "resize_cols_kernel", "frame": "1920x1080x3", "output": "640x360x3 fp32",
            "desc": "resize_normalize INTER_LINEAR 1920x1080x3 u8 NHWC -> 640x360x3 fp32 "
                    "(reference arithmetic) + per-channel normalize",
            "main": lambda stream=None: ops.resize_normalize(src, W_OUT, H_OUT, MEAN, STD, out=dst, stream=stream)}


def dry_run(args, world: int, rank: int) -> None:
    """The rank protocol of main() on CPU over gloo: barrier + max-over-ranks
    timing of exactly --steps stand-in steps (a small torch CPU resize; cfg5
    also all-reduces a (c, 2) fp64 sums tensor as its real step does).  The
    JSON line is marked "dry_run" and carries no roofline: it measures nothing."""
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo")
        world = dist.get_world_size()
    x = torch.rand(4, 3, 108, 192)

    def step():
        torch.nn.functional.interpolate(x, size=(36, 64), mode="bilinear", align_corners=False)
        if args.workload == "cubic_stats" and world > 1:
            s = torch.ones(3, 2, dtype=torch.float64)
            dist.all_reduce(s)
            assert float(s[0, 0]) == world

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    if world > 1:
        dist.barrier()
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        print(json.dumps({"metric": "dry run (launcher check, not a measurement)", "value": None, "unit": None,
                          "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": round(float(t[0]) * 1e3 / args.steps, 4), "dry_run": True,
                          "config": {"workload": args.workload, "parallelism": f"dp{world}"}}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))  # before anything touches the GPU
    world = int(env_world or "1")
    if world != args.gpus:
        print(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}: the rank count must equal --gpus",
              file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        return dry_run(args, world, rank)

    import torch
    import torch.distributed as dist
    # VACV_BENCH_BACKEND=gloo runs the world > 1 protocol (barriers, the
    # MAX-over-ranks merge, cfg5's all-reduce) without RCCL, so it can be
    # exercised with several ranks on ONE GPU (ranks share the devices
    # round-robin); the driver's multi-GPU runs use the default, nccl = RCCL.
    backend = os.environ.get("VACV_BENCH_BACKEND", "nccl")
    if backend not in ("nccl", "gloo"):
        print(f"bench: VACV_BENCH_BACKEND={backend}: nccl or gloo", file=sys.stderr)
        sys.exit(2)
    if world > 1:
        ndev = torch.cuda.device_count()  # (counting does not initialise the GPU)
        if backend == "nccl":
            if local >= ndev:
                print(f"bench: rank {local} has no GPU ({ndev} visible); RCCL needs one GPU per rank",
                      file=sys.stderr)
                sys.exit(2)
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            local = local % max(ndev, 1)
            torch.cuda.set_device(local)
            dist.init_process_group("gloo")
        world = dist.get_world_size()  # what the process group agreed on, reported as n_gpus
    dev = torch.device("cuda", local if world > 1 else 0)
    torch.cuda.set_device(dev)

    ensure_built(rank, world)
    from vacv_amd import ops
    from vacv_amd.roofline import HBM_PEAK_GBS

    wl = make_workload(args.workload, args.batch, dev, rank, world, ops)
    B = wl["batch"]
    if world > 1:
        # value = B * world * px and cfg5's global count assume equal shards
        sizes = [None] * world
        dist.all_gather_object(sizes, B)
        if len(set(sizes)) != 1:
            print(f"bench: unequal per-rank batches {sizes}", file=sys.stderr)
            sys.exit(2)
    stream = torch.cuda.current_stream(dev)
    launch = wl["main"]       # the dominant kernel (timed alone for the roofline)
    extra = wl.get("extra")   # the rest of the step (e.g. cfg5's stats + all-reduce)

    for _ in range(args.warmup):
        launch()  # also builds and caches the resize plan (a one-time upload)
        if extra:
            extra()
    torch.cuda.synchronize(dev)

    # One step = one vacv_resize_normalize launch over the whole batch.  With
    # --graph it is captured once into a HIP graph and replayed (every replay
    # runs the full kernel); the default launches it from Python each step.
    graph = None
    if args.graph and not extra:
        try:
            # capture on a stream of our own, warmed first: the library keys its
            # per-stream workspaces (cfg5's fixed-point accumulators) by stream,
            # so their one-time allocation and zeroing happen before the capture
            # instead of being recorded into it
            cap = torch.cuda.Stream(dev)
            cap.wait_stream(torch.cuda.current_stream(dev))
            wl["main"](stream=cap)
            cap.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=cap):
                wl["main"](stream=cap)
            graph = g
            stream = torch.cuda.current_stream(dev)
        except Exception as e:  # capture unsupported: eager launches
            print(f"bench: graph capture failed ({e}); eager launches", file=sys.stderr)
            graph = None

    def step():
        if graph is not None:
            graph.replay()
        else:
            launch()

    if graph is not None:
        graph.replay()  # the instantiated graph's first replay, before the timed region
        torch.cuda.synchronize(dev)

    # the timed region: exactly K steps, nothing else queued between them
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    region = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    t0 = time.perf_counter()
    region[0].record(stream)
    for i in range(args.steps):
        step()
        if extra:
            extra()
    region[1].record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    gpu_step_ms = region[0].elapsed_time(region[1]) / args.steps  # GPU time per step, one event pair
    # the statistics the last timed step produced (the kernel-only re-timing
    # below overwrites the workload's buffers with per-rank sums)
    step_sums = wl["stats"]["sums"].clone() if (extra and "stats" in wl) else None

    # The dominant kernel's average duration (roofline): the timed region's
    # GPU time / K, from that one HIP event pair on the launch stream, where a
    # step is the launch alone (back-to-back launches: the region is the
    # kernels; for cfg5 it also holds the 4.5 us fixed_sums_kernel, so the
    # figure is conservative).  No events between the steps: an event pair
    # between two launches idled the GPU ~8-10 us (rocprofv3 kernel trace:
    # back-to-back cfg5 launches 0 us apart, 10 us apart with events), ~5 % of
    # a step.  With an extra (multi-GPU cfg5: the all-reduce), the main launch
    # alone is timed again, K times, each bracketed by events.
    if extra is None:
        kern_ms = gpu_step_ms
    else:
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
        for i in range(args.steps):
            ev[i][0].record(stream)
            step()
            ev[i][1].record(stream)
        torch.cuda.synchronize(dev)
        kern_ms = sum(a.elapsed_time(b) for a, b in ev) / args.steps

    # cfg5 across ranks: the step's statistics must be the GLOBAL ones -- the
    # all-reduced sums equal the sum of every rank's own shard sums (recomputed
    # here, gathered to the host, added in rank order)
    stats_check = None
    if world > 1 and step_sums is not None:
        import numpy as np
        from vacv_amd import INTER_CUBIC
        mine = ops.resize_channel_sums(wl["inputs"], 224, 224, INTER_CUBIC, per_image=False)[1].cpu().numpy()
        every = [None] * world
        dist.all_gather_object(every, mine)
        want = np.sum(np.stack(every), axis=0)
        got = step_sums.cpu().numpy()
        rel = float(np.max(np.abs(got - want) / np.maximum(np.abs(want), 1.0)))
        stats_check = {"max_rel_diff": rel, "ok": bool(rel <= 1e-9)}
        if not stats_check["ok"]:
            print(f"bench: global statistics differ from the ranks' sums (rel {rel:g})", file=sys.stderr)
            sys.exit(3)

    t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, kern_ms = float(t[0]), float(t[1])
    ms_per_step = elapsed * 1e3 / args.steps

    n_img = B * world
    value = n_img * wl["px"] / (ms_per_step / 1e3) / 1e6
    b_alg = wl["b_alg"]  # per launch (one GPU's batch)
    achieved = b_alg / (kern_ms / 1e3) / 1e9
    traffic = pmc_traffic(args.workload)

    out = None
    if rank == 0:
        # the host-CPU leg runs at N = 1 only (the multi-GPU lines time the GPUs)
        cpu = None if (args.no_cpu_baseline or world > 1) else cpu_baseline(args.cpu_seconds, args.workload)
        out = {
            "metric": "Mpixels/sec per op (resize/warp/normalize) at 1080p; achieved HBM GB/s vs peak",
            "value": round(value, 2),
            "unit": "Mpixels/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (torch.randint u8 frames resident in HBM)",
            "config": {"workload": wl["desc"], "global_batch": n_img, "batch_per_gpu": B,
                       "parallelism": f"dp{world}", "frame": wl["frame"], "output": wl["output"],
                       "graph": graph is not None, "backend": backend if world > 1 else None},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "kernel": wl["kernel"], "kernel_ms": round(kern_ms, 4), "alg_bytes_per_launch": b_alg,
                         "gpu_ms_per_step": round(gpu_step_ms, 4)},
            "cpu_baseline": cpu,
        }
        if stats_check is not None:
            out["global_stats_check"] = stats_check
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
