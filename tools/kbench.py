#!/usr/bin/env python3
"""Kernel micro-bench for profiling (rocprofv3 wraps this; no CPU work).

  python tools/kbench.py --op resize_normalize --iters 20
Prints one JSON line per op: average launch time from HIP events and the
algorithmic GB/s (vacv_amd.roofline)."""
import argparse
import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "arm-neon-opencv_amd"))

MEAN = [103.94, 116.78, 123.68]
STD = [57.375, 57.12, 58.395]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--op", default="resize_normalize")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--only", default="", help="run only the cases whose name contains this")
    ap.add_argument("--sweep", default="",
                    help="kernel-variant knobs (VACV_TUNE_*, vacv_set_tuning) to sweep, "
                         "e.g. 'DIRECT_ALIGN=0,1;RESIZE_WORK=2,4'")
    a = ap.parse_args()
    import torch
    import vacv_amd
    from vacv_amd import ops
    from vacv_amd.roofline import resize_bytes
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev)
    g.manual_seed(1)

    def frames(n, h, w, c=3):
        return torch.randint(0, 256, (n, h, w, c), dtype=torch.uint8, device=dev, generator=g)

    cases = {}
    if a.op in ("resize_normalize", "all"):
        n = a.batch or 256
        src = frames(n, 1080, 1920)
        out = torch.empty((n, 360, 640, 3), dtype=torch.float32, device=dev)
        cases["resize_normalize_1080p_640x360"] = (lambda src=src, out=out: ops.resize_normalize(src, 640, 360, MEAN, STD, out=out),
                                                   n * resize_bytes(1920, 1080, 3, 640, 360, 1, 4), n * 1920 * 1080)
    if a.op in ("resize", "all"):
        n = a.batch or 256
        src = frames(n, 1080, 1920)
        o1 = torch.empty((n, 360, 640, 3), dtype=torch.uint8, device=dev)
        o2 = torch.empty((n, 720, 1280, 3), dtype=torch.uint8, device=dev)
        cases["resize_1080p_640x360_u8"] = (lambda src=src, o1=o1: ops.resize(src, 640, 360, out=o1),
                                            n * resize_bytes(1920, 1080, 3, 640, 360, 1, 1), n * 1920 * 1080)
        cases["resize_1080p_1280x720_u8"] = (lambda src=src, o2=o2: ops.resize(src, 1280, 720, out=o2),
                                             n * resize_bytes(1920, 1080, 3, 1280, 720, 1, 1), n * 1920 * 1080)
    if a.op in ("resize_other", "all"):
        # INTER_NEAREST / INTER_AREA (OpenCV-delegated modes): read the frame, write the output
        n = a.batch or 256
        src = frames(n, 1080, 1920)
        o3 = torch.empty((n, 360, 640, 3), dtype=torch.uint8, device=dev)
        o2 = torch.empty((n, 540, 960, 3), dtype=torch.uint8, device=dev)
        cases["area_1080p_640x360_u8"] = (
            lambda src=src, o=o3: ops.resize(src, 640, 360, interpolation=vacv_amd.INTER_AREA, out=o),
            n * (1920 * 1080 * 3 + 640 * 360 * 3), n * 1920 * 1080)
        cases["area_1080p_960x540_u8"] = (
            lambda src=src, o=o2: ops.resize(src, 960, 540, interpolation=vacv_amd.INTER_AREA, out=o),
            n * (1920 * 1080 * 3 + 960 * 540 * 3), n * 1920 * 1080)
        # nearest reads one pixel in (1920/640)^2 = 9 (whole 64 B lines of them, all of 1 in 3 rows)
        cases["nearest_1080p_640x360_u8"] = (
            lambda src=src, o=o3: ops.resize(src, 640, 360, interpolation=vacv_amd.INTER_NEAREST, out=o),
            n * (360 * 1920 * 3 + 640 * 360 * 3), n * 1920 * 1080)
    if a.op in ("lanczos", "all"):
        # INTER_LANCZOS4: every source row is weighted (8 taps at a 3x downscale)
        n = a.batch or 256
        src = frames(n, 1080, 1920)
        o3 = torch.empty((n, 360, 640, 3), dtype=torch.uint8, device=dev)
        cases["lanczos_1080p_640x360_u8"] = (
            lambda src=src, o=o3: ops.resize(src, 640, 360, interpolation=vacv_amd.INTER_LANCZOS4, out=o),
            n * (1920 * 1080 * 3 + 640 * 360 * 3), n * 1920 * 1080)
        of = torch.empty((n, 360, 640, 3), dtype=torch.float32, device=dev)
        cases["lanczos_normalize_1080p_640x360"] = (
            lambda src=src, o=of: ops.resize_normalize(src, 640, 360, MEAN, STD, interpolation=vacv_amd.INTER_LANCZOS4,
                                                       out=o),
            n * (1920 * 1080 * 3 + 640 * 360 * 12), n * 1920 * 1080)
    if a.op in ("warp", "all"):
        n = a.batch or 128
        src = frames(n, 720, 1280)
        o = torch.empty_like(src)
        m = ops.rotation_matrix(0.9, 15.0, (640, 360, 640, 360))
        cases["warp_720p_rot15_u8"] = (lambda src=src, m=m, o=o: ops.warp_affine(src, m, 1280, 720, out=o), n * 2 * 1280 * 720 * 3,
                                       n * 1280 * 720)
        for rot in (0.0, 5.0, 45.0):
            mr = ops.rotation_matrix(0.9, rot, (640, 360, 640, 360))
            cases[f"warp_720p_rot{int(rot)}_u8"] = (lambda src=src, m=mr, o=o: ops.warp_affine(src, m, 1280, 720, out=o),
                                                   n * 2 * 1280 * 720 * 3, n * 1280 * 720)
        # INTER_NEAREST (OpenCV's fixed-point map): the source pixels it reads, ~1/0.81 of a frame at scale 0.9
        cases["warp_nearest_720p_rot15_u8"] = (
            lambda src=src, m=m, o=o: ops.warp_affine(src, m, 1280, 720, flags=vacv_amd.INTER_NEAREST, out=o),
            n * 2 * 1280 * 720 * 3, n * 1280 * 720)
        of = torch.empty((n, 720, 1280, 3), dtype=torch.float32, device=dev)
        cases["warp_normalize_720p_rot15"] = (lambda src=src, m=m, of=of: ops.warp_affine_normalize(src, m, 1280, 720, MEAN, STD, out=of),
                                              n * 5 * 1280 * 720 * 3, n * 1280 * 720)
    if a.op in ("cvt", "all"):
        n = a.batch or 256
        yuv = torch.randint(0, 256, (n, 1620, 1920), dtype=torch.uint8, device=dev, generator=g)
        o = torch.empty((n, 1080, 1920, 3), dtype=torch.float32, device=dev)
        cases["nv21_bgr_normalize_1080p"] = (lambda yuv=yuv, o=o: ops.cvt_color_normalize(yuv, mean=MEAN, std=STD, out=o),
                                             n * (1920 * 1620 + 1920 * 1080 * 12), n * 1920 * 1080)
    if a.op in ("cvt_cv", "all"):
        # the OpenCV colour codes (k_color_cv.hip): YUV420 in, 3 or 4 channels out; gray -> BGR
        n = a.batch or 256
        yuv = torch.randint(0, 256, (n, 1620, 1920), dtype=torch.uint8, device=dev, generator=g)
        o4 = torch.empty((n, 1080, 1920, 4), dtype=torch.uint8, device=dev)
        o3 = torch.empty((n, 1080, 1920, 3), dtype=torch.uint8, device=dev)
        cases["nv21_bgra_1080p"] = (lambda yuv=yuv, o=o4: ops.cvt_color(yuv, vacv_amd.COLOR_YUV2BGRA_NV21, out=o),
                                    n * (1920 * 1620 + 1920 * 1080 * 4), n * 1920 * 1080)
        cases["yv12_bgr_1080p"] = (lambda yuv=yuv, o=o3: ops.cvt_color(yuv, vacv_amd.COLOR_YUV2BGR_YV12, out=o),
                                   n * (1920 * 1620 + 1920 * 1080 * 3), n * 1920 * 1080)
        gray = yuv[:, :1080]
        cases["gray_bgr_1080p"] = (lambda g_=gray, o=o3: ops.cvt_color(g_, vacv_amd.COLOR_GRAY2BGR, out=o),
                                   n * 1920 * 1080 * 4, n * 1920 * 1080)
    if a.op in ("yuv_resize", "all"):
        from vacv_amd.roofline import yuv_resize_bytes
        n = a.batch or 256
        yuv = torch.randint(0, 256, (n, 1620, 1920), dtype=torch.uint8, device=dev, generator=g)
        o1 = torch.empty((n, 3, 360, 640), dtype=torch.float32, device=dev)
        o2 = torch.empty((n, 3, 224, 224), dtype=torch.float32, device=dev)
        cases["nv21_resize_normalize_1080p_640x360_chw"] = (
            lambda yuv=yuv, o1=o1: ops.cvt_color_resize_normalize(yuv, 640, 360, MEAN, STD, out=o1),
            n * yuv_resize_bytes(1920, 1080, 640, 360), n * 1920 * 1080)
        o3 = torch.empty((n, 360, 640, 3), dtype=torch.float32, device=dev)
        cases["nv21_resize_normalize_1080p_640x360_hwc"] = (
            lambda yuv=yuv, o3=o3: ops.cvt_color_resize_normalize(yuv, 640, 360, MEAN, STD, layout=vacv_amd.NHWC, out=o3),
            n * yuv_resize_bytes(1920, 1080, 640, 360), n * 1920 * 1080)
        o4 = torch.empty((n, 360, 640, 3), dtype=torch.uint8, device=dev)
        cases["nv21_resize_1080p_640x360_u8"] = (
            lambda yuv=yuv, o4=o4: ops.cvt_color_resize(yuv, 640, 360, out=o4),
            n * yuv_resize_bytes(1920, 1080, 640, 360, out_esize=1), n * 1920 * 1080)
        cases["nv21_resize_normalize_1080p_224_chw"] = (
            lambda yuv=yuv, o2=o2: ops.cvt_color_resize_normalize(yuv, 224, 224, MEAN, STD, out=o2),
            n * yuv_resize_bytes(1920, 1080, 224, 224), n * 1920 * 1080)
    if a.op in ("cubic", "all"):
        n = a.batch or 128
        src = frames(n, 1440, 2560)
        o = torch.empty((n, 224, 224, 3), dtype=torch.float32, device=dev)
        cases["cubic_1440p_224_u8_f32"] = (lambda src=src, o=o: ops.resize(src, 224, 224, interpolation=vacv_amd.INTER_CUBIC, out=o),
                                           n * resize_bytes(2560, 1440, 3, 224, 224, 1, 4, cubic=True), n * 2560 * 1440)
        cases["cubic_stats_1440p_224"] = (
            lambda src=src, o=o: ops.resize_mean_stddev(src, 224, 224, interpolation=vacv_amd.INTER_CUBIC,
                                                        per_image=False, out=o),
            n * resize_bytes(2560, 1440, 3, 224, 224, 1, 4, cubic=True), n * 2560 * 1440)
    if a.op in ("match", "all"):
        # correlation MACs: (W-w+1)(H-h+1) * w*h*c; bytes: image + result
        n = a.batch or 8
        src = frames(n, 720, 1280)
        tpl = frames(1, 64, 64)[0]
        o = torch.empty((n, 720 - 63, 1280 - 63), dtype=torch.float32, device=dev)
        for m, name in ((2, "ccorr"), (5, "ccoeff_normed")):
            cases[f"match_720p_64x64_{name}"] = (lambda src=src, tpl=tpl, o=o, m=m: ops.match_template(src, tpl, m, out=o),
                                                 n * (1280 * 720 * 3 + 657 * 1217 * 4), n * 1280 * 720)
        # GMAC/s of the correlation, for its compute roofline (v_dot4_u32_u8)
        macs = n * 657 * 1217 * 64 * 64 * 3
        cases["match_720p_64x64_ccorr_macs"] = (lambda src=src, tpl=tpl, o=o: ops.match_template(src, tpl, 2, out=o),
                                                macs, n * 1280 * 720)
    if a.op in ("dtype", "all", "calib"):
        n = a.batch or 64
        src = frames(n, 1080, 1920)
        o = torch.empty((n, 1080, 1920, 3), dtype=torch.float32, device=dev)
        cases["u8_to_f32_1080p"] = (lambda src=src, o=o: ops.change_dtype(src, torch.float32, out=o) if False else
                                    ops.change_dtype(src, torch.float32), n * 1920 * 1080 * 15, n * 1920 * 1080)
    if a.op in ("layout", "all"):
        n = a.batch or 256
        src = frames(n, 360, 640)
        cases["hwc_to_chw_640x360_u8"] = (lambda src=src: ops.change_layout(src, vacv_amd.NCHW),
                                          n * 640 * 360 * 6, n * 640 * 360)
    if a.only:
        cases = {k: v for k, v in cases.items() if a.only in k}
    import itertools
    knobs = [kv.split("=", 1) for kv in a.sweep.split(";") if kv]
    combos = list(itertools.product(*[[(k, v) for v in vals.split(",")] for k, vals in knobs])) or [()]
    for fn, _, _ in cases.values():  # clocks ramp before the first timed case
        for _ in range(100):
            fn()
    torch.cuda.synchronize()
    for combo in combos:
        for k, v in combo:
            ops.set_tuning(k, int(v))
        tag = " ".join(f"{k}={v}" for k, v in combo)
        run_cases(cases, a.iters, tag)


def run_cases(cases, iters, tag):
    import torch
    for name, (fn, nbytes, px) in cases.items():
        for _ in range(10):  # clocks settle before the timed launches
            fn()
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
        s = torch.cuda.current_stream()
        for e0, e1 in ev:
            e0.record(s)
            fn()
            e1.record(s)
        torch.cuda.synchronize()
        ms = sorted(e0.elapsed_time(e1) for e0, e1 in ev)
        med = ms[len(ms) // 2]
        if name.endswith("_macs"):
            # a compute rate, not bytes: u8 multiply-adds of the correlation
            # per second, against the dense i8 MFMA peak (~5 POP/s = 2.5
            # PMAC/s, MI355X_MICROARCH.md; the kernel's nibble split issues
            # twice these MACs on the matrix cores)
            rate = {"GMAC_s": round(nbytes / med / 1e6, 1), "frac_i8_mfma_dense": round(nbytes / med / 1e6 / 2.5e6, 4)}
        else:
            rate = {"alg_GBps": round(nbytes / med / 1e6, 1), "frac_8TBps": round(nbytes / med / 1e6 / 8000, 4)}
        print(json.dumps({"case": name, **({"knobs": tag} if tag else {}), "ms_median": round(med, 4),
                          "ms_min": round(ms[0], 4), **rate, "Mpx_s": round(px / med / 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
