#!/usr/bin/env python3
"""Generate the committed golden fixtures from the REFERENCE's own code.

Run in the build container (needs /root/reference):
    make -C oracle ref && python tests/golden/make_golden.py

It drives oracle/_ref/libvacv_ref.so -- the reference's pixel loops
(resize_naive.cpp, warp_affine_naive.cpp, normalize_naive.cpp,
cvt_color.cpp, image_util.cpp) compiled from /root/reference by
oracle/Makefile -- on

  * synthetic images: oracle.synthetic_image(seed, h, w, c), i.e. per-channel
    gradients ((x*(37+11k))//w + (y*(53+7k))//h + 29k) mod 256 plus splitmix64
    noise in [-64, 63], clipped to u8;
  * the reference's test images (src/test/res/*.jp*, copied verbatim to
    tests/golden/res/), decoded with PIL and reordered to BGR (cv::imread's
    channel order; PIL and OpenCV decoders may differ by a few LSB, which
    does not matter because every comparison runs on the same decoded bytes).

Outputs:
  small_cases.npz  full input/output arrays of small cases (every op/mode)
  digests.json     SHA-256 of the reference outputs at the BASELINE configs
                   and the reference harness cases (src/test/src/impl/*.cpp)
Nothing here is reference source: these are data (inputs and the outputs the
reference computed from them).
"""
from __future__ import annotations

import hashlib
import json
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
sys.path.insert(0, str(REPO / "oracle"))

from oracle import Oracle, Reference, build_reference, synthetic_image  # noqa: E402

RES = HERE / "res"
MEAN = np.array([103.94, 116.78, 123.68], np.float32)
STD = np.array([57.375, 57.12, 58.395], np.float32)
HARNESS_M = np.array([0.849158, 0.012257, -474.827, -0.01225, 0.849158, -379.18], np.float32)  # test_warp_affine.cpp:31-32


def load_bgr(name: str) -> np.ndarray:
    from PIL import Image
    im = Image.open(RES / name).convert("RGB")
    return np.ascontiguousarray(np.asarray(im, dtype=np.uint8)[:, :, ::-1])


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def noisy_f32(img: np.ndarray, seed: int) -> np.ndarray:
    rng = np.random.default_rng(seed)
    return (img.astype(np.float32) + rng.standard_normal(img.shape).astype(np.float32) * 3.0).astype(np.float32)


def main() -> None:
    if not build_reference():
        sys.exit("reference sources unavailable: fixtures can only be generated in the build container")
    R, O = Reference(), Oracle()
    arrays: dict[str, np.ndarray] = {}
    cases: list[dict] = []

    def add(kind: str, inputs: dict, outputs: dict, **meta):
        # inputs are stored once per distinct content (keyed by digest)
        idx = len(cases)
        rec = {"kind": kind, "id": idx, **meta, "inputs": {}, "outputs": []}
        for k, v in inputs.items():
            key = "in_" + sha(v)[:16] + "_" + str(v.dtype)
            arrays[key] = v
            rec["inputs"][k] = key
        for k, v in outputs.items():
            arrays[f"c{idx}_out_{k}"] = v
            rec["outputs"].append(k)
        cases.append(rec)

    small = [(11, 23, 37, 1), (12, 48, 64, 3), (13, 61, 97, 3), (14, 5, 7, 3), (15, 16, 16, 4)]
    outs = [(20, 11), (33, 29), (111, 40), (7, 5), (2, 2), (160, 90)]
    real176 = load_bgr("176x144.jpg")

    # ---- bilinear (resize_naive.cpp:10-128) --------------------------------
    for seed, h, w, c in small:
        img = synthetic_image(seed, h, w, c)
        f = noisy_f32(img, seed)
        for wo, ho in outs:
            cc = c if c in (1, 3) else None
            u8 = R.resize_linear(img, wo, ho)
            add("resize_linear_u8", {"src": img}, {"dst": u8}, w_out=wo, h_out=ho)
            add("resize_linear_f32", {"src": f}, {"dst": R.resize_linear(f, wo, ho)}, w_out=wo, h_out=ho)
            if cc and h >= 4 and w >= 4:
                add("resize_cubic_f32", {"src": f}, {"dst": R.resize_cubic(f, wo, ho)}, w_out=wo, h_out=ho)
    for wo, ho in [(64, 48), (300, 200), (88, 72), (45, 45)]:
        add("resize_linear_u8", {"src": real176}, {"dst": R.resize_linear(real176, wo, ho)}, w_out=wo, h_out=ho)
        f = real176.astype(np.float32)
        add("resize_cubic_f32", {"src": f}, {"dst": R.resize_cubic(f, wo, ho)}, w_out=wo, h_out=ho)
    # the shipped hwc wrapper (valid when w_out == h_out, resize_naive.cpp:531-545)
    f = real176.astype(np.float32)
    add("resize_cubic_f32", {"src": f}, {"dst": R.resize_cubic(f, 56, 56, wrapper=True)}, w_out=56, h_out=56)

    # ---- affine (warp_affine_naive.cpp), M inverted by oracle_invert_affine --
    mats = [
        np.array([0.5, 0.1, 3.0, -0.2, 0.7, 5.0], np.float32),
        O.rotation_matrix(0.9, 15.0, [32, 24, 32, 24]),
        O.rotation_matrix(1.3, -40.0, [10, 10, 20, 8]),
        np.array([1.25, 0.0, -2.0, 0.0, 1.25, -2.0], np.float32),
    ]
    for seed, h, w, c in small[:3]:
        img = synthetic_image(seed, h, w, c)
        f = noisy_f32(img, seed + 100)
        for mi, m in enumerate(mats):
            inv = O.invert_affine(m)
            for wo, ho in [(64, 48), (33, 17)]:
                add("warp_affine_u8", {"src": img, "m": m}, {"dst": R.warp_affine_inv(img, inv, wo, ho)},
                    w_out=wo, h_out=ho)
                add("warp_affine_f32", {"src": f, "m": m}, {"dst": R.warp_affine_inv(f, inv, wo, ho)},
                    w_out=wo, h_out=ho)

    # ---- colour (image_util.cpp:9-41, cvt_color.cpp:39-135) -----------------
    for seed, h, w in [(21, 16, 24), (22, 36, 50), (23, 2, 2)]:
        bgr = synthetic_image(seed, h, w, 3)
        nv = R.bgr2nv21(bgr)
        add("bgr2nv21", {"src": bgr}, {"dst": nv})
        add("nv21_to_bgr", {"src": nv}, {"dst": R.nv21_to_bgr(nv)})
    rng = np.random.default_rng(5)
    yuv = rng.integers(0, 256, (48 * 3 // 2, 64), dtype=np.uint8)
    add("nv21_to_bgr", {"src": yuv}, {"dst": R.nv21_to_bgr(yuv)})
    nv176 = R.bgr2nv21(real176)
    add("bgr2nv21", {"src": real176}, {"dst": nv176})
    add("nv21_to_bgr", {"src": nv176}, {"dst": R.nv21_to_bgr(nv176)})

    # ---- normalize / mean_stddev (normalize_naive.cpp:7-90) ----------------
    for seed, h, w, c in [(31, 20, 30, 3), (32, 9, 13, 1)]:
        f = noisy_f32(synthetic_image(seed, h, w, c), seed)
        m, s = (MEAN, STD) if c == 3 else (MEAN[:1], STD[:1])
        add("normalize", {"src": f, "mean": m, "std": s}, {"dst": R.normalize(f, m, s)})
        rm, rs = R.mean_stddev(f)
        add("mean_stddev_ref", {"src": f}, {"mean": rm, "std": rs})
    for name in ["176x144.jpg", "284x214.jpg"]:
        f = load_bgr(name).astype(np.float32)
        rm, rs = R.mean_stddev(f)
        add("mean_stddev_ref", {"src": f}, {"mean": rm, "std": rs}, image=name)

    np.savez_compressed(HERE / "small_cases.npz", **arrays)

    # ---- digests at the BASELINE configs + reference harness cases --------
    dig: dict[str, dict] = {}
    b1080 = load_bgr("1920x1080.jpeg")
    b720 = load_bgr("1280x720.jpg")
    b720g = load_bgr("1280x720_grey.jpg")
    b1440 = load_bgr("2560x1440.jpeg")
    b640 = load_bgr("640x360.jpg")
    dig["input_1920x1080"] = {"sha256": sha(b1080)}
    dig["input_1280x720"] = {"sha256": sha(b720)}
    dig["input_1280x720_grey"] = {"sha256": sha(b720g)}
    dig["input_2560x1440"] = {"sha256": sha(b1440)}
    dig["input_640x360"] = {"sha256": sha(b640)}

    r = R.resize_linear(b1080, 640, 360)
    dig["cfg2_resize_1080p_640x360_u8"] = {"sha256": sha(r)}
    dig["cfg2_resize_1080p_1280x720_u8"] = {"sha256": sha(R.resize_linear(b1080, 1280, 720))}
    dig["target_resize_normalize_1080p_640x360"] = {
        "sha256": sha(R.normalize(r.astype(np.float32), MEAN, STD))}
    syn = synthetic_image(2, 1080, 1920, 3)
    dig["cfg2_synthetic_seed2_640x360_u8"] = {"sha256": sha(R.resize_linear(syn, 640, 360))}
    dig["target_synthetic_seed2_resize_normalize"] = {
        "sha256": sha(R.normalize(R.resize_linear(syn, 640, 360).astype(np.float32), MEAN, STD))}

    nv = R.bgr2nv21(b1080)
    bgr = R.nv21_to_bgr(nv)
    dig["cfg3_nv21_1080p"] = {"sha256": sha(nv)}
    dig["cfg3_nv21_to_bgr_1080p"] = {"sha256": sha(bgr)}
    dig["cfg3_nv21_bgr_normalize_1080p"] = {"sha256": sha(R.normalize(bgr.astype(np.float32), MEAN, STD))}

    rot = O.rotation_matrix(0.9, 15.0, [640, 360, 640, 360])
    dig["cfg4_rotation_matrix"] = {"m": [float(x) for x in rot]}
    dig["cfg4_warp_1280x720_rot15_u8"] = {"sha256": sha(R.warp_affine_inv(b720, O.invert_affine(rot), 1280, 720))}

    f1440 = b1440.astype(np.float32)
    cub = R.resize_cubic(f1440, 224, 224, wrapper=True)
    dig["cfg5_cubic_1440p_224_f32"] = {"sha256": sha(cub)}
    rm, rs = R.mean_stddev(cub)
    dig["cfg5_cubic_mean_stddev_ref"] = {"mean": [float(x) for x in rm], "std": [float(x) for x in rs]}

    # reference harness (src/test/src/impl/*.cpp)
    dig["harness_resize_hwc_u8_2560x1440_320x180"] = {"sha256": sha(R.resize_linear(b1440, 320, 180))}
    dig["harness_resize_hwc_f32_2560x1440_320x180"] = {"sha256": sha(R.resize_linear(f1440, 320, 180))}
    inv = O.invert_affine(HARNESS_M)
    dig["harness_warp_inverse_M"] = {"m": [float(x) for x in inv]}
    dig["harness_warp_hwc_u8_240"] = {"sha256": sha(R.warp_affine_inv(b720, inv, 240, 240))}
    dig["harness_warp_hwc_f32_240"] = {"sha256": sha(R.warp_affine_inv(b720.astype(np.float32), inv, 240, 240))}
    rot2 = O.rotation_matrix(1.073914, -3.314525, [738.518372, 537.672852, 204.766998, 73.329681])
    dig["harness_rotation_matrix"] = {"m": [float(x) for x in rot2]}
    dig["harness_rotation_u8_140x210"] = {"sha256": sha(R.warp_affine_inv(b720g, O.invert_affine(rot2), 140, 210))}
    for name, key in [("176x144.jpg", "176"), ("640x360.jpg", "640"), ("1280x720.jpg", "1280")]:
        im = load_bgr(name)
        nvx = R.bgr2nv21(im)
        dig[f"harness_nv21_{key}"] = {"sha256": sha(nvx), "bgr_sha256": sha(R.nv21_to_bgr(nvx))}
    for name in ["176x144.jpg", "284x214.jpg"]:
        f = load_bgr(name).astype(np.float32)
        rm, rs = R.mean_stddev(f)
        dig[f"harness_normalize_auto_{name}"] = {"sha256": sha(R.normalize(f, rm, rs)),
                                                 "mean": [float(x) for x in rm], "std": [float(x) for x in rs]}

    meta = {"cases": cases, "digests": dig, "mean": [float(x) for x in MEAN], "std": [float(x) for x in STD],
            "generator": "tests/golden/make_golden.py via oracle/_ref/libvacv_ref.so"}
    (HERE / "digests.json").write_text(json.dumps(meta, indent=1))
    print(f"{len(cases)} small cases, {len(dig)} digests")


if __name__ == "__main__":
    main()
