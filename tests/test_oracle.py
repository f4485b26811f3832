"""Pin the CPU oracle (oracle/vacv_oracle.c) to the reference.

Every small golden case (tests/golden/small_cases.npz, produced by the
reference's own loops via tests/golden/make_golden.py) must be reproduced
bit for bit; the large BASELINE-config and harness cases are checked by
SHA-256.  When oracle/_ref (the reference built from /root/reference) is
present, random cases are also cross-checked live.
"""
from __future__ import annotations

import hashlib

import numpy as np
import pytest

from conftest import load_bgr


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def run_case(O, kind, inp, meta):
    if kind in ("resize_linear_u8", "resize_linear_f32"):
        return {"dst": O.resize_linear(inp["src"], meta["w_out"], meta["h_out"])}
    if kind == "resize_cubic_f32":
        return {"dst": O.resize_cubic(inp["src"], meta["w_out"], meta["h_out"])}
    if kind in ("warp_affine_u8", "warp_affine_f32"):
        return {"dst": O.warp_affine(inp["src"], inp["m"], meta["w_out"], meta["h_out"])}
    if kind == "bgr2nv21":
        return {"dst": O.bgr2nv21(inp["src"])}
    if kind == "nv21_to_bgr":
        return {"dst": O.yuv420sp_to_bgr(inp["src"], v_first=True)}
    if kind == "normalize":
        return {"dst": O.normalize(inp["src"], inp["mean"], inp["std"])}
    if kind == "mean_stddev_ref":
        m, s = O.mean_stddev_ref(inp["src"])
        return {"mean": m, "std": s}
    raise KeyError(kind)


def test_small_cases_bit_exact(oracle, golden):
    meta, arrays = golden
    kinds = set()
    for case in meta["cases"]:
        inp = {k: arrays[v] for k, v in case["inputs"].items()}
        got = run_case(oracle, case["kind"], inp, case)
        for k in case["outputs"]:
            want = arrays[f"c{case['id']}_out_{k}"]
            g = got[k]
            assert g.shape == want.shape, (case["kind"], case["id"])
            assert g.dtype == want.dtype
            assert np.array_equal(g.view(np.uint8), want.view(np.uint8)), (case["kind"], case["id"], case)
        kinds.add(case["kind"])
    assert kinds == {"resize_linear_u8", "resize_linear_f32", "resize_cubic_f32", "warp_affine_u8",
                     "warp_affine_f32", "bgr2nv21", "nv21_to_bgr", "normalize", "mean_stddev_ref"}


@pytest.fixture(scope="module")
def images(golden):
    meta, _ = golden
    d = meta["digests"]
    imgs = {"1080": load_bgr("1920x1080.jpeg"), "720": load_bgr("1280x720.jpg"),
            "720g": load_bgr("1280x720_grey.jpg"), "1440": load_bgr("2560x1440.jpeg")}
    for key, name in [("1080", "input_1920x1080"), ("720", "input_1280x720"), ("720g", "input_1280x720_grey"),
                      ("1440", "input_2560x1440")]:
        if sha(imgs[key]) != d[name]["sha256"]:
            pytest.skip("this PIL decodes the test JPEGs differently from the fixture generator")
    return imgs


def test_config_digests(oracle, golden, images):
    meta, _ = golden
    d = meta["digests"]
    mean = np.array(meta["mean"], np.float32)
    std = np.array(meta["std"], np.float32)
    O = oracle
    r = O.resize_linear(images["1080"], 640, 360)
    assert sha(r) == d["cfg2_resize_1080p_640x360_u8"]["sha256"]
    assert sha(O.resize_linear(images["1080"], 1280, 720)) == d["cfg2_resize_1080p_1280x720_u8"]["sha256"]
    assert sha(O.normalize(O.u8_to_f32(r), mean, std)) == d["target_resize_normalize_1080p_640x360"]["sha256"]
    nv = O.bgr2nv21(images["1080"])
    assert sha(nv) == d["cfg3_nv21_1080p"]["sha256"]
    bgr = O.yuv420sp_to_bgr(nv)
    assert sha(bgr) == d["cfg3_nv21_to_bgr_1080p"]["sha256"]
    assert sha(O.normalize(O.u8_to_f32(bgr), mean, std)) == d["cfg3_nv21_bgr_normalize_1080p"]["sha256"]
    rot = O.rotation_matrix(0.9, 15.0, [640, 360, 640, 360])
    assert rot.tolist() == pytest.approx(d["cfg4_rotation_matrix"]["m"], abs=0)
    assert sha(O.warp_affine(images["720"], rot, 1280, 720)) == d["cfg4_warp_1280x720_rot15_u8"]["sha256"]
    cub = O.resize_cubic(O.u8_to_f32(images["1440"]), 224, 224)
    assert sha(cub) == d["cfg5_cubic_1440p_224_f32"]["sha256"]
    m, s = O.mean_stddev_ref(cub)
    assert m.tolist() == d["cfg5_cubic_mean_stddev_ref"]["mean"]
    assert s.tolist() == d["cfg5_cubic_mean_stddev_ref"]["std"]


def test_harness_digests(oracle, golden, images):
    meta, _ = golden
    d = meta["digests"]
    O = oracle
    assert sha(O.resize_linear(images["1440"], 320, 180)) == d["harness_resize_hwc_u8_2560x1440_320x180"]["sha256"]
    f1440 = O.u8_to_f32(images["1440"])
    assert sha(O.resize_linear(f1440, 320, 180)) == d["harness_resize_hwc_f32_2560x1440_320x180"]["sha256"]
    M = np.array([0.849158, 0.012257, -474.827, -0.01225, 0.849158, -379.18], np.float32)
    inv = O.invert_affine(M)
    assert inv.tolist() == d["harness_warp_inverse_M"]["m"]
    # the survey's recorded run of the reference: M is mutated to
    # [1.177392 -0.016995 552.613 ; 0.016985 1.177392 454.508]
    assert np.allclose(inv, [1.177392, -0.016995, 552.613, 0.016985, 1.177392, 454.508], atol=5e-4)
    assert sha(O.warp_affine(images["720"], M, 240, 240)) == d["harness_warp_hwc_u8_240"]["sha256"]
    assert sha(O.warp_affine(O.u8_to_f32(images["720"]), M, 240, 240)) == d["harness_warp_hwc_f32_240"]["sha256"]
    rot2 = O.rotation_matrix(1.073914, -3.314525, [738.518372, 537.672852, 204.766998, 73.329681])
    assert rot2.tolist() == d["harness_rotation_matrix"]["m"]
    assert sha(O.warp_affine(images["720g"], rot2, 140, 210)) == d["harness_rotation_u8_140x210"]["sha256"]


def test_layout_dtype_crop_semantics(oracle):
    """tensor.cpp:160-182 / :459-502 and crop.cpp:44-125 live behind the
    unbuildable Tensor code; they are index maps, pinned here against numpy's
    definition of the same maps."""
    from oracle import synthetic_image
    O = oracle
    img = synthetic_image(3, 37, 53, 3)
    chw = O.hwc_to_chw(img)
    assert np.array_equal(chw, img.transpose(2, 0, 1))
    assert np.array_equal(O.chw_to_hwc(chw), img)
    f = np.linspace(-3, 300, 999, dtype=np.float32)
    u = O.f32_to_u8(f)
    want = np.where(f > 0, np.trunc(f), 0).astype(np.int64) & 0xFF
    assert np.array_equal(u, want.astype(np.uint8))
    assert np.array_equal(O.u8_to_f32(img), img.astype(np.float32))
    assert np.array_equal(O.crop(img, 10, 20, 30, 15), img[20:35, 10:40])
    assert np.array_equal(O.crop(chw, 5, 6, 7, 8, chw=True), chw[:, 6:14, 5:12])


def test_exact_stats(oracle):
    from oracle import synthetic_image
    img = synthetic_image(9, 123, 77, 3)
    m, s = oracle.mean_stddev_exact(img)
    f = img.astype(np.float64).reshape(-1, 3)
    assert np.allclose(m, f.mean(0), rtol=0, atol=1e-5)
    assert np.allclose(s, f.std(0), rtol=1e-6)


@pytest.mark.skipif(not __import__("oracle").Reference.available(), reason="oracle/_ref not built")
def test_live_cross_check_random(oracle):
    """Random shapes against the reference loops (only where /root/reference built)."""
    from oracle import Reference
    R = Reference()
    rng = np.random.default_rng(1234)
    for _ in range(40):
        h, w = int(rng.integers(2, 90)), int(rng.integers(2, 90))
        c = int(rng.choice([1, 3]))
        img = rng.integers(0, 256, (h, w, c) if c > 1 else (h, w), dtype=np.uint8)
        wo, ho = int(rng.integers(1, 120)), int(rng.integers(1, 120))
        assert np.array_equal(oracle.resize_linear(img, wo, ho), R.resize_linear(img, wo, ho))
        f = img.astype(np.float32) * np.float32(0.37) - np.float32(11.0)
        assert np.array_equal(oracle.resize_linear(f, wo, ho).view(np.uint32), R.resize_linear(f, wo, ho).view(np.uint32))
        if h >= 4 and w >= 4:
            a, b = oracle.resize_cubic(f, wo, ho), R.resize_cubic(f, wo, ho)
            assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
        m = np.array([rng.uniform(0.3, 2), rng.uniform(-0.5, 0.5), rng.uniform(-20, 20),
                      rng.uniform(-0.5, 0.5), rng.uniform(0.3, 2), rng.uniform(-20, 20)], np.float32)
        inv = oracle.invert_affine(m)
        assert np.array_equal(oracle.warp_affine(img, m, wo, ho), R.warp_affine_inv(img, inv, wo, ho))


def test_resize_nearest_restatement(oracle):
    """OpenCV 2.4 resizeNN as restated in oracle/vacv_oracle.c (parity
    unpinned: no reference entry or fixture covers nearest): an integer
    downscale picks every k-th pixel, same size is a copy, an upscale
    repeats pixels, and indices never pass the last row/column."""
    import numpy as np
    from oracle import synthetic_image
    img = synthetic_image(3, 30, 40, 3)
    assert np.array_equal(oracle.resize_nearest(img, 20, 10), img[::3, ::2])
    assert np.array_equal(oracle.resize_nearest(img, 40, 30), img)
    up = oracle.resize_nearest(img, 80, 60)
    assert np.array_equal(up[::2, ::2], img) and np.array_equal(up[1::2, 1::2], img)
    odd = oracle.resize_nearest(img, 7, 11)
    xs = [min(int(np.floor(x * (1.0 / (7 / 40)))), 39) for x in range(7)]
    ys = [min(int(np.floor(y * (1.0 / (11 / 30)))), 29) for y in range(11)]
    assert np.array_equal(odd, img[ys][:, xs])


def test_resize_area_restatement(oracle):
    """OpenCV 2.4 resizeAreaFast_ as restated in oracle/vacv_oracle.c (parity
    unpinned), against an independent numpy statement: u8 = rint_half_even(
    fp32(block sum) * fp32(1/area)), except 2x2 blocks with 1, 3 or 4
    channels, which take ResizeAreaFastVec's fast_mode (sum + 2) >> 2 (half
    up); fp32 = the block mean with OpenCV's grouping (exact here:
    small-integer fp32 inputs sum exactly)."""
    import numpy as np
    from oracle import synthetic_image
    for c in (1, 2, 3, 4):
        img = synthetic_image(4 + c, 30, 42, c)
        if c == 1:
            img = img.reshape(30, 42)
        for ax, ay in [(1, 1), (2, 2), (3, 2), (2, 3), (6, 5), (7, 3)]:
            wo, ho = 42 // ax, 30 // ay
            blk = img.reshape(ho, ay, wo, ax, c).astype(np.int64).sum(axis=(1, 3))
            if ax == 2 and ay == 2 and c != 2:
                want = ((blk + 2) >> 2).astype(np.uint8)
            else:
                want = np.rint(blk.astype(np.float32) * np.float32(1.0 / (ax * ay))).astype(np.uint8)
            got = oracle.resize_area(img, wo, ho)
            assert np.array_equal(got.reshape(want.shape), want), (ax, ay, c)
    img = synthetic_image(4, 30, 42, 3)
    for ax, ay in [(1, 1), (2, 2), (3, 2), (6, 5), (7, 3)]:
        wo, ho = 42 // ax, 30 // ay
        blk = img.reshape(ho, ay, wo, ax, 3).astype(np.int64).sum(axis=(1, 3))
        f = img.astype(np.float32)
        wantf = blk.astype(np.float32) * np.float32(np.float32(1) / np.float32(ax * ay))
        assert np.array_equal(oracle.resize_area(f, wo, ho), wantf), (ax, ay)
    # ties round to even: a 2x1 block of (1, 2) averages 1.5 -> 2, (2, 3) -> 2
    tie = np.array([[[1], [2], [2], [3]]], np.uint8).reshape(1, 4)
    assert oracle.resize_area(tie, 2, 1).tolist() == [[2, 2]]
    # 2x2 ties (sum = 4k + 2) round half UP for cn 1/3/4 and half to even
    # for cn 2 (the generic path): sums 2 -> 1, 6 -> 2, 10 -> 3, 14 -> 4
    for c in (1, 2, 3, 4):
        sums = np.array([2, 6, 10, 14], np.int64)
        blk = np.zeros((2, 8, c), np.uint8)
        for j, sm in enumerate(sums):
            q = [sm // 4 + (1 if t < sm % 4 else 0) for t in range(4)]
            blk[0, 2 * j], blk[0, 2 * j + 1], blk[1, 2 * j], blk[1, 2 * j + 1] = q
        got = oracle.resize_area(blk if c > 1 else blk[:, :, 0], 4, 1).reshape(4, c)[:, 0].tolist()
        want = [1, 2, 3, 4] if c != 2 else [0, 2, 2, 4]
        assert got == want, (c, got)


def test_warp_border_modes_restatement(oracle):
    """The non-CONSTANT warp border modes of oracle/vacv_oracle.c (a build
    extension, parity unpinned) against an independent numpy statement:
    OpenCV 2.4 borderInterpolate's loops run literally, the naive sampler's
    float coordinates and fixed-point weights."""
    import numpy as np
    from oracle import synthetic_image

    def interp(p, n, mode):  # core/base.hpp borderInterpolate, as written
        if 0 <= p < n:
            return p
        if mode == 1:
            return 0 if p < 0 else n - 1
        if mode == 3:
            return p % n
        d = 1 if mode == 4 else 0
        if n == 1:
            return 0
        while not 0 <= p < n:
            p = -p - 1 + d if p < 0 else n - 1 - (p - n) - d
        return p

    img = synthetic_image(21, 9, 13, 2)
    m = np.array([0.8, 0.3, -4.0, -0.25, 0.9, 3.5], np.float32)
    inv = oracle.invert_affine(m)
    f32 = np.float32
    for mode in (1, 2, 3, 4):
        got = oracle.warp_affine(img, m, 20, 15, border_mode=mode)
        for y in range(15):
            for x in range(20):
                fx = f32(f32(inv[0] * f32(x)) + f32(inv[1] * f32(y))) + inv[2]
                fy = f32(f32(inv[3] * f32(x)) + f32(inv[4] * f32(y))) + inv[5]
                ix, iy = int(np.floor(fx)), int(np.floor(fy))
                if 0 <= ix <= 11 and 0 <= iy <= 7:
                    continue  # the naive sampler's own pixels: pinned by the golden vectors
                ax, ay = f32(fx - f32(ix)), f32(fy - f32(iy))
                wx0 = int(f32(f32(f32(1) - ax) * f32(2048)) + f32(0.5))
                wy0 = int(f32(f32(f32(1) - ay) * f32(2048)) + f32(0.5))
                wx1, wy1 = 2048 - wx0, 2048 - wy0
                x0, x1 = interp(ix, 13, mode), interp(ix + 1, 13, mode)
                y0, y1 = interp(iy, 9, mode), interp(iy + 1, 9, mode)
                for k in range(2):
                    v = (int(img[y0, x0, k]) * wx0 * wy0 + int(img[y1, x0, k]) * wx0 * wy1 +
                         int(img[y0, x1, k]) * wx1 * wy0 + int(img[y1, x1, k]) * wx1 * wy1) >> 22
                    assert got[y, x, k] == v, (mode, x, y, k)


def test_resize_area_any_restatement(oracle):
    """OpenCV 2.4 resizeArea_ (fractional INTER_AREA down-scales) and the
    area-mode bilinear (up-scales) as restated in oracle/vacv_oracle.c (a
    build extension, parity unpinned), against an independent numpy
    statement of imgwarp.cpp's computeResizeAreaTab / row loop and of the
    area-mode tap formula with the fixed-point rows."""
    import math
    import numpy as np
    from oracle import synthetic_image
    f32 = np.float32

    def tab(ssize, dsize, scale):
        out = [[] for _ in range(dsize)]
        for dx in range(dsize):
            fsx1 = dx * scale
            fsx2 = fsx1 + scale
            cell = min(scale, ssize - fsx1)
            sx1, sx2 = math.ceil(fsx1), math.floor(fsx2)
            sx2 = min(sx2, ssize - 1)
            sx1 = min(sx1, sx2)
            if sx1 - fsx1 > 1e-3:
                out[dx].append((sx1 - 1, f32((sx1 - fsx1) / cell)))
            for sx in range(sx1, sx2):
                out[dx].append((sx, f32(1.0 / cell)))
            if fsx2 - sx2 > 1e-3:
                out[dx].append((sx2, f32(min(min(fsx2 - sx2, 1.0), cell) / cell)))
        return out

    img = synthetic_image(31, 17, 23, 2)
    for wo, ho in [(10, 7), (15, 11), (22, 16)]:
        xt, yt = tab(23, wo, 23 / wo), tab(17, ho, 17 / ho)
        got = oracle.resize_area_any(img, wo, ho)
        for y in range(ho):
            for x in range(wo):
                for c in range(2):
                    sm = None
                    for sy, beta in yt[y]:
                        buf = f32(0)
                        for sx, al in xt[x]:
                            buf = f32(buf + f32(f32(img[sy, sx, c]) * al))
                        t = f32(beta * buf)
                        sm = t if sm is None else f32(sm + t)
                    assert got[y, x, c] == min(255, max(0, int(np.rint(sm)))), (wo, ho, x, y, c)

    def up_tap(d, n, scale, inv):
        sx = math.floor(d * scale)
        fx = f32((d + 1) - (sx + 1) * inv)
        fx = f32(0) if fx <= 0 else f32(fx - f32(math.floor(fx)))
        if sx >= n - 1:
            sx, fx = n - 1, f32(0)
        return sx, min(sx + 1, n - 1), fx

    for wo, ho in [(40, 30), (60, 9)]:  # up in both axes; up in x, down in y
        got = oracle.resize_area_any(img, wo, ho)
        ix, iy = wo / 23, ho / 17
        for y in range(ho):
            y0, y1, fy = up_tap(y, 17, 1 / iy, iy)
            b0, b1 = int(np.rint(f32(f32(1) - fy) * f32(2048))), int(np.rint(fy * f32(2048)))
            for x in range(wo):
                x0, x1, fx = up_tap(x, 23, 1 / ix, ix)
                a0, a1 = int(np.rint(f32(f32(1) - fx) * f32(2048))), int(np.rint(fx * f32(2048)))
                for c in range(2):
                    h0 = int(img[y0, x0, c]) * a0 + int(img[y0, x1, c]) * a1
                    h1 = int(img[y1, x0, c]) * a0 + int(img[y1, x1, c]) * a1
                    v = (((h0 >> 4) * b0) >> 16) + (((h1 >> 4) * b1) >> 16) + 2
                    assert got[y, x, c] == min(255, max(0, v >> 2)), (wo, ho, x, y, c)


def test_match_template_restatement(oracle):
    """oracle_match_template (cv::matchTemplate restated, parity unpinned)
    against an independent numpy statement of templmatch.cpp's formulas."""
    import numpy as np
    from oracle import synthetic_image
    img = synthetic_image(61, 20, 26, 3).astype(np.float64)
    tpl = img[4:11, 6:15].copy()
    h, w, cn = tpl.shape
    H, W = img.shape[:2]
    inv_area = 1.0 / (h * w)
    tm = tpl.reshape(-1, cn).mean(0)
    td = np.sqrt(np.maximum((tpl.reshape(-1, cn) ** 2).mean(0) - tm * tm, 0))
    for method in range(6):
        got = oracle.match_template(img.astype(np.uint8), tpl.astype(np.uint8), method)
        want = np.zeros((H - h + 1, W - w + 1))
        norm = float((td ** 2).sum())
        sum2 = norm + float((tm ** 2).sum())
        tmean = tm if method in (4, 5) else np.zeros(cn)
        if method not in (4, 5):
            norm = sum2
        tsum2 = sum2 / inv_area
        tnorm = np.sqrt(norm) / np.sqrt(inv_area)
        for y in range(H - h + 1):
            for x in range(W - w + 1):
                win = img[y:y + h, x:x + w]
                num = float(np.float32((win * tpl).sum()))
                if method == 2:
                    want[y, x] = num
                    continue
                S = win.reshape(-1, cn).sum(0)
                Q = float((win ** 2).sum())
                m2 = 0.0
                if method in (4, 5):
                    for c in range(cn):
                        m2 += S[c] * S[c]
                        num -= S[c] * tmean[c]
                    m2 *= inv_area
                if method in (0, 1):
                    num = max(Q - 2 * num + tsum2, 0.0)
                if method in (1, 3, 5):
                    t = np.sqrt(max(Q - m2, 0.0)) * tnorm
                    num = num / t if abs(num) < t else (np.sign(num) if abs(num) < t * 1.125 else (1 if method == 1 else 0))
                want[y, x] = num
        np.testing.assert_allclose(got, want.astype(np.float32), rtol=2e-6, atol=1e-6, err_msg=str(method))


def test_cv_color_restatement(oracle):
    """cv::cvtColor codes the reference delegates to OpenCV (cvt_color.cpp:
    139-141): YUV420sp -> RGBA/BGRA (94-97), YV12 -> BGR (99) and GRAY2BGR (8).
    oracle/vacv_oracle.c restates OpenCV 2.4's BT.601 fixed point; here an
    independent numpy statement of the same formula (vectorised, int64) over
    random frames and the saturating extremes.  Parity unpinned: no OpenCV
    runs here; the constants are those of OpenCV 2.4.13.4's own YUV2RGBA_NV12
    kernel text."""
    rng = np.random.default_rng(11)
    h, w = 10, 14
    for yuv in (rng.integers(0, 256, (h * 3 // 2, w), dtype=np.uint8),
                np.tile(np.array([0, 255], np.uint8), (h * 3 // 2, w // 2))):
        Y = yuv[:h].astype(np.int64)
        for code, (layout, dcn, bidx) in oracle.CV_YUV_CODES.items():
            if layout <= 1:
                pairs = yuv[h:].reshape(h // 2, w // 2, 2).astype(np.int64)
                U, V = (pairs[..., 0], pairs[..., 1]) if layout == 0 else (pairs[..., 1], pairs[..., 0])
            else:
                planes = yuv[h:].reshape(-1)
                q = (h // 2) * (w // 2)
                p0, p1 = planes[:q].reshape(h // 2, w // 2), planes[q:2 * q].reshape(h // 2, w // 2)
                V, U = (p0, p1) if layout == 2 else (p1, p0)
            u = np.repeat(np.repeat(U.astype(np.int64) - 128, 2, 0), 2, 1)
            v = np.repeat(np.repeat(V.astype(np.int64) - 128, 2, 0), 2, 1)
            yy = np.maximum(Y - 16, 0) * 1220542
            r = np.clip((yy + (1 << 19) + 1673527 * v) >> 20, 0, 255)
            g = np.clip((yy + (1 << 19) - 852492 * v - 409993 * u) >> 20, 0, 255)
            b = np.clip((yy + (1 << 19) + 2116026 * u) >> 20, 0, 255)
            want = np.zeros((h, w, dcn), np.uint8)
            want[..., bidx], want[..., 1], want[..., 2 - bidx] = b, g, r
            if dcn == 4:
                want[..., 3] = 255
            assert np.array_equal(oracle.yuv420_cv(yuv, code), want), code
    gray = rng.integers(0, 256, (5, 7), dtype=np.uint8)
    assert np.array_equal(oracle.gray_to_bgr(gray), np.repeat(gray[..., None], 3, 2))
    gf = rng.standard_normal((5, 7)).astype(np.float32)
    want4 = np.concatenate([np.repeat(gf[..., None], 3, 2), np.ones((5, 7, 1), np.float32)], 2)
    assert np.array_equal(oracle.gray_to_bgr(gf, 4), want4)


def test_warp_nearest_restatement(oracle):
    """cv::warpAffine INTER_NEAREST (the reference hands it to OpenCV,
    warp_affine.cpp:114-118): oracle_warp_affine_nn against an independent
    numpy statement of OpenCV 2.4's fixed point (fp64 inverse, AB_BITS = 10,
    half-to-even rounding) and remap's nearest sampler, for a forward and an
    inverse map (WARP_INVERSE_MAP), CONSTANT / REPLICATE / WRAP borders.
    Parity unpinned."""
    rng = np.random.default_rng(17)
    img = rng.integers(0, 256, (23, 31, 3), dtype=np.uint8)
    m = oracle.rotation_matrix(0.8, 27.0, [15, 11, 18, 9])
    inv32 = oracle.invert_affine(m)
    for inverse in (False, True):
        if inverse:
            given = inv32
            M = inv32.astype(np.float64)
        else:
            given = m
            f = m.astype(np.float64)
            D = f[0] * f[4] - f[1] * f[3]
            D = 1.0 / D if D != 0 else 0.0
            M = np.array([f[4] * D, f[1] * -D, 0.0, f[3] * -D, f[0] * D, 0.0])
            M[2] = -M[0] * f[2] - M[1] * f[5]
            M[5] = -M[3] * f[2] - M[4] * f[5]
        ys, xs = np.mgrid[0:19, 0:29]
        X0 = np.rint((M[1] * ys + M[2]) * 1024.0).astype(np.int64) + 512
        Y0 = np.rint((M[4] * ys + M[5]) * 1024.0).astype(np.int64) + 512
        X = np.clip((X0 + np.rint(M[0] * xs * 1024.0).astype(np.int64)) >> 10, -32768, 32767)
        Y = np.clip((Y0 + np.rint(M[3] * xs * 1024.0).astype(np.int64)) >> 10, -32768, 32767)
        inside = (X >= 0) & (X < 31) & (Y >= 0) & (Y < 23)
        for mode in (0, 1, 3):
            if mode == 0:
                want = np.zeros((19, 29, 3), np.uint8)
                want[...] = (7, 8, 9)
                want[inside] = img[Y[inside], X[inside]]
            else:
                bx = np.clip(X, 0, 30) if mode == 1 else np.mod(X, 31)
                by = np.clip(Y, 0, 22) if mode == 1 else np.mod(Y, 23)
                want = img[by, bx]
            got = oracle.warp_affine_nn(img, given, 29, 19, inverse_map=inverse, border_mode=mode, border=(7, 8, 9, 0))
            assert np.array_equal(got, want), (inverse, mode)


def _lanczos_numpy(img, w_out, h_out):
    """An independent numpy statement of OpenCV 2.4's INTER_LANCZOS4
    (interpolateLanczos4 + resize()'s tables + replicate borders), u8 only:
    separable integer sums in fixed point, the column pass on every source
    row first, then the 8-row pass."""
    h, w, c = img.shape
    f32 = np.float32

    def coeffs(x):
        x = f32(x)
        if x < np.finfo(np.float32).eps:
            out = np.zeros(8, np.float32)
            out[3] = 1
            return out
        s45 = 0.70710678118654752440084436210485
        cs = [(1, 0), (-s45, -s45), (0, 1), (s45, -s45), (-1, 0), (s45, s45), (0, -1), (-s45, s45)]
        y0 = -float(x + f32(3)) * 3.1415926535897932384626433832795 * 0.25
        s0, c0 = np.sin(y0), np.cos(y0)
        out = np.zeros(8, np.float32)
        tot = f32(0)
        for i in range(8):
            y = -float(x + f32(3) - f32(i)) * 3.1415926535897932384626433832795 * 0.25
            out[i] = f32((cs[i][0] * s0 + cs[i][1] * c0) / (y * y))
            tot = f32(tot + out[i])
        return (out * f32(f32(1) / tot)).astype(np.float32)

    def table(n_in, n_out):
        sc = 1.0 / (n_out / n_in)
        idx, wts = [], []
        for d in range(n_out):
            fx = f32((d + 0.5) * sc - 0.5)
            s = int(np.floor(fx))
            fx = f32(fx - f32(s))
            cf = coeffs(fx)
            wts.append(np.clip(np.rint(cf * f32(2048)), -32768, 32767).astype(np.int64))
            idx.append(np.clip(np.arange(s - 3, s + 5), 0, n_in - 1))
        return np.array(idx), np.array(wts)

    xi, xw = table(w, w_out)
    yi, yw = table(h, h_out)
    src = img.astype(np.int64)
    rows = (src[:, xi, :] * xw[None, :, :, None]).sum(axis=2)          # (h, w_out, c)
    acc = (rows[yi, :, :] * yw[:, :, None, None]).sum(axis=1)         # (h_out, w_out, c)
    return np.clip((acc + (1 << 21)) >> 22, 0, 255).astype(np.uint8)


def test_lanczos4_restatement(oracle):
    """INTER_LANCZOS4 (the reference hands it to cv::resize, resize.cpp:46-48;
    cv.h:33): oracle_resize_lanczos4 against an independent numpy statement
    for u8 down- and up-scales with 1 and 3 channels, and the identity at
    equal size (coefficients (0, 0, 0, 1, 0, ...)) for u8 and fp32.  Parity
    unpinned: OpenCV is not runnable here."""
    rng = np.random.default_rng(23)
    for (h, w, c), (wo, ho) in [((21, 34, 3), (13, 9)), ((17, 12, 1), (29, 40)), ((32, 48, 3), (48, 20)),
                                ((9, 9, 3), (5, 7))]:
        img = rng.integers(0, 256, (h, w, c), dtype=np.uint8)
        got = oracle.resize_lanczos4(img if c > 1 else img[..., 0], wo, ho)
        want = _lanczos_numpy(img, wo, ho)
        assert np.array_equal(got.reshape(want.shape), want), (h, w, c, wo, ho)
    img = rng.integers(0, 256, (15, 22, 3), dtype=np.uint8)
    assert np.array_equal(oracle.resize_lanczos4(img, 22, 15), img)
    f = rng.standard_normal((15, 22, 3)).astype(np.float32)
    assert np.array_equal(oracle.resize_lanczos4(f, 22, 15), f)
