"""GPU parity: every operator through the C ABI against the oracle.

Bar (DESIGN.md "Parity"): integer / byte / index outputs are bit-exact;
fp32 outputs are value-exact (the kernels perform the reference's IEEE
operations in the reference's order; the only permitted difference is the
sign of an exact zero where a zero-weight tap row is skipped instead of
multiplied by 0).  Statistics are compared with the tolerances written next
to each assert.
"""
from __future__ import annotations

import hashlib

import numpy as np
import pytest

from conftest import load_bgr
from oracle import synthetic_image

pytestmark = pytest.mark.gpu

MEAN = np.array([103.94, 116.78, 123.68], np.float32)
STD = np.array([57.375, 57.12, 58.395], np.float32)


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.fixture(scope="module")
def ops(hip_device):
    from vacv_amd import ops
    return ops


@pytest.fixture(scope="module")
def dev(hip_device):
    return hip_device


def to_dev(a, dev):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def host(t):
    import torch
    torch.cuda.synchronize()
    return t.cpu().numpy()


def assert_same(got, want, what=""):
    assert got.shape == want.shape, (what, got.shape, want.shape)
    assert got.dtype == want.dtype, (what, got.dtype, want.dtype)
    if got.dtype.kind == "f":
        bad = ~((got == want) | (np.isnan(got) & np.isnan(want)))
        assert not bad.any(), f"{what}: {bad.sum()} of {bad.size} differ, max |d| {np.nanmax(np.abs(got - want))}"
    else:
        bad = got != want
        assert not bad.any(), f"{what}: {bad.sum()} of {bad.size} differ"


def batch(images):
    return np.stack(images)


# ---------------------------------------------------------------------------
# resize

SIZES = [((23, 37), 1), ((48, 64), 3), ((61, 97), 3), ((5, 7), 3), ((16, 16), 4), ((144, 176), 3), ((2, 2), 1)]
OUTS = [(20, 11), (33, 29), (111, 40), (7, 5), (2, 2), (160, 90), (1, 1), (300, 7)]


@pytest.mark.parametrize("direct", [1, 2, 3])
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_resize_linear_u8_hwc(ops, dev, oracle, mode, direct):
    # direct 1: the default dispatch (gather kernel for one-tap-row
    # geometries, staged kernel otherwise); 2: the gather kernel everywhere;
    # 3: the column-strip kernel for two-tap geometries it applies to
    with ops.tuning(RESIZE_DIRECT=min(direct, 2), RESIZE_STRIP=1 if direct == 3 else 0):
        _resize_linear_u8_hwc(ops, dev, oracle, mode)


def _resize_linear_u8_hwc(ops, dev, oracle, mode):
    for i, ((h, w), c) in enumerate(SIZES):
        imgs = [synthetic_image(100 * i + k, h, w, c) for k in range(3)]
        src = to_dev(batch(imgs) if c > 1 else batch(imgs)[..., None], dev)
        for wo, ho in OUTS:
            out = host(ops.resize(src, wo, ho, mode=mode))
            for k in range(3):
                want = oracle.resize_linear(imgs[k], wo, ho, mode=mode)
                got = out[k] if c > 1 else out[k, ..., 0]
                assert_same(got, want, f"u8 mode{mode} {h}x{w}x{c}->{ho}x{wo}")


def test_resize_linear_chw_and_fp32(ops, dev, oracle):
    from vacv_amd import NCHW
    rng = np.random.default_rng(7)
    for i, ((h, w), c) in enumerate(SIZES):
        img = synthetic_image(7 + i, h, w, c)
        img = img if c > 1 else img[..., None]
        chw = np.ascontiguousarray(img.transpose(2, 0, 1))
        f = (img.astype(np.float32) + rng.standard_normal(img.shape).astype(np.float32)).astype(np.float32)
        for wo, ho in OUTS:
            out = host(ops.resize(to_dev(chw[None], dev), wo, ho, layout=NCHW))[0]
            for k in range(c):
                assert_same(out[k], oracle.resize_linear(chw[k], wo, ho), f"chw {h}x{w} k{k}")
            outf = host(ops.resize(to_dev(f[None], dev), wo, ho))[0]
            wantf = oracle.resize_linear(f if c > 1 else f[..., 0], wo, ho)
            assert_same(outf if c > 1 else outf[..., 0], wantf, f"f32 {h}x{w}x{c}->{ho}x{wo}")


def test_resize_cubic(ops, dev, oracle):
    from vacv_amd import INTER_CUBIC, NCHW
    rng = np.random.default_rng(11)
    for i, ((h, w), c) in enumerate(SIZES):
        if h < 4 or w < 4:
            continue
        img = synthetic_image(50 + i, h, w, c)
        img = img if c > 1 else img[..., None]
        f = (img.astype(np.float32) * np.float32(0.5) + rng.standard_normal(img.shape).astype(np.float32) * 4).astype(np.float32)
        for wo, ho in OUTS + [(224, 224)]:
            got = host(ops.resize(to_dev(f[None], dev), wo, ho, interpolation=INTER_CUBIC))[0]
            want = oracle.resize_cubic(f if c > 1 else f[..., 0], wo, ho)
            assert_same(got if c > 1 else got[..., 0], want, f"cubic f32 {h}x{w}x{c}->{ho}x{wo}")
            # u8 input: the u8 -> fp32 conversion the reference needs first, fused
            got8 = host(ops.resize(to_dev(img[None], dev), wo, ho, interpolation=INTER_CUBIC))[0]
            want8 = oracle.resize_cubic(oracle.u8_to_f32(img if c > 1 else img[..., 0]), wo, ho)
            assert_same(got8 if c > 1 else got8[..., 0], want8, f"cubic u8 {h}x{w}x{c}->{ho}x{wo}")
        chw = np.ascontiguousarray(f.transpose(2, 0, 1))
        got = host(ops.resize(to_dev(chw[None], dev), 31, 17, interpolation=INTER_CUBIC, layout=NCHW))[0]
        for k in range(c):
            assert_same(got[k], oracle.resize_cubic(chw[k], 31, 17), "cubic chw")


def test_cubic_direct_and_staged_agree(ops, dev, oracle):
    """u8 cubic runs on the per-pixel gather kernel (k_cubic_direct.hip) unless
    VACV_TUNE_CUBIC_DIRECT = 0 selects the staged kernel (k_resize.hip).  Both are
    the reference's arithmetic, so they agree bit for bit: BASELINE cfg5 at
    full size (2560x1440 -> 224x224, batch 6), normalized, a pitched source,
    NCHW planes and an upscale; image 0 is also checked against the oracle."""
    import torch
    from vacv_amd import INTER_CUBIC, NCHW
    imgs = np.stack([synthetic_image(90 + k, 1440, 2560, 3) for k in range(6)])
    src = to_dev(imgs, dev)
    big = torch.zeros((2, 1450, 2600, 3), dtype=torch.uint8, device=dev)
    big[:, 3:1443, 7:2567] = src[:2]
    view = big[:, 3:1443, 7:2567]
    # black frames with sparse white lines: exact zeros next to negative lobes,
    # for the rows the direct kernel does not read (weight 0) -- compared as bits
    stripes = np.zeros((2, 1440, 2560, 3), np.uint8)
    stripes[:, ::37] = 255
    stripes[:, :, ::53] = 255
    sdev = to_dev(stripes, dev)
    cases = [lambda: ops.resize(src, 224, 224, interpolation=INTER_CUBIC),
             lambda: ops.resize(sdev, 224, 224, interpolation=INTER_CUBIC),
             lambda: ops.resize_normalize(src, 224, 224, MEAN, STD, interpolation=INTER_CUBIC),
             lambda: ops.resize(view, 300, 171, interpolation=INTER_CUBIC),
             lambda: ops.resize(src[:1, :100, :90], 250, 333, interpolation=INTER_CUBIC),
             lambda: ops.resize(ops.change_layout(src[:2], NCHW), 97, 61, interpolation=INTER_CUBIC, layout=NCHW)]
    for i, fn in enumerate(cases):
        with ops.tuning(CUBIC_DIRECT=0):
            b = fn()
        # 1: the column kernel where it applies; 2: the row-major gather kernel
        # (its non-SUMS instances, kOutNorm included, exchange through LDS)
        for knob in (1, 2):
            with ops.tuning(CUBIC_DIRECT=knob):
                a = fn()
            torch.cuda.synchronize(dev)
            assert torch.equal(a.view(torch.int32), b.view(torch.int32)), \
                f"case {i}, CUBIC_DIRECT={knob}: {(a != b).sum().item()} values differ"
    got = host(ops.resize(src[:1], 224, 224, interpolation=INTER_CUBIC))[0]
    assert_same(got, oracle.resize_cubic(oracle.u8_to_f32(imgs[0]), 224, 224), "cfg5 image 0 vs oracle")
    got = host(ops.resize(sdev[:1], 224, 224, interpolation=INTER_CUBIC))[0]
    want = oracle.resize_cubic(oracle.u8_to_f32(stripes[0]), 224, 224)
    assert np.array_equal(got.view(np.uint32), np.asarray(want, np.float32).view(np.uint32)), "stripes vs oracle, bitwise"
    del src, big, sdev
    torch.cuda.empty_cache()


def test_resize_channel_sums(ops, dev, oracle):
    """vacv_resize_channel_sums / vacv_resize_mean_stddev: the resize output is
    unchanged and the sums match vacv_channel_sums of that output.  u8 -> fp32
    cubic (cfg5) fuses the sums into the cubic kernel: the column kernel adds
    fp64 per lane, wave and workgroup, then into per-image fixed-point int64
    accumulators (atomics: integer sums, order-free) that one small launch
    converts; the gather kernel (16-byte unaligned destination rows) adds fp32
    over <= 2 pixels per lane and reduces the per-workgroup partials in a
    fixed order.  Within 1e-6 relative of the fp64 sums, the derived mean /
    stddev within SURVEY 8(c)'s |d mean| <= 1e-3 and |d std| / std <= 1e-4 of
    the oracle's exact statistics, and bit-identical run to run (whatever
    order the workgroups finish in).  The batch statistic of cfg5 (2560x1440 -> 224x224 cubic) at full
    size, plus odd sizes with partial column blocks / row groups / waves."""
    import torch
    from vacv_amd import INTER_CUBIC, NCHW
    imgs = np.stack([synthetic_image(300 + k, 1440, 2560, 3) for k in range(4)])
    src = to_dev(imgs, dev)
    for per_image in (True, False):
        out, sums = ops.resize_channel_sums(src, 224, 224, INTER_CUBIC, per_image=per_image)
        _, again = ops.resize_channel_sums(src, 224, 224, INTER_CUBIC, per_image=per_image)
        ref = ops.resize(src, 224, 224, interpolation=INTER_CUBIC)
        assert torch.equal(out, ref)
        assert torch.equal(sums, again), "fused sums differ run to run"
        want = ops.channel_sums(ref, per_image=per_image)
        torch.cuda.synchronize(dev)
        rel = ((sums - want).abs() / want.abs().clamp(min=1.0)).max().item()
        assert rel <= 1e-6, rel
        count = 224 * 224 * (1 if per_image else 4)
        mean, std = ops.stats_from_sums(sums, count)
        host_out = host(ref).astype(np.float64).reshape(4, -1, 3)
        exact = host_out if per_image else host_out.reshape(1, -1, 3)
        em, es = exact.mean(axis=1), exact.std(axis=1)
        assert np.abs(host(mean) - em).max() <= 1e-3
        assert (np.abs(host(std) - es) / es).max() <= 1e-4
        # vacv_resize_mean_stddev (the one-GPU cfg5 call): the same sums, and the
        # statistics its reduction launch derives equal vacv_stats_from_sums'
        out2, sums2, mean2, std2 = ops.resize_mean_stddev(src, 224, 224, INTER_CUBIC, per_image=per_image)
        assert torch.equal(out2, ref) and torch.equal(sums2, sums)
        assert torch.equal(mean2, mean) and torch.equal(std2, std)
        for _ in range(8):  # the atomic accumulation: same bits whatever the finishing order
            _, s3, m3, d3 = ops.resize_mean_stddev(src, 224, 224, INTER_CUBIC, per_image=per_image)
            assert torch.equal(s3, sums) and torch.equal(m3, mean) and torch.equal(d3, std)
    odd = to_dev(np.stack([synthetic_image(310 + k, 301, 257, 3) for k in range(3)]), dev)
    # 61 x 37: 732-byte output rows -> the gather kernel (5 workgroups, the
    # last one partial); 68 x 37: 816-byte rows -> the column kernel (a
    # 4-column last block, a 1-row last row group)
    for ow, oh in ((61, 37), (68, 37)):
        out, sums = ops.resize_channel_sums(odd, ow, oh, INTER_CUBIC, per_image=True)
        assert torch.equal(out, ops.resize(odd, ow, oh, interpolation=INTER_CUBIC))
        want = ops.channel_sums(out)
        torch.cuda.synchronize(dev)
        assert ((sums - want).abs() / want.abs().clamp(min=1.0)).max().item() <= 1e-6
        for per_image in (True, False):
            _, s2, m2, d2 = ops.resize_mean_stddev(odd, ow, oh, INTER_CUBIC, per_image=per_image)
            count = ow * oh * (1 if per_image else 3)
            want = ops.channel_sums(out, per_image=per_image)
            wm, wd = ops.stats_from_sums(want, count)
            torch.cuda.synchronize(dev)
            assert ((s2 - want).abs() / want.abs().clamp(min=1.0)).max().item() <= 1e-6
            assert (m2 - wm).abs().max().item() <= 1e-3 and ((d2 - wd).abs() / wd).max().item() <= 1e-4
    # NCHW planes and odd sizes
    chw = ops.change_layout(src[:2, :301, :257].contiguous(), NCHW)
    out, sums = ops.resize_channel_sums(chw, 61, 37, INTER_CUBIC, layout=NCHW)
    want = ops.channel_sums(out, layout=NCHW)
    torch.cuda.synchronize(dev)
    assert ((sums - want).abs() / want.abs().clamp(min=1.0)).max().item() <= 1e-12
    # u8 bilinear: identical to the two calls (three with the statistics)
    out, sums = ops.resize_channel_sums(src, 640, 360)
    assert torch.equal(out, ops.resize(src, 640, 360))
    assert torch.equal(sums, ops.channel_sums(out))
    _, s2, m2, d2 = ops.resize_mean_stddev(src, 640, 360, per_image=True)
    wm, wd = ops.stats_from_sums(sums, 640 * 360)
    assert torch.equal(s2, sums) and torch.equal(m2, wm) and torch.equal(d2, wd)
    del src
    torch.cuda.empty_cache()


def test_resize_mean_stddev_random_geometry(ops, dev, oracle):
    """cfg5's fused call at seeded random geometries (u8 -> fp32 cubic, 1-4
    channels, batches of 3, per-image and batch statistics): the image equals
    the oracle's cubic resize bit for bit, the fused sums are within 1e-6
    relative of vacv_channel_sums of that output, the statistics within
    SURVEY 8(c)'s bounds of the exact fp64 ones, and a repeat gives the same
    bits (fixed-point accumulators)."""
    import torch
    from vacv_amd import INTER_CUBIC
    rng = np.random.default_rng(20260422)
    for t in range(12):
        c = 1 + t % 4
        h, w = int(rng.integers(8, 900)), int(rng.integers(8, 1500))
        ho, wo = int(rng.integers(4, 300)), int(rng.integers(4, 300))
        per_image = t % 3 != 2
        imgs = np.stack([synthetic_image(6000 + 3 * t + k, h, w, c).reshape(h, w, c) for k in range(3)])
        src = to_dev(imgs, dev)
        out, sums, mean, std = ops.resize_mean_stddev(src, wo, ho, INTER_CUBIC, per_image=per_image)
        _, s2, m2, d2 = ops.resize_mean_stddev(src, wo, ho, INTER_CUBIC, per_image=per_image)
        want = ops.channel_sums(out, per_image=per_image)
        torch.cuda.synchronize(dev)
        what = f"{w}x{h}x{c} -> {wo}x{ho} per_image={per_image}"
        assert torch.equal(s2, sums) and torch.equal(m2, mean) and torch.equal(d2, std), what + " repeat"
        assert ((sums - want).abs() / want.abs().clamp(min=1.0)).max().item() <= 1e-6, what
        ho_ = host(out)
        for k in range(3):
            r = oracle.resize_cubic(oracle.u8_to_f32(imgs[k] if c > 1 else imgs[k][..., 0]), wo, ho)
            assert_same(ho_[k].reshape(ho, wo, c), r.reshape(ho, wo, c), what + " image")
        ex = ho_.astype(np.float64).reshape(3, -1, c)
        ex = ex if per_image else ex.reshape(1, -1, c)
        em, es = ex.mean(axis=1), ex.std(axis=1)
        assert np.abs(host(mean).reshape(em.shape) - em).max() <= 1e-3, what
        assert (np.abs(host(std).reshape(es.shape) - es) / np.maximum(es, 1e-6)).max() <= 1e-4, what


def test_resize_nearest(ops, dev, oracle):
    """INTER_NEAREST (OpenCV 2.4 resizeNN semantics, parity unpinned -- see
    oracle/vacv_oracle.c): u8 and fp32, NHWC c = 1..4 and NCHW, down- and
    upscales, same size (a copy), the normalize epilogue, a pitched source."""
    import torch
    from vacv_amd import INTER_NEAREST, NCHW
    rng = np.random.default_rng(31)
    for i, ((h, w), c) in enumerate(SIZES + [((1080, 1920), 3)]):
        img = synthetic_image(600 + i, h, w, c)
        img = img if c > 1 else img[..., None]
        f = (img.astype(np.float32) + rng.standard_normal(img.shape).astype(np.float32)).astype(np.float32)
        for wo, ho in OUTS + [(w, h), (640, 360), (3 * w, 2 * h)]:
            sq = (lambda a: a) if c > 1 else (lambda a: a[..., 0])
            got = host(ops.resize(to_dev(img[None], dev), wo, ho, interpolation=INTER_NEAREST))[0]
            assert_same(sq(got), oracle.resize_nearest(sq(img), wo, ho), f"nearest u8 {h}x{w}x{c}->{ho}x{wo}")
            gotf = host(ops.resize(to_dev(f[None], dev), wo, ho, interpolation=INTER_NEAREST))[0]
            assert_same(sq(gotf), oracle.resize_nearest(sq(f), wo, ho), f"nearest f32 {h}x{w}x{c}->{ho}x{wo}")
        chw = np.ascontiguousarray(img.transpose(2, 0, 1))
        got = host(ops.resize(to_dev(chw[None], dev), 33, 21, interpolation=INTER_NEAREST, layout=NCHW))[0]
        for k in range(c):
            assert_same(got[k], oracle.resize_nearest(chw[k], 33, 21), "nearest chw")
        if c == 3:
            got = host(ops.resize_normalize(to_dev(img[None], dev), 50, 40, MEAN, STD, interpolation=INTER_NEAREST))[0]
            want = oracle.normalize(oracle.u8_to_f32(oracle.resize_nearest(img, 50, 40)), MEAN, STD)
            assert_same(got, want, "nearest normalize")
    big = torch.zeros((1, 80, 90, 3), dtype=torch.uint8, device=dev)
    img = synthetic_image(5, 61, 77, 3)
    big[0, 7:68, 3:80] = to_dev(img, dev)
    got = host(ops.resize(big[:, 7:68, 3:80], 30, 20, interpolation=INTER_NEAREST))[0]
    assert_same(got, oracle.resize_nearest(img, 30, 20), "nearest pitched")


def test_nearest_area_kernel_variants_agree(ops, dev, oracle):
    """Every INTER_NEAREST / u8 INTER_AREA kernel variant gives the same bytes
    at BASELINE's 1080p frame: nearest row-staged per wave (default where the
    source is 16-byte aligned, its row fits 16 KiB and the sample stride is
    short) vs row-staged per workgroup (VACV_TUNE_NEAREST_KERNEL = 1) vs the
    per-pixel kernel (0); area 16-byte column
    units (default) vs 16-byte LDS column sums (3) vs dword column sums (2) vs
    per-pixel (1); plus an fp32 row
    past 64 KiB (5600 px x 3 ch: the per-pixel fallback) and a strong
    horizontal downscale (wide stride: the per-pixel kernel) vs the oracle."""
    import torch
    from vacv_amd import INTER_AREA, INTER_NEAREST
    imgs = np.stack([synthetic_image(750 + k, 1080, 1920, 3) for k in range(2)])
    src = to_dev(imgs, dev)
    for wo, ho in [(640, 360), (960, 540), (1280, 720), (3000, 1500)]:
        a = ops.resize(src, wo, ho, interpolation=INTER_NEAREST)
        for knob in (1, 0):  # row per workgroup, per-pixel (default: row per wave)
            with ops.tuning(NEAREST_KERNEL=knob):
                b = ops.resize(src, wo, ho, interpolation=INTER_NEAREST)
            assert torch.equal(a, b), f"nearest variant {knob} differs -> {wo}x{ho}"
        if wo <= 1920:
            an = ops.resize_normalize(src, wo, ho, MEAN, STD, interpolation=INTER_NEAREST)
            for knob in (1, 0):
                with ops.tuning(NEAREST_KERNEL=knob):
                    bn = ops.resize_normalize(src, wo, ho, MEAN, STD, interpolation=INTER_NEAREST)
                assert torch.equal(an, bn), f"nearest normalize variant {knob} differs -> {wo}x{ho}"
    assert_same(host(a)[1], oracle.resize_nearest(imgs[1], 3000, 1500), "nearest upscale")
    for wo, ho in [(640, 360), (960, 540), (480, 270)]:
        a = ops.resize(src, wo, ho, interpolation=INTER_AREA)
        for knob in (1, 2, 3):
            with ops.tuning(AREA_KERNEL=knob):
                b = ops.resize(src, wo, ho, interpolation=INTER_AREA)
            assert torch.equal(a, b), f"area variant {knob} differs -> {wo}x{ho}"
        assert_same(host(a)[0], oracle.resize_area(imgs[0], wo, ho), f"area 1080p -> {wo}x{ho}")
    wide = synthetic_image(760, 9, 5600, 3).astype(np.float32) + 0.25
    got = host(ops.resize(to_dev(wide[None], dev), 700, 4, interpolation=INTER_NEAREST))[0]
    assert_same(got, oracle.resize_nearest(wide, 700, 4), "nearest fp32 row > 64 KiB")
    strided = synthetic_image(761, 40, 4096, 3).astype(np.float32)
    got = host(ops.resize(to_dev(strided[None], dev), 32, 20, interpolation=INTER_NEAREST))[0]
    assert_same(got, oracle.resize_nearest(strided, 32, 20), "nearest 128x horizontal downscale")


def test_resize_area(ops, dev, oracle):
    """INTER_AREA at integer downscales (OpenCV 2.4 resizeAreaFast_, parity
    unpinned -- see oracle/vacv_oracle.c): u8 (half-to-even rounding; 2x2
    blocks of 1/3/4 channels half up, ResizeAreaFastVec's fast_mode) and fp32
    (OpenCV's four-tap summation order, bit-exact), NHWC c = 1..4 and NCHW,
    block sizes 1x1 .. 7x5 incl. areas that are not a multiple of 4, the
    widen / normalize epilogues, a pitched source, and BASELINE's 1080p frame
    at 1/2 and 1/3."""
    import torch
    from vacv_amd import INTER_AREA, NCHW
    rng = np.random.default_rng(37)
    for i, ((h, w), c) in enumerate([((60, 84), 1), ((60, 84), 2), ((60, 84), 3), ((60, 84), 4),
                                     ((1080, 1920), 3)]):
        img = synthetic_image(700 + i, h, w, c)
        img = img if c > 1 else img[..., None]
        f = (img.astype(np.float32) + rng.standard_normal(img.shape).astype(np.float32)).astype(np.float32)
        sq = (lambda a: a) if c > 1 else (lambda a: a[..., 0])
        blocks = [(2, 2), (3, 3)] if h == 1080 else [(1, 1), (2, 2), (3, 2), (4, 4), (7, 5), (6, 3), (12, 1)]
        for ax, ay in blocks:
            wo, ho = w // ax, h // ay
            got = host(ops.resize(to_dev(img[None], dev), wo, ho, interpolation=INTER_AREA))[0]
            assert_same(sq(got), oracle.resize_area(sq(img), wo, ho), f"area u8 {h}x{w}x{c}/{ax}x{ay}")
            gotf = host(ops.resize(to_dev(f[None], dev), wo, ho, interpolation=INTER_AREA))[0]
            assert_same(sq(gotf), oracle.resize_area(sq(f), wo, ho), f"area f32 {h}x{w}x{c}/{ax}x{ay}")
        if c == 3:
            chw = np.ascontiguousarray(img.transpose(2, 0, 1))
            got = host(ops.resize(to_dev(chw[None], dev), w // 3, h // 2, interpolation=INTER_AREA, layout=NCHW))[0]
            for k in range(c):
                assert_same(got[k], oracle.resize_area(chw[k], w // 3, h // 2), "area chw")
            got = host(ops.resize(to_dev(chw[None], dev), w // 2, h // 2, interpolation=INTER_AREA, layout=NCHW))[0]
            for k in range(c):  # NCHW planes are 1-channel: the 2x2 fast_mode rounding
                assert_same(got[k], oracle.resize_area(chw[k], w // 2, h // 2), "area chw 2x2")
            got = host(ops.resize_normalize(to_dev(img[None], dev), w // 2, h // 2, MEAN, STD,
                                            interpolation=INTER_AREA))[0]
            want = oracle.normalize(oracle.u8_to_f32(oracle.resize_area(img, w // 2, h // 2)), MEAN, STD)
            assert_same(got, want, "area normalize")
    big = torch.zeros((1, 80, 90, 3), dtype=torch.uint8, device=dev)
    img = synthetic_image(6, 60, 78, 3)
    big[0, 7:67, 3:81] = to_dev(img, dev)
    got = host(ops.resize(big[:, 7:67, 3:81], 26, 20, interpolation=INTER_AREA))[0]
    assert_same(got, oracle.resize_area(img, 26, 20), "area pitched")
    # 2x2 ties: block sums 4k + 2 round half UP for 1/3/4 channels
    # (ResizeAreaFastVec fast_mode) and half to even for 2 (generic path)
    for c in (1, 2, 3, 4):
        blk = np.zeros((2, 8, c), np.uint8)
        for j, sm in enumerate([2, 6, 10, 14]):
            q = [sm // 4 + (1 if t < sm % 4 else 0) for t in range(4)]
            blk[0, 2 * j], blk[0, 2 * j + 1], blk[1, 2 * j], blk[1, 2 * j + 1] = q
        got = host(ops.resize(to_dev(blk[None], dev), 4, 1, interpolation=INTER_AREA))[0]
        want = [1, 2, 3, 4] if c != 2 else [0, 2, 2, 4]
        assert got.reshape(4, c)[:, 0].tolist() == want, (c, got)
        big = np.tile(blk, (64, 96, 1))  # the column-sum kernel (16-byte aligned rows)
        got = host(ops.resize(to_dev(big[None], dev), 384, 64, interpolation=INTER_AREA))[0]
        assert_same(got.reshape(64, 384, c), oracle.resize_area(big, 384, 64).reshape(64, 384, c), f"area tie c{c}")


def test_area_unit_kernel(ops, dev, oracle):
    """The streaming u8 INTER_AREA kernels (area_u8_unit_kernel, k_pixel.hip:
    16-byte aligned rows, AX in {2, 4} with 1-4 channels, AX = 3 with one;
    area_lane_kernel: AX = 3 with 3 or 4 channels):
    bit-exact against the oracle and against the LDS column-sum kernel
    (VACV_TUNE_AREA_KERNEL = 3) for every instance, with row pitches padded
    so that a row's last unit is partial (and, on the last row, its chunks
    reach past the plane's end), u8 / fp32 / normalised output, NCHW planes
    and a destination that forbids the vector stores."""
    import torch
    from vacv_amd import INTER_AREA, NCHW
    # (3, *, 3) and (3, *, 4): area_lane_kernel (whole source dwords per lane;
    # 300-pixel rows take its 16-byte loads, the others its dword loads)
    cases = [(2, 2, 1), (2, 2, 2), (2, 2, 3), (2, 2, 4), (3, 3, 1), (3, 1, 1), (4, 4, 1), (4, 2, 2), (4, 4, 3),
             (4, 3, 4), (2, 3, 3), (2, 5, 1), (3, 3, 3), (3, 3, 4), (3, 2, 3), (3, 4, 4)]
    for i, (ax, ay, c) in enumerate(cases):
        for wo, ho in [(37, 11), (64, 9)] + ([(300, 5), (1027, 3)] if ax == 3 and c >= 3 else []):
            w, h = wo * ax, ho * ay
            pitch = -(-(w * c + 1) // 16) * 16  # 16-byte rows, padded
            imgs = [synthetic_image(790 + 10 * i + k, h, w, c).reshape(h, w, c) for k in range(2)]
            flat = np.zeros(2 * h * pitch, np.uint8)
            for k in range(2):
                for y in range(h):
                    o = (k * h + y) * pitch
                    flat[o:o + w * c] = imgs[k][y].reshape(-1)
            view = to_dev(flat, dev).as_strided((2, h, w, c), (h * pitch, pitch, c, 1))
            got = ops.resize(view, wo, ho, interpolation=INTER_AREA)
            gh = host(got)
            for k in range(2):
                want = oracle.resize_area(imgs[k] if c > 1 else imgs[k][..., 0], wo, ho)
                assert_same(gh[k].reshape(want.shape), want, f"area unit {ax}x{ay} c{c} -> {wo}x{ho}")
            with ops.tuning(AREA_KERNEL=3):
                ref = ops.resize(view, wo, ho, interpolation=INTER_AREA)
                refn = ops.resize_normalize(view, wo, ho, MEAN[:c], STD[:c], interpolation=INTER_AREA) if c in (1, 3) else None
            assert torch.equal(got, ref), f"unit vs colsum {ax}x{ay} c{c}"
            if refn is not None:
                gotn = ops.resize_normalize(view, wo, ho, MEAN[:c], STD[:c], interpolation=INTER_AREA)
                assert torch.equal(gotn, refn), f"unit vs colsum normalize {ax}x{ay} c{c}"
            # a destination at an odd offset: element-wise stores
            out = torch.zeros((2, ho, wo + 1, c), dtype=torch.uint8, device=dev)[:, :, 1:]
            ops.resize(view, wo, ho, interpolation=INTER_AREA, out=out)
            assert torch.equal(out, ref), f"unit unaligned dst {ax}x{ay} c{c}"
    img = synthetic_image(799, 64, 96, 3)
    chw = to_dev(np.ascontiguousarray(img.transpose(2, 0, 1))[None], dev)
    got = host(ops.resize(chw, 48, 32, interpolation=INTER_AREA, layout=NCHW))[0]
    for k in range(3):
        assert_same(got[k], oracle.resize_area(np.ascontiguousarray(img[..., k]), 48, 32), "area unit chw")


def test_resize_lanczos4(ops, dev, oracle):
    """INTER_LANCZOS4 (k_lanczos.hip; the reference hands it to cv::resize,
    resize.cpp:46-48, cv.h:33): bit-exact against the oracle's OpenCV 2.4
    restatement (parity unpinned) for u8 and fp32, 1-4 channels, down- and
    up-scales, NCHW planes, the normalise epilogue, and cv::resize's fx / fy
    form."""
    import torch
    from vacv_amd import INTER_LANCZOS4, NCHW
    rng = np.random.default_rng(41)
    for i, ((h, w), c) in enumerate([((60, 84), 1), ((45, 70), 2), ((64, 96), 3), ((33, 50), 4)]):
        img = synthetic_image(820 + i, h, w, c)
        img = img if c > 1 else img[..., None]
        f = (img.astype(np.float32) + rng.standard_normal(img.shape).astype(np.float32)).astype(np.float32)
        sq = (lambda a: a) if c > 1 else (lambda a: a[..., 0])
        for wo, ho in [(w // 3, h // 2), (w * 2 + 1, h + 7), (w - 1, h * 3)]:
            got = host(ops.resize(to_dev(img[None], dev), wo, ho, interpolation=INTER_LANCZOS4))[0]
            assert_same(sq(got), oracle.resize_lanczos4(sq(img), wo, ho), f"lanczos u8 {h}x{w}x{c}->{ho}x{wo}")
            gotf = host(ops.resize(to_dev(f[None], dev), wo, ho, interpolation=INTER_LANCZOS4))[0]
            assert_same(sq(gotf), oracle.resize_lanczos4(sq(f), wo, ho), f"lanczos f32 {h}x{w}x{c}->{ho}x{wo}")
        if c == 3:
            chw = np.ascontiguousarray(img.transpose(2, 0, 1))
            got = host(ops.resize(to_dev(chw[None], dev), 41, 37, interpolation=INTER_LANCZOS4, layout=NCHW))[0]
            for k in range(c):
                assert_same(got[k], oracle.resize_lanczos4(chw[k], 41, 37), "lanczos chw")
            got = host(ops.resize_normalize(to_dev(img[None], dev), 50, 30, MEAN, STD, interpolation=INTER_LANCZOS4))[0]
            want = oracle.normalize(oracle.u8_to_f32(oracle.resize_lanczos4(img, 50, 30)), MEAN, STD)
            assert_same(got, want, "lanczos normalize")
            got = host(ops.resize(to_dev(img[None], dev), 0, 0, interpolation=INTER_LANCZOS4, fx=0.7, fy=0.45))[0]
            wo, ho = int(round(w * 0.7)), int(round(h * 0.45))
            assert_same(got, oracle.resize_lanczos4(img, wo, ho, 0.7, 0.45), "lanczos fx/fy")
    # sources narrower than the 8-pixel row window (lanczos_small_kernel):
    # every column is a border column of HResizeLanczos4
    for i, (h, w, c) in enumerate([(20, 5, 3), (9, 7, 1), (13, 4, 4), (6, 6, 2)]):
        img = synthetic_image(840 + i, h, w, c)
        img = img if c > 1 else img[..., None]
        f = (img.astype(np.float32) + rng.standard_normal(img.shape).astype(np.float32)).astype(np.float32)
        sq = (lambda a: a) if c > 1 else (lambda a: a[..., 0])
        for wo, ho in [(3, 11), (17, 5), (w + 1, h - 1)]:
            got = host(ops.resize(to_dev(img[None], dev), wo, ho, interpolation=INTER_LANCZOS4))[0]
            assert_same(sq(got), oracle.resize_lanczos4(sq(img), wo, ho), f"lanczos u8 narrow {h}x{w}x{c}->{ho}x{wo}")
            gotf = host(ops.resize(to_dev(f[None], dev), wo, ho, interpolation=INTER_LANCZOS4))[0]
            assert_same(sq(gotf), oracle.resize_lanczos4(sq(f), wo, ho), f"lanczos f32 narrow {h}x{w}x{c}->{ho}x{wo}")
        if c == 3:
            got = host(ops.resize_normalize(to_dev(img[None], dev), 9, 14, MEAN, STD, interpolation=INTER_LANCZOS4))[0]
            want = oracle.normalize(oracle.u8_to_f32(oracle.resize_lanczos4(img, 9, 14)), MEAN, STD)
            assert_same(got, want, "lanczos normalize narrow")
    big = np.stack([synthetic_image(830 + k, 1080, 1920, 3) for k in range(2)])
    got = host(ops.resize(to_dev(big, dev), 640, 360, interpolation=INTER_LANCZOS4))
    assert_same(got[1], oracle.resize_lanczos4(big[1], 640, 360), "lanczos 1080p -> 640x360")
    # u8: the register-ring kernel (default: staged source runs, 1 or 2 KiB
    # per wave row -- 3x and 10x downscales, an upscale) against the LDS-ring
    # kernel (LANCZOS_KERNEL=1) and its own per-lane windows (=2) on batches
    # of 1, 5 and 64 frames -- different band heights, so different
    # band-relative coefficient tables -- and on all three output types; the
    # oracle pins one frame of each
    src = to_dev(np.stack([synthetic_image(850 + k, 270, 481, 3) for k in range(64)]), dev)
    for n in (1, 5, 64):
        for wo, ho in [(160, 90), (333, 401), (48, 30)]:
            calls = [lambda: ops.resize(src[:n], wo, ho, interpolation=INTER_LANCZOS4),
                     lambda: ops.resize_normalize(src[:n], wo, ho, MEAN, STD, interpolation=INTER_LANCZOS4)]
            for j, fn in enumerate(calls):
                a = fn()
                for knob in (1, 2):
                    with ops.tuning(LANCZOS_KERNEL=knob):
                        b = fn()
                    torch.cuda.synchronize(dev)
                    assert torch.equal(a.view(torch.uint8), b.view(torch.uint8)), \
                        f"lanczos kernels differ n={n} {wo}x{ho} call {j} LANCZOS_KERNEL={knob}"
            k = n - 1
            full = host(ops.resize(src[:n], wo, ho, interpolation=INTER_LANCZOS4))
            assert_same(full[k], oracle.resize_lanczos4(host(src[k]), wo, ho), f"lanczos batch n={n} {wo}x{ho}")
    # the cached tables' staged-run count depends on the channel count: the
    # same geometry on 1-channel planes, then 3- and 4-channel pixels (6x and
    # 10x downscales, where cc = 1 needs fewer loads per lane than cc >= 3)
    for wo, ho in [(320, 60), (192, 36)]:
        for c, layout in [(3, NCHW), (3, None), (4, None), (1, None)]:
            img = synthetic_image(870 + c, 360, 1920, c)
            img = img if c > 1 else img[..., None]
            t = to_dev((np.ascontiguousarray(img.transpose(2, 0, 1)) if layout == NCHW else img)[None], dev)
            kw = dict(interpolation=INTER_LANCZOS4, **({"layout": NCHW} if layout == NCHW else {}))
            a = ops.resize(t, wo, ho, **kw)
            with ops.tuning(LANCZOS_KERNEL=1):
                b = ops.resize(t, wo, ho, **kw)
            torch.cuda.synchronize(dev)
            assert torch.equal(a, b), f"lanczos cc={c} layout={layout} {wo}x{ho} after another channel count"


def test_resize_area_any_scale(ops, dev, oracle):
    """INTER_AREA at non-integer scales (OpenCV 2.4 cv::resize restated,
    parity unpinned -- oracle/vacv_oracle.c oracle_resize_area_any):
    resizeArea_ weight tables for down-scales, the area-mode bilinear for
    up-scales and mixed scales; u8 and fp32, NHWC c = 1..4 and NCHW, the
    normalize epilogue, cv::resize's fx / fy form (dsize derived, inv_scale =
    fx), and 1080p -> 1280x720 / 800x600 at full size."""
    from vacv_amd import INTER_AREA, NCHW
    rng = np.random.default_rng(41)
    for i, c in enumerate((1, 2, 3, 4)):
        img = synthetic_image(800 + i, 60, 84, c)
        img = img if c > 1 else img[..., None]
        f = (img.astype(np.float32) + rng.standard_normal(img.shape).astype(np.float32)).astype(np.float32)
        sq = (lambda a: a) if c > 1 else (lambda a: a[..., 0])
        for wo, ho in [(33, 21), (50, 37), (83, 59), (100, 77), (30, 90), (168, 61), (84, 25)]:
            got = host(ops.resize(to_dev(img[None], dev), wo, ho, interpolation=INTER_AREA))[0]
            assert_same(sq(got), oracle.resize_area_any(sq(img), wo, ho), f"area u8 c{c} -> {wo}x{ho}")
            gotf = host(ops.resize(to_dev(f[None], dev), wo, ho, interpolation=INTER_AREA))[0]
            assert_same(sq(gotf), oracle.resize_area_any(sq(f), wo, ho), f"area f32 c{c} -> {wo}x{ho}")
    img = synthetic_image(810, 60, 84, 3)
    chw = np.ascontiguousarray(img.transpose(2, 0, 1))
    got = host(ops.resize(to_dev(chw[None], dev), 37, 26, interpolation=INTER_AREA, layout=NCHW))[0]
    for k in range(3):
        assert_same(got[k], oracle.resize_area_any(chw[k], 37, 26), "area any chw")
    got = host(ops.resize_normalize(to_dev(img[None], dev), 50, 37, MEAN, STD, interpolation=INTER_AREA))[0]
    want = oracle.normalize(oracle.u8_to_f32(oracle.resize_area_any(img, 50, 37)), MEAN, STD)
    assert_same(got, want, "area any normalize")
    for fx, fy in [(0.3, 0.7), (2.5, 1.25), (0.5, 0.5)]:
        got = host(ops.resize(to_dev(img[None], dev), 0, 0, interpolation=INTER_AREA, fx=fx, fy=fy))[0]
        wo, ho = int(round(84 * fx)), int(round(60 * fy))
        assert_same(got, oracle.resize_area_any(img, wo, ho, fx, fy), f"area fx={fx} fy={fy}")
    big = np.stack([synthetic_image(820 + k, 1080, 1920, 3) for k in range(2)])
    for wo, ho in [(1280, 720), (800, 600)]:
        got = host(ops.resize(to_dev(big, dev), wo, ho, interpolation=INTER_AREA))
        assert_same(got[1], oracle.resize_area_any(big[1], wo, ho), f"area 1080p -> {wo}x{ho}")


def test_resize_nearest_scaled(ops, dev, oracle):
    """cv::resize's fx / fy form for INTER_NEAREST: dsize = round(w * fx) and
    ifx = 1 / fx (not w_in / w_out)."""
    from vacv_amd import INTER_NEAREST
    img = synthetic_image(830, 61, 77, 3)
    for fx, fy in [(0.3, 0.7), (2.5, 1.25), (1.0 / 3, 0.6)]:
        got = host(ops.resize(to_dev(img[None], dev), 0, 0, interpolation=INTER_NEAREST, fx=fx, fy=fy))[0]
        wo, ho = int(round(77 * fx)), int(round(61 * fy))
        want = np.empty((ho, wo, 3), np.uint8)
        for y in range(ho):
            sy = min(int(np.floor(y * (1.0 / fy))), 60)
            for x in range(wo):
                want[y, x] = img[sy, min(int(np.floor(x * (1.0 / fx))), 76)]
        assert_same(got, want, f"nearest fx={fx} fy={fy}")


def test_resize_full_size_batch(ops, dev, oracle):
    """BASELINE cfg2 at full size: 1920x1080 -> 640x360 / 1280x720, batch of 3,
    plus a pitched source (a sub-window of a wider buffer)."""
    imgs = [synthetic_image(2 + k, 1080, 1920, 3) for k in range(3)]
    src = to_dev(batch(imgs), dev)
    for wo, ho in [(640, 360), (1280, 720), (224, 224), (2560, 1440)]:
        out = host(ops.resize(src, wo, ho))
        for k in range(3):
            assert_same(out[k], oracle.resize_linear(imgs[k], wo, ho), f"1080p->{wo}x{ho}")
    wide = to_dev(synthetic_image(99, 200, 300, 3), dev)
    view = wide[10:150, 20:220]  # pitched rows
    got = host(ops.resize(view, 77, 55))
    want = oracle.resize_linear(np.ascontiguousarray(synthetic_image(99, 200, 300, 3)[10:150, 20:220]), 77, 55)
    assert_same(got, want, "pitched")


def test_resize_u8_kernels_agree_and_pitched_out(ops, dev, oracle):
    """u8 bilinear with one weighted source row per output row runs on the
    per-pixel gather kernel (k_resize_direct.hip), the rest on the LDS-staged
    strip kernel; VACV_TUNE_RESIZE_DIRECT = 2 forces the gather kernel for every
    geometry and 0 the strip kernel.  Both must give identical bytes / floats
    at full size (one-tap and two-tap geometries), and the gather kernel must
    honour a pitched (sub-window) destination in every store path: 16-byte
    chunks mapped per row (row bytes a multiple of 16) and the byte
    fallback."""
    import torch
    imgs = [synthetic_image(60 + k, 1080, 1920, 3) for k in range(2)]
    src = to_dev(batch(imgs), dev)
    for wo, ho in [(640, 360), (1280, 720), (333, 129), (64, 1000)]:
        for mode in (0, 1, 2):
            with ops.tuning(RESIZE_DIRECT=2):
                a8 = ops.resize(src, wo, ho, mode=mode)
                an = ops.resize_normalize(src, wo, ho, MEAN, STD, mode=mode)
            with ops.tuning(RESIZE_DIRECT=0):
                b8 = ops.resize(src, wo, ho, mode=mode)
                bn = ops.resize_normalize(src, wo, ho, MEAN, STD, mode=mode)
            assert torch.equal(a8, b8), f"u8 kernels differ {wo}x{ho} mode {mode}"
            assert torch.equal(an, bn), f"normalize kernels differ {wo}x{ho} mode {mode}"
    small = synthetic_image(61, 97, 151, 3)
    s = to_dev(small[None], dev)
    with ops.tuning(RESIZE_DIRECT=2):
        for wo, ho, dt in [(80, 50, torch.uint8), (77, 55, torch.uint8), (64, 31, torch.float32), (41, 23, torch.float32)]:
            big = torch.zeros((1, ho + 9, wo + 24, 3), dtype=dt, device=dev)
            view = big[:, 4:4 + ho, 8:8 + wo]
            if dt == torch.uint8:
                ops.resize(s, wo, ho, out=view)
                want = oracle.resize_linear(small, wo, ho)
            else:
                ops.resize_normalize(s, wo, ho, MEAN, STD, out=view)
                want = oracle.normalize(oracle.u8_to_f32(oracle.resize_linear(small, wo, ho)), MEAN, STD)
            got = host(big)
            assert_same(got[0, 4:4 + ho, 8:8 + wo], want, f"pitched out {wo}x{ho} {dt}")
            rim = got.copy()
            rim[0, 4:4 + ho, 8:8 + wo] = 0
            assert not rim.any(), f"pitched out {wo}x{ho}: wrote outside the window"


def test_resize_strip_kernel(ops, dev, oracle):
    """Two-tap u8 bilinear on the column-strip kernel (k_resize_strip.hip,
    VACV_TUNE_RESIZE_STRIP = 1; it needs a source row pitch that is a multiple
    of 16): bit-exact against the oracle for every mode and channel count,
    down- and up-scales, odd output widths (partial lane quads, byte stores);
    at full size identical to the staged kernel for u8 / fp32 / normalised
    output, NCHW planes and a pitched destination."""
    import torch
    from vacv_amd import NCHW
    cases = [((48, 64), 3), ((16, 16), 4), ((144, 176), 3), ((61, 96), 1), ((40, 32), 2), ((97, 160), 3)]
    for i, ((h, w), c) in enumerate(cases):
        imgs = [synthetic_image(300 + 10 * i + k, h, w, c).reshape(h, w, c) for k in range(2)]
        src = to_dev(np.stack(imgs), dev)
        for wo, ho in OUTS + [(w * 2 // 3, h * 2 // 3), (w + 5, h * 3), (w - 3, h - 1)]:
            for mode in (0, 1, 2):
                wants = [oracle.resize_linear(imgs[k] if c > 1 else imgs[k][..., 0], wo, ho, mode=mode) for k in range(2)]
                for sv in (1, 2):  # 64- and 128-column strips
                    with ops.tuning(RESIZE_STRIP=sv):
                        out = host(ops.resize(src, wo, ho, mode=mode))
                    for k in range(2):
                        assert_same(out[k].reshape(wants[k].shape), wants[k], f"strip{sv} {h}x{w}x{c}->{ho}x{wo} mode {mode}")
    big = [synthetic_image(330 + k, 1080, 1920, 3) for k in range(2)]
    src = to_dev(np.stack(big), dev)
    chw = to_dev(np.ascontiguousarray(np.stack(big).transpose(0, 3, 1, 2)), dev)
    for wo, ho in [(1280, 720), (1000, 999), (333, 129)]:
        for mode in (0, 1, 2):
            res = {}
            for strip in (1, 2, 0):
                with ops.tuning(RESIZE_STRIP=strip):
                    res[strip] = (ops.resize(src, wo, ho, mode=mode),
                                  ops.resize_normalize(src, wo, ho, MEAN, STD, mode=mode),
                                  ops.resize(chw, wo, ho, mode=mode, layout=NCHW))
            for sv in (1, 2):
                for a, b in zip(res[sv], res[0]):
                    assert torch.equal(a, b), f"strip{sv} vs staged {wo}x{ho} mode {mode}"
    s1 = to_dev(big[0][None, :200, :320].copy(), dev)
    for wo, ho, dt in [(211, 150, torch.uint8), (200, 151, torch.uint8), (150, 140, torch.float32)]:
        buf = torch.zeros((1, ho + 9, wo + 23, 3), dtype=dt, device=dev)
        view = buf[:, 4:4 + ho, 7:7 + wo]
        with ops.tuning(RESIZE_STRIP=1):
            if dt == torch.uint8:
                ops.resize(s1, wo, ho, out=view)
                want = oracle.resize_linear(big[0][:200, :320].copy(), wo, ho)
            else:
                ops.resize_normalize(s1, wo, ho, MEAN, STD, out=view)
                want = oracle.normalize(oracle.u8_to_f32(oracle.resize_linear(big[0][:200, :320].copy(), wo, ho)), MEAN, STD)
        got = host(buf)
        assert_same(got[0, 4:4 + ho, 7:7 + wo], want, f"strip pitched out {wo}x{ho} {dt}")
        got[0, 4:4 + ho, 7:7 + wo] = 0
        assert not got.any(), f"strip pitched out {wo}x{ho}: wrote outside the window"


def test_resize_normalize(ops, dev, oracle):
    from vacv_amd import INTER_CUBIC
    imgs = [synthetic_image(40 + k, 1080, 1920, 3) for k in range(2)]
    src = to_dev(batch(imgs), dev)
    out = host(ops.resize_normalize(src, 640, 360, MEAN, STD))
    for k in range(2):
        want = oracle.normalize(oracle.u8_to_f32(oracle.resize_linear(imgs[k], 640, 360)), MEAN, STD)
        assert_same(out[k], want, "resize_normalize u8")
    # fp32 input, cubic, odd sizes
    f = oracle.u8_to_f32(synthetic_image(5, 61, 97, 3))
    got = host(ops.resize_normalize(to_dev(f[None], dev), 45, 33, MEAN, STD, interpolation=INTER_CUBIC))[0]
    assert_same(got, oracle.normalize(oracle.resize_cubic(f, 45, 33), MEAN, STD), "cubic normalize")
    got = host(ops.resize_normalize(to_dev(f[None], dev), 45, 33, MEAN, STD))[0]
    assert_same(got, oracle.normalize(oracle.resize_linear(f, 45, 33), MEAN, STD), "f32 linear normalize")
    # auto statistics: exact per-image stats of the resized image
    out = host(ops.resize_normalize(src, 640, 360))
    for k in range(2):
        r = oracle.resize_linear(imgs[k], 640, 360)
        m, s = oracle.mean_stddev_exact(r)
        assert_same(out[k], oracle.normalize(oracle.u8_to_f32(r), m, s), "resize_normalize auto")


def test_resize_normalize_random_geometry(ops, dev, oracle):
    """Seeded random geometries for the headline op (u8 HWC -> fp32
    normalised, resize_naive.cpp:10-68 then the normalize): down- and
    up-scales, 1-4 channels, widths that are not multiples of the column
    blocks, batches of 3 -- whichever kernel the dispatcher picks matches the
    oracle bit for bit; the plain u8 resize of the same batch too."""
    rng = np.random.default_rng(20260419)
    for t in range(16):
        c = 1 + t % 4
        h, w = int(rng.integers(9, 700)), int(rng.integers(9, 1300))
        f = rng.uniform(0.2, 1.6, 2)
        ho, wo = max(1, int(h * f[0])), max(1, int(w * f[1]))
        mu = np.concatenate([MEAN, [1.0]]).astype(np.float32)[:c]
        sd = np.concatenate([STD, [2.0]]).astype(np.float32)[:c]
        imgs = [synthetic_image(7000 + 3 * t + k, h, w, c).reshape(h, w, c) for k in range(3)]
        src = to_dev(np.stack(imgs), dev)
        out = host(ops.resize_normalize(src, wo, ho, mu, sd))
        out8 = host(ops.resize(src, wo, ho))
        for k in range(3):
            r = oracle.resize_linear(imgs[k] if c > 1 else imgs[k][..., 0], wo, ho).reshape(ho, wo, c)
            assert_same(out8[k], r, f"u8 {w}x{h}x{c} -> {wo}x{ho}")
            want = oracle.normalize(oracle.u8_to_f32(r), mu, sd).reshape(ho, wo, c)
            assert_same(out[k], want, f"normalize {w}x{h}x{c} -> {wo}x{ho}")


def test_resize_random_geometry_interpolations(ops, dev, oracle):
    """Seeded random geometries (scale 0.15-3 per axis, 1-4 channels, batches
    of 2) for INTER_NEAREST, INTER_AREA, INTER_CUBIC (u8 in, fp32 out) and
    INTER_LANCZOS4, u8 and fp32 sources: the dispatcher's pick is bit-exact
    against the oracle's OpenCV 2.4 restatements (parity unpinned, as in the
    per-mode tests above)."""
    from vacv_amd import INTER_AREA, INTER_CUBIC, INTER_LANCZOS4, INTER_NEAREST
    rng = np.random.default_rng(20260420)
    for t in range(24):
        interp = (INTER_NEAREST, INTER_AREA, INTER_CUBIC, INTER_LANCZOS4)[t % 4]
        c = 1 + (t // 4) % 4
        h, w = int(rng.integers(4, 300)), int(rng.integers(4, 500))
        f = rng.uniform(0.15, 3.0, 2)
        ho, wo = max(1, int(h * f[0])), max(1, int(w * f[1]))
        imgs = np.stack([synthetic_image(8000 + 2 * t + k, h, w, c).reshape(h, w, c) for k in range(2)])
        fl = imgs.astype(np.float32) * np.float32(0.75) + np.float32(0.125)
        got = host(ops.resize(to_dev(imgs, dev), wo, ho, interpolation=interp))
        gotf = host(ops.resize(to_dev(fl, dev), wo, ho, interpolation=interp))
        what = f"interp {interp} {w}x{h}x{c} -> {wo}x{ho}"
        for k in range(2):
            sq = (lambda a: a) if c > 1 else (lambda a: a[..., 0])
            if interp == INTER_NEAREST:
                want, wantf = oracle.resize_nearest(sq(imgs[k]), wo, ho), oracle.resize_nearest(sq(fl[k]), wo, ho)
            elif interp == INTER_AREA:
                want, wantf = oracle.resize_area_any(sq(imgs[k]), wo, ho), oracle.resize_area_any(sq(fl[k]), wo, ho)
            elif interp == INTER_CUBIC:
                want = oracle.resize_cubic(oracle.u8_to_f32(sq(imgs[k])), wo, ho)
                wantf = oracle.resize_cubic(sq(fl[k]), wo, ho)
            else:
                want, wantf = oracle.resize_lanczos4(sq(imgs[k]), wo, ho), oracle.resize_lanczos4(sq(fl[k]), wo, ho)
            assert_same(got[k].reshape(ho, wo, c), want.reshape(ho, wo, c), what + " u8")
            assert_same(gotf[k].reshape(ho, wo, c), wantf.reshape(ho, wo, c), what + " f32")


def test_resize_normalize_bench_batch(ops, dev, oracle):
    """The bench workload at its full size (256 x 1080p, one launch): images
    spread over the batch match the oracle bit for bit, every image equals the
    kernel's own single-image result (batch invariance), and a stripe of the
    batch has the oracle's checksum."""
    import torch
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    src = torch.randint(0, 256, (256, 1080, 1920, 3), dtype=torch.uint8, device=dev, generator=g)
    out = ops.resize_normalize(src, 640, 360, MEAN, STD)
    torch.cuda.synchronize(dev)
    for k in (0, 1, 77, 128, 255):
        img = host(src[k])
        want = oracle.normalize(oracle.u8_to_f32(oracle.resize_linear(img, 640, 360)), MEAN, STD)
        assert_same(host(out[k]), want, f"bench batch image {k}")
    for k in (3, 200):
        single = ops.resize_normalize(src[k:k + 1], 640, 360, MEAN, STD)
        assert torch.equal(single[0], out[k]), f"batch invariance {k}"
    # 64-column wave blocks (VACV_TUNE_RESIZE_TILE_W = 64) against the default
    # 128-column blocks of this geometry: the whole batch, bit for bit
    with ops.tuning(RESIZE_TILE_W=64):
        out64 = ops.resize_normalize(src, 640, 360, MEAN, STD)
    torch.cuda.synchronize(dev)
    assert torch.equal(out64.view(torch.int32), out.view(torch.int32)), "64- vs 128-column blocks"
    del out64
    # u8 resize of the same batch: per-image checksums of a stripe vs the oracle
    r8 = ops.resize(src, 640, 360)
    for k in range(16, 24):
        assert sha(host(r8[k])) == sha(oracle.resize_linear(host(src[k]), 640, 360)), f"u8 stripe {k}"
    del src, out, r8
    torch.cuda.empty_cache()


# ---------------------------------------------------------------------------
# warp affine

def test_warp_affine(ops, dev, oracle):
    from vacv_amd import NCHW
    mats = [np.array([0.5, 0.1, 3.0, -0.2, 0.7, 5.0], np.float32),
            oracle.rotation_matrix(0.9, 15.0, [32, 24, 32, 24]),
            oracle.rotation_matrix(1.3, -40.0, [10, 10, 20, 8]),
            np.array([1.25, 0.0, -2.0, 0.0, 1.25, -2.0], np.float32),
            np.array([1, 0, 0, 0, 1, 0], np.float32),
            np.array([0, 0, 0, 0, 0, 0], np.float32)]
    rng = np.random.default_rng(3)
    for i, ((h, w), c) in enumerate(SIZES[:5]):
        img = synthetic_image(70 + i, h, w, c)
        img = img if c > 1 else img[..., None]
        f = (img.astype(np.float32) + rng.standard_normal(img.shape).astype(np.float32)).astype(np.float32)
        for m in mats:
            for wo, ho in [(64, 48), (33, 17), (5, 3)]:
                got = host(ops.warp_affine(to_dev(img[None], dev), m, wo, ho))[0]
                want = oracle.warp_affine(img if c > 1 else img[..., 0], m, wo, ho)
                assert_same(got if c > 1 else got[..., 0], want, f"warp u8 {h}x{w}x{c}")
                gotf = host(ops.warp_affine(to_dev(f[None], dev), m, wo, ho))[0]
                wantf = oracle.warp_affine(f if c > 1 else f[..., 0], m, wo, ho)
                assert_same(gotf if c > 1 else gotf[..., 0], wantf, f"warp f32 {h}x{w}x{c}")
        chw = np.ascontiguousarray(img.transpose(2, 0, 1))
        got = host(ops.warp_affine(to_dev(chw[None], dev), mats[1], 40, 30, layout=NCHW))[0]
        for k in range(c):
            assert_same(got[k], oracle.warp_affine(chw[k], mats[1], 40, 30), "warp chw")


def test_warp_affine_config_and_harness(ops, dev, oracle, golden):
    meta, _ = golden
    d = meta["digests"]
    b720 = load_bgr("1280x720.jpg")
    if sha(b720) != d["input_1280x720"]["sha256"]:
        pytest.skip("PIL decodes differently here")
    rot = ops.rotation_matrix(0.9, 15.0, (640, 360, 640, 360))
    assert rot.tolist() == d["cfg4_rotation_matrix"]["m"]
    imgs = np.stack([b720, synthetic_image(4, 720, 1280, 3)])
    out = host(ops.warp_affine(to_dev(imgs, dev), rot, 1280, 720))
    assert sha(out[0]) == d["cfg4_warp_1280x720_rot15_u8"]["sha256"]
    assert_same(out[1], oracle.warp_affine(imgs[1], rot, 1280, 720), "cfg4 synthetic")
    M = np.array([0.849158, 0.012257, -474.827, -0.01225, 0.849158, -379.18], np.float32)
    assert sha(host(ops.warp_affine(to_dev(b720, dev), M, 240, 240))) == d["harness_warp_hwc_u8_240"]["sha256"]
    rot2 = ops.rotation_matrix(1.073914, -3.314525, (738.518372, 537.672852, 204.766998, 73.329681))
    g = load_bgr("1280x720_grey.jpg")
    assert sha(host(ops.warp_affine(to_dev(g, dev), rot2, 140, 210))) == d["harness_rotation_u8_140x210"]["sha256"]
    # normalize fused
    got = host(ops.warp_affine_normalize(to_dev(imgs, dev), rot, 1280, 720, MEAN, STD))
    want = oracle.normalize(oracle.u8_to_f32(oracle.warp_affine(imgs[1], rot, 1280, 720)), MEAN, STD)
    assert_same(got[1], want, "warp_affine_normalize")


def test_warp_cfg4_as_benchmarked(ops, dev, oracle, golden):
    """cfg4 exactly as `bench.py --workload warp` runs it: 720p u8 frames,
    rotation 15 / scale 0.9 about (640, 360), default dispatch (the frames
    kernel with its default frames per workgroup: 128 frames are full groups,
    131 leave a partial last group).  Frame 0 is the reference's own
    1280x720.jpg and must give the cfg4 digest made by the reference's
    warp_affine_naive (warp_affine_naive.cpp:9-58); frames 1, 63, 64, 127 and
    130 are compared with the oracle; the whole batch with the per-pixel
    gather kernel (VACV_TUNE_WARP_KERNEL = 0); the fused normalize likewise."""
    import torch
    meta, _ = golden
    d = meta["digests"]
    b720 = load_bgr("1280x720.jpg")
    if sha(b720) != d["input_1280x720"]["sha256"]:
        pytest.skip("PIL decodes differently here")
    rot = ops.rotation_matrix(0.9, 15.0, (640, 360, 640, 360))
    g = torch.Generator(device=dev)
    g.manual_seed(1234)
    for n in (128, 131):
        src = torch.randint(0, 256, (n, 720, 1280, 3), dtype=torch.uint8, device=dev, generator=g)
        src[0].copy_(to_dev(b720, dev))
        dst = torch.empty_like(src)
        ops.warp_affine(src, rot, 1280, 720, out=dst)  # the bench call
        got = host(dst)
        assert sha(got[0]) == d["cfg4_warp_1280x720_rot15_u8"]["sha256"], f"cfg4 digest, batch {n}"
        for k in (1, 63, 64, 127, 130):
            if k < n:
                assert_same(got[k], oracle.warp_affine(host(src[k]), rot, 1280, 720), f"cfg4 frame {k} of {n}")
        with ops.tuning(WARP_KERNEL=0):
            want = ops.warp_affine(src, rot, 1280, 720)
        assert torch.equal(dst, want), f"cfg4 batch {n}: frames kernel vs gather kernel"
        del want
        gotn = ops.warp_affine_normalize(src, rot, 1280, 720, MEAN, STD)
        for k in (0, 64, n - 1):
            wn = oracle.normalize(oracle.u8_to_f32(got[k]), MEAN, STD)
            assert_same(host(gotn[k]), wn, f"cfg4 normalize frame {k} of {n}")
        with ops.tuning(WARP_KERNEL=0):
            assert torch.equal(gotn, ops.warp_affine_normalize(src, rot, 1280, 720, MEAN, STD)), \
                f"cfg4 normalize batch {n}"
        del src, dst, gotn
        torch.cuda.empty_cache()


def test_warp_frames_plan_cache_keys(ops, dev, oracle):
    """The frames kernel's LDS plan depends on the channel count and on the
    output kind (byte output adds a store-exchange area).  Calls that share a
    matrix and sizes but differ in those must not share a plan: fp32 output
    first, then u8 output; 1 channel first, then 4; each compared with the
    gather kernel at 720p x 8 frames (full-size tiles, many workgroups per CU)."""
    import torch
    rng = np.random.default_rng(77)
    for a, (first, then) in enumerate([(("norm", 3), ("u8", 3)), (("u8", 1), ("u8", 4)), (("f32", 4), ("u8", 4))]):
        m = ops.rotation_matrix(0.9, 11.0 + a + 0.37, (640, 360, 640, 360))  # a matrix no other test uses
        for kind, c in (first, then):
            src = to_dev(rng.integers(0, 256, (8, 720, 1280, c), dtype=np.uint8), dev)
            mu = np.concatenate([MEAN, [1.0]]).astype(np.float32)[:c]
            sd = np.concatenate([STD, [2.0]]).astype(np.float32)[:c]

            def run():
                if kind == "norm":
                    return ops.warp_affine_normalize(src, m, 1280, 720, mu, sd)
                s = src if kind == "u8" else src.float()
                return ops.warp_affine(s, m, 1280, 720)
            got = run()
            with ops.tuning(WARP_KERNEL=0):
                want = run()
            assert torch.equal(got, want), f"{kind} c={c} after {first}"


def test_match_template(ops, dev, oracle):
    """match_template (match_template.cpp:13-41 -> cv::matchTemplate; OpenCV
    2.4's six methods restated in oracle/vacv_oracle.c, parity unpinned):
    u8 bit-exact (integer correlation, identical double formula); fp32 within
    1e-5 (window sums in another order); c = 1, 3, 4; a batch against one
    template; a template as large as the image; a flat template under
    CCOEFF_NORMED (all ones); a larger template (cv::matchTemplate swaps)."""
    import torch
    rng = np.random.default_rng(53)
    for c in (1, 3, 4):
        imgs = np.stack([synthetic_image(900 + 10 * c + k, 70, 301, c).reshape(70, 301, c) for k in range(2)])
        tpl = np.ascontiguousarray(imgs[1, 20:37, 150:173])
        for m in range(6):
            got = host(ops.match_template(to_dev(imgs, dev), to_dev(tpl, dev), m))
            for k in range(2):
                want = oracle.match_template(imgs[k], tpl, m)
                assert_same(got[k], want, f"match u8 c{c} method {m} image {k}")
        f = (imgs[0].astype(np.float32) * np.float32(0.5) + rng.standard_normal(imgs[0].shape).astype(np.float32))
        tf = np.ascontiguousarray(f[5:16, 40:61])
        for m in range(6):
            got = host(ops.match_template(to_dev(f, dev), to_dev(tf, dev), m))
            want = oracle.match_template(f, tf, m)
            np.testing.assert_allclose(got, want, rtol=1e-5, atol=1e-5 * max(1.0, float(np.abs(want).max())),
                                       err_msg=f"match f32 c{c} method {m}")
    img = synthetic_image(950, 40, 50, 1)
    full = host(ops.match_template(to_dev(img, dev), to_dev(img, dev), 5))
    assert full.shape == (1, 1) and abs(float(full[0, 0]) - 1.0) < 1e-6
    flat = np.full((5, 7), 9, np.uint8)
    ones = host(ops.match_template(to_dev(img, dev), to_dev(flat, dev), 5))
    assert (ones == 1.0).all()
    small = np.ascontiguousarray(img[3:10, 4:15])
    sw = host(ops.match_template(to_dev(small, dev), to_dev(img, dev), 0))  # swapped: img is the template
    assert_same(sw, oracle.match_template(img, small, 0), "match swapped")
    # the u8 correlation on the matrix cores (default where its image block
    # fits) and on the v_dot4 kernel (VACV_TUNE_MATCH_KERNEL = 0): identical,
    # at a size with several output tiles, partial tiles and every method
    big = np.stack([synthetic_image(960 + k, 203, 301, 3).reshape(203, 301, 3) for k in range(3)])
    btpl = np.ascontiguousarray(big[1, 50:97, 100:141])
    for m in range(6):
        a = host(ops.match_template(to_dev(big, dev), to_dev(btpl, dev), m))
        with ops.tuning(MATCH_KERNEL=0):
            b = host(ops.match_template(to_dev(big, dev), to_dev(btpl, dev), m))
        assert_same(a, b, f"match mfma vs dot4 method {m}")
    for c in (1, 4):  # other channel counts through the matrix cores, against the oracle
        im = synthetic_image(970 + c, 90, 150, c).reshape(90, 150, c)
        tp = np.ascontiguousarray(im[10:43, 20:77])
        got = host(ops.match_template(to_dev(im[None], dev), to_dev(tp, dev), 2))
        assert_same(got[0], oracle.match_template(im, tp, 2), f"match mfma c{c}")
    # the largest sums the matrix-core plan takes: all-255 image and a
    # 226 x 141 template (K*h = 31,866, the LDS plan's limit is about 32k;
    # 255^2 * 31,866 = 2.07e9, next to 2^31), recombined in int64
    sat = np.full((300, 400), 255, np.uint8)
    stpl = np.full((141, 226), 255, np.uint8)
    got = host(ops.match_template(to_dev(sat, dev), to_dev(stpl, dev), 2))
    assert_same(got, oracle.match_template(sat, stpl, 2), "match mfma int32 limit")
    assert (got == np.float32(255.0 * 255.0 * 226 * 141)).all()
    with ops.tuning(MATCH_KERNEL=0):
        assert_same(host(ops.match_template(to_dev(sat, dev), to_dev(stpl, dev), 2)), got, "match dot4 int32 limit")
    # u8 window statistics as uint32 box sums (match_vsum_u8_kernel /
    # match_finish_u8_kernel): the saturated image puts 255^2 * 31,866 =
    # 2.07e9 in every window's square sum (uint32, exact) -- every method;
    # and a row too wide for the workgroup's LDS prefix rows (2,800 x 3
    # channels) takes the double integral images, against the oracle too
    for m in (0, 1, 3, 4, 5):
        assert_same(host(ops.match_template(to_dev(sat, dev), to_dev(stpl, dev), m)),
                    oracle.match_template(sat, stpl, m), f"match box sums saturated method {m}")
    wide = synthetic_image(980, 20, 2800, 3).reshape(20, 2800, 3)
    wtpl = np.ascontiguousarray(wide[4:11, 100:109])
    for m in (1, 5):
        assert_same(host(ops.match_template(to_dev(wide[None], dev), to_dev(wtpl, dev), m))[0],
                    oracle.match_template(wide, wtpl, m), f"match integral images wide row method {m}")
    # minMaxIdx on a match result finds the template's position
    got = ops.match_template(to_dev(img, dev), to_dev(small, dev), 0)
    mn, mx, imn, imx = ops.min_max_idx(got)
    want = oracle.min_max_idx(host(got))
    assert (mn, mx, imn, imx) == want and imn == (3, 4), ((mn, mx, imn, imx), want)


def test_min_max_idx(ops, dev, oracle):
    """minMaxIdx (match_template.cpp:43-46 -> cv::minMaxIdx): first min / max
    in row-major order, masks, ties, NaNs skipped, u8 and fp32, an all-masked
    input (0, 0, -1s), sizes past one workgroup's share."""
    rng = np.random.default_rng(59)
    for h, w in [(1, 1), (7, 13), (333, 517), (1080, 1920)]:
        a = rng.standard_normal((h, w)).astype(np.float32)
        if h * w > 4:
            a[h // 2, w // 3] = np.nan
            a.flat[h * w - 1] = a.min()  # a later tie of the minimum
        assert ops.min_max_idx(to_dev(a, dev)) == oracle.min_max_idx(a), (h, w)
        u = rng.integers(0, 256, (h, w), dtype=np.uint8)
        assert ops.min_max_idx(to_dev(u, dev)) == oracle.min_max_idx(u), (h, w, "u8")
        m = (rng.random((h, w)) < 0.3).astype(np.uint8)
        assert ops.min_max_idx(to_dev(u, dev), to_dev(m, dev)) == oracle.min_max_idx(u, m), (h, w, "mask")
    z = np.zeros((5, 6), np.uint8)
    assert ops.min_max_idx(to_dev(z, dev)) == (0.0, 0.0, (0, 0), (0, 0))
    assert ops.min_max_idx(to_dev(z, dev), to_dev(z, dev)) == (0.0, 0.0, (-1, -1), (-1, -1))


def test_warp_border_modes(ops, dev, oracle):
    """BORDER_REPLICATE / REFLECT / WRAP / REFLECT_101 / TRANSPARENT (the
    reference hands them to OpenCV, warp_affine.cpp:114-118; here the naive
    sampler with OpenCV's borderInterpolate taps, parity unpinned --
    oracle/vacv_oracle.c): u8 and fp32, NHWC c = 1 and 3 and NCHW, the
    batched and per-pixel kernels, maps that reach far outside the source (a
    shrink with a large offset), the normalize epilogue; TRANSPARENT keeps
    the destination's bytes where the sampler has no taps."""
    import torch
    from vacv_amd import NCHW
    mats = [ops.rotation_matrix(0.7, 33.0, (40, 30, 50, 35)),
            np.array([0.3, 0.05, 70.0, -0.04, 0.35, -20.0], np.float32),   # shrink + big offset: wraps often
            np.array([-1.6, 0.1, 150.0, 0.2, 1.3, -9.5], np.float32)]       # flip + up-scale
    for c in (1, 3):
        img = synthetic_image(300 + c, 61, 83, c).reshape(61, 83, c)
        f = img.astype(np.float32) * np.float32(0.75) + np.float32(0.125)
        for m in mats:
            for mode in (1, 2, 3, 4):
                for knob in (2, 0):
                    with ops.tuning(WARP_KERNEL=knob):
                        got = host(ops.warp_affine(to_dev(img[None], dev), m, 97, 71, border_mode=mode))[0]
                        gotf = host(ops.warp_affine(to_dev(f[None], dev), m, 97, 71, border_mode=mode))[0]
                    want = oracle.warp_affine(img, m, 97, 71, border_mode=mode).reshape(71, 97, c)
                    assert_same(got.reshape(71, 97, c), want, f"border {mode} u8 c{c} kernel={knob}")
                    wantf = oracle.warp_affine(f, m, 97, 71, border_mode=mode).reshape(71, 97, c)
                    assert_same(gotf.reshape(71, 97, c), wantf, f"border {mode} f32 c{c}")
            prev = np.full((71, 97, c), 77, np.uint8)
            for knob in (2, 0):
                with ops.tuning(WARP_KERNEL=knob):
                    out = to_dev(prev[None], dev)
                    ops.warp_affine(to_dev(img[None], dev), m, 97, 71, border_mode=5, out=out)
                want = oracle.warp_affine(img, m, 97, 71, border_mode=5, dst=prev.reshape(71, 97, c) if c > 1
                                          else prev.reshape(71, 97)).reshape(71, 97, c)
                assert_same(host(out)[0].reshape(71, 97, c), want, f"transparent c{c} kernel={knob}")
    img = synthetic_image(310, 61, 83, 3)
    chw = to_dev(np.ascontiguousarray(img.transpose(2, 0, 1))[None], dev)
    got = host(ops.warp_affine(chw, mats[1], 97, 71, border_mode=4, layout=NCHW))[0]
    for k in range(3):
        assert_same(got[k], oracle.warp_affine(np.ascontiguousarray(img[..., k]), mats[1], 97, 71, border_mode=4),
                    "border chw")
    got = host(ops.warp_affine_normalize(to_dev(img[None], dev), mats[0], 97, 71, MEAN, STD, border_mode=1))[0]
    want = oracle.normalize(oracle.u8_to_f32(oracle.warp_affine(img, mats[0], 97, 71, border_mode=1)), MEAN, STD)
    assert_same(got, want, "border normalize")


# the LDS-staged warp kernel with 2 (default), 3 and 4 boxes in its LDS ring
FRAMES_VARIANTS = [dict(WARP_KERNEL=4, WARP_SLOTS=2), dict(WARP_KERNEL=4, WARP_SLOTS=3),
                   dict(WARP_KERNEL=4, WARP_SLOTS=4)]


@pytest.mark.parametrize("variant", range(len(FRAMES_VARIANTS)))
def test_warp_frames_kernel(ops, dev, oracle, variant):
    """The LDS-staged kernel (k_warp_frames.hip: per-pixel taps computed once
    for kf frames, the source boxes copied into an LDS ring of 2-4 slots by
    LDS-DMA) is the default for u8 BORDER_CONSTANT warps (1-4 channels, NCHW
    planes as frames); border-only tiles skip the sampling.  Against the per-pixel
    gather kernel (VACV_TUNE_WARP_KERNEL = 0) at full size over frames per
    workgroup 1, 2, 3, 16 and tile heights 16 / 32 (odd batch: a partial last
    frame group), u8 / fp32 / normalised outputs, a non-zero border value and a
    pitched destination; against the oracle at odd sizes where the source box
    reaches the plane's last bytes (the bytewise tail path)."""
    import torch
    V = FRAMES_VARIANTS[variant]
    n = 7
    imgs = np.stack([synthetic_image(500 + k, 720, 1280, 3) for k in range(n)])
    src = to_dev(imgs, dev)
    mats = [ops.rotation_matrix(0.9, 15.0, (640, 360, 640, 360)),
            ops.rotation_matrix(0.9, 45.0, (640, 360, 640, 360)),
            ops.rotation_matrix(1.2, -100.0, (640, 360, 600, 350)),
            np.array([1, 0, -0.5, 0, 1, -0.5], np.float32)]
    for m in mats:
        with ops.tuning(WARP_KERNEL=0):
            want = ops.warp_affine(src, m, 1280, 720, border_value=(7, 200, 31, 0))
            wantn = ops.warp_affine_normalize(src, m, 1280, 720, MEAN, STD)
        for th in (16, 32):
            for kf in (1, 2, 3, 16):
                with ops.tuning(**V, WARP_FRAMES=kf, WARP_TILE_H=th):
                    got = ops.warp_affine(src, m, 1280, 720, border_value=(7, 200, 31, 0))
                    assert torch.equal(got, want), f"frames kernel {m.tolist()} th={th} kf={kf}"
            with ops.tuning(**V, WARP_TILE_H=th):
                assert torch.equal(ops.warp_affine_normalize(src, m, 1280, 720, MEAN, STD), wantn), \
                    f"frames kernel normalize {m.tolist()} th={th}"
    # pitched destination (dword-aligned quads and bytewise columns)
    for x0 in (4, 5):
        big = torch.zeros((n, 130, 230, 3), dtype=torch.uint8, device=dev)
        view = big[:, 3:123, x0:x0 + 200]
        with ops.tuning(**V):
            ops.warp_affine(src, mats[2], 200, 120, out=view)
        g = host(big)
        for k in (0, n - 1):
            assert_same(g[k, 3:123, x0:x0 + 200], oracle.warp_affine(imgs[k], mats[2], 200, 120), f"pitched {x0}")
        g[:, 3:123, x0:x0 + 200] = 0
        assert not g.any(), "frames kernel wrote outside the window"
    for c in (1, 2, 3, 4):  # odd sizes: the source box reaches the plane's last group
        ims = np.stack([synthetic_image(600 + 7 * c + k, 97, 143, c).reshape(97, 143, c) for k in range(3)])
        mu = np.concatenate([MEAN, [1.0]]).astype(np.float32)[:c]
        sd = np.concatenate([STD, [2.0]]).astype(np.float32)[:c]
        for m in mats:
            for wo, ho in ((143, 97), (121, 83)):
                with ops.tuning(**V, WARP_FRAMES=2):
                    got = host(ops.warp_affine(to_dev(ims, dev), m, wo, ho))
                    gotf = host(ops.warp_affine_normalize(to_dev(ims, dev), m, wo, ho, mu, sd))
                for k in range(3):
                    want = oracle.warp_affine(ims[k] if c > 1 else ims[k, ..., 0], m, wo, ho).reshape(ho, wo, c)
                    assert_same(got[k].reshape(ho, wo, c), want, f"frames c={c} {wo}x{ho} {m.tolist()}")
                    wantf = oracle.normalize(oracle.u8_to_f32(want), mu, sd)
                    assert_same(gotf[k].reshape(ho, wo, c), wantf.reshape(ho, wo, c), f"frames norm c={c}")


    # pitched sources: rows padded to a multiple of 4 bytes (the frames
    # kernel) and a source starting 1 byte into its allocation (dword-
    # misaligned: the gather kernels)
    bigs = to_dev(np.zeros((n, 100, 192, 3), np.uint8), dev)  # rows of 576 bytes
    bigs[:, 2:99, 4:147] = to_dev(imgs[:, 100:197, 300:443], dev)
    for view, tag in ((bigs[:, 2:99, 4:147], "row-padded"),
                      (to_dev(np.ascontiguousarray(imgs[:, 100:197, 300:443]), dev), "dense")):
        with ops.tuning(**V):
            got = host(ops.warp_affine(view, mats[0], 121, 83))
        for k in (0, n - 1):
            assert_same(got[k], oracle.warp_affine(np.ascontiguousarray(imgs[k, 100:197, 300:443]), mats[0], 121, 83)
                        .reshape(83, 121, 3), f"pitched source {tag}")
    flat = torch.zeros(n * 97 * 143 * 3 + 1, dtype=torch.uint8, device=dev)
    mis = flat[1:].view(n, 97, 143, 3)
    mis.copy_(to_dev(np.ascontiguousarray(imgs[:, 100:197, 300:443]), dev))
    got = host(ops.warp_affine(mis, mats[0], 121, 83))
    assert_same(got[n - 1], oracle.warp_affine(np.ascontiguousarray(imgs[n - 1, 100:197, 300:443]), mats[0], 121, 83)
                .reshape(83, 121, 3), "misaligned source")
    # NCHW planes are frames of their own (3 planes x 3 images)
    from vacv_amd import NCHW
    ims = np.stack([synthetic_image(650 + k, 97, 143, 3) for k in range(3)])
    chw = to_dev(np.ascontiguousarray(ims.transpose(0, 3, 1, 2)), dev)
    with ops.tuning(**V, WARP_FRAMES=2):
        got = host(ops.warp_affine(chw, mats[0], 121, 83, layout=NCHW))
        gotn = host(ops.warp_affine_normalize(chw, mats[0], 121, 83, MEAN, STD, layout=NCHW))
    for k in range(3):
        for ch in range(3):
            want = oracle.warp_affine(np.ascontiguousarray(ims[k, ..., ch]), mats[0], 121, 83)
            assert_same(got[k, ch], want.reshape(83, 121), f"frames chw {k} {ch}")
            wn = oracle.normalize(oracle.u8_to_f32(want.reshape(83, 121, 1)), MEAN[ch:ch + 1], STD[ch:ch + 1])
            assert_same(gotn[k, ch], wn.reshape(83, 121), f"frames chw norm {k} {ch}")

def test_warp_random_matrices(ops, dev, oracle):
    """Seeded random affine maps (any rotation, anisotropic scale 0.4-2.5,
    shear, the source centre jittered by up to half a frame), odd sizes, 1-4
    channels, u8 and fp32 sources, all five sampling border modes, batches of
    2: whichever kernel the planner picks (the LDS ring for u8 CONSTANT, the
    gather kernels for boxes over its LDS plan, fp32 and the other borders)
    is bit-exact against the oracle (warp_affine_naive.cpp:9-62, inverse as
    warp_affine.cpp:121-133), and so is the normalize epilogue."""
    rng = np.random.default_rng(20260418)
    for t in range(40):
        c = 1 + t % 4
        h, w = int(rng.integers(13, 150)), int(rng.integers(13, 190))
        ho, wo = int(rng.integers(7, 140)), int(rng.integers(7, 180))
        a = np.deg2rad(rng.uniform(-180.0, 180.0))
        sx, sy = rng.uniform(0.4, 2.5, 2)
        A = np.array([[np.cos(a), -np.sin(a)], [np.sin(a), np.cos(a)]]) @ np.array([[sx, rng.uniform(-0.6, 0.6)],
                                                                                   [0.0, sy]])
        tv = np.array([wo / 2, ho / 2]) - A @ np.array([w / 2, h / 2]) + rng.uniform(-0.5, 0.5, 2) * (wo, ho)
        m = np.concatenate([A, tv[:, None]], 1).astype(np.float32).reshape(6)
        mode = 0 if (t // 4) % 2 == 0 else int(rng.integers(1, 5))  # half on the LDS ring's CONSTANT path
        ims = np.stack([synthetic_image(9000 + 2 * t + k, h, w, c).reshape(h, w, c) for k in range(2)])
        fl = ims.astype(np.float32) * np.float32(0.75) + np.float32(0.125)
        mu = np.concatenate([MEAN, [1.0]]).astype(np.float32)[:c]
        sd = np.concatenate([STD, [2.0]]).astype(np.float32)[:c]
        got = host(ops.warp_affine(to_dev(ims, dev), m, wo, ho, border_mode=mode))
        gotf = host(ops.warp_affine(to_dev(fl, dev), m, wo, ho, border_mode=mode))
        gotn = host(ops.warp_affine_normalize(to_dev(ims, dev), m, wo, ho, mu, sd, border_mode=mode))
        what = f"case {t}: {w}x{h}x{c} -> {wo}x{ho} border {mode} m={m.tolist()}"
        for k in range(2):
            src = ims[k] if c > 1 else ims[k, ..., 0]
            want = oracle.warp_affine(src, m, wo, ho, border_mode=mode).reshape(ho, wo, c)
            assert_same(got[k].reshape(ho, wo, c), want, what)
            wantf = oracle.warp_affine(fl[k] if c > 1 else fl[k, ..., 0], m, wo, ho, border_mode=mode)
            assert_same(gotf[k].reshape(ho, wo, c), wantf.reshape(ho, wo, c), what + " f32")
            wantn = oracle.normalize(oracle.u8_to_f32(want), mu, sd)
            assert_same(gotn[k].reshape(ho, wo, c), wantn.reshape(ho, wo, c), what + " normalize")
        # INTER_NEAREST on the same map (every other case through WARP_INVERSE_MAP
        # with the host-inverted matrix), a non-zero border value
        from vacv_amd import INTER_NEAREST, WARP_INVERSE_MAP
        inv = t % 2 == 1
        mm = oracle.invert_affine(m) if inv else m
        bv = (7, 200, 31, 99)
        gotnn = host(ops.warp_affine(to_dev(ims, dev), mm, wo, ho, flags=INTER_NEAREST | (WARP_INVERSE_MAP if inv else 0),
                                     border_mode=mode, border_value=bv))
        for k in range(2):
            src = ims[k] if c > 1 else ims[k, ..., 0]
            want = oracle.warp_affine_nn(src, mm, wo, ho, inverse_map=inv, border_mode=mode, border=bv)
            assert_same(gotnn[k].reshape(ho, wo, c), want.reshape(ho, wo, c), what + f" nearest inv={inv}")


def test_warp_nearest_staged(ops, dev, oracle):
    """INTER_NEAREST on the LDS-staged kernel (warp_exp_kernel<..., NN>: 3-channel
    u8, BORDER_CONSTANT, dword-aligned rows): seeded random maps on 4-aligned
    widths, u8 and normalised fp32 output, through WARP_INVERSE_MAP every other
    case, against the oracle's OpenCV restatement (parity unpinned); and cfg4's
    720p rot-15 map on 6 frames, bit-identical to the gather kernel
    (VACV_TUNE_WARP_KERNEL = 5) and to the oracle on frames 0 and 5."""
    import torch
    from vacv_amd import INTER_NEAREST, WARP_INVERSE_MAP
    rng = np.random.default_rng(20261018)
    bv = (7, 200, 31, 99)
    for t in range(16):
        h, w = int(rng.integers(20, 160)), 4 * int(rng.integers(5, 48))
        ho, wo = int(rng.integers(9, 140)), 4 * int(rng.integers(3, 45))
        a = np.deg2rad(rng.uniform(-180.0, 180.0))
        sx, sy = rng.uniform(0.5, 1.8, 2)
        A = np.array([[np.cos(a), -np.sin(a)], [np.sin(a), np.cos(a)]]) @ np.array([[sx, rng.uniform(-0.4, 0.4)],
                                                                                   [0.0, sy]])
        tv = np.array([wo / 2, ho / 2]) - A @ np.array([w / 2, h / 2]) + rng.uniform(-0.5, 0.5, 2) * (wo, ho)
        m = np.concatenate([A, tv[:, None]], 1).astype(np.float32).reshape(6)
        inv = t % 2 == 1
        mm = oracle.invert_affine(m) if inv else m
        fl = INTER_NEAREST | (WARP_INVERSE_MAP if inv else 0)
        ims = np.stack([synthetic_image(9500 + 2 * t + k, h, w, 3) for k in range(2)])
        got = host(ops.warp_affine(to_dev(ims, dev), mm, wo, ho, flags=fl, border_value=bv))
        gotn = host(ops.warp_affine_normalize(to_dev(ims, dev), mm, wo, ho, MEAN, STD, flags=fl, border_value=bv))
        what = f"case {t}: {w}x{h} -> {wo}x{ho} inv={inv} m={m.tolist()}"
        for k in range(2):
            want = oracle.warp_affine_nn(ims[k], mm, wo, ho, inverse_map=inv, border=bv).reshape(ho, wo, 3)
            assert_same(got[k].reshape(ho, wo, 3), want, what)
            assert_same(gotn[k].reshape(ho, wo, 3), oracle.normalize(oracle.u8_to_f32(want), MEAN, STD),
                        what + " normalize")
    m = ops.rotation_matrix(0.9, 15.0, (640, 360, 640, 360))
    src = torch.randint(0, 256, (6, 720, 1280, 3), dtype=torch.uint8, device=dev,
                        generator=torch.Generator(device=dev).manual_seed(5))
    a = ops.warp_affine(src, m, 1280, 720, flags=INTER_NEAREST)
    with ops.tuning(WARP_KERNEL=5):
        b = ops.warp_affine(src, m, 1280, 720, flags=INTER_NEAREST)
    torch.cuda.synchronize(dev)
    assert torch.equal(a, b), f"{(a != b).sum().item()} bytes differ from the gather kernel"
    for k in (0, 5):
        want = oracle.warp_affine_nn(host(src[k]), m, 1280, 720)
        assert_same(host(a[k]), want.reshape(720, 1280, 3), f"cfg4 nearest frame {k}")
    del src, a, b
    torch.cuda.empty_cache()


def test_warp_kernels_agree(ops, dev, oracle):
    """u8 BORDER_CONSTANT warps run on the LDS-staged frames kernel
    (k_warp_frames.hip) unless its box plan does not fit (e.g. a 4x
    down-scale); then on the batched gather kernel (warp_u8_kernel) where a 64-pixel output row
    spans few source rows, else on the per-pixel kernel (warp_kernel).
    VACV_TUNE_WARP_KERNEL = 4 / 2 / 0 forces one of them and VACV_TUNE_WARP_PX
    switches the gather kernels' lane blocks per wave.  Identical outputs at
    full size for rotations, flips, shears, strong down-scales, fused
    normalisation, NCHW planes and a pitched destination."""
    import torch
    from vacv_amd import NCHW
    imgs = np.stack([synthetic_image(80 + k, 720, 1280, 3) for k in range(2)])
    src = to_dev(imgs, dev)
    mats = [ops.rotation_matrix(0.9, 15.0, (640, 360, 640, 360)),
            ops.rotation_matrix(1.7, -130.0, (640, 360, 500, 300)),
            np.array([-1, 0, 1279, 0, 1, 0], np.float32),            # horizontal flip
            np.array([1.3, 0.2, 100.0, -0.1, 1.45, 50.0], np.float32),  # shear + up-scale
            np.array([0.25, 0.0, 0.0, 0.0, 0.25, 0.0], np.float32),   # 4x down: footprint over budget
            np.array([1, 0, 0.5, 0, 1, -0.25], np.float32)]
    for m in mats:
        for wo, ho in [(1280, 720), (333, 211)]:
            with ops.tuning(WARP_KERNEL=2):
                a = ops.warp_affine(src, m, wo, ho)
                an = ops.warp_affine_normalize(src, m, wo, ho, MEAN, STD)
            with ops.tuning(WARP_KERNEL=4):
                t = ops.warp_affine(src, m, wo, ho)
                tn = ops.warp_affine_normalize(src, m, wo, ho, MEAN, STD)
            with ops.tuning(WARP_KERNEL=0):
                b = ops.warp_affine(src, m, wo, ho)
                bn = ops.warp_affine_normalize(src, m, wo, ho, MEAN, STD)
                assert torch.equal(a, b), f"warp kernels differ {m.tolist()} {wo}x{ho}"
                assert torch.equal(an, bn), f"warp normalize kernels differ {m.tolist()} {wo}x{ho}"
                assert torch.equal(t, b), f"staged warp differs {m.tolist()} {wo}x{ho}"
                assert torch.equal(tn, bn), f"staged warp normalize differs {m.tolist()} {wo}x{ho}"
                for px in (4, 5, 8, 10):
                    with ops.tuning(WARP_PX=px):
                        assert torch.equal(ops.warp_affine(src, m, wo, ho), b), f"gather PX={px}"
                        assert torch.equal(ops.warp_affine_normalize(src, m, wo, ho, MEAN, STD), bn), \
                            f"gather PX={px} norm"
    for c in (1, 2, 3, 4):  # every pixel width, odd sizes, both kernels vs the oracle
        im = synthetic_image(90 + c, 97, 143, c)
        for m in mats[:2] + mats[3:4]:
            for wo in (121, 128):  # byte stores / the aligned 4-pixel stores, partial tiles
                want = oracle.warp_affine(im, m, wo, 83).reshape(83, wo, c)
                for flag in (4, 2, 0):
                    with ops.tuning(WARP_KERNEL=flag):
                        got = host(ops.warp_affine(to_dev(im.reshape(1, 97, 143, c), dev), m, wo, 83))[0]
                    assert_same(got.reshape(83, wo, c), want, f"warp c={c} {wo} kernel={flag}")
    chw = to_dev(np.ascontiguousarray(imgs.transpose(0, 3, 1, 2)), dev)
    got = host(ops.warp_affine(chw, mats[0], 300, 200, layout=NCHW))
    for k in range(3):
        assert_same(got[1, k], oracle.warp_affine(np.ascontiguousarray(imgs[1, ..., k]), mats[0], 300, 200), "warp chw")
    big = torch.zeros((1, 130, 230, 3), dtype=torch.uint8, device=dev)
    view = big[:, 3:123, 5:205]
    ops.warp_affine(src[:1], mats[1], 200, 120, out=view)
    g = host(big)
    assert_same(g[0, 3:123, 5:205], oracle.warp_affine(imgs[0], mats[1], 200, 120), "warp pitched out")
    g[0, 3:123, 5:205] = 0
    assert not g.any(), "warp kernel wrote outside the window"


# ---------------------------------------------------------------------------
# colour

@pytest.mark.parametrize("v_first,rgb", [(True, False), (False, False), (True, True), (False, True)])
def test_cvt_color(ops, dev, oracle, v_first, rgb):
    import vacv_amd as V
    code = {(True, False): V.COLOR_YUV2BGR_NV21, (False, False): V.COLOR_YUV2BGR_NV12,
            (True, True): V.COLOR_YUV2RGB_NV21, (False, True): V.COLOR_YUV2RGB_NV12}[(v_first, rgb)]
    rng = np.random.default_rng(17)
    for h, w in [(2, 2), (16, 24), (36, 50), (144, 176), (1080, 1920), (6, 10)]:
        yuv = np.stack([rng.integers(0, 256, (h * 3 // 2, w), dtype=np.uint8) for _ in range(2)])
        out = host(ops.cvt_color(to_dev(yuv, dev), code))
        for k in range(2):
            assert_same(out[k], oracle.yuv420sp_to_bgr(yuv[k], v_first=v_first, rgb=rgb), f"cvt {h}x{w}")
        outn = host(ops.cvt_color_normalize(to_dev(yuv, dev), code, MEAN, STD))
        for k in range(2):
            want = oracle.normalize(oracle.u8_to_f32(oracle.yuv420sp_to_bgr(yuv[k], v_first=v_first, rgb=rgb)), MEAN, STD)
            assert_same(outn[k], want, "cvt normalize")


def test_cvt_color_pipeline_digests(ops, dev, oracle, golden):
    meta, _ = golden
    d = meta["digests"]
    b = load_bgr("1920x1080.jpeg")
    if sha(b) != d["input_1920x1080"]["sha256"]:
        pytest.skip("PIL decodes differently here")
    nv = oracle.bgr2nv21(b)
    assert sha(nv) == d["cfg3_nv21_1080p"]["sha256"]
    bgr = host(ops.cvt_color(to_dev(nv, dev)))
    assert sha(bgr) == d["cfg3_nv21_to_bgr_1080p"]["sha256"]
    out = host(ops.cvt_color_normalize(to_dev(nv, dev), mean=MEAN, std=STD))
    assert sha(out) == d["cfg3_nv21_bgr_normalize_1080p"]["sha256"]


def test_cvt_color_cfg3_as_benchmarked(ops, dev, oracle, golden):
    """BASELINE cfg3 exactly as bench.py --workload cvt_normalize runs it: 256
    NV21 1080p frames (1920 x 1620 u8, drawn on the device as bench.py draws
    them) -> cvt_color_normalize into a preallocated (256, 1080, 1920, 3) fp32
    output of 6.37 GB, the only BASELINE output past 2^32 bytes.  Frame 0 is
    the reference's 1080p test image (its NV21 must hash to the reference's
    cfg3 digest); frames 127, 128, 200 and 255 -- 200 and 255 start beyond
    the 4 GiB output offset -- must equal the oracle bit for bit.  The same
    for cvt_color's u8 output (1.59 GB) once.
    Reference: cvt_color.cpp:39-135, normalize_naive.cpp:74-90."""
    import torch
    meta, _ = golden
    d = meta["digests"]
    b = load_bgr("1920x1080.jpeg")
    if sha(b) != d["input_1920x1080"]["sha256"]:
        pytest.skip("PIL decodes differently here")
    nv = oracle.bgr2nv21(b)
    g = torch.Generator(device=dev)
    g.manual_seed(1234)
    yuv = torch.randint(0, 256, (256, 1620, 1920), dtype=torch.uint8, device=dev, generator=g)
    yuv[0] = to_dev(nv, dev)
    out = torch.empty((256, 1080, 1920, 3), dtype=torch.float32, device=dev)
    assert out.numel() * 4 > 200 * 1080 * 1920 * 12 > 2 ** 32
    ops.cvt_color_normalize(yuv, mean=MEAN, std=STD, out=out)
    assert sha(host(out[0])) == d["cfg3_nv21_bgr_normalize_1080p"]["sha256"]
    for k in (127, 128, 200, 255):
        want = oracle.normalize(oracle.u8_to_f32(oracle.yuv420sp_to_bgr(host(yuv[k]))), MEAN, STD)
        assert_same(host(out[k]), want, f"cfg3 frame {k}")
    del out
    torch.cuda.empty_cache()
    bgr = torch.empty((256, 1080, 1920, 3), dtype=torch.uint8, device=dev)
    ops.cvt_color(yuv, out=bgr)
    assert sha(host(bgr[0])) == d["cfg3_nv21_to_bgr_1080p"]["sha256"]
    for k in (128, 255):
        assert_same(host(bgr[k]), oracle.yuv420sp_to_bgr(host(yuv[k])), f"cvt_color u8 frame {k}")
    del bgr, yuv
    torch.cuda.empty_cache()


# ---------------------------------------------------------------------------
# fused camera frame -> model input

def _yuv_chain(oracle, yuv, w, h, v_first, rgb, mode, mean=None, std=None, chw=False, u8=False):
    """The reference's own chain, step by step, on the oracle: cvt_color ->
    resize INTER_LINEAR u8 -> change_dtype FP32 -> normalize -> change_layout."""
    r = oracle.resize_linear(oracle.yuv420sp_to_bgr(yuv, v_first=v_first, rgb=rgb), w, h, mode)
    if not u8:
        r = oracle.u8_to_f32(r)
        if mean is not None:
            r = oracle.normalize(r, mean, std)
    return oracle.hwc_to_chw(r) if chw else r


def test_cvt_color_resize_random_geometry(ops, dev, oracle):
    """Seeded random even frame sizes and output sizes (scale 0.1-2.5) for the
    four semi-planar codes: cvt_color, cvt_color_normalize and the fused
    cvt_color_resize_normalize (NHWC / NCHW) match the reference's step-by-step
    chain on the oracle bit for bit (cvt_color.cpp:39-135, resize_naive.cpp,
    normalize_naive.cpp:74-90)."""
    import vacv_amd as V
    codes = [(V.COLOR_YUV2BGR_NV21, True, False), (V.COLOR_YUV2BGR_NV12, False, False),
             (V.COLOR_YUV2RGB_NV21, True, True), (V.COLOR_YUV2RGB_NV12, False, True)]
    rng = np.random.default_rng(20260421)
    for t in range(16):
        code, v_first, rgb = codes[t % 4]
        h, w = 2 * int(rng.integers(1, 300)), 2 * int(rng.integers(1, 500))
        f = rng.uniform(0.1, 2.5, 2)
        ho, wo = max(1, int(h * f[0])), max(1, int(w * f[1]))
        yuv = np.stack([rng.integers(0, 256, (h * 3 // 2, w), dtype=np.uint8) for _ in range(2)])
        ydev = to_dev(yuv, dev)
        bgr = host(ops.cvt_color(ydev, code))
        bgrn = host(ops.cvt_color_normalize(ydev, code, MEAN, STD))
        what = f"code {code} {w}x{h} -> {wo}x{ho}"
        for k in range(2):
            want = oracle.yuv420sp_to_bgr(yuv[k], v_first=v_first, rgb=rgb)
            assert_same(bgr[k], want, what + " cvt")
            assert_same(bgrn[k], oracle.normalize(oracle.u8_to_f32(want), MEAN, STD), what + " cvt normalize")
        for layout, chw in ((V.NHWC, False), (V.NCHW, True)):
            got = host(ops.cvt_color_resize_normalize(ydev, wo, ho, MEAN, STD, code, layout=layout))
            for k in range(2):
                assert_same(got[k], _yuv_chain(oracle, yuv[k], wo, ho, v_first, rgb, 0, MEAN, STD, chw=chw),
                            what + f" resize normalize chw={chw}")


@pytest.mark.parametrize("v_first,rgb", [(True, False), (False, True)])
def test_cvt_color_resize(ops, dev, oracle, v_first, rgb):
    import vacv_amd as V
    code = {(True, False): V.COLOR_YUV2BGR_NV21, (False, True): V.COLOR_YUV2RGB_NV12}[(v_first, rgb)]
    rng = np.random.default_rng(29)
    cases = [((36, 50), (17, 11)), ((144, 176), (64, 48)), ((120, 160), (224, 224)), ((1080, 1920), (640, 360)),
             ((1080, 1920), (224, 224)), ((4, 4), (3, 5)), ((360, 640), (640, 360)),
             # point-sampling geometries (odd integer steps: every tap weight 2048)
             # on 64-column blocks: 3x to 320x120, 5x to 100x50
             ((360, 960), (320, 120)), ((250, 500), (100, 50))]
    for (h, w), (wo, ho) in cases:
        yuv = np.stack([rng.integers(0, 256, (h * 3 // 2, w), dtype=np.uint8) for _ in range(2)])
        ydev = to_dev(yuv, dev)
        for mode in (0, 1, 2):
            got = host(ops.cvt_color_resize(ydev, wo, ho, code, mode=mode))
            for k in range(2):
                assert_same(got[k], _yuv_chain(oracle, yuv[k], wo, ho, v_first, rgb, mode, u8=True),
                            f"u8 nhwc {h}x{w}->{wo}x{ho} mode {mode}")
        got = host(ops.cvt_color_resize(ydev, wo, ho, code, layout=V.NCHW))
        for k in range(2):
            assert_same(got[k], _yuv_chain(oracle, yuv[k], wo, ho, v_first, rgb, 0, chw=True, u8=True), "u8 nchw")
        got = host(ops.cvt_color_resize(ydev, wo, ho, code, dtype=__import__("torch").float32))
        for k in range(2):
            assert_same(got[k], _yuv_chain(oracle, yuv[k], wo, ho, v_first, rgb, 0), "f32 nhwc")
        for layout, chw in ((V.NCHW, True), (V.NHWC, False)):
            got = host(ops.cvt_color_resize_normalize(ydev, wo, ho, MEAN, STD, code, layout=layout))
            for k in range(2):
                assert_same(got[k], _yuv_chain(oracle, yuv[k], wo, ho, v_first, rgb, 0, MEAN, STD, chw=chw),
                            f"normalize {'nchw' if chw else 'nhwc'} {h}x{w}->{wo}x{ho}")
        # auto statistics: per-image exact stats of the resized image
        got = host(ops.cvt_color_resize_normalize(ydev, wo, ho, code=code))
        for k in range(2):
            r = _yuv_chain(oracle, yuv[k], wo, ho, v_first, rgb, 0, u8=True)
            m, s = oracle.mean_stddev_exact(r)
            want = oracle.hwc_to_chw(oracle.normalize(oracle.u8_to_f32(r), m, s))
            assert_same(got[k], want, "auto stats")


def test_cvt_color_resize_batch_and_pitch(ops, dev, oracle):
    """Full-size batch (64 x NV21 1080p -> 224x224 CHW fp32, one launch): images
    across the batch match the oracle chain; a pitched NCHW destination (a
    slice of a wider buffer) gets the same values."""
    import torch
    import vacv_amd as V
    g = torch.Generator(device=dev)
    g.manual_seed(11)
    yuv = torch.randint(0, 256, (64, 1620, 1920), dtype=torch.uint8, device=dev, generator=g)
    out = ops.cvt_color_resize_normalize(yuv, 224, 224, MEAN, STD)
    for k in (0, 31, 63):
        want = _yuv_chain(oracle, host(yuv[k]), 224, 224, True, False, 0, MEAN, STD, chw=True)
        assert_same(host(out[k]), want, f"batch image {k}")
    big = torch.full((2, 3, 230, 240), -7.0, dtype=torch.float32, device=dev)
    view = big[:, :, 3:227, 5:229]
    ops.cvt_color_resize_normalize(yuv[:2], 224, 224, MEAN, STD, out=view)
    assert torch.equal(view, out[:2])
    assert bool((big[:, :, :3] == -7.0).all()) and bool((big[:, :, :, :5] == -7.0).all())
    # the column-stationary kernel (yuv_cols_kernel, default where the
    # destination's block rows are 16-byte aligned) and the row-major one
    # (VACV_TUNE_RESIZE_DIRECT = 2) agree bit for bit: the bench workload
    # (640x360 NCHW fp32), NHWC fp32 / u8, NCHW u8, a two-tap geometry
    for wo, ho, layout, kw in ((640, 360, V.NCHW, {}), (640, 360, V.NHWC, {}), (1280, 720, V.NCHW, {}),
                               (300, 200, V.NHWC, {})):
        for fn in (lambda: ops.cvt_color_resize_normalize(yuv[:8], wo, ho, MEAN, STD, layout=layout),
                   lambda: ops.cvt_color_resize(yuv[:8], wo, ho, layout=layout)):
            a = fn()
            with ops.tuning(RESIZE_DIRECT=2):
                b = fn()
            # 64-column blocks instead of the 128-column ones (CW = 2) of the
            # odd-step geometries (1080p -> 640x360)
            with ops.tuning(RESIZE_TILE_W=64):
                c = fn()
            # the point-sampling instance (odd integer steps) against the
            # blending one (RESIZE_DIRECT = 3)
            with ops.tuning(RESIZE_DIRECT=3):
                e = fn()
            torch.cuda.synchronize(dev)
            assert torch.equal(a, b), f"{wo}x{ho} layout {layout}: {(a != b).sum().item()} values differ"
            assert torch.equal(a, c), f"{wo}x{ho} layout {layout} 64-column blocks: {(a != c).sum().item()} differ"
            assert torch.equal(a, e), f"{wo}x{ho} layout {layout} without POINT: {(a != e).sum().item()} differ"
    # the fused op equals the unfused GPU chain (cvt_color, resize_normalize, layout)
    bgr = ops.cvt_color(yuv[:4])
    chain = ops.change_layout(ops.resize_normalize(bgr, 224, 224, MEAN, STD), V.NCHW)
    assert torch.equal(chain, out[:4])
    del yuv, out, big
    torch.cuda.empty_cache()


# ---------------------------------------------------------------------------
# normalize / stats

def test_normalize_and_stats(ops, dev, oracle):
    from vacv_amd import NCHW
    rng = np.random.default_rng(23)
    for (h, w), c in [((144, 176), 3), ((20, 30), 1), ((33, 17), 4), ((1080, 1920), 3)]:
        img = synthetic_image(h + w, h, w, c)
        img = img if c > 1 else img[..., None]
        f = (img.astype(np.float32) * np.float32(0.9) + rng.standard_normal(img.shape).astype(np.float32)).astype(np.float32)
        mean = np.arange(c, dtype=np.float32) * 7 + 50
        std = np.arange(c, dtype=np.float32) * 3 + 40
        got = host(ops.normalize(to_dev(f[None], dev), mean, std))[0]
        assert_same(got, oracle.normalize(f, mean, std), "normalize f32")
        got = host(ops.normalize(to_dev(img[None], dev), mean, std))[0]
        assert_same(got, oracle.normalize(oracle.u8_to_f32(img), mean, std), "normalize u8")
        # exact statistics: u8 sums are integers (bit-exact)
        sums = host(ops.channel_sums(to_dev(img[None], dev)))[0].reshape(-1)
        assert np.array_equal(sums, oracle.channel_sums(img)), "u8 channel sums exact"
        m, s = ops.mean_stddev(to_dev(img[None], dev))
        me, se = oracle.mean_stddev_exact(img)
        assert_same(host(m)[0], me, "mean exact")
        assert_same(host(s)[0], se, "std exact")
        # fp32: fp64 sums in a different order -> tolerance vs exact double
        mf, sf = ops.mean_stddev(to_dev(f[None], dev))
        ref = f.reshape(-1, c).astype(np.float64)
        assert np.allclose(host(mf)[0], ref.mean(0), rtol=0, atol=1e-3)          # |dmean| <= 1e-3
        assert np.allclose(host(sf)[0], ref.std(0), rtol=1e-4, atol=0)           # |dstd|/std <= 1e-4
        # reference fp32 sequential stats (normalize_naive.cpp:7-72) vs ours
        rm, rs = oracle.mean_stddev_ref(f)
        assert np.allclose(host(mf)[0], rm, rtol=0, atol=0.5)
        assert np.allclose(host(sf)[0], rs, rtol=1e-2)
        # auto normalize = normalize with our exact stats
        got = host(ops.normalize(to_dev(img[None], dev)))[0]
        assert_same(got, oracle.normalize(oracle.u8_to_f32(img), me, se), "normalize auto")
        chw = np.ascontiguousarray(f.transpose(2, 0, 1))
        got = host(ops.normalize(to_dev(chw[None], dev), mean, std, layout=NCHW))[0]
        for k in range(c):
            assert_same(got[k], oracle.normalize(chw[k], mean[k:k + 1], std[k:k + 1]), "normalize chw")
        mc, sc = ops.mean_stddev(to_dev(chw[None], dev), layout=NCHW)
        assert np.allclose(host(mc)[0], ref.mean(0), atol=1e-3)


def test_batch_global_stats(ops, dev, oracle):
    imgs = np.stack([synthetic_image(300 + k, 224, 224, 3) for k in range(5)])
    sums = host(ops.channel_sums(to_dev(imgs, dev), per_image=False))[0].reshape(-1)
    assert np.array_equal(sums, oracle.channel_sums(imgs.reshape(-1, 224, 3)))


# ---------------------------------------------------------------------------
# crop / layout / dtype

def test_crop_layout_dtype(ops, dev, oracle):
    import torch
    from vacv_amd import NCHW, NHWC
    for (h, w), c in [((360, 640), 3), ((37, 53), 1), ((21, 33), 4), ((144, 176), 3)]:
        img = synthetic_image(h * w, h, w, c)
        img = img if c > 1 else img[..., None]
        src = to_dev(np.stack([img, img[::-1].copy()]), dev)
        for rect in [(0, 0, w // 2, h // 2), (10.7, 20.2, w - 1.5, h - 3.9), (3, 1, 8, 6)]:
            if int(np.float32(rect[2]) - np.float32(rect[0])) < 1 or int(np.float32(rect[3]) - np.float32(rect[1])) < 1:
                continue
            got = host(ops.crop(src, rect))
            l, t = int(rect[0]), int(rect[1])
            cw, chh = int(np.float32(rect[2]) - np.float32(rect[0])), int(np.float32(rect[3]) - np.float32(rect[1]))
            want = oracle.crop(img if c > 1 else img[..., 0], l, t, cw, chh)
            assert_same(got[0] if c > 1 else got[0, ..., 0], want, f"crop {rect}")
        chw = host(ops.change_layout(src, NCHW))
        assert_same(chw[0], oracle.hwc_to_chw(img), "hwc->chw")
        back = host(ops.change_layout(to_dev(chw, dev), NHWC, layout=NCHW))
        assert_same(back[0], img, "chw->hwc")
        got = host(ops.crop(to_dev(chw, dev), (2, 3, 9, 11), layout=NCHW))
        assert_same(got[0], oracle.crop(chw[0], 2, 3, 7, 8, chw=True), "crop chw")
        f = host(ops.change_dtype(src, torch.float32))
        assert_same(f[0], oracle.u8_to_f32(img), "u8->f32")
        ff = (np.random.default_rng(1).standard_normal(img.shape) * 200 + 100).astype(np.float32)
        u = host(ops.change_dtype(to_dev(ff[None], dev), torch.uint8))
        assert_same(u[0], oracle.f32_to_u8(ff), "f32->u8")
    # fp32 / fp16 layout change
    x = np.random.default_rng(2).standard_normal((2, 17, 19, 3)).astype(np.float32)
    assert_same(host(ops.change_layout(to_dev(x, dev), NCHW)), x.transpose(0, 3, 1, 2), "f32 layout")
    x16 = x.astype(np.float16)
    assert_same(host(ops.change_layout(to_dev(x16, dev), NCHW)), x16.transpose(0, 3, 1, 2), "f16 layout")


def test_error_statuses(ops, dev):
    import torch
    import vacv_amd as V
    x = torch.zeros((1, 8, 8, 3), dtype=torch.uint8, device=dev)
    with pytest.raises(V.VacvError) as e:
        ops.crop(x, (4, 4, 12, 12))           # rect outside the image
    assert e.value.status == V._lib.ERR_INVALID_ARG
    with pytest.raises(V.VacvError) as e:
        ops.resize(x, 4, 4, interpolation=5)  # no such mode (resize.cpp:46-49 recurses on it)
    assert e.value.status == V._lib.ERR_UNSUPPORTED
    with pytest.raises(V.VacvError) as e:  # BORDER_ISOLATED has no meaning for warp_affine
        ops.warp_affine(x, np.eye(2, 3, dtype=np.float32), 8, 8, border_mode=16)
    assert e.value.status == V._lib.ERR_UNSUPPORTED
    with pytest.raises(V.VacvError) as e:  # TRANSPARENT in place
        ops.warp_affine(x, np.eye(2, 3, dtype=np.float32), 8, 8, border_mode=V.BORDER_TRANSPARENT, out=x)
    assert e.value.status == V._lib.ERR_INVALID_ARG
    with pytest.raises(V.VacvError):
        ops.resize(x, 4, 4, interpolation=V.INTER_CUBIC, out=torch.zeros((1, 4, 4, 3), dtype=torch.uint8, device=dev))
    with pytest.raises(ValueError):
        ops.normalize(x.float(), mean=[1, 2, 3])
    odd = torch.zeros((1, 9, 5), dtype=torch.uint8, device=dev)
    with pytest.raises(V.VacvError):
        ops.cvt_color(odd)


def test_cvt_color_opencv_codes(ops, dev, oracle):
    """The cvt_color codes the reference hands to cv::cvtColor (cvt_color.cpp:
    139-141): NV12/NV21 -> RGBA/BGRA (94-97) and YV12 -> BGR (99) with OpenCV
    2.4's BT.601 fixed point, GRAY2BGR (8) for u8 and fp32 -- bit-exact with
    the oracle's restatement (parity unpinned: no OpenCV runs here), batches,
    odd block counts, a pitched 4-channel destination (byte stores) and the
    saturating extremes."""
    import torch
    from vacv_amd import (COLOR_GRAY2BGR, COLOR_YUV2BGR_YV12, COLOR_YUV2BGRA_NV12, COLOR_YUV2BGRA_NV21,
                          COLOR_YUV2RGBA_NV12, COLOR_YUV2RGBA_NV21)
    rng = np.random.default_rng(91)
    # widths 616 / 1032: the wave-per-row-pair kernel's partial last wave (13
    # and 1 live lanes: the odd-lane BGR tail); it is also checked against
    # the lane-strided 8 x 2 kernel (RESIZE_DIRECT = 2)
    for h, w in ((6, 10), (72, 130), (10, 616), (8, 1032), (1080, 1920)):
        yuv = rng.integers(0, 256, (3, h * 3 // 2, w), dtype=np.uint8)
        yuv[0, :h // 2] = 255
        yuv[0, h:] = 0
        for code in (COLOR_YUV2RGBA_NV12, COLOR_YUV2BGRA_NV12, COLOR_YUV2RGBA_NV21, COLOR_YUV2BGRA_NV21,
                     COLOR_YUV2BGR_YV12):
            a = ops.cvt_color(to_dev(yuv, dev), code)
            got = host(a)
            for k in range(3):
                assert_same(got[k], oracle.yuv420_cv(yuv[k], code), f"cvt code {code} {w}x{h} image {k}")
            with ops.tuning(RESIZE_DIRECT=2):
                b = ops.cvt_color(to_dev(yuv, dev), code)
            assert torch.equal(a, b), f"cvt code {code} {w}x{h}: the two 8 x 2 kernels differ"
    # a pitched RGBA destination (rows not 8-byte aligned: the byte-store path)
    yuv = rng.integers(0, 256, (2, 30, 26), dtype=np.uint8)
    big = torch.zeros((2, 20, 31, 4), dtype=torch.uint8, device=dev)
    view = big[:, 0:20, 1:27]
    from vacv_amd import _lib as L
    from vacv_amd.ops import NHWC, check, describe
    import ctypes
    src = to_dev(yuv, dev)
    check("vacv_cvt_color", L.load().vacv_cvt_color(ctypes.byref(describe(src.unsqueeze(-1), NHWC)),
                                                    ctypes.byref(describe(view, NHWC)), COLOR_YUV2BGRA_NV21, None))
    g = host(big)
    for k in range(2):
        assert_same(g[k, :, 1:27], oracle.yuv420_cv(yuv[k], COLOR_YUV2BGRA_NV21), "pitched rgba")
    g[:, :, 1:27] = 0
    assert not g.any(), "cvt_color wrote outside the window"
    # 53 wide: elementwise (unaligned rows); 64 / 1920 / 1104 wide: units with
    # vector loads and stores (gray_x_kernel: a wave per row's 64 units, the
    # last one partial at 1920 and 1104); a pitched source (a 61-wide slice of 64)
    for dt in (np.uint8, np.float32):
        for shape, crop in (((2, 37, 53), 53), ((2, 36, 64), 64), ((2, 8, 1920), 1920), ((2, 5, 1104), 1104),
                            ((2, 9, 64), 61)):
            full = (rng.integers(0, 256, shape).astype(dt) * (dt(0.5) if dt == np.float32 else 1)).astype(dt)
            gray = full[:, :, :crop]
            a = ops.cvt_color(to_dev(full, dev)[:, :, :crop], COLOR_GRAY2BGR)
            got = host(a)
            for k in range(2):
                assert_same(got[k], oracle.gray_to_bgr(np.ascontiguousarray(gray[k])), f"gray2bgr {dt} {shape} {crop}")
            with ops.tuning(RESIZE_DIRECT=2):  # gray_kernel: lanes write their own pixels
                b = ops.cvt_color(to_dev(full, dev)[:, :, :crop], COLOR_GRAY2BGR)
            assert torch.equal(a, b), f"gray2bgr {dt} {shape} {crop}: the unit kernels differ"


def test_warp_flags_nearest_and_inverse_map(ops, dev, oracle):
    """cv::warpAffine flags the reference hands to OpenCV (warp_affine.cpp:
    114-118): INTER_NEAREST (OpenCV 2.4's fixed point, restated in
    oracle_warp_affine_nn: bit-exact, parity unpinned) with every border mode,
    u8 / fp32, NHWC c = 1 / 3 / 4 and NCHW, the normalize epilogue; and
    WARP_INVERSE_MAP: INTER_LINEAR with m already inverted equals the forward
    call bit for bit (the same float inverse) on every kernel, cfg4's size
    included."""
    import torch
    from vacv_amd import INTER_NEAREST, NCHW, WARP_INVERSE_MAP
    mats = [ops.rotation_matrix(0.7, 33.0, (40, 30, 50, 35)),
            np.array([0.3, 0.05, 70.0, -0.04, 0.35, -20.0], np.float32),
            np.array([-1.6, 0.1, 150.0, 0.2, 1.3, -9.5], np.float32)]
    bv = (7, 200, 31, 99)
    for c in (1, 3, 4):
        img = synthetic_image(400 + c, 61, 83, c).reshape(61, 83, c)
        f = img.astype(np.float32) * np.float32(0.75) + np.float32(0.125)
        for m in mats:
            for inv in (False, True):
                mm = oracle.invert_affine(m) if inv else m
                fl = INTER_NEAREST | (WARP_INVERSE_MAP if inv else 0)
                # 97 wide: byte-aligned rows for c = 1, 3 (the per-pixel kernel);
                # 96 wide (and c = 4): 4-pixel units with packed stores
                for mode in (0, 1, 2, 3, 4):
                    for dw, dh in ((97, 71), (96, 70)):
                        got = host(ops.warp_affine(to_dev(img[None], dev), mm, dw, dh, flags=fl, border_mode=mode,
                                                   border_value=bv))[0].reshape(dh, dw, c)
                        want = oracle.warp_affine_nn(img, mm, dw, dh, inverse_map=inv, border_mode=mode,
                                                     border=bv).reshape(dh, dw, c)
                        assert_same(got, want, f"nearest c{c} {dw}x{dh} inv={inv} mode {mode}")
                gotf = host(ops.warp_affine(to_dev(f[None], dev), mm, 97, 71, flags=fl, border_mode=1))[0]
                wantf = oracle.warp_affine_nn(f, mm, 97, 71, inverse_map=inv, border_mode=1)
                assert_same(gotf.reshape(71, 97, c), wantf.reshape(71, 97, c), f"nearest f32 c{c}")
                prev = np.full((71, 97, c), 77, np.uint8)
                out = to_dev(prev[None], dev)
                ops.warp_affine(to_dev(img[None], dev), mm, 97, 71, flags=fl, border_mode=5, out=out)
                want = oracle.warp_affine_nn(img, mm, 97, 71, inverse_map=inv, border_mode=5,
                                             dst=prev if c > 1 else prev[..., 0]).reshape(71, 97, c)
                assert_same(host(out)[0].reshape(71, 97, c), want, f"nearest transparent c{c}")
    img = synthetic_image(410, 61, 83, 3)
    chw = np.ascontiguousarray(img.transpose(2, 0, 1))
    got = host(ops.warp_affine(to_dev(chw[None], dev), mats[0], 97, 71, flags=INTER_NEAREST, layout=NCHW))[0]
    for k in range(3):
        assert_same(got[k], oracle.warp_affine_nn(chw[k], mats[0], 97, 71), "nearest chw")
    gn = host(ops.warp_affine_normalize(to_dev(img[None], dev), mats[0], 97, 71, MEAN, STD, flags=INTER_NEAREST))[0]
    want = oracle.normalize(oracle.u8_to_f32(oracle.warp_affine_nn(img, mats[0], 97, 71)), MEAN, STD)
    assert_same(gn, want, "nearest normalize")
    # WARP_INVERSE_MAP with INTER_LINEAR: the LDS-staged kernel (cfg4 size) and the gathers
    imgs = np.stack([synthetic_image(420 + k, 720, 1280, 3) for k in range(2)])
    src = to_dev(imgs, dev)
    rot = ops.rotation_matrix(0.9, 15.0, (640, 360, 640, 360))
    inv = oracle.invert_affine(rot)
    for knob in (4, 2, 0):
        with ops.tuning(WARP_KERNEL=knob):
            a = ops.warp_affine(src, rot, 1280, 720)
            b = ops.warp_affine(src, inv, 1280, 720, flags=1 | WARP_INVERSE_MAP)
        assert torch.equal(a, b), f"inverse map kernel {knob}"
    assert_same(host(b)[1], oracle.warp_affine(imgs[1], rot, 1280, 720), "inverse map vs oracle")
