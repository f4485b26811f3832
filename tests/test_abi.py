"""The C ABI without a GPU: library loads, exports exactly what
include/vacv_hip.h declares, and the host-only entry points (matrices,
argument validation, status strings) behave like the reference."""
from __future__ import annotations

import ctypes
import re
import subprocess

import numpy as np
import pytest


@pytest.fixture(scope="module")
def lib():
    import vacv_amd
    if not vacv_amd._lib.HIP_LIB.exists():
        vacv_amd._lib.build()
    return vacv_amd._lib.load()


def header_functions():
    import vacv_amd
    text = vacv_amd._lib.HEADER.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(vacv_[a-z0-9_]+)\s*\(", text)))


def test_header_matches_exports_and_binding(lib):
    import vacv_amd
    declared = header_functions()
    assert len(declared) >= 18
    assert declared == sorted(vacv_amd._lib.SIGNATURES), "ctypes binding out of sync with the header"
    out = subprocess.run(["nm", "-D", "--defined-only", str(vacv_amd._lib.HIP_LIB)], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r" T (vacv_[a-z0-9_]+)$", out, flags=re.M))
    assert set(declared) <= exported, set(declared) - exported
    assert exported <= set(declared), f"undeclared exports: {exported - set(declared)}"


def test_version_and_status(lib):
    import vacv_amd
    hdr = vacv_amd._lib.HEADER.read_text()
    declared = int(re.search(r"#define VACV_ABI_VERSION (\d+)", hdr).group(1))
    assert vacv_amd._lib.ABI_VERSION == declared, "binding and header disagree on the ABI version"
    assert lib.vacv_abi_version() == declared
    # the binding's tuning keys are the header's enum, and the library's
    count = int(re.search(r"VACV_TUNE_COUNT = (\d+)", hdr).group(1))
    assert len(vacv_amd._lib.TUNE) == count and sorted(vacv_amd._lib.TUNE.values()) == list(range(count))
    for name, key in vacv_amd._lib.TUNE.items():
        assert re.search(rf"VACV_TUNE_{name} = {key},", hdr), name
    assert lib.vacv_set_tuning(count - 1, -1) == 0 and lib.vacv_set_tuning(count, -1) == -1
    assert lib.vacv_status_string(0) == b"ok"
    assert lib.vacv_status_string(-2) == b"unsupported"


def test_rotation_and_inverse_match_oracle(lib, oracle):
    from vacv_amd import ops
    for scale, rot, aux in [(0.9, 15.0, (640, 360, 640, 360)), (1.073914, -3.314525,
                                                                 (738.518372, 537.672852, 204.766998, 73.329681)),
                            (2.0, 90.0, (0, 0, 0, 0)), (0.3, -179.5, (12.5, -3, 7, 1e3))]:
        assert np.array_equal(ops.rotation_matrix(scale, rot, aux), oracle.rotation_matrix(scale, rot, aux))
    rng = np.random.default_rng(0)
    for _ in range(200):
        m = rng.uniform(-3, 3, 6).astype(np.float32)
        assert np.array_equal(ops.invert_affine(m), oracle.invert_affine(m))
    assert np.array_equal(ops.invert_affine(np.zeros(6, np.float32)), np.zeros(6, np.float32))


def test_argument_validation_without_device(lib):
    """Descriptor checks happen before any HIP call."""
    from vacv_amd._lib import VacvImage
    null = VacvImage(None, 1, 8, 8, 3, 2, 1, 0, 0, 0)
    good = VacvImage(0x1000, 1, 8, 8, 3, 2, 1, 0, 0, 0)
    assert lib.vacv_crop(ctypes.byref(null), ctypes.byref(good), 0, 0, None) == -1
    bad_dtype = VacvImage(0x1000, 1, 8, 8, 3, 9, 1, 0, 0, 0)
    assert lib.vacv_resize(ctypes.byref(bad_dtype), ctypes.byref(good), 1, 0, None) == -2
    small_pitch = VacvImage(0x1000, 1, 8, 8, 3, 2, 1, 10, 0, 0)
    assert lib.vacv_resize(ctypes.byref(small_pitch), ctypes.byref(good), 1, 0, None) == -1
    dst = VacvImage(0x2000, 1, 4, 4, 3, 2, 1, 0, 0, 0)
    assert lib.vacv_crop(ctypes.byref(good), ctypes.byref(dst), 6, 0, None) == -1      # rect outside
    assert lib.vacv_resize(ctypes.byref(good), ctypes.byref(dst), 5, 0, None) == -2    # no such mode (LANCZOS4 = 4 runs)
    dst3 = VacvImage(0x2000, 1, 3, 3, 3, 2, 1, 0, 0, 0)
    assert lib.vacv_resize_scaled(ctypes.byref(good), ctypes.byref(dst3), 3, 0, 0.0, 0.5, None) == -1  # fx <= 0
    assert lib.vacv_resize_scaled(ctypes.byref(good), ctypes.byref(dst3), 1, 0, 0.5, 0.5, None) == -2  # LINEAR
    up = VacvImage(0x2000, 1, 16, 16, 3, 2, 1, 0, 0, 0)
    assert lib.vacv_resize(ctypes.byref(good), ctypes.byref(dst), 1, 7, None) == -1    # bad mode
    m = (ctypes.c_float * 6)(1, 0, 0, 0, 1, 0)
    assert lib.vacv_warp_affine(ctypes.byref(good), ctypes.byref(dst), m, 1, 16, None, None) == -2  # BORDER_ISOLATED
    assert lib.vacv_warp_affine(ctypes.byref(good), ctypes.byref(dst), m, 2, 0, None, None) == -2  # CUBIC
    yuv = VacvImage(0x1000, 1, 7, 9, 1, 2, 1, 0, 0, 0)
    bgr = VacvImage(0x2000, 1, 7, 6, 3, 2, 1, 0, 0, 0)
    assert lib.vacv_cvt_color(ctypes.byref(yuv), ctypes.byref(bgr), 93, None) == -1   # odd width
    assert lib.vacv_cvt_color(ctypes.byref(yuv), ctypes.byref(bgr), 98, None) == -2   # YUV2RGB_YV12 (not in cv.h)
    assert lib.vacv_cvt_color(ctypes.byref(yuv), ctypes.byref(bgr), 8, None) == -1    # GRAY2BGR: dst is not (7, 9, 3)
    rgba = VacvImage(0x2000, 1, 8, 6, 3, 2, 1, 0, 0, 0)
    yuv8 = VacvImage(0x1000, 1, 8, 9, 1, 2, 1, 0, 0, 0)
    assert lib.vacv_cvt_color(ctypes.byref(yuv8), ctypes.byref(rgba), 96, None) == -1  # RGBA needs 4 channels
    f = VacvImage(0x1000, 1, 8, 8, 3, 0, 1, 0, 0, 0)
    mean = (ctypes.c_float * 3)(1, 2, 3)
    assert lib.vacv_normalize(ctypes.byref(good), ctypes.byref(f), mean, None, None) == -1  # one of mean/std
    assert lib.vacv_image_bytes(ctypes.byref(good)) == 8 * 8 * 3
    chw = VacvImage(0x1000, 2, 5, 4, 3, 0, 0, 0, 0, 0)
    assert lib.vacv_image_bytes(ctypes.byref(chw)) == 5 * 4 * 3 * 4


def test_no_oracle_in_product():
    """The product library and package never reference the oracle."""
    import vacv_amd
    root = vacv_amd._lib.PKG_ROOT
    for p in list(root.rglob("*.py")) + list(root.rglob("*.hip")) + list(root.rglob("*.cpp")) + list(root.rglob("*.h*")):
        text = p.read_text(errors="ignore")
        assert "import oracle" not in text and "from oracle" not in text and "vacv_oracle" not in text, p
    out = subprocess.run(["nm", "-D", str(vacv_amd._lib.HIP_LIB)], capture_output=True, text=True, check=True).stdout
    assert "oracle_" not in out and "ref_" not in out
