"""The drop-in boundary: the reference's own test harness,
/root/reference/src/test/src/** (CMakeLists.txt:4-24 builds it as va_cv_ut),
compiles UNCHANGED against this build's source-compatible headers and its
va_cv:: / vision:: symbols all resolve in lib/libvacv.so.

How: the harness sources are copied into a temporary tree (never into the
repository) laid out as the reference's src/, whose common/, cv/ and util/
are symlinks to arm-neon-opencv_amd/src -- so the harness's relative
includes ("../../../cv/cv.h") land on this build's headers, exactly as a
maintainer swapping the library would see them.  They are compiled with the
reference's own flags (-std=c++14, src/test/CMakeLists.txt:11) and OpenCV
2.4.13.4's HEADERS from thirdparty/.  OpenCV's prebuilt binaries are never
linked, loaded or run: the link step is replaced by a symbol check -- every
symbol the harness objects leave undefined is either defined by libvacv.so or
belongs to OpenCV (cv::) / the C and C++ runtimes.

CPU only; skipped where /root/reference is absent (the GPU box)."""
from __future__ import annotations

import os
import re
import shutil
import subprocess
from pathlib import Path

import pytest

REF = Path("/root/reference")
REPO = Path(__file__).resolve().parent.parent
LIB = REPO / "arm-neon-opencv_amd" / "lib" / "libvacv.so"
OCV_INC = REF / "thirdparty" / "opencv_2.4.13.4" / "linux-x86_64" / "include"

pytestmark = pytest.mark.skipif(not (REF / "src" / "test" / "src").is_dir() or not OCV_INC.is_dir(),
                                reason="the reference tree is not present here")


def _nm(args):
    return subprocess.run(["nm"] + args, capture_output=True, text=True, check=True).stdout


def test_reference_harness_builds_against_vacv(tmp_path):
    if not LIB.exists():
        subprocess.run(["make", "-s", "-C", str(REPO / "arm-neon-opencv_amd"), "-j8"], check=True)
    src = tmp_path / "src"
    shutil.copytree(REF / "src" / "test" / "src", src / "test" / "src")
    for d in ("common", "cv", "util"):
        os.symlink(REPO / "arm-neon-opencv_amd" / "src" / d, src / d)
    cpps = sorted((src / "test" / "src").rglob("*.cpp"))
    assert len(cpps) >= 9, cpps  # test_main, cv_profile and the seven impl/test_*.cpp
    objs = []
    for cpp in cpps:
        obj = tmp_path / (cpp.stem + ".o")
        r = subprocess.run(["g++", "-std=c++14", "-c", str(cpp), "-o", str(obj), "-I", str(OCV_INC),
                            "-w"], capture_output=True, text=True)
        assert r.returncode == 0, f"{cpp.relative_to(src)} does not compile against vacv:\n{r.stderr[-3000:]}"
        objs.append(obj)
    undefined = set()
    for o in objs:
        undefined |= {l.strip()[2:] for l in _nm(["-C", "-u", str(o)]).splitlines() if l.strip().startswith("U ")}
    defined_here = set()
    for o in objs:
        defined_here |= {l.split(" ", 2)[-1] for l in _nm(["-C", "--defined-only", str(o)]).splitlines() if l.strip()}
    lib_syms = {l.split(" ", 2)[-1] for l in _nm(["-C", "-D", "--defined-only", str(LIB)]).splitlines() if l.strip()}
    missing = []
    for sym in sorted(undefined - defined_here):
        if sym in lib_syms:
            continue
        if sym.startswith(("cv::", "std::", "__cxa", "__gxx", "_Unwind", "__stack_chk", "operator ", "vtable for __cxxabiv1",
                           "typeinfo for std::", "vtable for std::", "__dso_handle", "_GLOBAL_OFFSET_TABLE_")):
            continue
        if re.fullmatch(r"[a-z_][a-z0-9_]*(@.*)?", sym) or sym.startswith("__"):
            continue  # C runtime (printf, memcpy, clock, ...)
        missing.append(sym)
    assert not missing, "harness symbols libvacv.so does not define:\n" + "\n".join(missing)
    # and the harness really uses the operator API (not an empty build)
    used = {s for s in undefined if s.startswith(("va_cv::", "vision::"))}
    for name in ("va_cv::resize", "va_cv::warp_affine", "va_cv::crop", "va_cv::normalize", "va_cv::cvt_color",
                 "vision::Tensor::change_layout", "vision::Tensor::change_dtype"):
        assert any(s.startswith(name) for s in used), name
