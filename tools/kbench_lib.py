#!/usr/bin/env python3
"""tools/kbench.py against another build of libvacv_hip.so (diagnosis builds,
e.g. `make LIB=lib_dbg1 OBJ=build_dbg1 EXTRA=-DVACV_FRAMES_DBG=1`):
  python tools/kbench_lib.py <dir with libvacv_hip.so> <kbench args...>"""
import runpy
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "arm-neon-opencv_amd"))
import vacv_amd._lib as L  # noqa: E402

L.HIP_LIB = Path(sys.argv[1]).resolve() / "libvacv_hip.so"
sys.argv = [str(REPO / "tools" / "kbench.py")] + sys.argv[2:]
runpy.run_path(sys.argv[0], run_name="__main__")
