"""Shared test setup.

Markers
  gpu  -- needs an MI355X (HIP device); these are the parity tests proper and
          call the product through its C ABI (lib/libvacv_hip.so).
Everything unmarked runs on the CPU: the oracle against the committed golden
fixtures, host-side logic, the C ABI's exported surface, and the multi-rank
(gloo) statistics exchange.
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

import numpy as np
import pytest

REPO = Path(__file__).resolve().parent.parent
PKG = REPO / "arm-neon-opencv_amd"
for p in (REPO / "oracle", PKG, REPO):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))

GOLDEN = REPO / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); parity tests through the C ABI")


@pytest.fixture(scope="session")
def oracle():
    from oracle import Oracle
    return Oracle()


@pytest.fixture(scope="session")
def golden():
    meta = json.loads((GOLDEN / "digests.json").read_text())
    arrays = np.load(GOLDEN / "small_cases.npz")
    return meta, arrays


@pytest.fixture(scope="session")
def hip_device():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import vacv_amd
    lib = vacv_amd._lib
    if not lib.HIP_LIB.exists():
        lib.build()
    lib.load()
    return torch.device("cuda:0")


def load_bgr(name: str) -> np.ndarray:
    from PIL import Image
    im = Image.open(GOLDEN / "res" / name).convert("RGB")
    return np.ascontiguousarray(np.asarray(im, dtype=np.uint8)[:, :, ::-1])
