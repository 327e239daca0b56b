"""The C-ABI library builds for gfx950, loads, and exports every symbol include/bugseg.h declares.
No compute calls: this runs on the CPU-only build container too."""
import ctypes
import re
import subprocess
from pathlib import Path

import pytest

from bugcar_image_segmentation_amd import _native as N

ROOT = Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "bugseg.h"


def declared_symbols():
    text = HEADER.read_text()
    return sorted(set(re.findall(r"\b(bugseg_[a-z_0-9]+)\s*\(", text)))


def test_header_declares_the_abi():
    syms = declared_symbols()
    assert set(N.EXPORTED) == set(syms), (set(N.EXPORTED) ^ set(syms))


def test_library_exports_every_declared_symbol(native_lib):
    for s in declared_symbols():
        assert hasattr(native_lib, s), s
    out = subprocess.run(["nm", "-D", "--defined-only", str(N.LIB_PATH)], capture_output=True, text=True).stdout
    for s in declared_symbols():
        assert re.search(rf"\bT {s}$", out, re.M), f"{s} not exported as a text symbol"


def test_library_carries_gfx950_code(native_lib):
    # the embedded HIP fat binary names its code objects by target triple + processor
    assert b"amdgcn-amd-amdhsa--gfx950" in N.LIB_PATH.read_bytes()


def test_version_and_error_paths(native_lib):
    assert native_lib.bugseg_version() == 100
    # argument validation happens before any device work
    assert native_lib.bugseg_create(0, 7, ctypes.byref(ctypes.c_void_p())) == N.EINVAL
    assert b"precision" in native_lib.bugseg_last_error(None)
    assert native_lib.bugseg_create(0, 0, None) == N.EINVAL
    assert native_lib.bugseg_destroy(None) == N.OK


def test_no_cpu_fallback_without_gpu(native_lib):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from bugcar_image_segmentation_amd.models import ENET
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        ENET(weights=b"BSG1")
