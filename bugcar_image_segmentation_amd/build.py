"""Build the native engine libbugseg.so in-tree for gfx950 (hipcc, no torch extension machinery).

The shared library is plain HIP C++ behind the C ABI of include/bugseg.h; it links only the HIP
runtime (libamdhip64.so.7). Loaded after `import torch`, it binds to the same HIP runtime torch
uses, so torch device pointers and streams can be handed straight to it.
"""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
OBJ = PKG / "_build"
LIB = PKG / "libbugseg.so"
SOURCES = ["conv_kernels.hip", "cls_kernels.hip", "init_kernels.hip", "bneck_kernels.hip", "bneck2_kernels.hip", "up_kernels.hip", "prep_kernels.hip",
           "bev_kernels.hip", "deeplab_kernels.hip", "bugseg_runtime.cpp", "deeplab_runtime.cpp"]
HEADERS = [CSRC / "bugseg_internal.h", CSRC / "deeplab_internal.h", CSRC / "mfma_common.h", CSRC / "cls_common.h", ROOT / "include" / "bugseg.h"]
ARCH = os.environ.get("BUGSEG_OFFLOAD_ARCH", "gfx950")
# per-source code-generation options. The class layer: MFMA results in ordinary VGPRs instead of AGPRs
# (removes the accumulator copies in and out of AGPRs; round 6, fp32 B = 64: 113.6 -> 107.5 us per launch;
# on every source it measured neutral-to-slower, so only here)
SOURCE_FLAGS = {"cls_kernels.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form=1"]}


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.sep not in c or os.path.exists(c)):
            return c
    raise RuntimeError("hipcc not found")


def _stale(target: Path, deps) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(Path(d).stat().st_mtime > t for d in deps)


def build_native(force: bool = False, verbose: bool = False, stamps: bool = False, variant: str = "",
                 defines=()) -> Path:
    """stamps=True: the debug variant libbugseg_stamps.so (-DBUGSEG_STAMPS: in-kernel phase clocks,
    scripts/stamp_probe.py); variant="name" with defines=("-DX=1", ...): an A/B build
    libbugseg_<name>.so (loaded through BUGSEG_LIB by measurement scripts). Neither is loaded by the
    product path."""
    if stamps:
        variant, defines = "stamps", ("-DBUGSEG_STAMPS", *defines)
    obj_dir = OBJ / variant if variant else OBJ
    lib = PKG / f"libbugseg_{variant}.so" if variant else LIB
    obj_dir.mkdir(parents=True, exist_ok=True)
    hipcc = _hipcc()
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function",
             f"-I{ROOT / 'include'}", f"-I{CSRC}", *defines]
    jobs = []
    for s in SOURCES:
        src = CSRC / s
        obj = obj_dir / (s + ".o")
        if force or _stale(obj, [src, *HEADERS]):
            lang = ["-x", "hip"] if s.endswith(".hip") else []
            jobs.append((obj, [hipcc, *flags, *SOURCE_FLAGS.get(s, []), *lang, "-c", str(src), "-o", str(obj)]))

    def run(job):
        obj, cmd = job
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        return obj

    with ThreadPoolExecutor(max_workers=min(4, max(1, len(jobs)))) as ex:
        list(ex.map(run, jobs))
    objs = [obj_dir / (s + ".o") for s in SOURCES]
    if force or jobs or _stale(lib, objs):
        tmp = lib.with_suffix(".so.tmp")
        cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(tmp), *map(str, objs)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, lib)
    return lib


if __name__ == "__main__":
    var = next((a.split("=", 1)[1] for a in sys.argv if a.startswith("--variant=")), "")
    print(build_native(force="--force" in sys.argv, verbose=True, stamps="--stamps" in sys.argv, variant=var,
                       defines=tuple(a for a in sys.argv if a.startswith("-D"))))
