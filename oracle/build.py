"""ORACLE — TEST INFRASTRUCTURE ONLY. Compiles the C restatement (ocv_ref.c) with gcc.

-ffp-contract=off and the x86-64 baseline ISA (SSE2, no FMA) keep every double operation the
separately rounded IEEE op written in the source, which is what the restated OpenCV code does.
"""
from __future__ import annotations

import subprocess
from pathlib import Path

HERE = Path(__file__).resolve().parent
OUT = HERE / "_build"
LIB = OUT / "libocvref.so"


def build_oracle(force: bool = False) -> Path:
    OUT.mkdir(exist_ok=True)
    src = HERE / "ocv_ref.c"
    if force or not LIB.exists() or src.stat().st_mtime > LIB.stat().st_mtime:
        cmd = ["gcc", "-O2", "-std=c11", "-ffp-contract=off", "-fPIC", "-shared", "-Wall", "-o", str(LIB), str(src), "-lm"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"oracle build failed: {' '.join(cmd)}\n{r.stderr}")
    return LIB


if __name__ == "__main__":
    print(build_oracle(force=True))
