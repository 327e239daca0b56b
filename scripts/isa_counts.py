"""Instruction mix per kernel of a device assembly file (hipcc -S --cuda-device-only): v_ instructions,
MFMAs, the split-f16 conversions (v_fma_mix*, v_cvt_pk_f16_f32), LDS and global memory ops.

usage: python scripts/isa_counts.py file.s [name-substring]"""
import re
import sys

PATS = {"v_": r"^\s+v_", "mfma": r"v_mfma", "mix": r"v_fma_mix", "cvtpk": r"v_cvt_pk_f16_f32", "ds_read": r"ds_read",
        "ds_write": r"ds_write", "vmem_ld": r"(buffer|global)_load", "vmem_st": r"(buffer|global)_store"}
s = open(sys.argv[1]).read()
flt = sys.argv[2] if len(sys.argv) > 2 else ""
for m in re.finditer(r"^(_Z\w+):[^\n]*\n(.*?)^\s+s_endpgm", s, re.S | re.M):
    name, body = m.group(1), m.group(2)
    if flt not in name:
        continue
    counts = " ".join(f"{k}:{len(re.findall(p, body, re.M)):5d}" for k, p in PATS.items())
    print(f"{name[:64]:64s} {counts}")
