"""Per-kernel register / spill / occupancy table for one HIP source (compile-only, no GPU).

    python scripts/resusage.py bugcar_image_segmentation_amd/csrc/bneck_kernels.hip [-DNAME=VALUE ...]
"""
import re
import subprocess
import sys
import tempfile
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(src, *defines):
    with tempfile.TemporaryDirectory() as d:
        cmd = ["/opt/rocm/bin/hipcc", *defines, "--offload-arch=gfx950", "-O3", "-std=c++17",
               f"-I{ROOT}/include", f"-I{ROOT}/bugcar_image_segmentation_amd/csrc", "-x", "hip", "-c", src,
               "-o", os.path.join(d, "o.o"), "-Rpass-analysis=kernel-resource-usage"]
        r = subprocess.run(cmd, capture_output=True, text=True)
    rows, cur = [], None
    for line in r.stderr.splitlines():
        m = re.search(r"remark:\s+(.*?) \[-Rpass", line)
        if not m:
            continue
        t = m.group(1)
        if t.startswith("Function Name:"):
            cur = {"name": t.split(":", 1)[1].strip()}
            rows.append(cur)
        elif cur is not None and ":" in t:
            k, v = t.split(":", 1)
            cur[k.strip()] = v.strip()
    for c in rows:
        print(f"{c.get('VGPRs', '?'):>4} vgpr {c.get('AGPRs', '?'):>3} agpr  spill v{c.get('VGPRs Spill', '?')} "
              f"s{c.get('SGPRs Spill', '?')}  occ {c.get('Occupancy [waves/SIMD]', '?')}  "
              f"lds {c.get('LDS Size [bytes/block]', '?'):>6}  {c['name']}")
    if r.returncode:
        print(r.stderr[-3000:])
        sys.exit(r.returncode)


if __name__ == "__main__":
    main(sys.argv[1], *sys.argv[2:])
