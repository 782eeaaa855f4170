#!/usr/bin/env python3
"""Per-kernel resources (SGPR, VGPR, scratch, LDS, occupancy) of a HIP source for gfx950.
usage: python tools/kres.py bwt-mtf-huffman-compressor_amd/csrc/bwt.hip [name-filter]
SGPR > 80 costs residency on gfx950 (MI355X_MICROARCH.md: 82-96 -> 7 waves/SIMD)."""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
out = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "--offload-device-only",
                      "-c", "-o", "/dev/null", src, "-Rpass-analysis=kernel-resource-usage"],
                     capture_output=True, text=True).stderr
cur = None
rows = []
for line in out.splitlines():
    m = re.search(r"remark: (.*)", line)
    if not m:
        continue
    t = m.group(1)
    if t.startswith("Function Name:"):
        name = t.split(":", 1)[1].strip()
        short = re.search(r"(k_[A-Za-z0-9_]+?)(E|I|$)", name)
        tmpl = re.search(r"ILj(\d+)ELj(\d+)E", name)
        cur = {"name": (short.group(1) if short else name) + (f"<{tmpl.group(1)},{tmpl.group(2)}>" if tmpl else "")}
        rows.append(cur)
    elif cur is not None:
        k, _, v = t.partition(":")
        cur[k.strip()] = v.strip().split()[0] if v.strip() else ""
for r in rows:
    if flt and flt not in r["name"]:
        continue
    print(f"{r['name']:34s} sgpr {r.get('TotalSGPRs','?'):>4} vgpr {r.get('VGPRs','?'):>4} agpr {r.get('AGPRs','?'):>3} "
          f"scratch {r.get('ScratchSize [bytes/lane]','?'):>4} lds {r.get('LDS Size [bytes/block]','?'):>6} "
          f"occ {r.get('Occupancy [waves/SIMD]','?')}")
