#!/usr/bin/env python3
"""Per-kernel VGPR/SGPR/spill/occupancy table from hipcc -Rpass-analysis output."""
import re
import subprocess
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "fft-convolution_amd/csrc/kernels.hip"
flt = sys.argv[2] if len(sys.argv) > 2 else ""
out = subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-c", src, "-o",
                      "/tmp/_res.o", "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"remark: Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[[^\]]*\])?: (\d+)", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = m.group(2)
for k, v in rows.items():
    if flt and flt not in k:
        continue
    dm = subprocess.run(["llvm-cxxfilt", k], capture_output=True, text=True).stdout.strip() if False else k
    print(f"{dm[:75]:75s} vgpr={v.get('VGPRs','?'):>4} sgpr={v.get('SGPRs','?'):>4} vspill={v.get('VGPRs Spill','?')} "
          f"sspill={v.get('SGPRs Spill','?')} occ={v.get('Occupancy','?')} lds={v.get('LDS Size','?')}")
