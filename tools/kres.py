#!/usr/bin/env python3
"""Per-kernel register / LDS / occupancy summary of t2_kernels.hip (hipcc -Rpass-analysis), e.g.
python tools/kres.py [-Dflags...]"""
import re
import subprocess
import sys

import os
src = os.environ.get("KRES_SRC", "gr-dvbt2ll_amd/csrc/t2_kernels.hip")
cmd = ["/opt/rocm/bin/hipcc", "-std=c++17", "-O3", "-fPIC", "--offload-arch=gfx950", "-munsafe-fp-atomics",
       "-Rpass-analysis=kernel-resource-usage", "-c", src, "-o", "/tmp/kres.o"] + sys.argv[1:]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark:\s+(Function Name|VGPRs|AGPRs|TotalSGPRs|SGPRs Spill|VGPRs Spill|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|"
                  r"LDS Size \[bytes/block\]): (\S+)", line)
    if not m:
        continue
    k, v = m.groups()
    if k == "Function Name":
        cur = {"name": subprocess.run(["c++filt", v], capture_output=True, text=True).stdout.strip()[:60]}
        rows.append(cur)
    else:
        cur["VGPRs_spill" if k == "VGPRs Spill" else k.split()[0]] = v
for r in rows:
    print("%-60s vgpr %4s agpr %3s sgpr %4s (spill %3s) vspill %3s scratch %4s occ %2s" % (
        r["name"], r.get("VGPRs"), r.get("AGPRs"), r.get("TotalSGPRs"), r.get("SGPRs"), r.get("VGPRs_spill"), r.get("ScratchSize"), r.get("Occupancy")))
