#!/usr/bin/env python3
"""VGPRs, spills and occupancy of every pass kernel in pt_kernels.hip (compile-only, no GPU).

    python tools/regcheck.py [extra hipcc flags...]
"""
import re
import subprocess
import sys

cmd = ["/opt/rocm/bin/hipcc", "-x", "hip", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
       "-fno-fast-math", "-fno-slp-vectorize", *sys.argv[1:], "-Iinclude", "-Ipathtracerwithcuda_amd/csrc", "-c",
       "pathtracerwithcuda_amd/csrc/pt_kernels.hip", "-o", "/tmp/regcheck.o", "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"remark: Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+(VGPRs|VGPRs Spill|SGPRs Spill|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]): (\d+)", line)
    if m and cur:
        rows[cur][m.group(1).split(" [")[0]] = int(m.group(2))
for k, v in rows.items():
    if "pass_kernel" in k:
        print(f"{k[:60]:60s} vgpr {v.get('VGPRs')} vspill {v.get('VGPRs Spill')} scratch {v.get('ScratchSize')} occ {v.get('Occupancy')}")
