#!/bin/bash
# Print VGPR / SGPR / spill / occupancy of every kernel in pt_kernels.hip (compile-only, no GPU).
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math -fno-slp-vectorize $EXTRA \
  -Iinclude -Ipathtracerwithcuda_amd/csrc -c pathtracerwithcuda_amd/csrc/pt_kernels.hip -o /tmp/regcheck.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 | grep -E "Function Name|VGPRs:|Spill|Occupancy|ScratchSize" \
  | sed 's/.*remark: //; s/ \[-Rpass-analysis=kernel-resource-usage\]//' | paste - - - - - - - | grep -E "pass_kernel"
