# Builds the PT_DUP diagnostic libraries (pt_kernels.hip: one phase run twice on opaque copies) into
# pathtracerwithcuda_amd/lib_dup{1..4}: 1 shading, 2 box stage, 3 triangle stage, 4 path generation.
# Compile-only (runs here); tools/gpu_dup.sh measures them.
set -e
cd "$(dirname "$0")/.."
for k in 1 2 3 4; do
  PT_LIBDIR=$PWD/pathtracerwithcuda_amd/lib_dup$k PT_EXTRA_FLAGS="-DPT_DUP=$k" python -c "from pathtracerwithcuda_amd.build import build; build(force=True)" &
done
wait
ls -la pathtracerwithcuda_amd/lib_dup*/libpt_hip.so
