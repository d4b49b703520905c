# Builds the PT_DUP diagnostic libraries (one phase run twice on opaque copies of its inputs) into
# pathtracerwithcuda_amd/lib_dup{1..4}: 1 shading, 2 box stage, 3 triangle stage, 4 path generation.
# The phase duplicates are not in the product source: they come back with profiles/r06/pruned/experiment_arms.patch
# applied in reverse to a copy of csrc/. Compile-only (runs here); tools/gpu_dup.sh measures them.
set -e
cd "$(dirname "$0")/.."
SRC=$(mktemp -d)
trap 'rm -rf "$SRC"' EXIT
cp -r pathtracerwithcuda_amd/csrc "$SRC/csrc"
cp -r include "$SRC/include"  # the sources include ../../include
(cd "$SRC" && mkdir -p pathtracerwithcuda_amd && mv csrc pathtracerwithcuda_amd/ &&
 patch -s -p1 -R < "$OLDPWD/profiles/r06/pruned/experiment_arms.patch")
for k in 1 2 3 4; do
  PT_CSRC=$SRC/pathtracerwithcuda_amd/csrc PT_LIBDIR=$PWD/pathtracerwithcuda_amd/lib_dup$k PT_EXTRA_FLAGS="-DPT_DUP=$k" \
    python -c "from pathtracerwithcuda_amd.build import build; build(force=True)" &
done
wait
ls -la pathtracerwithcuda_amd/lib_dup*/libpt_hip.so
