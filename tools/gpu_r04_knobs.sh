# Round-4 step: bench-knob sweep at the current kernel (metric, the driver's --steps 20 --warmup 5, two rounds
# over the list), then the reference ABI with a moving camera and with a still one.
#   gpurun --timeout 1200 -- bash tools/gpu_r04_knobs.sh <tag> "VAR=a" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-knobs}
shift
mkdir -p gpurun_out/$TAG
for r in 1 2; do
for v in "$@"; do
  n=${v//[= ]/_}
  env $v timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/$TAG/b_${n}_$r.json 2> gpurun_out/$TAG/b_${n}_$r.err || exit $?
  echo "$v $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], d['config']['ms_per_frame_latency'])" gpurun_out/$TAG/b_${n}_$r.json)" | tee -a gpurun_out/$TAG/summary.txt
done
done
if [ -n "$ABI" ]; then
  timeout -k 10 300 python tools/abi_rate.py --moving --frames 8 > gpurun_out/$TAG/abi_moving.json 2> gpurun_out/$TAG/abi_moving.err || exit $?
  cat gpurun_out/$TAG/abi_moving.json
  timeout -k 10 300 python tools/abi_rate.py --frames 4 > gpurun_out/$TAG/abi_still.json 2> gpurun_out/$TAG/abi_still.err || exit $?
  cat gpurun_out/$TAG/abi_still.json
  PT_ABI_PASS_CACHE=0 timeout -k 10 300 python tools/abi_rate.py --moving --frames 8 > gpurun_out/$TAG/abi_moving_nocache.json 2> gpurun_out/$TAG/abi_moving_nocache.err || exit $?
  cat gpurun_out/$TAG/abi_moving_nocache.json
fi
