# PT_DUP phase-cost experiment (pt_kernels.hip): for the product build and each diagnostic build that
# runs one phase twice, one timed bench and one SQ counter pass. The differences to the product
# build are the VALU instructions and wall time of that phase.
#   gpurun -- bash tools/gpu_dup.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-dup}
mkdir -p gpurun_out/$TAG
for d in lib lib_dup1 lib_dup2 lib_dup3 lib_dup4; do
  L=/root/repo/pathtracerwithcuda_amd/$d
  PT_LIBDIR=$L timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/$TAG/bench_$d.json 2>/dev/null || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], 'Mrays/s', d['roofline']['avg_launch_ms'], 'ms/launch')" gpurun_out/$TAG/bench_$d.json $d
  PT_LIBDIR=$L timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/$TAG/$d -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/$TAG/pmc_$d.log 2>&1 || { tail -5 gpurun_out/$TAG/pmc_$d.log; exit 1; }
done
for d in lib lib_dup1 lib_dup2 lib_dup3 lib_dup4; do echo "== $d"; python3 tools/pmc_summary.py gpurun_out/$TAG/$d; done > gpurun_out/$TAG/summary.txt 2>&1
cat gpurun_out/$TAG/summary.txt
