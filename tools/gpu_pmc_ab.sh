# SQ counters of the bench kernel for two builds (one frame in flight): gpurun -- bash tools/gpu_pmc_ab.sh <tag> <libdir> <libdir>
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
mkdir -p gpurun_out/$TAG
for d in "$@"; do
  PT_BENCH_INFLIGHT=1 PT_LIBDIR=$GRAFT_REPO_ROOT/pathtracerwithcuda_amd/$d timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/$TAG/$d -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline > gpurun_out/$TAG/$d.log 2>&1 || exit $?
  echo "== $d"; python3 tools/pmc_summary.py gpurun_out/$TAG/$d
done
