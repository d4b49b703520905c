# Round-3 N1 experiment (profiles/r03/coal): the walk step's records as coalesced loads staged through LDS.
#   git apply profiles/r03/coal/coalesced_lds_walk.patch
#   PT_LIBDIR=$PWD/pathtracerwithcuda_amd/lib_coal PT_EXTRA_FLAGS=-DPT_COAL=1 python -m pathtracerwithcuda_amd.build
#   gpurun -- bash tools/gpu_coal.sh     (parity with lib_coal, A/B against lib, vector-memory and SQ counters)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/coal2
PT_LIBDIR=$GRAFT_REPO_ROOT/pathtracerwithcuda_amd/lib_coal timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/coal2/pytest_coal.log 2>&1 || { tail -30 gpurun_out/coal2/pytest_coal.log; exit 1; }
tail -1 gpurun_out/coal2/pytest_coal.log
ROUNDS=3 bash tools/gpu_libab4.sh coal2 lib lib_coal || exit $?
PT_LIBDIR=$GRAFT_REPO_ROOT/pathtracerwithcuda_amd/lib_coal PMC_ENV=PT_BENCH_INFLIGHT=1 bash tools/gpu_pmc.sh coal2/pmc "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_TA_BUSY_sum TD_TC_STALL_sum TD_TD_BUSY_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum GRBM_GUI_ACTIVE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT" | grep -A12 "pass_kernel_u"
