cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/uprof_defer
for t in 6 16; do
PT_LIBDIR=$GRAFT_REPO_ROOT/pathtracerwithcuda_amd/lib PT_TRI_MIN=$t timeout -k 10 120 python tools/uprof.py > gpurun_out/uprof_defer/base_t$t.txt 2>&1 || exit $?
PT_LIBDIR=$GRAFT_REPO_ROOT/pathtracerwithcuda_amd/lib_defer PT_TRI_MIN=$t timeout -k 10 120 python tools/uprof.py > gpurun_out/uprof_defer/defer_t$t.txt 2>&1 || exit $?
done
tail -n 30 gpurun_out/uprof_defer/*.txt
