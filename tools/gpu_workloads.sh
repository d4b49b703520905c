# GPU step: the bench line at the other BASELINE.json configurations (bench.py --workload c2|c3|c4|c5,
# 1 GPU, three frames in flight) into gpurun_out/<tag>/.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-workloads}
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python bench.py --workload c2 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/$TAG/c2.json || exit $?
cut -c1-220 gpurun_out/$TAG/c2.json
timeout -k 10 300 python bench.py --workload c3 --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/$TAG/c3.json || exit $?
cut -c1-220 gpurun_out/$TAG/c3.json
timeout -k 10 400 python bench.py --workload c4 --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG/c4.json || exit $?
cut -c1-220 gpurun_out/$TAG/c4.json
timeout -k 10 500 python bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG/c5.json || exit $?
cut -c1-220 gpurun_out/$TAG/c5.json
