# GPU step: the driver-shaped bench line (20 steps, 5 warmup) and one-off C4 / C2 workload lines into
# gpurun_out/<tag>/ (a baseline for A/Bs on the same box generation).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-base}
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/$TAG/metric.json 2> gpurun_out/$TAG/metric.err || exit $?
cut -c1-200 gpurun_out/$TAG/metric.json
for w in $WORKLOADS; do
  timeout -k 10 400 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG/$w.json 2> gpurun_out/$TAG/$w.err || exit $?
  cut -c1-200 gpurun_out/$TAG/$w.json
done
