# The one GPU-side runner (replaces the per-round tools/gpu_r0x_*.sh scripts). Every step writes under
# gpurun_out/<tag>/ and stops at the first failure (no retries).
#
#   gpurun -- bash tools/gpu.sh tests <tag> [pytest args...]     # default: the whole -m gpu suite
#   gpurun -- bash tools/gpu.sh ab <tag> <variant>...            # bench A/B, ROUNDS (2) alternating rounds
#        variant = base | lib:<dir under pathtracerwithcuda_amd/> | env:VAR=a,VAR2=b | lib:<dir>+env:VAR=a
#        BENCH_ARGS (default: the driver's --steps 20 --warmup 5) and TESTS=1 (parity of each lib first)
#   gpurun -- bash tools/gpu.sh workloads <tag>                   # the metric line + c1..c5 (+ c4 --medium-bound)
#   gpurun -- bash tools/gpu.sh profile <tag>                     # rocprof traces + PMC passes + PT_UPROF + PT_DUP
#   gpurun -- bash tools/gpu.sh wlprofile <tag>                   # c1..c5 (+ c4 --medium-bound): trace + PMC passes
#   gpurun -- bash tools/gpu.sh orbit <tag>                       # static vs per-frame camera, with and without groups
#   gpurun -- bash tools/gpu.sh rccl <tag>                        # bench --rccl + its rocprofv3 RCCL API trace
#   gpurun -- bash tools/gpu.sh rehearsal <tag>                   # N = 2..8 gloo ranks on the one GPU (bench.py's
#                                                                  # N > 1 path; tools/gpu_multirank_rehearsal.sh)
#   gpurun -- bash tools/gpu.sh shares <tag>                      # rank 0's share of N = 2, 4, 8 under PMC
#                                                                  # (tools/gpu_share_pmc.sh) for the N > 1 roofline
#   gpurun -- bash tools/gpu.sh tile <tag> [tile_scaling.py args] # per-rank share timing on one GPU
#   gpurun -- bash tools/gpu.sh abi <tag>                         # the reference ABI's PCIe-inclusive rate
# Summaries for profiles/: python tools/traffic_summary.py / tools/pmc_summary.py / tools/lane_weighted.py.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
STEP=$1
TAG=$2
shift 2
T=gpurun_out/$TAG
mkdir -p $T
PKG=$PWD/pathtracerwithcuda_amd
line() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], d['value'], 'Mrays/s', d['ms_per_step'], 'ms/frame', r['avg_launch_ms'], 'ms/launch', 'frac', r['frac'], 'timed', r.get('frac_timed_mode'))" "$1" "$2"; }

# runs bench.py once under a variant spec, appending its JSON line to $T/bench_<name>.json
run_variant() {
  local v=$1 name=$(echo $1 | tr ':=,/+' '_____') libdir="" envs=""
  for part in $(echo $v | tr '+' ' '); do
    case $part in
      base) ;;
      lib:*) libdir=$PKG/${part#lib:} ;;
      env:*) envs=$(echo ${part#env:} | tr ',' ' ') ;;
    esac
  done
  env ${libdir:+PT_LIBDIR=$libdir} $envs timeout -k 10 300 python3 bench.py ${BENCH_ARGS:---steps 20 --warmup 5} \
    --no-cpu-baseline > $T/cur.json 2>> $T/bench_err.log || return $?
  cat $T/cur.json >> $T/bench_$name.json
  line $T/cur.json "$v"
}

case $STEP in
tests)
  if [ $# -gt 0 ]; then args=("$@"); else args=(tests -m gpu); fi
  timeout -k 10 1100 python3 -u -m pytest "${args[@]}" -x -v --timeout 400 --timeout-method thread > $T/pytest_gpu.log 2>&1
  rc=$?; tail -4 $T/pytest_gpu.log; exit $rc ;;
ab)
  if [ -n "$TESTS" ]; then
    for v in "$@"; do
      case $v in lib:*) d=${v#lib:}; d=${d%%+*}
        PT_LIBDIR=$PKG/$d timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 \
          --timeout-method thread > $T/pytest_$d.log 2>&1 || { echo "parity FAILED with $d"; tail -30 $T/pytest_$d.log; exit 1; }
        echo "$d: $(tail -1 $T/pytest_$d.log)" ;;
      esac
    done
  fi
  for r in $(seq ${ROUNDS:-2}); do for v in "$@"; do run_variant $v || exit $?; done; done ;;
workloads)
  timeout -k 10 300 python3 bench.py > $T/bench.json 2> $T/bench.err || exit $?
  line $T/bench.json metric
  for w in c1 c2 c3 c4 c5; do
    timeout -k 10 600 python3 bench.py --workload $w --no-cpu-baseline > $T/wl_$w.json 2> $T/wl_$w.err || exit $?
    line $T/wl_$w.json $w
  done
  timeout -k 10 600 python3 bench.py --workload c4 --medium-bound --no-cpu-baseline > $T/wl_c4_mb.json 2> $T/wl_c4_mb.err || exit $?
  line $T/wl_c4_mb.json c4_medium_bound ;;
profile)
  B="python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-alt-tree"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $T/trace_timed -o run -- $B > $T/trace_timed.log 2>&1 || exit $?
  export PT_BENCH_INFLIGHT=1 PT_BENCH_GROUP=1  # one frame per launch, one at a time: the roofline's solo launch
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $T/trace -o run -- python3 bench.py --steps 10 --warmup 1 --no-cpu-baseline --no-alt-tree > $T/trace.log 2>&1 || exit $?
  P="python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-alt-tree"
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $T/pmc_fetch -o run -- $P > $T/pmc_fetch.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $T/pmc_write -o run -- $P > $T/pmc_write.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $T/pmc_sq -o run -- $P > $T/pmc_sq.log 2>&1 || exit $?
  # the timed mode's own kernel: the MULTI instance over one 8-frame launch
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY --output-format csv -d $T/pmc_sq_group8 -o run -- python3 tools/share_render.py --n 1 --frames 2 --group 8 > $T/pmc_sq_group8.log 2>&1 || exit $?
  unset PT_BENCH_INFLIGHT PT_BENCH_GROUP
  timeout -k 10 120 python3 tools/uprof.py metric > $T/uprof_metric.json 2> $T/uprof_metric.err || exit $?
  if [ -d $PKG/lib_dup1 ]; then bash tools/gpu_dup.sh $TAG/dup > $T/dup.log 2>&1 || exit $?; tail -4 $T/dup.log; fi
  echo profile done ;;
wlprofile)
  # the other configurations' roofline inputs, each workload's solo launch (one frame per launch, one in flight):
  # kernel trace, FETCH_SIZE, WRITE_SIZE and SQ passes; then per workload
  #   python tools/traffic_summary.py gpurun_out/<tag>/<w> profiles/<round>/workloads/<w> --workload <key> --kernel "pass_kernel_u<"
  export PT_BENCH_INFLIGHT=1 PT_BENCH_GROUP=1
  for w in ${WORKLOADS:-c1 c2 c3 c4 c4mb c5}; do
    a="--workload ${w%mb} --no-cpu-baseline --no-alt-tree"; [ "$w" = c4mb ] && a="$a --medium-bound"
    st="--steps 3 --warmup 1"; sp="--steps 1 --warmup 0"
    case $w in c1) st="--steps 40 --warmup 2"; sp="--steps 4 --warmup 0" ;; c5) st="--steps 1 --warmup 0" ;; esac
    mkdir -p $T/$w
    timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $T/$w/trace -o run -- python3 bench.py $a $st > $T/$w/trace.log 2>&1 || exit $?
    timeout -s KILL 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $T/$w/pmc_fetch -o run -- python3 bench.py $a $sp > $T/$w/pmc_fetch.log 2>&1 || exit $?
    timeout -s KILL 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $T/$w/pmc_write -o run -- python3 bench.py $a $sp > $T/$w/pmc_write.log 2>&1 || exit $?
    timeout -s KILL 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $T/$w/pmc_sq -o run -- python3 bench.py $a $sp > $T/$w/pmc_sq.log 2>&1 || exit $?
    echo "$w profiled"
  done ;;
orbit)
  for r in 1 2; do
    for v in "" "--orbit 0.01"; do for g in 8 1; do
      n=$(echo "o${v#--orbit }_g$g" | tr -d ' ')
      PT_BENCH_GROUP=$g timeout -k 10 300 python3 bench.py --no-cpu-baseline $v > $T/cur.json 2>> $T/bench_err.log || exit $?
      cat $T/cur.json >> $T/bench_$n.json; line $T/cur.json $n
    done; done
  done ;;
rccl)
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --rccl > $T/rccl.json 2> $T/rccl.err || exit $?
  line $T/rccl.json rccl
  timeout -k 10 300 rocprofv3 --rccl-trace --kernel-trace --stats --output-format csv -d $T/rccl_trace -o run -- python3 bench.py --no-cpu-baseline --rccl --steps 10 --warmup 2 > $T/rccl_trace.log 2>&1 || exit $? ;;
rehearsal)
  bash tools/gpu_multirank_rehearsal.sh $TAG ;;
shares)
  bash tools/gpu_share_pmc.sh > $T/share_pmc.log 2>&1 || exit $?; tail -20 $T/share_pmc.log ;;
tile)
  timeout -k 10 900 python3 tools/tile_scaling.py "$@" > $T/tile.json 2> $T/tile.err || exit $?; cat $T/tile.json ;;
abi)
  timeout -k 10 300 python3 tools/abi_rate.py > $T/abi_rate.json 2> $T/abi_rate.err || exit $?; cat $T/abi_rate.json
  timeout -k 10 300 python3 tools/abi_rate.py --moving > $T/abi_rate_moving.json 2> $T/abi_rate_moving.err || exit $?
  cat $T/abi_rate_moving.json ;;
*)
  echo "unknown step $STEP"; exit 2 ;;
esac
