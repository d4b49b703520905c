# End-of-batch policy: the last K frames of the timed batch on the whole grid (PT_BENCH_LAST_FULL=K), N = 1,
# the driver's --steps 20 --warmup 5, two rounds.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/lastfull
for r in 1 2; do for k in 0 1 2 3; do
  PT_BENCH_LAST_FULL=$k timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/lastfull/k${k}_$r.json 2>/dev/null || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('last_full', sys.argv[2], d['value'], 'Mrays/s', d['ms_per_step'], 'ms/frame')" gpurun_out/lastfull/k${k}_$r.json $k
done; done
