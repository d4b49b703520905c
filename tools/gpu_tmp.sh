mkdir -p gpurun_out/wl
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/wl/metric.json 2> gpurun_out/wl/metric.err || exit $?
timeout -k 10 300 python bench.py --workload c3 --steps 2 --warmup 1 > gpurun_out/wl/c3.json 2> gpurun_out/wl/c3.err || exit $?
timeout -k 10 400 python bench.py --workload c4 --steps 1 --warmup 1 > gpurun_out/wl/c4.json 2> gpurun_out/wl/c4.err || exit $?
timeout -k 10 500 python bench.py --workload c5 --steps 1 --warmup 0 > gpurun_out/wl/c5.json 2> gpurun_out/wl/c5.err || exit $?
for f in metric c3 c4 c5; do python3 -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['config']; print(sys.argv[2], d['value'], 'Mrays/s', d['ms_per_step'], 'ms/frame', c['segments_per_frame'], 'seg/frame', d['roofline']['frac'])" gpurun_out/wl/$f.json $f; done
