timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread 2>&1 | tail -2 && mkdir -p gpurun_out/acc && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/acc/t -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/acc/b.json 2>/dev/null && python3 -c "
import csv,glob,json
for f in glob.glob('gpurun_out/acc/t/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'accumulate' in r['Name'] or 'pass_kernel_u' in r['Name']: print(r['Name'][:40], r['AverageNs'])
d=json.load(open('gpurun_out/acc/b.json')); print(d['value'], d['ms_per_step'])"
