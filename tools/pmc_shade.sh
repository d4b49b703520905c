set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in "PT_SHADE_MIN=40" "PT_SHADE_MIN=24" "PT_SHADE_MIN=56"; do
  d=gpurun_out/pmc2/$(echo $v | tr '= ' '__')
  mkdir -p $d
  env $v timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_THREAD_CYCLES_VALU SQ_INSTS_LDS --output-format csv -d $d -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $d.log 2>&1 || exit $?
  echo "== $v"; python3 tools/pmc_summary.py $(dirname $d) 2>/dev/null | grep -A9 "pass_kernel_u" | head -0
done
python3 - <<'PY'
import csv, glob, os
for d in sorted(glob.glob("gpurun_out/pmc2/*/")):
    agg = {}
    for f in glob.glob(d + "**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "pass_kernel_u" in r["Kernel_Name"]:
                agg.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    print(os.path.basename(d.rstrip("/")), {k: "%.4g" % (sum(v)/len(v)) for k, v in sorted(agg.items())})
PY
