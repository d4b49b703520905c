"""Lane-weighted VALU of the bench kernel (verdict r02 item 3): SQ_INSTS_VALU counts a wave-instruction
as full however many of its 64 lanes are active. The PT_DUP builds split the instructions by phase
(tools/gpu_dup.sh: one phase run twice, the difference is its count) and the PT_UPROF counters give each
phase's active lanes (tools/uprof.py); the weighted count is sum(VALU_phase x lanes_phase / 64).

    python tools/lane_weighted.py <dup summary dir> <uprof json> [--workload KEY]

Phases and their lanes: shading (lanes per shading batch), box stage (walking lanes per walk step),
triangle stage (lanes per triangle batch), path generation (lanes per refill that started a path), and
the rest ("control": refills, segment starts, mesh changes, loop bookkeeping) at the lanes holding a path
per wave round. With --workload the result is recorded in profiles/traffic.json for bench.py.
"""
import argparse
import glob
import json
import os
import csv

ap = argparse.ArgumentParser()
ap.add_argument("dup")
ap.add_argument("uprof")
ap.add_argument("--workload", default=None)
ap.add_argument("--kernel", default="pass_kernel_u<8, false, 0, false>")
args = ap.parse_args()


def valu(d):
    vals = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == "SQ_INSTS_VALU" and args.kernel in r["Kernel_Name"]:
                vals.append(float(r["Counter_Value"]))
    if not vals:
        raise SystemExit(f"no SQ_INSTS_VALU for {args.kernel!r} under {d}")
    return sum(vals) / len(vals)


base = valu(os.path.join(args.dup, "lib"))
phase = {name: valu(os.path.join(args.dup, f"lib_dup{k}")) - base
         for k, name in ((1, "shading"), (2, "box"), (3, "triangle"), (4, "generation"))}
phase["control"] = base - sum(phase.values())
u = json.load(open(args.uprof))
lanes = {"shading": u["lanes_per_shade_batch"], "box": u["lanes_per_walk_step"], "triangle": u["lanes_per_tri_batch"],
         "generation": u["lanes_per_gen_batch"], "control": u["live_lanes_per_round"]}
weighted = sum(phase[k] * lanes[k] / 64.0 for k in phase)
out = {"valu_insts_per_launch": round(base), "valu_lane_weighted_per_launch": round(weighted),
       "lane_efficiency": round(weighted / base, 4),
       "phases": {k: {"valu": round(phase[k]), "share": round(phase[k] / base, 4), "lanes": lanes[k]} for k in phase}}
print(json.dumps(out, indent=1))
if args.workload:
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles", "traffic.json")
    d = json.load(open(path))
    d.setdefault(args.workload, {})["valu_lane_weighted_per_launch"] = out["valu_lane_weighted_per_launch"]
    d[args.workload]["lane_weighted_source"] = (f"{os.path.relpath(args.dup)} (PT_DUP phase split) x "
                                                f"{os.path.relpath(args.uprof)} (PT_UPROF lanes per phase)")
    json.dump(d, open(path, "w"), indent=1)
