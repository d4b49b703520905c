"""Per-kernel HBM traffic from two separate rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE).

    python tools/traffic_summary.py gpurun_out/<tag> profiles/<round> [--workload KEY --kernel SUBSTR]

Writes <out>/pmc_summary.json (mean KB per dispatch per kernel) and, with --workload, records the
dominant kernel's per-launch HBM bytes in profiles/traffic.json (read by bench.py as roofline.traffic).
Corrections per MI355X_MICROARCH.md §HBM: counters are in KB (x1024); on gfx950 FETCH_SIZE reports
half the bytes of 16-B-per-lane reads, so it is doubled; WRITE_SIZE is taken as is.
"""
import argparse
import csv
import glob
import json
import os

ap = argparse.ArgumentParser()
ap.add_argument("src")
ap.add_argument("out")
ap.add_argument("--workload", default=None)
ap.add_argument("--kernel", default="pass_kernel_u<6, false, false, 2, true>")
ap.add_argument("--round", default=None)
args = ap.parse_args()

agg = {}
for sub, counter in (("pmc_fetch", "FETCH_SIZE"), ("pmc_write", "WRITE_SIZE"), ("pmc_sq", "SQ_INSTS_VALU")):
    for f in glob.glob(os.path.join(args.src, sub, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            k = r["Kernel_Name"].split("(")[0]
            agg.setdefault(k, {}).setdefault(counter, []).append(float(r["Counter_Value"]))

summary = {k: {c: {"dispatches": len(v), ("mean" if c.startswith("SQ_") else "mean_kb"): sum(v) / len(v)}
                 for c, v in d.items()} for k, d in agg.items()}
os.makedirs(args.out, exist_ok=True)
json.dump(summary, open(os.path.join(args.out, "pmc_summary.json"), "w"), indent=1)

if args.workload:
    hits = [k for k in summary if args.kernel in k]
    if len(hits) != 1:
        raise SystemExit(f"kernel {args.kernel!r} matched {hits}")
    k = hits[0]
    fetch = summary[k]["FETCH_SIZE"]["mean_kb"] * 1024 * 2
    write = summary[k]["WRITE_SIZE"]["mean_kb"] * 1024
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles", "traffic.json")
    d = json.load(open(path)) if os.path.exists(path) else {}
    d[args.workload] = {
        "hbm_bytes_per_launch": round(fetch + write),
        "fetch_bytes": round(fetch),
        "write_bytes": round(write),
        "source": f"{os.path.relpath(args.out)}/pmc_summary.json (rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, "
                  "separate passes; FETCH_SIZE x2 gfx950 correction, KB x1024)",
        "kernel": k,
        # wave-level VALU instructions per launch (pmc_sq pass), for bench.py's VALU-busy figure
        "valu_insts_per_launch": (round(summary[k]["SQ_INSTS_VALU"]["mean"]) if "SQ_INSTS_VALU" in summary[k]
                                  else None),
        "round": args.round or os.path.basename(os.path.normpath(args.out)),
    }
    rec = d[args.workload]
    # the timed mode's kernel (frame groups: the MULTI instance), from the pmc_sq_group8 pass of tools/gpu.sh
    # profile (tools/share_render.py --group 8: one launch of 8 frames), VALU per frame
    # pmc_sq_group<G>: one launch of G frames (G = 8 for the 1-GPU frame; min(8 N, 20) for a 1/N share, as the
    # driver's 20 steps run it)
    for gdir in sorted(glob.glob(os.path.join(args.src, "pmc_sq_group*"))):
        if not os.path.isdir(gdir):
            continue
        G = int(os.path.basename(gdir)[len("pmc_sq_group"):])
        multi = {}
        for f in glob.glob(os.path.join(gdir, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if r["Counter_Name"] == "SQ_INSTS_VALU" and "pass_kernel_u<" in r["Kernel_Name"] and ", true>" in r["Kernel_Name"]:
                    multi.setdefault(r["Kernel_Name"].split("(")[0], []).append(float(r["Counter_Value"]))
        if multi:
            mk, mv = next(iter(multi.items()))
            rec["valu_insts_per_frame_timed"] = round(sum(mv) / len(mv) / G)
            rec["valu_insts_per_frame_timed_source"] = (f"{os.path.relpath(args.out)}/pmc_sq_group{G}.json: SQ_INSTS_VALU "
                                                        f"of {mk} (the MULTI instance the timed launches run) over one "
                                                        f"{G}-frame launch / {G}")
            json.dump({mk: {"SQ_INSTS_VALU_per_launch": sum(mv) / len(mv), "frames_per_launch": G}},
                      open(os.path.join(args.out, f"pmc_sq_group{G}.json"), "w"), indent=1)
    # the solo launch's average duration in rocprofv3's kernel trace (one frame in flight)
    for f in glob.glob(os.path.join(args.src, "trace", "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if args.kernel in r["Name"]:
                rec["rocprof_avg_launch_ms"] = round(float(r["AverageNs"]) / 1e6, 4)
                rec["rocprof_avg_launch_source"] = (f"{os.path.relpath(args.out)}/kernel_stats_one_in_flight.csv "
                                                    f"({r['Calls']} solo launches)")
                import shutil
                shutil.copy(f, os.path.join(args.out, "kernel_stats_one_in_flight.csv"))
    for f in glob.glob(os.path.join(args.src, "trace_timed", "**", "*kernel_stats.csv"), recursive=True):
        import shutil
        shutil.copy(f, os.path.join(args.out, "kernel_stats_timed_mode.csv"))
    json.dump(d, open(path, "w"), indent=1)
    print(k, d[args.workload])
