"""State-machine occupancy of pass_kernel_u on a benchmark frame (PT_UPROF=1 instance of the kernel):
rounds, walk steps and walking lanes per step, shading / triangle batches and their lanes."""
import ctypes as C
import json
import os
import sys

os.environ["PT_UPROF"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import pathtracerwithcuda_amd as pt  # noqa: E402

# argv[1]: a bench.py workload (default "metric"); one frame of its 8 passes in one launch
wl = bench.Workload(sys.argv[1] if len(sys.argv) > 1 else "metric", tree=bench.DEFAULT_TREE)
r = pt.Renderer(0)
scene, cfg, cam = wl.scene, wl.cfg, wl.cam
r.upload(scene, cfg)
r.setup_frame(wl.width, wl.height)
TILE = int(os.environ.get("PT_UPROF_TILE", "1"))  # >1: rank 0's bands of an N-way tiled frame
if TILE > 1:
    r.set_tiling(bench.BAND_ROWS, TILE, 0)
SHARE = int(os.environ.get("PT_UPROF_SHARE", "100"))  # percent of the occupancy grid (frames in flight)
if SHARE != 100:
    r.set_grid_share(SHARE)
r.render(cam, cfg, 1, 8, write_u8=2)
r.synchronize()
r.stats_reset()
r.render(cam, cfg, 1, 8, write_u8=2)
r.synchronize()
buf = (C.c_ulonglong * 48)()
pt.lib().pt_stats_all(r._ctx, buf, 48)
v = list(buf)
names = ["rounds", "walk_steps", "walking_lanes", "shade_batches", "lanes_shaded", "tri_batches", "tri_lanes", "refilled",
         "cyc_refill", "cyc_shade", "cyc_walk", "drained_steps_lanes", "parked_lanes", "ready_lanes", "idle_lanes", "cyc_next_segment"]
d = {n: v[16 + i] for i, n in enumerate(names)}
d["segments"] = v[0]
d["lanes_per_walk_step"] = round(d["walking_lanes"] / max(d["walk_steps"], 1), 2)
d["lanes_per_shade_batch"] = round(d["lanes_shaded"] / max(d["shade_batches"], 1), 2)
d["lanes_per_tri_batch"] = round(d["tri_lanes"] / max(d["tri_batches"], 1), 2)
d["walk_steps_per_round"] = round(d["walk_steps"] / max(d["rounds"], 1), 2)
tot = d["cyc_refill"] + d["cyc_shade"] + d["cyc_walk"]
for k in ("cyc_refill", "cyc_shade", "cyc_walk"):
    d[k.replace("cyc", "frac")] = round(d[k] / max(tot, 1), 3)
d["cyc_per_walk_round"] = round(d["cyc_walk"] / max(d["rounds"] - d["shade_batches"], 1))
d["cyc_per_shade_batch"] = round(d["cyc_shade"] / max(d["shade_batches"], 1))
for k in ("parked_lanes", "ready_lanes", "idle_lanes"):
    d[k + "_per_walk_step"] = round(d[k] / max(d["walk_steps"], 1), 2)
d["drained_walk_steps"] = d["drained_steps_lanes"] & 0xffffffff
d["drained_walking_lanes"] = d.pop("drained_steps_lanes") >> 32
d["drained_frac_of_walk_steps"] = round(d["drained_walk_steps"] / max(d["walk_steps"], 1), 3)
d["drained_lanes_per_walk_step"] = round(d["drained_walking_lanes"] / max(d["drained_walk_steps"], 1), 2)
d["next_segment_frac_of_shade"] = round(d["cyc_next_segment"] / max(d["cyc_shade"], 1), 3)
# timeline (stats[32..41], real-time clock at 100 MHz): waves' start, first drained refill, end
M = (1 << 64) - 1
tl = v[32:44]
if tl[8]:
    t0 = M ^ tl[0]
    us = lambda t: round((t - t0) / 100.0, 1)  # noqa: E731
    d["tl_waves"] = tl[8]
    d["tl_start_last_us"] = us(tl[1])
    d["tl_drain_first_us"] = us(M ^ tl[2])
    d["tl_drain_last_us"] = us(tl[3])
    d["tl_end_first_us"] = us(M ^ tl[4])
    d["tl_end_last_us"] = us(tl[5])
    d["tl_wave_tail_avg_us"] = round(tl[6] / tl[8] / 100.0, 1)
    d["tl_wave_life_avg_us"] = round(tl[7] / tl[8] / 100.0, 1)
    d["tl_segments_after_drain_frac"] = round(tl[9] / max(d["segments"], 1), 3)
    d["gen_batches"] = tl[10]
    d["lanes_per_gen_batch"] = round(d["refilled"] / max(tl[10], 1), 2)
    d["live_lanes_per_round"] = round(tl[11] / max(d["rounds"], 1), 2)
print(json.dumps(d))
