#!/usr/bin/env python3
"""Benchmark of the radiance loop: Mrays/s and ms/frame at 1920x1080, 8 spp, 8 bounces on the
Cornell + OBJ-mesh scene (BASELINE.json `metric`), on 1 GPU or tiled across N GPUs of one node.

A step is one frame: 8 passes over the 1920x1080 frame and its 8-bit gamma output. Frames are rendered in
groups (pt_render_frames: G frames per persistent HIP launch, each through its own camera, plus one accumulate
launch) on two renderer contexts, queued with no host synchronisation. With N > 1 each rank renders its
interleaved 8-row bands of G = 8 N frames per launch and rank 0 gathers every rank's 8-bit rows with one RCCL
gather per group (torch.distributed "nccl"; the float running sums stay on their ranks, as the reference's
float image stays on the device; --collective gather moves them too, --collective reduce sums the float stack on
rank 0, the north star's RCCL reduce). Each rank of a multi-GPU run works under a stage watchdog and a collective
timeout (--stage-timeout, 180 s): a rank stuck in a stage exits 124 with a stderr line naming it and the stage, and
the line reports every rank's render and collective time per launch (config.per_rank). With the default gather8 the
same frames are then timed again with the reduce (config.collective.reduce_leg; PT_BENCH_REDUCE_LEG=0 skips it).
The host-synchronised single-frame latency is reported beside it. Mrays/s = ray segments traced (the live-ray counts the
reference's thread_shrink returns, summed over passes and depths and over ranks) / wall time.

    python bench.py [--gpus N --steps K --warmup W]   (defaults: 20 timed frames after 5, C4/C5 3 after 1)
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 --master-port P bench.py --gpus N
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

WIDTH, HEIGHT, SPP, DEPTH = 1920, 1080, 8, 8
# The BVH the timed frames walk by default: PT_BVH_SAH (pt_host.cpp, a surface-area tree with the walk's expected
# dependent steps minimised), whose frames equal the reference tree's bit for bit on the metric, C2 and C4 frames
# (profiles/r06/tree/); every N = 1 line re-checks that (config.image_matches_reference_tree) and times the reference
# LBVH beside it (config.alt_tree). PT_BENCH_TREE / --tree lbvh puts the reference tree in the headline.
DEFAULT_TREE = os.environ.get("PT_BENCH_TREE", "sah")
KNOT = (350, 100)  # 70,000 triangles: the ~70k-triangle bunny stand-in
CAMERA = dict(pitch=0.08, radius=12.5, center=(0.0, 1.2, 0.0))
BAND_ROWS = int(os.environ.get("PT_BAND_ROWS", "8"))  # rows per interleaved band of the tiled frame
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
HBM_MEASURED_GBS = 6290.0  # MI355X_MICROARCH.md:36: 6.29 TB/s measured (float4 copy), "≈6.3 TB/s achievable" (:296)
SIMDS = 256 * 4  # 256 CUs x 4 SIMDs
CLOCK_HZ = 2.4e9  # MI355X_MICROARCH.md: max clock 2400 MHz


def algorithmic_bytes(counts: dict, sphere_count: int, leaf_size: int, pixels: int, passes: int) -> float:
    """SURVEY.md §8(d) per-segment byte model in the reference's data layout:
    100 B path state per segment (alive index 4, ray in 24, scattering 24, throughput R/W 24,
    ray out 24) + 16 B per sphere + 32 B per BVH node + 4 B per leaf slot + 36 B per triangle test
    + 120 B per mesh hit (normals 36, material 84) + 84 B per sphere hit + 16 B (bilinear sky) and
    24 B (radiance R/W) per miss; plus 115 B per pixel per pass (init, raygen, gamma, 8-bit)."""
    seg = counts["segments"]
    b = (100.0 * seg + 16.0 * sphere_count * seg + 32.0 * counts["nodes"] + 4.0 * counts["tris"] * (1 if leaf_size == 1 else 1)
         + 36.0 * counts["tris"] + 120.0 * counts["hit_mesh"] + 84.0 * counts["hit_sphere"] + 40.0 * counts["miss"])
    return b + 115.0 * pixels * passes


def extend_bytes(counts: dict, sphere_count: int) -> float:
    """The BVH-walk share of the same model (what one wavefront extend launch must move): ray in 24 B,
    16 B per sphere, 32 B per node, 4 + 36 B per triangle test, hit record out 16 B."""
    seg = counts["segments"]
    return (24.0 + 16.0 + 16.0 * sphere_count) * seg + 32.0 * counts["nodes"] + 40.0 * counts["tris"]


GOLDEN = os.path.join(ROOT, "tests", "golden")


class ReferenceAssetsMissing(RuntimeError):
    """The reference's own assets are not packed here (tests skip their C5 / reference-scene cases)."""


def asset_root() -> str:
    """A reference-style working directory (res/configuration, res/scene, res/obj, res/texture) holding the
    scene fixtures of tests/golden/res and the reference's own meshes, textures and lobby skybox from
    tests/golden/ref_assets.tar.xz, unpacked once per pack into the temp directory. The pack is not in git (the
    reference states no license for its assets): __graft_entry__.build() writes it from a reference
    checkout (tools/pack_ref_assets.py), and it travels to the GPU box with the tree like the built libraries.
    /root/reference is not read here: it does not exist on the GPU box."""
    import hashlib
    import shutil
    import tarfile
    import tempfile

    pack = os.path.join(GOLDEN, "ref_assets.tar.xz")
    if not os.path.exists(pack):
        raise ReferenceAssetsMissing(f"{pack} is absent: run tools/pack_ref_assets.py with the reference checkout")
    digest = hashlib.sha256(open(pack, "rb").read()).hexdigest()[:16]
    fixtures = hashlib.sha256()
    for d, _, fs in sorted(os.walk(os.path.join(GOLDEN, "res"))):
        for f in sorted(fs):
            fixtures.update(os.path.relpath(os.path.join(d, f), GOLDEN).encode())
            fixtures.update(open(os.path.join(d, f), "rb").read())
    root = os.path.join(tempfile.gettempdir(), f"pt_assets_{digest}_{fixtures.hexdigest()[:12]}")
    if not os.path.isdir(os.path.join(root, "res")):
        tmp = f"{root}.tmp{os.getpid()}"
        shutil.rmtree(tmp, ignore_errors=True)
        shutil.copytree(os.path.join(GOLDEN, "res"), os.path.join(tmp, "res"))
        with tarfile.open(pack, "r:xz") as tar:
            for m in tar.getmembers():  # plain files under res/ only
                if not m.isfile() or not m.name.startswith("res/") or ".." in m.name.split("/"):
                    raise RuntimeError(f"unexpected member {m.name!r} in {pack}")
                tar.extract(m, tmp)
        for d, _, fs in os.walk(tmp):
            for f in fs:
                os.chmod(os.path.join(d, f), 0o644)
        try:
            os.rename(tmp, root)
        except OSError:  # another process unpacked it first
            shutil.rmtree(tmp, ignore_errors=True)
    return root


def procedural_texture(w: int, h: int, seed: int) -> np.ndarray:
    """RGBA8 texture (top row first): checker tiles with per-tile colour noise."""
    rng = np.random.default_rng(seed)
    tiles = rng.integers(40, 255, (8, 8, 3))
    y, x = np.mgrid[0:h, 0:w]
    c = tiles[(y * 8 // h) % 8, (x * 8 // w) % 8]
    img = np.concatenate([c, np.full((h, w, 1), 255)], -1)
    img[..., :3] = (img[..., :3] * (0.75 + 0.25 * ((x // 16 + y // 16) % 2))[..., None]).astype(np.int64)
    return img.astype(np.uint8)


class Workload:
    """One benchmark workload: scene, configuration, camera and frame size. `metric` is the configuration
    BASELINE.json's metric is quoted on (the default line); c2 is BASELINE.json's second config (1280x720,
    diffuse-only mesh, no spheres); c3-c5 are the heavier BASELINE.json configs
    (1 GPU or tiled), for one-off measurements of the same path at their sizes."""

    # BVH builders a workload can be built with: the reference's Morton LBVH (its config default MortonCodeCUDA,
    # Bvh/bvh.cpp:862-1047) and PT_BVH_SAH, the surface-area tree (a stated-tolerance mode)
    TREES = {"lbvh": 2, "sah": 3}

    def __init__(self, name: str, tree: str = "lbvh", leaf: int = 1):
        import pathtracerwithcuda_amd as pt

        self.name = name
        self.tree, self.leaf = tree, leaf  # leaf: BvhLeafNodeTriangleNum (the reference's config: 1)
        method = self.TREES[tree]
        cam_kw = dict(CAMERA)
        if name == "metric":
            self.width, self.height, self.spp, self.depth = WIDTH, HEIGHT, SPP, DEPTH
            self.scene = pt.cornell_scene(pt.torus_knot(*KNOT), method=method, leaf_size=leaf)
            self.key = f"cornell+knot{KNOT[0] * KNOT[1] * 2}_{WIDTH}x{HEIGHT}_spp{SPP}_d{DEPTH}"
            self.desc = ("Cornell box (cornell.obj walls, cube.obj light, iron+glass spheres) + torus knot, "
                         f"{self.scene.triangle_count} triangles, {self.scene.view.sphere_num} spheres")
            self.data = "synthetic: procedural 70k-triangle torus knot (bunny stand-in) + procedural 512^2 cube map"
        elif name == "c1":  # BASELINE.json configs[0]: spheres-only Cornell box, 512x512, 4 spp, 4 bounces
            self.width, self.height, self.spp, self.depth = 512, 512, 4, 4
            self.scene = pt.cornell_spheres_scene()
            cam_kw = dict(pitch=0.05, radius=11.0, center=(0.0, 1.2, 0.0))  # inside the box
            self.key = "c1_cornell_spheres_512x512_spp4_d4"
            self.desc = ("cornell_box_simple.json without meshes: five r=1000 wall spheres, a light sphere, iron + "
                         f"glass spheres ({self.scene.view.sphere_num} spheres, no BVH)")
            self.data = "synthetic: spheres-only Cornell box (cornell_box_simple.json materials) + procedural 512^2 cube map"
        elif name == "c2":  # Cornell + ~70k-triangle mesh, diffuse only, 1280x720
            self.width, self.height, self.spp, self.depth = 1280, 720, 8, 8
            self.scene = pt.cornell_scene(pt.torus_knot(*KNOT), mesh_material="diffuse_white", spheres=False,
                                          method=method, leaf_size=leaf)
            self.key = f"c2_cornell+knot{KNOT[0] * KNOT[1] * 2}_diffuse_1280x720_spp8_d8"
            self.desc = ("Cornell box (cornell.obj walls, cube.obj light) + torus knot, diffuse only (specular 0, "
                         f"n = 1.000293), no spheres, {self.scene.triangle_count} triangles")
            self.data = "synthetic: procedural 70k-triangle torus knot (bunny stand-in) + procedural 512^2 cube map"
        elif name == "c3":  # micro_surface.json: six GGX spheres, skybox, depth of field
            self.width, self.height, self.spp, self.depth = 1920, 1080, 64, 8
            sc = pt.Scene()
            for i, x in enumerate(np.linspace(-2.5, 2.5, 6)):
                sc.add_sphere((float(x), 0.4, 0.0), 0.45, f"Micro{i + 1}")
            walls = [sc.add_material(m) for m in ("wall_white", "wall_green", "wall_red", "wall_white", "wall_white")]
            sc.add_mesh(pt.cornell_shapes(), walls, position=(0.0, -0.8, 1.0), scale=(0.1, 0.1, 0.3))
            sc.add_mesh([pt.cube_shape()], [sc.add_material("light")], position=(0.0, 3.1, 0.0),
                        scale=(0.85, 0.05, 0.85))
            sc.set_cube_map(pt.procedural_cube_map(512))
            self.scene = sc.build(leaf_size=leaf, method=method)
            cam_kw.update(aperture=0.1, focal=12.5)
            self.key = "c3_microfacet_sky_dof_1920x1080_spp64_d8"
            self.desc = "six GGX spheres (roughness 0.01..1, silver n=0.04 k=2.65), Cornell walls + light, skybox, DoF 0.1"
            self.data = "synthetic: micro_surface.json spheres + procedural 512^2 cube map"
        elif name == "c4":  # ~800k-triangle mesh with the dragon's subsurface material
            self.width, self.height, self.spp, self.depth = 1920, 1080, 256, 8
            self.scene = pt.cornell_scene(pt.torus_knot(1000, 400), mesh_material="DragonGreen", method=method,
                                          leaf_size=leaf)
            self.key = "c4_knot800000_sss_1920x1080_spp256_d8"
            self.desc = (f"Cornell box + {self.scene.triangle_count - 22}-triangle torus knot (dragon stand-in) "
                         "with DragonGreen subsurface scattering (sigma_a (40,3,14), sigma_s' 400)")
            self.data = "synthetic: procedural 800k-triangle torus knot + procedural 512^2 cube map"
        elif name == "c5":  # multi-mesh, diffuse + specular texture maps, 4K
            self.width, self.height, self.spp, self.depth = 3840, 2160, 1024, 12
            # tests/golden/res/scene/c5_vanille_gallery.json, loaded by the reference-format scene parser from the
            # reference's own assets: two vanille.obj (25,786 triangles, 15 shapes, vanille.json's per-shape
            # materials and its five TGA diffuse maps, 256^2-1024^2) + human, cow, monkey, cup, with sponza
            # *_spec.tga specular maps (512^2 RGBA, 512^2 RGB, 1024^2 RGB), in the Cornell walls under the
            # cube light, lobby skybox
            root = asset_root()
            cfg = pt.configuration(max_tracer_depth=self.depth, bvh_build=method, bvh_leaf_node_triangle_num=leaf)
            self.scene = pt.load_scene(os.path.join(root, "res", "scene", "c5_vanille_gallery.json"), root_dir=root,
                                       config=cfg)
            cam_kw = dict(pitch=0.1, radius=9.0, center=(0.0, 0.9, 0.0))  # the room's front opening
            self.key = "c5_vanille_gallery_3840x2160_spp1024_d12"
            self.desc = (f"two vanille.obj + human/cow/monkey/cup in the Cornell walls, {self.scene.triangle_count} "
                         "triangles, vanille TGA diffuse maps + sponza *_spec.tga specular maps, lobby skybox")
            self.data = "the reference's own meshes, TGA maps and lobby skybox (tests/golden/ref_assets.tar.xz)"
        else:
            raise SystemExit(f"unknown workload {name!r}")
        self.cfg = pt.configuration(max_tracer_depth=self.depth, bvh_leaf_node_triangle_num=leaf)
        self.cam_kw = cam_kw
        self.cam = pt.camera(self.width, self.height, **cam_kw)


def cpu_baseline(wl: "Workload", threads: int) -> dict:
    """The reference's CPU fallback semantics (Core/path_tracer_cpu.cpp: MSVC rand, libm, MSVC's unfused
    arithmetic), as
    restated by the oracle, on the same frame: one whole frame (all of its passes), so ms/frame is measured,
    not extrapolated."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # cpu_baseline leg only

    oracle.lib()
    # whole frames until at least 2 s have passed (one frame of the metric workload, ~50 of C1's small one)
    frames, segments = 0, 0
    t0 = time.perf_counter()
    while True:
        _, _, st = oracle.render(wl.scene.view, wl.cam, wl.cfg, 1, wl.spp, rng="msvc", math="libm", arith="plain",
                                 threads=threads, with_u8=True)
        frames += 1
        segments += st["segments"]
        dt = time.perf_counter() - t0
        if dt >= 2.0 or frames >= 200:
            break
    what = "one whole" if frames == 1 else f"{frames} whole"
    return {"value": round(segments / dt / 1e6, 3), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": f"{what} {wl.width}x{wl.height} {wl.spp}-spp depth-{wl.depth} frame{'s' if frames > 1 else ''} "
                      f"({segments} ray segments, {dt:.2f} s), oracle in reference-CPU-fallback mode (MSVC rand, libm, "
                      "no FMA), OpenMP",
            "ms_per_frame": round(dt * 1000 / frames, 1)}


def host_threads(requested: int = 0) -> tuple[int, str]:
    """The host cores this job may use: every CPU of its affinity mask, unless the environment limits
    OpenMP (the GPU boxes export OMP_NUM_THREADS = their CPU share for one GPU)."""
    if requested:
        return requested, "--cpu-threads"
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and 0 < int(omp) < aff:
        return int(omp), f"OMP_NUM_THREADS={omp} (this job's CPU share; {aff} CPUs in the affinity mask)"
    return aff, f"all {aff} CPUs of the affinity mask"


def load_profile(workload: str) -> dict:
    """The dominant kernel's PMC figures for this workload (profiles/traffic.json, written by
    tools/traffic_summary.py from separate rocprofv3 --pmc passes): HBM bytes and VALU instructions."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    if not os.path.exists(path):
        return {}
    try:
        return json.load(open(path)).get(workload) or {}
    except Exception:
        return {}


def init_distributed(dist, backend: str, world: int, local: int, timeout_s: float, device=None) -> None:
    """The process group of a multi-GPU run: env:// rendezvous from torch.distributed.run, or a
    one-rank in-process group (bench.py --rccl run directly), with a collective timeout, so that a collective whose
    peer never arrives raises instead of waiting forever ("nccl" is RCCL on ROCm; device_id binds the communicator
    to this rank's GPU). The StageWatch beside it ends a rank that is stuck anywhere else."""
    import datetime

    # the collective timeout outlasts the stage limit, so the StageWatch names the stuck stage first
    kw = {"timeout": datetime.timedelta(seconds=max(1.0, float(timeout_s) + 60.0))}
    if backend == "nccl" and device is not None:
        kw["device_id"] = device
    if world == 1 and "MASTER_ADDR" not in os.environ:
        dist.init_process_group(backend, store=dist.HashStore(), rank=0, world_size=1, **kw)
    else:
        dist.init_process_group(backend, **kw)


def rank_breakdown(dist, frames, world: int, device) -> dict:
    """Per rank, the timed run's mean render and collective time per launch (StageClock: HIP events on the renderer
    streams, launch start -> passes rendered -> collective done), gathered to every rank: where a slow multi-GPU
    point spends its time. Every rank calls it (a collective)."""
    import torch

    t = [x for f in frames for x in f.clock.timings()]
    n = len(t)
    mine = [sum(a for a, _ in t) / max(n, 1), sum(b for _, b in t) / max(n, 1),
            max((a for a, _ in t), default=0.0), max((b for _, b in t), default=0.0), float(n)]
    if dist.get_backend() == "gloo":  # the rehearsal's gloo group: host tensors
        device = "cpu"
    x = torch.tensor(mine, dtype=torch.float64, device=device)
    parts = [torch.zeros_like(x) for _ in range(world)]
    dist.all_gather(parts, x)
    rows = [q.tolist() for q in parts]
    return {
        "render_ms_per_launch": [round(r[0], 4) for r in rows],
        "collective_ms_per_launch": [round(r[1], 4) for r in rows],
        "render_ms_per_launch_max_over_ranks": round(max(r[0] for r in rows), 4),
        "collective_ms_per_launch_max_over_ranks": round(max(r[1] for r in rows), 4),
        "render_ms_slowest_launch": round(max(r[2] for r in rows), 4),
        "collective_ms_slowest_launch": round(max(r[3] for r in rows), 4),
        "launches_timed_per_rank": [int(r[4]) for r in rows],
        "source": "HIP events on each rank's renderer streams: launch start -> passes rendered -> collective done "
                  "(frames in flight overlap, so a launch's render time includes waiting for the GPU)",
    }


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # defaults: the driver's 20 timed frames after 5 warm-up frames for the 1080p workloads (0.13 s of GPU time
    # at the metric frame), 3 after 1 for the heavy C4/C5 frames
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--warmup", type=int, default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--save-image", default="")
    ap.add_argument("--schedule", choices=["persistent", "wavefront"], default=None,
                    help="kernel schedule (default: the library's, PT_MODE)")
    ap.add_argument("--medium-bound", action="store_true",
                    help="tolerance mode pt_set_medium_bound: in-medium segments walk with min_t starting at their "
                         "free-flight distance (not proven bit-exact; DESIGN.md §4.2)")
    ap.add_argument("--workload", choices=["metric", "c1", "c2", "c3", "c4", "c5"], default="metric",
                    help="metric: BASELINE.json's metric configuration (default); c1: its CPU-path plumbing config "
                         "(the line then carries that frame's CPU-path time as cpu_baseline); c2-c5: its other configs")
    ap.add_argument("--tree", choices=list(Workload.TREES), default=DEFAULT_TREE,
                    help="the BVH the timed frames walk: lbvh, the reference's Morton LBVH (Bvh/bvh.cpp:862-1047, its "
                         "config default), or sah, PT_BVH_SAH (DESIGN.md §5)")
    ap.add_argument("--no-alt-tree", action="store_true",
                    help="at N = 1 the line also times the other tree on the same frames (config.alt_tree) and checks "
                         "that both render the same image; this skips both")
    ap.add_argument("--orbit", type=float, default=0.0, metavar="RAD",
                    help="advance the camera's yaw by RAD per frame (an interactive caller's moving camera); every "
                         "frame then has its own camera, 0 (default) keeps one camera for all frames")
    ap.add_argument("--collective", choices=["gather8", "gather", "reduce"], default=None,
                    help="the frame collective of a multi-GPU run (default: PT_FRAME_COLLECTIVE, else gather8 with frame "
                         "groups): gather8 moves each rank's 8-bit rows to rank 0 (the float running sums stay on their "
                         "ranks), gather moves the float rows too, reduce sums the float buffers on rank 0 (north_star's "
                         "RCCL reduce of the accumulation buffer)")
    ap.add_argument("--stage-timeout", type=float, default=float(os.environ.get("PT_BENCH_STAGE_TIMEOUT", "180")),
                    help="multi-GPU runs: seconds a rank may spend in one stage (init, upload, warm-up, timed run, "
                         "collectives, self-check) before it exits with 124 and a stderr line naming the rank and the "
                         "stage; also the collective timeout of the process group")
    ap.add_argument("--rccl", action="store_true",
                    help="at N = 1: run the multi-GPU path anyway, through a one-rank RCCL (torch 'nccl') group: "
                         "bands = 1, the frame's gather / reduce, barrier and all-reduce on RCCL, and the "
                         "image_matches_1gpu self-check")
    args = ap.parse_args()
    # stdout carries exactly ONE line, the JSON result: everything else the process prints — the scene loader's
    # progress, RCCL's version banner at communicator init (printed to stdout by the library itself) — goes to
    # stderr, at the file-descriptor level so that native code's writes follow it
    sys.stdout.flush()
    result_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    heavy = args.workload in ("c4", "c5")
    if args.steps is None:
        args.steps = 3 if heavy else 20
    if args.warmup is None:
        args.warmup = 1 if heavy else 5

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"[bench] --gpus {args.gpus} but WORLD_SIZE {world}: launch N>1 with torch.distributed.run",
              file=sys.stderr)
        if world == 1 and args.gpus > 1:
            return 2

    # HIP hardware queues per process (read when HIP initialises, before any device call): with 4, more
    # than three frames in flight share queues and serialise (4 frames on 33 % grids: 7.89 ms at N = 1);
    # with 8 they overlap (profiles/r02/scaling/hw_queues.txt). The GPU boxes EXPORT GPU_MAX_HW_QUEUES=4,
    # so the value is set here, not defaulted (PT_BENCH_HW_QUEUES overrides it; at most 32 on this pool).
    # Tiled (N > 1): 16, so RCCL's own streams get queues of their own beside the five renderer streams
    # instead of queueing behind a persistent pass launch (16 and 8 measured equal for the share itself)
    hw_queues = os.environ.get("PT_BENCH_HW_QUEUES", "16" if world > 1 or args.rccl else "8")
    os.environ["GPU_MAX_HW_QUEUES"] = hw_queues
    # Tiled shares batch triangle tests from 3 parked lanes instead of 6: a small share spends most of its
    # launch in the tail, where few lanes walk (8-way share 0.869-0.871 vs 0.887-0.897 ms; at N = 1 it is
    # -0.2 %, so the library default stays 6; profiles/r03/scaling/share8_knobs.txt)
    if world > 1:
        os.environ.setdefault("PT_TRI_MIN", "3")
    import torch
    import torch.distributed as dist

    import pathtracerwithcuda_amd as pt

    # PT_BENCH_BACKEND / PT_BENCH_SHARE_GPU: rehearsal of the N > 1 path on a one-GPU box (gloo, every
    # rank on device 0); the driver's multi-GPU runs use the defaults (RCCL, one GPU per rank)
    backend = os.environ.get("PT_BENCH_BACKEND", "nccl")
    if os.environ.get("PT_BENCH_SHARE_GPU"):
        local = 0
    # the multi-GPU code path: every N > 1 run, and N = 1 with --rccl (a one-rank group in this process)
    distributed = world > 1 or args.rccl
    # fail-fast: every stage of a multi-GPU rank runs under a watchdog (pt.StageWatch), and collectives time out
    watch = pt.StageWatch(rank, args.stage_timeout if distributed else 0.0)
    if distributed:
        watch.stage("init process group")
        torch.cuda.set_device(local)
        init_distributed(dist, backend, world, local, args.stage_timeout, torch.device("cuda", local))
        watch.stage("scene and upload")
    # frames in flight: one renderer context (own stream, image and pass buffers) per frame in flight,
    # so the next frame's workgroups fill the previous frame's tail; 1 = one at a time.
    # Each launch takes 1 / (F - 1) of the occupancy-sized grid (pt_set_grid_share). Measured best
    # (profiles/r02/scaling/hw_queues.txt, ms per frame of rank 0's share): three frames on half grids
    # for the whole frame (6.04 vs 6.13 with five), five on quarter grids for a tiled share (0.99 vs 1.08
    # at N = 8, 1.76 vs 1.80 at N = 4, 3.24 vs 3.26 at N = 2). At N = 1 the two running launches of a 1080p
    # frame take 45 % each rather than half: the queued third frame's first waves then start beside them
    # (+0.27 %, 3 of 3 rounds, profiles/r03/grid_share/). Not for the 0.4-4 s C4/C5 frames, whose tails are
    # a small part of them: there the 10 % left to the third frame sits idle (C4 -3.8 %)
    # Frames per launch (pt_render_frames, pathtracerwithcuda_amd.FrameGroup): each context renders G frames of
    # the view in one pass launch (and, tiled, moves them with one gather per group), so the frames share one launch's
    # start and tail. Every frame is still rendered whole, with its own 8-bit output. Measured
    # (profiles/r04/group/), two contexts on the whole grid against one frame per launch on three (N = 1, 45 %
    # grids) or five (tiled, 25 %) contexts: the bench line at N = 1 13662-13697 Mrays/s with 8 frames per
    # launch (8 + 8 + 4 over 20 steps) vs 13441-13475 (4: 13534-13550, 10: 13603-13638); rank 0's share per
    # frame over 20 frames (tools/tile_scaling.py --total 20) 8-way 0.744-0.750 ms vs 0.877-0.895, 4-way
    # 1.371-1.372 vs 1.551-1.555 (8 per launch), 2-way 2.690-2.693 vs 2.863-2.867 (4 per launch). Not for the
    # 0.1-ms C1 frame (27132-27561 vs 33068-33337 with 4 per launch: host-bound) nor the 0.4-4 s C4/C5 frames,
    # whose tails are a small part of them.
    # Nor for frames of more than one pass launch (C3's 64 passes: 25107 vs 25870 Mrays/s with 8 per launch):
    # their launches already follow each other on a context.
    wl = Workload(args.workload, tree=args.tree)
    # At 8 waves (profiles/r04/group/group_size_n2_n4.txt) 8 per launch beats 4 at N = 2 too (2.595-2.605 vs
    # 2.653-2.659 ms per frame). The tail is paid per launch and lasts about 1 ms whatever the share (the last
    # paths in flight), so a rank's launch carries 8 whole frames' units at every N: G = 8 N frames of a 1/N
    # share (round 5, profiles/r05/group_n/: rank 0's 8-way share over 20 frames 0.721 ms per frame with 8 per
    # launch, 0.679 with all 20 in one launch, 0.636 with 40 over 40 frames; 4-way 1.310 -> 1.272). At N = 1
    # it stays 8 (8 + 8 + 4 over the driver's 20 steps); the launch never holds more frames than the run has.
    group = int(os.environ.get("PT_BENCH_GROUP", "0")) or (
        1 if heavy or args.workload == "c1" or wl.spp > 8 else 8 * world)
    inflight = int(os.environ.get("PT_BENCH_INFLIGHT", "0")) or (
        2 if group > 1 else 3 if world == 1 else 5)
    collective = args.collective or os.environ.get("PT_FRAME_COLLECTIVE") or ("gather8" if group > 1 else "gather")
    if group == 1 and collective == "gather8":
        collective = "gather"  # one frame per launch: rank 0 gathers the float rows and writes the 8-bit image
    grid_share = int(os.environ.get("PT_BENCH_GRID_SHARE", "0")) or (
        (45 if inflight == 3 and not heavy and group == 1 else 100 // (inflight - 1)) if inflight >= 3 else 100)
    scene, cfg, cam = wl.scene, wl.cfg, wl.cam
    width, height, spp = wl.width, wl.height, wl.spp
    rs, frames = [], []
    for _ in range(inflight):
        q = pt.Renderer(local)
        q.set_schedule(args.schedule)
        q.set_grid_share(grid_share)
        if args.medium_bound:
            q.set_medium_bound(True)
        q.upload(scene, cfg)
        rs.append(q)
        if group > 1:
            # buffers for the most frames one launch of this run holds (the warm-up's or the timed run's)
            # tiled, a group moves only its 8-bit rows to rank 0 ("gather8"): the frame the reference's application
            # takes from the device each frame (Main/window.cpp:391); the float running sums stay on their ranks
            frames.append(pt.FrameGroup(q, width, height, max(1, min(group, max(args.steps, args.warmup))),
                                        dist if distributed else None, BAND_ROWS, device=f"cuda:{local}",
                                        collective=collective))
        else:
            frames.append(pt.TiledFrame(q, width, height, dist if distributed else None, BAND_ROWS,
                                        device=f"cuda:{local}" if distributed else None, collective=collective))
    r = rs[0]
    schedule = r.schedule()

    # roofline inputs: one instrumented (untimed) frame for the visit counts
    watch.stage("instrumented frame")
    r.set_instrumented(True)
    r.stats_reset()
    r.render(cam, cfg, 1, spp, write_u8=0)
    r.synchronize()
    counts = r.stats_all()
    r.set_instrumented(False)

    nframe = 0

    # PT_BENCH_LAST_FULL: how many frames at the end of a batch take the whole grid (default 1)
    last_full = int(os.environ.get("PT_BENCH_LAST_FULL", "1"))

    # --orbit: frame i of the run (warm-up frames first) is seen from the bench camera turned by i * RAD of yaw,
    # as an interactive caller's camera moves between frames; without it every frame shares the one camera
    def camera_of(i: int):
        if not args.orbit:
            return cam
        return pt.camera(width, height, yaw=float(i) * args.orbit, **wl.cam_kw)

    frame_no = 0  # frames issued so far (warm-up included): the camera index
    last_launch = None  # (context index, cameras) of the most recent launch

    def run(k: int) -> None:
        # the last launch of a batch has no launch behind it to fill the CUs it leaves: it takes the whole
        # grid (every frame is still rendered completely, in order, on its own context). With frame groups a
        # launch takes the next min(G, frames left) frames.
        nonlocal nframe, frame_no, last_launch
        launches = [min(group, k - i) for i in range(0, k, group)]
        for j, n in enumerate(launches):
            q = frames[nframe % inflight]
            full = grid_share < 100 and j >= len(launches) - last_full
            if full:
                rs[nframe % inflight].set_grid_share(100)
            cams = [camera_of(frame_no + f) for f in range(n)]
            if group > 1:
                q.launch(cams, cfg, spp)
            else:
                q.launch(cams[0], cfg, spp)
            if full:
                rs[nframe % inflight].set_grid_share(grid_share)
            last_launch = (nframe % inflight, cams)
            nframe += 1
            frame_no += n

    watch.stage("warm-up")
    run(args.warmup)
    torch.cuda.synchronize()
    for q in rs:
        q.stats_reset()
    for f in frames:
        f.clock.reset()
    if distributed:
        watch.stage("barrier before the timed run")
        dist.barrier()
    torch.cuda.synchronize()
    watch.stage("timed run")
    t0 = time.perf_counter()
    run(args.steps)
    torch.cuda.synchronize()
    if distributed:
        watch.stage("barrier after the timed run")
        dist.barrier()
    elapsed = time.perf_counter() - t0
    breakdown = None
    if distributed:
        watch.stage("per-rank breakdown")
        breakdown = rank_breakdown(dist, frames, world, torch.device("cuda", local))

    # The distributed path must produce the 1-GPU frame. Outside the timed region, rank 0 takes the last TIMED
    # launch's first and last frame (with frame groups: the MULTI kernel's frames, as every timed frame is made)
    # and renders each again alone on a fresh untiled context over the whole grid, through the same camera, and
    # compares them bitwise (float running sum and 8-bit image); the line carries config.image_matches_1gpu and a
    # mismatch exits 3
    matches_1gpu = None
    solo_frame = None
    watch.stage("self-check")
    if distributed and group > 1:
        # "gather8": the float rows of the last timed launch's frames to rank 0 for the check (every rank)
        frames[last_launch[0]].collect_float()
        frames[last_launch[0]].synchronize()
    if distributed and rank == 0:
        ctx, cams = last_launch
        picks = sorted({0, len(cams) - 1})
        got = [frames[ctx].download(f) if group > 1 else frames[ctx].download() for f in picks]
        solo = pt.Renderer(local)
        try:
            if args.medium_bound:
                solo.set_medium_bound(True)
            solo.upload(scene, cfg)
            solo.setup_frame(width, height)
            matches_1gpu = True
            for f, (tiled, tiled8) in zip(picks, got):
                solo.render(cams[f], cfg, 1, spp, write_u8=2)
                one, one8 = solo.download()
                if f == 0:
                    solo_frame = (one, one8)  # also the reference for the reduce leg's frames (one camera)
                matches_1gpu &= bool(np.array_equal(tiled.view(np.uint32).reshape(-1), one.view(np.uint32).reshape(-1))
                                     and np.array_equal(tiled8.reshape(-1), one8.reshape(-1)))
        finally:
            solo.close()
    timed_kernel = rs[0].last_kernel()  # the timed launches' kernel (frame groups: the MULTI instance)
    segments = sum(q.stats()["segments"] for q in rs)
    # dominant kernel: the pass kernel (persistent schedule) or the BVH-walk extend kernel (wavefront)
    kind = 0 if schedule == "persistent" else 1
    kernel_ms = sum(q.kernel_time_kind(kind)[0] for q in rs)
    launches = sum(q.kernel_time_kind(kind)[1] for q in rs)
    # single-frame latency (one frame at a time, host-synchronised), reported beside the throughput; the
    # dominant kernel's launch duration for the roofline is taken here too, with no other frame in flight
    # (with frames in flight the HIP events of one launch also span the overlapping launch's work)
    # --save-image: the last timed launch's first frame (the frame the self-check compares), taken before the latency
    # frames and the other tree's leg reuse the contexts
    saved8 = None
    if args.save_image and rank == 0:
        ctx_s, _ = last_launch
        _, saved8 = frames[ctx_s].download(0) if group > 1 else frames[ctx_s].download()
    watch.stage("single-frame latency")
    lat_frames = max(3, min(5, args.steps))
    r.set_grid_share(100)
    r.stats_reset()
    if distributed:
        dist.barrier()
    t1 = time.perf_counter()
    for _ in range(lat_frames):
        frames[0].render(cam, cfg, spp)
    if distributed:
        dist.barrier()
    latency = (time.perf_counter() - t1) / max(lat_frames, 1)
    solo_ms, solo_launches = r.kernel_time_kind(kind)

    # The north star's collective beside the default (N > 1 with frame groups): the same K frames with
    # "reduce" (every rank's float stack summed on rank 0, which then writes the 8-bit images) in place of "gather8",
    # timed the same way (warm-up, barrier, max over ranks) on the same contexts; config.collective.reduce_leg
    reduce_leg = None
    if distributed and world > 1 and group > 1 and collective == "gather8" \
            and os.environ.get("PT_BENCH_REDUCE_LEG", "1") != "0":
        watch.stage("reduce leg")
        for f in frames:
            f.collective = "reduce"
        try:
            run(max(1, args.warmup))
            torch.cuda.synchronize()
            for q in rs:
                q.stats_reset()
            for f in frames:
                f.clock.reset()
            dist.barrier()
            torch.cuda.synchronize()
            tr = time.perf_counter()
            run(args.steps)
            torch.cuda.synchronize()
            dist.barrier()
            red = torch.tensor([time.perf_counter() - tr, sum(q.stats()["segments"] for q in rs)],
                               dtype=torch.float64, device=f"cuda:{local}")
            r_break = rank_breakdown(dist, frames, world, torch.device("cuda", local))
            # rank 0 holds the reduced frames: the last launch's first frame must be the 1-GPU frame too (one camera
            # for every frame unless --orbit)
            reduce_matches = None
            if rank == 0 and solo_frame is not None and not args.orbit:
                got_f, got_8 = frames[last_launch[0]].download(0)
                reduce_matches = bool(np.array_equal(got_f.view(np.uint32).reshape(-1), solo_frame[0].view(np.uint32).reshape(-1))
                                      and np.array_equal(got_8.reshape(-1), solo_frame[1].reshape(-1)))
        finally:
            for f in frames:
                f.collective = collective
        r_elapsed = torch.tensor([float(red[0])], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(r_elapsed, op=dist.ReduceOp.MAX)
        r_seg = red[1:].clone()
        dist.all_reduce(r_seg)
        reduce_leg = {"value": round(float(r_seg.item()) / float(r_elapsed.item()) / 1e6, 3),
                      "ms_per_step": round(float(r_elapsed.item()) / args.steps * 1000.0, 3),
                      "collective_ms_per_launch_max_over_ranks":
                          r_break.get("collective_ms_per_launch_max_over_ranks") if r_break else None,
                      "render_ms_per_launch_max_over_ranks":
                          r_break.get("render_ms_per_launch_max_over_ranks") if r_break else None,
                      "image_matches_1gpu": reduce_matches}
        if reduce_matches is False:
            matches_1gpu = False  # the line says so and the run exits 3

    # The other tree on the same frames (N = 1): the reference's LBVH beside PT_BVH_SAH, or the other way round, timed
    # the same way (warm-up, K timed frames, one-frame-in-flight launches for the roofline), and one frame of each
    # compared bit for bit (the trees' closest hits differ only where the walk order decides them)
    alt = None
    if world == 1 and not distributed and not args.no_alt_tree and scene.view.mesh_num > 0:  # (no BVH, no tree)
        alt_tree = "lbvh" if args.tree == "sah" else "sah"
        awl = Workload(args.workload, tree=alt_tree)
        for q in rs:
            q.synchronize()
            q.upload(awl.scene, cfg)
        run(args.warmup)
        torch.cuda.synchronize()
        for q in rs:
            q.stats_reset()
        torch.cuda.synchronize()
        ta = time.perf_counter()
        run(args.steps)
        torch.cuda.synchronize()
        a_elapsed = time.perf_counter() - ta
        a_segments = sum(q.stats()["segments"] for q in rs)
        r.set_grid_share(100)
        r.stats_reset()
        for _ in range(lat_frames):
            frames[0].render(cam, cfg, spp)
        a_ms, a_n = r.kernel_time_kind(kind)
        chk = pt.Renderer(local)
        try:
            chk.set_schedule(args.schedule)
            imgs = []
            for sc_ in (wl.scene, awl.scene):
                chk.upload(sc_, cfg)
                chk.setup_frame(width, height)
                chk.render(cam, cfg, 1, spp, write_u8=2)
                imgs.append(chk.download())
        finally:
            chk.close()
        (f0, u0), (f1, u1) = imgs
        differ = int((f0.view(np.uint32) != f1.view(np.uint32)).any(axis=-1).sum())
        alt = {"tree": alt_tree, "scene": awl.scene, "elapsed": a_elapsed, "segments": a_segments,
               "avg_launch_s": a_ms / max(a_n, 1) / 1000.0, "pixels_differ": differ,
               "pixels_differ_u8": int((u0 != u1).any(axis=-1).sum()), "key": awl.key}

    if distributed:
        watch.stage("max over ranks")
        t = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        s = torch.tensor([segments], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(s)
        segments = int(s.item())
        c = torch.tensor([counts[k] for k in sorted(counts)], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(c)
        counts = {k: int(v) for k, v in zip(sorted(counts), c.tolist())}

    if rank != 0:
        if distributed:
            watch.stage("destroy process group")
            dist.destroy_process_group()
        watch.close()
        return 0
    watch.stage("report")

    if saved8 is not None:
        from pathtracerwithcuda_amd.imageio import write_png
        write_png(args.save_image, np.asarray(saved8).reshape(height, width, 3))

    value = segments / elapsed / 1e6
    ms_per_step = elapsed / args.steps * 1000.0
    avg_launch_s = solo_ms / max(solo_launches, 1) / 1000.0  # one frame at a time (see above)
    launches_per_frame = launches / max(args.steps, 1)
    # the roofline prices the solo launch, which renders ONE frame; with frame groups a timed launch renders up
    # to G frames: pass launches per frame = pass launches per group launch (every frame of a group takes the
    # same batches of passes)
    frame_launches = launches / max(1, -(-args.steps // group))
    if schedule == "persistent":
        # one launch = a batch of passes over the frame (this rank's bands when tiled)
        bytes_per_launch = algorithmic_bytes(counts, scene.view.sphere_num, cfg.bvh_leaf_node_triangle_num,
                                             width * height, spp) / world / frame_launches
        kernel_name = r.last_kernel()
    else:
        # one launch = one depth of one pass
        bytes_per_launch = extend_bytes(counts, scene.view.sphere_num) / world / frame_launches
        kernel_name = "extend_kernel<LEAF1=true,STATS=false>"
    workload = wl.key
    # profiles/traffic.json keys: the workload, then "/sah" for the PT_BVH_SAH tree (the reference tree unsuffixed)
    suffix = ("" if schedule == "persistent" else "/wavefront") + ("/medium_bound" if args.medium_bound else "")
    key = workload + ("/sah" if args.tree == "sah" and scene.view.mesh_num > 0 else "") + suffix
    # N > 1: rank 0's share profiled on its own (tools/gpu_share_pmc.sh, "<key>/tiled<N>"); otherwise the
    # whole 1-GPU frame's profile, of which a rank of N runs 1/N
    prof = load_profile(f"{key}/tiled{world}") if world > 1 else {}
    per_rank = bool(prof)
    if not per_rank:
        prof = load_profile(key)
    scale = 1.0 if per_rank or world == 1 else 1.0 / world
    traffic = float(prof["hbm_bytes_per_launch"]) * scale if prof.get("hbm_bytes_per_launch") else None
    valu_insts = float(prof["valu_insts_per_launch"]) * scale if prof.get("valu_insts_per_launch") else None
    # The resource that binds this kernel is VALU issue behind a dependent-load chain, not HBM
    # (DESIGN.md §4): a wave64 VALU instruction issues over 2 cycles of its SIMD-32
    # (MI355X_MICROARCH.md, Wave scheduling), so the chip issues at most SIMDS x clock / 2 wave-level
    # VALU instructions per second. achieved = SQ_INSTS_VALU per launch (rocprofv3 --pmc, profiles/)
    # / the launch's duration measured here with HIP events on the renderer's stream, one frame in flight.
    valu_peak = SIMDS * CLOCK_HZ / 2.0 / 1e9  # G wave-instructions / s
    valu_achieved = valu_insts / avg_launch_s / 1e9 if valu_insts else None
    # The same roofline over the timed mode's own clock: the TIMED kernel's VALU per frame / ms_per_step (frames in
    # flight overlap, so this is what the timed figure implies per GPU). With frame groups the timed launches run
    # the MULTI instance, which issues fewer instructions per frame than the solo launch (it shares one drain among
    # its frames): its own count is profiled separately (profiles/traffic.json valu_insts_per_frame_timed, a
    # --pmc SQ_INSTS_VALU pass over an 8-frame launch) and used here; without that record the field stays null.
    if group > 1:
        vt = prof.get("valu_insts_per_frame_timed")
        valu_timed_frame = float(vt) * scale if vt else None
    else:
        valu_timed_frame = valu_insts * frame_launches if valu_insts else None
    valu_timed = valu_timed_frame / (ms_per_step / 1000.0) / 1e9 if valu_timed_frame else None
    # the solo launch's duration as rocprofv3's kernel trace averages it (recorded with the counters): the same
    # fraction priced on the profiler's clock instead of this run's HIP events
    rp_ms = prof.get("rocprof_avg_launch_ms")
    valu_rocprof = valu_insts / (float(rp_ms) / 1000.0) / 1e9 if (valu_insts and rp_ms and world == 1) else None
    # Lane-weighted: a wave-instruction counts active lanes / 64 (PT_UPROF lanes per phase x the PT_DUP VALU
    # split per phase, tools/lane_weighted.py, recorded in profiles/traffic.json)
    valu_lanes = float(prof["valu_lane_weighted_per_launch"]) * scale if prof.get("valu_lane_weighted_per_launch") else None
    hbm = None
    if traffic is not None:
        hbm_gbs = traffic / avg_launch_s / 1e9
        hbm = {"achieved": round(hbm_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
               "frac": round(hbm_gbs / HBM_PEAK_GBS, 4), "bytes_per_launch": round(traffic),
               "frac_of_measured": round(hbm_gbs / HBM_MEASURED_GBS, 4), "measured_peak": HBM_MEASURED_GBS,
               "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (gfx950 FETCH x2), profiles/traffic.json"}
    valu = {"achieved": round(valu_achieved, 1) if valu_achieved else None, "peak": valu_peak,
            "unit": "G VALU wave-instructions/s",
            "frac": round(valu_achieved / valu_peak, 4) if valu_achieved else None}
    line = {
        "metric": "Mrays/sec + ms/frame @1920x1080, 8spp, 8-bounce; 1/2/4/8 GPU",
        "value": round(value, 3),
        "unit": "Mrays/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": wl.data,
        "config": {
            "workload": workload,
            "scene": wl.desc,
            "width": width, "height": height, "spp": spp, "max_depth": wl.depth,
            "parallelism": f"tiled{world}" if distributed else "single",
            "schedule": schedule,
            "medium_bound": bool(args.medium_bound),
            "band_rows": BAND_ROWS if world > 1 else None,
            "ms_per_frame": round(ms_per_step, 3),
            "frames_in_flight": inflight,
            "frames_per_launch": group,
            "hw_queues": int(hw_queues),
            "grid_share_pct": grid_share,
            "ms_per_frame_latency": round(latency * 1000.0, 3),
            "camera_samples_per_s_M": round(width * height * spp * args.steps / elapsed / 1e6, 3),
            "segments_per_frame": segments // max(args.steps, 1),
            "orbit_rad_per_frame": args.orbit,
        },
        "roofline": {
            "bound": "valu",
            **{k: valu[k] for k in ("achieved", "peak", "unit", "frac")},
            "traffic": round(traffic) if traffic is not None else None,
            "hbm": hbm,
            "valu": valu,
            "valu_insts_per_launch": round(valu_insts) if valu_insts else None,
            "frac_rocprof_avg": round(valu_rocprof / valu_peak, 4) if valu_rocprof else None,
            "rocprof_avg_launch_ms": rp_ms if valu_rocprof else None,
            "frac_timed_mode": round(valu_timed / valu_peak, 4) if valu_timed else None,
            "valu_insts_per_frame_timed": round(valu_timed_frame) if valu_timed_frame else None,
            "frac_lane_weighted": round(valu_lanes / avg_launch_s / 1e9 / valu_peak, 4) if valu_lanes else None,
            "valu_lane_weighted_per_launch": round(valu_lanes) if valu_lanes else None,
            "kernel": kernel_name,
            "kernel_timed": timed_kernel,
            "counters_from": ("one GPU" if world == 1 else
                              f"rank 0's share of {world}, profiled on its own" if per_rank else
                              f"the 1-GPU frame's profile / {world}"),
            "avg_launch_ms": round(avg_launch_s * 1000, 4),
            "avg_launch_source": "HIP events on the renderer stream, one frame in flight",
            "avg_launch_ms_frames_in_flight": round(kernel_ms / max(launches, 1), 4),
            "launches_per_frame": round(launches_per_frame, 3),
            # SURVEY.md §8(d)'s reference-layout bytes: what the reference's AoS walk would load per launch,
            # mostly served by L1/L2/MALL here; a cache-level figure, not an HBM fraction
            "algorithmic_bytes_per_launch": round(bytes_per_launch),
            "counts_per_frame": counts,
        },
        "cpu_baseline": None,
    }
    # The roofline that binds is whichever resource the kernel is closer to: VALU issue (the metric frame, C2, C3, C5)
    # or HBM (C4's 51-MB tree: 0.61 of HBM against 0.51 of VALU, profiles/r05/workloads/); the other stays beside it
    rf = line["roofline"]
    if hbm is not None and (valu["frac"] is None or hbm["frac"] > valu["frac"]):
        rf.update(bound="hbm", achieved=hbm["achieved"], peak=hbm["peak"], unit=hbm["unit"], frac=hbm["frac"])
    line["config"]["tree"] = args.tree
    if alt is not None:
        aprof = load_profile(alt["key"] + ("/sah" if alt["tree"] == "sah" and scene.view.mesh_num > 0 else "") + suffix)
        a_valu = aprof.get("valu_insts_per_launch")
        a_hbm = aprof.get("hbm_bytes_per_launch")
        a_vf = float(a_valu) / alt["avg_launch_s"] / 1e9 / valu_peak if a_valu else None
        a_hf = float(a_hbm) / alt["avg_launch_s"] / 1e9 / HBM_PEAK_GBS if a_hbm else None
        a_bound = "hbm" if (a_hf is not None and (a_vf is None or a_hf > a_vf)) else "valu"
        line["config"]["alt_tree"] = {
            "tree": alt["tree"],
            "value": round(alt["segments"] / alt["elapsed"] / 1e6, 3),
            "ms_per_step": round(alt["elapsed"] / args.steps * 1000.0, 3),
            "avg_launch_ms": round(alt["avg_launch_s"] * 1000.0, 4),
            "roofline": {"bound": a_bound, "frac": round(a_hf if a_bound == "hbm" else a_vf, 4) if (a_vf or a_hf) else None,
                         "valu_frac": round(a_vf, 4) if a_vf else None, "hbm_frac": round(a_hf, 4) if a_hf else None,
                         "valu_insts_per_launch": a_valu, "hbm_bytes_per_launch": a_hbm},
            "segments_per_frame": alt["segments"] // max(args.steps, 1),
            # one frame of each tree through the same camera, compared bit for bit
            "image_pixels_differ": alt["pixels_differ"], "image_pixels_differ_u8": alt["pixels_differ_u8"],
        }
        line["config"]["image_matches_reference_tree"] = alt["pixels_differ"] == 0 and alt["pixels_differ_u8"] == 0
    if distributed:
        line["config"]["image_matches_1gpu"] = matches_1gpu
        line["config"]["collective"] = {"backend": dist.get_backend(), "world_size": world,
                                        "frame_collective": frames[0].collective}
        if reduce_leg is not None:
            line["config"]["collective"]["reduce_leg"] = reduce_leg
        line["config"]["per_rank"] = breakdown
    if world == 1 and not args.no_cpu_baseline and args.workload in ("metric", "c1"):
        threads, why = host_threads(args.cpu_threads)
        line["cpu_baseline"] = cpu_baseline(wl, threads)
        line["cpu_baseline"]["cpu"] = platform.processor() or platform.machine()
        line["cpu_baseline"]["threads_from"] = why
    print(json.dumps(line), file=result_out, flush=True)
    if distributed:
        watch.stage("destroy process group")
        dist.destroy_process_group()
    watch.close()
    if distributed and not matches_1gpu:
        print("[bench] the tiled frame differs from the 1-GPU frame", file=sys.stderr)
        return 3
    return 0


if __name__ == "__main__":
    sys.exit(main())
