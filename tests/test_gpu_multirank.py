"""The N > 1 frame pipeline on the HIP renderer: 2 and 3 ranks, every rank on cuda:0 (this pool's boxes
have one GPU), gloo between the ranks, through the same TiledFrame/renderer code bench.py runs with
RCCL on an 8-GPU node (band tiling, two or five frames in flight on their own HIP streams, the frame's one
collective — a gather of the ranks' rows or a reduce of the float buffer — and rank 0's 8-bit
output). Rank 0's images must equal the oracle's single-frame render bit for bit."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import oracle
import pathtracerwithcuda_amd as pt

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gpu_multirank_worker as worker  # noqa: E402


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("ranks,collective,inflight", [(2, "gather", 5), (3, "reduce", 2)])
def test_tiled_frames_on_hip_equal_the_oracle(require_gpu, tmp_path, ranks, collective, inflight):
    out = str(tmp_path / "mr")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ranks}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(HERE, "gpu_multirank_worker.py"), out, collective, str(2 * inflight + 1), str(inflight)]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    res = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env)
    assert res.returncode == 0, res.stderr[-4000:]
    sc = worker.scene()
    cfg = pt.configuration(max_tracer_depth=8)
    cam = pt.camera(worker.W, worker.H, **worker.CAM)
    ref, ref8, _ = oracle.render(sc.view, cam, cfg, 1, worker.SPP)
    for k in range(inflight):
        img = np.load(f"{out}_{k}_f.npy")
        img8 = np.load(f"{out}_{k}_u8.npy")
        assert np.array_equal(img.view(np.uint32), ref.view(np.uint32)), f"context {k}: float image"
        assert np.array_equal(img8, ref8), f"context {k}: 8-bit image"


def test_rccl_one_rank_metric_frame(require_gpu, tmp_path):
    """RCCL itself on the one-GPU box: torch.distributed "nccl" with a one-rank group, initialised as bench.py
    initialises its N-GPU runs (torch.distributed.run env:// rendezvous, device_id), carries the metric frame
    through the production collective path — a FrameGroup of three frames in one MULTI launch with one RCCL
    gather, the bench's "gather8" group (8-bit rows per launch, the float rows on demand), and a TiledFrame with
    one RCCL reduce — plus an all-reduce and a barrier. Every frame equals the
    oracle's whole frame bit for bit, and librccl is the library the process loaded."""
    import bench

    out = str(tmp_path / "rccl")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(HERE, "gpu_rccl_worker.py"), out]
    res = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert res.returncode == 0, res.stderr[-4000:]
    import json
    facts = json.load(open(f"{out}_facts.json"))
    assert facts["backend"] == "nccl" and facts["world_size"] == 1, facts
    assert "MULTI" in facts["group_kernel"], facts
    assert facts["all_reduce"] == [1.5, 2.5] and any("librccl" in p for p in facts["rccl_loaded"]), facts
    wl = bench.Workload("metric")
    turned = pt.camera(wl.width, wl.height, yaw=0.35, **wl.cam_kw)
    ref, ref8, _ = oracle.render(wl.scene.view, wl.cam, wl.cfg, 1, wl.spp)
    ref_t, ref8_t, _ = oracle.render(wl.scene.view, turned, wl.cfg, 1, wl.spp)
    for tag, (want, want8) in (("group0", (ref, ref8)), ("group1", (ref_t, ref8_t)), ("group2", (ref, ref8)),
                               ("reduce", (ref, ref8)), ("g8_0", (ref, ref8)), ("g8_1", (ref_t, ref8_t))):
        img = np.load(f"{out}_{tag}_f.npy")
        img8 = np.load(f"{out}_{tag}_u8.npy")
        assert np.array_equal(img.view(np.uint32), want.view(np.uint32)), f"{tag}: float image"
        assert np.array_equal(img8, want8), f"{tag}: 8-bit image"


def test_bench_rccl_one_rank_self_check(require_gpu, tmp_path):
    """bench.py --rccl at N = 1: the timed run on the distributed path over a one-rank RCCL group (gather, frame
    groups, barrier, max-over-ranks all-reduce) and its image_matches_1gpu self-check, which re-renders the last
    timed launch's first and last frame alone; the line must say true, and the run must exit 0."""
    import json
    cmd = [sys.executable, os.path.join(os.path.dirname(HERE), "bench.py"), "--rccl", "--steps", "10", "--warmup",
           "2", "--no-cpu-baseline", "--orbit", "0.01"]
    res = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert res.returncode == 0, res.stderr[-4000:]
    line = json.loads(res.stdout.strip().splitlines()[-1])
    assert line["config"]["image_matches_1gpu"] is True, line["config"]
    assert line["config"]["collective"]["backend"] == "nccl", line["config"]
    assert line["config"]["frames_per_launch"] == 8 and line["config"]["orbit_rad_per_frame"] == 0.01, line["config"]


@pytest.mark.parametrize("ranks,collective,inflight,group", [(2, "gather", 3, 4), (3, "reduce", 2, 3),
                                                            (3, "gather8", 2, 4)])
def test_frame_groups_on_hip_equal_the_oracle(require_gpu, tmp_path, ranks, collective, inflight, group):
    """bench.py's PT_BENCH_GROUP path: FrameGroup contexts (pt_render_frames, one collective per group) with
    frames in flight; every frame of every context equals the oracle's frame of its camera."""
    out = str(tmp_path / "mg")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ranks}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(HERE, "gpu_multirank_worker.py"), out, collective, str(2 * inflight + 1), str(inflight),
           str(group)]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    res = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env)
    assert res.returncode == 0, res.stderr[-4000:]
    sc = worker.scene()
    cfg = pt.configuration(max_tracer_depth=8)
    for j in range(group):
        cam = pt.camera(worker.W, worker.H, yaw=0.3 * j, **worker.CAM)
        ref, ref8, _ = oracle.render(sc.view, cam, cfg, 1, worker.SPP)
        for k in range(inflight):
            img = np.load(f"{out}_{k}_{j}_f.npy")
            img8 = np.load(f"{out}_{k}_{j}_u8.npy")
            assert np.array_equal(img.view(np.uint32), ref.view(np.uint32)), f"context {k} frame {j}: float"
            assert np.array_equal(img8, ref8), f"context {k} frame {j}: 8-bit"


def test_rank0_continues_accumulating_after_gather8_groups(require_gpu, tmp_path):
    """gather8 (bench.py's tiled default) moves only the 8-bit rows per group, leaving each rank's float running sums on
    that rank. A caller that keeps accumulating on rank 0 — continuation passes add into the running sum
    (Core/path_tracer.cpp:40-67, path_tracer_kernel.cu:644-651) — first calls collect_float(); rank 0's sum then
    continues to the oracle's 2 SPP-pass sum bit for bit, over every row, its own and the other ranks'."""
    out = str(tmp_path / "cont")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=3",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(HERE, "gpu_multirank_worker.py"), out, "gather8", "3", "2", "3", "continue"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    res = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env)
    assert res.returncode == 0, res.stderr[-4000:]
    sc = worker.scene()
    cfg = pt.configuration(max_tracer_depth=8)
    cam = pt.camera(worker.W, worker.H, yaw=0.0, **worker.CAM)
    ref, ref8, _ = oracle.render(sc.view, cam, cfg, 1, 2 * worker.SPP)
    img = np.load(f"{out}_cont_f.npy")
    img8 = np.load(f"{out}_cont_u8.npy")
    assert np.array_equal(img.view(np.uint32), ref.view(np.uint32)), f"{(img != ref).any(axis=1).sum()} pixels differ"
    assert np.array_equal(img8, ref8)
