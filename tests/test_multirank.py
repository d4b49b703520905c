"""Multi-rank frame logic on the CPU: world_size 2 over gloo, through the same TiledFrame that
bench.py uses on the GPU box (band ownership, per-rank render, reduce to rank 0, 8-bit finalize).

The per-rank renderer here is a CPU stand-in with the Renderer frame interface, backed by the
oracle (test infrastructure). The HIP kernels' band tiling is covered on the GPU by
tests/test_gpu_parity.py::test_band_tiling_partitions_the_frame. The bar is the same as one GPU:
the reduced float image and its 8-bit output must equal a single full-frame render bitwise.
"""
import ctypes as C
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
import pathtracerwithcuda_amd as pt

W, H, SPP, BAND = 40, 27, 2, 4


class OracleFrameRenderer:
    """CPU stand-in for pathtracerwithcuda_amd.Renderer's frame interface."""

    def __init__(self, scene):
        self.scene = scene
        self.tiling = (1, 1, 0)

    def setup_frame(self, width, height, image_ptr=None):
        self.w, self.h = width, height
        n = width * height
        if image_ptr:
            self.img = np.ctypeslib.as_array((C.c_float * (n * 3)).from_address(image_ptr)).reshape(n, 3)
        else:
            self.img = np.zeros((n, 3), np.float32)
        self.img8 = np.zeros((n, 3), np.uint8)

    def set_tiling(self, band_rows, band_count, band_index):
        self.tiling = (band_rows, band_count, band_index)

    def render(self, cam, cfg, first_pass, pass_count, write_u8=0):
        assert first_pass == 1  # pass 1 overwrites: the owned pixels receive the whole sum
        px = pt.owned_pixels(self.w, self.h, *self.tiling)
        img, img8, _ = oracle.render(self.scene.view, cam, cfg, first_pass, pass_count, pixels=px)
        self.img[px] = img
        if write_u8:
            self.img8[px] = img8

    def render_frames(self, cams, cfg, images, images256, first_pass, pass_count, write_u8=0):
        assert first_pass == 1
        px = pt.owned_pixels(self.w, self.h, *self.tiling)
        for f, cam in enumerate(cams):
            img, img8, _ = oracle.render(self.scene.view, cam, cfg, first_pass, pass_count, pixels=px)
            images[f].numpy().reshape(-1, 3)[px] = img
            if write_u8 and images256 is not None:
                images256[f].numpy().reshape(-1, 3)[px] = img8

    def synchronize(self):
        pass

    def finalize_u8(self, cfg, pass_):
        self.img8[:] = oracle.gamma_u8(cfg, self.img, pass_)

    def finalize_u8_image(self, cfg, pass_, image, image256):
        image256.numpy().reshape(-1, 3)[:] = oracle.gamma_u8(cfg, image.numpy().reshape(-1, 3), pass_)


def _scene():
    return pt.cornell_scene(pt.torus_knot(40, 12), cube_length=16)


def _setup():
    cfg = pt.configuration(max_tracer_depth=5)
    cam = pt.camera(W, H, pitch=0.08, radius=12.5, center=(0, 1.2, 0))
    return cfg, cam


def _worker(rank, world, port, out_dir, collective="gather", inflight=1):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        scene = _scene()
        cfg, cam = _setup()
        if inflight == 1:
            r = OracleFrameRenderer(scene)
            frame = pt.TiledFrame(r, W, H, dist, BAND, device="cpu", collective=collective)
            assert frame.world == world and frame.rank == rank and frame.collect
            for _ in range(2):  # a second frame must not see the first one's reduced sum (bench renders many)
                frame.render(cam, cfg, SPP)
        else:
            # bench.py's frames in flight: one renderer + TiledFrame per frame in flight, frames queued with
            # launch() round-robin and synchronised at the end; every context must hold a whole frame
            rs = [OracleFrameRenderer(scene) for _ in range(inflight)]
            frames = [pt.TiledFrame(q, W, H, dist, BAND, device="cpu", collective=collective) for q in rs]
            for i in range(2 * inflight + 1):
                frames[i % inflight].launch(cam, cfg, SPP)
            for f in frames:
                f.synchronize()
            if rank == 0:
                for q in rs[1:]:
                    assert np.array_equal(q.img.view(np.uint32), rs[0].img.view(np.uint32))
                    assert np.array_equal(q.img8, rs[0].img8)
            r = rs[0]
        np.savez(os.path.join(out_dir, f"rank{rank}.npz"), img=r.img.copy(), img8=r.img8.copy(),
                 owned=pt.owned_pixels(W, H, BAND, world, rank))
    finally:
        dist.destroy_process_group()


CAM_YAWS = (0.0, 0.5, -0.6)


def _group_worker(rank, world, port, out_dir, collective):
    """bench.py's frame groups (PT_BENCH_GROUP): FrameGroup renders up to three frames per launch, each through
    its own camera, and moves them with one collective; a launch of fewer frames follows a full one."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        scene = _scene()
        cfg, _ = _setup()
        cams = [pt.camera(W, H, yaw=y, pitch=0.08, radius=12.5, center=(0, 1.2, 0)) for y in CAM_YAWS]
        # "gather8>reduce": bench.py's reduce leg, the live group switched from gather8 to the reduce between launches
        first, then = collective.split(">") if ">" in collective else (collective, collective)
        g = pt.FrameGroup(OracleFrameRenderer(scene), W, H, 3, dist, BAND, device="cpu", collective=first)
        def frames_of(n):
            if g.collective != "gather8":
                return [g.download(f) for f in range(n)]
            # gather8: rank 0 has every frame's 8-bit image after the launch; the float rows follow on demand
            img8 = [g.download(f)[1] for f in range(n)]
            g.collect_float()
            g.synchronize()
            return [(g.download(f)[0], img8[f]) for f in range(n)]

        g.launch(cams, cfg, SPP)
        g.synchronize()
        full = frames_of(3)
        g.collective = then
        g.launch(cams[1:], cfg, SPP)  # two frames: the stack's third frame is left as it was
        g.synchronize()
        two = frames_of(2)
        np.savez(os.path.join(out_dir, f"rank{rank}.npz"), img=np.stack([a for a, _ in full]),
                 img8=np.stack([b for _, b in full]), img2=np.stack([a for a, _ in two]),
                 img82=np.stack([b for _, b in two]))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world,collective", [(2, "gather"), (3, "gather"), (2, "reduce"), (1, "gather"),
                                              (1, "reduce"), (2, "gather8"), (3, "gather8"), (1, "gather8"),
                                              (3, "gather8>reduce")])
def test_frame_group_equals_single_renders(tmp_path, world, collective):
    """World size 1 is bench.py --rccl's path: a one-rank group still takes the collective (band count 1, the
    gather's own piece placed, or the reduce of the one buffer)."""
    mp.start_processes(_group_worker, args=(world, _free_port(), str(tmp_path), collective), nprocs=world,
                       join=True, start_method="spawn")
    r0 = np.load(tmp_path / "rank0.npz")
    cfg, _ = _setup()
    scene = _scene()  # keep alive: the view points into it
    for f, y in enumerate(CAM_YAWS):
        cam = pt.camera(W, H, yaw=y, pitch=0.08, radius=12.5, center=(0, 1.2, 0))
        ref, ref8, _ = oracle.render(scene.view, cam, cfg, 1, SPP)
        assert np.array_equal(r0["img"][f].reshape(-1, 3).view(np.uint32), ref.view(np.uint32)), f
        assert np.array_equal(r0["img8"][f].reshape(-1, 3), ref8), f
        if f >= 1:
            assert np.array_equal(r0["img2"][f - 1].reshape(-1, 3).view(np.uint32), ref.view(np.uint32)), f
            assert np.array_equal(r0["img82"][f - 1].reshape(-1, 3), ref8), f


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_owned_pixels_partition_the_frame():
    for world in (1, 2, 3, 8):
        parts = [pt.owned_pixels(W, H, BAND, world, k) for k in range(world)]
        allpx = np.concatenate(parts)
        assert np.array_equal(np.sort(allpx), np.arange(W * H))
        for k, p in enumerate(parts):
            rows = np.unique(p // W)
            assert np.array_equal(rows, pt.owned_rows(H, BAND, world, k))
            assert all((y // BAND) % world == k for y in rows)


@pytest.mark.parametrize("n,partial", [(17, True), (135, True), (16, False), (5, False), (9, True)])
def test_deal_bands_gives_every_region_its_costliest_bands_first(n, partial):
    """renderer.deal_bands: a permutation of the local bands that keeps a partial last band last; the
    launch's 8 regions (band positions by midpoint) each receive ranked bands in rank order, and the
    first band of every non-empty region comes from the top of the ranking."""
    from pathtracerwithcuda_amd.renderer import deal_bands
    full = n - 1 if partial else n
    rng = np.random.default_rng(n)
    ranked = [int(b) for b in rng.permutation(full)]
    order = deal_bands(ranked, n, 8)
    assert sorted(order) == list(range(n))
    if partial:
        assert order[-1] == n - 1
    rank_of = {b: i for i, b in enumerate(ranked)}
    region = [min(7, (2 * p + 1) * 8 // (2 * n)) for p in range(full)]
    firsts = []
    for r in range(8):
        ranks = [rank_of[order[p]] for p in range(full) if region[p] == r]
        assert ranks == sorted(ranks)
        if ranks:
            firsts.append(ranks[0])
    assert sorted(firsts) == list(range(len(firsts)))


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world,collective,inflight", [(2, "gather", 1), (2, "reduce", 1), (3, "gather", 1),
                                                       (2, "gather", 2), (2, "reduce", 3), (1, "gather", 1),
                                                       (1, "reduce", 2)])
def test_two_rank_tiled_frame_equals_single_render(tmp_path, world, collective, inflight):
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path), collective, inflight), nprocs=world, join=True,
                       start_method="spawn")
    rs = [np.load(tmp_path / f"rank{k}.npz") for k in range(world)]
    r0 = rs[0]
    cfg, cam = _setup()
    scene = _scene()  # keep alive: the view points into it
    ref, ref8, _ = oracle.render(scene.view, cam, cfg, 1, SPP)
    # rank 0 holds the reduced frame and its 8-bit image
    assert np.array_equal(r0["img"].view(np.uint32), ref.view(np.uint32))
    assert np.array_equal(r0["img8"], ref8)
    # the ranks' bands are disjoint and cover the frame (non-root buffers are scratch after the collective)
    owned = np.concatenate([r["owned"] for r in rs])
    assert np.array_equal(np.sort(owned), np.arange(W * H))


def _stage_run(tmp_path, world, stall, limit):
    import subprocess
    import sys
    import time

    here = os.path.dirname(os.path.abspath(__file__))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(here, "dist_stage_worker.py"), str(tmp_path / "st"), str(stall), str(limit)]
    t0 = time.monotonic()
    res = subprocess.run(cmd, capture_output=True, text=True, timeout=240,
                         env=dict(os.environ, OMP_NUM_THREADS="1", PYTHONUNBUFFERED="1"))
    return res, time.monotonic() - t0


@pytest.mark.timeout(300)
def test_stalled_rank_fails_the_job_within_the_stage_limit(tmp_path):
    """bench.py's fail-fast path (init_distributed's collective timeout + pt.StageWatch) over gloo: rank 1's renderer
    hangs before its group's gather; the job must exit non-zero well before its outer limit, with a stderr line naming
    a rank and the stage it was stuck in (rank 1 in its render, rank 0 in the gather: both are 'timed run')."""
    res, took = _stage_run(tmp_path, 2, 1, 6)
    assert res.returncode != 0, res.stderr[-3000:]
    assert took < 120, took
    assert "stage 'timed run' did not finish within 6 s" in res.stderr, res.stderr[-3000:]
    assert "rank 1: stage" in res.stderr or "rank 0: stage" in res.stderr, res.stderr[-3000:]
    assert not (tmp_path / "st_breakdown.json").exists()


@pytest.mark.timeout(300)
def test_rank_breakdown_reports_every_rank(tmp_path):
    """The same job without a stall: rank_breakdown (bench.py's config.per_rank) lists both ranks' render and
    collective time per launch over the two timed launches."""
    import json

    res, _ = _stage_run(tmp_path, 2, -1, 120)
    assert res.returncode == 0, res.stderr[-3000:]
    bd = json.load(open(tmp_path / "st_breakdown.json"))
    assert bd["launches_timed_per_rank"] == [2, 2], bd
    assert len(bd["render_ms_per_launch"]) == 2 and min(bd["render_ms_per_launch"]) > 0, bd
    assert len(bd["collective_ms_per_launch"]) == 2 and min(bd["collective_ms_per_launch"]) >= 0, bd
    assert bd["render_ms_per_launch_max_over_ranks"] == max(bd["render_ms_per_launch"]), bd


def test_stage_watch_names_the_stage_and_exits():
    """pt.StageWatch alone: a stage that outlives its limit ends the process with exit code 124 and one stderr line;
    a stage left in time does not."""
    import subprocess
    import sys

    code = ("import time, pathtracerwithcuda_amd as pt\n"
            "w = pt.StageWatch(3, 1.0)\n"
            "w.stage('quick'); time.sleep(0.3)\n"
            "w.stage('stuck gather'); time.sleep(30)\n")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60, cwd=root)
    assert res.returncode == 124, (res.returncode, res.stderr)
    assert "[bench] rank 3: stage 'stuck gather' did not finish within 1 s" in res.stderr, res.stderr
    assert "quick" not in res.stderr
