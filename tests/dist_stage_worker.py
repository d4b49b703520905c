"""Worker of tests/test_multirank.py's fail-fast tests, launched by torch.distributed.run like bench.py's N-GPU runs:
bench.py's own distributed pieces (init_distributed with its collective timeout, pt.StageWatch stages named as bench
names them, rank_breakdown) around FrameGroup launches on the oracle-backed CPU renderer, over gloo.

    dist_stage_worker.py OUT_PREFIX STALL_RANK STAGE_TIMEOUT_S

STALL_RANK >= 0: that rank's renderer hangs in its second launch, before the group's gather, as a lost GPU or a hung
kernel would; every rank must then exit non-zero within about STAGE_TIMEOUT_S with a line naming the rank and stage.
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))


def main() -> int:
    out, stall, limit = sys.argv[1], int(sys.argv[2]), float(sys.argv[3])
    import torch.distributed as dist

    import bench
    import pathtracerwithcuda_amd as pt
    from test_multirank import BAND, SPP, W, H, OracleFrameRenderer, _scene, _setup

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    watch = pt.StageWatch(rank, limit)
    watch.stage("init process group")
    bench.init_distributed(dist, "gloo", world, 0, limit)
    watch.stage("scene and upload")
    scene = _scene()
    cfg, cam = _setup()

    class Renderer(OracleFrameRenderer):
        launches = 0

        def render_frames(self, *a, **k):
            Renderer.launches += 1
            if rank == stall and Renderer.launches == 2:
                time.sleep(3600)  # never returns: the watchdog must end this process
            return super().render_frames(*a, **k)

    g = pt.FrameGroup(Renderer(scene), W, H, 2, dist, BAND, device="cpu", collective="gather8")
    watch.stage("warm-up")
    g.launch([cam, cam], cfg, SPP)
    g.clock.reset()
    watch.stage("timed run")
    for _ in range(2):
        g.launch([cam, cam], cfg, SPP)
    watch.stage("per-rank breakdown")
    bd = bench.rank_breakdown(dist, [g], world, "cpu")
    watch.stage("destroy process group")
    dist.destroy_process_group()
    watch.close()
    if rank == 0:
        json.dump(bd, open(f"{out}_breakdown.json", "w"))
    return 0


if __name__ == "__main__":
    sys.exit(main())
