"""One rank of tests/test_gpu_multirank.py::test_rccl_one_rank_metric_frame: the production collective path on
RCCL (torch.distributed "nccl") with a one-rank group on the one-GPU box, initialised exactly as bench.py
initialises an N-GPU run (env:// rendezvous from torch.distributed.run, device_id given). The metric frame goes
through a FrameGroup (three frames in one MULTI launch, one RCCL gather of the group), a "gather8" FrameGroup
(two frames: their 8-bit rows with the launch, the float rows by collect_float) and a TiledFrame (one RCCL
reduce of the float buffer); the images and the collective's facts are saved for the test to check.

    python -m torch.distributed.run --nproc-per-node 1 ... gpu_rccl_worker.py <out-prefix>
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main() -> int:
    out = sys.argv[1]
    os.environ["GPU_MAX_HW_QUEUES"] = "16"  # as bench.py sets it for the distributed path
    import torch
    import torch.distributed as dist

    import bench
    import pathtracerwithcuda_amd as pt

    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    wl = bench.Workload("metric")
    cams = [wl.cam, pt.camera(wl.width, wl.height, yaw=0.35, **wl.cam_kw), wl.cam]
    facts = {"backend": dist.get_backend(), "world_size": dist.get_world_size()}
    q = pt.Renderer(local)
    try:
        q.upload(wl.scene, wl.cfg)
        g = pt.FrameGroup(q, wl.width, wl.height, 3, dist, bench.BAND_ROWS, device=f"cuda:{local}",
                          collective="gather")
        g.launch(cams, wl.cfg, wl.spp)
        g.synchronize()
        facts["group_kernel"] = q.last_kernel()
        for f in range(3):
            img, img8 = g.download(f)
            np.save(f"{out}_group{f}_f.npy", img.reshape(-1, 3))
            np.save(f"{out}_group{f}_u8.npy", img8.reshape(-1, 3))
    finally:
        q.close()
    q = pt.Renderer(local)
    try:
        # bench.py's tiled group: only the 8-bit rows move with the launch; the float rows on demand
        q.upload(wl.scene, wl.cfg)
        g = pt.FrameGroup(q, wl.width, wl.height, 3, dist, bench.BAND_ROWS, device=f"cuda:{local}",
                          collective="gather8")
        g.launch(cams[:2], wl.cfg, wl.spp)
        g.synchronize()
        img8s = [g.download(f)[1] for f in range(2)]
        g.collect_float()
        g.synchronize()
        for f in range(2):
            np.save(f"{out}_g8_{f}_f.npy", g.download(f)[0].reshape(-1, 3))
            np.save(f"{out}_g8_{f}_u8.npy", img8s[f].reshape(-1, 3))
    finally:
        q.close()
    q = pt.Renderer(local)
    try:
        q.upload(wl.scene, wl.cfg)
        t = pt.TiledFrame(q, wl.width, wl.height, dist, bench.BAND_ROWS, device=f"cuda:{local}", collective="reduce")
        t.render(wl.cam, wl.cfg, wl.spp)
        img, img8 = t.download()
        np.save(f"{out}_reduce_f.npy", np.asarray(img).reshape(-1, 3))
        np.save(f"{out}_reduce_u8.npy", np.asarray(img8).reshape(-1, 3))
    finally:
        q.close()
    # an all-reduce on RCCL as well (bench.py's max-over-ranks time and segment sums)
    x = torch.tensor([1.5, 2.5], dtype=torch.float64, device=f"cuda:{local}")
    dist.all_reduce(x, op=dist.ReduceOp.MAX)
    dist.barrier()
    facts["all_reduce"] = x.tolist()
    facts["rccl_loaded"] = sorted({ln.split()[-1] for ln in open("/proc/self/maps") if "rccl" in ln.split()[-1]})
    dist.destroy_process_group()
    json.dump(facts, open(f"{out}_facts.json", "w"))
    return 0


if __name__ == "__main__":
    sys.exit(main())
