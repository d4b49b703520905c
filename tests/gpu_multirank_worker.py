"""Worker of tests/test_gpu_multirank.py, launched N times by torch.distributed.run on ONE GPU (every
rank on cuda:0, gloo between them): the bench.py frame pipeline (TiledFrame over renderer contexts,
INFLIGHT frames in flight, each launch on 1 / (INFLIGHT - 1) of the grid from three on and the last
frame on the whole grid, rank 0 collecting the frame) on the HIP renderer. Rank 0 saves each
context's float image and 8-bit image for the test to compare with the oracle.

With GROUP > 1 every context is a FrameGroup: each launch renders GROUP frames, frame j through the camera
turned by yaw 0.3 j (GROUP cameras), moved by one collective; rank 0 saves every frame of every context.

With CONTINUE ("continue", gather8 groups only): after the groups, every rank gathers the float rows (collect_float),
and rank 0 alone carries on accumulating frame 0 of its first context, passes SPP+1 .. 2 SPP over the whole frame
(untiled) into that running sum, as a caller adding passes to the image it was handed would; it saves that sum.

    worker.py OUT_PREFIX COLLECTIVE LAUNCHES [INFLIGHT [GROUP [CONTINUE]]]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

W, H, SPP = 96, 64, 4
CAM = dict(pitch=0.08, radius=12.5, center=(0.0, 1.2, 0.0))


def scene():
    import pathtracerwithcuda_amd as pt
    return pt.cornell_scene(pt.torus_knot(80, 24), cube_length=32)


def main() -> int:
    out, collective, frames = sys.argv[1], sys.argv[2], int(sys.argv[3])
    inflight = int(sys.argv[4]) if len(sys.argv) > 4 else 2
    group = int(sys.argv[5]) if len(sys.argv) > 5 else 1
    cont = len(sys.argv) > 6 and sys.argv[6] == "continue"
    share = 100 // (inflight - 1) if inflight >= 3 else 100
    import torch.distributed as dist

    import pathtracerwithcuda_amd as pt

    dist.init_process_group("gloo")
    rank = dist.get_rank()
    sc = scene()
    cfg = pt.configuration(max_tracer_depth=8)
    cam = pt.camera(W, H, **CAM)
    rs, fr = [], []
    for _ in range(inflight):  # one renderer context per frame in flight (bench.py)
        r = pt.Renderer(0)
        r.set_grid_share(share)
        r.upload(sc, cfg)
        rs.append(r)
        if group > 1:
            fr.append(pt.FrameGroup(r, W, H, group, dist, 8, device="cuda:0", collective=collective))
        else:
            fr.append(pt.TiledFrame(r, W, H, dist, 8, device="cuda:0", collective=collective))
    cams = [pt.camera(W, H, yaw=0.3 * j, **CAM) for j in range(group)]
    for i in range(frames):
        last = i == frames - 1 and share < 100
        if last:
            rs[i % inflight].set_grid_share(100)
        fr[i % inflight].launch(cams if group > 1 else cam, cfg, SPP)
    for f in fr:
        f.synchronize()
    if group > 1 and collective == "gather8":  # the float rows stay on their ranks until asked for (every rank)
        for f in fr:
            f.collect_float()
            f.synchronize()
    if rank == 0:
        for k, (r, f) in enumerate(zip(rs, fr)):
            if group > 1:
                for j in range(group):
                    img, img8 = f.download(j)
                    np.save(f"{out}_{k}_{j}_f.npy", img.reshape(-1, 3))
                    np.save(f"{out}_{k}_{j}_u8.npy", img8.reshape(-1, 3))
            else:
                _, img8 = r.download()
                np.save(f"{out}_{k}_f.npy", f.image.cpu().numpy().reshape(-1, 3))
                np.save(f"{out}_{k}_u8.npy", img8.reshape(-1, 3))
    if cont and rank == 0:
        # gather8 left each rank's float rows on that rank; collect_float (above) brought them to rank 0. Now the
        # caller continues frame 0 on rank 0 alone, untiled: passes SPP+1 .. 2 SPP add into the collected sum
        r, f = rs[0], fr[0]
        r.set_tiling(8, 1, 0)
        r.setup_frame(W, H, f.images[0].data_ptr())
        r.render(cams[0], cfg, SPP + 1, SPP, write_u8=2)
        r.synchronize()
        _, img8 = r.download()
        np.save(f"{out}_cont_f.npy", f.images[0].cpu().numpy().reshape(-1, 3))
        np.save(f"{out}_cont_u8.npy", img8.reshape(-1, 3))
    dist.barrier()
    for r in rs:
        r.close()
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
