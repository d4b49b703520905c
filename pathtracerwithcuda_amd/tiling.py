"""Frame tiling across ranks and the one-collective frame of the multi-GPU path.

Every pixel's path depends only on (pass, global pixel index, depth) and the read-only scene
(path_tracer_kernel.cu:324,415), so a frame shards with no exchange while rendering. Rank r of N
owns the rows y with (y // band_rows) % N == r: interleaved bands balance sky against mesh. Each
rank renders all passes of its rows into its full-size float accumulation buffer; then one
collective brings the frame to rank 0, which writes the 8-bit gamma image:

- "gather" (default): each rank packs its own rows (1/N of the frame) and rank 0 gathers them (RCCL
  send/recv over xGMI on the GPU box: rank 0 receives N-1 pieces of 1/N of the frame, one per link)
  and places them. Every pixel of rank 0's buffer is rewritten each frame.
- "reduce" (PT_FRAME_COLLECTIVE=reduce): the buffers, zero outside each rank's rows, are summed on
  rank 0 (a ring reduce moves about the whole buffer per rank); the buffer is cleared every frame.

Either way the result is bit-identical to one GPU (disjoint pixels; summing zeros is exact).

`launch` queues all of a frame (passes, collective, 8-bit output) on the renderer's HIP stream with
no host synchronisation. A persistent pass launch ends with a tail in which the frame's longest paths
finish on a mostly idle GPU (about 0.85 ms on the bench frame); with two or three
TiledFrames, each on its own renderer context, frames are in flight together and the next frame's
workgroups fill that tail.

The renderer is anything with the pathtracerwithcuda_amd.Renderer frame interface (setup_frame,
set_tiling, render, synchronize, finalize_u8); tests/test_multirank.py drives this same code
with gloo on the CPU.
"""
from __future__ import annotations

import os

import numpy as np


def owned_rows(height: int, band_rows: int, band_count: int, band_index: int) -> np.ndarray:
    """Rows owned by one rank (DevTiling, csrc/pt_scene.h)."""
    y = np.arange(height)
    return y[(y // band_rows) % band_count == band_index]


def owned_pixels(width: int, height: int, band_rows: int, band_count: int, band_index: int) -> np.ndarray:
    """Pixel indices owned by one rank, in the kernel's unit order (unit_to_pixel, csrc/pt_work.h)."""
    rows = owned_rows(height, band_rows, band_count, band_index)
    return (rows[:, None] * width + np.arange(width)[None, :]).reshape(-1).astype(np.int32)


class StageClock:
    """Per launch of a TiledFrame / FrameGroup: when it started, when its passes were rendered and when its collective
    was done, as HIP events on the renderer's stream (a CUDA frame) or host clock readings (a host-side renderer, whose
    steps run in host order). timings() gives (render_ms, collective_ms) per launch since the last reset():
    bench.py's per-rank breakdown of a multi-GPU run."""

    def __init__(self, stream=None):
        self.stream = stream
        self.marks: list[list] = []

    def reset(self) -> None:
        self.marks = []

    def _now(self):
        if self.stream is None:
            import time

            return time.perf_counter()
        import torch

        ev = torch.cuda.Event(enable_timing=True)
        ev.record(self.stream)
        return ev

    def start(self) -> None:
        self.marks.append([self._now()])

    def mark(self) -> None:
        if self.marks:
            self.marks[-1].append(self._now())

    def timings(self) -> list[tuple[float, float]]:
        out = []
        for m in self.marks:
            if len(m) != 3:
                continue
            if self.stream is None:
                out.append(((m[1] - m[0]) * 1e3, (m[2] - m[1]) * 1e3))
            else:
                m[2].synchronize()
                out.append((m[0].elapsed_time(m[1]), m[1].elapsed_time(m[2])))
        return out


def _placement(rows, most: int, device):
    """Where the gather's landing rows go on rank 0: row i of rank k's piece (k >= 1) is landing row
    k * most + i and frame row rows[k][i] (rank 0's own rows are rendered in place). Empty for one rank."""
    import torch

    if len(rows) == 1:
        empty = torch.zeros(0, dtype=torch.long, device=device)
        return empty, empty
    src = [k * most + torch.arange(len(rows[k]), device=device) for k in range(1, len(rows))]
    return torch.cat(src), torch.cat([rows[k] for k in range(1, len(rows))])


class TiledFrame:
    """One frame of `spp` passes on this rank's bands, collected on rank 0 (world > 1)."""

    def __init__(self, renderer, width: int, height: int, dist=None, band_rows: int = 8, device=None,
                 collective: str | None = None):
        self.r = renderer
        self.width, self.height = width, height
        self.dist = dist if (dist is not None and dist.is_available() and dist.is_initialized()) else None
        self.world = self.dist.get_world_size() if self.dist else 1
        self.rank = self.dist.get_rank() if self.dist else 0
        self.band_rows = band_rows
        self.collective = collective or os.environ.get("PT_FRAME_COLLECTIVE", "gather")
        if self.collective not in ("gather", "reduce"):
            raise ValueError(f"unknown frame collective {self.collective!r}")
        self.image = None
        self.stream = None  # the renderer's HIP stream as a torch stream (CUDA buffers only)
        # the collective path runs whenever a process group is given, a one-rank group included (bench.py --rccl:
        # RCCL's reduce / gather on the one-GPU box, bands = 1)
        self.collect = self.dist is not None
        if self.collect:
            import torch

            self.image = torch.zeros(width * height * 3, dtype=torch.float32, device=device)
            renderer.setup_frame(width, height, self.image.data_ptr())
            renderer.set_tiling(band_rows, self.world, self.rank)
            # rows of every rank, and one equal-size (padded) packing buffer per rank for the gather
            self.rows = [torch.as_tensor(owned_rows(height, band_rows, self.world, k), device=device)
                         for k in range(self.world)]
            most = max(len(rw) for rw in self.rows)
            self.part = torch.zeros(most, width, 3, dtype=torch.float32, device=device)
            self.parts = None
            if self.rank == 0:
                # the gather lands in one [world, most, width, 3] buffer; one index map places every other
                # rank's rows with a single gather + scatter (not one indexing pass per rank)
                self.landing = torch.zeros(self.world, most, width, 3, dtype=torch.float32, device=device)
                self.parts = list(self.landing.unbind(0))
                self.src_rows, self.dst_rows = _placement(self.rows, most, device)
            if self.image.is_cuda and hasattr(renderer, "stream_handle"):
                self.stream = torch.cuda.ExternalStream(renderer.stream_handle(), device=self.image.device)
        else:
            renderer.setup_frame(width, height)
        self.clock = StageClock(self.stream)

    def _on_stream(self):
        """Torch work of the frame goes on the renderer's stream (in order with its passes)."""
        import contextlib

        if self.stream is None:
            return contextlib.nullcontext()
        import torch

        return torch.cuda.stream(self.stream)

    def launch(self, cam, cfg, spp: int) -> None:
        """Queues passes 1..spp, then (world > 1) the frame's one collective and rank 0's 8-bit output,
        all in order on the renderer's HIP stream: no host synchronisation, so several TiledFrames
        (one renderer context each) can have frames in flight and one frame's tail overlaps the next
        frame's start. With a host-side renderer (no stream) every step runs in host order."""
        if not self.collect:
            self.r.render(cam, cfg, 1, spp, write_u8=2)
            return
        with self._on_stream():
            self.clock.start()
            if self.collective == "reduce":
                # rows outside this rank's bands must be zero for the reduce, and rank 0's buffer still
                # holds the previous frame's sum: clear it (ordered before the passes on this stream)
                self.image.zero_()
            self.r.render(cam, cfg, 1, spp, write_u8=0)
            if self.stream is None:
                self.r.synchronize()
            self.clock.mark()
            if self.collective == "reduce":
                self.dist.reduce(self.image, dst=0)  # the one collective of the frame
            else:
                img = self.image.view(self.height, self.width, 3)
                mine = self.rows[self.rank]
                self.part[:len(mine)] = img[mine]
                self.dist.gather(self.part, gather_list=self.parts, dst=0)  # the one collective of the frame
                if self.rank == 0:
                    img[self.dst_rows] = self.landing.view(-1, self.width, 3)[self.src_rows]
            self.clock.mark()
            if self.rank == 0:
                self.r.finalize_u8(cfg, spp)

    def synchronize(self) -> None:
        self.r.synchronize()
        if self.stream is not None:
            self.stream.synchronize()

    def render(self, cam, cfg, spp: int) -> None:
        """Passes 1..spp; rank 0 ends with the full float image and its 8-bit output."""
        self.launch(cam, cfg, spp)
        self.synchronize()

    def download(self):
        """Rank 0's frame after a render: the float running sum and the 8-bit image (numpy)."""
        return self.r.download()


class FrameGroup:
    """`frames` frames per launch on this rank's bands (pt_render_frames), then one collective per group for all
    of them: the group's float images are one [frames, height * width * 3] buffer, so the gather moves every
    frame's rows in one call (with a second for the ranks' own 8-bit rows; the reduce sums the whole stack and
    rank 0 writes the 8-bit images). The frames share one pass launch's start
    and tail instead of each paying its own, which is most of a small share's cost. Frame f
    of a launch is bit-identical to a TiledFrame's frame through the same camera.

    "gather8" moves only the 8-bit rows per group: rank 0 ends with every frame's 8-bit image, the frame the
    reference's application takes from the device each frame (Main/window.cpp:391 copies pixels_256_device
    only; the float running sum stays on the device for the next passes), while each rank keeps the float
    running sums of its own rows; collect_float() gathers those on demand. A quarter of the gather's bytes
    (3 B per pixel, not 15).

    The renderer additionally needs render_frames and finalize_u8_image (the Renderer interface)."""

    def __init__(self, renderer, width: int, height: int, frames: int, dist=None, band_rows: int = 8,
                 device=None, collective: str | None = None):
        import torch

        self.r = renderer
        self.width, self.height, self.frames = width, height, frames
        self.dist = dist if (dist is not None and dist.is_available() and dist.is_initialized()) else None
        self.world = self.dist.get_world_size() if self.dist else 1
        self.rank = self.dist.get_rank() if self.dist else 0
        self.band_rows = band_rows
        self.collective = collective or os.environ.get("PT_FRAME_COLLECTIVE", "gather")
        if self.collective not in ("gather", "gather8", "reduce"):
            raise ValueError(f"unknown frame collective {self.collective!r}")
        device = device or "cuda:0"
        n = width * height * 3
        self.stack = torch.zeros(frames, n, dtype=torch.float32, device=device)
        self.stack8 = torch.zeros(frames, n, dtype=torch.uint8, device=device)
        self.images = list(self.stack.unbind(0))
        self.images8 = list(self.stack8.unbind(0))
        renderer.setup_frame(width, height, self.images[0].data_ptr())  # the frame geometry
        self.stream = None
        self.last = 0  # frames of the last launch
        self.collect = self.dist is not None  # a one-rank group included (TiledFrame)
        if self.collect:
            renderer.set_tiling(band_rows, self.world, self.rank)
            self.rows = [torch.as_tensor(owned_rows(height, band_rows, self.world, k), device=device)
                         for k in range(self.world)]
            most = max(len(rw) for rw in self.rows)
            self.most = most
            self.part = torch.zeros(frames, most, width, 3, dtype=torch.float32, device=device)
            # the gather also moves each rank's 8-bit rows, written by its own accumulate launch (the same per-pixel
            # gamma function as a finalize on rank 0, which then has none to run): 3 B more per pixel on the links
            self.part8 = torch.zeros(frames, most, width, 3, dtype=torch.uint8, device=device)
            self.parts = self.parts8 = None
            if self.rank == 0:
                self.landing = torch.zeros(self.world, frames, most, width, 3, dtype=torch.float32, device=device)
                self.landing8 = torch.zeros(self.world, frames, most, width, 3, dtype=torch.uint8, device=device)
                self.parts = list(self.landing.unbind(0))
                self.parts8 = list(self.landing8.unbind(0))
                self.src_rows, self.dst_rows = _placement(self.rows, most, device)
        if self.stack.is_cuda and hasattr(renderer, "stream_handle"):
            self.stream = torch.cuda.ExternalStream(renderer.stream_handle(), device=self.stack.device)
        self.clock = StageClock(self.stream)

    def _on_stream(self):
        import contextlib

        if self.stream is None:
            return contextlib.nullcontext()
        import torch

        return torch.cuda.stream(self.stream)

    def launch(self, cams, cfg, spp: int) -> None:
        """Queues passes 1..spp of len(cams) <= frames frames (frame f through cams[f]), then (world > 1) the
        group's collective (gather: the float and the 8-bit rows of every rank; gather8: the 8-bit rows; reduce: the
        float stack, then rank 0's 8-bit outputs), in order on the renderer's stream."""
        n = len(cams)
        if not 1 <= n <= self.frames:
            raise ValueError(f"1..{self.frames} cameras per launch, got {n}")
        self.last = n
        if not self.collect:
            with self._on_stream():
                self.r.render_frames(list(cams), cfg, self.images[:n], self.images8[:n], 1, spp, write_u8=2)
            return
        with self._on_stream():
            self.clock.start()
            if self.collective == "reduce":
                self.stack[:n].zero_()  # rows outside this rank's bands must be zero for the reduce
                self.r.render_frames(list(cams), cfg, self.images[:n], None, 1, spp, write_u8=0)
                if self.stream is None:
                    self.r.synchronize()
                self.clock.mark()
                self.dist.reduce(self.stack, dst=0)  # the one collective of the group
                self.clock.mark()
                if self.rank == 0:
                    for f in range(n):
                        self.r.finalize_u8_image(cfg, spp, self.images[f], self.images8[f])
                return
            self.r.render_frames(list(cams), cfg, self.images[:n], self.images8[:n], 1, spp, write_u8=2)
            if self.stream is None:
                self.r.synchronize()
            self.clock.mark()
            if self.collective == "gather":
                self._gather_rows(self.stack, self.part, self.parts, self.landing if self.rank == 0 else None, n)
            self._gather_rows(self.stack8, self.part8, self.parts8, self.landing8 if self.rank == 0 else None, n)
            self.clock.mark()

    def _gather_rows(self, stack, part, parts, landing, n: int) -> None:
        """Frames 0..n-1 of `stack`: every rank's own rows to rank 0 (one gather of n frames' pieces; a launch of
        fewer frames than the group moves only its own), placed there."""
        img = stack.view(self.frames, self.height, self.width, 3)
        mine = self.rows[self.rank]
        part[:n, :len(mine)] = img[:n, mine]
        self.dist.gather(part[:n], gather_list=[p[:n] for p in parts] if parts is not None else None, dst=0)
        if landing is not None:
            land = landing[:, :n].transpose(0, 1).reshape(n, self.world * self.most, self.width, 3)
            img[:n, self.dst_rows] = land[:, self.src_rows]

    def collect_float(self) -> None:
        """"gather8": the float running sums of the last launch's frames, which stay on the ranks that rendered
        their rows, gathered to rank 0 (a collective: every rank calls it). Queued on the renderer's stream; other
        collectives need nothing."""
        if not self.collect or self.collective != "gather8":
            return
        with self._on_stream():
            self._gather_rows(self.stack, self.part, self.parts, self.landing if self.rank == 0 else None, self.last)

    def synchronize(self) -> None:
        self.r.synchronize()
        if self.stream is not None:
            self.stream.synchronize()

    def render(self, cam, cfg, spp: int) -> None:
        """One frame (frame 0 of the group); rank 0 ends with its float image and 8-bit output."""
        self.launch([cam], cfg, spp)
        self.synchronize()

    def download(self, frame: int = 0):
        """Frame `frame` of the last launch as (float image, 8-bit image), numpy [height, width, 3]."""
        shape = (self.height, self.width, 3)
        return (self.stack[frame].cpu().numpy().reshape(shape).copy(),
                self.stack8[frame].cpu().numpy().reshape(shape).copy())


class StageWatch:
    """Fail-fast for one rank of a multi-GPU run: the rank names the stage it is in (stage()), and a watchdog thread
    ends the process when a stage outlives its limit, with one stderr line naming the rank and the stage, and exit
    code 124. A rank whose peer never reaches a collective (a stalled or lost rank) thus exits non-zero on its own
    instead of waiting for the job's outer time limit, and torch.distributed.run then ends the other ranks. The
    thread only reads a clock: it works while the main thread is blocked in a collective or a device wait (those
    release the GIL)."""

    def __init__(self, rank: int, limit_s: float, tag: str = "[bench]", exit_code: int = 124):
        import threading
        import time

        self.rank, self.limit_s, self.tag, self.exit_code = rank, float(limit_s), tag, exit_code
        self._time = time.monotonic
        self._name, self._since, self._limit = "start", self._time(), self.limit_s
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._watch, name="stage-watch", daemon=True)
        if self.limit_s > 0:
            self._thread.start()

    def stage(self, name: str, limit_s: float | None = None) -> None:
        self._name, self._since = name, self._time()
        self._limit = self.limit_s if limit_s is None else float(limit_s)

    def _watch(self) -> None:
        import sys

        while not self._stop.wait(0.25):
            waited = self._time() - self._since
            if waited > self._limit:
                print(f"{self.tag} rank {self.rank}: stage '{self._name}' did not finish within {self._limit:.0f} s "
                      f"({waited:.1f} s); exiting with {self.exit_code}", file=sys.stderr, flush=True)
                os._exit(self.exit_code)

    def close(self) -> None:
        self._stop.set()
