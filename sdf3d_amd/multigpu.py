"""Multi-device frame driver: interleaved row-block tiling + gather to rank 0.

One process per GPU (torch.distributed; "nccl" is RCCL over xGMI on ROCm).
Rank r of N renders the 8-row blocks r, r+N, r+2N, ... of every frame
(sdf_tiling {8, r, N}: per-rank work within 1.006x of the mean at N = 8,
SURVEY.md 8(e), where contiguous bands are 1.75x), packed densely.  Rank 0
gathers the N packed parts and scatters the rows into the frame
(sdf_deinterleave).  The reference has no multi-device path at all (one GL
context, /root/reference/Code/src/main.cpp:48,53).

Pipelining: two buffer sets.  The gather of frame i is asynchronous (RCCL
runs on its own stream) and rank 0 deinterleaves it on a side stream, so
frame i+1 renders while frame i is in flight; a buffer is reused only after
the collective (and on rank 0 the deinterleave) that read it has finished.

The render and deinterleave steps are injected, so the same driver runs the
HIP kernels on GPUs (bench.py) and a CPU stand-in under the gloo backend
(tests/test_multigpu_cpu.py).
"""
from __future__ import annotations

from typing import Callable, Optional

import numpy as np


def owned_rows_py(height: int, rank: int, world: int, block_rows: int = 8) -> int:
    """Rows of an interleaved tiling, in Python (mirror of sdf_owned_rows)."""
    nblocks = (height + block_rows - 1) // block_rows
    rows = 0
    for b in range(rank, nblocks, world):
        rows += min(block_rows, height - b * block_rows)
    return rows


def owned_row_ids(height: int, rank: int, world: int, block_rows: int = 8) -> np.ndarray:
    """Frame rows (y) owned by `rank`, in packed order."""
    y = np.arange(height)
    b = y // block_rows
    return y[(b % world) == rank] if world > 1 else y


def deinterleave_index(height: int, world: int, stride: int, block_rows: int = 8) -> np.ndarray:
    """For every frame row y, its row index in the gathered parts buffer
    (part r occupies rows [r*stride, (r+1)*stride))."""
    y = np.arange(height)
    b = y // block_rows
    r = b % world
    pr = (b // world) * block_rows + (y - b * block_rows)
    return r * stride + pr


class FrameDriver:
    def __init__(self, width: int, height: int, rank: int, world: int, device,
                 render_fn: Callable, deinterleave_fn: Callable, block_rows: int = 8,
                 nbuf: int = 2, dist=None, dtype=None, wire_channels: int = 4):
        import torch
        self.torch = torch
        self.W, self.H = width, height
        self.rank, self.world = rank, world
        self.B = block_rows
        self.device = device
        self.render_fn = render_fn          # render_fn(out_rows_tensor, stream) -> None
        self.deinterleave_fn = deinterleave_fn  # (parts, world, stride, W, H, B, out, stream)
        self.dist = dist
        self.rows = owned_rows_py(height, rank, world, block_rows)
        self.stride = owned_rows_py(height, 0, world, block_rows)  # rank 0 owns the most
        self.gpu = getattr(device, "type", str(device)).startswith("cuda")
        self.nbuf = nbuf if world > 1 else 1
        dtype = dtype or torch.float32   # the framebuffer format on the wire
        mk = lambda *shape: torch.empty(shape, dtype=dtype, device=device)  # noqa: E731
        wc = wire_channels   # 3: RGB32F wire, alpha restored by the deinterleave
        self.local = [mk(self.stride, width, wc if world > 1 else 4) for _ in range(self.nbuf)]
        self.works = [None] * self.nbuf
        self.root = rank == 0
        if world > 1 and self.root:
            self.gathered = [mk(world * self.stride, width, wc) for _ in range(self.nbuf)]
            self.frames = [mk(height, width, 4) for _ in range(self.nbuf)]
            self.deint_done = [None] * self.nbuf
        self.stream = torch.cuda.current_stream(device) if self.gpu else None
        self.side = torch.cuda.Stream(device=device) if (self.gpu and world > 1) else None

    def step(self, i: int, ev_before=None, ev_after=None) -> None:
        """Render frame i (and start its gather).  Optional events bracket the
        render launch on the render stream (kernel timing)."""
        torch = self.torch
        b = i % self.nbuf
        if self.world > 1 and self.works[b] is not None:
            self.works[b].wait()            # the gather of frame i - nbuf has read local[b]
            self.works[b] = None
            if not self.gpu and self.root:
                self._cpu_finish(b)
        if ev_before is not None:
            ev_before.record(self.stream)
        self.render_fn(self.local[b][:self.rows], self.stream)
        if ev_after is not None:
            ev_after.record(self.stream)
        if self.world == 1:
            return
        dist = self.dist
        if self.root:
            if self.gpu and self.deint_done[b] is not None:
                self.stream.wait_event(self.deint_done[b])  # deinterleave i-nbuf read gathered[b]
            glist = [self.gathered[b][r * self.stride:(r + 1) * self.stride]
                     for r in range(self.world)]
            self.works[b] = dist.gather(self.local[b], gather_list=glist, dst=0, async_op=True)
            if self.gpu:
                with torch.cuda.stream(self.side):
                    self.works[b].wait()    # side stream waits for the collective
                    self.deinterleave_fn(self.gathered[b], self.world, self.stride, self.W,
                                         self.H, self.B, self.frames[b], self.side)
                    ev = torch.cuda.Event()
                    ev.record(self.side)
                    self.deint_done[b] = ev
        else:
            self.works[b] = dist.gather(self.local[b], gather_list=None, dst=0, async_op=True)

    def _cpu_finish(self, b: int) -> None:
        self.deinterleave_fn(self.gathered[b], self.world, self.stride, self.W, self.H, self.B,
                             self.frames[b], None)

    def drain(self) -> None:
        for b, w in enumerate(self.works):
            if w is not None:
                w.wait()
                self.works[b] = None
                if not self.gpu and self.root and self.world > 1:
                    self._cpu_finish(b)
        if self.gpu:
            self.torch.cuda.synchronize(self.device)

    def frame(self, i: int):
        """Rank 0's assembled frame of step i (valid after drain())."""
        if self.world == 1:
            return self.local[0][:self.H]
        if not self.root:
            return None
        return self.frames[i % self.nbuf]


def deinterleave_torch(parts, world, stride, W, H, B, out, stream=None):
    """CPU stand-in for sdf_deinterleave (index math of deinterleave.hip;
    3-channel parts get alpha = 1)."""
    import torch
    idx = torch.as_tensor(deinterleave_index(H, world, stride, B), device=parts.device)
    rows = parts.index_select(0, idx)
    if rows.shape[-1] == 3:
        out[..., :3].copy_(rows)
        out[..., 3] = 1.0
    else:
        out.copy_(rows)
    return out
