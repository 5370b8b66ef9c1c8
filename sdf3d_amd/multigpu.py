"""Multi-device frame driver: interleaved row-block tiling + gather to rank 0.

One process per GPU (torch.distributed; "nccl" is RCCL over xGMI on ROCm).
Rank r of N renders the 8-row blocks r, r+N, r+2N, ... of every frame
(sdf_tiling {8, r, N}: per-rank work within 1.006x of the mean at N = 8,
SURVEY.md 8(e), where contiguous bands are 1.75x), packed densely.  Rank 0
gathers the N parts and assembles the frame.  With the TILES wire the
shares can be unequal (shares = (a, b): rank 0 owns a blocks and every other
rank b per period of a + b (N - 1), choose_shares): rank 0 also decodes the
other ranks' streams, so at N = 8 it gets 1 block in 22.  The reference has no
multi-device path at all (one GL context, /root/reference/Code/src/main.cpp:48,53).

Wire formats (what crosses xGMI):
  "raw"    the packed rows themselves (RGBA, or RGB32F with alpha restored),
           scattered into the frame by sdf_deinterleave.
  "tiles"  the TILES stream (include/sdf_abi.h): lossless compressed RGB32F,
           ~3.2 instead of 12 bytes per pixel on the 4K CSG frame, written by
           the render kernel and decoded straight into the frame rows by
           sdf_tiles_decode.  Streams vary in length, so the ranks agree on
           each frame's byte count (an all-reduce MAX of one integer) before
           gathering that many bytes from every rank.

Collective streams: the TILES size agreement has a process group of its
own (its own RCCL communicator and stream) so it never queues behind a
gather.

Pipelining: nbuf buffer sets and one render stream per set, so frame
i+1 starts while frame i's slowest tiles finish (a launch of one rank's
share ends with its slowest 8x8 tile: ~0.11 ms for 1/8 of the 4K frame on
one stream, ~0.05 ms per frame on alternating streams) and while frame i is
gathered (RCCL) and assembled on rank 0 (TILES: on frame i's own render
stream; raw rows: on a side stream).  In "tiles" mode the gather of frame i
is issued `lag` steps later (after frame i + lag's render is enqueued), once
frame i's agreed size has reached the host: the agreed size is copied into
pinned host memory on the frame's stream and read after an event wait, so
with lag >= 2 the host finds it there without stalling and always keeps
frames queued ahead of the GPU (with lag 1 it waits for the frame just
rendered while only one frame is queued).  Every collective is issued in
the same order on all ranks, in an order that keeps the single RCCL stream
from holding one frame's transfer behind the next one's render.  A buffer
is reused only after the collective (and on rank 0 the assembly) that read
it has finished: lag <= nbuf - 1.

The render and assembly steps are injected, so the same driver runs the HIP
kernels on GPUs (bench.py) and CPU stand-ins under the gloo backend
(tests/test_multigpu_cpu.py).
"""
from __future__ import annotations

from typing import Callable, Optional

import numpy as np

from . import abi


def share_blocks(rank: int, world: int, shares=(1, 1)) -> tuple[int, int, int, int]:
    """(first block, run, period, step) of `rank` in the tiling with shares
    (a, b): per period of P = a + b (world - 1) blocks rank 0 owns the first
    a, rank r >= 1 the b blocks a + r - 1 + j (world - 1), j < b, interleaved
    with the other peers' (renderer.tiling, sdf_tiling.run_step)."""
    a, b = shares
    period = a + b * (world - 1)
    if rank == 0:
        return (0, a, period, 1)
    return (a + rank - 1, b, period, world - 1 if b > 1 else 1)


def owned_row_ids(height: int, rank: int, world: int, block_rows: int = 8,
                  shares=(1, 1)) -> np.ndarray:
    """Frame rows (y) owned by `rank`, in packed order."""
    first, run, period, step = share_blocks(rank, world, shares)
    y = np.arange(height)
    b = y // block_rows
    o = (b - first) % period
    return y[(b >= first) & (o % step == 0) & (o // step < run)]


def owned_rows_py(height: int, rank: int, world: int, block_rows: int = 8,
                  shares=(1, 1)) -> int:
    """Rows of a rank's tiling, in Python (mirror of sdf_owned_rows)."""
    return int(owned_row_ids(height, rank, world, block_rows, shares).size)


# Per-frame costs of the 4K CSG frame (C4) on one MI355X, in ms of one whole
# frame (tools/root_probe.py, profiles/r01_root_probe_C4.json): the rows
# rendered straight into the frame; the rows rendered as a TILES stream
# (render + encoding); the TILES decode (0.047 alone, 0.043 beside rank 0's
# own render: rank 0's per-frame time minus its render share); the floor of a lone small render
# (its launch ends with its slowest tiles: 1/15 and 1/22 of the frame both
# take ~0.027 ms alone, but beside the decode, as rank 0 runs them, the
# tail overlaps and the two simply add); and the wire: the whole frame's
# TILES stream (3.21 B/pixel, 26.6 MB) over one xGMI link at ~65 GB/s per
# direction (85% of half the 153 GB/s bidirectional link figure) -- every
# peer ships its share to rank 0 over its own link, concurrently.
FRAME_COSTS_MS = {"render": 0.373, "render_tiles": 0.444, "decode": 0.043, "floor": 0.026,
                  "wire": 0.41}

# Shares measured best on one MI355X with rank 0's and the busiest peer's
# per-frame GPU work (tools/root_probe.py, 4 streams, shading-term TILES;
# profiles/r03_share_probe_C4.json), max(rank 0, peer) ms per frame:
#   N = 2: 1:1 0.188, 4:3 0.204, 3:2 0.212
#   N = 4: 3:4 0.102, 4:5 0.103, 2:3 0.105, 1:1 0.112
#   N = 8: 2:7 0.0532, 1:4 0.0538, 1:3 0.0548
# Round 5 at N = 8, rank 0's whole loop with rotated (non-resident) peer
# streams and the busiest peer (tools/root_rccl_probe.py, root_probe.py;
# profiles/r05_root_rccl_probe_*.json, r05_root_probe_exact_C4_*.json),
# max(rank 0, peer) ms per frame: exact 1:7 0.0735, 1:4 0.0739, 2:7 0.0762;
# fast rank 0 1:7 0.0564, 1:4 0.0612, 2:7 0.0630 -- and with RCCL's transfer
# work on rank 0 too, 1:7 is the lightest (exact 0.126 against 0.137-0.140).
# The cost model below serves the other world sizes (and explicit costs).
MEASURED_SHARES = {2: (1, 1), 4: (3, 4), 8: (1, 7)}


def choose_shares(world: int, costs=None, max_blocks: int = 4) -> tuple[int, int]:
    """Shares (a, b) for the TILES frame driver: rank 0 renders its rows in
    place and decodes everyone else's, so it gets fewer rows.  Minimises the
    larger of rank 0's per-frame work, max(a/P render + (1 - a/P) decode,
    floor), and a peer's, max(b/P render_tiles, floor, b/P wire) (P = a + b
    (world - 1): a peer's frames are pipelined, so its period is the slower of
    its render and its link); ties go to the shorter period.  Measured at
    N = 8 (rank 0 / busiest peer GPU work, ms per frame, escape-coded TILES):
    1:2 0.064 / 0.057, 1:3 0.058 / 0.060, 1:4 0.055 / 0.061, 2:7 0.055 /
    0.062 (profiles/r01_root_probe_C4.json)."""
    if world <= 1:
        return (1, 1)
    if costs is None and world in MEASURED_SHARES:
        return MEASURED_SHARES[world]
    c = costs or FRAME_COSTS_MS
    best = None
    for period_first in range(2, 2 * max_blocks + 1):
        for a in range(1, max_blocks + 1):
            for b in range(1, max_blocks + 1):
                if a + b != period_first:
                    continue
                P = a + b * (world - 1)
                floor = c.get("floor", 0.0)
                root = max(a / P * c["render"] + (1 - a / P) * c["decode"], floor)
                peer = max(b / P * c["render_tiles"], floor, b / P * c.get("wire", 0.0))
                t = max(root, peer)
                if best is None or t < best[0] * (1 - 1e-6):
                    best = (t, (a, b))
    return best[1]


def deinterleave_index(height: int, world: int, stride: int, block_rows: int = 8) -> np.ndarray:
    """For every frame row y, its row index in the gathered parts buffer
    (part r occupies rows [r*stride, (r+1)*stride))."""
    y = np.arange(height)
    b = y // block_rows
    r = b % world
    pr = (b // world) * block_rows + (y - b * block_rows)
    return r * stride + pr


def tiles_data_offset(width: int, rows: int) -> int:
    """Offset of the plane data in a TILES stream of `rows` packed rows
    (include/sdf_abi.h): header, offset table, 16-B heads."""
    n = ((width + 7) // 8) * ((rows + 7) // 8)
    return (abi.TILES_HEADER_BYTES + 4 * n + 15) // 16 * 16 + 16 * n


class FrameDriver:
    def __init__(self, width: int, height: int, rank: int, world: int, device,
                 render_fn: Callable, deinterleave_fn: Callable, block_rows: int = 8,
                 nbuf: int = 3, dist=None, dtype=None, wire_channels: int = 4,
                 wire: str = "raw", wire_bytes: Optional[int] = None,
                 root_render_fn: Optional[Callable] = None, shares=(1, 1),
                 lag: int = 2, collectives_at_world1: bool = False):
        import collections

        import torch
        self.torch = torch
        self.W, self.H = width, height
        self.rank, self.world = rank, world
        self.B = block_rows
        self.device = device
        self.render_fn = render_fn          # render_fn(out_buffer, stream) -> None
        # "tiles" mode, rank 0: render its own rows straight into the frame
        # (root_render_fn(frame, stream), SDF_TILING_FRAME_ROWS) and send an
        # empty stream (ntiles = 0, skipped by the decode)
        self.root_render_fn = root_render_fn if (wire == "tiles" and rank == 0) else None
        # raw: (parts, world, stride_rows, W, H, B, out, stream)
        # tiles: (parts, world, part_stride_bytes, W, H, B, out, stream)
        self.deinterleave_fn = deinterleave_fn
        self.dist = dist
        self.shares = tuple(shares)
        if self.shares != (1, 1) and (wire != "tiles" or world == 1):
            raise ValueError("unequal shares need the tiles wire (the raw rows' "
                             "sdf_deinterleave takes the plain interleave)")
        self.rows = owned_rows_py(height, rank, world, block_rows, self.shares)
        # the largest part sizes every rank's buffers
        self.stride = max(owned_rows_py(height, r, world, block_rows, self.shares)
                          for r in range(world))
        self.gpu = getattr(device, "type", str(device)).startswith("cuda")
        self.nbuf = nbuf
        # collectives_at_world1: run the N > 1 code path with one rank (host
        # cost probes of the collectives, tools/driver_probe.py)
        self.multi = world > 1 or collectives_at_world1
        self.wire = wire if self.multi else "raw"
        self.lag = lag
        if self.wire == "tiles" and not 1 <= lag <= nbuf - 1:
            raise ValueError(f"lag must be in [1, nbuf - 1] (nbuf {nbuf}), got {lag}")
        self.root = rank == 0
        self.works = [None] * nbuf
        if self.wire == "tiles":
            if wire_bytes is None:
                from .renderer import tiles_bytes
                wire_bytes = tiles_bytes(width, self.stride)
            self.cap = wire_bytes                     # part pitch in bytes
            # the largest part's stream header is the longest: its data
            # offset + the largest `used` covers every rank's stream
            self.data_off = tiles_data_offset(width, self.stride)
            self.local = [torch.zeros((self.cap,), dtype=torch.uint8, device=device)
                          for _ in range(nbuf)]
            self.size_works = [None] * nbuf
            self.pending = collections.deque()        # (i, b) rendered, not yet shipped
            if self.gpu:
                # agreed sizes land here (pinned: an async copy on the frame's
                # stream, read after its event)
                self.size_host = torch.zeros((nbuf,), dtype=torch.int32, pin_memory=True)
                self.size_ev = [torch.cuda.Event() for _ in range(nbuf)]
            # the size agreement runs in its own process group: its own RCCL
            # communicator and stream, so frame i's all-reduce completes
            # while frame i-1's gather is still on the links, and the
            # gathers go back to back (in one group they would alternate
            # with the all-reduces and the host's turnaround between them)
            self.size_group = dist.new_group(ranks=list(range(world))) if dist else None
            if self.root:
                self.gathered = [torch.empty((world * self.cap,), dtype=torch.uint8,
                                             device=device) for _ in range(nbuf)]
        else:
            dtype = dtype or torch.float32   # the framebuffer format on the wire
            mk = lambda *shape: torch.empty(shape, dtype=dtype, device=device)  # noqa: E731
            wc = wire_channels   # 3: RGB32F wire, alpha restored by the deinterleave
            self.local = [mk(self.stride, width, wc if self.multi else 4) for _ in range(nbuf)]
            if self.multi and self.root:
                self.gathered = [mk(world * self.stride, width, wc) for _ in range(nbuf)]
        if self.multi and self.root:
            self.frames = [torch.empty((height, width, 4), dtype=torch.float32 if self.wire ==
                                       "tiles" else (dtype or torch.float32), device=device)
                           for _ in range(nbuf)]
            self.asm_done = [None] * nbuf
        if self.gpu:
            self.streams = [torch.cuda.Stream(device=device) for _ in range(nbuf)]
            self.side = torch.cuda.Stream(device=device) if self.multi else None
        else:
            self.streams = [None] * nbuf
            self.side = None

    def _ctx(self, stream):
        import contextlib
        return self.torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext()

    def step(self, i: int, ev_before=None, ev_after=None) -> None:
        """Render frame i (and ship frame i, or in "tiles" mode frame i-1).
        Optional events bracket the render launch on its stream."""
        b = i % self.nbuf
        s = self.streams[b]
        if self.works[b] is not None:       # the gather of frame i - nbuf read local[b]
            with self._ctx(s):
                self.works[b].wait()
            self.works[b] = None
            if not self.gpu and self.root and self.wire == "raw":
                self._cpu_finish(b)
        out = self.local[b] if self.wire == "tiles" else self.local[b][:self.rows]
        if not self.multi:
            # no collectives: the stream goes to the calls explicitly (a
            # stream context costs more host time than a small frame renders)
            if ev_before is not None:
                ev_before.record(s)
            self.render_fn(out, s)
            if ev_after is not None:
                ev_after.record(s)
            return
        with self._ctx(s):
            if ev_before is not None:
                ev_before.record(s)
            if self.root_render_fn is not None:
                self.root_render_fn(self.frames[b], s)
            else:
                self.render_fn(out, s)
            if ev_after is not None:
                ev_after.record(s)
        if self.wire == "tiles":
            self._step_tiles(i, b, s)
        else:
            self._step_raw(b, s)

    # ---- raw rows ------------------------------------------------------------
    def _step_raw(self, b, s):
        torch, dist = self.torch, self.dist
        with self._ctx(s):
            if self.root:
                if self.gpu and self.asm_done[b] is not None:
                    s.wait_event(self.asm_done[b])   # assembly of i - nbuf read gathered[b]
                glist = [self.gathered[b][r * self.stride:(r + 1) * self.stride]
                         for r in range(self.world)]
                self.works[b] = dist.gather(self.local[b], gather_list=glist, dst=0,
                                            async_op=True)
            else:
                self.works[b] = dist.gather(self.local[b], gather_list=None, dst=0,
                                            async_op=True)
        if self.root and self.gpu:
            with torch.cuda.stream(self.side):
                self.works[b].wait()            # side stream waits for the collective
                self.deinterleave_fn(self.gathered[b], self.world, self.stride, self.W,
                                     self.H, self.B, self.frames[b], self.side)
                ev = torch.cuda.Event()
                ev.record(self.side)
                self.asm_done[b] = ev

    def _cpu_finish(self, b: int) -> None:
        self.deinterleave_fn(self.gathered[b], self.world, self.stride, self.W, self.H, self.B,
                             self.frames[b], None)

    # ---- TILES streams -------------------------------------------------------
    def _step_tiles(self, i, b, s):
        import torch.distributed as tdist
        if len(self.pending) >= self.lag:
            self._ship(*self.pending.popleft())
        with self._ctx(s):
            # the ranks agree on the largest `used` (header word 0, reduced in
            # place: the decoder reads only the offset table and the heads)
            self.size_works[b] = self.dist.all_reduce(self._used(b), op=tdist.ReduceOp.MAX,
                                                      group=self.size_group, async_op=True)
            if self.gpu:
                self.size_works[b].wait()          # stream s waits for the reduction
                self.size_host[b:b + 1].copy_(self._used(b), non_blocking=True)
                self.size_ev[b].record(s)
        self.pending.append((i, b))

    def _used(self, b):
        return self.local[b][:4].view(self.torch.int32)

    def _ship(self, i, b):
        """Gather frame i's streams (their agreed length) and assemble on rank 0."""
        torch, dist = self.torch, self.dist
        s = self.streams[b]
        with self._ctx(s):
            # host wait: frame i rendered (and its size reduced) everywhere
            if self.gpu:
                self.size_ev[b].synchronize()
                used = int(self.size_host[b])
            else:
                self.size_works[b].wait()
                used = int(self._used(b).item())
            count = self.data_off + used
            self.size_works[b] = None
            if self.root:
                # the decode of frame i - nbuf, which read gathered[b], is
                # already on stream s, which the gather waits for
                glist = [self.gathered[b][r * self.cap:r * self.cap + count]
                         for r in range(self.world)]
                self.works[b] = dist.gather(self.local[b][:count], gather_list=glist, dst=0,
                                            async_op=True)
            else:
                self.works[b] = dist.gather(self.local[b][:count], gather_list=None, dst=0,
                                            async_op=True)
        if self.root:
            if self.gpu:
                # the decode goes on the frame's own render stream: the next
                # render into frames[b] (frame i + nbuf) has to follow it
                # anyway, and measured on one MI355X (tools/root_probe.py)
                # the root's frame period is 0.074 ms this way against 0.093
                # with the decodes on a side stream of their own
                with torch.cuda.stream(s):
                    self.works[b].wait()
                    self.deinterleave_fn(self.gathered[b], self.world, self.cap, self.W, self.H,
                                         self.B, self.frames[b], s, shares=self.shares)
            else:
                self.works[b].wait()
                self.works[b] = None
                self.deinterleave_fn(self.gathered[b], self.world, self.cap, self.W, self.H,
                                     self.B, self.frames[b], None, shares=self.shares)

    def drain(self) -> None:
        while self.wire == "tiles" and self.pending:
            self._ship(*self.pending.popleft())
        for b, w in enumerate(self.works):
            if w is not None:
                w.wait()
                self.works[b] = None
                if not self.gpu and self.root and self.multi and self.wire == "raw":
                    self._cpu_finish(b)
        if self.gpu:
            self.torch.cuda.synchronize(self.device)

    def frame(self, i: int):
        """Rank 0's assembled frame of step i (valid after drain(); the last
        nbuf frames are kept)."""
        if not self.multi:
            return self.local[i % self.nbuf][:self.H]
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
