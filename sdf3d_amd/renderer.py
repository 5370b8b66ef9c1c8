"""Host-side renderer over the C-ABI (Python mirror of the C++ ``sdf::Renderer``).

One ``Renderer.render`` call is one frame of the reference's draw,
``gl->plot(sh, proj_mode)`` (/root/reference/Code/src/main.cpp:95): the scene,
camera, light and material go in, an RGBA float framebuffer comes out.  The
framebuffer lives in device memory allocated through PyTorch (plumbing only);
all arithmetic runs in the HIP kernels of ``libsdf3d.so``.
"""
from __future__ import annotations

import ctypes as C

from . import abi
from .scenes import Frame


def tiling(rank: int = 0, world: int = 1, block_rows: int = 8,
           frame_rows: bool = False, shares: tuple[int, int] = (1, 1)) -> abi.sdf_tiling:
    """Interleaved row-block tiling of `world` devices.

    shares = (a, b): per period of P = a + b (world - 1) blocks, rank 0 owns
    the first a blocks and rank r >= 1 the b blocks a + r - 1 + j (world - 1),
    j < b, interleaved with the other peers' (so a frame whose block count is
    not a multiple of P gives the last partial period to distinct ranks;
    (1, 1): device r owns blocks r, r + world, ...).  frame_rows: write the
    rows at their frame positions of a full-height buffer
    (SDF_TILING_FRAME_ROWS)."""
    a, b = shares
    if a < 1 or b < 1:
        raise ValueError(f"shares must be >= 1, got {shares}")
    t = abi.sdf_tiling()
    t.block_rows = block_rows
    t.block_stride = a + b * (world - 1)
    t.first_block = 0 if rank == 0 else a + rank - 1
    t.block_run = a if rank == 0 else b
    t.run_step = 1 if rank == 0 or b == 1 else world - 1
    t.flags = abi.TILING_FRAME_ROWS if frame_rows else 0
    return t


def buffer_rows(height: int, t: abi.sdf_tiling | None = None) -> int:
    """Rows of the output buffer of a render with tiling `t`."""
    if t is not None and t.flags & abi.TILING_FRAME_ROWS:
        return height
    return owned_rows(height, t)


def owned_rows(height: int, t: abi.sdf_tiling | None = None) -> int:
    n = abi.load_library().sdf_owned_rows(height, C.byref(t) if t is not None else None)
    if n < 0:
        abi.check(n, "sdf_owned_rows")
    return n


def torch_dtype(fmt: int):
    """torch element type of a framebuffer format."""
    import torch
    return {abi.FORMAT_RGBA32F: torch.float32, abi.FORMAT_RGBA16F: torch.float16,
            abi.FORMAT_RGBA8: torch.uint8, abi.FORMAT_RGB32F: torch.float32,
            abi.FORMAT_TILES: torch.uint8, abi.FORMAT_SHADE32F: torch.float32}[fmt]


def tiles_bytes(width: int, rows: int) -> int:
    """Capacity of a TILES stream (sdf_tiles_bytes)."""
    n = abi.load_library().sdf_tiles_bytes(width, rows)
    if n < 0:
        abi.check(int(n), "sdf_tiles_bytes")
    return int(n)


def tiles_stream_bytes(stream) -> int:
    """Meaningful prefix of a TILES stream on the host: table + used records."""
    import numpy as np
    used, n = np.frombuffer(bytes(stream[:8].cpu().numpy()), dtype=np.uint32)
    return (abi.TILES_HEADER_BYTES + 4 * int(n) + 15) // 16 * 16 + 16 * int(n) + int(used)


def channels(fmt: int) -> int:
    return abi.FORMAT_CHANNELS[fmt]


class Renderer:
    """Renders frames on one HIP device through ``sdf_render``."""

    def __init__(self, device=None):
        import torch
        self.torch = torch
        self.lib = abi.load_library()
        if not torch.cuda.is_available():
            raise RuntimeError("no HIP device visible: the renderer has no CPU path")
        self.device = torch.device(device if device is not None else "cuda")
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())

    def _on_device(self):
        """The HIP calls must run with this renderer's device current; enter
        a device context only when it is not (the context costs host time)."""
        import contextlib
        if self.torch.cuda.current_device() == self.device.index:
            return contextlib.nullcontext()
        return self.torch.cuda.device(self.device)

    def _stream(self, stream):
        if stream is None:
            stream = self.torch.cuda.current_stream(self.device)
        return C.c_void_p(stream.cuda_stream)

    def alloc(self, frame: Frame, t: abi.sdf_tiling | None = None, steps: bool = False):
        rows = buffer_rows(frame.params.height, t)
        w = frame.params.width
        fmt = frame.params.output_format
        if fmt == abi.FORMAT_TILES:
            rgba = self.torch.empty((tiles_bytes(w, rows),), dtype=self.torch.uint8,
                                    device=self.device)
        else:
            rgba = self.torch.empty((rows, w, channels(fmt)), dtype=torch_dtype(fmt),
                                    device=self.device)
        st = (self.torch.empty((rows, w, 2), dtype=self.torch.int32, device=self.device)
              if steps else None)
        return rgba, st

    def schedule(self, rows: int, period: int = 1) -> "Schedule":
        """A render schedule for frames of `rows` packed rows (sdf_schedule):
        pass it to ``render(..., schedule=)`` to dispatch the rows' 8-row
        blocks costliest first (bit-identical output)."""
        return Schedule(self, rows, period)

    def render(self, frame: Frame, t: abi.sdf_tiling | None = None, out=None,
               steps=False, stream=None, schedule: "Schedule | None" = None):
        """Render the rows owned by tiling `t` (None = whole frame).

        Returns (rgba[rows, W, 4] float32, steps[rows, W, 2] int32 or None), both
        on the device, asynchronous on `stream` (default: torch's current).
        `schedule`: dispatch order of the row blocks (sdf_render_scheduled)."""
        torch = self.torch
        rows = buffer_rows(frame.params.height, t)
        w = frame.params.width
        if out is None:
            rgba, st = self.alloc(frame, t, steps is True)
        else:
            rgba = out
            st = None
        if isinstance(steps, torch.Tensor):
            st = steps
        if frame.params.output_format == abi.FORMAT_TILES:
            if rows and (rgba.dtype != torch.uint8 or rgba.numel() < tiles_bytes(w, rows)
                         or not rgba.is_contiguous() or rgba.device != self.device):
                raise ValueError(f"a TILES stream needs a contiguous uint8 tensor of "
                                 f">= {tiles_bytes(w, rows)} bytes on {self.device}")
        else:
            dt = torch_dtype(frame.params.output_format)
            ch = channels(frame.params.output_format)
            if tuple(rgba.shape) != (rows, w, ch) or rgba.dtype != dt \
                    or not rgba.is_contiguous() or rgba.device != self.device:
                raise ValueError(f"rgba must be a contiguous {dt} ({rows}, {w}, {ch}) tensor "
                                 f"on {self.device}")
        if st is not None and (tuple(st.shape) != (rows, w, 2) or st.dtype != torch.int32
                               or not st.is_contiguous()):
            raise ValueError(f"steps must be a contiguous int32 ({rows}, {w}, 2) tensor")
        with self._on_device():
            args = (C.byref(frame.scene), C.byref(frame.camera), C.byref(frame.light),
                    C.byref(frame.material), C.byref(frame.params),
                    C.byref(t) if t is not None else None,
                    C.c_void_p(rgba.data_ptr()),
                    C.c_void_p(st.data_ptr()) if st is not None else None)
            if schedule is None:
                rc = self.lib.sdf_render(*args, self._stream(stream))
            else:
                rc = self.lib.sdf_render_scheduled(*args, schedule.handle, self._stream(stream))
        abi.check(rc, "sdf_render")
        return rgba, st

    def render_multi(self, frame: Frame, devices, shares=(0, 0), out=None, stream=None):
        """One RGBA32F frame rendered across `devices` (device indices of this
        process, this renderer's device first) through sdf_render_multi: the
        root renders its rows in place and decodes the other devices' TILES
        streams through peer-mapped memory.  Returns the (H, W, 4) frame on
        this renderer's device, asynchronous on `stream`."""
        torch = self.torch
        devs = [int(d) for d in devices]
        if not devs or devs[0] != self.device.index:
            raise ValueError("devices[0] must be this renderer's device")
        p = frame.params
        if out is None:
            out = torch.empty((p.height, p.width, 4), dtype=torch.float32, device=self.device)
        if (tuple(out.shape) != (p.height, p.width, 4) or out.dtype != torch.float32
                or not out.is_contiguous() or out.device != self.device):
            raise ValueError("out must be a contiguous float32 (H, W, 4) tensor on the root")
        arr = (C.c_int32 * len(devs))(*devs)
        with self._on_device():
            rc = self.lib.sdf_render_multi(
                C.byref(frame.scene), C.byref(frame.camera), C.byref(frame.light),
                C.byref(frame.material), C.byref(frame.params), len(devs), arr,
                int(shares[0]), int(shares[1]), C.c_void_p(out.data_ptr()), self._stream(stream))
        abi.check(rc, "sdf_render_multi")
        return out

    def render_frames(self, frame: Frame, cameras, outs, steps=None, stream=None):
        """Whole frames of `frame`'s scene, frame i through cameras[i] into
        outs[i] (and its iteration counts into steps[i]), by the persistent
        frame-sequence kernel (sdf_render_frames): the same pixels as one
        ``render`` per camera.  Asynchronous on `stream`; returns `outs`."""
        torch = self.torch
        n = len(cameras)
        if len(outs) != n or (steps is not None and len(steps) != n):
            raise ValueError("one output (and one steps buffer) per camera")
        p = frame.params
        if p.output_format == abi.FORMAT_TILES:
            raise ValueError("frame sequences take plain formats, not TILES")
        dt, ch = torch_dtype(p.output_format), channels(p.output_format)
        for o in outs:
            if tuple(o.shape) != (p.height, p.width, ch) or o.dtype != dt \
                    or not o.is_contiguous() or o.device != self.device:
                raise ValueError(f"outputs must be contiguous {dt} ({p.height}, {p.width}, {ch}) "
                                 f"tensors on {self.device}")
        for s in steps or ():
            if tuple(s.shape) != (p.height, p.width, 2) or s.dtype != torch.int32 \
                    or not s.is_contiguous() or s.device != self.device:
                raise ValueError("steps must be contiguous int32 (H, W, 2) tensors")
        cams = (abi.sdf_camera * max(n, 1))(*cameras)
        ptrs = (C.c_void_p * max(n, 1))(*[o.data_ptr() for o in outs])
        sptrs = (C.c_void_p * max(n, 1))(*[s.data_ptr() for s in steps]) if steps else None
        with self._on_device():
            rc = self.lib.sdf_render_frames(
                C.byref(frame.scene), cams, n, C.byref(frame.light), C.byref(frame.material),
                C.byref(frame.params), ptrs, sptrs, self._stream(stream))
        abi.check(rc, "sdf_render_frames")
        return outs

    def heatmap(self, steps, which: int = 0, max_steps: int = 128, fmt: int = abi.FORMAT_RGBA8,
                out=None, stream=None):
        """Turbo-coloured view of a `steps` tensor (rows, W, 2) from render()."""
        torch = self.torch
        if steps.dtype != torch.int32 or steps.shape[-1] != 2 or not steps.is_contiguous():
            raise ValueError("steps must be a contiguous int32 (..., 2) tensor")
        count = steps.numel() // 2
        if out is None:
            out = torch.empty((*steps.shape[:-1], channels(fmt)), dtype=torch_dtype(fmt),
                              device=self.device)
        with torch.cuda.device(self.device):
            rc = self.lib.sdf_heatmap(C.c_void_p(steps.data_ptr()), count, which, max_steps,
                                      fmt, C.c_void_p(out.data_ptr()), self._stream(stream))
        abi.check(rc, "sdf_heatmap")
        return out

    def deinterleave(self, parts, nparts: int, part_stride_rows: int, width: int,
                     height: int, block_rows: int = 8, out=None, stream=None,
                     fmt: int | None = None):
        """Scatter gathered packed row blocks (nparts x part_stride_rows rows)
        into a full (height, width, 4) frame on this device."""
        torch = self.torch
        if fmt is None:
            fmt = {torch.float32: abi.FORMAT_RGBA32F, torch.float16: abi.FORMAT_RGBA16F,
                   torch.uint8: abi.FORMAT_RGBA8}[parts.dtype]
            if parts.shape[-1] == 3:
                fmt = abi.FORMAT_RGB32F
        if out is None:
            out = torch.empty((height, width, 4), dtype=torch_dtype(fmt), device=self.device)
        if parts.numel() < nparts * part_stride_rows * width * channels(fmt) \
                or not parts.is_contiguous() or parts.dtype != torch_dtype(fmt) \
                or out.dtype != parts.dtype or tuple(out.shape) != (height, width, 4) \
                or not out.is_contiguous():
            raise ValueError("parts/frame buffers of the wrong size, layout or format")
        with torch.cuda.device(self.device):
            rc = self.lib.sdf_deinterleave(C.c_void_p(parts.data_ptr()), nparts,
                                           part_stride_rows, width, height, block_rows, fmt,
                                           C.c_void_p(out.data_ptr()), self._stream(stream))
        abi.check(rc, "sdf_deinterleave")
        return out

    def tiles_decode(self, parts, nparts: int, part_stride: int, width: int, height: int,
                     block_rows: int = 8, out=None, stream=None, tilings=None):
        """Decode `nparts` TILES streams (uint8, pitch `part_stride` bytes; part
        r from tiling {block_rows, r, nparts}, or from tilings[r] when given)
        into a (height, width, 4) float32 frame on this device
        (sdf_tiles_decode / sdf_tiles_decode_tilings)."""
        torch = self.torch
        if out is None:
            out = torch.empty((height, width, 4), dtype=torch.float32, device=self.device)
        if parts.dtype != torch.uint8 or not parts.is_contiguous() \
                or parts.numel() < nparts * part_stride or out.dtype != torch.float32 \
                or tuple(out.shape) != (height, width, 4) or not out.is_contiguous():
            raise ValueError("TILES parts / RGBA32F frame of the wrong size, layout or type")
        with self._on_device():
            if tilings is None:
                rc = self.lib.sdf_tiles_decode(C.c_void_p(parts.data_ptr()), nparts, part_stride,
                                               width, height, block_rows,
                                               C.c_void_p(out.data_ptr()), self._stream(stream))
            else:
                if len(tilings) != nparts:
                    raise ValueError("one tiling per part")
                arr = (abi.sdf_tiling * nparts)(*tilings)
                rc = self.lib.sdf_tiles_decode_tilings(C.c_void_p(parts.data_ptr()), nparts,
                                                       part_stride, arr, width, height,
                                                       C.c_void_p(out.data_ptr()),
                                                       self._stream(stream))
        abi.check(rc, "sdf_tiles_decode")
        return out

    def tiles_decode_checked(self, parts, nparts: int, part_stride: int, width: int, height: int,
                             tilings, used=None, out=None, status=None, stream=None):
        """sdf_tiles_decode_checked: the decode of tiles_decode(tilings=...)
        for streams that crossed a wire.  `used`: each part's expected data
        bytes (-1: its header's); `status`: a uint32 device tensor of nparts
        words (zeroed here) that receives each part's SDF_TILES_BAD_* bits,
        or None for a synchronous call that raises (SDF_E_COMM) when some
        part was malformed.  Returns (frame, status)."""
        torch = self.torch
        if out is None:
            out = torch.empty((height, width, 4), dtype=torch.float32, device=self.device)
        if parts.dtype != torch.uint8 or not parts.is_contiguous() \
                or parts.numel() < nparts * part_stride or out.dtype != torch.float32 \
                or tuple(out.shape) != (height, width, 4) or not out.is_contiguous() \
                or len(tilings) != nparts:
            raise ValueError("TILES parts / RGBA32F frame of the wrong size, layout or type")
        if status is not None:
            if status.dtype != torch.int32 or status.numel() < nparts or not status.is_contiguous():
                raise ValueError("status: nparts int32 words (holding uint32 codes)")
            status.zero_()
        arr = (abi.sdf_tiling * nparts)(*tilings)
        u = None if used is None else (C.c_int64 * nparts)(*[int(x) for x in used])
        with self._on_device():
            rc = self.lib.sdf_tiles_decode_checked(
                C.c_void_p(parts.data_ptr()), nparts, part_stride, arr, u, width, height,
                C.c_void_p(out.data_ptr()),
                None if status is None else C.c_void_p(status.data_ptr()), self._stream(stream))
        abi.check(rc, "sdf_tiles_decode_checked")
        return out, status


class Schedule:
    """sdf_schedule: the dispatch order of a frame's 8-row blocks, costliest
    first, learnt from the cycles the kernels measured in earlier frames
    (include/sdf_abi.h).  One per stream; ``close()`` frees it."""

    def __init__(self, renderer: "Renderer", rows: int, period: int = 1):
        self.lib = renderer.lib
        self.handle = C.c_void_p()
        with renderer._on_device():
            abi.check(self.lib.sdf_schedule_create(int(rows), int(period), C.byref(self.handle)),
                      "sdf_schedule_create")

    def order(self) -> list[int]:
        """blockIdx.y -> 8-row block ([] until the first cost snapshot landed)."""
        buf = (C.c_int32 * 512)()
        n = self.lib.sdf_schedule_order(self.handle, buf, 512)
        if n < 0:
            abi.check(n, "sdf_schedule_order")
        return list(buf[:n])

    def close(self) -> None:
        if self.handle:
            self.lib.sdf_schedule_destroy(self.handle)
            self.handle = C.c_void_p()

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass
