"""Python handle on the native multi-device frame driver (include/sdf_abi.h
``sdf_comm_*`` / ``sdf_driver_*``, sdf3d_amd/csrc/driver.cpp).

One process per GPU, as launched by torchrun.  torch.distributed is used
once, to hand every rank the RCCL unique ids of the driver's two
communicators (stream lengths; stream data, each on its own HIP stream);
from then on every per-frame call is one ctypes call into the library,
which renders, agrees the TILES stream lengths (RCCL
all-gather), ships the streams to rank 0 (RCCL send/recv) and decodes them
there -- the same sequence as ``multigpu.FrameDriver`` (whose gloo
rehearsal in tests/test_multigpu_cpu.py pins the collective order) at a
fraction of its host cost (tools/driver_probe.py).  The driver loads the
RCCL library this process already has mapped (PyTorch's), so one RCCL
instance serves both.
"""
from __future__ import annotations

import ctypes as C
import os

from . import abi
from .scenes import Frame


def loaded_rccl_path() -> str:
    """Path of the librccl this process has mapped (PyTorch loads one with
    its HIP backend), else PyTorch's bundled one, else the system's."""
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                path = line.rsplit(None, 1)[-1] if "/" in line else ""
                if "librccl" in os.path.basename(path):
                    return path
    except OSError:  # pragma: no cover - non-Linux
        pass
    try:
        import torch
        p = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
        if os.path.exists(p):
            return p
    except ImportError:  # pragma: no cover
        pass
    return "librccl.so.1"


class Comm:
    """One RCCL communicator over the torch.distributed world (collective:
    every rank constructs it, in the same order).

    Failure is agreed, never one-sided: rank 0 broadcasts a status byte with
    the id (so a failed sdf_comm_unique_id fails every rank at the same
    collective), sdf_comm_create gives up after `timeout_ms` when a peer never
    joins, and the ranks all-reduce their outcome, so either every rank holds
    the communicator or every rank raises (and bench.py falls back on all of
    them together)."""

    def __init__(self, dist, device, rccl_path: str | None = None, timeout_ms: int = 120000):
        import torch
        self.lib = abi.load_library()
        self.path = (rccl_path or loaded_rccl_path()).encode()
        self.handle = C.c_void_p()
        rank, world = dist.get_rank(), dist.get_world_size()
        msg = torch.zeros(abi.COMM_ID_BYTES + 1, dtype=torch.uint8)   # [ok, id]
        err = None
        if rank == 0:
            buf = (C.c_uint8 * abi.COMM_ID_BYTES)()
            rc = self.lib.sdf_comm_unique_id(self.path, buf)
            if rc == abi.SDF_OK:
                msg[0] = 1
                msg[1:] = torch.frombuffer(bytearray(bytes(buf)), dtype=torch.uint8)
            else:
                err = abi.SdfError(rc, "sdf_comm_unique_id")
        on_dev = dist.get_backend() == "nccl"
        t = msg.to(device) if on_dev else msg
        dist.broadcast(t, src=0)
        msg = t.cpu()
        ok = int(msg[0]) == 1
        if ok:
            raw = bytes(msg[1:].numpy().tobytes())
            with torch.cuda.device(device):
                rc = self.lib.sdf_comm_create(self.path, raw, world, rank, int(timeout_ms),
                                              C.byref(self.handle))
            if rc != abi.SDF_OK:
                ok, err = False, abi.SdfError(rc, "sdf_comm_create")
        elif err is None:
            err = abi.SdfError(abi.SDF_E_COMM, "rank 0 could not make a communicator id")
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32)
        flag = flag.to(device) if on_dev else flag
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        if int(flag.item()) != 1:
            self.close()
            raise err or abi.SdfError(abi.SDF_E_COMM, "a peer could not join the communicator")

    def close(self):
        if self.handle:
            self.lib.sdf_comm_destroy(self.handle)
            self.handle = C.c_void_p()


class NativeFrameDriver:
    """The frame loop in C++ (sdf_driver_*).  ``step()`` enqueues one frame;
    ``drain()`` ships everything and waits; ``read_frame(i, out)`` copies
    rank 0's frame i (one of the last ``nbuf``) into a torch tensor.
    ``batch``: frames per ship (one length all-gather and one send/recv group
    per batch; nbuf % batch == 0, lag <= nbuf - batch)."""

    def __init__(self, frame: Frame, rank: int, world: int, device, shares=(1, 1), nbuf: int = 4,
                 lag: int = 2, dist=None, root_as_peer: bool = False, timeout_ms: int = 60000,
                 rccl_path: str | None = None, batch: int = 1):
        import torch
        self.torch = torch
        self.lib = abi.load_library()
        self.device = torch.device(device)
        self.frame_desc = frame
        self.rank, self.world, self.nbuf = rank, world, nbuf
        self.comms = []
        cfg = abi.sdf_driver_config(rank=rank, world=world, share_root=shares[0],
                                    share_peer=shares[1], nbuf=nbuf, lag=lag,
                                    flags=abi.DRIVER_ROOT_AS_PEER if root_as_peer else 0,
                                    timeout_ms=timeout_ms, batch=batch)
        if world > 1 or root_as_peer:
            if dist is None:
                raise ValueError("a multi-rank driver needs torch.distributed for its comm ids")
            try:
                for _ in range(2):
                    self.comms.append(Comm(dist, self.device, rccl_path))
            except Exception:
                self._close_comms()
                raise
        self.handle = C.c_void_p()
        with torch.cuda.device(self.device):
            rc = self.lib.sdf_driver_create(
                C.byref(frame.scene), C.byref(frame.camera), C.byref(frame.light),
                C.byref(frame.material), C.byref(frame.params), C.byref(cfg),
                *([c.handle for c in self.comms] or [None, None]), C.byref(self.handle))
        if rc != abi.SDF_OK:
            self._close_comms()
            abi.check(rc, "sdf_driver_create")
        self._idx = C.c_int64()

    def step(self) -> int:
        rc = self.lib.sdf_driver_step(self.handle, C.byref(self._idx))
        if rc != abi.SDF_OK:
            abi.check(rc, "sdf_driver_step")
        return self._idx.value

    def set_camera(self, camera) -> None:
        abi.check(self.lib.sdf_driver_set_camera(self.handle, C.byref(camera)),
                  "sdf_driver_set_camera")

    def drain(self) -> None:
        abi.check(self.lib.sdf_driver_drain(self.handle), "sdf_driver_drain")

    def read_frame(self, index: int, out=None, stream=None):
        """Rank 0's frame `index` as a (H, W, 4) tensor of the frame format."""
        from .renderer import channels, torch_dtype
        torch = self.torch
        p = self.frame_desc.params
        if out is None:
            out = torch.empty((p.height, p.width, channels(p.output_format)),
                              dtype=torch_dtype(p.output_format), device=self.device)
        s = stream or torch.cuda.current_stream(self.device)
        abi.check(self.lib.sdf_driver_read_frame(
            self.handle, index, C.c_void_p(out.data_ptr()),
            out.numel() * out.element_size(), C.c_void_p(s.cuda_stream)), "sdf_driver_read_frame")
        return out

    def stats(self) -> dict:
        """Host time of the driver's calls: frames, seconds in step/drain, and
        the seconds of that spent waiting on the GPU or a peer."""
        out = (C.c_double * 7)()
        abi.check(self.lib.sdf_driver_stats(self.handle, out, 7), "sdf_driver_stats")
        n = max(out[0], 1.0)
        us = lambda x: round(x / n * 1e6, 2)  # noqa: E731
        return {"frames": int(out[0]), "call_s": out[1], "wait_s": out[2],
                "host_us_per_frame": us(out[1] - out[2]),
                "enqueue_us_per_frame": {"render": us(out[3]), "lengths": us(out[4]),
                                         "transfer_group": us(out[5]), "decode": us(out[6])}}

    def close(self) -> None:
        if self.handle:
            rc = self.lib.sdf_driver_destroy(self.handle)
            self.handle = C.c_void_p()
            self._close_comms()
            abi.check(rc, "sdf_driver_destroy")

    def _close_comms(self) -> None:
        for c in self.comms:
            c.close()
        self.comms = []

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass
