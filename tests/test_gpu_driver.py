"""The native frame driver (sdf_driver_*, sdf3d_amd/csrc/driver.cpp) on one
GPU: its frames must equal a one-device sdf_render bit for bit.

  - world 1, no communicator: whole frames on alternating streams;
  - world 1 with ROOT_AS_PEER over a one-rank RCCL process group: every
    frame goes the multi-rank way (TILES stream, RCCL all-gather of its
    length, RCCL send/recv to rank 0 = itself, decode into the frame).
RCCL refuses two ranks on one GPU, so the multi-rank collective order is
pinned by the gloo rehearsal of the same sequence (test_multigpu_cpu.py)."""
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def nccl_world1():
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    yield dist
    dist.destroy_process_group()


def _reference(frame):
    from sdf3d_amd import Renderer
    rd = Renderer("cuda:0")
    ref, _ = rd.render(frame)
    torch.cuda.synchronize()
    return ref


@pytest.mark.parametrize("cfg,W,H,pose", [("C3", 200, 120, 1), ("C2", 96, 64, 2),
                                          ("C5", 64, 40, 0), ("C4", 3840, 2160, 0)])
def test_native_local_frames(cfg, W, H, pose):
    from sdf3d_amd import abi, scenes
    from sdf3d_amd.driver import NativeFrameDriver
    f = scenes.config(cfg, W, H, precision=abi.PRECISION_FAST, pose=pose)
    drv = NativeFrameDriver(f, 0, 1, "cuda:0", nbuf=3, lag=1)
    for _ in range(5):
        last = drv.step()
    drv.drain()
    got = drv.read_frame(last)
    torch.cuda.synchronize()
    drv.close()
    assert torch.equal(got.view(torch.int32), _reference(f).view(torch.int32))


@pytest.mark.parametrize("cfg,W,H,lag,nbuf", [("C3", 200, 120, 2, 4), ("C3", 77, 45, 1, 2),
                                              ("C5", 160, 90, 3, 4), ("C4", 3840, 2160, 2, 4)])
def test_native_root_as_peer(nccl_world1, cfg, W, H, lag, nbuf):
    from sdf3d_amd import abi, scenes
    from sdf3d_amd.driver import NativeFrameDriver
    f = scenes.config(cfg, W, H, precision=abi.PRECISION_FAST)
    drv = NativeFrameDriver(f, 0, 1, "cuda:0", nbuf=nbuf, lag=lag, dist=nccl_world1,
                            root_as_peer=True, timeout_ms=20000)
    idx = [drv.step() for _ in range(2 * nbuf + 1)]
    drv.drain()
    ref = _reference(f)
    for i in idx[-nbuf:]:
        got = drv.read_frame(i)
        torch.cuda.synchronize()
        assert torch.equal(got.view(torch.int32), ref.view(torch.int32)), i
    drv.close()


def test_native_camera_change(nccl_world1):
    """Frames after set_camera use the new camera (and only those)."""
    from sdf3d_amd import abi, scenes
    from sdf3d_amd.driver import NativeFrameDriver
    f0 = scenes.config("C3", 128, 72, precision=abi.PRECISION_FAST, pose=0)
    f1 = scenes.config("C3", 128, 72, precision=abi.PRECISION_FAST, pose=2)
    drv = NativeFrameDriver(f0, 0, 1, "cuda:0", nbuf=4, lag=2, dist=nccl_world1,
                            root_as_peer=True)
    a = drv.step()
    drv.set_camera(f1.camera)
    b = drv.step()
    drv.drain()
    ga, gb = drv.read_frame(a), drv.read_frame(b)
    torch.cuda.synchronize()
    drv.close()
    assert torch.equal(ga.view(torch.int32), _reference(f0).view(torch.int32))
    assert torch.equal(gb.view(torch.int32), _reference(f1).view(torch.int32))


def test_native_bad_config():
    from sdf3d_amd import abi, scenes
    from sdf3d_amd.driver import NativeFrameDriver
    f = scenes.config("C3", 64, 64, precision=abi.PRECISION_FAST)
    with pytest.raises(abi.SdfError):
        NativeFrameDriver(f, 0, 1, "cuda:0", nbuf=3, lag=3)       # lag > nbuf - 1
    ft = f.copy()
    ft.params.output_format = abi.FORMAT_TILES
    with pytest.raises(abi.SdfError):
        NativeFrameDriver(ft, 0, 1, "cuda:0", nbuf=3, lag=1)      # TILES is a wire, not a frame
