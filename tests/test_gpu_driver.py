"""The native frame driver (sdf_driver_*, sdf3d_amd/csrc/driver.cpp) on one
GPU: its frames must equal a one-device sdf_render bit for bit.

  - world 1, no communicator: whole frames on alternating streams;
  - world 1 with ROOT_AS_PEER over a one-rank RCCL process group: every
    frame goes the multi-rank way (TILES stream, RCCL all-gather of its
    length, RCCL send/recv to rank 0 = itself, decode into the frame).
RCCL refuses two ranks on one GPU, so the multi-rank collective order is
pinned by the gloo rehearsal of the same sequence (test_multigpu_cpu.py)."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _free_port():
    from netutil import free_port
    return free_port()


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


ROOT = __import__("pathlib").Path(__file__).resolve().parent.parent
SHMCOMM = ROOT / "tests" / "shmcomm" / "libshmcomm.so"


def test_frame_not_shipped_is_refused(nccl_world1):
    """a frame whose peers' rows have not been shipped yet (the
    last `lag` frames stepped, before sdf_driver_drain) is refused, not
    handed out half-assembled."""
    from sdf3d_amd import abi, scenes
    from sdf3d_amd.driver import NativeFrameDriver
    f = scenes.config("C3", 96, 64, precision=abi.PRECISION_FAST)
    drv = NativeFrameDriver(f, 0, 1, "cuda:0", nbuf=4, lag=2, dist=nccl_world1,
                            root_as_peer=True)
    idx = [drv.step() for _ in range(3)]
    with pytest.raises(abi.SdfError):
        drv.read_frame(idx[-1])          # not shipped yet (lag 2)
    drv.read_frame(idx[0])               # shipped at step 2
    drv.drain()
    got = drv.read_frame(idx[-1])
    torch.cuda.synchronize()
    drv.close()
    assert torch.equal(got.view(torch.int32), _reference(f).view(torch.int32))


@pytest.mark.parametrize("nproc,cfg,shares,batch,streams,nonblocking,lag", [
    (2, "C3", None, 2, 4, True, 0), (3, "C3", "1:2", 1, 4, False, 0),
    (3, "C3", None, 4, 8, True, 0), (8, "C3", None, 4, 8, False, 0),
    (8, "C4", None, 0, 0, False, 0),
    # 16 buffer sets on the driver's 4 render streams, batches of
    # 8 shipped 8 frames late -- buffer sets share streams, and their waits
    # must not form a cycle across ranks
    (3, "C3", None, 8, 16, False, 8), (2, "C5", None, 8, 16, True, 8),
    # the Mandelbulb at world 8 (4K, default shares)
    (8, "C5", None, 0, 0, False, 0)])
def test_native_driver_multirank(tmp_path, nproc, cfg, shares, batch, streams, nonblocking, lag):
    """The native C++ driver's multi-rank sequence (render, RCCL-style length
    all-gather, send/recv of the TILES streams to rank 0, decode) with
    `nproc` ranks sharing this GPU: bench.py --driver native over the
    stand-in communications library tests/shmcomm (RCCL refuses two ranks on
    one GPU), in its asynchronous mode (required): calls return once
    enqueued and hold only their own stream, on the GPU, until the data is in
    place, and one FIFO engine per rank makes any cross-communicator order
    mismatch between ranks an error.  Rank 0's assembled last frame must equal a single-device
    render bit for bit; the 8-rank C4 case is the round-end N = 8 bench's
    configuration (4K, default 1:7 shares, batches of 2 frames).  Frames
    are shipped in batches (1, 2, 4: one length all-gather and one send/recv
    group per batch; the warm-up's drain closes a short batch, so the next
    batch starts on a new buffer set).  `nonblocking`: the stand-in answers
    ncclInProgress for creation, all-gathers and groups (as RCCL's
    non-blocking communicators may) and enqueues them later, so work the
    driver recorded behind an unsettled call would run before it."""
    import json
    import sys
    assert SHMCOMM.exists(), "build() must produce tests/shmcomm/libshmcomm.so"
    from netutil import run_launcher

    def cmd(port):
        c = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node",
             str(nproc), "--master-addr", "127.0.0.1", "--master-port", str(port), "--tee", "2",
             str(ROOT / "bench.py"), "--gpus", str(nproc), "--steps", "6", "--warmup", "2",
             "--backend", "gloo", "--comm-lib", str(SHMCOMM), "--driver", "native",
             "--config", cfg, "--no-display", "--clock-warm-s", "0"]
        c += ["--batch", str(batch)] if batch else []
        c += ["--streams", str(streams)] if streams else []
        c += ["--lag", str(lag), "--steps", "20"] if lag else []
        return c + (["--shares", shares] if shares else [])
    env = dict(os.environ, SHMCOMM_TIMEOUT_MS="60000", GPU_MAX_HW_QUEUES="8",
               SHMCOMM_REQUIRE_ASYNC="1", SHMCOMM_STATS="1")
    if nonblocking:
        env["SHMCOMM_NONBLOCKING"] = "1"
    r = run_launcher(cmd, timeout=400, cwd=ROOT, env=env)
    if r.returncode != 0:   # the ranks' own error lines first (torchrun's summary is long)
        import re
        bad = [l for l in (r.stderr or "").splitlines()
               if re.search(r"terminate|what\(\)|Error|error|Assert|abort|SIG", l)
               and "error_file" not in l]
        raise AssertionError("\n".join(bad[:60]) + "\n----\n" + r.stderr[-3000:])
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert d["n_gpus"] == nproc and d["frame_verified"] is True, d
    assert d["config"]["driver"].startswith("native"), d["config"]
    assert d["config"]["wire"] == "tiles"
    assert d["config"]["batch"] == (batch or 2), d["config"]
    if nproc == 8:
        assert d["config"]["tiling"].startswith("8-row blocks, rank 0 1 / others 7")
    import re
    counts = [int(m) for m in re.findall(r"shmcomm: inprogress_returns=(\d+)", r.stderr)]
    assert len(counts) >= nproc, r.stderr[-2000:]
    if nonblocking:   # every rank's creations, all-gathers and groups answered "in progress"
        assert min(counts) > 2, counts
    else:
        assert max(counts) == 0, counts


def _read_ppm(path):
    import numpy as np
    data = open(path, "rb").read()
    parts = data.split(b"\n", 3)
    w, h = map(int, parts[1].split())
    return np.frombuffer(parts[3], dtype=np.uint8).reshape(h, w, 3)


@pytest.mark.parametrize("world", [2, 3])
def test_cpp_driver_multirank_arcball(tmp_path, world):
    """examples/sdf_main.cpp as `world` processes on this GPU (RANK /
    WORLD_SIZE set, ids exchanged through files, stand-in communications
    library), camera from sdf::Arcball's scripted navigation (SDF3D_NAV):
    rank 0's last frame equals the Python path's render of the same V_mat
    (sdf3d_amd.camera.Arcball) to 1 LSB of the 8-bit image, and that render
    passes the oracle parity policy."""
    import subprocess
    import sys

    import numpy as np
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle
    from parity import assert_parity, compare, quantize
    from sdf3d_amd import Renderer, abi, scenes
    from test_camera import nav_views
    exe = ROOT / "sdf3d_amd" / "bin" / "sdf_main"
    frames, W, H = 40, 160, 96
    out = tmp_path / "f.ppm"
    procs = []
    port = str(_free_port())     # the launch tag of the id files (sdf3d.hpp exchange_id)
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK="0",
                   SDF3D_RCCL=str(SHMCOMM), SDF3D_ID_DIR=str(tmp_path),
                   SDF3D_RUN_ID=f"t{os.getpid()}_{world}", SDF3D_NAV="arcball",
                   SHMCOMM_TIMEOUT_MS="60000", GPU_MAX_HW_QUEUES="8",
                   SHMCOMM_REQUIRE_ASYNC="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([str(exe), str(W), str(H), str(frames), str(out), "csg8"],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                      text=True))
    outs = [p.communicate(timeout=300) for p in procs]
    for p, (so, se) in zip(procs, outs):
        assert p.returncode == 0, se[-2000:]
    assert f"rank 0 of {world}" in outs[0][0]
    img = _read_ppm(out)
    f = scenes.config("C3", W, H, precision=abi.PRECISION_EXACT)   # sdf_main's default
    scenes.set_view(f, nav_views(frames)[-1])
    rd = Renderer("cuda:0")
    rgba, st = rd.render(f, steps=True)
    torch.cuda.synchronize()
    rgba, st = rgba.cpu().numpy(), st.cpu().numpy()
    want = quantize(rgba, abi.FORMAT_RGBA8)[::-1, :, :3]
    assert np.abs(img.astype(int) - want.astype(int)).max() <= 1
    ref, rst = oracle.render(f)
    assert_parity(compare(f, rgba, st, ref, rst), what="arcball")


def test_native_driver_refuses_malformed_stream():
    """a receive whose content no longer matches its header
    (the stand-in overwrites frame 2's offset table) makes rank 0's decode
    skip the bad tiles and the driver fail with SDF_E_COMM -- no fault, the
    frame before it and frame 2's other tiles intact."""
    import json
    import subprocess
    import sys
    from netutil import free_port
    from sdf3d_amd import abi
    # SDF3D_DRIVER_DEBUG=2: the probe reads the failed driver's frames (a
    # failed driver refuses them otherwise, test_failed_driver_refuses_frames)
    env = dict(os.environ, SHMCOMM_CORRUPT_RECV="3", SHMCOMM_TIMEOUT_MS="20000",
               GPU_MAX_HW_QUEUES="8", SDF3D_DRIVER_DEBUG="2")
    r = subprocess.run([sys.executable, str(ROOT / "tests" / "driver_fault_probe.py"),
                        str(free_port())], capture_output=True, text=True, timeout=180,
                       cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert d["error"] == abi.SDF_E_COMM, d
    assert d["frame1_exact"] and d["frame2_exact_outside"], d


def test_failed_driver_refuses_frames():
    """once a malformed stream has failed the driver, its frames
    are refused with the driver's error (the bad tiles hold older pixels)."""
    import json
    import subprocess
    import sys
    from netutil import free_port
    from sdf3d_amd import abi
    env = dict(os.environ, SHMCOMM_CORRUPT_RECV="3", SHMCOMM_TIMEOUT_MS="20000",
               GPU_MAX_HW_QUEUES="8", SDF3D_DRIVER_DEBUG="0")
    r = subprocess.run([sys.executable, str(ROOT / "tests" / "driver_fault_probe.py"),
                        str(free_port())], capture_output=True, text=True, timeout=180,
                       cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert d["error"] == abi.SDF_E_COMM, d
    assert d["read_error"] == abi.SDF_E_COMM, d


def test_reused_buffer_set_refuses_its_old_frame(nccl_world1):
    """after a drain closes a short batch the next batch
    starts on a new buffer set, so later frames reuse buffer sets out of
    index order; a frame whose buffer set now holds a newer frame must be
    refused (sdf_driver_frame's owner check), not handed out with another
    frame's pixels.  nbuf 8, batches of 4: frames 0-1, drain, frames 2-7 land
    in sets 4-7 and 0-1, so frame 0's set holds frame 6."""
    from sdf3d_amd import abi, scenes
    from sdf3d_amd.driver import NativeFrameDriver
    f = scenes.config("C3", 96, 64, precision=abi.PRECISION_FAST)
    drv = NativeFrameDriver(f, 0, 1, "cuda:0", nbuf=8, lag=2, dist=nccl_world1,
                            root_as_peer=True, batch=4)
    first = [drv.step() for _ in range(2)]
    drv.drain()
    later = [drv.step() for _ in range(6)]
    drv.drain()
    with pytest.raises(abi.SdfError):
        drv.read_frame(first[0])         # its buffer set now holds a later frame
    got = drv.read_frame(later[-1])
    torch.cuda.synchronize()
    drv.close()
    assert torch.equal(got.view(torch.int32), _reference(f).view(torch.int32))
