"""Multi-rank path on the CPU: the FrameDriver used by bench.py, run with
the gloo backend (world size 2 and 3) and a CPU stand-in for the render
kernel (the oracle) and for sdf_deinterleave.  Rank 0's assembled frames
must equal whole-frame renders bit for bit (pixels are independent)."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
import tiles_ref
from sdf3d_amd import renderer as R, scenes
from sdf3d_amd.multigpu import (FrameDriver, deinterleave_index, deinterleave_torch,
                                owned_row_ids, owned_rows_py)


def free_port():
    from netutil import free_port as pick
    return pick()


def frame_for(step):
    return scenes.config("C3", 72, 43, pose=step % 4)


def tiles_decode_cpu(parts, world, cap, W, H, B, out, stream=None, shares=(1, 1)):
    """CPU stand-in for sdf_tiles_decode(_tilings): decode every rank's
    stream with the NumPy reference and put its rows in place."""
    p = parts.numpy()
    for r in range(world):
        rows = owned_rows_py(H, r, world, B, shares)
        if rows == 0 or int(np.frombuffer(p[r * cap + 4:r * cap + 8].tobytes(), np.uint32)[0]) == 0:
            continue   # no stream (rank 0 rendered its rows in place)
        part = tiles_ref.decode(p[r * cap:(r + 1) * cap], W, rows)
        out[torch.as_tensor(owned_row_ids(H, r, world, B, shares))] = torch.from_numpy(part)
    return out


def _worker(rank, world, port, q, wire_channels=4, direct=False, shares=(1, 1), lag=2, nbuf=3):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        step_box = [0]
        tiles = wire_channels == "tiles"

        def render_fn(out, stream):
            f = frame_for(step_box[0])
            rgba, _ = oracle.render(f, R.tiling(rank, world, 8, shares=shares), nthreads=1)
            if tiles:
                st = tiles_ref.encode(rgba)
                out[:st.size] = torch.from_numpy(st)
            else:
                out.copy_(torch.from_numpy(rgba[..., :out.shape[-1]].copy()))

        f0 = frame_for(0)
        W, H = f0.params.width, f0.params.height
        def root_fn(frame, stream):
            # rank 0's rows straight into the frame (SDF_TILING_FRAME_ROWS)
            f = frame_for(step_box[0])
            rgba, _ = oracle.render(f, R.tiling(0, world, 8, shares=shares), nthreads=1)
            frame[torch.as_tensor(owned_row_ids(H, 0, world, 8, shares))] = torch.from_numpy(rgba)

        if tiles:
            big = max(owned_rows_py(H, r, world, 8, shares) for r in range(world))
            drv = FrameDriver(W, H, rank, world, torch.device("cpu"), render_fn,
                              tiles_decode_cpu, dist=dist, wire="tiles",
                              wire_bytes=tiles_ref.capacity(W, big),
                              root_render_fn=root_fn if direct else None, shares=shares,
                              lag=lag, nbuf=nbuf)
        else:
            drv = FrameDriver(W, H, rank, world, torch.device("cpu"),
                              render_fn, deinterleave_torch, dist=dist,
                              wire_channels=wire_channels)
        frames = []
        for i in range(6):
            step_box[0] = i
            drv.step(i)
        drv.drain()
        if rank == 0:
            # buffers hold the last nbuf frames
            for i in range(6 - nbuf, 6):
                frames.append((i, drv.frame(i).clone().numpy()))
            q.put(frames)
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,wire,direct,shares,lag,nbuf", [
    (2, 4, False, (1, 1), 2, 3), (3, 4, False, (1, 1), 2, 3), (2, 3, False, (1, 1), 2, 3),
    (2, "tiles", False, (1, 1), 2, 3), (3, "tiles", True, (1, 1), 2, 3),
    (3, "tiles", True, (1, 2), 2, 4), (4, "tiles", False, (2, 3), 2, 3),
    (2, "tiles", True, (1, 1), 1, 3), (3, "tiles", True, (1, 2), 3, 4)])
def test_frame_driver_gloo(world, wire, direct, shares, lag, nbuf):
    """wire = 3: the lossless RGB32F wire format (alpha restored on rank 0);
    "tiles": the compressed TILES streams (NumPy codec standing in for the
    kernels), variable-length, with the per-frame size agreement, shipped
    `lag` steps after the render over `nbuf` buffer sets; shares: unequal
    row shares (rank 0 fewer)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, wire, direct, shares, lag, nbuf))
             for r in range(world)]
    for p in procs:
        p.start()
    frames = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for i, got in frames:
        want, _ = oracle.render(frame_for(i), nthreads=1)
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), i


@pytest.mark.parametrize("H", [1, 43, 600, 2160])
@pytest.mark.parametrize("world,shares", [(2, (1, 2)), (8, (1, 3)), (5, (3, 2))])
def test_share_index_math_matches_c_abi(H, world, shares):
    seen = np.zeros(H, dtype=int)
    for r in range(world):
        n = owned_rows_py(H, r, world, 8, shares)
        assert n == R.owned_rows(H, R.tiling(r, world, 8, shares=shares))
        ids = owned_row_ids(H, r, world, 8, shares)
        assert len(ids) == n
        seen[ids] += 1
    assert (seen == 1).all()


def test_choose_shares():
    from sdf3d_amd.multigpu import FRAME_COSTS_MS, choose_shares
    assert choose_shares(1) == (1, 1)
    a, b = choose_shares(2)
    assert a >= b                           # the one peer's link is the slower leg
    no_wire = dict(FRAME_COSTS_MS, wire=0.0)
    assert choose_shares(2, no_wire) == (1, 1)   # root's decode is cheap next to half a frame
    a, b = choose_shares(8)
    assert a < b                            # rank 0 decodes 7 streams: fewer rows
    # with a free decode the shares balance renders alone
    assert choose_shares(8, {"render": 1.0, "render_tiles": 1.0, "decode": 0.0}) == (1, 1)
    # the measured defaults (tools/root_probe.py, profiles/r03_share_probe_C4.json;
    # N = 8 round 5: r05_root_rccl_probe_exact_C4.json)
    assert [choose_shares(w) for w in (2, 4, 8)] == [(1, 1), (3, 4), (1, 7)]
    # every default tiling covers the frame exactly once
    for w in range(2, 9):
        a, b = choose_shares(w)
        seen = np.zeros(2160, dtype=int)
        for r in range(w):
            seen[owned_row_ids(2160, r, w, shares=(a, b))] += 1
        assert (seen == 1).all()


@pytest.mark.parametrize("H", [1, 8, 43, 600, 2160])
@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_index_math_matches_c_abi(H, world):
    stride = owned_rows_py(H, 0, world)
    seen = np.zeros(H, dtype=int)
    for r in range(world):
        n = owned_rows_py(H, r, world)
        assert n == R.owned_rows(H, R.tiling(r, world, 8))
        ids = owned_row_ids(H, r, world)
        assert len(ids) == n
        seen[ids] += 1
    assert (seen == 1).all()
    idx = deinterleave_index(H, world, stride)
    # row y of the frame comes from its owner's packed position
    for r in range(world):
        ids = owned_row_ids(H, r, world)
        assert np.array_equal(idx[ids], r * stride + np.arange(len(ids)))


def test_lag_bound():
    """A buffer set is reused after nbuf steps: it must have been shipped by then."""
    with pytest.raises(ValueError):
        FrameDriver(16, 16, 0, 1, torch.device("cpu"), None, None, wire="tiles", nbuf=3, lag=3,
                    collectives_at_world1=True, wire_bytes=4096)


@pytest.mark.parametrize("world,shares", [(1, (1, 1)), (2, (4, 3)), (4, (1, 1)), (8, (1, 2)),
                                          (5, (3, 2)), (8, (1, 3)), (4, (3, 4))])
def test_native_driver_tilings_match(world, shares):
    """The native driver's shares (sdf_share_tiling) are the Python driver's."""
    import ctypes as C
    from sdf3d_amd import abi
    lib = abi.load_library()
    for r in range(world):
        t = abi.sdf_tiling()
        assert lib.sdf_share_tiling(r, world, shares[0], shares[1], C.byref(t)) == 0
        want = R.tiling(r, world, 8, shares=shares)
        for H in (43, 2160):
            assert R.owned_rows(H, t) == R.owned_rows(H, want) == owned_rows_py(H, r, world, 8, shares)
        if world > 1:
            assert (t.block_rows, t.first_block, t.block_stride, t.block_run, t.run_step) == \
                (want.block_rows, want.first_block, want.block_stride, want.block_run,
                 want.run_step)
    bad = abi.sdf_tiling()
    assert lib.sdf_share_tiling(world, world, 1, 1, C.byref(bad)) == abi.SDF_E_INVALID_ARG


@pytest.mark.parametrize("world,shares,busiest", [(8, (1, 3), 296), (4, (3, 4), 576),
                                                  (2, (1, 1), 1080)])
def test_share_rows_balanced_on_4k(world, shares, busiest):
    """The peers' interleaved runs (sdf_tiling.run_step) spread a 4K frame's
    last partial period over distinct ranks: at N = 8, 1:3 (270 blocks,
    period 22) no peer owns more than 37 blocks (consecutive runs gave one
    peer 39, 312 rows), and the rows still partition the frame."""
    rows = [R.owned_rows(2160, R.tiling(r, world, 8, shares=shares)) for r in range(world)]
    assert sum(rows) == 2160 and max(rows[1:]) == busiest
    ids = np.concatenate([owned_row_ids(2160, r, world, 8, shares) for r in range(world)])
    assert np.array_equal(np.sort(ids), np.arange(2160))


def _comm_fail_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from sdf3d_amd import abi
        from sdf3d_amd.driver import Comm
        try:
            # rank 0 cannot load the communications library: it must not be
            # the only rank to give up (the others would wait in a collective)
            Comm(dist, "cpu", rccl_path="/nonexistent/librccl.so" if rank == 0 else None)
            q.put((rank, "created"))
        except abi.SdfError as e:
            q.put((rank, f"raised {e.code}"))
        # the ranks are still in step: a later collective completes
        t = torch.ones(1)
        dist.all_reduce(t)
        q.put((rank, f"sum {int(t.item())}"))
    finally:
        dist.destroy_process_group()


def test_comm_failure_is_agreed():
    """sdf3d_amd.driver.Comm fails on every rank together (status
    broadcast with the id), so no rank is left blocked in a collective."""
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_comm_fail_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(120)
        assert p.exitcode == 0
    got = sorted(q.get(timeout=10) for _ in range(2 * world))
    from sdf3d_amd import abi
    for r in range(world):
        assert (r, f"raised {abi.SDF_E_COMM}") in got and (r, f"sum {world}") in got
