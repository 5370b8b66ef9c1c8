"""TEST INFRASTRUCTURE (tests/test_gpu_driver.py): the native frame driver
over the stand-in communications library with one of rank 0's receives
corrupted (SHMCOMM_CORRUPT_RECV, tests/shmcomm/shmcomm.cpp): the decode must
find the stream malformed, the driver fail with SDF_E_COMM, and the frames
and tiles not concerned stay intact.  One JSON line on stdout.

    SHMCOMM_CORRUPT_RECV=3 python tests/driver_fault_probe.py PORT
"""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    import numpy as np
    import torch
    import torch.distributed as dist
    from sdf3d_amd import Renderer, abi, scenes
    from sdf3d_amd.driver import NativeFrameDriver
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=sys.argv[1])
    dist.init_process_group("gloo", rank=0, world_size=1)
    f = scenes.config("C3", 160, 96, precision=abi.PRECISION_FAST, pose=1)
    drv = NativeFrameDriver(f, 0, 1, "cuda:0", nbuf=8, lag=2, dist=dist, root_as_peer=True,
                            timeout_ms=20000, rccl_path=str(ROOT / "tests/shmcomm/libshmcomm.so"))
    err, at, steps = None, None, 0
    try:
        for _ in range(6):
            drv.step()
            steps += 1
        at = "drain"
        drv.drain()
    except abi.SdfError as e:
        err, at = e.code, at or "step"
    rd = Renderer("cuda:0")
    ref, _ = rd.render(f)
    if os.environ.get("SDF3D_DRIVER_DEBUG", "0") < "2":
        # a failed driver refuses its frames (driver.cpp sdf_driver_frame)
        try:
            drv.read_frame(1)
            read_error = 0
        except abi.SdfError as e:
            read_error = e.code
        print(json.dumps({"error": err, "at": at, "steps": steps, "read_error": read_error}),
              flush=True)
        drv.handle and drv.lib.sdf_driver_destroy(drv.handle)
        drv.handle = None
        drv._close_comms()
        dist.destroy_process_group()
        return
    f1 = drv.read_frame(1)            # received intact
    f2 = drv.read_frame(2)            # its table entries 0..15 overwritten
    torch.cuda.synchronize()
    ref, f1, f2 = ref.cpu().numpy(), f1.cpu().numpy(), f2.cpu().numpy()
    tx = (160 + 7) // 8
    bad = np.zeros((96, 160), dtype=bool)
    for t in range(16):
        y, x = divmod(t, tx)
        bad[8 * y:8 * y + 8, 8 * x:8 * x + 8] = True
    same = lambda a, b: bool(np.array_equal(a.view(np.uint32), b.view(np.uint32)))  # noqa: E731
    print(json.dumps({"error": err, "at": at, "steps": steps,
                      "frame1_exact": same(f1, ref),
                      "frame2_exact_outside": same(f2[~bad], ref[~bad])}), flush=True)
    drv.handle and drv.lib.sdf_driver_destroy(drv.handle)
    drv.handle = None
    drv._close_comms()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
