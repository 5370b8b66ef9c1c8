"""TEST INFRASTRUCTURE (tests/test_gpu_shmcomm.py): sdf_comm_create (the
native driver's communicator creation, sdf3d_amd/csrc/driver.cpp) over the
stand-in tests/shmcomm/libshmcomm.so in its non-blocking mode
(SHMCOMM_NONBLOCKING=1: ncclCommInitRankConfig answers ncclInProgress and
joins on a helper thread), for a 2-rank communicator whose second rank never
joins.  The creation must give up after its limit with SDF_E_TIMEOUT and
abort the half-made communicator (ncclCommAbort), which stops the join.
Prints one JSON line.

    python create_probe.py <timeout_ms>
"""
import ctypes as C
import json
import sys
import time
from pathlib import Path

import torch

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent.parent))
LIB = HERE / "libshmcomm.so"


def main():
    timeout_ms = int(sys.argv[1])
    torch.cuda.set_device(0)
    from sdf3d_amd import abi
    lib = abi.load_library()
    uid = (C.c_uint8 * abi.COMM_ID_BYTES)()
    assert lib.sdf_comm_unique_id(str(LIB).encode(), uid) == abi.SDF_OK
    h = C.c_void_p()
    t0 = time.perf_counter()
    rc = lib.sdf_comm_create(str(LIB).encode(), bytes(uid), 2, 0, timeout_ms, C.byref(h))
    el = time.perf_counter() - t0
    shm = C.CDLL(str(LIB))   # the same instance the driver loaded
    shm.shmcomm_counts.restype = C.c_ulonglong
    print(json.dumps({"rc": rc, "seconds": round(el, 3), "handle_null": not h.value,
                      "inprogress_returns": shm.shmcomm_counts(0),
                      "aborts": shm.shmcomm_counts(1)}), flush=True)


if __name__ == "__main__":
    main()
