"""TEST INFRASTRUCTURE (tests/test_gpu_shmcomm.py): one rank of a 2-rank
run of the asynchronous stand-in (tests/shmcomm/libshmcomm.so) driven
through its RCCL symbols with ctypes.

    python order_probe.py <rank> <id_dir> <mode>

mode "same": both ranks issue all-gathers on communicators A then B, three
times; the results must be right and the calls must return before the GPU
has run them (a 0.4 s busy kernel sits on the stream first).
mode "crossed": rank 1 issues B then A -- a cross-communicator order the
stand-in's single FIFO engine cannot serve: the communicators must report
an asynchronous error within SHMCOMM_TIMEOUT_MS and the stream must still
drain (no GPU stream left waiting).  Prints one JSON line."""
import ctypes as C
import json
import os
import sys
import time
from pathlib import Path

import torch

LIB = Path(__file__).resolve().parent / "libshmcomm.so"


class UniqueId(C.Structure):
    _fields_ = [("internal", C.c_char * 128)]


def main():
    rank, id_dir, mode = int(sys.argv[1]), Path(sys.argv[2]), sys.argv[3]
    torch.cuda.set_device(0)
    lib = C.CDLL(str(LIB))
    comms = []
    for name in ("A", "B"):
        uid = UniqueId()
        f = id_dir / f"{name}.id"
        if rank == 0:
            assert lib.ncclGetUniqueId(C.byref(uid)) == 0
            tmp = f.with_suffix(".tmp")
            tmp.write_bytes(bytes(uid.internal).ljust(128, b"\0"))
            os.replace(tmp, f)
        else:
            while not f.exists():
                time.sleep(0.01)
            uid.internal = f.read_bytes()[:128].rstrip(b"\0")
        comm = C.c_void_p()
        assert lib.ncclCommInitRank(C.byref(comm), 2, uid, rank) == 0
        comms.append(comm)
    s = torch.cuda.Stream()
    ncclInt32 = 2
    out = {"rank": rank, "mode": mode}
    send = torch.full((4,), 10 * rank + 1, dtype=torch.int32, device="cuda")
    recvs = [torch.zeros(8, dtype=torch.int32, device="cuda") for _ in range(6)]
    order = [0, 1] if (mode == "same" or rank == 0) else [1, 0]
    with torch.cuda.stream(s):
        torch.cuda._sleep(int(1.0e9))              # ~0.4-0.7 s of GPU work first
        t0 = time.perf_counter()
        rcs = []
        for rep in range(3):
            for k in order:
                rcs.append(lib.ncclAllGather(C.c_void_p(send.data_ptr()),
                                             C.c_void_p(recvs[2 * rep + k].data_ptr()), 4,
                                             ncclInt32, comms[k], C.c_void_p(s.cuda_stream)))
        out["issue_s"] = round(time.perf_counter() - t0, 4)
    out["async_engine"] = int(lib.shmcomm_async_engine())
    out["rcs"] = rcs
    t0 = time.perf_counter()
    s.synchronize()
    out["drain_s"] = round(time.perf_counter() - t0, 3)
    errs = []
    for comm in comms:
        e = C.c_int(0)
        lib.ncclCommGetAsyncError(comm, C.byref(e))
        errs.append(e.value)
    out["async_errors"] = errs
    if mode == "same":
        want = [1] * 4 + [11] * 4
        out["correct"] = all(r.cpu().tolist() == want for r in recvs)
    for comm in comms:
        lib.ncclCommDestroy(comm)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
