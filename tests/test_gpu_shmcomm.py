"""The asynchronous stand-in communications library (tests/shmcomm), the
substrate of the native driver's multi-rank tests (test_gpu_driver.py):
its calls return once enqueued, like RCCL's, with the caller's stream held
on the GPU until the data is in place; and its single per-process FIFO
engine turns ranks that issue calls on two communicators in different orders
into a reported error (SHMCOMM_TIMEOUT_MS), never a hang."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
HERE = Path(__file__).resolve().parent
PROBE = HERE / "shmcomm" / "order_probe.py"


def run_pair(tmp_path, mode, timeout_ms):
    # every stream its own hardware queue (tests/shmcomm/shmcomm.cpp)
    env = dict(os.environ, SHMCOMM_TIMEOUT_MS=str(timeout_ms), GPU_MAX_HW_QUEUES="16")
    env.pop("SHMCOMM_SYNC", None)
    procs = [subprocess.Popen([sys.executable, str(PROBE), str(r), str(tmp_path), mode],
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env)
             for r in range(2)]
    outs = [p.communicate(timeout=150) for p in procs]
    for p, (so, se) in zip(procs, outs):
        assert p.returncode == 0, se[-2000:]
    return [json.loads(so.strip().splitlines()[-1]) for so, _ in outs]


def test_calls_are_asynchronous_and_correct(tmp_path):
    for r in run_pair(tmp_path, "same", 30000):
        assert r["correct"] and r["async_errors"] == [0, 0] and r["rcs"] == [0] * 6, r
        # six all-gathers issued behind ~0.4-0.7 s of GPU work return at once
        assert r["async_engine"] == 1, r
        assert r["issue_s"] < 0.2 and r["drain_s"] > 0.2, r


def test_crossed_communicator_order_is_an_error_not_a_hang(tmp_path):
    res = run_pair(tmp_path, "crossed", 3000)
    assert any(e != 0 for r in res for e in r["async_errors"]), res
    for r in res:
        assert r["drain_s"] < 60, r     # the streams were released


def test_nonblocking_creation_timeout_aborts(tmp_path):
    """sdf_comm_create over a non-blocking communicator
    (ncclCommInitRankConfig answers ncclInProgress) whose peer never joins
    gives SDF_E_TIMEOUT after its limit and aborts the half-made
    communicator (no join left running, no handle returned)."""
    env = dict(os.environ, SHMCOMM_NONBLOCKING="1", SHMCOMM_TIMEOUT_MS="60000",
               GPU_MAX_HW_QUEUES="16")
    r = subprocess.run([sys.executable, str(HERE / "shmcomm" / "create_probe.py"), "1500"],
                       capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["rc"] == -6 and d["handle_null"], d            # SDF_E_TIMEOUT
    assert d["inprogress_returns"] >= 1 and d["aborts"] == 1, d
    assert 1.4 < d["seconds"] < 30, d
