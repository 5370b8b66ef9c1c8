"""Rendezvous ports for the multi-process tests (test infrastructure).

A port from bind(0) comes from the kernel's ephemeral range, where any
outgoing connection on the box (another test's store client, another job's
socket) may take it again before the launched ranks listen on it: that is a
rendezvous failure (EADDRINUSE) before any rank has started work.  So ports
are picked at random below the ephemeral range (Linux: 32768-60999) and
checked free, and a launch that fails on exactly that error is started again
once with a new port.
"""
from __future__ import annotations

import random
import socket
import subprocess
import sys
import warnings

_ADDR_IN_USE = ("EADDRINUSE", "address already in use", "Address already in use")


def free_port() -> int:
    rng = random.Random()
    for _ in range(200):
        port = rng.randrange(20000, 32000)
        with socket.socket() as s:
            try:
                s.bind(("127.0.0.1", port))
            except OSError:
                continue
            return port
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_launcher(make_cmd, attempts: int = 2, **kw) -> subprocess.CompletedProcess:
    """subprocess.run(make_cmd(port), capture_output=True, text=True, **kw),
    launched again with a new port when the rendezvous could not listen."""
    r = None
    for attempt in range(attempts):
        port = free_port()
        r = subprocess.run(make_cmd(port), capture_output=True, text=True, **kw)
        if r.returncode == 0 or not any(m in (r.stderr or "") for m in _ADDR_IN_USE):
            return r
        if attempt + 1 < attempts:
            # every re-launch is visible in the test report: a
            # failure whose stderr merely mentions the error text gets a
            # second run, and that must not go unseen
            tail = (r.stderr or "")[-1500:]
            msg = (f"netutil: launch on port {port} failed with rc {r.returncode} and an "
                   f"address-in-use message; launching again. stderr tail:\n{tail}")
            print(msg, file=sys.stderr, flush=True)
            warnings.warn(msg, RuntimeWarning)
    return r
