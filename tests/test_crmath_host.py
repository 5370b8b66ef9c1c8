"""The exhaustive part of the one-step Markstein division proof
(sdf3d_amd/csrc/cr_math.h div_refined / div_prepared), run on the host CPU:
the divisor mantissas the proof's margin argument does not cover (with a
margin: the 64 largest) against every numerator mantissa, plus a random
sample of general normal pairs (tests/crmath/markstein_window.c).  IEEE
binary32 arithmetic with round-to-nearest-even is the same on the host and on
gfx950 (v_mul_f32 / v_fma_f32 / the division it replaces), so the host run
checks the kernel's operation sequence."""
import json
import shutil
import subprocess
from pathlib import Path

import pytest

HERE = Path(__file__).resolve().parent


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_markstein_one_step_window(tmp_path):
    exe = tmp_path / "markstein_window"
    subprocess.run(["gcc", "-O2", "-o", str(exe), str(HERE / "crmath" / "markstein_window.c"),
                    "-lm"], check=True)
    r = subprocess.run([str(exe), "64", "20000000"], capture_output=True, text=True, timeout=600)
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert r.returncode == 0, (out, r.stderr[-500:])
    assert out["window_checked"] == 64 * 2 * (1 << 23)
    assert out["window_bad"] == 0 and out["sample_bad"] == 0
