"""The exact kernel's correctly rounded building blocks (sdf3d_amd/csrc/
cr_math.h), checked EXHAUSTIVELY on the GPU by tests/crmath/crmath_check.hip:

  * cr_sqrt(x) is bit-identical to IEEE sqrtf(x) for all 2^32 inputs (the
    oracle's sqrtf; voxel_fragment.frag's length() / sqrt);
  * rcp_fast(x) is bit-identical to IEEE 1.0f / x on its domain [2^-100,
    2^100) (the Mandelbulb's 1 / sqrt(k3), k3 in [1e-30, 4]);
  * cr_log(x) is bit-identical to (float)log((double)x) -- the oracle's
    cr_logf (oracle/sdf_oracle.c), the Mandelbulb DE's log -- for all 2^32
    inputs;
  * the smooth-min's h = n / k by div_scaled and (round 6) the whole
    max(k - |e|, 0) / k by smin_h: its bits equal IEEE n / k, or (only where
    h < 2^-77) h*h*k/4 does, over 2^32 SAMPLED (k, n) pairs with
    k log-uniform over every positive exponent and n over [0, k], and over
    2^32 more from its edge families (denormal k, k near FLT_MAX, n * sc
    underflowing, tiny normal k) -- its proof is Markstein's theorem;
  * shade.h spec_pow (exact precision's x^n by repeated squaring in fp64) is
    bit-identical to the library (float)pow((double)x, n) for every float x
    in [0, 1.0001] and every integer n in [0, 64].

With those, the exact-precision kernel stays bit-exact with the oracle
(test_gpu_parity.py's full-size exact cases)."""
import json
import subprocess
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
EXE = Path(__file__).resolve().parent / "crmath" / "crmath_check"


@pytest.fixture(scope="module")
def results():
    assert EXE.exists(), "build() must produce tests/crmath/crmath_check"
    r = subprocess.run([str(EXE)], capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr
    d = json.loads(r.stdout.strip().splitlines()[-1])
    out = Path("gpurun_out")
    out.mkdir(exist_ok=True)
    (out / "crmath_check.json").write_text(json.dumps(d, indent=1))
    print(json.dumps(d))
    return d


def test_cr_sqrt_is_ieee_sqrt_everywhere(results):
    r = results["sqrt"]
    assert r["inputs"] == 2**32 and r["mismatch"] == 0, r
    # the fast path covers [2^-100, 2^100): 200 binades of 2^23 floats
    assert r["fast_path"] == 200 * 2**23, r


def test_cr_sqrt_one_compare_guard_is_ieee_on_every_finite_input(results):
    """SDF_CRM_SQRT_GUARD 1 (the CSG units): guard x >= 2^-100 only; the one
    input it gets wrong is +INF, which the working range keeps away."""
    r = results["sqrtbounded"]
    assert r["inputs"] == 2**32 and r["mismatch"] == 1 and r["effective"] == 0, r
    assert r["first"] == [0x7F800000], r
    # [2^-100, +INF]: 228 binades and +INF itself
    assert r["fast_path"] == 228 * 2**23 + 1, r


def test_sqrt_fast_path_exact_on_every_normal_from_2_pow_minus_100(results):
    """The unguarded fast path on EVERY positive normal float: no mismatch
    from 2^-100 up to FLT_MAX (what the one-compare guard admits); below
    2^-100 ("effective") it fails, and both guards keep it out."""
    r = results["sqrtwide"]
    assert r["fast_path"] == 254 * 2**23, r
    assert r["mismatch"] == r["effective"] > 0, r


def test_rcp_fast_is_ieee_reciprocal_on_its_domain(results):
    r = results["rcp"]
    assert r["fast_path"] == 200 * 2**23 and r["mismatch"] == 0, r


def test_cr_log_is_the_oracles_log_everywhere(results):
    r = results["log"]
    assert r["inputs"] == 2**32 and r["mismatch"] == 0, r
    # almost every positive normal float takes the fast path
    assert r["fast_path"] > 0.999 * 254 * 2**23, r


def test_smooth_min_division_is_bit_identical_where_it_counts(results):
    r = results["smin"]
    assert r["effective"] == 0, r


def test_smooth_min_division_edge_families(results):
    r = results["sminedge"]
    assert r["inputs"] == 2**32 and r["effective"] == 0, r


def test_smooth_min_h_by_one_clamped_fma(results):
    """cr_math.h smin_h (round 6): max(k - |e|, 0) / k with the subtraction,
    the max and the scaling in one clamped FMA -- h*h*k/4 bit-identical to
    the IEEE form on 2^32 sampled (k, e) pairs and 2^32 from edge families."""
    for name in ("sminh", "sminhedge"):
        r = results[name]
        assert r["inputs"] == 2**32 and r["effective"] == 0, (name, r)


def test_integer_pow_is_the_library_pow(results):
    r = results["pow"]
    assert r["inputs"] == 0x3F800347 and r["mismatch"] == 0, r


def test_hardware_min_max_equal_the_select_where_used(results):
    """render_kernel.inc hw_min / hw_max (exact precision) replace the GLSL
    select only where the operands make them equal; the signed-zero and NaN
    pairs those proofs rest on are checked on the hardware."""
    r = results["minmax"]
    assert r["mismatch"] == 0 and r["fast_path"] == 22, r


def test_rcp_fast_negative_half(results):
    r = results["rcpneg"]
    assert r["fast_path"] == 200 * 2**23 and r["mismatch"] == 0, r


def test_markstein_divisions_are_ieee(results):
    """normalize / the Mandelbulb's divisions / the shadow march's division
    by one reciprocal and one Markstein step (cr_math.h div_one,
    div_refined; round 6, proof in cr_math.h and tests/test_crmath_host.py):
    bit-identical to IEEE a / b on 2^32 sampled pairs, inside the guard by
    the step itself ("effective" 0), everywhere with the guard's fall-back
    ("mismatch" 0)."""
    r = results["div"]
    assert r["inputs"] == 2**32 and r["mismatch"] == 0 and r["effective"] == 0, r
    assert r["fast_path"] > 0.7 * 2**32, r
