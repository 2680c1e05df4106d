"""The GPU path at the extremes of its two exactness bounds (tests/worstcase.py builds the inputs;
tests/test_worstcase_bounds.py shows on CPU that the same inputs break a basis with one prime fewer):

* the key switch over 31-bit primes: every digit of every product's c2 is -B/2 and the key is
  sign-aligned, so coefficient 0 reaches m G' n (B/2) floor(q/2) -- cfg3 (bfv_mul_and_relin, m = 1),
  cfg4 (dbfv_mul, limb 1 sums m = 2 products: the wide basis), cfg5 (dbfv_mul, limb 7 sums m = 8,
  int8 digits, psum);
* psum: every product's c1 tensor at 2 n floor(Q/2)^2 (cfg4, cfg5).
Each is bit-exact against the C restatement of the reference (oracle/c), computed in-test at cfg3 /
cfg4 and pinned by committed digests at cfg5 (tests/golden/make_golden.py --worst-digests); the
pinned item rides in the bench's production batch (two pipeline lanes).
"""

import hashlib
import json
import os

import numpy as np
import pytest

from oracle import params as P, cref
from exacto_amd._ffi import HipContext
from bridge import uniform_residues
import worstcase as W

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.uint64).tobytes()).hexdigest()


def pad(a, b, to, q, n, seed):
    rng = np.random.default_rng(seed)
    k = a.shape[0]
    if to > k:
        a = np.concatenate([a, uniform_residues(rng, (to - k,) + a.shape[1:-2], q, n)])
        b = np.concatenate([b, uniform_residues(rng, (to - k,) + b.shape[1:-2], q, n)])
    return a, b


def test_worst_case_key_switch_cfg3(gpu_available):
    prm = P.cfg3_params(4096)
    q, n, G = prm.ct_basis.moduli, 4096, prm.gadget_digits
    ct1, ct2, rlk, gp = W.digit_case_bfv(q, prm.plain_modulus, prm.gadget_base, G, n)
    assert gp == G - 1
    want = cref.bfv_mul_and_relin(prm, ct1, ct2, rlk, threads=8)
    ctx = HipContext.from_params(prm)
    assert ctx.ks32_primes == 3
    ctx.load_relin_key(rlk)
    c1, c2 = pad(ct1, ct2, 200, q, n, 1)      # 200 products: two lanes of 100
    got = ctx.bfv_mul_and_relin(c1, c2)
    assert np.array_equal(got[:1], want)
    # the sign-aligned key's L1 norms exceed the lazy basis' bound: the narrow basis runs it
    assert not ctx.ks32_lazy


def test_worst_case_digits_lazy_basis_cfg3(gpu_available):
    """The same extreme digits (every one -B/2) with a uniform key: its norms (~n q / 4 per row) fit
    the lazy basis (primes below 2^30), which then runs the key switch at its digit bound."""
    prm = P.cfg3_params(4096)
    q, n, G = prm.ct_basis.moduli, 4096, prm.gadget_digits
    ct1, ct2, _, _ = W.digit_case_bfv(q, prm.plain_modulus, prm.gadget_base, G, n)
    rlk = uniform_residues(np.random.default_rng(30), (G, 2), q, n)
    want = cref.bfv_mul_and_relin(prm, ct1, ct2, rlk, threads=8)
    ctx = HipContext.from_params(prm)
    ctx.load_relin_key(rlk)
    c1, c2 = pad(ct1, ct2, 200, q, n, 3)
    got = ctx.bfv_mul_and_relin(c1, c2)
    assert ctx.ks32_lazy
    assert np.array_equal(got[:1], want)
    assert np.array_equal(got[1:3], cref.bfv_mul_and_relin(prm, c1[1:3], c2[1:3], rlk, threads=8))


@pytest.mark.parametrize("kind", ["digits", "tensor"])
def test_worst_case_dbfv_cfg4(gpu_available, kind):
    dp = P.cfg4_params(4096)
    prm = dp.bfv_params
    q, n, d, G = prm.ct_basis.moduli, 4096, dp.num_digits, prm.gadget_digits
    if kind == "digits":
        a, b, rlk, _ = W.digit_case_dbfv(q, prm.plain_modulus, prm.gadget_base, G, n, d)
    else:
        a, b, rlk = W.tensor_case_dbfv(q, n, d, G)
    want = cref.dbfv_mul(dp, a, b, rlk, threads=8)
    ctx = HipContext.from_params(prm)
    assert ctx.psum_max >= 2
    ctx.load_relin_key(rlk)
    a2, b2 = pad(a, b, 64, q, n, 2)           # 192 products: two lanes
    out, _ = ctx.dbfv_mul(d, dp.base, dp.plain_modulus, a2, b2)
    assert np.array_equal(out[:1], want)


@pytest.mark.parametrize("name", ["worst_cfg5_digits", "worst_cfg5_tensor"])
def test_worst_case_dbfv_cfg5(gpu_available, name):
    import sys
    sys.path.insert(0, GOLD)
    from make_golden import worst_inputs
    with open(os.path.join(GOLD, "digests.json")) as f:
        spec = json.load(f)[name]
    dp, a, b, rlk = worst_inputs(spec)
    assert sha(np.concatenate([a.ravel(), b.ravel(), rlk.ravel()])) == spec["sha256_inputs"]
    prm = dp.bfv_params
    q, n, d = prm.ct_basis.moduli, spec["n"], dp.num_digits
    ctx = HipContext.from_params(prm)
    assert ctx.psum_max >= 8
    ctx.load_relin_key(rlk)
    a2, b2 = pad(a, b, 8, q, n, 3)            # the bench's batch of 8: two lanes of 144 products
    out, _ = ctx.dbfv_mul(d, dp.base, dp.plain_modulus, a2, b2)
    assert sha(out[:1]) == spec["sha256_out"]
