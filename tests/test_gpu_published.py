"""GPU parity at the reference's own published configurations, at production batch sizes.

* compact_bfv (presets.rs:24-35; README.md:153 publishes its bfv_mul_and_relin at ~390 us): the
  literal HPS multiplier with one aux prime (eval.rs:157-332), G = 3.  A batch spanning several
  pipeline chunks and both lanes, against the C oracle (oracle/c, bit-exact restatement).
* u64_dbfv (presets.rs:61-75; reports/paper_reproduction.md:9 publishes its dbfv_mul at 31.395 ms):
  d = 8, b = 256, p = 2^64 over one 60-bit q with two HPS aux primes (eval.rs:349-404), G = 8.
  Every one of the d^2 products is an HPS product; the oracle multiplies all 64 of them.
"""

import numpy as np
import pytest

from oracle import cref
from oracle import params as P
from exacto_amd._ffi import HipContext, PATH_HPS
from bridge import uniform_residues

pytestmark = pytest.mark.gpu


def _need_cref():
    if not cref.available():
        pytest.skip("oracle/c not built")


def test_compact_bfv_production_batch(gpu_available):
    _need_cref()
    prm = P.compact_bfv()
    q, n = prm.ct_basis.moduli, prm.ring_degree
    rng = np.random.default_rng(0xE7AC7001)
    # the library's default chunk at compact_bfv is 7168 products, so B = 1100 is ONE chunk split in
    # halves over the two lanes; set_chunk(512) then makes it 512 + 512 + 76 (chunk and lane
    # boundaries).  The bench's own B = 8192 (7168 + 1024) is test_gpu_bench_shapes.py's cfg1 case.
    B = 1100
    ct1 = uniform_residues(rng, (B, 2), q, n)
    ct2 = uniform_residues(rng, (B, 2), q, n)
    rlk = uniform_residues(rng, (prm.gadget_digits, 2), q, n)
    ctx = HipContext.from_params(prm)
    assert ctx.path == PATH_HPS and ctx.G == 3
    ctx.load_relin_key(rlk)
    got = ctx.bfv_mul_and_relin(ct1, ct2)
    want = cref.bfv_mul_and_relin(prm, ct1, ct2, rlk, threads=16)
    assert np.array_equal(got, want)
    ctx.set_chunk(512)
    assert np.array_equal(ctx.bfv_mul_and_relin(ct1, ct2), want)
    # one product alone (the published single-call case) is the same as inside the batch
    assert np.array_equal(ctx.bfv_mul_and_relin(ct1[777:778], ct2[777:778]), want[777:778])


@pytest.mark.parametrize("B", [1, 3])
def test_u64_dbfv_dbfv_mul(gpu_available, B):
    _need_cref()
    dp = P.u64_dbfv()
    prm = dp.bfv_params
    q, n = prm.ct_basis.moduli, prm.ring_degree
    rng = np.random.default_rng(0xE7AC70A0 + B)
    a = uniform_residues(rng, (B, dp.num_digits, 2), q, n)
    b = uniform_residues(rng, (B, dp.num_digits, 2), q, n)
    rlk = uniform_residues(rng, (prm.gadget_digits, 2), q, n)
    ctx = HipContext.from_params(prm)
    assert ctx.path == PATH_HPS and ctx.G == 8
    ctx.load_relin_key(rlk)
    got, _ = ctx.dbfv_mul(dp.num_digits, dp.base, dp.plain_modulus, a, b)
    want = cref.dbfv_mul(dp, a, b, rlk, threads=16)
    assert np.array_equal(got, want)
