"""dBFV psum: each output limb's c0 / c1 scaled once from the sum of its products' tensors
(ntt_inv_tensor_sum_kernel + exact_psum_sp_kernel) instead of per product and summed after
(dbfv_combine_kernel, EXACTO_PSUM=0).

Reference: dbfv_mul (src/dbfv/eval.rs:82-149): d^2 bfv_mul_and_relin (src/bfv/eval.rs:73-82, the
exact tensor-and-round of eval.rs:113-147, 711-831), summed per output limb, then reduce
(src/dbfv/reduction.rs:15-93).  The sum of the rounded products equals one rounding of the summed
tensors plus the per-product corrections, an integer identity while |sum| < P / 2 (checked at
context creation).  Bit-exact: integer work.  Covers both BASELINE dBFV configurations (cfg4: n =
4096, 3 limbs, per-component tensor kernel; cfg5: n = 8192, 4 limbs, the (item, prime) tensor
kernel), batches spanning several chunks on both pipeline lanes (chunks hold whole dBFV items),
chains, and the C restatement of the reference on single products.
"""

import os

import numpy as np
import pytest

from oracle import params as P, cref
from exacto_amd._ffi import HipContext
from bridge import uniform_residues

pytestmark = pytest.mark.gpu


def _ctx(prm, psum: bool, chunk=0, var="EXACTO_PSUM"):
    old = os.environ.get(var)
    os.environ[var] = "1" if psum else "0"
    try:
        ctx = HipContext.from_params(prm, device=0)
    finally:
        if old is None:
            del os.environ[var]
        else:
            os.environ[var] = old
    if chunk:
        ctx.set_chunk(chunk)
    return ctx


@pytest.mark.parametrize("B,chunk", [(1, 0), (5, 4), (4, 0)])
def test_psum_cfg4_matches_per_product(gpu_available, B, chunk):
    """cfg4 (d = 2, 3 products per item): chunk 4 rounds down to 3 products = one item per chunk."""
    dp = P.cfg4_params(4096)
    prm = dp.bfv_params
    q, n, d = prm.ct_basis.moduli, 4096, 2
    rng = np.random.default_rng(4040 + B)
    a = uniform_residues(rng, (B, d, 2), q, n)
    b = uniform_residues(rng, (B, d, 2), q, n)
    rlk = uniform_residues(rng, (prm.gadget_digits, 2), q, n)
    outs = []
    for on in (True, False):
        ctx = _ctx(prm, on, chunk)
        assert (ctx.psum_max >= 2) if on else ctx.psum_max == 0
        ctx.load_relin_key(rlk)
        outs.append(ctx.dbfv_mul(d, dp.base, dp.plain_modulus, a, b)[0])
    assert np.array_equal(outs[0], outs[1])
    if cref.available():
        i = B - 1
        p01 = cref.bfv_mul_and_relin(prm, a[i:i + 1, 0], b[i:i + 1, 1], rlk, threads=4)[0]
        p10 = cref.bfv_mul_and_relin(prm, a[i:i + 1, 1], b[i:i + 1, 0], rlk, threads=4)[0]
        Q = np.array(q, dtype=object)[None, :, None]
        assert np.array_equal(outs[0][i, 1].astype(object), (p01.astype(object) + p10.astype(object)) % Q)


def test_psum_cfg5_chunks_and_chain(gpu_available):
    """cfg5 (d = 8, 36 products per item, up to 8 per limb): two items in two chunks of 36."""
    dp = P.cfg5_params(8192)
    prm = dp.bfv_params
    q, n, d = prm.ct_basis.moduli, 8192, dp.num_digits
    rng = np.random.default_rng(5050)
    a = uniform_residues(rng, (2, d, 2), q, n)
    b = uniform_residues(rng, (2, d, 2), q, n)
    rlk = uniform_residues(rng, (prm.gadget_digits, 2), q, n)
    res = []
    for on in (True, False):
        ctx = _ctx(prm, on, 40)
        assert (ctx.psum_max >= 8) if on else ctx.psum_max == 0
        ctx.load_relin_key(rlk)
        out = ctx.dbfv_mul(d, dp.base, dp.plain_modulus, a, b)[0]
        chain = ctx.dbfv_mul_chain(d, dp.base, dp.plain_modulus, a, b, 2)
        res.append((out, chain))
    assert np.array_equal(res[0][0], res[1][0])
    assert np.array_equal(res[0][1], res[1][1])


def test_int8_digits_cfg5(gpu_available):
    """cfg5's gadget base 256: the products' digits summed per limb are written and read as int8
    (every balanced digit lies in [-128, 127]); identical to the int16 form (EXACTO_DIGIT8=0)."""
    dp = P.cfg5_params(8192)
    prm = dp.bfv_params
    q, n, d = prm.ct_basis.moduli, 8192, dp.num_digits
    rng = np.random.default_rng(5151)
    a = uniform_residues(rng, (1, d, 2), q, n)
    b = uniform_residues(rng, (1, d, 2), q, n)
    rlk = uniform_residues(rng, (prm.gadget_digits, 2), q, n)
    res = []
    for on in (True, False):
        ctx = _ctx(prm, on, var="EXACTO_DIGIT8")
        ctx.load_relin_key(rlk)
        res.append(ctx.dbfv_mul(d, dp.base, dp.plain_modulus, a, b)[0])
    assert np.array_equal(res[0], res[1])


@pytest.mark.parametrize("chain", [False, True])
def test_dbfv_item_groups_match_one_pass(gpu_available, chain):
    """A batch whose buffers exceed EXACTO_DBFV_GROUP_MB runs in groups of whole items
    (dbfv_mul_core); 1 MB forces one item per group at cfg4 (4.4 MB per item).  Items are
    independent, so every group size gives the one-pass result, for dbfv_mul and for a chain (whose
    constant right operand's extensions are then recomputed per group)."""
    dp = P.cfg4_params(4096)
    prm = dp.bfv_params
    q, n, d, B = prm.ct_basis.moduli, 4096, 2, 3
    rng = np.random.default_rng(5151)
    a = uniform_residues(rng, (B, d, 2), q, n)
    b = uniform_residues(rng, (B, d, 2), q, n)
    rlk = uniform_residues(rng, (prm.gadget_digits, 2), q, n)
    outs = []
    for mb in ("1", None):
        old = os.environ.get("EXACTO_DBFV_GROUP_MB")
        if mb:
            os.environ["EXACTO_DBFV_GROUP_MB"] = mb
        try:
            ctx = HipContext.from_params(prm, device=0)
        finally:
            if old is None:
                os.environ.pop("EXACTO_DBFV_GROUP_MB", None)
            else:
                os.environ["EXACTO_DBFV_GROUP_MB"] = old
        ctx.load_relin_key(rlk)
        if chain:
            outs.append(ctx.dbfv_mul_chain(d, dp.base, dp.plain_modulus, a, b, 2))
        else:
            outs.append(ctx.dbfv_mul(d, dp.base, dp.plain_modulus, a, b)[0])
    assert np.array_equal(outs[0], outs[1])


def test_psum_cfg5_two_halves_vs_limbwise(gpu_available):
    """The cfg5 bench path as it runs by default -- psum, int8 digit sums, the ks32 digit-sum key
    switch, and a batch that fits one chunk split into two halves on both pipeline lanes (B = 4:
    144 products, 2 x 72) -- against the other key-switch formulation: 60-bit limb-wise MAC
    (EXACTO_KS32=0) and per-product scaling summed by dbfv_combine (EXACTO_PSUM=0)."""
    dp = P.cfg5_params(8192)
    prm = dp.bfv_params
    q, n, d, B = prm.ct_basis.moduli, 8192, dp.num_digits, 4
    rng = np.random.default_rng(5252)
    a = uniform_residues(rng, (B, d, 2), q, n)
    b = uniform_residues(rng, (B, d, 2), q, n)
    rlk = uniform_residues(rng, (prm.gadget_digits, 2), q, n)
    outs = []
    for envs in ({}, {"EXACTO_KS32": "0", "EXACTO_PSUM": "0"}):
        old = {k: os.environ.get(k) for k in envs}
        os.environ.update(envs)
        try:
            ctx = HipContext.from_params(prm, device=0)
        finally:
            for k, v in old.items():
                if v is None:
                    del os.environ[k]
                else:
                    os.environ[k] = v
        assert (ctx.psum_max >= 8) if not envs else ctx.psum_max == 0
        ctx.load_relin_key(rlk)
        outs.append(ctx.dbfv_mul(d, dp.base, dp.plain_modulus, a, b)[0])
    assert np.array_equal(outs[0], outs[1])
