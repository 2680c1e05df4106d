"""The persistent LDS-DMA forward NTT (ntt_fwd_pipe_kernel, n = 4096, EXACTO_NTT_PIPE=1) against the
oracle and against the default one-workgroup-per-polynomial kernel (ntt_fwd_pin_kernel), on batches
large enough that every resident workgroup streams several polynomials through its LDS
halves, with mixed primes, and on the int16 gadget-digit source of bfv_mul_and_relin.

Bit-exact: integer work.  Reference: concrete-ntt Plan::fwd (src/ring/ntt.rs:42-55).
"""

import os

import numpy as np
import pytest

from oracle.ring import CoeffPoly, NttPoly, make_plan
from oracle import params as P
from exacto_amd._ffi import HipContext
from bridge import uniform_residues

pytestmark = pytest.mark.gpu

QS = [1152921504606830593, 1152921504606748673, 1152921504606683137]


def _ctx(pipe: bool, *args, **kw):
    old = os.environ.get("EXACTO_NTT_PIPE")
    os.environ["EXACTO_NTT_PIPE"] = "1" if pipe else "0"
    try:
        return HipContext(*args, **kw)
    finally:
        if old is None:
            del os.environ["EXACTO_NTT_PIPE"]
        else:
            os.environ["EXACTO_NTT_PIPE"] = old


def _ctx_params(pipe: bool, prm):
    old = os.environ.get("EXACTO_NTT_PIPE")
    os.environ["EXACTO_NTT_PIPE"] = "1" if pipe else "0"
    try:
        return HipContext.from_params(prm, device=0)
    finally:
        if old is None:
            del os.environ["EXACTO_NTT_PIPE"]
        else:
            os.environ["EXACTO_NTT_PIPE"] = old


@pytest.mark.parametrize("B", [1, 171, 700])
def test_pipe_fwd_rns_batch(gpu_available, B):
    """B ciphertext limbs-sets of 3 primes (3B polynomials; 2100 > the 510 resident workgroups)."""
    import torch
    n = 4096
    rng = np.random.default_rng(B)
    a = uniform_residues(rng, (B,), QS, n)
    a[0, 0] = QS[0] - 1                      # extreme magnitudes in the first and last rows
    a[-1, -1] = np.where(np.arange(n) % 2 == 0, QS[-1] - 1, 0)
    outs = []
    for pipe in (True, False):
        ctx = _ctx(pipe, n, QS, plain_modulus=65537)
        d = torch.from_numpy(a.copy().view(np.int64)).cuda()
        ctx.rns_fwd_dev(d, B)
        ctx.synchronize()
        outs.append(d.cpu().numpy().view(np.uint64).copy())
        if pipe:
            ctx.rns_inv_dev(d, B)
            ctx.synchronize()
            assert np.array_equal(d.cpu().numpy().view(np.uint64), a), "roundtrip"
    assert np.array_equal(outs[0], outs[1])
    for (b, i) in {(0, 0), (B - 1, 2), (B // 2, 1)}:
        plan = make_plan(n, QS[i])
        want = NttPoly.from_coeff_poly(CoeffPoly([int(x) for x in a[b, i]], QS[i]), plan).evals
        assert [int(x) for x in outs[0][b, i]] == want


def test_pipe_bfv_mul_and_relin_matches_unpipelined(gpu_available):
    """cfg3 shape (n=4096, 3x60-bit, base 2^16, G=12): the digit NTTs read int16 sources; 24
    products give 864 digit polynomials, so workgroups run more than one iteration."""
    import torch
    prm = P.cfg3_params(4096)
    rng = np.random.default_rng(33)
    B = 24
    q = prm.ct_basis.moduli
    ct1 = uniform_residues(rng, (B, 2), q, 4096)
    ct2 = uniform_residues(rng, (B, 2), q, 4096)
    rlk = uniform_residues(rng, (prm.gadget_digits, 2), q, 4096)
    outs = []
    for pipe in (True, False):
        ctx = _ctx_params(pipe, prm)
        ctx.load_relin_key(rlk)
        outs.append(ctx.bfv_mul_and_relin(ct1, ct2))
    assert np.array_equal(outs[0], outs[1])
