"""The hand-scheduled inverse NTT (ntt_inv_asm_kernel and the fused tensor + inverse with the
generated InvRoundAsm rounds, n = 4096 / 8192) against the oracle and against the
compiler-scheduled kernels it replaces (EXACTO_NTT_ASM_INV=0).

Bit-exact: integer work.  Reference: concrete-ntt Plan::inv + normalize (src/ring/ntt.rs:58-67);
the tensor path is bfv_mul_no_relin's exact multi-limb product (src/bfv/eval.rs:113-147).
"""

import os

import numpy as np
import pytest

from oracle.ring import CoeffPoly, NttPoly, make_plan
from oracle import params as P
from exacto_amd._ffi import HipContext
from bridge import uniform_residues

pytestmark = pytest.mark.gpu

QS = [1152921504606830593, 1152921504606748673, 1152921504606683137, 1152921504606601217]


def _with_env(value, make):
    old = os.environ.get("EXACTO_NTT_ASM_INV")
    os.environ["EXACTO_NTT_ASM_INV"] = value
    try:
        return make()
    finally:
        if old is None:
            del os.environ["EXACTO_NTT_ASM_INV"]
        else:
            os.environ["EXACTO_NTT_ASM_INV"] = old


@pytest.mark.parametrize("n,L,B", [(4096, 3, 5), (8192, 4, 3)])
def test_inverse_matches_compiler_kernel_and_oracle(gpu_available, n, L, B):
    import torch
    qs = QS[:L]
    rng = np.random.default_rng(n + B)
    a = uniform_residues(rng, (B,), qs, n)
    a[0, 0] = qs[0] - 1                                   # extremes: all q-1, alternating q-1 / 0
    a[-1, -1] = np.where(np.arange(n) % 2 == 0, qs[-1] - 1, 0)
    a[B // 2, 0] = 0
    outs = []
    for asm in ("1", "0"):
        ctx = _with_env(asm, lambda: HipContext(n, qs, plain_modulus=65537))
        d = torch.from_numpy(a.copy().view(np.int64)).cuda()
        torch.cuda.synchronize()
        ctx.rns_inv_dev(d, B)
        ctx.synchronize()
        outs.append(d.cpu().numpy().view(np.uint64).copy())
    assert np.array_equal(outs[0], outs[1])
    for (b, i) in {(0, 0), (B - 1, L - 1), (B // 2, 1)}:
        plan = make_plan(n, qs[i])
        want = NttPoly(list(int(x) for x in a[b, i]), qs[i], plan).to_coeff_poly().coeffs
        assert [int(x) for x in outs[0][b, i]] == want, (b, i)


@pytest.mark.parametrize("n,L,B", [(4096, 3, 6), (8192, 4, 2)])
def test_tensor_inverse_matches_compiler_kernel(gpu_available, n, L, B):
    """bfv_mul_and_relin through the fused tensor + inverse NTT (every auxiliary prime of the exact
    path is also in the asm window) is bit-identical with the compiler-scheduled rounds."""
    prm = P.cfg3_params(n) if L == 3 else P.cfg5_params(n).bfv_params
    q = prm.ct_basis.moduli
    rng = np.random.default_rng(90 + n)
    ct1 = uniform_residues(rng, (B, 2), q, n)
    ct2 = uniform_residues(rng, (B, 2), q, n)
    ct1[0, 0, 0] = q[0] - 1
    rlk = uniform_residues(rng, (prm.gadget_digits, 2), q, n)
    outs = []
    for asm in ("1", "0"):
        ctx = _with_env(asm, lambda: HipContext.from_params(prm, device=0))
        ctx.load_relin_key(rlk)
        outs.append(ctx.bfv_mul_and_relin(ct1, ct2))
    assert np.array_equal(outs[0], outs[1])
