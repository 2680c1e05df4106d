"""GPU parity of bfv_add / bfv_sub / bfv_neg (reference src/bfv/eval.rs:14-60) against the oracle
(oracle/bfv.py:52-79), including mixed degrees: the longer operand's extra components pass through
(eval.rs:21-22), and under subtraction ct2's are negated (eval.rs:41-42).  Bit-exact, NTT domain,
host and device entry points, cfg3's 3x60-bit basis and the compact single-prime basis."""

import numpy as np
import pytest

from oracle import bfv as obfv
from oracle import params as P
from exacto_amd._ffi import HipContext, ExactoError
from bridge import ct_to_np, np_to_ct, uniform_residues

pytestmark = pytest.mark.gpu


def _oracle(fn, ct1, ct2, prm):
    return np.stack([ct_to_np(fn(np_to_ct(ct1[b], prm), np_to_ct(ct2[b], prm))) for b in range(ct1.shape[0])])


@pytest.mark.parametrize("p1,p2", [(2, 2), (3, 2), (2, 3), (1, 3), (3, 3)])
def test_bfv_add_sub_mixed_degree(gpu_available, p1, p2):
    n = 64
    prm = P.cfg3_params(n)
    q = prm.ct_basis.moduli
    rng = np.random.default_rng(100 + 10 * p1 + p2)
    B = 3
    ct1 = uniform_residues(rng, (B, p1), q, n)
    ct2 = uniform_residues(rng, (B, p2), q, n)
    ctx = HipContext.from_params(prm)
    assert np.array_equal(ctx.bfv_add(ct1, ct2), _oracle(obfv.bfv_add, ct1, ct2, prm))
    assert np.array_equal(ctx.bfv_sub(ct1, ct2), _oracle(obfv.bfv_sub, ct1, ct2, prm))
    want_neg = np.stack([ct_to_np(obfv.bfv_neg(np_to_ct(ct1[b], prm))) for b in range(B)])
    assert np.array_equal(ctx.bfv_neg(ct1), want_neg)


def test_bfv_add_sub_edge_values(gpu_available):
    # zeros and q - 1 in every limb: sums wrap to q - 2, differences 0 - (q-1) = 1, neg(0) = 0
    n = 16
    prm = P.cfg3_params(n)
    q = np.array(prm.ct_basis.moduli, dtype=np.uint64)
    top = np.broadcast_to((q - 1)[None, None, :, None], (2, 2, 3, n)).copy()
    zero = np.zeros_like(top)
    ctx = HipContext.from_params(prm)
    assert np.array_equal(ctx.bfv_add(top, top), _oracle(obfv.bfv_add, top, top, prm))
    assert np.array_equal(ctx.bfv_sub(zero, top), _oracle(obfv.bfv_sub, zero, top, prm))
    assert np.array_equal(ctx.bfv_neg(zero), zero)


def test_bfv_add_dev_in_place_and_alias_rule(gpu_available):
    import torch
    prm = P.compact_bfv()       # cfg1: one 40-bit prime, n = 1024
    q = prm.ct_basis.moduli
    n = prm.ring_degree
    rng = np.random.default_rng(7)
    B = 4
    ct1 = uniform_residues(rng, (B, 3), q, n)
    ct2 = uniform_residues(rng, (B, 2), q, n)
    want = _oracle(obfv.bfv_sub, ct1, ct2, prm)
    ctx = HipContext.from_params(prm)
    dev = torch.device("cuda", 0)
    a = torch.from_numpy(ct1.view(np.int64)).to(dev)
    b = torch.from_numpy(ct2.view(np.int64)).to(dev)
    ctx.bfv_sub_dev(a, 3, b, 2, a, B)      # in place over the longer operand: allowed
    ctx.synchronize()
    assert np.array_equal(a.cpu().numpy().view(np.uint64), want)
    with pytest.raises(ExactoError) as e:  # over the shorter one: rejected, never silently wrong
        ctx.bfv_add_dev(a, 3, b, 2, b, B)
    assert e.value.variant == "InvalidParam"
    # a partial overlap (output shifted by one component into ct1) is rejected too
    big = torch.zeros((B + 1) * 3 * n, dtype=torch.int64, device=dev)
    x = big[: B * 3 * n]
    o = big[n: n + B * 3 * n]
    with pytest.raises(ExactoError) as e:
        ctx.bfv_add_dev(x, 3, b, 2, o, B)
    assert e.value.variant == "InvalidParam"
