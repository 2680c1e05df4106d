"""GPU parity of the NTT engine (K1/K2) and RNS pointwise ops (K3) against the oracle.

Reference tests mirrored: src/ring/ntt.rs:170-212 (roundtrip, NTT-mul == mul_naive, NTT-add),
src/ring/rns.rs:299-338.  Bit-exact: integer work.
"""

import numpy as np
import pytest

from oracle.ring import CoeffPoly, NttPoly, make_plan
from exacto_amd._ffi import HipContext, ExactoError

pytestmark = pytest.mark.gpu

CFG2_Q = 1152921504606830593


def oracle_fwd(coeffs, n, q):
    plan = make_plan(n, q)
    return NttPoly.from_coeff_poly(CoeffPoly([int(x) for x in coeffs], q), plan).evals


@pytest.mark.parametrize("n,q", [(16, 65537), (32, 65537), (64, 65537), (256, 65537),
                                 (1024, 1099509805057), (1024, 562949953443841),
                                 (2048, CFG2_Q), (4096, CFG2_Q), (8192, CFG2_Q),
                                 (16384, 1152921504606748673), (4096, 1152921504606748673),
                                 (4096, 2305843009213554689), (4096, 4611686018427322369),
                                 (1024, 4611686018427322369)])
def test_ntt_fwd_matches_oracle(gpu_available, n, q):
    rng = np.random.default_rng(n + q % 1000)
    ctx = HipContext(n, [q], plain_modulus=257)
    a = rng.integers(0, q, size=(3, n), dtype=np.uint64)
    got = ctx.ntt_fwd(a)
    for r in range(3):
        assert [int(x) for x in got[r]] == oracle_fwd(a[r], n, q)
    back = ctx.ntt_inv(got)
    assert np.array_equal(back, a)


def test_ntt_kat_roundtrip_and_mul(gpu_available):
    # ntt.rs:170-195: n=16, q=65537
    n, q = 16, 65537
    ctx = HipContext(n, [q], plain_modulus=257)
    x = np.array([[1, 2, 3, 4, 5, 6, 7, 8] + [0] * 8], dtype=np.uint64)
    assert np.array_equal(ctx.ntt_inv(ctx.ntt_fwd(x)), x)
    a = np.array([[1, 1] + [0] * 14], dtype=np.uint64)
    fa = ctx.ntt_fwd(a)
    prod = (fa.astype(object) * fa.astype(object)) % q
    c = ctx.ntt_inv(np.array(prod, dtype=np.uint64))
    assert [int(v) for v in c[0][:4]] == [1, 2, 1, 0]


def test_ntt_mul_matches_naive_random(gpu_available):
    n, q = 64, 65537
    rng = np.random.default_rng(5)
    ctx = HipContext(n, [q], plain_modulus=257)
    a = rng.integers(0, q, size=(1, n), dtype=np.uint64)
    b = rng.integers(0, q, size=(1, n), dtype=np.uint64)
    fa, fb = ctx.ntt_fwd(a), ctx.ntt_fwd(b)
    prod = np.array((fa.astype(object) * fb.astype(object)) % q, dtype=np.uint64)
    got = ctx.ntt_inv(prod)
    want = CoeffPoly([int(v) for v in a[0]], q).mul_naive(CoeffPoly([int(v) for v in b[0]], q))
    assert [int(v) for v in got[0]] == want.coeffs


def test_cfg2_pointwise_pipeline(gpu_available):
    """BASELINE configs[1]: batched fwd NTT, pointwise mul, inv NTT at n=4096, 60-bit q."""
    import torch
    n, q = 4096, CFG2_Q
    B = 64
    rng = np.random.default_rng(2)
    ctx = HipContext(n, [q], plain_modulus=65537)
    a = rng.integers(0, q, size=(B, n), dtype=np.uint64)
    b = rng.integers(0, q, size=(B, n), dtype=np.uint64)
    da = torch.from_numpy(a.view(np.int64)).cuda()
    db = torch.from_numpy(b.view(np.int64)).cuda()
    ctx.rns_fwd_dev(da, B)
    ctx.rns_fwd_dev(db, B)
    ctx.rns_mul_dev(da, db, da, B)
    ctx.rns_inv_dev(da, B)
    ctx.synchronize()
    got = da.cpu().numpy().view(np.uint64)
    # oracle on 2 polys (full check), negacyclic schoolbook identity on all via evaluation at X=1?
    plan = make_plan(n, q)
    for r in (0, B - 1):
        fa = NttPoly.from_coeff_poly(CoeffPoly([int(x) for x in a[r]], q), plan)
        fb = NttPoly.from_coeff_poly(CoeffPoly([int(x) for x in b[r]], q), plan)
        assert [int(x) for x in got[r]] == fa.mul(fb).to_coeff_poly().coeffs
    # every row: a(psi) * b(psi) == c(psi) at psi = first evaluation point (size-independent check)
    psi = plan.psi
    pw = [pow(psi, i, q) for i in range(n)]
    for r in range(B):
        ev = lambda v: sum(int(x) * w for x, w in zip(v, pw)) % q
        assert ev(got[r]) == ev(a[r]) * ev(b[r]) % q


def test_rns_pointwise_ops(gpu_available):
    import torch
    n = 1024
    qs = [1152921504606830593, 1152921504606748673, 1152921504606683137]
    ctx = HipContext(n, qs, plain_modulus=65537)
    rng = np.random.default_rng(9)
    a = np.stack([rng.integers(0, q, size=(4, n), dtype=np.uint64) for q in qs], axis=1)
    b = np.stack([rng.integers(0, q, size=(4, n), dtype=np.uint64) for q in qs], axis=1)
    da = torch.from_numpy(a.view(np.int64)).cuda()
    db = torch.from_numpy(b.view(np.int64)).cuda()
    out = torch.empty_like(da)
    A, Bo = a.astype(object), b.astype(object)
    Q = np.array(qs, dtype=object)[None, :, None]
    for op, want in [("add", (A + Bo) % Q), ("sub", (A - Bo) % Q), ("mul", (A * Bo) % Q)]:
        getattr(ctx, f"rns_{op}_dev")(da, db, out, 4)
        ctx.synchronize()
        assert np.array_equal(out.cpu().numpy().view(np.uint64).astype(object), want), op
    ctx.rns_neg_dev(da, out, 4)
    ctx.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint64).astype(object), (-A) % Q)
    s = (1 << 63) + 12345
    ctx.rns_scalar_mul_dev(da, s, out, 4)
    ctx.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint64).astype(object), (A * (s % Q)) % Q)


def test_limb_out_of_range(gpu_available):
    ctx = HipContext(16, [65537], plain_modulus=257)
    with pytest.raises(ExactoError) as e:
        ctx.ntt_fwd(np.zeros((1, 16), dtype=np.uint64), limb=3)
    assert e.value.variant == "DimensionMismatch"


@pytest.mark.parametrize("n,q", [(16, 65537), (4096, CFG2_Q), (8192, 1152921504606748673),
                                 (4096, 4611686018427322369), (2048, 2305843009213554689)])
def test_ntt_extreme_inputs(gpu_available, n, q):
    # worst-case magnitudes for the lazy bounds: all q-1, alternating 0/q-1, and the inverse
    # applied to all-(q-1) evaluations
    ctx = HipContext(n, [q], plain_modulus=257)
    top = np.full(n, q - 1, dtype=np.uint64)
    alt = np.where(np.arange(n) % 2 == 0, q - 1, 0).astype(np.uint64)
    a = np.stack([top, alt, top[::-1].copy()])
    got = ctx.ntt_fwd(a)
    for r in range(2):
        assert [int(x) for x in got[r]] == oracle_fwd(a[r], n, q)
    assert np.array_equal(ctx.ntt_inv(got), a)
    inv_top = ctx.ntt_inv(top[None, :])
    assert np.array_equal(ctx.ntt_fwd(inv_top), top[None, :])


@pytest.mark.parametrize("n,qs", [(16, [65537]), (256, [65537, 1099509805057]), (1024, [1099509805057]),
                                  (4096, [CFG2_Q]), (8192, [CFG2_Q, 1152921504606748673]),
                                  (4096, [1152921504606830593, 1152921504606748673, 1152921504606683137]),
                                  (4096, [4611686018427322369]), (16384, [1152921504606748673])])
def test_rns_mul_inv_fused_matches_composition(gpu_available, n, qs):
    """exacto_rns_mul_inv_dev (pointwise product fused into the inverse) against rns_mul + rns_inv
    (ntt.rs:119-129 then 58-67) on the same inputs, in place (out = a) and out of place, with
    extreme residues; n = 16 also against mul_naive (ntt.rs:181-195)."""
    import torch
    L = len(qs)
    B = 5
    rng = np.random.default_rng(n + L)
    ctx = HipContext(n, qs, plain_modulus=257)
    q = np.array(qs, dtype=np.uint64)[None, :, None]
    a = (rng.integers(0, 1 << 63, size=(B, L, n), dtype=np.uint64) % q).astype(np.uint64)
    b = (rng.integers(0, 1 << 63, size=(B, L, n), dtype=np.uint64) % q).astype(np.uint64)
    a[0] = q[0] - 1
    b[0, :, ::2] = q[0, :, 0:1] - 1
    da = torch.from_numpy(a.view(np.int64)).cuda()
    db = torch.from_numpy(b.view(np.int64)).cuda()
    ref = da.clone()
    torch.cuda.synchronize()  # the context's stream does not wait for torch's (the clone)
    ctx.rns_mul_dev(ref, db, ref, B)
    ctx.rns_inv_dev(ref, B)
    out = torch.empty_like(da)
    ctx.rns_mul_inv_dev(da, db, out, B)
    ctx.rns_mul_inv_dev(da, db, da, B)       # in place
    ctx.synchronize()
    want = ref.cpu().numpy()
    assert np.array_equal(out.cpu().numpy(), want)
    assert np.array_equal(da.cpu().numpy(), want)
    if n == 16:
        fa = ctx.ntt_inv(a.reshape(-1, n)[:1])   # coefficient-domain operands: INTT of the inputs
        fb = ctx.ntt_inv(b.reshape(-1, n)[:1])
        naive = CoeffPoly([int(v) for v in fa[0]], qs[0]).mul_naive(CoeffPoly([int(v) for v in fb[0]], qs[0]))
        assert [int(v) for v in want.view(np.uint64)[0, 0]] == naive.coeffs


@pytest.mark.parametrize("n,qs", [(16, [65537]), (1024, [1099509805057, 562949953443841]), (4096, [CFG2_Q]),
                                  (4096, [1152921504606830593, 1152921504606748673, 1152921504606683137]),
                                  (8192, [CFG2_Q, 1152921504606748673]), (4096, [4611686018427322369])])
def test_rns_polymul_matches_composition(gpu_available, n, qs):
    """exacto_rns_polymul_dev (one kernel per product at n = 4096 / 8192 with special primes, the
    composition otherwise) against rns_fwd x2 + rns_mul + rns_inv, in place and out of place; the
    reference's own negacyclic identity (ntt.rs:181-195) against mul_naive on the first product."""
    import torch
    L = len(qs)
    B = 4
    rng = np.random.default_rng(3 * n + L)
    ctx = HipContext(n, qs, plain_modulus=257)
    q = np.array(qs, dtype=np.uint64)[None, :, None]
    a = (rng.integers(0, 1 << 63, size=(B, L, n), dtype=np.uint64) % q).astype(np.uint64)
    b = (rng.integers(0, 1 << 63, size=(B, L, n), dtype=np.uint64) % q).astype(np.uint64)
    a[1] = q[0] - 1
    b[1, :, 1::2] = q[0, :, 0:1] - 1
    da = torch.from_numpy(a.view(np.int64)).cuda()
    db = torch.from_numpy(b.view(np.int64)).cuda()
    ra, rb = da.clone(), db.clone()
    torch.cuda.synchronize()  # the context's stream does not wait for torch's (the clones)
    ctx.rns_fwd_dev(ra, B)
    ctx.rns_fwd_dev(rb, B)
    ctx.rns_mul_dev(ra, rb, ra, B)
    ctx.rns_inv_dev(ra, B)
    out = torch.empty_like(da)
    ctx.rns_polymul_dev(da, db, out, B)
    ctx.rns_polymul_dev(da, db, db, B)   # in place on b
    ctx.synchronize()
    want = ra.cpu().numpy()
    assert np.array_equal(out.cpu().numpy(), want)
    assert np.array_equal(db.cpu().numpy(), want)
    if n <= 1024:
        naive = CoeffPoly([int(v) for v in a[0, 0]], qs[0]).mul_naive(CoeffPoly([int(v) for v in b[0, 0]], qs[0]))
        assert [int(v) for v in want.view(np.uint64)[0, 0]] == naive.coeffs


def test_fused_product_entry_points_edge_cases(gpu_available):
    """count = 0 is a no-op; a null buffer is InvalidParam (the library's pointer checks), for the
    fused product + inverse and the one-kernel product."""
    import ctypes
    import torch
    n = 4096
    ctx = HipContext(n, [CFG2_Q], plain_modulus=257)
    a = torch.zeros((1, 1, n), dtype=torch.int64, device="cuda")
    ctx.rns_mul_inv_dev(a, a, a, 0)
    ctx.rns_polymul_dev(a, a, a, 0)
    for fn in ("exacto_rns_mul_inv_dev", "exacto_rns_polymul_dev"):
        rc = getattr(ctx._lib, fn)(ctx._h, None, ctypes.c_void_p(a.data_ptr()), ctypes.c_void_p(a.data_ptr()), 1)
        assert rc != 0, fn
    # all-zero operands: the product is zero
    ctx.rns_polymul_dev(a, a, a, 1)
    ctx.synchronize()
    assert not a.any()
