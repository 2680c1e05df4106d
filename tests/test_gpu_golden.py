"""GPU vs committed golden fixtures, dBFV, and full-size properties.

* every tests/golden/vectors.npz case (bfv_mul_and_relin, bfv_mul_no_relin, dbfv_mul) bit-exact;
* full-size cfg3 (n=4096, 3x60-bit) against the committed C-oracle digest;
* BASELINE configs[3] (dBFV d=2 over cfg3's basis) at full size vs oracle on sampled rows;
* size-independent properties at batch scale: chunking invariance, batch-position invariance,
  agreement of mul_no_relin + relinearize with the fused path;
* dBFV decrypt-level tests mirroring dbfv/eval.rs:223-313.
"""

import hashlib
import json
import os
import random

import numpy as np
import pytest

from oracle import bfv as obfv, dbfv as odbfv, params as P, cref
from exacto_amd._ffi import HipContext, ExactoError
from bridge import ct_to_np, cts_to_np, np_to_ct, np_to_rlk, rlk_to_np, uniform_residues

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _meta():
    with open(os.path.join(GOLD, "vectors_meta.json")) as f:
        return json.load(f)


def _ctx(m):
    aux = [int(x) for x in m["aux_moduli"]]
    return HipContext(m["n"], [int(x) for x in m["ct_moduli"]], aux, m["plain"], m["gadget_base"])


@pytest.mark.parametrize("name", [k for k, v in _meta().items() if "d" not in v])
def test_bfv_vectors(gpu_available, name):
    m = _meta()[name]
    z = np.load(os.path.join(GOLD, "vectors.npz"))
    ctx = _ctx(m)
    ctx.load_relin_key(z[f"{name}__rlk"])
    ct1, ct2 = z[f"{name}__ct1"], z[f"{name}__ct2"]
    assert np.array_equal(ctx.bfv_mul_and_relin(ct1, ct2), z[f"{name}__out"])
    assert np.array_equal(ctx.bfv_mul_no_relin(ct1, ct2), z[f"{name}__out3"])
    assert np.array_equal(ctx.relinearize(z[f"{name}__out3"]), z[f"{name}__out"])


@pytest.mark.parametrize("name", [k for k, v in _meta().items() if "d" in v])
def test_dbfv_vectors(gpu_available, name):
    m = _meta()[name]
    z = np.load(os.path.join(GOLD, "vectors.npz"))
    ctx = _ctx(m)
    ctx.load_relin_key(z[f"{name}__rlk"])
    out, depth = ctx.dbfv_mul(m["d"], m["base"], m["dbfv_plain"], z[f"{name}__a"], z[f"{name}__b"])
    assert np.array_equal(out, z[f"{name}__out"])
    assert (depth == 1).all()


def test_cfg3_full_size_digest(gpu_available):
    with open(os.path.join(GOLD, "digests.json")) as f:
        spec = json.load(f)["cfg3_full"]
    prm = P.cfg3_params(spec["n"])
    rng = np.random.default_rng(spec["seed"])
    q, n = prm.ct_basis.moduli, prm.ring_degree
    ct1 = uniform_residues(rng, (spec["batch"], 2), q, n)
    ct2 = uniform_residues(rng, (spec["batch"], 2), q, n)
    rlk = uniform_residues(rng, (prm.gadget_digits, 2), q, n)
    sha = lambda a: hashlib.sha256(np.ascontiguousarray(a, dtype=np.uint64).tobytes()).hexdigest()
    assert sha(np.concatenate([ct1.ravel(), ct2.ravel(), rlk.ravel()])) == spec["sha256_inputs"]
    ctx = HipContext.from_params(prm)
    ctx.load_relin_key(rlk)
    assert sha(ctx.bfv_mul_and_relin(ct1, ct2)) == spec["sha256_out"]


def test_cfg3_batch_properties(gpu_available):
    """Batch of 300 at full size: chunk-size invariance, position invariance, sampled oracle rows."""
    import torch
    prm = P.cfg3_params(4096)
    q, n, L = prm.ct_basis.moduli, 4096, 3
    B = 300
    rng = np.random.default_rng(77)
    ct1 = uniform_residues(rng, (B, 2), q, n)
    ct2 = uniform_residues(rng, (B, 2), q, n)
    ct2[123] = ct2[5]
    ct1[123] = ct1[5]  # duplicated pair at another position (and another chunk)
    rlk = uniform_residues(rng, (prm.gadget_digits, 2), q, n)
    ctx = HipContext.from_params(prm)
    stream = torch.cuda.current_stream()
    ctx.set_stream(stream.cuda_stream)
    ctx.load_relin_key(rlk)
    d1 = torch.from_numpy(ct1.view(np.int64)).cuda()
    d2 = torch.from_numpy(ct2.view(np.int64)).cuda()
    outs = []
    for chunk in (128, 37, 300):
        ctx.set_chunk(chunk)
        o = torch.empty_like(d1)
        ctx.bfv_mul_and_relin_dev(d1, d2, o, B)
        ctx.synchronize()
        outs.append(o.cpu().numpy().view(np.uint64))
    assert np.array_equal(outs[0], outs[1]) and np.array_equal(outs[0], outs[2])
    assert np.array_equal(outs[0][123], outs[0][5])
    # mul_no_relin + relinearize == fused
    o3 = torch.empty((B, 3, L, n), dtype=torch.int64, device="cuda")
    ctx.bfv_mul_no_relin_dev(d1, d2, o3, B)
    o2 = torch.empty_like(d1)
    ctx.relinearize_dev(o3, 3, o2, B)
    ctx.synchronize()
    assert np.array_equal(o2.cpu().numpy().view(np.uint64), outs[0])
    if cref.available():
        rows = [0, 127, 128, 299]
        want = cref.bfv_mul_and_relin(prm, ct1[rows], ct2[rows], rlk, threads=4)
        assert np.array_equal(outs[0][rows], want)


def test_cfg4_full_size_dbfv(gpu_available):
    """BASELINE configs[3]: dBFV p=2^16, b=256, d=2 over n=4096 / 3x60-bit (t=260111)."""
    dp = P.cfg4_params(4096)
    prm = dp.bfv_params
    q, n, d = prm.ct_basis.moduli, 4096, 2
    B = 3
    rng = np.random.default_rng(404)
    a = uniform_residues(rng, (B, d, 2), q, n)
    b = uniform_residues(rng, (B, d, 2), q, n)
    rlk = uniform_residues(rng, (prm.gadget_digits, 2), q, n)
    ctx = HipContext.from_params(prm)
    ctx.load_relin_key(rlk)
    out, _ = ctx.dbfv_mul(d, dp.base, dp.plain_modulus, a, b)
    if not cref.available():
        pytest.skip("oracle/c not built")
    # oracle: limb0 = a0*b0, limb1 = a0*b1 + a1*b0 (reps all zero at p = b^d), via the C restatement
    i = 1
    p00 = cref.bfv_mul_and_relin(prm, a[i:i + 1, 0], b[i:i + 1, 0], rlk, threads=4)[0]
    p01 = cref.bfv_mul_and_relin(prm, a[i:i + 1, 0], b[i:i + 1, 1], rlk, threads=4)[0]
    p10 = cref.bfv_mul_and_relin(prm, a[i:i + 1, 1], b[i:i + 1, 0], rlk, threads=4)[0]
    Q = np.array(q, dtype=object)[None, :, None]
    assert np.array_equal(out[i, 0], p00)
    assert np.array_equal(out[i, 1].astype(object), (p01.astype(object) + p10.astype(object)) % Q)


def test_dbfv_depth_guard_and_errors(gpu_available):
    dp = P.compact_dbfv()
    prm = dp.bfv_params
    ctx = HipContext.from_params(prm)
    rng = np.random.default_rng(0)
    a = uniform_residues(rng, (2, 2, 2), prm.ct_basis.moduli, 1024)
    ctx.load_relin_key(uniform_residues(rng, (prm.gadget_digits, 2), prm.ct_basis.moduli, 1024))
    with pytest.raises(ExactoError) as e:
        ctx.dbfv_mul(2, 16, 256, a, a, depth_a=[1, 0], depth_b=[0, 0])
    assert e.value.variant == "NotImplemented"
    assert "chained dBFV multiplication requires ciphertext-level lattice reduction" in str(e.value)
    with pytest.raises(ExactoError) as e:
        ctx.dbfv_mul(2, 15, 256, a, a)
    assert "base^digits = 225 < plain_modulus = 256" in str(e.value)


def test_dbfv_nonzero_reps(gpu_available):
    """p not a power of b: degree reduction folds limbs with nonzero small representatives."""
    prm = P.BfvParamsBuilder().ring_degree(32).plain_modulus(12289).ct_moduli(P.Q3).build()
    dp = P.DbfvParams(prm, 7, 4, 1000)
    assert odbfv.needed_pairs(dp) != [(i, j) for i in range(4) for j in range(4) if i + j < 4]
    rng = np.random.default_rng(12)
    q = prm.ct_basis.moduli
    a = uniform_residues(rng, (1, 4, 2), q, 32)
    b = uniform_residues(rng, (1, 4, 2), q, 32)
    rlk = uniform_residues(rng, (prm.gadget_digits, 2), q, 32)
    ctx = HipContext.from_params(prm)
    ctx.load_relin_key(rlk)
    out, _ = ctx.dbfv_mul(4, 7, 1000, a, b)
    A = odbfv.DbfvCiphertext([np_to_ct(a[0, k], prm) for k in range(4)], 4, 0, dp)
    Bc = odbfv.DbfvCiphertext([np_to_ct(b[0, k], prm) for k in range(4)], 4, 0, dp)
    want = odbfv.dbfv_mul(A, Bc, np_to_rlk(rlk, prm))
    assert np.array_equal(out[0], np.stack([ct_to_np(l) for l in want.limbs]))


def test_dbfv_decrypt_level(gpu_available):
    """dbfv/eval.rs:223-290 on the GPU path: 3*7, carries over b = 16."""
    dp = P.compact_dbfv()
    prm = dp.bfv_params
    rng = random.Random(42)
    sk = obfv.gen_secret_key(prm, rng)
    rlk = obfv.gen_relin_key(sk, rng)
    ctx = HipContext.from_params(prm)
    ctx.load_relin_key(rlk_to_np(rlk))
    for x, y in [(3, 7), (15, 15), (10, 20), (12, 12)]:
        ca = odbfv.dbfv_encrypt_scalar_sk(x, sk, dp, rng)
        cb = odbfv.dbfv_encrypt_scalar_sk(y, sk, dp, rng)
        A = np.stack([ct_to_np(l) for l in ca.limbs])[None]
        B = np.stack([ct_to_np(l) for l in cb.limbs])[None]
        out, _ = ctx.dbfv_mul(2, 16, 256, A, B)
        r = odbfv.DbfvCiphertext([np_to_ct(out[0, k], prm) for k in range(2)], 2, 1, dp)
        assert odbfv.dbfv_decrypt_scalar(r, sk) == (x * y) % 256


def test_cfg5_full_size(gpu_available):
    """BASELINE configs[4] at full size: n=8192, 4x60-bit limbs, gadget 256 (G=30), t=1040407, d=8.
    bfv_mul_and_relin bit-exact vs the C restatement on one row; one dbfv_mul's output limbs equal
    the sums of the GPU's own (oracle-checked) BFV products; a depth-2 chain equals two dbfv_mul."""
    dp = P.cfg5_params(8192)
    prm = dp.bfv_params
    q, n, d = prm.ct_basis.moduli, 8192, dp.num_digits
    rng = np.random.default_rng(505)
    rlk = uniform_residues(rng, (prm.gadget_digits, 2), q, n)
    ctx = HipContext.from_params(prm)
    ctx.load_relin_key(rlk)
    ct1 = uniform_residues(rng, (2, 2), q, n)
    ct2 = uniform_residues(rng, (2, 2), q, n)
    got = ctx.bfv_mul_and_relin(ct1, ct2)
    if cref.available():
        assert np.array_equal(got[1], cref.bfv_mul_and_relin(prm, ct1[1:], ct2[1:], rlk, threads=1)[0])
    a = uniform_residues(rng, (1, d, 2), q, n)
    b = uniform_residues(rng, (1, d, 2), q, n)
    out, _ = ctx.dbfv_mul(d, dp.base, dp.plain_modulus, a, b)
    Q = np.array(q, dtype=object)[:, None]
    for k in (0, 1, 7):  # p = 2^64 = b^d: every reduction rep is zero, limb k = sum_{i+j=k} a_i b_j
        prods = ctx.bfv_mul_and_relin(a[0, :k + 1], b[0, k::-1])
        want = (prods.astype(object).sum(axis=0) % Q)
        assert np.array_equal(out[0, k].astype(object), want), k
    chain = ctx.dbfv_mul_chain(d, dp.base, dp.plain_modulus, a, b, 2)
    step2, _ = ctx.dbfv_mul(d, dp.base, dp.plain_modulus, out, b)
    assert np.array_equal(chain, step2)


def _dbfv_digest_case(name, fill_to):
    """The pinned items of a full-size dBFV digest, padded with other random items to the production
    batch (psum, int8 / int16 digit sums, two-lane halves: all library defaults)."""
    import sys
    sys.path.insert(0, GOLD)
    from make_golden import dbfv_digest_inputs
    with open(os.path.join(GOLD, "digests.json")) as f:
        spec = json.load(f)[name]
    dp, a, b, rlk = dbfv_digest_inputs(spec)
    sha = lambda x: hashlib.sha256(np.ascontiguousarray(x, dtype=np.uint64).tobytes()).hexdigest()
    assert sha(np.concatenate([a.ravel(), b.ravel(), rlk.ravel()])) == spec["sha256_inputs"]
    k = a.shape[0]
    if fill_to > k:
        rng = np.random.default_rng(99)
        q, n, d = dp.bfv_params.ct_basis.moduli, spec["n"], dp.num_digits
        a = np.concatenate([a, uniform_residues(rng, (fill_to - k, d, 2), q, n)])
        b = np.concatenate([b, uniform_residues(rng, (fill_to - k, d, 2), q, n)])
    ctx = HipContext.from_params(dp.bfv_params)
    ctx.load_relin_key(rlk)
    return spec, dp, ctx, a, b, k, sha


def test_cfg4_full_size_dbfv_digest(gpu_available):
    """BASELINE configs[3] at full size: 4 pinned dbfv_mul items in a batch of 64 (192 products: two
    pipeline lanes, psum, wide-basis digit sums) against the C restatement's digest."""
    spec, dp, ctx, a, b, k, sha = _dbfv_digest_case("cfg4_full", 64)
    assert ctx.psum_max >= 2
    out, _ = ctx.dbfv_mul(dp.num_digits, dp.base, dp.plain_modulus, a, b)
    assert sha(out[:k]) == spec["sha256_out"]


def test_cfg5_full_size_dbfv_digest(gpu_available):
    """BASELINE configs[4] at full size (n = 8192, 4x60-bit, d = 8): one pinned dbfv_mul item in the
    bench's batch of 8 (288 products: two lanes of 144, psum, int8 digit sums)."""
    spec, dp, ctx, a, b, k, sha = _dbfv_digest_case("cfg5_full", 8)
    out, _ = ctx.dbfv_mul(dp.num_digits, dp.base, dp.plain_modulus, a, b)
    got = [sha(out[0, j]) for j in range(dp.num_digits)]
    assert got == spec["sha256_out_item0_limbs"], [j for j in range(len(got)) if got[j] != spec["sha256_out_item0_limbs"][j]]
    assert sha(out[:k]) == spec["sha256_out"]


def test_cfg5_full_size_chain_digest(gpu_available):
    """The bench's cfg5 workload itself: a depth-4 dbfv_mul chain (paper_repro.rs:203-236 guard-bypass
    semantics) of one pinned item in a batch of 8, against the C restatement's digest."""
    spec, dp, ctx, a, b, k, sha = _dbfv_digest_case("cfg5_chain4", 8)
    out = ctx.dbfv_mul_chain(dp.num_digits, dp.base, dp.plain_modulus, a, b, spec["depth"])
    assert sha(out[:k]) == spec["sha256_out"]
