"""GPU parity of bfv_mul_no_relin / relinearize / bfv_mul_and_relin against the oracle.

Bit-exact on the same inputs (uniform random residues and genuine encryptions), for
every dispatch branch of eval.rs:89-108:
  * exact multi-limb path (eval.rs:113-147) — cfg3's 3x60-bit basis at small n and n=4096,
    plus the reference's own multi-prime Q < 2^64 parameters (eval.rs:903-927);
  * literal HPS, one aux prime (compact_bfv, presets.rs:24-35) and two (u64_dbfv basis);
  * schoolbook (no aux, single q) and its overflow guard.
"""

import random

import numpy as np
import pytest

from oracle import bfv as obfv
from oracle import params as P
from exacto_amd._ffi import HipContext, ExactoError, PATH_EXACT_RNS, PATH_HPS, PATH_SCHOOLBOOK
from bridge import ct_to_np, cts_to_np, np_to_ct, np_to_rlk, rlk_to_np, uniform_residues

pytestmark = pytest.mark.gpu


def random_case(params, B, seed, num_keys=None):
    rng = np.random.default_rng(seed)
    q = params.ct_basis.moduli
    n = params.ring_degree
    ct1 = uniform_residues(rng, (B, 2), q, n)
    ct2 = uniform_residues(rng, (B, 2), q, n)
    G = params.gadget_digits if num_keys is None else num_keys
    rlk = uniform_residues(rng, (G, 2), q, n)
    return ct1, ct2, rlk


def oracle_mul(params, ct1, ct2, rlk_np, relin=True):
    rlk = np_to_rlk(rlk_np, params)
    outs = []
    for b in range(ct1.shape[0]):
        c1, c2 = np_to_ct(ct1[b], params), np_to_ct(ct2[b], params)
        r = obfv.bfv_mul_and_relin(c1, c2, rlk) if relin else obfv.bfv_mul_no_relin(c1, c2)
        outs.append(ct_to_np(r))
    return np.stack(outs)


def run_case(params, B, seed, num_keys=None, check_no_relin=True):
    ctx = HipContext.from_params(params)
    ct1, ct2, rlk = random_case(params, B, seed, num_keys)
    ctx.load_relin_key(rlk)
    got = ctx.bfv_mul_and_relin(ct1, ct2)
    want = oracle_mul(params, ct1, ct2, rlk)
    assert np.array_equal(got, want)
    if check_no_relin:
        got3 = ctx.bfv_mul_no_relin(ct1, ct2)
        assert np.array_equal(got3, oracle_mul(params, ct1, ct2, rlk, relin=False))
        assert np.array_equal(ctx.relinearize(got3), got)
    return ctx


def test_exact_multiprime_small_q(gpu_available):
    # eval.rs:903-927 parameters: Q = 65537 * 1099509805057 < 2^64, base 8
    prm = (P.BfvParamsBuilder().ring_degree(16).plain_modulus(257)
           .ct_moduli([65537, 1099509805057]).sigma(3.2).gadget_base(8).build())
    ctx = run_case(prm, 4, 1)
    assert ctx.path == PATH_EXACT_RNS


@pytest.mark.parametrize("n", [16, 256, 1024])
def test_exact_cfg3_basis_small_n(gpu_available, n):
    run_case(P.cfg3_params(n), 2, 10 + n)


def test_exact_cfg3_full_size(gpu_available):
    """BASELINE configs[2] at full size: n=4096, 3x60-bit limbs, base 2^16 (G=12)."""
    run_case(P.cfg3_params(4096), 1, 33, check_no_relin=False)


def test_exact_cfg5_basis(gpu_available):
    """u64 profile basis (4x60-bit, gadget 256 -> G=30), t=1040407, at reduced n."""
    prm = (P.BfvParamsBuilder().ring_degree(64).plain_modulus(1040407).ct_moduli(P.Q4)
           .gadget_base(256).build())
    run_case(prm, 2, 55)


def test_hps_one_aux_compact(gpu_available):
    ctx = run_case(P.compact_bfv(), 2, 3)
    assert ctx.path == PATH_HPS


def test_hps_two_aux(gpu_available):
    prm = P.u64_dbfv().bfv_params
    run_case(prm, 1, 4, check_no_relin=False)


def test_hps_two_aux_small_n(gpu_available):
    prm = (P.BfvParamsBuilder().ring_degree(256).plain_modulus(1040407)
           .ct_moduli([1152921504606830593]).aux_moduli([18014398509998081, 36028797018972161])
           .gadget_base(256).build())
    run_case(prm, 3, 44)


def test_schoolbook_path(gpu_available):
    prm = (P.BfvParamsBuilder().ring_degree(16).plain_modulus(17).ct_moduli([65537])
           .gadget_base(4).build())
    ctx = run_case(prm, 3, 6)
    assert ctx.path == PATH_SCHOOLBOOK


def _guard_case(aux):
    # dbfv/eval.rs:385-453 parameters: n=4096, t=1040407, q=18014398509506561, base 256
    q = 18014398509506561
    ctx = HipContext(4096, [q], aux, 1040407, 256)
    rng = np.random.default_rng(101)
    ct = uniform_residues(rng, (1, 2), [q], 4096)
    ctx.load_relin_key(uniform_residues(rng, (ctx.G, 2), [q], 4096))
    with pytest.raises(ExactoError) as e:
        ctx.bfv_mul_and_relin(ct, ct)
    return e.value


def test_schoolbook_overflow_guard(gpu_available):
    err = _guard_case([])
    assert err.variant == "NotImplemented"
    assert "schoolbook BFV multiplication can overflow i128" in str(err)


def test_hps_single_aux_too_small(gpu_available):
    err = _guard_case([36028797018972161])
    assert err.variant == "InvalidParam"
    assert "single aux prime too small" in str(err)


def test_relin_key_truncation(gpu_available):
    # keyswitch.rs:86-89: only min(G, rlk.len) digits are used
    prm = P.cfg3_params(64)
    run_case(prm, 2, 77, num_keys=5)
    run_case(prm, 1, 78, num_keys=0, check_no_relin=False)


def test_degree_errors(gpu_available):
    prm = P.cfg3_params(16)
    ctx = HipContext.from_params(prm)
    rng = np.random.default_rng(0)
    ct3 = uniform_residues(rng, (1, 3), prm.ct_basis.moduli, 16)
    ctx.load_relin_key(uniform_residues(rng, (prm.gadget_digits, 2), prm.ct_basis.moduli, 16))
    with pytest.raises(ExactoError) as e:
        ctx.bfv_mul_no_relin(ct3, ct3)
    assert "multiplication requires degree-1 ciphertexts" in str(e.value)
    ct4 = uniform_residues(rng, (1, 4), prm.ct_basis.moduli, 16)
    with pytest.raises(ExactoError) as e:
        ctx.relinearize(ct4)
    assert "relinearization only supports degree-2 ciphertexts" in str(e.value)
    ct2 = uniform_residues(rng, (2, 2), prm.ct_basis.moduli, 16)
    assert np.array_equal(ctx.relinearize(ct2), ct2)
    # keyswitch.rs:63-65 clones a ciphertext of fewer than 3 polys: one-poly items, batched,
    # keep their own layout ([B][1][L][n]), on the host and the device entry points
    ct1 = uniform_residues(rng, (3, 1), prm.ct_basis.moduli, 16)
    assert np.array_equal(ctx.relinearize(ct1), ct1)
    import torch
    d_in = torch.from_numpy(ct1.view(np.int64)).cuda()
    d_out = torch.full((3 + 2, 1, prm.ct_basis.num_moduli(), 16), -1, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()  # the context's stream does not wait for torch's
    ctx.relinearize_dev(d_in, 1, d_out, 3)
    ctx.synchronize()
    got = d_out.cpu().numpy()
    assert np.array_equal(got[:3].view(np.uint64), ct1)
    assert (got[3:] == -1).all()  # nothing written past the B*1*L*n output words


def test_missing_key(gpu_available):
    prm = P.cfg3_params(16)
    ctx = HipContext.from_params(prm)
    rng = np.random.default_rng(0)
    ct = uniform_residues(rng, (1, 2), prm.ct_basis.moduli, 16)
    with pytest.raises(ExactoError) as e:
        ctx.bfv_mul_and_relin(ct, ct)
    assert e.value.variant == "MissingKey"


@pytest.mark.parametrize("which", ["compact", "multi"])
def test_decrypt_level(gpu_available, which):
    """Functional tests mirroring eval.rs:883-927 (3*7 = 21; multi-prime products)."""
    if which == "compact":
        prm = P.compact_bfv()
        cases = [(3, 7)]
    else:
        prm = (P.BfvParamsBuilder().ring_degree(16).plain_modulus(257)
               .ct_moduli([65537, 1099509805057]).sigma(3.2).gadget_base(8).build())
        cases = [(3, 7), (10, 20), (0, 5)]
    rng = random.Random(42)
    sk = obfv.gen_secret_key(prm, rng)
    rlk = obfv.gen_relin_key(sk, rng)
    ctx = HipContext.from_params(prm)
    ctx.load_relin_key(rlk_to_np(rlk))
    for a, b in cases:
        c1 = obfv.encrypt_sk(obfv.encode_scalar(a, prm), sk, rng)
        c2 = obfv.encrypt_sk(obfv.encode_scalar(b, prm), sk, rng)
        got = ctx.bfv_mul_and_relin(cts_to_np([c1]), cts_to_np([c2]))[0]
        assert np.array_equal(got, ct_to_np(obfv.bfv_mul_and_relin(c1, c2, rlk)))
        dec = obfv.decrypt(np_to_ct(got, prm), sk)
        assert obfv.decode_scalar(dec) == (a * b) % prm.plain_modulus


def test_exact_path_with_62bit_primes(gpu_available):
    """Primes >= 2^60 take the non-lazy forward NTT; results must not change."""
    prm = (P.BfvParamsBuilder().ring_degree(64).plain_modulus(65537)
           .ct_moduli([4611686018427322369, 2305843009213554689]).build())
    run_case(prm, 2, 91)
