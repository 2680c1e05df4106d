"""Key generation and encryption on the GPU: exacto_gen_{secret,public,relin}_key,
exacto_encrypt_{sk,pk}.

Reference: bfv/keygen.rs:64-162, bfv/encrypt.rs:29-106, 181-229, sampling/{uniform,gaussian}.rs.
The random stream is this library's own (ChaCha20 in counter mode; the reference's ChaCha20Rng
stream is not reproducible here and the hot path does not depend on it), so parity is checked
(1) exactly on the structure the reference's samplers give every polynomial (a CoeffPoly modulo
the first prime, reduced modulo each q_i), (2) statistically with the reference's own sampler
test bounds (sampling/gaussian.rs:60-82: |mean| < 0.5, |var - sigma^2| < 2, |x| <= ceil(6 sigma)),
and (3) at decryption level, with the GPU and the oracle decryptors, including products
relinearised with a GPU-generated key.
"""
import numpy as np
import pytest

from oracle import bfv as obfv, params as P
from oracle.ring import CoeffPoly
from exacto_amd._ffi import HipContext, ExactoError
from bridge import np_to_ct, np_to_rns

pytestmark = pytest.mark.gpu

KEY = [0x0123456789ABCDEF, 0xFEDCBA9876543210, 0x0F1E2D3C4B5A6978, 0x8796A5B4C3D2E1F0]


def coeffs(ctx, ntt_poly):
    """[L][n] NTT-domain residues -> [L][n] coefficients (GPU inverse NTT, parity-tested)."""
    out = np.empty_like(ntt_poly)
    for i in range(ntt_poly.shape[0]):
        out[i] = ctx.ntt_inv(ntt_poly[i][None, :].copy(), limb=i)[0]
    return out


def check_literal_rns(c, moduli):
    """Reference sampling semantics: limb i == (limb-0 value as an integer in [0, q0)) mod q_i."""
    for i in range(1, len(moduli)):
        assert np.array_equal(c[i], c[0] % np.uint64(moduli[i]))


def centred(v, q):
    v = v.astype(object)
    return np.array([int(x) - q if x > q // 2 else int(x) for x in v], dtype=np.int64)


def sk_obj(sk_np, prm):
    return obfv.SecretKey(np_to_rns(sk_np, prm.ct_basis), prm, None)


@pytest.mark.parametrize("which", ["compact", "cfg3_n1024"])
def test_samplers_follow_reference_semantics(gpu_available, which):
    prm = {"compact": P.compact_bfv, "cfg3_n1024": lambda: P.cfg3_params(1024)}[which]()
    ctx = HipContext.from_params(prm)
    q = prm.ct_basis.moduli
    n = prm.ring_degree
    sk = ctx.gen_secret_key(KEY, stream=1)
    s = coeffs(ctx, sk)
    check_literal_rns(s, q)
    vals, counts = np.unique(s[0], return_counts=True)
    assert set(int(v) for v in vals) <= {0, 1, q[0] - 1}
    assert all(abs(c - n / 3) < 5 * np.sqrt(n * 2 / 9) for c in counts) and len(counts) == 3
    # relinearisation key: rlk0_i + a_i s - base^i s^2 = -e_i, a_i uniform mod q0
    rlk = ctx.gen_relin_key(sk, KEY, stream=2)
    assert rlk.shape == (prm.gadget_digits, 2, len(q), n)
    skp = np_to_rns(sk, prm.ct_basis)
    s2 = skp.mul(skp)
    errs = []
    for g in range(prm.gadget_digits):
        a = coeffs(ctx, rlk[g, 1])
        check_literal_rns(a, q)
        assert (a[0] < np.uint64(q[0])).all()
        gi = s2.scalar_mul(pow(prm.gadget_base, g))
        neg_e = np_to_rns(rlk[g, 0], prm.ct_basis).add(np_to_rns(rlk[g, 1], prm.ct_basis).mul(skp)).sub(gi)
        ne = coeffs(ctx, np.array([c.evals for c in neg_e.components], dtype=np.uint64))
        e = np.stack([(np.uint64(qi) - ne[i]) % np.uint64(qi) for i, qi in enumerate(q)])
        check_literal_rns(e, q)
        errs.append(centred(e[0], q[0]))
    x = np.concatenate(errs).astype(np.float64)
    assert abs(x.mean()) < 0.5
    assert abs(x.var() - 3.2 ** 2) < 2.0
    assert np.abs(x).max() <= int(np.ceil(6 * 3.2))
    # uniform: mean of a's limb-0 coefficients ~ q0/2
    a_all = np.concatenate([coeffs(ctx, rlk[g, 1])[0] for g in range(prm.gadget_digits)]).astype(np.float64)
    assert abs(a_all.mean() / q[0] - 0.5) < 0.02


def test_determinism_and_streams(gpu_available):
    prm = P.compact_bfv()
    ctx = HipContext.from_params(prm)
    a = ctx.gen_secret_key(KEY, stream=5)
    assert np.array_equal(a, ctx.gen_secret_key(KEY, stream=5))
    assert not np.array_equal(a, ctx.gen_secret_key(KEY, stream=6))
    k2 = list(KEY)
    k2[3] ^= 1
    assert not np.array_equal(a, ctx.gen_secret_key(k2, stream=5))


@pytest.mark.parametrize("which", ["compact", "small", "cfg3_n1024", "cfg3"])
def test_encrypt_decrypt(gpu_available, which):
    prm = {"compact": P.compact_bfv, "small": P.small_bfv, "cfg3_n1024": lambda: P.cfg3_params(1024),
           "cfg3": P.cfg3_params}[which]()
    ctx = HipContext.from_params(prm)
    n, p = prm.ring_degree, prm.plain_modulus
    sk = ctx.gen_secret_key(KEY, stream=11)
    pk = ctx.gen_public_key(sk, KEY, stream=12)
    rng = np.random.default_rng(4)
    pt = rng.integers(0, p, size=(4, n), dtype=np.uint64)
    ct_sk = ctx.encrypt_sk(pt, sk, KEY, stream=13)
    ct_pk = ctx.encrypt_pk(pt, pk, KEY, stream=14)
    for ct in (ct_sk, ct_pk):
        assert np.array_equal(ctx.bfv_decrypt(ct, sk), pt)
        for b in (0, 3):  # the oracle's decryptor agrees (encrypt.rs:111-178)
            assert obfv.decrypt(np_to_ct(ct[b], prm), sk_obj(sk, prm)).coeffs == [int(v) for v in pt[b]]
    # c1 of a secret-key encryption is the uniform a: reference sampling semantics
    check_literal_rns(coeffs(ctx, ct_sk[0, 1]), prm.ct_basis.moduli)


@pytest.mark.parametrize("which", ["compact", "cfg3_n1024"])
def test_products_with_gpu_generated_relin_key(gpu_available, which):
    prm = {"compact": P.compact_bfv, "cfg3_n1024": lambda: P.cfg3_params(1024)}[which]()
    ctx = HipContext.from_params(prm)
    n, p = prm.ring_degree, prm.plain_modulus
    sk = ctx.gen_secret_key(KEY, stream=21)
    ctx.gen_relin_key(sk, KEY, stream=22, resident=True)   # straight into the resident key
    msgs = [(3, 7), (0, 5), (p - 1, 2), (12, 12)]
    pa = np.zeros((4, n), dtype=np.uint64)
    pb = np.zeros((4, n), dtype=np.uint64)
    for i, (a, b) in enumerate(msgs):
        pa[i, 0], pb[i, 0] = a, b
    ca = ctx.encrypt_sk(pa, sk, KEY, stream=23)
    cb = ctx.encrypt_sk(pb, sk, KEY, stream=24)
    prod = ctx.bfv_mul_and_relin(ca, cb)
    dec = ctx.bfv_decrypt(prod, sk)
    assert [int(d[0]) for d in dec] == [(a * b) % p for a, b in msgs]
    assert not dec[:, 1:].any()
    # the same key as an explicit buffer reproduces the resident one
    rlk = ctx.gen_relin_key(sk, KEY, stream=22)
    ctx2 = HipContext.from_params(prm)
    ctx2.load_relin_key(rlk)
    assert np.array_equal(ctx2.bfv_mul_and_relin(ca, cb), prod)


def test_errors(gpu_available):
    prm = P.compact_bfv()
    ctx = HipContext.from_params(prm)
    sk = ctx.gen_secret_key(KEY)
    with pytest.raises(ExactoError) as e:
        ctx.encrypt_sk(np.zeros((1, prm.ring_degree), dtype=np.uint64), sk, KEY, sigma=-1.0)
    assert e.value.variant == "InvalidParam"
    with pytest.raises(ValueError):
        ctx.gen_secret_key([1, 2, 3])


def test_resident_relin_key_under_boot_debug(gpu_available):
    """exacto_gen_relin_key with rlk = NULL (straight into the resident key) under EXACTO_DEBUG_BOOT=1:
    the host-call debug print once dereferenced the NULL host output (fixed in 355108a).  The switch
    is read once per process, so the call runs in a child process."""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    code = (
        "import sys; sys.path[:0] = [%r, %r]\n"
        "import torch; torch.cuda.init()\n"
        "import numpy as np\n"
        "from oracle import params as P\n"
        "from exacto_amd._ffi import HipContext\n"
        "prm = P.compact_bfv(); ctx = HipContext.from_params(prm)\n"
        "K = %r\n"
        "sk = ctx.gen_secret_key(K, stream=31)\n"
        "ctx.gen_relin_key(sk, K, stream=32, resident=True)\n"
        "pa = np.zeros((1, 1024), dtype=np.uint64); pa[0, 0] = 6\n"
        "ca = ctx.encrypt_sk(pa, sk, K, stream=33)\n"
        "d = ctx.bfv_decrypt(ctx.bfv_mul_and_relin(ca, ca), sk)\n"
        "assert int(d[0, 0]) == 36, d[0, :4]\n"
        "print('ok')\n" % (os.path.dirname(here), here, KEY))
    env = dict(os.environ, EXACTO_DEBUG_BOOT="1")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]
