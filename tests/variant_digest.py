"""Digests of the hot path's outputs under the kernel / path selection switches of this process's
environment (run as a child process by tests/test_gpu_variants.py: each switch is read once per
process).  Prints one JSON object {case: sha256}.  argv: the case groups to run (default: all).

Case groups:
  cfg3    bfv_mul_and_relin, n = 4096, 3 limbs (forward, inverse, tensor, ks32 key switch), 160
          products in pipeline chunks of 64 (three chunks: both lanes, or three with EXACTO_LANES=3)
  cfg4    dbfv_mul d = 2 (n = 4096, 3 limbs: psum, the wide 31-bit basis for int32 digit sums)
  cfg5    dbfv_mul and a depth-2 chain of 3 items (n = 8192, 4 limbs: psum, the n = 8192 tensor kernels,
          the chain split over two streams)
  hps     compact_bfv products (one aux prime) and a u64_dbfv dbfv_mul (two aux primes, digit sums)
  polymul the fused NTT product at n = 4096 / 8192, out of place and in place on b
"""

import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)

from bridge import uniform_residues  # noqa: E402
from oracle import params as P  # noqa: E402
from exacto_amd._ffi import HipContext  # noqa: E402

GROUPS = ("cfg3", "cfg4", "cfg5", "hps", "polymul")


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.uint64).tobytes()).hexdigest()


def cfg3(out):
    prm = P.cfg3_params(4096)
    q, n = prm.ct_basis.moduli, 4096
    rng = np.random.default_rng(7001)
    ct1 = uniform_residues(rng, (160, 2), q, n)
    ct2 = uniform_residues(rng, (160, 2), q, n)
    rlk = uniform_residues(rng, (prm.gadget_digits, 2), q, n)
    ctx = HipContext.from_params(prm)
    ctx.set_chunk(64)
    ctx.load_relin_key(rlk)
    out["cfg3_mul_relin"] = sha(ctx.bfv_mul_and_relin(ct1, ct2))


def cfg4(out):
    dp = P.cfg4_params(4096)
    prm = dp.bfv_params
    q, d = prm.ct_basis.moduli, dp.num_digits
    rng = np.random.default_rng(7006)
    a = uniform_residues(rng, (3, d, 2), q, 4096)
    b = uniform_residues(rng, (3, d, 2), q, 4096)
    rlk = uniform_residues(rng, (prm.gadget_digits, 2), q, 4096)
    ctx = HipContext.from_params(prm)
    ctx.load_relin_key(rlk)
    out["cfg4_dbfv_mul"] = sha(ctx.dbfv_mul(d, dp.base, dp.plain_modulus, a, b)[0])


def cfg5(out):
    dp = P.cfg5_params(8192)
    prm5 = dp.bfv_params
    q5, d = prm5.ct_basis.moduli, dp.num_digits
    rng = np.random.default_rng(7002)
    # three items: the chain batch splits 2 + 1 over the context and its twin (EXACTO_CHAIN_SPLIT)
    a = uniform_residues(rng, (3, d, 2), q5, 8192)
    b = uniform_residues(rng, (3, d, 2), q5, 8192)
    rlk5 = uniform_residues(rng, (prm5.gadget_digits, 2), q5, 8192)
    ctx5 = HipContext.from_params(prm5)
    ctx5.load_relin_key(rlk5)
    out["cfg5_dbfv_mul"] = sha(ctx5.dbfv_mul(d, dp.base, dp.plain_modulus, a, b)[0])
    out["cfg5_chain2"] = sha(ctx5.dbfv_mul_chain(d, dp.base, dp.plain_modulus, a, b, 2))


def hps(out):
    cb = P.compact_bfv()
    rng = np.random.default_rng(7004)
    qc = cb.ct_basis.moduli
    h1 = uniform_residues(rng, (8, 2), qc, 1024)
    h2 = uniform_residues(rng, (8, 2), qc, 1024)
    hk = uniform_residues(rng, (cb.gadget_digits, 2), qc, 1024)
    hc = HipContext.from_params(cb)
    hc.load_relin_key(hk)
    out["compact_mul_relin"] = sha(hc.bfv_mul_and_relin(h1, h2))
    out["compact_mul_no_relin"] = sha(hc.bfv_mul_no_relin(h1, h2))
    du = P.u64_dbfv()
    pu = du.bfv_params
    rng = np.random.default_rng(7005)
    qu = pu.ct_basis.moduli
    ua = uniform_residues(rng, (2, du.num_digits, 2), qu, 4096)
    ub = uniform_residues(rng, (2, du.num_digits, 2), qu, 4096)
    uk = uniform_residues(rng, (pu.gadget_digits, 2), qu, 4096)
    uc = HipContext.from_params(pu)
    uc.load_relin_key(uk)
    out["u64dbfv_dbfv_mul"] = sha(uc.dbfv_mul(du.num_digits, du.base, du.plain_modulus, ua, ub)[0])


def polymul(out):
    import torch
    for nn, qs in ((4096, [1152921504606830593]), (8192, [1152921504606830593, 1152921504606748673])):
        rng = np.random.default_rng(7003 + nn)
        c = HipContext(nn, qs, plain_modulus=257)
        qa = np.array(qs, dtype=np.uint64)[None, :, None]
        x = (rng.integers(0, 1 << 63, size=(4, len(qs), nn), dtype=np.uint64) % qa).astype(np.uint64)
        y = (rng.integers(0, 1 << 63, size=(4, len(qs), nn), dtype=np.uint64) % qa).astype(np.uint64)
        dx = torch.from_numpy(x.view(np.int64)).cuda()
        dy = torch.from_numpy(y.view(np.int64)).cuda()
        o = torch.empty_like(dx)
        c.rns_polymul_dev(dx, dy, o, 4)
        c.rns_polymul_dev(dx, dy, dy, 4)   # in place on b
        c.synchronize()
        out[f"polymul_{nn}"] = sha(o.cpu().numpy().view(np.uint64))
        out[f"polymul_{nn}_inplace"] = sha(dy.cpu().numpy().view(np.uint64))


def main():
    # torch's HIP runtime first, as in the pytest parent and the bench: both the library and torch's
    # bundled libamdhip64 carry the soname libamdhip64.so.7, and the process keeps whichever loads
    # first (with the library first, torch.cuda found no GPU on a round-4 box)
    import torch
    torch.cuda.init()
    out = {}
    for g in (sys.argv[1:] or GROUPS):
        globals()[g](out)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
