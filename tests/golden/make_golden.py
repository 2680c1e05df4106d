#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/.

1. kats.json — the reference's own known-answer tests for this path.  Every entry cites the
   reference test (path:line) whose assertion it transcribes; expected values are the literal
   numbers of those assertions, or the plain-integer expression the assertion itself states
   (e.g. modular.rs:135 asserts barrett_reduce(123456789) == 123456789 % m).  No reference code
   is executed (it is Rust and cannot be built here).
2. vectors.npz — seeded inputs and oracle outputs (Python restatement, cross-checked with the
   C restatement) for every dispatch branch at small sizes, plus dBFV cases.
3. digests.json — SHA-256 of the C-oracle output for full-size cfg3 (n=4096, 3x60-bit) on
   seeded inputs; the GPU tests regenerate the inputs and compare digests.

   --dbfv-digests adds full-size cfg4 / cfg5 dbfv_mul and cfg5 depth-4 chain digests of the C
   restatement of dbfv_mul (all d^2 products, sums, reduce).

Run: python tests/golden/make_golden.py   (takes ~1 minute)
     python tests/golden/make_golden.py --dbfv-digests   (~10 minutes on 8 cores)
     python tests/golden/make_golden.py --worst-digests  (~5 minutes: tests/worstcase.py inputs at cfg5)
"""

import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

from oracle import bfv as obfv, dbfv as odbfv, params as P  # noqa: E402
from bridge import ct_to_np, np_to_ct, np_to_rlk, uniform_residues  # noqa: E402

M = 65537


def kats():
    k = []

    def add(src, fn, args, expected):
        k.append({"source": src, "fn": fn, "args": args, "expected": expected})

    # src/ring/modular.rs tests (m = 65537)
    add("src/ring/modular.rs:131", "barrett_reduce", [0, M], 0)
    add("src/ring/modular.rs:132", "barrett_reduce", [1, M], 1)
    add("src/ring/modular.rs:133", "barrett_reduce", [M, M], 0)
    add("src/ring/modular.rs:134", "barrett_reduce", [M + 1, M], 1)
    add("src/ring/modular.rs:135", "barrett_reduce", [123456789, M], 123456789 % M)
    add("src/ring/modular.rs:142", "mod_mul", [1234, 5678, M], (1234 * 5678) % M)
    add("src/ring/modular.rs:143", "mod_mul", [0, 5678, M], 0)
    add("src/ring/modular.rs:144", "mod_mul", [1, 5678, M], 5678)
    add("src/ring/modular.rs:150", "mod_add", [100, 200, M], 300)
    add("src/ring/modular.rs:151", "mod_add", [M - 1, 2, M], 1)
    add("src/ring/modular.rs:152", "mod_sub", [200, 100, M], 100)
    add("src/ring/modular.rs:153", "mod_sub", [100, 200, M], M - 100)
    add("src/ring/modular.rs:159", "mod_neg", [0, M], 0)
    add("src/ring/modular.rs:160", "mod_neg", [1, M], M - 1)
    add("src/ring/modular.rs:167", "mod_pow", [2, 10, M], 1024)
    add("src/ring/modular.rs:168", "mod_pow", [2, 16, M], 65536 % M)
    add("src/ring/modular.rs:169", "mod_pow", [3, 0, M], 1)
    add("src/ring/modular.rs:178", "mod_inv_times_a", [12345, M], 1)
    add("src/ring/modular.rs:188", "montgomery_check", [M], 0)
    add("src/ring/modular.rs:201", "montgomery_reduce_am", [12345, M], 0)
    # src/ring/poly.rs tests (Z_17[X]/(X^4+1))
    add("src/ring/poly.rs:185-190", "poly_add", [[1, 2, 3, 4], [5, 6, 7, 8], 17], [6, 8, 10, 12])
    add("src/ring/poly.rs:190", "poly_sub", [[6, 8, 10, 12], [5, 6, 7, 8], 17], [1, 2, 3, 4])
    add("src/ring/poly.rs:194-198", "poly_neg_add_is_zero", [[1, 0, 3, 16], 17], [0, 0, 0, 0])
    add("src/ring/poly.rs:202-207", "mul_naive", [[1, 1, 0, 0], [1, 1, 0, 0], 17], [1, 2, 1, 0])
    add("src/ring/poly.rs:210-218", "mul_naive", [[0, 0, 0, 1], [0, 0, 0, 1], 17], [0, 0, 16, 0])
    add("src/ring/poly.rs:221-225", "scalar_mul", [[1, 2, 3, 4], 3, 17], [3, 6, 9, 12])
    add("src/ring/poly.rs:228-233", "centered_coeffs", [[0, 1, 16, 9], 17], [0, 1, -1, -8])
    # src/ring/ntt.rs tests (n = 16, q = 65537)
    add("src/ring/ntt.rs:170-178", "ntt_roundtrip", [[1, 2, 3, 4, 5, 6, 7, 8], 16, M], [1, 2, 3, 4, 5, 6, 7, 8])
    add("src/ring/ntt.rs:181-195", "ntt_mul", [[1, 1], [1, 1], 16, M], [1, 2, 1] + [0] * 13)
    add("src/ring/ntt.rs:198-212", "ntt_add", [[1, 2, 3], [4, 5, 6], 16, M], [5, 7, 9] + [0] * 13)
    # src/ring/rns.rs tests (single prime 65537, n = 16)
    add("src/ring/rns.rs:299-306", "rns_roundtrip", [[1, 2, 3, 4, 5, 6, 7, 8], 16, [M]], [1, 2, 3, 4, 5, 6, 7, 8] + [0] * 8)
    add("src/ring/rns.rs:309-322", "rns_add", [[1, 2, 3, 4, 5, 6, 7, 8], [10, 20, 30, 40, 50, 60, 70, 80], 16, [M]],
        [11, 22, 33, 44, 55, 66, 77, 88] + [0] * 8)
    add("src/ring/rns.rs:325-338", "rns_mul", [[1, 1], [1, 1], 16, [M]], [1, 2, 1] + [0] * 13)
    # src/bfv/keyswitch.rs tests
    add("src/bfv/keyswitch.rs:111-119", "gadget_decompose", [[42], M, 16, 2], [[65531], [3]])
    add("src/bfv/keyswitch.rs:122-144", "gadget_reconstruct", [[12345, 54321, 100, 0], M, 16, 4], [12345, 54321, 100, 0])
    add("src/bfv/keyswitch.rs:147-152", "gadget_decompose_digit0", [[M - 1], M, 16, 4], M - 1)
    # src/bfv/encrypt.rs:300-330 — Delta = floor(Q/p) residues for Q = q0*q1
    q0, q1 = 1099509805057, 562949953443841
    delta = (q0 * q1) // 257
    add("src/bfv/encrypt.rs:300-330", "delta_residues", [[q0, q1], 257], [delta % q0, delta % q1])
    # decrypt-level functional tests (values the reference asserts)
    add("src/bfv/eval.rs:883-900", "bfv_mul_decrypt", ["compact_bfv", 3, 7], 21)
    add("src/bfv/eval.rs:903-927", "bfv_mul_decrypt_multiprime", [[16, 257, [65537, 1099509805057], 8],
                                                                  [[3, 7], [10, 20], [0, 5]]], [21, 200, 0])
    add("src/dbfv/eval.rs:223-237", "dbfv_mul_decrypt", ["compact_dbfv", 3, 7], 21)
    add("src/dbfv/eval.rs:272-290", "dbfv_mul_decrypt_many", ["compact_dbfv", [[15, 15], [10, 20], [12, 12]]],
        [(15 * 15) % 256, (10 * 20) % 256, (12 * 12) % 256])
    add("src/dbfv/eval.rs:292-313", "dbfv_depth_guard", ["compact_dbfv"],
        "chained dBFV multiplication requires ciphertext-level lattice reduction")
    add("src/dbfv/eval.rs:385-416", "hps_single_aux_guard", [[4096, 1040407, [18014398509506561], [36028797018972161], 256]],
        "single aux prime too small")
    add("src/dbfv/eval.rs:419-453", "schoolbook_guard", [[4096, 1040407, [18014398509506561], [], 256]],
        "schoolbook BFV multiplication can overflow i128")
    return k


def bfv_case(name, prm, B, seed, num_keys=None):
    rng = np.random.default_rng(seed)
    q, n = prm.ct_basis.moduli, prm.ring_degree
    ct1 = uniform_residues(rng, (B, 2), q, n)
    ct2 = uniform_residues(rng, (B, 2), q, n)
    G = prm.gadget_digits if num_keys is None else num_keys
    rlk = uniform_residues(rng, (G, 2), q, n)
    rk = np_to_rlk(rlk, prm)
    out, out3 = [], []
    for b in range(B):
        c1, c2 = np_to_ct(ct1[b], prm), np_to_ct(ct2[b], prm)
        m = obfv.bfv_mul_no_relin(c1, c2)
        out3.append(ct_to_np(m))
        out.append(ct_to_np(obfv.relinearize(m, rk)))
    aux = prm.aux_basis.moduli if prm.aux_basis is not None else []
    meta = {"n": n, "ct_moduli": [str(x) for x in q], "aux_moduli": [str(x) for x in aux],
            "plain": prm.plain_modulus, "gadget_base": prm.gadget_base, "gadget_digits": prm.gadget_digits}
    return name, meta, {"ct1": ct1, "ct2": ct2, "rlk": rlk, "out": np.stack(out), "out3": np.stack(out3)}


def dbfv_case(name, dprm, B, seed):
    prm = dprm.bfv_params
    rng = np.random.default_rng(seed)
    q, n, d = prm.ct_basis.moduli, prm.ring_degree, dprm.num_digits
    a = uniform_residues(rng, (B, d, 2), q, n)
    b = uniform_residues(rng, (B, d, 2), q, n)
    rlk = uniform_residues(rng, (prm.gadget_digits, 2), q, n)
    rk = np_to_rlk(rlk, prm)
    outs = []
    for i in range(B):
        A = odbfv.DbfvCiphertext([np_to_ct(a[i, k], prm) for k in range(d)], d, 0, dprm)
        Bc = odbfv.DbfvCiphertext([np_to_ct(b[i, k], prm) for k in range(d)], d, 0, dprm)
        r = odbfv.dbfv_mul(A, Bc, rk)
        outs.append(np.stack([ct_to_np(l) for l in r.limbs]))
    aux = prm.aux_basis.moduli if prm.aux_basis is not None else []
    meta = {"n": n, "ct_moduli": [str(x) for x in q], "aux_moduli": [str(x) for x in aux],
            "plain": prm.plain_modulus, "gadget_base": prm.gadget_base, "gadget_digits": prm.gadget_digits,
            "d": d, "base": dprm.base, "dbfv_plain": dprm.plain_modulus}
    return name, meta, {"a": a, "b": b, "rlk": rlk, "out": np.stack(outs)}


def bfv_cases():
    B = P.BfvParamsBuilder
    yield bfv_case("multiprime16", B().ring_degree(16).plain_modulus(257).ct_moduli([65537, 1099509805057])
                   .gadget_base(8).build(), 2, 101)
    yield bfv_case("cfg1_compact", P.compact_bfv(), 1, 102)
    yield bfv_case("cfg3_n64", P.cfg3_params(64), 2, 103)
    yield bfv_case("cfg3_n64_3keys", P.cfg3_params(64), 1, 104, num_keys=3)
    yield bfv_case("cfg5basis_n32", B().ring_degree(32).plain_modulus(1040407).ct_moduli(P.Q4)
                   .gadget_base(256).build(), 1, 105)
    yield bfv_case("hps2_n64", B().ring_degree(64).plain_modulus(1040407).ct_moduli([1152921504606830593])
                   .aux_moduli([18014398509998081, 36028797018972161]).gadget_base(256).build(), 2, 106)
    yield bfv_case("schoolbook16", B().ring_degree(16).plain_modulus(17).ct_moduli([65537]).gadget_base(4).build(),
                   2, 107)
    yield bfv_case("oddbase16", B().ring_degree(16).plain_modulus(17).ct_moduli([65537, 1099509805057])
                   .gadget_base(5).build(), 2, 108)


def dbfv_cases():
    yield dbfv_case("dbfv_compact", P.compact_dbfv(), 1, 201)
    yield dbfv_case("dbfv_cfg4_n32", P.cfg4_params(32), 2, 202)
    yield dbfv_case("dbfv_cfg5basis_n16", P.cfg5_params(16), 1, 203)


DIGEST_SPEC = {"config": "cfg3", "n": 4096, "batch": 2, "seed": 3003,
               "generator": "numpy.random.default_rng(seed); ct1, ct2 = uniform_residues((B,2)); "
                            "rlk = uniform_residues((G,2))  (tests/bridge.py)"}


def digest_inputs(spec):
    prm = P.cfg3_params(spec["n"])
    rng = np.random.default_rng(spec["seed"])
    q, n = prm.ct_basis.moduli, prm.ring_degree
    ct1 = uniform_residues(rng, (spec["batch"], 2), q, n)
    ct2 = uniform_residues(rng, (spec["batch"], 2), q, n)
    rlk = uniform_residues(rng, (prm.gadget_digits, 2), q, n)
    return prm, ct1, ct2, rlk


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.uint64).tobytes()).hexdigest()


# Full-size dBFV digests (BASELINE configs[3] and [4]), from the C restatement of dbfv_mul
# (oracle/c oracle_dbfv_mul: all d^2 products, per-limb sums, reduce): inputs regenerated from the
# seed, item 0 of each list is the pinned item.  The chain is paper_repro's guard-bypass chain
# (src/bin/paper_repro.rs:203-236: acc <- dbfv_mul(acc, y) with mul_depth reset, `depth` steps).
DBFV_DIGESTS = {
    "cfg4_full": {"config": "cfg4", "n": 4096, "items": 4, "seed": 4004, "depth": 1},
    "cfg5_full": {"config": "cfg5", "n": 8192, "items": 1, "seed": 5005, "depth": 1},
    "cfg5_chain4": {"config": "cfg5", "n": 8192, "items": 1, "seed": 5006, "depth": 4},
}
DBFV_GEN = ("numpy.random.default_rng(seed); a, b = uniform_residues((items, d, 2)); "
            "rlk = uniform_residues((G, 2))  (tests/bridge.py)")


def dbfv_digest_inputs(spec):
    dp = P.cfg4_params(spec["n"]) if spec["config"] == "cfg4" else P.cfg5_params(spec["n"])
    prm = dp.bfv_params
    rng = np.random.default_rng(spec["seed"])
    q, n, d = prm.ct_basis.moduli, prm.ring_degree, dp.num_digits
    a = uniform_residues(rng, (spec["items"], d, 2), q, n)
    b = uniform_residues(rng, (spec["items"], d, 2), q, n)
    rlk = uniform_residues(rng, (prm.gadget_digits, 2), q, n)
    return dp, a, b, rlk


def dbfv_digests(threads):
    from oracle import cref
    out = {}
    for name, spec in DBFV_DIGESTS.items():
        dp, a, b, rlk = dbfv_digest_inputs(spec)
        acc = a
        for _ in range(spec["depth"]):
            acc = cref.dbfv_mul(dp, acc, b, rlk, threads=threads)
        e = dict(spec, generator=DBFV_GEN)
        e["sha256_inputs"] = sha(np.concatenate([a.ravel(), b.ravel(), rlk.ravel()]))
        e["sha256_out"] = sha(acc)
        e["sha256_out_item0_limbs"] = [sha(acc[0, k]) for k in range(acc.shape[1])]
        out[name] = e
        print(name, e["sha256_out"], flush=True)
    return out


# Worst-case inputs of the two exactness bounds (tests/worstcase.py): every digit -B/2 with a
# sign-aligned key (the key switch over 31-bit primes) and tensors at 2 n floor(Q/2)^2 (psum), at
# cfg5 size, where the C restatement needs minutes (cfg3 / cfg4 are checked in-test).
WORST = {
    "worst_cfg5_digits": {"config": "cfg5", "n": 8192, "kind": "digits", "d": 8},
    "worst_cfg5_tensor": {"config": "cfg5", "n": 8192, "kind": "tensor", "d": 8},
}


def worst_inputs(spec):
    import worstcase as W
    dp = P.cfg5_params(spec["n"]) if spec["config"] == "cfg5" else P.cfg4_params(spec["n"])
    prm = dp.bfv_params
    q, n, d, G = prm.ct_basis.moduli, prm.ring_degree, dp.num_digits, prm.gadget_digits
    if spec["kind"] == "digits":
        a, b, rlk, _ = W.digit_case_dbfv(q, prm.plain_modulus, prm.gadget_base, G, n, d)
    else:
        a, b, rlk = W.tensor_case_dbfv(q, n, d, G)
    return dp, a, b, rlk


def worst_digests(threads):
    from oracle import cref
    out = {}
    for name, spec in WORST.items():
        dp, a, b, rlk = worst_inputs(spec)
        r = cref.dbfv_mul(dp, a, b, rlk, threads=threads)
        e = dict(spec)
        e["sha256_inputs"] = sha(np.concatenate([a.ravel(), b.ravel(), rlk.ravel()]))
        e["sha256_out"] = sha(r)
        out[name] = e
        print(name, e["sha256_out"], flush=True)
    return out


# The bench's production shapes (bench.py DEFAULT_BATCH), so that the exact batch the bench times,
# at the library's default chunking and pipeline lanes, is compared against the C restatement:
#   cfg3    bfv_mul_and_relin, B = 1024 (two 512-product chunks on two lanes; eval.rs:73-147)
#   cfg1    bfv_mul_and_relin on compact_bfv, B = 8192 (chunks of 7168 + 1024; eval.rs:157-332)
#   u64dbfv dbfv_mul on u64_dbfv, B = 64 items (4096 HPS products, chunks of 1152; dbfv/eval.rs:82-149)
#   cfg2    INTT(NTT(a) . NTT(b)) of B = 16384 coefficient-domain polys (ntt.rs:181-195)
#   cfg4    dbfv_mul d = 2 over cfg3's basis, B = 1024 items (3072 products with psum digit sums across
#           six 512-product chunks; dbfv/eval.rs:82-149)
#   cfg5    dbfv_mul chain of depth 4 (paper_repro.rs:203-236: acc <- dbfv_mul(acc, y)), B = 8 chains at
#           n = 8192, every chain digested on its own
# Inputs are regenerated from the seed by the GPU test (numpy default_rng, tests/bridge.py); the
# digests of row blocks name the failing rows when one differs.
BENCH_DIGESTS = {
    "cfg3_bench": {"config": "cfg3", "n": 4096, "batch": 1024, "seed": 3301, "block": 128},
    "cfg1_bench": {"config": "cfg1", "n": 1024, "batch": 8192, "seed": 1101, "block": 1024},
    "u64dbfv_bench": {"config": "u64dbfv", "n": 4096, "batch": 64, "seed": 6401, "block": 8},
    "cfg2_bench": {"config": "cfg2", "n": 4096, "batch": 16384, "seed": 2201, "block": 2048},
    "cfg4_bench": {"config": "cfg4", "n": 4096, "batch": 1024, "seed": 4401, "block": 128},
    "cfg5_bench": {"config": "cfg5", "n": 8192, "batch": 8, "seed": 5501, "block": 1, "depth": 4},
}
DBFV_CFGS = ("u64dbfv", "cfg4", "cfg5")
BENCH_GEN = ("numpy.random.default_rng(seed); bfv: ct1, ct2 = uniform_residues((B, 2)), rlk = "
             "uniform_residues((G, 2)); dbfv: a, b = uniform_residues((B, d, 2)), rlk; cfg2: a, b = "
             "uniform_residues((B,))  (tests/bridge.py)")


def bench_params(cfg, n):
    if cfg == "cfg3":
        return P.cfg3_params(n)
    if cfg == "cfg1":
        return P.compact_bfv()
    if cfg == "u64dbfv":
        return P.u64_dbfv()
    if cfg == "cfg2":
        return P.BfvParamsBuilder().ring_degree(n).plain_modulus(65537).ct_moduli([P.Q3[0]]).build()
    if cfg == "cfg4":
        return P.cfg4_params(n)
    if cfg == "cfg5":
        return P.cfg5_params(n)
    raise ValueError(cfg)


def bench_digest_inputs(spec):
    """(params, x, y, rlk) of a BENCH_DIGESTS entry; x, y are ct1/ct2, a/b or the cfg2 operands."""
    prm = bench_params(spec["config"], spec["n"])
    dbfv = spec["config"] in DBFV_CFGS
    bp = prm.bfv_params if dbfv else prm
    rng = np.random.default_rng(spec["seed"])
    q, n, B = bp.ct_basis.moduli, bp.ring_degree, spec["batch"]
    pre = (B,) if spec["config"] == "cfg2" else (B, prm.num_digits, 2) if dbfv else (B, 2)
    x = uniform_residues(rng, pre, q, n)
    y = uniform_residues(rng, pre, q, n)
    rlk = None if spec["config"] == "cfg2" else uniform_residues(rng, (bp.gadget_digits, 2), q, n)
    return prm, x, y, rlk


def bench_output(spec, prm, x, y, rlk, threads):
    from oracle import cref
    if spec["config"] == "cfg2":
        return cref.polymul(spec["n"], prm.ct_basis.moduli[0], x, y, threads=threads)
    if spec["config"] in DBFV_CFGS:
        acc = x
        for _ in range(spec.get("depth", 1)):
            acc = cref.dbfv_mul(prm, acc, y, rlk, threads=threads)
        return acc
    return cref.bfv_mul_and_relin(prm, x, y, rlk, threads=threads)


def input_digest(x, y, rlk):
    parts = [x.ravel(), y.ravel()] + ([] if rlk is None else [rlk.ravel()])
    return sha(np.concatenate(parts))


def bench_digests(threads, names=None):
    import time
    out = {}
    for name, spec in BENCH_DIGESTS.items():
        if names and name not in names:
            continue
        t0 = time.time()
        prm, x, y, rlk = bench_digest_inputs(spec)
        r = bench_output(spec, prm, x, y, rlk, threads)
        e = dict(spec, generator=BENCH_GEN)
        e["sha256_inputs"] = input_digest(x, y, rlk)
        e["sha256_out"] = sha(r)
        blk = spec["block"]
        e["sha256_out_blocks"] = [sha(r[i:i + blk]) for i in range(0, spec["batch"], blk)]
        out[name] = e
        print(name, e["sha256_out"], f"{time.time() - t0:.1f} s", flush=True)
    return out


def main():
    if "--bench-digests" in sys.argv:   # minutes: cfg3's 1024 BigInt schoolbook tensors dominate
        names = [a for a in sys.argv[1:] if not a.startswith("--")]
        with open(os.path.join(HERE, "digests.json")) as f:
            dg = json.load(f)
        dg.update(bench_digests(threads=os.cpu_count() or 1, names=names))
        with open(os.path.join(HERE, "digests.json"), "w") as f:
            json.dump(dg, f, indent=1)
        return
    if "--worst-digests" in sys.argv:
        with open(os.path.join(HERE, "digests.json")) as f:
            dg = json.load(f)
        dg.update(worst_digests(threads=os.cpu_count() or 1))
        with open(os.path.join(HERE, "digests.json"), "w") as f:
            json.dump(dg, f, indent=1)
        return
    if "--dbfv-digests" in sys.argv:   # minutes of CPU: BigInt schoolbook tensors at n = 8192
        with open(os.path.join(HERE, "digests.json")) as f:
            dg = json.load(f)
        dg.update(dbfv_digests(threads=os.cpu_count() or 1))
        with open(os.path.join(HERE, "digests.json"), "w") as f:
            json.dump(dg, f, indent=1)
        return
    with open(os.path.join(HERE, "kats.json"), "w") as f:
        json.dump(kats(), f, indent=1)
    arrays, meta = {}, {}
    for name, m, arr in list(bfv_cases()) + list(dbfv_cases()):
        meta[name] = m
        for k, v in arr.items():
            arrays[f"{name}__{k}"] = v
    np.savez_compressed(os.path.join(HERE, "vectors.npz"), **arrays)
    with open(os.path.join(HERE, "vectors_meta.json"), "w") as f:
        json.dump(meta, f, indent=1)
    from oracle import cref
    prm, ct1, ct2, rlk = digest_inputs(DIGEST_SPEC)
    out = cref.bfv_mul_and_relin(prm, ct1, ct2, rlk, threads=2)
    spec = dict(DIGEST_SPEC)
    spec["sha256_inputs"] = sha(np.concatenate([ct1.ravel(), ct2.ravel(), rlk.ravel()]))
    spec["sha256_out"] = sha(out)
    path = os.path.join(HERE, "digests.json")
    dg = json.load(open(path)) if os.path.exists(path) else {}
    dg["cfg3_full"] = spec
    with open(path, "w") as f:
        json.dump(dg, f, indent=1)
    print("wrote kats.json, vectors.npz, vectors_meta.json, digests.json")


if __name__ == "__main__":
    main()
