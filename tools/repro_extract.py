#!/usr/bin/env python3
"""Localises a wrong batched coefficient extraction at n = 16 with device-generated Galois keys
(G = 17 digits): batched automorphisms for B = 1..6 against the oracle, then extractions of
every (j0, J) window shape."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle import bfv as obfv, bootstrap as ob, params as P  # noqa: E402
from exacto_amd._ffi import HipContext  # noqa: E402
from bridge import ct_to_np, np_to_ct, np_to_rlk, uniform_residues  # noqa: E402

prm = (P.BfvParamsBuilder().ring_degree(16).plain_modulus(97).ct_moduli([1125899906842817])
       .sigma(3.2).gadget_base(8).build())
n, q = prm.ring_degree, prm.ct_basis.moduli
ctx = HipContext.from_params(prm)
KEY = [42, 0, 0, 1]
sk = ctx.gen_secret_key(KEY, stream=1)
els, gks = ctx.gen_trace_galois_keys(sk, KEY, stream=100)
keys = {k: obfv.GaloisKey(np_to_rlk(gks[e], prm).keys, k, prm) for e, k in enumerate(els)}
rng = np.random.default_rng(5)
bad = 0
for B in range(1, 7):
    cts = uniform_residues(rng, (B, 2), q, n)
    for e, k in enumerate(els[:3]):
        got = ctx.bfv_apply_automorphism(cts, k, gks[e])
        errs = [b for b in range(B)
                if not np.array_equal(got[b], ct_to_np(obfv.bfv_apply_automorphism(np_to_ct(cts[b], prm), keys[k])))]
        if errs:
            print(f"automorphism B={B} k={k}: wrong items {errs}")
            bad += 1
ct = uniform_residues(rng, (2,), q, n)
want = [ct_to_np(ob.extract_coefficient(np_to_ct(ct, prm), j, keys)) for j in range(n)]
for J in range(1, 7):
    for j0 in (0, 1, 5):
        got = ctx.extract_coefficients(ct, j0, J, els, gks)
        errs = [j0 + t for t in range(J) if not np.array_equal(got[t], want[j0 + t])]
        if errs:
            print(f"extract j0={j0} J={J}: wrong {errs}")
            bad += 1
print("REPRO", "FAIL" if bad else "OK")
