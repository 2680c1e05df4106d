"""Test helpers: move data between oracle objects and the C-ABI flat layout.

Layout (include/exacto_hip.h): ciphertext batch [B][poly][limb][n] uint64, NTT domain in
this build's documented convention — the oracle (oracle/ring.py NttPlan) implements the
same convention, so NTT-domain arrays compare directly.
"""

from __future__ import annotations

import numpy as np

from oracle import bfv as obfv
from oracle.ring import NttPoly, RnsPoly


def rns_to_np(p: RnsPoly) -> np.ndarray:
    return np.array([c.evals for c in p.components], dtype=np.uint64)


def ct_to_np(ct) -> np.ndarray:
    return np.stack([rns_to_np(p) for p in ct.c])


def cts_to_np(cts) -> np.ndarray:
    return np.stack([ct_to_np(c) for c in cts])


def rlk_to_np(rlk) -> np.ndarray:
    if not rlk.keys:
        return np.zeros((0, 2, 1, 1), dtype=np.uint64)
    return np.stack([np.stack([rns_to_np(k0), rns_to_np(k1)]) for k0, k1 in rlk.keys])


def np_to_rns(a: np.ndarray, basis) -> RnsPoly:
    return RnsPoly([NttPoly([int(x) for x in a[i]], q, plan)
                    for i, (q, plan) in enumerate(zip(basis.moduli, basis.plans))], basis.ring_degree)


def np_to_ct(a: np.ndarray, params):
    return obfv.BfvCiphertext([np_to_rns(a[k], params.ct_basis) for k in range(a.shape[0])], params)


def np_to_rlk(a: np.ndarray, params):
    keys = [(np_to_rns(a[g, 0], params.ct_basis), np_to_rns(a[g, 1], params.ct_basis))
            for g in range(a.shape[0])]
    return obfv.RelinKey(keys, params)


def uniform_residues(rng: np.random.Generator, shape_prefix, moduli, n) -> np.ndarray:
    """Uniform canonical residues: shape prefix + [L][n], limb i uniform in [0, q_i)."""
    out = np.empty(tuple(shape_prefix) + (len(moduli), n), dtype=np.uint64)
    for i, q in enumerate(moduli):
        out[..., i, :] = rng.integers(0, q, size=tuple(shape_prefix) + (n,), dtype=np.uint64)
    return out
