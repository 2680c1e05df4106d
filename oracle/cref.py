"""ctypes wrapper of oracle/c/liboracle.so — the C restatement of the reference algorithm.

TEST ORACLE / CPU BASELINE ONLY (see oracle/__init__.py).  Cross-checked against the
Python restatement in tests/test_oracle.py.
"""

from __future__ import annotations

import ctypes as C
import os

import numpy as np

_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "c", "liboracle.so")
_lib = None


def available() -> bool:
    return os.path.exists(_PATH)


def _load():
    global _lib
    if _lib is None:
        lib = C.CDLL(_PATH)
        P, I, U = C.c_void_p, C.c_int, C.c_uint64
        lib.oracle_bfv_mul.argtypes = [I, I, P, I, P, U, U, I, P, P, P, I, P, I, I, I]
        lib.oracle_bfv_mul.restype = I
        lib.oracle_ntt.argtypes = [I, U, P, I, I, I]
        lib.oracle_ntt.restype = I
        lib.oracle_dbfv_mul.argtypes = [I, I, P, I, P, U, U, I, I, U, U, P, P, P, I, P, I, I]
        lib.oracle_dbfv_mul.restype = I
        lib.oracle_polymul.argtypes = [I, U, P, P, P, I, I]
        lib.oracle_polymul.restype = I
        _lib = lib
    return _lib


def _u64(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.uint64))


def bfv_mul(params, ct1, ct2, rlk=None, relin=True, threads=1):
    """bfv_mul_and_relin (relin=True) or bfv_mul_no_relin of batches [B][2][L][n] (NTT domain)."""
    lib = _load()
    ct1, ct2 = _u64(ct1), _u64(ct2)
    B, _, L, n = ct1.shape
    q = _u64(params.ct_basis.moduli)
    aux = _u64(params.aux_basis.moduli) if params.aux_basis is not None else np.zeros(1, np.uint64)
    K = len(params.aux_basis.moduli) if params.aux_basis is not None else 0
    if rlk is None:
        rlk = np.zeros((0, 2, L, n), dtype=np.uint64)
    rlk = _u64(rlk)
    out = np.zeros((B, 2 if relin else 3, L, n), dtype=np.uint64)
    rc = lib.oracle_bfv_mul(n, L, q.ctypes.data, K, aux.ctypes.data, params.plain_modulus,
                            params.gadget_base, params.gadget_digits, ct1.ctypes.data,
                            ct2.ctypes.data, rlk.ctypes.data if rlk.size else None, rlk.shape[0],
                            out.ctypes.data, B, 1 if relin else 0, threads)
    if rc != 0:
        raise ValueError("oracle_bfv_mul: unsupported parameters")
    return out


def bfv_mul_and_relin(params, ct1, ct2, rlk, threads=1):
    return bfv_mul(params, ct1, ct2, rlk, True, threads)


def dbfv_mul(dparams, a, b, rlk, threads=1):
    """dbfv_mul + reduce (dbfv/eval.rs:82-149, reduction.rs:15-93) of batches a, b = [B][d][2][L][n]
    (NTT domain), all d^2 products, depth guard left to the caller (paper_repro's chains reset it)."""
    lib = _load()
    prm = dparams.bfv_params
    a, b, rlk = _u64(a), _u64(b), _u64(rlk)
    B, d, _, L, n = a.shape
    q = _u64(prm.ct_basis.moduli)
    aux = _u64(prm.aux_basis.moduli) if prm.aux_basis is not None else np.zeros(1, np.uint64)
    K = len(prm.aux_basis.moduli) if prm.aux_basis is not None else 0
    out = np.zeros_like(a)
    rc = lib.oracle_dbfv_mul(n, L, q.ctypes.data, K, aux.ctypes.data, prm.plain_modulus, prm.gadget_base,
                             prm.gadget_digits, d,
                             dparams.base, dparams.plain_modulus, a.ctypes.data, b.ctypes.data,
                             rlk.ctypes.data if rlk.size else None, rlk.shape[0], out.ctypes.data, B, threads)
    if rc != 0:
        raise ValueError("oracle_dbfv_mul: unsupported parameters")
    return out


def polymul(n, q, a, b, threads=1):
    """INTT(NTT(a) (.) NTT(b)) of coefficient-domain polys [count][n] mod q (ntt.rs:181-195)."""
    lib = _load()
    a, b = _u64(a), _u64(b)
    out = np.empty_like(a)
    lib.oracle_polymul(n, q, a.ctypes.data, b.ctypes.data, out.ctypes.data, a.size // n, threads)
    return out


def ntt(n, q, polys, inverse=False, threads=1):
    lib = _load()
    a = _u64(polys).copy()
    lib.oracle_ntt(n, q, a.ctypes.data, a.size // n, 1 if inverse else 0, threads)
    return a
