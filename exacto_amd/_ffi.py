"""ctypes binding of the C ABI in include/exacto_hip.h (libexacto_hip.so, built in-tree).

This is the only way the Python side reaches the GPU path; there is no CPU fallback:
if the shared library is missing, importing anything that needs it raises.
"""

from __future__ import annotations

import ctypes as C
import os

import numpy as np

_LIB_PATH = os.environ.get("EXACTO_HIP_LIB") or os.path.join(
    os.path.dirname(os.path.abspath(__file__)), "lib", "libexacto_hip.so")  # env: kernel-variant builds (tools/)

VARIANTS = ("InvalidParam", "DimensionMismatch", "ModulusMismatch", "InvalidRingDegree",
            "DecryptionError", "DecompositionError", "LatticeError", "MissingKey", "NotImplemented")

PATH_EXACT_RNS, PATH_HPS, PATH_SCHOOLBOOK = 0, 1, 2


class ExactoError(Exception):
    """Mirror of reference src/error.rs ExactoError: ``variant`` + Display text."""

    def __init__(self, code: int, message: str):
        super().__init__(message)
        self.code = code
        self.variant = VARIANTS[code - 1] if 1 <= code <= 9 else "HipError"


NTT_ORDER = 1   # exacto_hip.h EXACTO_NTT_ORDER: evaluation k at (k mod 16) n/16 + k/16


class CtxInfo(C.Structure):
    _fields_ = [("ring_degree", C.c_size_t), ("num_ct_moduli", C.c_size_t),
                ("num_aux_moduli", C.c_size_t), ("num_internal_aux", C.c_size_t),
                ("gadget_digits", C.c_size_t), ("gadget_base", C.c_uint64),
                ("plain_modulus", C.c_uint64), ("mul_path", C.c_int), ("device", C.c_int),
                ("ks32_primes", C.c_int), ("psum_max", C.c_int),
                ("ks32_lazy", C.c_int), ("ntt_order", C.c_int), ("dbfv_key_switch", C.c_int)]


_lib = None

# (name, argtypes, restype)
_P = C.c_void_p
_SZ = C.c_size_t
_U64 = C.c_uint64
_SIGS = [
    ("exacto_ctx_create", [C.POINTER(_P), _SZ, _P, _SZ, _P, _SZ, _U64, _U64, C.c_int], C.c_int),
    ("exacto_ctx_destroy", [_P], None),
    ("exacto_ctx_get_info", [_P, C.POINTER(CtxInfo)], C.c_int),
    ("exacto_ctx_set_stream", [_P, _P], C.c_int),
    ("exacto_ctx_set_chunk", [_P, _SZ], C.c_int),
    ("exacto_synchronize", [_P], C.c_int),
    ("exacto_ctx_load_relin_key", [_P, _P, _SZ], C.c_int),
    ("exacto_ctx_load_relin_key_dev", [_P, _P, _SZ], C.c_int),
    ("exacto_ctx_relin_key_buffer", [_P, _SZ], _P),
    ("exacto_ntt_fwd", [_P, _P, _SZ, _SZ], C.c_int),
    ("exacto_ntt_inv", [_P, _P, _SZ, _SZ], C.c_int),
    ("exacto_ntt_fwd_dev", [_P, _P, _SZ, _SZ], C.c_int),
    ("exacto_ntt_inv_dev", [_P, _P, _SZ, _SZ], C.c_int),
    ("exacto_rns_fwd_dev", [_P, _P, _SZ], C.c_int),
    ("exacto_rns_inv_dev", [_P, _P, _SZ], C.c_int),
    ("exacto_rns_add_dev", [_P, _P, _P, _P, _SZ], C.c_int),
    ("exacto_rns_sub_dev", [_P, _P, _P, _P, _SZ], C.c_int),
    ("exacto_rns_neg_dev", [_P, _P, _P, _SZ], C.c_int),
    ("exacto_rns_mul_dev", [_P, _P, _P, _P, _SZ], C.c_int),
    ("exacto_rns_mul_inv_dev", [_P, _P, _P, _P, _SZ], C.c_int),
    ("exacto_rns_polymul_dev", [_P, _P, _P, _P, _SZ], C.c_int),
    ("exacto_rns_scalar_mul_dev", [_P, _P, _U64, _P, _SZ], C.c_int),
    ("exacto_bfv_add", [_P, _P, _SZ, _P, _SZ, _P, _SZ], C.c_int),
    ("exacto_bfv_add_dev", [_P, _P, _SZ, _P, _SZ, _P, _SZ], C.c_int),
    ("exacto_bfv_sub", [_P, _P, _SZ, _P, _SZ, _P, _SZ], C.c_int),
    ("exacto_bfv_sub_dev", [_P, _P, _SZ, _P, _SZ, _P, _SZ], C.c_int),
    ("exacto_bfv_neg", [_P, _P, _SZ, _P, _SZ], C.c_int),
    ("exacto_bfv_neg_dev", [_P, _P, _SZ, _P, _SZ], C.c_int),
    ("exacto_bfv_mul_no_relin", [_P, _P, _SZ, _P, _SZ, _P, _SZ], C.c_int),
    ("exacto_bfv_mul_no_relin_dev", [_P, _P, _SZ, _P, _SZ, _P, _SZ], C.c_int),
    ("exacto_relinearize", [_P, _P, _SZ, _P, _SZ], C.c_int),
    ("exacto_relinearize_dev", [_P, _P, _SZ, _P, _SZ], C.c_int),
    ("exacto_bfv_mul_and_relin", [_P, _P, _P, _P, _SZ], C.c_int),
    ("exacto_bfv_mul_and_relin_dev", [_P, _P, _P, _P, _SZ], C.c_int),
    ("exacto_gadget_decompose_dev", [_P, _P, _P, _SZ, _SZ], C.c_int),
    ("exacto_dbfv_mul", [_P, _SZ, _U64, _U64, _P, _P, _P, _SZ, _P, _P, _P], C.c_int),
    ("exacto_dbfv_mul_dev", [_P, _SZ, _U64, _U64, _P, _P, _P, _SZ, _P, _P, _P], C.c_int),
    ("exacto_dbfv_mul_chain", [_P, _SZ, _U64, _U64, _P, _P, _P, _SZ, _SZ], C.c_int),
    ("exacto_dbfv_mul_limbs", [_P, _SZ, _U64, _U64, _P, _P, _P, _SZ, _P, _SZ], C.c_int),
    ("exacto_dbfv_mul_limbs_dev", [_P, _SZ, _U64, _U64, _P, _P, _P, _SZ, _P, _SZ], C.c_int),
    ("exacto_bfv_decrypt", [_P, _P, _SZ, _P, _P, _SZ], C.c_int),
    ("exacto_bfv_decrypt_dev", [_P, _P, _SZ, _P, _P, _SZ], C.c_int),
    ("exacto_dbfv_decrypt", [_P, _SZ, _U64, _U64, _P, _P, _P, _SZ], C.c_int),
    ("exacto_dbfv_decrypt_dev", [_P, _SZ, _U64, _U64, _P, _P, _P, _SZ], C.c_int),
    ("exacto_dbfv_decrypt_poly", [_P, _SZ, _U64, _U64, _P, _P, _P, _SZ], C.c_int),
    ("exacto_dbfv_decrypt_poly_dev", [_P, _SZ, _U64, _U64, _P, _P, _P, _SZ], C.c_int),
    ("exacto_dbfv_mul_chain_dev", [_P, _SZ, _U64, _U64, _P, _P, _P, _SZ, _SZ], C.c_int),
    ("exacto_gen_secret_key", [_P, _P, _U64, _P], C.c_int),
    ("exacto_gen_secret_key_dev", [_P, _P, _U64, _P], C.c_int),
    ("exacto_gen_public_key", [_P, _P, C.c_double, _P, _U64, _P], C.c_int),
    ("exacto_gen_public_key_dev", [_P, _P, C.c_double, _P, _U64, _P], C.c_int),
    ("exacto_gen_relin_key", [_P, _P, C.c_double, _P, _U64, _SZ, _P], C.c_int),
    ("exacto_gen_relin_key_dev", [_P, _P, C.c_double, _P, _U64, _SZ, _P], C.c_int),
    ("exacto_encrypt_sk", [_P, _P, _P, C.c_double, _P, _U64, _P, _SZ], C.c_int),
    ("exacto_encrypt_sk_dev", [_P, _P, _P, C.c_double, _P, _U64, _P, _SZ], C.c_int),
    ("exacto_encrypt_pk", [_P, _P, _P, C.c_double, _P, _U64, _P, _SZ], C.c_int),
    ("exacto_encrypt_pk_dev", [_P, _P, _P, C.c_double, _P, _U64, _P, _SZ], C.c_int),
    ("exacto_gen_galois_key", [_P, _P, _U64, C.c_double, _P, _U64, _SZ, _P], C.c_int),
    ("exacto_gen_galois_key_dev", [_P, _P, _U64, C.c_double, _P, _U64, _SZ, _P], C.c_int),
    ("exacto_bfv_apply_automorphism", [_P, _P, _SZ, _U64, _P, _SZ, _P, _SZ], C.c_int),
    ("exacto_bfv_apply_automorphism_dev", [_P, _P, _SZ, _U64, _P, _SZ, _P, _SZ], C.c_int),
    ("exacto_bfv_plain_mul", [_P, _P, _SZ, _P, _P, _SZ], C.c_int),
    ("exacto_bfv_plain_mul_dev", [_P, _P, _SZ, _P, _P, _SZ], C.c_int),
    ("exacto_bfv_plain_add", [_P, _P, _SZ, _P, _P, _SZ], C.c_int),
    ("exacto_bfv_plain_add_dev", [_P, _P, _SZ, _P, _P, _SZ], C.c_int),
    ("exacto_bfv_inner_product", [_P, _P, _P, _SZ, _SZ, _P], C.c_int),
    ("exacto_bfv_inner_product_dev", [_P, _P, _P, _SZ, _SZ, _P], C.c_int),
    ("exacto_bfv_monomial_mul", [_P, _P, _SZ, _U64, _P, _SZ], C.c_int),
    ("exacto_bfv_monomial_mul_dev", [_P, _P, _SZ, _U64, _P, _SZ], C.c_int),
    ("exacto_bfv_trace", [_P, _P, _SZ, _P, _SZ, _P, _SZ, _P, _SZ], C.c_int),
    ("exacto_bfv_trace_dev", [_P, _P, _SZ, _P, _SZ, _P, _SZ, _P, _SZ], C.c_int),
    ("exacto_required_trace_elements", [_SZ, _P, _SZ], _SZ),
    ("exacto_extract_coefficients", [_P, _P, _U64, _SZ, _P, _SZ, _P, _SZ, _P], C.c_int),
    ("exacto_extract_coefficients_dev", [_P, _P, _U64, _SZ, _P, _SZ, _P, _SZ, _P], C.c_int),
    ("exacto_slots_to_coeffs", [_P, _P, _SZ, _SZ, _P], C.c_int),
    ("exacto_slots_to_coeffs_dev", [_P, _P, _SZ, _SZ, _P], C.c_int),
    ("exacto_lagrange_interpolate", [_P, _SZ, _U64, _P], C.c_int),
    ("exacto_compute_rounding_poly", [_U64, _U64, _U64, _P], C.c_int),
    ("exacto_trivial_encrypt", [_P, _P, _P, _SZ], C.c_int),
    ("exacto_trivial_encrypt_dev", [_P, _P, _P, _SZ], C.c_int),
    ("exacto_eval_poly", [_P, _P, _P, _SZ, _P, _SZ], C.c_int),
    ("exacto_eval_poly_dev", [_P, _P, _P, _SZ, _P, _SZ], C.c_int),
    ("exacto_bootstrap_key_material", [_P, _P, _P, _P, _P], C.c_int),
    ("exacto_bootstrap_key_material_dev", [_P, _P, _P, _P, _P], C.c_int),
    ("exacto_bfv_bootstrap", [_P, _P, _P, _SZ, _P, _P, _SZ, _U64, _P, _SZ, _P, _SZ, _P, _SZ], C.c_int),
    ("exacto_bfv_bootstrap_dev", [_P, _P, _P, _SZ, _P, _P, _SZ, _U64, _P, _SZ, _P, _SZ, _P, _SZ], C.c_int),
    ("exacto_rccl_unique_id", [_P], C.c_int),
    ("exacto_rccl_comm_init", [C.POINTER(_P), C.c_int, _P, C.c_int, C.c_int], C.c_int),
    ("exacto_rccl_comm_destroy", [_P], C.c_int),
    ("exacto_rccl_comm_count", [_P, C.POINTER(C.c_int)], C.c_int),
    ("exacto_ctx_broadcast_relin_key", [_P, _P, C.c_int, _SZ], C.c_int),
    ("exacto_broadcast_galois_key", [_P, _P, C.c_int, _P, _SZ], C.c_int),
    ("exacto_rccl_allgather_u64", [_P, _P, _P, _P, _SZ], C.c_int),
    ("exacto_rccl_sync", [_P, _P], C.c_int),
    ("exacto_last_error", [C.c_char_p, _SZ], _SZ),
    ("exacto_prof_enable", [_P, C.c_int], C.c_int),
    ("exacto_prof_read", [_P, C.c_int, C.POINTER(_U64), C.POINTER(C.c_double),
                          C.POINTER(C.c_double), C.POINTER(_U64)], C.c_int),
    ("exacto_prof_kernels", [_P, C.c_int, C.c_char_p, _SZ], _SZ),
    ("exacto_version", [], C.c_char_p),
]

EXPORTED_SYMBOLS = [s[0] for s in _SIGS]


def lib_path() -> str:
    return _LIB_PATH


def load() -> C.CDLL:
    """Load libexacto_hip.so (raises if it has not been built: no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            raise RuntimeError(f"{_LIB_PATH} not built; run `python -c 'import __graft_entry__ as g; g.build()'`")
        lib = C.CDLL(_LIB_PATH)
        for name, args, res in _SIGS:
            f = getattr(lib, name)
            f.argtypes = args
            f.restype = res
        _lib = lib
    return _lib


def last_error() -> str:
    lib = load()
    buf = C.create_string_buffer(4096)
    lib.exacto_last_error(buf, 4096)
    return buf.value.decode("utf-8", "replace")


def check(rc: int):
    if rc != 0:
        raise ExactoError(rc, last_error())


def lagrange_interpolate(values, p: int) -> list[int]:
    """digit_extract.rs:37-90 (host-only entry point)."""
    v = np.ascontiguousarray(np.asarray(values, dtype=np.uint64))
    out = np.zeros(max(v.size, 1), dtype=np.uint64)
    check(load().exacto_lagrange_interpolate(v.ctypes.data, v.size, p, out.ctypes.data))
    return [int(x) for x in out[:v.size]]


def compute_rounding_poly(t_orig: int, q_prime: int, t_boot: int) -> list[int]:
    """digit_extract.rs:19-30 (host-only entry point)."""
    out = np.zeros(max(t_boot, 1), dtype=np.uint64)
    check(load().exacto_compute_rounding_poly(t_orig, q_prime, t_boot, out.ctypes.data))
    return [int(x) for x in out[:t_boot]]


def bootstrap_key_material(orig: "HipContext", boot: "HipContext", sk):
    """bfv_host.rs:57-100, 289-330: (boot_sk [Lb][n] NTT domain, s_pt [n]) from sk [1][n]."""
    sk = _u64(sk)
    boot_sk = np.zeros((boot.L, boot.n), dtype=np.uint64)
    s_pt = np.zeros(boot.n, dtype=np.uint64)
    check(load().exacto_bootstrap_key_material(orig._h, boot._h, sk.ctypes.data, boot_sk.ctypes.data,
                                               s_pt.ctypes.data))
    return boot_sk, s_pt


def bfv_bootstrap_raw(orig: "HipContext", boot: "HipContext", ct, bsk, rpoly, q_prime, elements, gks):
    """bfv_host.rs:131-205 batched: ct [B][2][1][n] (orig) -> [B][2][Lb][n] (boot)."""
    ct, bsk, gks = _u64(ct), _u64(bsk), _u64(gks)
    rp = np.ascontiguousarray(np.asarray(rpoly, dtype=np.uint64))
    el = np.ascontiguousarray(np.asarray(elements, dtype=np.uint64))
    E = el.shape[0]
    out = np.zeros((ct.shape[0], 2, boot.L, boot.n), dtype=np.uint64)
    check(load().exacto_bfv_bootstrap(orig._h, boot._h, ct.ctypes.data, ct.shape[1], bsk.ctypes.data,
                                      rp.ctypes.data, rp.size, q_prime, el.ctypes.data if E else None, E,
                                      gks.ctypes.data if E else None, gks.shape[1] if E else 0, out.ctypes.data,
                                      ct.shape[0]))
    return out


def rccl_unique_id() -> bytes:
    """ncclGetUniqueId (128 bytes) through the library's RCCL (exacto_rccl_unique_id)."""
    buf = (C.c_uint8 * 128)()
    check(load().exacto_rccl_unique_id(buf))
    return bytes(buf)


class RcclComm:
    """An RCCL communicator (ncclComm_t) made by the library (exacto_rccl_comm_init) on `device`."""

    def __init__(self, nranks: int, uid: bytes, rank: int, device: int = 0):
        lib = load()
        buf = (C.c_uint8 * 128).from_buffer_copy(uid)
        h = C.c_void_p()
        check(lib.exacto_rccl_comm_init(C.byref(h), nranks, buf, rank, device))
        self._h, self._lib, self.nranks, self.rank = h, lib, nranks, rank

    @property
    def handle(self):
        return self._h

    def count(self) -> int:
        """ncclCommCount of the library's communicator: the ranks RCCL itself spans."""
        v = C.c_int(0)
        check(self._lib.exacto_rccl_comm_count(self._h, C.byref(v)))
        return v.value

    def close(self):
        if self._h:
            check(self._lib.exacto_rccl_comm_destroy(self._h))
            self._h = None


def required_trace_elements(n: int) -> list[int]:
    """coeffs_to_slots.rs:168-183 (host-only entry point of the library; no GPU needed)."""
    lib = load()
    count = lib.exacto_required_trace_elements(n, None, 0)
    out = (C.c_uint64 * max(count, 1))()
    lib.exacto_required_trace_elements(n, out, count)
    return [int(v) for v in out[:count]]


def _ptr(a) -> int | None:
    """Pointer of a numpy array (host) or a torch tensor (device or host)."""
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        assert a.flags["C_CONTIGUOUS"]
        return a.ctypes.data
    return a.data_ptr()  # torch.Tensor


def _u64(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.uint64))


class HipContext:
    """One device context = BfvParams (+ RnsBasis/NTT plans) on a GPU (exacto_ctx_create)."""

    def __init__(self, ring_degree: int, ct_moduli, aux_moduli=(), plain_modulus: int = 65537,
                 gadget_base: int = 0, device: int = 0):
        lib = load()
        ct = _u64(list(ct_moduli))
        aux = _u64(list(aux_moduli)) if len(aux_moduli) else None
        h = C.c_void_p()
        check(lib.exacto_ctx_create(C.byref(h), ring_degree, ct.ctypes.data, len(ct),
                                    aux.ctypes.data if aux is not None else None,
                                    0 if aux is None else len(aux), plain_modulus, gadget_base,
                                    device))
        self._h = h
        self._lib = lib
        info = CtxInfo()
        check(lib.exacto_ctx_get_info(h, C.byref(info)))
        self.n = info.ring_degree
        self.L = info.num_ct_moduli
        self.G = info.gadget_digits
        self.gadget_base = info.gadget_base
        self.path = info.mul_path
        self.num_internal_aux = info.num_internal_aux
        self.ks32_primes = info.ks32_primes
        self.psum_max = info.psum_max
        self.ct_moduli = [int(q) for q in ct_moduli]
        self.plain_modulus = int(info.plain_modulus)
        # the NTT-domain storage order this binding was written for (exacto_hip.h EXACTO_NTT_ORDER): keys and
        # ciphertexts kept from a library of another order would give wrong results silently
        if info.ntt_order != NTT_ORDER:
            raise RuntimeError(f"libexacto_hip uses NTT-domain order {info.ntt_order}, this binding expects {NTT_ORDER}")

    @property
    def ks32_lazy(self) -> bool:
        """The resident relinearisation key runs in the lazy 31-bit basis (decided at its first use)."""
        info = CtxInfo()
        check(self._lib.exacto_ctx_get_info(self._h, C.byref(info)))
        return bool(info.ks32_lazy)

    @property
    def dbfv_key_switch(self) -> int:
        """The last dbfv_mul's key switch: 1 summed digits (primary 31-bit basis), 2 summed (wide basis),
        0 per product, -1 none yet (exacto_ctx_info.dbfv_key_switch)."""
        info = CtxInfo()
        check(self._lib.exacto_ctx_get_info(self._h, C.byref(info)))
        return int(info.dbfv_key_switch)

    @classmethod
    def from_params(cls, params, device=0):
        """Build from an oracle-style / exacto_amd.params BfvParams object."""
        aux = params.aux_basis.moduli if params.aux_basis is not None else []
        return cls(params.ring_degree, params.ct_basis.moduli, aux, params.plain_modulus,
                   params.gadget_base, device)

    def close(self):
        if self._h:
            self._lib.exacto_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    # ---- configuration
    def set_stream(self, stream_handle: int | None):
        """Enqueue on this hipStream_t handle (0/None = the default stream)."""
        check(self._lib.exacto_ctx_set_stream(self._h, stream_handle or None))

    def set_chunk(self, chunk: int):
        check(self._lib.exacto_ctx_set_chunk(self._h, chunk))

    def synchronize(self):
        check(self._lib.exacto_synchronize(self._h))

    # ---- relinearisation key
    def load_relin_key(self, rlk: np.ndarray):
        rlk = _u64(rlk)
        nk = rlk.shape[0] if rlk.ndim == 4 else 0
        check(self._lib.exacto_ctx_load_relin_key(self._h, rlk.ctypes.data if nk else None, nk))

    def load_relin_key_dev(self, rlk_dev, num_keys: int):
        check(self._lib.exacto_ctx_load_relin_key_dev(self._h, _ptr(rlk_dev), num_keys))

    def relin_key_buffer(self, num_keys: int) -> int:
        p = self._lib.exacto_ctx_relin_key_buffer(self._h, num_keys)
        if not p:
            raise ExactoError(100, last_error())
        return p

    # ---- host-pointer API (synchronous, numpy uint64)
    def ntt_fwd(self, polys: np.ndarray, limb: int = 0) -> np.ndarray:
        a = _u64(polys).copy()
        check(self._lib.exacto_ntt_fwd(self._h, a.ctypes.data, a.size // self.n, limb))
        return a

    def ntt_inv(self, polys: np.ndarray, limb: int = 0) -> np.ndarray:
        a = _u64(polys).copy()
        check(self._lib.exacto_ntt_inv(self._h, a.ctypes.data, a.size // self.n, limb))
        return a

    def bfv_mul_no_relin(self, ct1: np.ndarray, ct2: np.ndarray) -> np.ndarray:
        ct1, ct2 = _u64(ct1), _u64(ct2)
        B = ct1.shape[0]
        out = np.zeros((B, 3, self.L, self.n), dtype=np.uint64)
        check(self._lib.exacto_bfv_mul_no_relin(self._h, ct1.ctypes.data, ct1.shape[1],
                                                ct2.ctypes.data, ct2.shape[1], out.ctypes.data, B))
        return out

    def relinearize(self, ct: np.ndarray) -> np.ndarray:
        ct = _u64(ct)
        B, polys = ct.shape[0], ct.shape[1]
        out = np.zeros((B, polys if polys < 3 else 2, self.L, self.n), dtype=np.uint64)
        check(self._lib.exacto_relinearize(self._h, ct.ctypes.data, polys, out.ctypes.data, B))
        return out

    def bfv_mul_and_relin(self, ct1: np.ndarray, ct2: np.ndarray) -> np.ndarray:
        ct1, ct2 = _u64(ct1), _u64(ct2)
        B = ct1.shape[0]
        out = np.zeros((B, 2, self.L, self.n), dtype=np.uint64)
        check(self._lib.exacto_bfv_mul_and_relin(self._h, ct1.ctypes.data, ct2.ctypes.data,
                                                 out.ctypes.data, B))
        return out

    def _addsub(self, fn, ct1, ct2):
        ct1, ct2 = _u64(ct1), _u64(ct2)
        B = ct1.shape[0]
        out = np.zeros((B, max(ct1.shape[1], ct2.shape[1]), self.L, self.n), dtype=np.uint64)
        check(fn(self._h, ct1.ctypes.data, ct1.shape[1], ct2.ctypes.data, ct2.shape[1], out.ctypes.data, B))
        return out

    def bfv_add(self, ct1: np.ndarray, ct2: np.ndarray) -> np.ndarray:
        """eval.rs:14-31 batched: ct1 [B][p1][L][n] + ct2 [B][p2][L][n] -> [B][max][L][n]."""
        return self._addsub(self._lib.exacto_bfv_add, ct1, ct2)

    def bfv_sub(self, ct1: np.ndarray, ct2: np.ndarray) -> np.ndarray:
        """eval.rs:34-51 batched (ct2's extra components negated)."""
        return self._addsub(self._lib.exacto_bfv_sub, ct1, ct2)

    def bfv_neg(self, ct: np.ndarray) -> np.ndarray:
        """eval.rs:54-60 batched."""
        ct = _u64(ct)
        out = np.zeros_like(ct)
        check(self._lib.exacto_bfv_neg(self._h, ct.ctypes.data, ct.shape[1], out.ctypes.data, ct.shape[0]))
        return out

    def dbfv_mul(self, d, base, plain, a: np.ndarray, b: np.ndarray, depth_a=None, depth_b=None):
        a, b = _u64(a), _u64(b)
        B = a.shape[0]
        out = np.zeros_like(a)
        da = np.ascontiguousarray(depth_a, dtype=np.uint32) if depth_a is not None else None
        db = np.ascontiguousarray(depth_b, dtype=np.uint32) if depth_b is not None else None
        dout = np.zeros(B, dtype=np.uint32)
        check(self._lib.exacto_dbfv_mul(self._h, d, base, plain, a.ctypes.data, b.ctypes.data,
                                        out.ctypes.data, B, _ptr(da), _ptr(db), dout.ctypes.data))
        return out, dout

    def dbfv_mul_chain(self, d, base, plain, x: np.ndarray, y: np.ndarray, depth: int):
        """paper_repro.rs:203-236 chain: x * y^depth, mul_depth reset before every step."""
        x, y = _u64(x), _u64(y)
        out = np.zeros_like(x)
        check(self._lib.exacto_dbfv_mul_chain(self._h, d, base, plain, x.ctypes.data, y.ctypes.data,
                                              out.ctypes.data, x.shape[0], depth))
        return out

    def bfv_decrypt(self, ct: np.ndarray, sk: np.ndarray) -> np.ndarray:
        """encrypt.rs:111-178 batched: ct [B][polys][L][n], sk [L][n] (NTT) -> [B][n] mod p."""
        ct, sk = _u64(ct), _u64(sk)
        out = np.zeros((ct.shape[0], ct.shape[-1]), dtype=np.uint64)
        check(self._lib.exacto_bfv_decrypt(self._h, ct.ctypes.data, ct.shape[1], sk.ctypes.data,
                                           out.ctypes.data, ct.shape[0]))
        return out

    def dbfv_decrypt(self, d, base, plain, ct: np.ndarray, sk: np.ndarray) -> np.ndarray:
        """dbfv/decrypt.rs:20-43: ct [B][d][2][L][n] -> [B] scalars."""
        ct, sk = _u64(ct), _u64(sk)
        out = np.zeros(ct.shape[0], dtype=np.uint64)
        check(self._lib.exacto_dbfv_decrypt(self._h, d, base, plain, ct.ctypes.data, sk.ctypes.data,
                                            out.ctypes.data, ct.shape[0]))
        return out

    def dbfv_decrypt_poly(self, d, base, plain, ct: np.ndarray, sk: np.ndarray) -> np.ndarray:
        """dbfv/decrypt.rs:48-79: ct [B][d][2][L][n] -> [B][n] mod p."""
        ct, sk = _u64(ct), _u64(sk)
        out = np.zeros((ct.shape[0], ct.shape[-1]), dtype=np.uint64)
        check(self._lib.exacto_dbfv_decrypt_poly(self._h, d, base, plain, ct.ctypes.data, sk.ctypes.data,
                                                 out.ctypes.data, ct.shape[0]))
        return out

    # ---- key generation / encryption (keygen.rs:64-162, encrypt.rs:29-106); key = 4 u64 words
    @staticmethod
    def _key(key):
        k = _u64(key).reshape(-1)
        if k.size != 4:
            raise ValueError("key must be 4 64-bit words")
        return k

    def gen_secret_key(self, key, stream=0) -> np.ndarray:
        k = self._key(key)
        sk = np.zeros((self.L, self.n), dtype=np.uint64)
        check(self._lib.exacto_gen_secret_key(self._h, k.ctypes.data, stream, sk.ctypes.data))
        return sk

    def gen_public_key(self, sk, key, stream=0, sigma=3.2) -> np.ndarray:
        k, sk = self._key(key), _u64(sk)
        pk = np.zeros((2, self.L, self.n), dtype=np.uint64)
        check(self._lib.exacto_gen_public_key(self._h, sk.ctypes.data, sigma, k.ctypes.data, stream, pk.ctypes.data))
        return pk

    def gen_relin_key(self, sk, key, stream=0, sigma=3.2, num_keys=None, resident=False):
        """resident=True: generate into the context's resident key (returns None)."""
        k, sk = self._key(key), _u64(sk)
        nk = self.G if num_keys is None else num_keys
        if resident:
            check(self._lib.exacto_gen_relin_key(self._h, sk.ctypes.data, sigma, k.ctypes.data, stream, nk, None))
            return None
        rlk = np.zeros((nk, 2, self.L, self.n), dtype=np.uint64)
        check(self._lib.exacto_gen_relin_key(self._h, sk.ctypes.data, sigma, k.ctypes.data, stream, nk,
                                             rlk.ctypes.data))
        return rlk

    def encrypt_sk(self, pt, sk, key, stream=0, sigma=3.2) -> np.ndarray:
        """pt [B][n] plaintext coefficients -> ct [B][2][L][n]."""
        k, pt, sk = self._key(key), _u64(pt), _u64(sk)
        ct = np.zeros((pt.shape[0], 2, self.L, self.n), dtype=np.uint64)
        check(self._lib.exacto_encrypt_sk(self._h, pt.ctypes.data, sk.ctypes.data, sigma, k.ctypes.data, stream,
                                          ct.ctypes.data, pt.shape[0]))
        return ct

    def encrypt_pk(self, pt, pk, key, stream=0, sigma=3.2) -> np.ndarray:
        k, pt, pk = self._key(key), _u64(pt), _u64(pk)
        ct = np.zeros((pt.shape[0], 2, self.L, self.n), dtype=np.uint64)
        check(self._lib.exacto_encrypt_pk(self._h, pt.ctypes.data, pk.ctypes.data, sigma, k.ctypes.data, stream,
                                          ct.ctypes.data, pt.shape[0]))
        return ct

    def gen_galois_key(self, sk, element, key, stream=0, sigma=3.2, num_keys=None) -> np.ndarray:
        """keygen.rs:171-209 -> [num_keys][2][L][n]."""
        k, sk = self._key(key), _u64(sk)
        nk = self.G if num_keys is None else num_keys
        gk = np.zeros((nk, 2, self.L, self.n), dtype=np.uint64)
        check(self._lib.exacto_gen_galois_key(self._h, sk.ctypes.data, element, sigma, k.ctypes.data, stream, nk,
                                              gk.ctypes.data))
        return gk

    def bfv_apply_automorphism(self, ct, element, gk) -> np.ndarray:
        """eval.rs:512-561 batched: ct [B][2][L][n], gk [K][2][L][n] -> [B][2][L][n]."""
        ct, gk = _u64(ct), _u64(gk)
        out = np.zeros((ct.shape[0], 2, self.L, self.n), dtype=np.uint64)
        check(self._lib.exacto_bfv_apply_automorphism(self._h, ct.ctypes.data, ct.shape[1], element,
                                                      gk.ctypes.data if gk.size else None, gk.shape[0],
                                                      out.ctypes.data, ct.shape[0]))
        return out

    def required_trace_elements(self, n=None) -> list[int]:
        return required_trace_elements(self.n if n is None else n)

    def gen_trace_galois_keys(self, sk, key, stream=0, elements=None, sigma=3.2):
        """gen_trace_galois_keys / gen_all_galois_keys (coeffs_to_slots.rs:151-197): one key per element,
        element e on ChaCha stream `stream + e`.  Returns (elements, gks [E][G][2][L][n])."""
        els = self.required_trace_elements() if elements is None else list(elements)
        gks = np.stack([self.gen_galois_key(sk, k, key, stream=stream + e, sigma=sigma) for e, k in enumerate(els)])
        return els, gks

    def extract_coefficients(self, ct, j0, count, elements, gks) -> np.ndarray:
        """coeffs_to_slots.rs:21-49 for j0 .. j0+count-1: ct [2][L][n] -> [count][2][L][n]."""
        ct = _u64(ct)
        el = np.ascontiguousarray(np.asarray(elements, dtype=np.uint64))
        gks = _u64(gks)
        E = el.shape[0]
        out = np.zeros((count, 2, self.L, self.n), dtype=np.uint64)
        check(self._lib.exacto_extract_coefficients(self._h, ct.ctypes.data, j0, count, el.ctypes.data if E else None,
                                                    E, gks.ctypes.data if E else None, gks.shape[1] if E else 0,
                                                    out.ctypes.data))
        return out

    def extract_coefficient(self, ct, j, elements, gks) -> np.ndarray:
        return self.extract_coefficients(ct, j, 1, elements, gks)[0]

    def coeffs_to_slots(self, ct, elements, gks) -> np.ndarray:
        """coeffs_to_slots.rs:103-115: all n coefficients, the n shifted copies traced together."""
        return self.extract_coefficients(ct, 0, self.n, elements, gks)

    def slots_to_coeffs(self, slots) -> np.ndarray:
        """coeffs_to_slots.rs:121-145: slots [S][polys][L][n] -> [polys][L][n]."""
        slots = _u64(slots)
        S = slots.shape[0]
        polys = slots.shape[1] if S else 2
        out = np.zeros((polys, self.L, self.n), dtype=np.uint64)
        check(self._lib.exacto_slots_to_coeffs(self._h, slots.ctypes.data, S, polys, out.ctypes.data))
        return out

    def trivial_encrypt_poly(self, pt) -> np.ndarray:
        """digit_extract.rs:179-189 batched: pt [B][n] -> (Delta m, 0) [B][2][L][n]."""
        pt = _u64(pt)
        pt = pt.reshape(-1, self.n)
        out = np.zeros((pt.shape[0], 2, self.L, self.n), dtype=np.uint64)
        check(self._lib.exacto_trivial_encrypt(self._h, pt.ctypes.data, out.ctypes.data, pt.shape[0]))
        return out

    def trivial_encrypt(self, values) -> np.ndarray:
        """digit_extract.rs:160-176 for each scalar m of `values`: (Delta (m mod t), 0)."""
        vals = [int(v) for v in np.atleast_1d(values)]
        pt = np.zeros((len(vals), self.n), dtype=np.uint64)
        pt[:, 0] = [v % self.plain_modulus for v in vals]
        return self.trivial_encrypt_poly(pt)

    def eval_poly(self, ct, coeffs) -> np.ndarray:
        """digit_extract.rs:101-157 on a batch ct [B][2][L][n]; needs the resident relin key."""
        ct = _u64(ct)
        cf = np.ascontiguousarray(np.asarray(coeffs, dtype=np.uint64))
        out = np.zeros_like(ct)
        check(self._lib.exacto_eval_poly(self._h, ct.ctypes.data, cf.ctypes.data if cf.size else None, cf.size,
                                         out.ctypes.data, ct.shape[0]))
        return out

    def _pt(self, pt, rows):
        pt = _u64(pt).reshape(rows, self.n)
        return pt

    def bfv_plain_mul(self, ct, pt) -> np.ndarray:
        """eval.rs:468-486 batched: ct [B][polys][L][n], pt [B][n] -> [B][polys][L][n]."""
        ct = _u64(ct)
        pt = self._pt(pt, ct.shape[0])
        out = np.zeros_like(ct)
        check(self._lib.exacto_bfv_plain_mul(self._h, ct.ctypes.data, ct.shape[1], pt.ctypes.data, out.ctypes.data,
                                             ct.shape[0]))
        return out

    def bfv_plain_add(self, ct, pt) -> np.ndarray:
        """eval.rs:489-503 batched: c0 + Delta m."""
        ct = _u64(ct)
        pt = self._pt(pt, ct.shape[0])
        out = np.zeros_like(ct)
        check(self._lib.exacto_bfv_plain_add(self._h, ct.ctypes.data, ct.shape[1], pt.ctypes.data, out.ctypes.data,
                                             ct.shape[0]))
        return out

    def bfv_inner_product(self, cts, pts) -> np.ndarray:
        """eval.rs:588-606: cts [K][polys][L][n], pts [K][n] -> [polys][L][n]."""
        cts = _u64(cts)
        K = cts.shape[0]
        pts = _u64(pts).reshape(K, self.n) if K else _u64(pts)
        polys = cts.shape[1] if K else 2
        out = np.zeros((polys, self.L, self.n), dtype=np.uint64)
        check(self._lib.exacto_bfv_inner_product(self._h, cts.ctypes.data, pts.ctypes.data, K, polys,
                                                 out.ctypes.data))
        return out

    def bfv_monomial_mul(self, ct, j) -> np.ndarray:
        """eval.rs:613-652 batched: X^j * ct."""
        ct = _u64(ct)
        out = np.zeros_like(ct)
        check(self._lib.exacto_bfv_monomial_mul(self._h, ct.ctypes.data, ct.shape[1], j, out.ctypes.data,
                                                ct.shape[0]))
        return out

    def bfv_trace(self, ct, elements, gks) -> np.ndarray:
        """eval.rs:572-586 batched: elements [E], gks [E][K][2][L][n] (the key of elements[e] at e)."""
        ct = _u64(ct)
        el = np.ascontiguousarray(np.asarray(elements, dtype=np.uint64))
        gks = _u64(gks)
        E = el.shape[0]
        nk = gks.shape[1] if E else 0
        out = np.zeros_like(ct)
        check(self._lib.exacto_bfv_trace(self._h, ct.ctypes.data, ct.shape[1], el.ctypes.data if E else None, E,
                                         gks.ctypes.data if E else None, nk, out.ctypes.data, ct.shape[0]))
        return out

    def gen_relin_key_dev(self, sk, key, stream, num_keys, rlk=None, sigma=3.2):
        k = self._key(key)
        check(self._lib.exacto_gen_relin_key_dev(self._h, self._p(sk), sigma, k.ctypes.data, stream, num_keys,
                                                 None if rlk is None else self._p(rlk)))

    def encrypt_sk_dev(self, pt, sk, key, stream, ct, batch, sigma=3.2):
        k = self._key(key)
        check(self._lib.exacto_encrypt_sk_dev(self._h, self._p(pt), self._p(sk), sigma, k.ctypes.data, stream,
                                              self._p(ct), batch))

    # ---- device-pointer API (asynchronous; torch tensors or raw ints)
    def _p(self, x):
        return x if isinstance(x, int) else _ptr(x)

    def ntt_fwd_dev(self, polys, count, limb=0):
        check(self._lib.exacto_ntt_fwd_dev(self._h, self._p(polys), count, limb))

    def ntt_inv_dev(self, polys, count, limb=0):
        check(self._lib.exacto_ntt_inv_dev(self._h, self._p(polys), count, limb))

    def rns_fwd_dev(self, polys, count):
        check(self._lib.exacto_rns_fwd_dev(self._h, self._p(polys), count))

    def rns_inv_dev(self, polys, count):
        check(self._lib.exacto_rns_inv_dev(self._h, self._p(polys), count))

    def rns_add_dev(self, a, b, out, count):
        check(self._lib.exacto_rns_add_dev(self._h, self._p(a), self._p(b), self._p(out), count))

    def rns_sub_dev(self, a, b, out, count):
        check(self._lib.exacto_rns_sub_dev(self._h, self._p(a), self._p(b), self._p(out), count))

    def rns_neg_dev(self, a, out, count):
        check(self._lib.exacto_rns_neg_dev(self._h, self._p(a), self._p(out), count))

    def rns_mul_dev(self, a, b, out, count):
        check(self._lib.exacto_rns_mul_dev(self._h, self._p(a), self._p(b), self._p(out), count))

    def rns_mul_inv_dev(self, a, b, out, count):
        """INTT(a (.) b) per limb, fused (exacto_rns_mul_inv_dev)."""
        check(self._lib.exacto_rns_mul_inv_dev(self._h, self._p(a), self._p(b), self._p(out), count))

    def rns_polymul_dev(self, a, b, out, count):
        """Negacyclic products of coefficient-domain polys (exacto_rns_polymul_dev)."""
        check(self._lib.exacto_rns_polymul_dev(self._h, self._p(a), self._p(b), self._p(out), count))

    def rns_scalar_mul_dev(self, a, scalar, out, count):
        check(self._lib.exacto_rns_scalar_mul_dev(self._h, self._p(a), scalar, self._p(out), count))

    def bfv_add_dev(self, a, polys1, b, polys2, out, batch):
        check(self._lib.exacto_bfv_add_dev(self._h, self._p(a), polys1, self._p(b), polys2, self._p(out), batch))

    def bfv_sub_dev(self, a, polys1, b, polys2, out, batch):
        check(self._lib.exacto_bfv_sub_dev(self._h, self._p(a), polys1, self._p(b), polys2, self._p(out), batch))

    def bfv_neg_dev(self, a, polys, out, batch):
        check(self._lib.exacto_bfv_neg_dev(self._h, self._p(a), polys, self._p(out), batch))

    def bfv_mul_no_relin_dev(self, ct1, ct2, out, batch):
        check(self._lib.exacto_bfv_mul_no_relin_dev(self._h, self._p(ct1), 2, self._p(ct2), 2,
                                                    self._p(out), batch))

    def relinearize_dev(self, ct, polys, out, batch):
        check(self._lib.exacto_relinearize_dev(self._h, self._p(ct), polys, self._p(out), batch))

    def bfv_mul_and_relin_dev(self, ct1, ct2, out, batch):
        check(self._lib.exacto_bfv_mul_and_relin_dev(self._h, self._p(ct1), self._p(ct2),
                                                     self._p(out), batch))

    def bfv_apply_automorphism_dev(self, ct, element, gk, num_keys, out, batch):
        check(self._lib.exacto_bfv_apply_automorphism_dev(self._h, self._p(ct), 2, element, self._p(gk), num_keys,
                                                          self._p(out), batch))

    def gadget_decompose_dev(self, coeffs, digits, batch, num_digits):
        check(self._lib.exacto_gadget_decompose_dev(self._h, self._p(coeffs), self._p(digits),
                                                    batch, num_digits))

    def dbfv_mul_dev(self, d, base, plain, a, b, out, batch, depth_a=None, depth_b=None):
        da = np.ascontiguousarray(depth_a, dtype=np.uint32) if depth_a is not None else None
        db = np.ascontiguousarray(depth_b, dtype=np.uint32) if depth_b is not None else None
        check(self._lib.exacto_dbfv_mul_dev(self._h, d, base, plain, self._p(a), self._p(b),
                                            self._p(out), batch, _ptr(da), _ptr(db), None))

    def dbfv_mul_limbs(self, d, base, plain, a: np.ndarray, b: np.ndarray, limbs) -> np.ndarray:
        """One GPU's output limbs of a split dbfv_mul: [B][len(limbs)][2][L][n], slot s = limb limbs[s]."""
        a, b = _u64(a), _u64(b)
        ls = np.ascontiguousarray(np.asarray(limbs, dtype=np.uint32))
        out = np.zeros((a.shape[0], ls.size, 2, self.L, self.n), dtype=np.uint64)
        check(self._lib.exacto_dbfv_mul_limbs(self._h, d, base, plain, a.ctypes.data, b.ctypes.data, out.ctypes.data,
                                              a.shape[0], ls.ctypes.data if ls.size else None, ls.size))
        return out

    def dbfv_mul_limbs_dev(self, d, base, plain, a, b, out, batch, limbs):
        ls = np.ascontiguousarray(np.asarray(limbs, dtype=np.uint32))
        check(self._lib.exacto_dbfv_mul_limbs_dev(self._h, d, base, plain, self._p(a), self._p(b), self._p(out),
                                                  batch, ls.ctypes.data if ls.size else None, ls.size))

    # ---- RCCL collectives (exacto_hip.h; comm = RcclComm)
    def broadcast_relin_key(self, comm: "RcclComm", root: int, num_keys: int):
        """Root's resident relinearisation key -> this context's resident key (ncclBroadcast, in place)."""
        check(self._lib.exacto_ctx_broadcast_relin_key(self._h, comm.handle, root, num_keys))

    def broadcast_galois_key(self, comm: "RcclComm", root: int, gk_dev, num_keys: int):
        check(self._lib.exacto_broadcast_galois_key(self._h, comm.handle, root, self._p(gk_dev), num_keys))

    def allgather_u64(self, comm: "RcclComm", send, recv, count: int):
        """recv = [nranks][count] u64 (ncclAllGather on the context stream)."""
        check(self._lib.exacto_rccl_allgather_u64(self._h, comm.handle, self._p(send), self._p(recv), count))

    def rccl_sync(self, comm: "RcclComm"):
        """Wait for the collectives on the context stream, at most $EXACTO_RCCL_TIMEOUT_S seconds
        (exacto_rccl_sync); raises ExactoError on expiry (the communicator is then aborted)."""
        check(self._lib.exacto_rccl_sync(self._h, comm.handle))

    def dbfv_mul_chain_dev(self, d, base, plain, x, y, out, batch, depth):
        check(self._lib.exacto_dbfv_mul_chain_dev(self._h, d, base, plain, self._p(x), self._p(y),
                                                  self._p(out), batch, depth))

    def bfv_decrypt_dev(self, ct, polys, sk, out, batch):
        check(self._lib.exacto_bfv_decrypt_dev(self._h, self._p(ct), polys, self._p(sk), self._p(out), batch))

    def dbfv_decrypt_dev(self, d, base, plain, ct, sk, out, batch, poly=False):
        fn = self._lib.exacto_dbfv_decrypt_poly_dev if poly else self._lib.exacto_dbfv_decrypt_dev
        check(fn(self._h, d, base, plain, self._p(ct), self._p(sk), self._p(out), batch))

    # ---- profiling
    def prof_enable(self, on=True):
        check(self._lib.exacto_prof_enable(self._h, 1 if on else 0))

    def prof_read(self, kind: int):
        nl, pl = C.c_uint64(), C.c_uint64()
        ms, by = C.c_double(), C.c_double()
        check(self._lib.exacto_prof_read(self._h, kind, C.byref(nl), C.byref(ms), C.byref(by),
                                         C.byref(pl)))
        return {"launches": nl.value, "ms": ms.value, "bytes": by.value, "polys": pl.value}

    def prof_kernels(self, kind: int) -> list[tuple[str, int, float]]:
        """The kernels that ran for family `kind` in the records prof_read consumed, as rocprofv3 names
        them, by descending time: [(name, launches, ms)] (exacto_prof_kernels)."""
        n = self._lib.exacto_prof_kernels(self._h, kind, None, 0)
        buf = C.create_string_buffer(n + 1)
        self._lib.exacto_prof_kernels(self._h, kind, buf, n + 1)
        out = []
        for part in filter(None, buf.value.decode().split("; ")):
            name, _, tail = part.rpartition(" (")
            cnt, ms = tail.rstrip(")").split(", ")
            out.append((name, int(cnt), float(ms.split()[0])))
        return out
