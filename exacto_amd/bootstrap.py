"""Bootstrapping host API — mirrors reference src/bootstrap/bfv_host.rs over the C ABI.

Everything here composes device entry points of libexacto_hip.so (no CPU arithmetic on the
ciphertexts): the key material and bfv_bootstrap are exacto_bootstrap_key_material and
exacto_bfv_bootstrap; keys come from the device samplers (ChaCha20 counter mode, see
csrc/keygen.hip), so they differ from the reference's ChaCha20Rng stream but have its
distributions.  The original scheme must use one ciphertext prime (the reference's modulus switch
reads moduli[0] after to_coeff_poly, bfv_host.rs:149-157).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import _ffi
from ._ffi import ExactoError, HipContext


@dataclass
class BootstrapKey:
    """bfv_host.rs:22-37."""
    bsk: np.ndarray              # [2][Lb][n], Enc_boot(s)
    boot: HipContext             # boot scheme context; its resident relin key is boot_rlk
    galois_elements: list[int]   # keys of galois_keys, in the order gks is stacked
    galois_keys: np.ndarray      # [E][G][2][Lb][n]
    rounding_poly: list[int]
    t_orig: int
    q_prime: int
    boot_sk: np.ndarray          # create_boot_sk (kept for tests / decryption under the boot scheme)


def gen_bootstrap_key(orig: HipContext, sk, boot: HipContext, q_prime: int, t_orig: int, key,
                      stream: int = 0) -> BootstrapKey:
    """gen_bootstrap_key (bfv_host.rs:49-124).  Streams stream .. stream+2+E are used for the bsk
    encryption, the boot relin key (made resident in `boot`) and the trace Galois keys."""
    boot_sk, s_pt = _ffi.bootstrap_key_material(orig, boot, sk)
    bsk = boot.encrypt_sk(s_pt[None], boot_sk, key, stream=stream)[0]
    boot.gen_relin_key(boot_sk, key, stream=stream + 1, resident=True)
    els, gks = boot.gen_trace_galois_keys(boot_sk, key, stream=stream + 2)
    rpoly = _ffi.compute_rounding_poly(t_orig, q_prime, boot.plain_modulus)
    return BootstrapKey(bsk, boot, els, gks, rpoly, t_orig, q_prime, boot_sk)


def bfv_bootstrap(orig: HipContext, ct, bsk: BootstrapKey) -> np.ndarray:
    """bfv_bootstrap (bfv_host.rs:131-205), batched: ct [B][2][1][n] -> [B][2][Lb][n]."""
    ct = np.asarray(ct, dtype=np.uint64)
    if ct.ndim == 3:
        return bfv_bootstrap(orig, ct[None], bsk)[0]
    return _ffi.bfv_bootstrap_raw(orig, bsk.boot, ct, bsk.bsk, bsk.rounding_poly, bsk.q_prime,
                                  bsk.galois_elements, bsk.galois_keys)


def dbfv_bootstrap(orig: HipContext, ct, bsk: BootstrapKey) -> np.ndarray:
    """dbfv_bootstrap (bfv_host.rs:213-236): every limb of ct [B][d][2][1][n] refreshed, all B*d
    limbs in one batched call; mul_depth restarts at 0 (the caller's depth counters)."""
    ct = np.asarray(ct, dtype=np.uint64)
    B, d = ct.shape[:2]
    out = bfv_bootstrap(orig, ct.reshape(B * d, *ct.shape[2:]), bsk)
    return out.reshape(B, d, *out.shape[1:])


def dbfv_mul_then_bootstrap(orig: HipContext, d: int, base: int, plain: int, a, b, bsk: BootstrapKey):
    """dbfv_mul_then_bootstrap (bfv_host.rs:242-250): returns (refreshed [B][d][2][Lb][n], depth 0s)."""
    prod, _ = orig.dbfv_mul(d, base, plain, a, b)
    out = dbfv_bootstrap(orig, prod, bsk)
    return out, np.zeros(out.shape[0], dtype=np.uint32)


def dbfv_mul_chain_then_bootstrap(orig: HipContext, d: int, base: int, plain: int, cts, bsk: BootstrapKey):
    """dbfv_mul_chain_then_bootstrap (bfv_host.rs:257-288) for chains whose inputs are all under the
    original parameters: the first product is taken under `orig` with its resident key, every later
    one under the boot scheme with boot_rlk (the reference's use_boot_rlk), each rhs refreshed first
    because its parameters differ from the accumulator's."""
    if len(cts) == 0:
        raise ExactoError(1, "invalid parameter: dbfv_mul_chain_then_bootstrap requires at least one ciphertext")
    acc = np.asarray(cts[0], dtype=np.uint64)
    on_boot = False
    for ct in cts[1:]:
        if not on_boot:
            acc, _ = dbfv_mul_then_bootstrap(orig, d, base, plain, acc, ct, bsk)
            on_boot = True
        else:
            rhs = dbfv_bootstrap(orig, ct, bsk)
            prod, _ = bsk.boot.dbfv_mul(d, base, plain, acc, rhs)
            acc = _boot_refresh(bsk, prod)
    return acc


def _boot_refresh(bsk: BootstrapKey, ct):
    """Refresh a dBFV ciphertext that already lives under the boot scheme: bootstrapping it takes the
    boot scheme as the original one (the reference's dbfv_bootstrap of a boot-parameter input)."""
    boot = bsk.boot
    if boot.L != 1:
        raise ExactoError(1, "invalid parameter: bootstrap requires a single-prime ciphertext modulus")
    return dbfv_bootstrap(boot, ct, bsk)
