"""Every selection switch the library reads gives bit-identical results: each alternative kernel or
path computes the same outputs as the default selection.

The switches are read once per process, so each variant runs tests/variant_digest.py in a child
process (sequentially, one GPU process at a time) over the case groups the switch affects, and the
digests are compared with the default's.  The default selection itself is pinned to the oracle by
the rest of the suite (test_gpu_golden.py digests, test_gpu_published.py, test_gpu_ntt.py,
test_gpu_psum.py); bit-exact, integer work.

Not listed (no effect on results): EXACTO_SCRATCH_POOL / EXACTO_DEBUG_SCRATCH / EXACTO_DEBUG_FILL /
EXACTO_LEAK_CTX (allocation diagnostics, tools/diag.sh), EXACTO_DEBUG_BOOT / EXACTO_DEBUG_WATCH /
EXACTO_DEBUG_ALLOC (bootstrap snapshots, write watch, allocation log), EXACTO_DBFV_GROUP_MB (tests/test_gpu_psum.py runs it),
EXACTO_PROF_RAW (profiling arithmetic), EXACTO_RCCL_LIB (library path), EXACTO_RCCL_TIMEOUT_S (collective deadline).
"""

import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
# name: (environment, case groups of tests/variant_digest.py)
VARIANTS = {
    "tensor_pin_both": ({"EXACTO_TENSOR_PIN": "1"}, ["cfg3", "cfg4"]),
    "tensor_pin_none": ({"EXACTO_TENSOR_PIN": "0"}, ["cfg5"]),
    "ntt_asm_off": ({"EXACTO_NTT_ASM": "0"}, ["cfg3", "cfg5", "hps"]),
    "ntt_asm_inv_off": ({"EXACTO_NTT_ASM_INV": "0"}, ["cfg3", "cfg5", "hps"]),
    "ntt_gen_off": ({"EXACTO_NTT_GEN": "0"}, ["hps"]),
    "ntt_genq_off": ({"EXACTO_NTT_GENQ": "0"}, ["hps"]),
    # no asm at all: the special primes then take the C++ rounds too (with NTT_ASM=0 alone they take
    # the generic-prime asm rounds)
    "ntt_asm_gen_off": ({"EXACTO_NTT_ASM": "0", "EXACTO_NTT_GEN": "0"}, ["cfg3", "hps"]),
    "one_lane": ({"EXACTO_DUAL_STREAM": "0"}, ["cfg3", "cfg5"]),
    "three_lanes": ({"EXACTO_LANES": "3"}, ["cfg3"]),
    "share_ext_off": ({"EXACTO_SHARE_EXT": "0"}, ["cfg4", "cfg5", "hps"]),
    "digit16_off": ({"EXACTO_DIGIT16": "0"}, ["cfg3", "cfg4"]),
    "digit8_off": ({"EXACTO_DIGIT8": "0"}, ["cfg5", "hps"]),
    "ks32_off": ({"EXACTO_KS32": "0"}, ["cfg3", "cfg4", "cfg5"]),
    "ks32_wide_off": ({"EXACTO_KS32_WIDE": "0"}, ["cfg4"]),
    "ks32_lazy_off": ({"EXACTO_KS32_LAZY": "0"}, ["cfg3", "cfg4", "cfg5"]),
    "ks32_wide_primary": ({"EXACTO_KS32_WIDE": "2"}, ["cfg3", "cfg4"]),
    "psum_off": ({"EXACTO_PSUM": "0"}, ["cfg4", "cfg5"]),
    # Garner over P instead of the rounded-float CRT in the SP scale and psum kernels
    "fp_crt_off": ({"EXACTO_FP_CRT": "0"}, ["cfg3", "cfg4", "cfg5"]),
    # Garner over Q for s = [p T]_Q in those kernels, and the float sum with a 1/4 band (about half the
    # coefficients then take the Garner fallback inside the same launch)
    "fpq_off": ({"EXACTO_FPQ": "0"}, ["cfg3", "cfg4", "cfg5"]),
    "fpq_band": ({"EXACTO_FPQ": "2"}, ["cfg3", "cfg4", "cfg5"]),
    # ... and in the 31-bit key switch's lift (ks32_crt)
    "ks_fpc_off": ({"EXACTO_KS_FPC": "0"}, ["cfg3", "cfg4", "cfg5"]),
    # a dBFV batch (dbfv_mul, chain) on one stream instead of two halves (the twin context)
    "chain_split_off": ({"EXACTO_CHAIN_SPLIT": "0"}, ["cfg4", "cfg5", "hps"]),
    "dot30_off": ({"EXACTO_DOT30": "0"}, ["cfg3", "cfg5"]),
    "xcd_remap_off": ({"EXACTO_XCD_REMAP": "0"}, ["cfg3", "cfg5"]),
    "mac_lds_off": ({"EXACTO_MAC_LDS": "0"}, ["hps"]),
    # HPS: the literal i128 scale against the division-free one, per-product relinearisation against
    # dbfv_mul's per-limb digit sums
    "hps_literal": ({"EXACTO_HPS_LITERAL": "1"}, ["hps"]),
    "hps_per_product": ({"EXACTO_HPS_SUM": "0"}, ["hps"]),
}
SWITCHES = sorted({k for env, _ in VARIANTS.values() for k in env})


def _digests(extra_env, groups):
    env = dict(os.environ)
    for k in SWITCHES:
        env.pop(k, None)
    env.update(extra_env)
    r = subprocess.run([sys.executable, os.path.join(HERE, "variant_digest.py"), *groups], env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout + r.stderr
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.fixture(scope="module")
def default_digests(gpu_available):
    return _digests({}, [])


def test_every_library_switch_is_covered():
    """Every runtime switch the library source reads is either a variant here or listed above as
    result-neutral."""
    import re
    src = os.path.join(os.path.dirname(HERE), "exacto_amd", "csrc")
    found = set()
    for f in os.listdir(src):
        if f.endswith((".hip", ".hpp")):
            with open(os.path.join(src, f)) as fh:
                found |= set(re.findall(r'(?:getenv|env_switch)\("(EXACTO_[A-Z0-9_]+)"', fh.read()))
    neutral = {"EXACTO_SCRATCH_POOL", "EXACTO_DEBUG_SCRATCH", "EXACTO_DEBUG_FILL", "EXACTO_DBFV_GROUP_MB",
               "EXACTO_PROF_RAW", "EXACTO_RCCL_LIB", "EXACTO_DEBUG_BOOT", "EXACTO_LEAK_CTX",
               "EXACTO_DEBUG_ALLOC", "EXACTO_DEBUG_WATCH", "EXACTO_RCCL_TIMEOUT_S"}
    assert found - neutral == set(SWITCHES), found ^ (set(SWITCHES) | neutral)


@pytest.mark.parametrize("name", sorted(VARIANTS))
def test_variant_matches_default(default_digests, name):
    env, groups = VARIANTS[name]
    got = _digests(env, groups)
    want = {k: v for k, v in default_digests.items() if k in got}
    assert got and got == want, {k: (got.get(k), v) for k, v in want.items() if got.get(k) != v}
