"""The kernel-selection switches give bit-identical results: every A/B alternative that ships in
the library (the pinned-home forward / tensor / polymul kernels against the asm, pipe, tensor3 +
tensor_c2 and register-resident forms; the fused ks32 lift + forward kernels against the separate
ones) computes the same outputs as the default selection.

Each switch is read once per process, so each variant runs tests/variant_digest.py in a child
process (sequentially, one GPU process at a time) and the digests are compared with the default's.
The default selection itself is pinned to the oracle by the rest of the suite (test_gpu_golden.py
digests, test_gpu_ntt.py, test_gpu_psum.py); bit-exact, integer work.
"""

import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
VARIANTS = {
    "tensor_pin_both": {"EXACTO_TENSOR_PIN": "1"},
    "tensor_pin_none": {"EXACTO_TENSOR_PIN": "0"},
    "asm_fwd_and_pipe": {"EXACTO_FWD_PIN": "0", "EXACTO_NTT_PIPE": "1"},
    "polymul_pin": {"EXACTO_POLYMUL_PIN": "1"},
    "crt_fwd_pin": {"EXACTO_CRT_FWD": "4"},
    "crt_fwd_3waves": {"EXACTO_CRT_FWD": "3"},
    # HPS: the literal i128 scale against the division-free one, per-product relinearisation against
    # dbfv_mul's per-limb digit sums
    "hps_literal": {"EXACTO_HPS_LITERAL": "1"},
    "hps_per_product": {"EXACTO_HPS_SUM": "0"},
}


def _digests(extra_env):
    env = dict(os.environ)
    for k in ("EXACTO_TENSOR_PIN", "EXACTO_FWD_PIN", "EXACTO_NTT_PIPE", "EXACTO_POLYMUL_PIN", "EXACTO_TENSOR3",
              "EXACTO_CRT_FWD", "EXACTO_HPS_LITERAL", "EXACTO_HPS_SUM"):
        env.pop(k, None)
    env.update(extra_env)
    r = subprocess.run([sys.executable, os.path.join(HERE, "variant_digest.py")], env=env, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, r.stdout + r.stderr
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.fixture(scope="module")
def default_digests(gpu_available):
    return _digests({})


@pytest.mark.parametrize("name", sorted(VARIANTS))
def test_variant_matches_default(default_digests, name):
    got = _digests(VARIANTS[name])
    assert got == default_digests, {k: (got.get(k), v) for k, v in default_digests.items() if got.get(k) != v}
