"""CPU check of the generated forward / inverse NTT asm rounds (exacto_amd/csrc/ntt_asm.inc): a
one-lane simulation of every round's instruction sequence against exact modular butterflies
(Cooley-Tukey forward, Gentleman-Sande inverse with n^-1 folded into the last stage), at the
input bounds the rounds assume, for the approximate and the exact Shoup quotient
(tools/asm_sim.py), and the committed .inc is what the generator emits today."""

import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import asm_sim  # noqa: E402
import gen_ntt_asm  # noqa: E402


def test_rounds_match_exact_arithmetic():
    rng = random.Random(7)
    for approx in (True, False):
        for logn in (12, 13):
            for r in range((logn + 3) // 4):
                for i in range(15):
                    q = asm_sim.PRIMES[i % len(asm_sim.PRIMES)]
                    asm_sim.check_round(logn, r, q, rng, approx)
                    asm_sim.check_inv_round(logn, r, q, rng, approx)
                    asm_sim.check_round_pinned(logn, r, q, rng, approx)
                    asm_sim.check_inv_round_pinned(logn, r, q, rng, approx)
            # the tensor kernels' last round: outputs congruent and below 2q (bound_out = 2)
            r = (logn + 3) // 4 - 1
            for i in range(15):
                q = asm_sim.PRIMES[i % len(asm_sim.PRIMES)]
                asm_sim.check_inv_round(logn, r, q, rng, approx, lazy_out=True)
                asm_sim.check_inv_round_pinned(logn, r, q, rng, approx, lazy_out=True)
                asm_sim.check_round_pinned(logn, r, q, rng, approx, lazy_out=True)


def test_lane_pair_exchange_and_permuted_last_round():
    """n = 8192 forward: the last exchange within lane pairs by DPP (EXACTO_XCHG_PIN_LP, two lanes
    simulated with quad_perm [1, 0, 3, 2]) leaves the LO = 0 layout in the PERM_LP homes, and the last
    round over those homes (EXACTO_FWD_PIN_13_3_LP[_LZ]) matches exact arithmetic."""
    rng = random.Random(23)
    for i in range(40):
        q = asm_sim.PRIMES[i % len(asm_sim.PRIMES)]
        asm_sim.check_lane_pair_xchg(rng, q, approx=True, lazy_out=bool(i % 2))


def test_generic_rounds_match_exact_arithmetic():
    # FwdRoundGenAsm / InvRoundGenAsm (any q < 2^60) at every size they are emitted for, over the
    # HPS primes of the published configurations and the ends of the range
    rng = random.Random(13)
    for logn in gen_ntt_asm.GEN_LOGN:
        for r in range((logn + 3) // 4):
            for i in range(2 * len(asm_sim.GENERIC_PRIMES)):
                q = asm_sim.GENERIC_PRIMES[i % len(asm_sim.GENERIC_PRIMES)]
                asm_sim.check_round(logn, r, q, rng, True, generic=True)
                asm_sim.check_inv_round(logn, r, q, rng, True, generic=True)


def test_small_prime_generic_rounds_match_exact_arithmetic():
    # FwdRoundGenAsm / InvRoundGenAsm<LOGN, R, QB < 60>: fewer reductions for q < 2^QB, at the
    # bounds the transform's earlier rounds leave (fwd_rounds / inv_rounds chain them)
    rng = random.Random(17)
    for logn, qbs in gen_ntt_asm.GEN_QBITS.items():
        for qb in qbs:
            qs = asm_sim.generic_primes(qb)
            for r in range((logn + 3) // 4):
                for i in range(3 * len(qs)):
                    asm_sim.check_round(logn, r, qs[i % len(qs)], rng, True, True, qb)
                    asm_sim.check_inv_round(logn, r, qs[i % len(qs)], rng, True, True, qb)


def test_tensor_products_match_exact_arithmetic():
    # MulNear60Asm: the 120-bit product folded twice through 2^60 == d, for every BASELINE prime
    # (the fifth entry of PRIMES has d = 2^32 - 3, outside the d < 2^24 this sequence needs)
    rng = random.Random(11)
    for i in range(2000):
        for w in (1, 2):
            asm_sim.check_mulpair(w, asm_sim.PRIMES[i % 4], rng)
            asm_sim.check_mulpair(w, asm_sim.PRIMES[i % 4], rng, bound=2)   # lazy extension operands


def test_committed_inc_is_current(tmp_path):
    out = tmp_path / "ntt_asm.inc"
    old = gen_ntt_asm.OUT
    gen_ntt_asm.OUT = str(out)
    try:
        gen_ntt_asm.main()
    finally:
        gen_ntt_asm.OUT = old
    with open(os.path.join(ROOT, "exacto_amd", "csrc", "ntt_asm.inc")) as f:
        assert f.read() == out.read_text(), "re-run tools/gen_ntt_asm.py"
