#!/usr/bin/env python3
"""One-lane simulator of the generated NTT asm rounds (tools/gen_ntt_asm.py), for CPU checks.

Runs each round's instruction sequence on random inputs at the bounds the round assumes and
checks the results against exact modular arithmetic: every output is congruent mod q to the
radix-2 Cooley-Tukey (forward) or Gentleman-Sande (inverse, n^-1 folded into the last stage)
butterflies of the round, below the bound the generator declares for the round's outputs, and
canonical after the final round.  This catches register-reuse and sequencing mistakes before a
GPU run (it does not model timing or hazards; pad_hazards() handles those).

Usage: python3 tools/asm_sim.py [trials]
"""

import os
import random
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gen_ntt_asm as G  # noqa: E402

M32 = (1 << 32) - 1
M64 = (1 << 64) - 1


class Lane:
    def __init__(self, named):
        self.v = {}
        self.s = {}        # carry / compare masks (this lane's bit) and SGPR pairs
        self.named = named  # name -> [value, bits]

    # ---------------------------------------------------------------- operands
    def rd32(self, op):
        op = op.strip()
        if op.startswith("%["):
            val, bits = self.named[op[2:-1]]
            assert bits == 32, op
            return val
        if op.startswith("v"):
            return self.v.get(int(op[1:]), 0xDEADBEEF)
        return int(op, 0) & M32

    def rd64(self, op):
        op = op.strip()
        if op.startswith("%["):
            val, bits = self.named[op[2:-1]]
            assert bits == 64, op
            return val
        m = re.fullmatch(r"v\[(\d+):(\d+)\]", op)
        if m:
            a = int(m.group(1))
            return self.v.get(a, 0xDEADBEEF) | (self.v.get(a + 1, 0xDEADBEEF) << 32)
        return int(op, 0) & M64

    def wr32(self, op, val):
        op = op.strip()
        if op.startswith("%["):
            raise AssertionError("32-bit write to a named operand " + op)
        self.v[int(op[1:])] = val & M32

    def wr64(self, op, val):
        op = op.strip()
        val &= M64
        if op.startswith("%["):
            name = op[2:-1]
            assert self.named[name][1] == 64
            self.named[name][0] = val
            return
        m = re.fullmatch(r"v\[(\d+):(\d+)\]", op)
        a = int(m.group(1))
        self.v[a] = val & M32
        self.v[a + 1] = val >> 32

    # ---------------------------------------------------------------- instructions
    def run(self, text):
        text = text.strip()
        if text.startswith("s_nop"):
            return
        mnem, _, rest = text.partition(" ")
        ops = [o.strip() for o in re.split(r",(?![^\[]*\])", rest)]
        if mnem == "v_mul_hi_u32":
            self.wr32(ops[0], (self.rd32(ops[1]) * self.rd32(ops[2])) >> 32)
        elif mnem == "v_mul_lo_u32":
            self.wr32(ops[0], self.rd32(ops[1]) * self.rd32(ops[2]))
        elif mnem == "v_mad_u64_u32":
            full = self.rd32(ops[2]) * self.rd32(ops[3]) + self.rd64(ops[4])
            self.s[ops[1]] = full >> 64
            self.wr64(ops[0], full)
        elif mnem == "v_mov_b32":
            self.wr32(ops[0], self.rd32(ops[1]))
        elif mnem == "v_cndmask_b32_e64":
            self.wr32(ops[0], self.rd32(ops[2]) if self.s[ops[3]] else self.rd32(ops[1]))
        elif mnem == "v_add_u32":
            self.wr32(ops[0], self.rd32(ops[1]) + self.rd32(ops[2]))
        elif mnem == "v_sub_u32":
            self.wr32(ops[0], self.rd32(ops[1]) - self.rd32(ops[2]))
        elif mnem == "v_sub_co_u32_e64":
            r = self.rd32(ops[2]) - self.rd32(ops[3])
            self.s[ops[1]] = 1 if r < 0 else 0
            self.wr32(ops[0], r)
        elif mnem == "v_subb_co_u32_e64":
            r = self.rd32(ops[2]) - self.rd32(ops[3]) - self.s[ops[4]]
            self.s[ops[1]] = 1 if r < 0 else 0
            self.wr32(ops[0], r)
        elif mnem == "v_cmp_le_u64_e64":
            self.s[ops[0]] = 1 if self.rd64(ops[1]) <= self.rd64(ops[2]) else 0
        elif mnem == "v_lshl_add_u64":
            self.wr64(ops[0], (self.rd64(ops[1]) << int(ops[2])) + self.rd64(ops[3]))
        elif mnem == "v_lshrrev_b32":
            self.wr32(ops[0], self.rd32(ops[2]) >> int(ops[1]))
        elif mnem == "v_lshlrev_b32":
            self.wr32(ops[0], self.rd32(ops[2]) << int(ops[1]))
        elif mnem == "v_ashrrev_i32":
            x = self.rd32(ops[2])
            if x >> 31:
                x -= 1 << 32
            self.wr32(ops[0], x >> int(ops[1]))
        elif mnem == "v_and_b32":
            self.wr32(ops[0], self.rd32(ops[1]) & self.rd32(ops[2]))
        elif mnem == "v_alignbit_b32":
            self.wr32(ops[0], ((self.rd32(ops[1]) << 32 | self.rd32(ops[2])) >> int(ops[3])) & M32)
        else:
            raise NotImplementedError(mnem)


def shoup(w, q):
    return (w << 64) // q


def _named(rd, x, tw, q, logn):
    """Operand values of one statement for a lane holding x[0..15] with twiddles tw[slot]."""
    n = 1 << logn
    n_inv = pow(n, -1, q)
    # psi_inv_rev[1] * n^-1: any constant below q exercises the same instructions
    last_w = (q - 12345) * n_inv % q
    K = dict(n0=((1 << 64) - q) & M32, n1=((1 << 64) - q) >> 32, ql=q & M32, qh=q >> 32, nq=(1 << 64) - q,
             nil=n_inv & M32, nih=n_inv >> 32, nsl=shoup(n_inv, q) & M32, nsh=shoup(n_inv, q) >> 32,
             lwl=last_w & M32, lwh=last_w >> 32, lsl=shoup(last_w, q) & M32, lsh=shoup(last_w, q) >> 32)
    named = {}
    for key, cons, expr in rd.ins:
        m = re.fullmatch(r"x(\d+)([lh])", key)
        if m:
            k = int(m.group(1))
            named[key] = [(x[k] if m.group(2) == "l" else x[k] >> 32) & M32, 32]
            continue
        m = re.fullmatch(r"t(\d+)(w0|w1|s0|s1)", key)
        if m:
            slot, part = int(m.group(1)), m.group(2)
            w = tw[slot]
            named[key] = [{"w0": w & M32, "w1": w >> 32, "s0": shoup(w, q) & M32,
                           "s1": shoup(w, q) >> 32}[part], 32]
            continue
        m = re.fullmatch(r"mq(\d+)", key)
        if m:
            named[key] = [int(m.group(1)) * q, 64]
            continue
        m = re.fullmatch(r"nmq(\d+)", key)
        if m:
            named[key] = [((1 << 64) - int(m.group(1)) * q) & M64, 64]
            continue
        m = re.fullmatch(r"q(\d+)([lh])", key)
        if m:
            cq = int(m.group(1)) * q
            named[key] = [(cq if m.group(2) == "l" else cq >> 32) & M32, 32]
            continue
        named[key] = [K[key], 64 if key == "nq" else 32]
    for k in range(16):
        named[f"x{k}"] = [x[k], 64]
    return named, n_inv, last_w


def _inputs(rng, bound_in):
    x = [rng.randrange(bound_in) for _ in range(16)]
    if rng.random() < 0.3:   # extremes
        x = [bound_in - 1 - rng.randrange(3) for _ in range(16)]
    return x


def check_round(logn, r, q, rng, approx=True, generic=False, qbits=60):
    if qbits < 60:
        rd = G.fwd_rounds(logn, approx, True, generic, qbits)[r]
    else:
        rd = G.Round(logn, r, approx, generic=generic)
    seq = rd.gen()
    bound_in = rd.bound_in * q
    x = _inputs(rng, bound_in)
    tw = [rng.randrange(q) for _ in range(15)]
    named, _, _ = _named(rd, x, tw, q, logn)
    lane = Lane(named)
    for ins in seq:
        lane.run(ins.text)
    got = [named[f"x{k}"][0] for k in range(16)]
    # exact model
    want = [v % q for v in x]
    for lb, bfs in rd.stages():
        for k0, k1, slot in bfs:
            t = want[k1] * tw[slot] % q
            want[k0], want[k1] = (want[k0] + t) % q, (want[k0] - t) % q
    for k in range(16):
        assert got[k] % q == want[k], (logn, r, k, got[k], want[k])
        if rd.last:
            assert got[k] < q, ("not canonical", logn, r, k, got[k])
        else:
            assert got[k] < rd.bound_out * q, ("bound", logn, r, k, got[k] / q)


def check_inv_round(logn, r, q, rng, approx=True, generic=False, qbits=60, lazy_out=False):
    rd = G.inv_rounds(logn, approx, generic, qbits)[r]
    rd = G.InvRound(logn, r, rd.bound_in, approx, generic, qbits, lazy_out=lazy_out)
    seq = rd.gen()
    x = _inputs(rng, rd.bound_in * q)
    tw = [rng.randrange(q) for _ in range(15)]
    named, n_inv, last_w = _named(rd, x, tw, q, logn)
    lane = Lane(named)
    for ins in seq:
        lane.run(ins.text)
    got = [named[f"x{k}"][0] for k in range(16)]
    want = [v % q for v in x]
    for final, bfs in rd.stages():
        for k0, k1, slot in bfs:
            u, w_ = want[k0], want[k1]
            if final:
                want[k0], want[k1] = (u + w_) * n_inv % q, (u - w_) * last_w % q
            else:
                want[k0], want[k1] = (u + w_) % q, (u - w_) * tw[slot] % q
    for k in range(16):
        assert got[k] % q == want[k], ("inv", logn, r, k, got[k], want[k])
        assert got[k] < rd.bound_out * q, ("inv bound", logn, r, k, got[k] / q, rd.bound_out)


def _run_pinned(rd, x, tw, q, logn):
    """Run a pinned statement: the values start and end in the home pairs G.PIN_BASE + 2k."""
    seq = rd.gen()
    named, n_inv, last_w = _named(rd, [0] * 16, tw, q, logn)
    lane = Lane(named)
    for k in range(16):
        lane.v[G.PIN_BASE + 2 * k] = x[k] & M32
        lane.v[G.PIN_BASE + 2 * k + 1] = x[k] >> 32
    for ins in seq:
        lane.run(ins.text)
    got = [lane.v[G.PIN_BASE + 2 * k] | (lane.v[G.PIN_BASE + 2 * k + 1] << 32) for k in range(16)]
    return got, n_inv, last_w


def check_round_pinned(logn, r, q, rng, approx=True, lazy_out=False):
    rd = G.Round(logn, r, approx, True, pinned=True, lazy_out=lazy_out)
    bound_in = q if r == 0 else 16 * q
    x = _inputs(rng, bound_in)
    tw = [rng.randrange(q) for _ in range(15)]
    got, _, _ = _run_pinned(rd, x, tw, q, logn)
    want = [v % q for v in x]
    for lb, bfs in rd.stages():
        for k0, k1, slot in bfs:
            t = want[k1] * tw[slot] % q
            want[k0], want[k1] = (want[k0] + t) % q, (want[k0] - t) % q
    for k in range(16):
        assert got[k] % q == want[k], ("pinned fwd", logn, r, k)
        assert got[k] < ((2 if lazy_out else 1) * q if rd.last else rd.bound_out * q), \
            ("pinned fwd bound", logn, r, k, got[k] / q)


def check_inv_round_pinned(logn, r, q, rng, approx=True, lazy_out=False):
    b = G.inv_rounds_pinned(logn, approx)[r].bound_in
    rd = G.InvRoundPinned(logn, r, b, approx, lazy_out=lazy_out)
    x = _inputs(rng, b * q)
    tw = [rng.randrange(q) for _ in range(15)]
    got, n_inv, last_w = _run_pinned(rd, x, tw, q, logn)
    want = [v % q for v in x]
    for final, bfs in rd.stages():
        for k0, k1, slot in bfs:
            u, w_ = want[k0], want[k1]
            if final:
                want[k0], want[k1] = (u + w_) * n_inv % q, (u - w_) * last_w % q
            else:
                want[k0], want[k1] = (u + w_) % q, (u - w_) * tw[slot] % q
    for k in range(16):
        assert got[k] % q == want[k], ("pinned inv", logn, r, k)
        assert got[k] < rd.bound_out * q, ("pinned inv bound", logn, r, k, got[k] / q)


def check_lane_pair_xchg(rng, q, approx=True, lazy_out=False):
    """The 8192-point forward's last exchange by DPP (G.LanePairXchg) on a lane pair, then the last
    round with the permuted homes (G.PERM_LP): the pair's 32 elements end where the LDS exchange
    (layout LO = 1 -> LO = 0) and the plain last round would leave them, congruent and in bound."""
    seq = G.LanePairXchg().gen()
    # element layout LO = 1: lane b (b = 0 even, 1 odd) holds element 2k + b as value k
    elems = [rng.randrange(16 * q) for _ in range(32)]
    lanes = []
    for b in (0, 1):
        ln = Lane({"tid": [b, 32]})   # %[tid]; only its parity matters
        for k in range(16):
            e = elems[2 * k + b]
            ln.v[G.PIN_BASE + 2 * k] = e & M32
            ln.v[G.PIN_BASE + 2 * k + 1] = e >> 32
        lanes.append(ln)
    for ins in seq:
        t = ins.text.strip()
        if t.startswith("s_nop"):
            continue
        mnem, _, rest = t.partition(" ")
        if mnem in ("v_mov_b32_dpp", "v_cndmask_b32_dpp"):
            # quad_perm [1, 0, 3, 2]: src0 is read from the partner lane, before this instruction writes
            ops = [o.strip() for o in rest.split(" quad_perm")[0].split(",")]
            src0 = [ln.rd32(ops[1]) for ln in lanes]
            for i, ln in enumerate(lanes):
                part = src0[1 - i]
                if mnem == "v_mov_b32_dpp":
                    ln.wr32(ops[0], part)
                else:   # D = VCC ? src1 : src0(partner)
                    ln.wr32(ops[0], ln.rd32(ops[2]) if ln.s["vcc"] else part)
            continue
        for ln in lanes:
            if mnem == "v_cmp_eq_u32_e32":
                ops = [o.strip() for o in rest.split(",")]
                ln.s["vcc"] = 1 if ln.rd32(ops[1]) == ln.rd32(ops[2]) else 0
            elif mnem == "v_cndmask_b32_e32":
                ops = [o.strip() for o in rest.split(",")]
                ln.wr32(ops[0], ln.rd32(ops[2]) if ln.s["vcc"] else ln.rd32(ops[1]))
            else:
                ln.run(t)
    # layout LO = 0: lane b holds element 16 b + k' as value k', in home PERM_LP[k']
    for b, ln in enumerate(lanes):
        for kk in range(16):
            h = G.PERM_LP[kk]
            got = ln.v[G.PIN_BASE + 2 * h] | (ln.v[G.PIN_BASE + 2 * h + 1] << 32)
            assert got == elems[16 * b + kk], ("lane-pair exchange", b, kk)
    # the permuted last round on each lane
    rd = G.Round(13, 3, approx, True, pinned=True, lazy_out=lazy_out, perm=G.PERM_LP)
    rseq = rd.gen()
    for b, ln in enumerate(lanes):
        x = [elems[16 * b + kk] for kk in range(16)]
        tw = [rng.randrange(q) for _ in range(15)]
        named, _, _ = _named(rd, [0] * 16, tw, q, 13)
        lane = Lane(named)
        for kk in range(16):
            h = G.PERM_LP[kk]
            lane.v[G.PIN_BASE + 2 * h] = x[kk] & M32
            lane.v[G.PIN_BASE + 2 * h + 1] = x[kk] >> 32
        for ins in rseq:
            lane.run(ins.text)
        want = [v % q for v in x]
        for lb, bfs in rd.stages():
            for k0, k1, slot in bfs:
                t = want[k1] * tw[slot] % q
                want[k0], want[k1] = (want[k0] + t) % q, (want[k0] - t) % q
        for kk in range(16):
            h = G.PERM_LP[kk]
            got = lane.v[G.PIN_BASE + 2 * h] | (lane.v[G.PIN_BASE + 2 * h + 1] << 32)
            assert got % q == want[kk] and got < (2 if lazy_out else 1) * q, ("permuted last round", b, kk)


def check_mulpair(w, q, rng, bound=1):
    """MulNear60Asm<w>: r_k == a_k b_k (mod q) and r_k < 2q for a_k, b_k < bound q (extremes
    included; bound 2: the extension transforms' lazy outputs)."""
    st = G.MulPair(w)
    seq = st.gen()
    d = (1 << 60) - q
    vals = []
    top = bound * q
    for k in range(w):
        if rng.random() < 0.3:
            a, b = top - 1 - rng.randrange(3), top - 1 - rng.randrange(3)
        else:
            a, b = rng.randrange(top), rng.randrange(top)
        vals.append((a, b))
    named = {"d": [d, 32], "e": [16 * d, 32]}
    for k, (a, b) in enumerate(vals):
        named.update({f"a{k}l": [a & M32, 32], f"a{k}h": [a >> 32, 32], f"b{k}l": [b & M32, 32],
                      f"b{k}h": [b >> 32, 32], f"r{k}": [0, 64]})
    lane = Lane(named)
    for ins in seq:
        lane.run(ins.text)
    for k, (a, b) in enumerate(vals):
        r = named[f"r{k}"][0]
        assert r % q == a * b % q and r < 2 * q, ("mulpair", w, k, a, b, r)


PRIMES = [1152921504606830593, 1152921504606748673, 1152921504606683137, 1152921504606601217,
          (1 << 60) - (1 << 32) + 3]  # the last: d = 2^32 - 3, the edge of the path (primality irrelevant here)
# the generic rounds: the HPS primes of compact_bfv (q, aux) and u64_dbfv (aux), odd values near both
# ends of (2^30, 2^60), and the special primes (any prime below 2^60 is in their domain)
GENERIC_PRIMES = [1099509805057, 562949953443841, 18014398509998081, 36028797018972161,
                  (1 << 60) - 1, (1 << 59) + 12345, (1 << 30) + 3] + PRIMES[:2]


def generic_primes(qbits):
    """The generic test primes below 2^qbits, and odd values at the top of that range."""
    return [q for q in GENERIC_PRIMES if q < (1 << qbits)] + [(1 << qbits) - 1, (1 << qbits) - 12345]


def main():
    trials = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    rng = random.Random(1)
    for approx in (True, False):
        for logn in (12, 13):
            for r in range((logn + 3) // 4):
                for i in range(trials):
                    check_round(logn, r, PRIMES[i % len(PRIMES)], rng, approx)
                    check_inv_round(logn, r, PRIMES[i % len(PRIMES)], rng, approx)
                    check_round_pinned(logn, r, PRIMES[i % len(PRIMES)], rng, approx)
                    check_inv_round_pinned(logn, r, PRIMES[i % len(PRIMES)], rng, approx)
    for logn in G.GEN_LOGN:
        for r in range((logn + 3) // 4):
            for i in range(trials):
                q = GENERIC_PRIMES[i % len(GENERIC_PRIMES)]
                check_round(logn, r, q, rng, True, generic=True)
                check_inv_round(logn, r, q, rng, True, generic=True)
        for qb in G.GEN_QBITS.get(logn, ()):
            qs = generic_primes(qb)
            for r in range((logn + 3) // 4):
                for i in range(trials):
                    check_round(logn, r, qs[i % len(qs)], rng, True, True, qb)
                    check_inv_round(logn, r, qs[i % len(qs)], rng, True, True, qb)
    for i in range(trials):
        for w in (1, 2):
            check_mulpair(w, PRIMES[i % 4], rng)
    print(f"asm_sim: all forward and inverse rounds of n=4096/8192 (approximate and exact Shoup "
          f"quotients) agree with exact arithmetic over {trials} trials each")


if __name__ == "__main__":
    main()
