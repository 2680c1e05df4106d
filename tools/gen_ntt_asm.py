#!/usr/bin/env python3
"""Generates exacto_amd/csrc/ntt_asm.inc: hand-scheduled gfx950 inline-asm rounds of the forward
negacyclic NTT (Cooley-Tukey, Harvey lazy butterflies, Shoup twiddles) for primes q in
(2^60 - 2^32, 2^60).  Run it after editing; the output is committed.

Why asm: gfx950 has no 64-bit add/sub/compare with carry-out to a VGPR, so every 64-bit
subtraction and every 65-bit sum is a VALU carry chain through an SGPR pair, and a VALU that
reads an SGPR written by a VALU needs 2 wait states.  hipcc schedules one butterfly at a time
and pads each chain with s_nop.  Here W butterflies are interleaved with explicit carry pairs, so
every carry read has its 2 wait states filled by independent work; pad_hazards() inserts s_nop
only where a gap remains (and is the safety net for the rule).

Issue costs measured on MI355X (tools/op_rate.hip, cycles per wave-instruction per SIMD): v_add /
v_sub / v_and / v_mov / v_lshrrev_b32 ~2.5; every multiply, mad, carry op, 64-bit op, add3,
cndmask_e64, bfi, alignbit ~4.2-5.  The sequence below is written for that table.

Register model: one asm statement per round keeps the 16 values of a thread in physical VGPR
pairs (clobbered) between stages, with one temp set per butterfly stream.  The values enter and
leave through "+v" u64 operands tied to x[k]; the first stage also takes the u32 halves of its
Y operands (and the high halves of the X operands it reduces) as inputs.  Tied operands are
written only by the round's last stage (or the final reduction), after every input was read.
Hazard rule (LLVM GCNHazardRecognizer, gfx940+ VALUWriteSGPRVALURead): a VALU reading an SGPR
written by a VALU (carry-in, cndmask mask) needs 2 wait states after the write.  gfx9 reads at
most one SGPR (or literal) per VALU instruction, so the carry-in of v_subb takes 2q's high word
from a VGPR.

Per-butterfly sequence (Y any 64-bit value, X < bound, T = Shoup(Y, w) in [0, 2q)), 15 slow +
2 fast instructions (the previous generator: 18 slow + 1 fast):
  qh = hi64(Y * ws) exact:  Z = mulhi(y0,s0); A = y1*s0 + Z; B = y0*s1 + A with the carry-out of
       v_mad_u64_u32 in an SGPR pair; D = (B.hi, carry) by v_mov + v_cndmask; qh = y1*s1 + D
  T  = lo64(Y*w + qh*(2^64-q)):  E = y0*w0; E += qh0*n0 (two mads); the high-word cross terms
       y0*w1 + y1*w0 + qh0*n1 + qh1*n0 as one mul_lo + three mads on a 32-bit chain (the high
       word of a mad's 64-bit addend never reaches the low word of its result); T.hi += chain
  out0 = X + T, out1 = X + (2q - T)        (v_lshl_add_u64, sub_co/subb)
Reduction of a value x < 2^64 for q = 2^60 - d, d < 2^32 (so 2^64 - q = (0xF0000000, d)):
  t = x.hi >> 28; r = x + t*(2^64 - q) = x - t*q, by one mad (low word d) and a subtraction of
  t << 28 from the high word; r = (x mod 2^60) + t*d < 2q.
Round-start reduction (rounds >= 1): only the 8 values that are X of the round's first stage are
reduced (< 2q; a Shoup input may be anything below 2^64, and both butterfly outputs are bounded
by X's bound + 2q per stage), so the round ends below 10q < 16q.
Final round: the reduction above, then r - q, selected by the sign of r - q (and-mask + add).
"""

import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "exacto_amd", "csrc", "ntt_asm.inc")

VBASE = int(os.environ.get("EXACTO_ASM_VBASE", "104"))   # first physical VGPR of the statements
W = int(os.environ.get("EXACTO_ASM_STREAMS", "2"))       # butterflies interleaved per group
SGPR_C = [80, 82, 84, 88, 90, 92][:max(W, 2)]            # carry pair of each stream
SGPR_SD = 86                  # sink for the carry-out of v_mad_u64_u32 where it is not used


def v(i):
    return f"v{i}"


def vp(i):
    return f"v[{i}:{i + 1}]"


def sp(i):
    return f"s[{i}:{i + 1}]"


class Ins:
    __slots__ = ("text", "rd", "wr", "valu")

    def __init__(self, text, rd=(), wr=(), valu=True):
        self.text, self.rd, self.wr, self.valu = text, set(rd), set(wr), valu


def interleave(streams):
    """Round-robin merge of instruction streams."""
    out = []
    its = [list(s) for s in streams]
    while any(its):
        for s in its:
            if s:
                out.append(s.pop(0))
    return out


def pad_hazards(seq):
    """Insert s_nop so that every SGPR read by a VALU is >= 2 wait states after its VALU write."""
    out = []
    last_write = {}
    clock = 0
    for ins in seq:
        need = 0
        if ins.valu:
            for r in ins.rd:
                if r in last_write:
                    gap = clock - last_write[r] - 1
                    need = max(need, 2 - gap)
        if need > 0:
            out.append(Ins(f"s_nop {need - 1}", valu=False))
            clock += need
        out.append(ins)
        clock += 1
        if ins.valu:
            for w in ins.wr:
                last_write[w] = clock - 1
    return out


class Round:
    """One forward round (stage bits BHI..LO of a 4-bit window) as one asm statement."""

    def __init__(self, logn, r):
        self.logn, self.r = logn, r
        self.lo = max(logn - 4 * (r + 1), 0)
        self.bhi = logn - 1 - 4 * r
        self.last = self.lo == 0
        self.uniform_tw = self.lo + 4 >= logn     # thigh == 0: twiddles are block-uniform (SGPR)
        self.ins = []                            # (name, constraint, expr)
        self.seen = set()

    def _in(self, key, cons, expr):
        if key not in self.seen:
            self.ins.append((key, cons, expr))
            self.seen.add(key)
        return "%[" + key + "]"

    def n0(self): return self._in("n0", "s", "K.n0")
    def n1(self): return self._in("n1", "s", "K.n1")
    def q2l(self): return self._in("q2l", "s", "K.q2l")
    def q2h(self): return self._in("q2h", "v", "K.q2h")
    def ql(self): return self._in("ql", "s", "K.ql")
    def qh(self): return self._in("qh", "s", "K.qh")
    def nq(self): return self._in("nq", "s", "K.nq")

    def xh(self, k): return self._in(f"x{k}h", "v", f"(uint32_t)(x[{k}] >> 32)")
    def xl(self, k): return self._in(f"x{k}l", "v", f"(uint32_t)x[{k}]")

    def tw(self, slot, part):
        c = "s" if self.uniform_tw else "v"
        expr = {"w0": f"(uint32_t)tw[{slot}].w", "w1": f"(uint32_t)(tw[{slot}].w >> 32)",
                "s0": f"(uint32_t)tw[{slot}].ws", "s1": f"(uint32_t)(tw[{slot}].ws >> 32)"}[part]
        return self._in(f"t{slot}{part}", c, expr)

    def stages(self):
        res, slot = [], 0
        for b in range(self.bhi, self.lo - 1, -1):
            lb = b - self.lo
            half = 1 << lb
            bfs = []
            for g in range(8 >> lb):
                for m in range(half):
                    k0 = g * 2 * half + m
                    bfs.append((k0, k0 + half, slot + g))
            slot += 8 >> lb
            res.append((lb, bfs))
        return res

    def reduce(self, dst, src_pair, src_hi, t, u):
        """dst (pair) = src - floor(src / 2^60) * q  in [0, 2q).  t, u: temp VGPRs."""
        return [
            Ins(f"v_lshrrev_b32 {v(t)}, 28, {src_hi}"),
            Ins(f"v_mad_u64_u32 {vp(dst)}, {sp(SGPR_SD)}, {v(t)}, {self.n0()}, {src_pair}", wr=[sp(SGPR_SD)]),
            Ins(f"v_lshlrev_b32 {v(u)}, 28, {v(t)}"),
            Ins(f"v_sub_u32 {v(dst + 1)}, {v(dst + 1)}, {v(u)}"),
        ]

    def gen(self):
        P = [VBASE + 2 * k for k in range(16)]
        TB = VBASE + 32
        # 10 VGPRs per stream: Z (Z.hi stays 0), A (= D = qh), B (then 2q - T), E (T), F (cross chain)
        temps = [dict(Z=TB + 10 * j, A=TB + 10 * j + 2, B=TB + 10 * j + 4, E=TB + 10 * j + 6,
                      F=TB + 10 * j + 8) for j in range(max(W, 2))]
        self.vmax = TB + 10 * len(temps)
        C = SGPR_C
        SD = sp(SGPR_SD)
        seq = [Ins("s_nop 1", valu=False)]      # an "s" operand may come straight from a VALU
        for t in temps:
            seq.append(Ins(f"v_mov_b32 {v(t['Z'] + 1)}, 0"))

        st = self.stages()
        nstage = len(st)
        if nstage < 2 and not self.last:
            raise SystemExit("single-stage non-final round not supported")
        first_lb = st[0][0]
        xop = {k: f"%[x{k}]" for k in range(16)}
        in_p = {k: False for k in range(16)}

        if self.r > 0:   # round-start reduction of the first stage's X values into P
            red = [k for k in range(16) if not (k >> first_lb) & 1]
            streams = [[] for _ in range(len(temps))]
            for i, k in enumerate(red):
                j = i % len(temps)
                t = temps[j]
                streams[j] += self.reduce(P[k], xop[k], self.xh(k), t["B"], t["B"] + 1)
                in_p[k] = True
            seq += interleave(streams)

        for si, (lb, bfs) in enumerate(st):
            direct_out = si == nstage - 1 and not self.last
            for pi in range(0, len(bfs), W):
                streams = []
                for j, (k0, k1, slot) in enumerate(bfs[pi:pi + W]):
                    t = temps[j]
                    c = sp(C[j])
                    Z, A, B, E, F = (t[n] for n in "ZABEF")
                    if in_p[k1]:
                        yl, yh = v(P[k1]), v(P[k1] + 1)
                    else:
                        yl, yh = self.xl(k1), self.xh(k1)
                    X = vp(P[k0]) if in_p[k0] else xop[k0]
                    w0, w1 = self.tw(slot, "w0"), self.tw(slot, "w1")
                    s0, s1 = self.tw(slot, "s0"), self.tw(slot, "s1")
                    o0, o1 = (xop[k0], xop[k1]) if direct_out else (vp(P[k0]), vp(P[k1]))
                    streams.append([
                        Ins(f"v_mul_hi_u32 {v(Z)}, {yl}, {s0}"),
                        Ins(f"v_mad_u64_u32 {vp(A)}, {SD}, {yh}, {s0}, {vp(Z)}", wr=[SD]),
                        Ins(f"v_mad_u64_u32 {vp(B)}, {c}, {yl}, {s1}, {vp(A)}", wr=[c]),
                        Ins(f"v_mad_u64_u32 {vp(E)}, {SD}, {yl}, {w0}, 0", wr=[SD]),
                        Ins(f"v_mov_b32 {v(A)}, {v(B + 1)}"),
                        Ins(f"v_mul_lo_u32 {v(F)}, {yl}, {w1}"),
                        Ins(f"v_cndmask_b32_e64 {v(A + 1)}, 0, 1, {c}", rd=[c]),
                        Ins(f"v_mad_u64_u32 {vp(F)}, {SD}, {yh}, {w0}, {vp(F)}", wr=[SD]),
                        Ins(f"v_mad_u64_u32 {vp(A)}, {SD}, {yh}, {s1}, {vp(A)}", wr=[SD]),
                        Ins(f"v_mad_u64_u32 {vp(E)}, {SD}, {v(A)}, {self.n0()}, {vp(E)}", wr=[SD]),
                        Ins(f"v_mad_u64_u32 {vp(F)}, {SD}, {v(A)}, {self.n1()}, {vp(F)}", wr=[SD]),
                        Ins(f"v_mad_u64_u32 {vp(F)}, {SD}, {v(A + 1)}, {self.n0()}, {vp(F)}", wr=[SD]),
                        Ins(f"v_sub_co_u32_e64 {v(B)}, {c}, {self.q2l()}, {v(E)}", wr=[c]),
                        Ins(f"v_add_u32 {v(E + 1)}, {v(E + 1)}, {v(F)}"),
                        Ins(f"v_subb_co_u32_e64 {v(B + 1)}, {c}, {self.q2h()}, {v(E + 1)}, {c}", rd=[c], wr=[c]),
                        # o1 first: o0 may be X's own register pair
                        Ins(f"v_lshl_add_u64 {o1}, {vp(B)}, 0, {X}"),
                        Ins(f"v_lshl_add_u64 {o0}, {vp(E)}, 0, {X}"),
                    ])
                    if not direct_out:
                        in_p[k0] = in_p[k1] = True
                seq += interleave(streams)

        if self.last:
            # canonical reduction of all 16 values (< 16q) into the tied operands:
            # r = x - floor(x/2^60)*q in [0, 2q); s = r - q; out = s + (q & sign(s))
            streams = [[] for _ in range(len(temps))]
            for k in range(16):
                j = k % len(temps)
                t = temps[j]
                R, S, M = P[k], t["E"], t["F"]
                streams[j] += self.reduce(R, vp(R), v(R + 1), t["B"], t["B"] + 1) + [
                    Ins(f"v_lshl_add_u64 {vp(S)}, {vp(R)}, 0, {self.nq()}"),
                    Ins(f"v_ashrrev_i32 {v(M)}, 31, {v(S + 1)}"),
                    Ins(f"v_and_b32 {v(M + 1)}, {self.qh()}, {v(M)}"),
                    Ins(f"v_and_b32 {v(M)}, {self.ql()}, {v(M)}"),
                    Ins(f"v_lshl_add_u64 {xop[k]}, {vp(S)}, 0, {vp(M)}"),
                ]
            seq += interleave(streams)

        return pad_hazards(seq)

    def emit(self):
        seq = self.gen()
        body = "\\n\\t".join(i.text for i in seq)
        clob = [f'"v{i}"' for i in range(VBASE, self.vmax)]
        clob += [f'"s{i}"' for p in SGPR_C + [SGPR_SD] for i in (p, p + 1)]
        clob.append('"memory"')   # keeps the next round's twiddle loads below the statement
        outs = ", ".join(f'[x{k}] "+v"(x[{k}])' for k in range(16))
        ins = ", ".join(f'[{k}] "{c}"({e})' for k, c, e in self.ins)
        nops = sum(1 for i in seq if i.text.startswith("s_nop"))
        valu = sum(1 for i in seq if i.valu)
        return (f"// round {self.r} of the {1 << self.logn}-point forward NTT: stage bits {self.bhi}..{self.lo}, "
                f"{valu} VALU, {nops} s_nop\n"
                f"template <> struct FwdRoundAsm<{self.logn}, {self.r}> {{\n"
                f"    static __device__ __forceinline__ void run(u64 (&x)[16], const TwPair (&tw)[15], "
                f"const AsmK& K) {{\n"
                f"        asm volatile(\"{body}\"\n            : {outs}\n            : {ins}\n"
                f"            : {', '.join(clob)});\n    }}\n}};\n")


def main():
    parts = ["// GENERATED by tools/gen_ntt_asm.py -- do not edit.\n"
             "// Hand-scheduled forward NTT rounds for primes in (2^60 - 2^32, 2^60); see the generator's docstring.\n"
             "// Included inside namespace exacto by ntt.hip.\n#pragma once\n\n"
             "struct AsmK {\n"
             "    uint32_t n0, n1;      // 2^64 - q (n1 = 0xF0000000 for the primes of this path)\n"
             "    uint32_t q2l, q2h;    // 2q\n"
             "    uint32_t ql, qh;      // q\n"
             "    u64 nq;               // 2^64 - q\n"
             "};\n\n"
             "__device__ __forceinline__ AsmK make_asmk(u64 q) {\n"
             "    AsmK K;\n"
             "    const u64 nq = (u64)0 - q, q2 = 2 * q;\n"
             "    K.n0 = (uint32_t)nq; K.n1 = (uint32_t)(nq >> 32);\n"
             "    K.q2l = (uint32_t)q2; K.q2h = (uint32_t)(q2 >> 32);\n"
             "    K.ql = (uint32_t)q; K.qh = (uint32_t)(q >> 32);\n"
             "    K.nq = nq;\n"
             "    return K;\n"
             "}\n\n"
             "template <int LOGN, int R> struct FwdRoundAsm;\n\n"]
    for logn in (12, 13):
        for r in range((logn + 3) // 4):
            parts.append(Round(logn, r).emit())
            parts.append("\n")
    with open(OUT, "w") as f:
        f.write("".join(parts))
    print("wrote", OUT)


if __name__ == "__main__":
    main()
