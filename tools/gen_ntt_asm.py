#!/usr/bin/env python3
"""Generates exacto_amd/csrc/ntt_asm.inc: hand-scheduled gfx950 inline-asm rounds of the forward
negacyclic NTT (Cooley-Tukey, Harvey lazy butterflies, Shoup twiddles) for primes in
(2^60 - 2^56, 2^60).  Run it after editing; the output is committed.

Why asm: gfx950 has no 64-bit add/sub/compare with carry-out to a VGPR, so every 64-bit
subtraction and every 65-bit sum is a VALU carry chain through an SGPR pair, and a VALU that
reads an SGPR written by a VALU needs 2 wait states.  hipcc schedules one butterfly at a time
and pads each chain with s_nop (~450 per wave of the 4096-point transform, ~14 % of its issue
slots).  Here two butterflies are interleaved with explicit carry pairs, so every carry read has
its 2 wait states filled by independent work; pad_hazards() inserts s_nop only where a gap
remains (and is the safety net for the rule).

Register model: one asm statement per round keeps the 16 values of a thread in physical VGPR
pairs (clobbered) between stages, with two temp sets (one per butterfly stream).  The values
enter and leave through "+v" u64 operands tied to x[k]; the first stage also takes the u32
halves of its Y operands as inputs.  Tied operands are written only by the round's last stage
(or the final reduction), after every input was read.  Hazard rule (LLVM GCNHazardRecognizer,
gfx940+ VALUWriteSGPRVALURead): a VALU reading an SGPR written by a VALU (carry-in, cndmask
mask) needs 2 wait states after the write.

Per-butterfly sequence (values < 16q < 2^64, T = Shoup(Y, w) in [0, 2q)):
  qh = hi64(Y * ws)  exact: mul_hi, 3 mad_u64_u32, 65-bit carry (add_co, addc, addc)
  T  = lo64(Y*w + qh*(2^64-q)): 2 mad (low words), 3 cross products (mul_lo/mad), add3
  out0 = X + T, out1 = X + (2q - T)        (v_lshl_add_u64, sub_co/subb)
Round-start reduction (rounds >= 1): only the 8 values that are X of the round's first stage are
brought under 8q (a Shoup input may be anything below 2^64, and both butterfly outputs are
bounded by X's bound + 2q), so the round ends below 16q.
Final round: canonical reduction r = x - floor(x / 2^60) * q in [0, 2q) (exact because
q > 2^60 - 2^56 and x < 16q), then one conditional subtraction.
"""

import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "exacto_amd", "csrc", "ntt_asm.inc")

VBASE = int(os.environ.get("EXACTO_ASM_VBASE", "104"))   # first physical VGPR of the statements
W = int(os.environ.get("EXACTO_ASM_STREAMS", "2"))       # butterflies interleaved per group
SGPR_C = [80, 82, 84, 88, 90, 92][:max(W, 3)]            # carry / compare pair of each stream
SGPR_SD = 86                  # sink for the carry-out of v_mad_u64_u32


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
    def q8(self): return self._in("q8", "s", "K.q8")
    def nq8l(self): return self._in("nq8l", "v", "K.nq8l")
    def nq8h(self): return self._in("nq8h", "v", "K.nq8h")
    def qq(self): return self._in("qq", "s", "K.q")
    def nql(self): return self._in("nql", "v", "K.nql")
    def nqh(self): return self._in("nqh", "v", "K.nqh")

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

    def gen(self):
        P = [VBASE + 2 * k for k in range(16)]
        TB = VBASE + 32
        # 10 VGPRs per stream: D reuses Z (Z.hi is re-zeroed after D's last read), Q and the
        # difference N reuse B (lifetimes [3,6], [9,13], [15,17] of the sequence below)
        temps = [dict(Z=TB + 10 * j, D=TB + 10 * j, B=TB + 10 * j + 2, Q=TB + 10 * j + 2,
                      A=TB + 10 * j + 4, E=TB + 10 * j + 6, F=TB + 10 * j + 8) for j in range(max(W, 2))]
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
        half_in = {}
        for k in range(16):
            if (k >> first_lb) & 1:
                half_in[k] = (self._in(f"x{k}l", "v", f"(uint32_t)x[{k}]"),
                              self._in(f"x{k}h", "v", f"(uint32_t)(x[{k}] >> 32)"))
        in_p = {k: False for k in range(16)}

        if self.r > 0:   # round-start reduction of the first stage's X values
            red = [k for k in range(16) if not (k >> first_lb) & 1]
            NS = max(W, 3)
            streams = [[] for _ in range(NS)]
            Ms = [temps[0]["A"], temps[0]["B"], temps[1]["A"]] if W < 3 else [t["A"] for t in temps]
            for i, k in enumerate(red):
                j = i % NS
                c, M = sp(C[j]), Ms[j]
                streams[j] += [
                    Ins(f"v_cmp_le_u64_e64 {c}, {self.q8()}, {xop[k]}", wr=[c]),
                    Ins(f"v_cndmask_b32_e64 {v(M)}, 0, {self.nq8l()}, {c}", rd=[c]),
                    Ins(f"v_cndmask_b32_e64 {v(M + 1)}, 0, {self.nq8h()}, {c}", rd=[c]),
                    Ins(f"v_lshl_add_u64 {vp(P[k])}, {vp(M)}, 0, {xop[k]}"),
                ]
                in_p[k] = True
            seq += interleave(streams)

        for si, (lb, bfs) in enumerate(st):
            direct_out = si == nstage - 1 and not self.last
            for pi in range(0, len(bfs), W):
                streams = []
                for j, (k0, k1, slot) in enumerate(bfs[pi:pi + W]):
                    t = temps[j]
                    c = sp(C[j])
                    Z, A, B, D, Q, E, F = (t[n] for n in "ZABDQEF")
                    if in_p[k1]:
                        yl, yh = v(P[k1]), v(P[k1] + 1)
                    else:
                        yl, yh = half_in[k1]
                    X = vp(P[k0]) if in_p[k0] else xop[k0]
                    w0, w1 = self.tw(slot, "w0"), self.tw(slot, "w1")
                    s0, s1 = self.tw(slot, "s0"), self.tw(slot, "s1")
                    o0, o1 = (xop[k0], xop[k1]) if direct_out else (vp(P[k0]), vp(P[k1]))
                    streams.append([
                        Ins(f"v_mul_hi_u32 {v(Z)}, {yl}, {s0}"),
                        Ins(f"v_mad_u64_u32 {vp(A)}, {SD}, {yh}, {s0}, {vp(Z)}", wr=[SD]),
                        Ins(f"v_mad_u64_u32 {vp(B)}, {SD}, {yl}, {s1}, 0", wr=[SD]),
                        Ins(f"v_add_co_u32_e64 {v(B)}, {c}, {v(B)}, {v(A)}", wr=[c]),
                        Ins(f"v_mad_u64_u32 {vp(E)}, {SD}, {yl}, {w0}, 0", wr=[SD]),
                        Ins(f"v_addc_co_u32_e64 {v(D)}, {c}, {v(B + 1)}, {v(A + 1)}, {c}", rd=[c], wr=[c]),
                        Ins(f"v_mul_lo_u32 {v(F)}, {yl}, {w1}"),
                        Ins(f"v_addc_co_u32_e64 {v(D + 1)}, {c}, 0, 0, {c}", rd=[c], wr=[c]),
                        Ins(f"v_mad_u64_u32 {vp(Q)}, {SD}, {yh}, {s1}, {vp(D)}", wr=[SD]),
                        Ins(f"v_mov_b32 {v(Z + 1)}, 0"),
                        Ins(f"v_mad_u64_u32 {vp(E)}, {SD}, {v(Q)}, {self.n0()}, {vp(E)}", wr=[SD]),
                        Ins(f"v_mad_u64_u32 {vp(F)}, {SD}, {yh}, {w0}, {vp(F)}", wr=[SD]),
                        Ins(f"v_mul_lo_u32 {v(A)}, {v(Q)}, {self.n1()}"),
                        Ins(f"v_mad_u64_u32 {vp(A)}, {SD}, {v(Q + 1)}, {self.n0()}, {vp(A)}", wr=[SD]),
                        Ins(f"v_sub_co_u32_e64 {v(B)}, {c}, {self.q2l()}, {v(E)}", wr=[c]),
                        Ins(f"v_add3_u32 {v(E + 1)}, {v(E + 1)}, {v(F)}, {v(A)}"),
                        Ins(f"v_subb_co_u32_e64 {v(B + 1)}, {c}, {self.q2h()}, {v(E + 1)}, {c}", rd=[c], wr=[c]),
                        Ins(f"v_lshl_add_u64 {o1}, {vp(B)}, 0, {X}"),
                        Ins(f"v_lshl_add_u64 {o0}, {vp(E)}, 0, {X}"),
                    ])
                    if not direct_out:
                        in_p[k0] = in_p[k1] = True
                seq += interleave(streams)

        if self.last:
            # canonical reduction of all 16 values (< 16q) into the tied operands
            NS = max(W, 3)
            streams = [[] for _ in range(NS)]
            if W < 3:
                Ms = [temps[0]["A"], temps[1]["A"], temps[0]["Q"]]
                Ts = [temps[0]["D"], temps[1]["D"], temps[1]["Q"]]
            else:
                Ms = [t["A"] for t in temps]
                Ts = [t["D"] for t in temps]
            for k in range(16):
                j = k % NS
                c, M, tq = sp(C[j]), Ms[j], Ts[j]
                R = P[k]
                streams[j] += [
                    Ins(f"v_lshrrev_b32 {v(tq)}, 28, {v(R + 1)}"),
                    Ins(f"v_mad_u64_u32 {vp(R)}, {SD}, {v(tq)}, {self.n0()}, {vp(R)}", wr=[SD]),
                    Ins(f"v_mul_lo_u32 {v(tq + 1)}, {v(tq)}, {self.n1()}"),
                    Ins(f"v_add_u32 {v(R + 1)}, {v(R + 1)}, {v(tq + 1)}"),
                    Ins(f"v_cmp_le_u64_e64 {c}, {self.qq()}, {vp(R)}", wr=[c]),
                    Ins(f"v_cndmask_b32_e64 {v(M)}, 0, {self.nql()}, {c}", rd=[c]),
                    Ins(f"v_cndmask_b32_e64 {v(M + 1)}, 0, {self.nqh()}, {c}", rd=[c]),
                    Ins(f"v_lshl_add_u64 {xop[k]}, {vp(M)}, 0, {vp(R)}"),
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
             "// Hand-scheduled forward NTT rounds for primes in (2^60 - 2^56, 2^60); see the generator's docstring.\n"
             "// Included inside namespace exacto by ntt.hip.\n#pragma once\n\n"
             "struct AsmK {\n"
             "    uint32_t n0, n1;      // 2^64 - q\n"
             "    uint32_t q2l, q2h;    // 2q\n"
             "    uint32_t nq8l, nq8h;  // 2^64 - 8q\n"
             "    uint32_t nql, nqh;    // 2^64 - q (VGPR copies for v_cndmask)\n"
             "    u64 q8, q;\n"
             "};\n\n"
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
