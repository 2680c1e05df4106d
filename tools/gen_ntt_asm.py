#!/usr/bin/env python3
"""Generates exacto_amd/csrc/ntt_asm.inc: hand-scheduled gfx950 inline-asm rounds of the forward
(Cooley-Tukey) and inverse (Gentleman-Sande) negacyclic NTT with Shoup twiddles, for primes q in
(2^60 - 2^32, 2^60).  Run it after editing; the output is committed.

Why asm: gfx950 has no 64-bit add/sub/compare with carry-out to a VGPR, so every 64-bit
subtraction and every 65-bit sum is a VALU carry chain through an SGPR pair, and a VALU that
reads an SGPR written by a VALU needs 2 wait states.  hipcc schedules one butterfly at a time
and pads each chain with s_nop (the compiler-scheduled inverse issued 12.9k VALU per 4096-point
polynomial, the forward below 7.7k).  Here W butterflies are interleaved with explicit carry
pairs, so every carry read has its 2 wait states filled by independent work; pad_hazards()
inserts s_nop only where a gap remains (and is the safety net for the rule).

Issue costs measured on MI355X (tools/op_rate.hip, cycles per wave-instruction per SIMD): v_add /
v_sub / v_and / v_mov / v_lshrrev_b32 ~2.5; every multiply, mad, carry op, 64-bit op, add3,
cndmask_e64, bfi, alignbit ~4.2-5.  The sequences below are written for that table.

Shoup product T = Y*w mod q for any Y < 2^64 (w < q, ws = floor(w * 2^64 / q)), 10 or 11 slow +
2 fast instructions:
  qh = hi64(Y * ws):  A = y1*s0 + Z with Z = mulhi(y0,s0) (exact) or Z = 0 (APPROX); B = y0*s1 + A
       with the carry-out of v_mad_u64_u32 in an SGPR pair; D = (B.hi, carry) by v_mov + v_cndmask;
       qh = y1*s1 + D.  Dropping the low-low partial product lowers qh by at most 1, so T grows
       from [0, 2q) to [0, 3q): one multiply less per butterfly for a wider bound.
  T  = lo64(Y*w + qh*(2^64-q)):  E = y0*w0; E += qh0*n0 (two mads); the high-word cross terms
       y0*w1 + y1*w0 + qh0*n1 + qh1*n0 as one mul_lo + three mads on a 32-bit chain (the high
       word of a mad's 64-bit addend never reaches the low word of its result); T.hi += chain.
Forward butterfly (X < bound, Y anything): out0 = X + T, out1 = X + (cq - T), c = 2 or 3.
Inverse butterfly (U, V with bounds mu + mv <= 16): D = U + (mv*q - V) (sub_co/subb + one 64-bit
add), U' = U + V, V' = T = Shoup(D, w).  Bounds are tracked per value at generation time; a value
that would push a sum past 16q is first reduced.
Reduction of a value x < 2^64 for q = 2^60 - d, d < 2^32 (so 2^64 - q = (0xF0000000, d)):
  t = x.hi >> 28; r = x + t*(2^64 - q) = x - t*q, by one mad (low word d) and a subtraction of
  t << 28 from the high word; r = (x mod 2^60) + t*d < 2q.
Forward round-start reduction (rounds >= 1): only the 8 values that are X of the round's first
stage are reduced (< 2q; a Shoup input may be anything below 2^64, and both butterfly outputs are
bounded by X's bound + cq per stage), so the round ends below 2q + 4cq <= 14q < 16q.
Final forward round: the reduction above, then r - q, selected by the sign of r - q (and-mask + add).
Final inverse stage: n^-1 folded in (x0 = (U+V)*n^-1, x1 = D*psi_inv_rev[1]*n^-1), exact Shoup,
then the same canonical reduction.
Generic rounds (FwdRoundGenAsm / InvRoundGenAsm, any q < 2^60: the HPS primes of compact_bfv and
u64_dbfv): the Shoup chain is the same (it only uses 2^64 - q); every reduction is instead a chain
of conditional subtractions of (bound/2) q, each c = (m q <= x) by one 64-bit compare, x + (2^64 -
m q) by one 64-bit add and two selects, in that order so the mask is read 2 instructions after its
write (no s_nop).  Forward: round start 8q, 4q, 2q; final chain down to q.

Register model: one asm statement per round.  The 16 values enter and leave through "+v" u64
operands tied to x[k]; the first stage also takes u32 halves of its inputs.  Tied operands are
written only once every input of the round has been read (the round's last stage, or the final
reduction).  Forward: values live in fixed VGPR pairs between stages, one temp set per butterfly
stream.  Inverse: values and temps share one pool of VGPR pairs with renaming (the sum overwrites
U's pair, the Shoup result's temp pair becomes V's home and V's old pair becomes the next temp).
Hazard rule (LLVM GCNHazardRecognizer, gfx940+ VALUWriteSGPRVALURead): a VALU reading an SGPR
written by a VALU (carry-in, cndmask mask) needs 2 wait states after the write.  gfx9 reads at
most one SGPR (or literal) per VALU instruction, so carry-in instructions take their other
constant operand (2q, 3q, m*q high words) from a VGPR.
"""

import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "exacto_amd", "csrc", "ntt_asm.inc")

VBASE = int(os.environ.get("EXACTO_ASM_VBASE", "104"))   # first physical VGPR of the statements
W = int(os.environ.get("EXACTO_ASM_STREAMS", "2"))       # butterflies interleaved per group
SGPR_C = [80, 82, 84, 88, 90, 92][:max(W, 2)]            # carry pair of each stream
SGPR_SD = 86                  # sink for the carry-out of v_mad_u64_u32 where it is not used
SGPR_RED = [80, 82, 84, 88]   # carry pairs of the generic rounds' four reduction streams
INV_BOUND_IN = 4              # inverse round 0 input bound (the fused tensor's c1 < 4q)
GEN_LOGN = (10, 12, 13)       # transform sizes with generic-prime rounds (cfg1: n = 1024; u64_dbfv: 4096)
# smaller-prime forms per size (q < 2^qbits): compact_bfv's q and p (2^40, 2^49) at n = 1024,
# u64_dbfv's auxiliary primes (2^54, 2^55) at n = 4096
GEN_QBITS = {10: (50,), 12: (56,)}


def v(i):
    return f"v{i}"


def vp(i):
    return f"v[{i}:{i + 1}]"


def sp(i):
    return f"s[{i}:{i + 1}]"


def lo(pair):
    """Low VGPR of a pair operand 'v[a:b]'."""
    return "v" + pair[2:pair.index(":")]


def hi(pair):
    return "v" + pair[pair.index(":") + 1:-1]


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


class Statement:
    """Operand bookkeeping of one asm statement."""

    def __init__(self):
        self.ins = []                            # (name, constraint, expr)
        self.seen = set()

    def _in(self, key, cons, expr):
        if key not in self.seen:
            self.ins.append((key, cons, expr))
            self.seen.add(key)
        return "%[" + key + "]"

    def n0(self): return self._in("n0", "s", "K.n0")
    def n1(self): return self._in("n1", "s", "K.n1")
    def ql(self): return self._in("ql", "s", "K.ql")
    def qh(self): return self._in("qh", "s", "K.qh")
    def nq(self): return self._in("nq", "s", "K.nq")

    def mq(self, m): return self._in(f"mq{m}", "s", f"K.q * {m}u")
    def nmq(self, m): return self._in(f"nmq{m}", "s", f"(u64)0 - K.q * {m}u")
    def cql(self, c): return self._in(f"q{c}l", "s", f"(uint32_t)(K.q * {c}u)")
    def cqh(self, c): return self._in(f"q{c}h", "v", f"(uint32_t)((K.q * {c}u) >> 32)")

    def xh(self, k): return self._in(f"x{k}h", "v", f"(uint32_t)(x[{k}] >> 32)")
    def xl(self, k): return self._in(f"x{k}l", "v", f"(uint32_t)x[{k}]")


def shoup_seq(st, yl, yh, w0, w1, s0, s1, T, c, approx, fixup=True, E=None, addend="0"):
    """Instructions computing E = addend + Shoup(Y, w) mod 2^64 (Shoup in [0, 2q) exact, [0, 3q)
    approx).  T: temp pairs Z (Z.hi == 0, exact only), A, B, E, F; c: this stream's carry SGPR pair.
    E: the result pair (default T['E']; must be addressable by halves); addend: a 64-bit operand
    added for free by the first mad (the forward butterfly's X).  fixup=False leaves out the last
    instruction (E.hi += F.lo) for the caller to place: E.lo is final before it."""
    SD = sp(SGPR_SD)
    Z, A, B, _, F = (T.get(n) for n in "ZABEF")
    E = E or T.get("E")
    seq = []
    if approx:
        seq.append(Ins(f"v_mad_u64_u32 {A}, {SD}, {yh}, {s0}, 0", wr=[SD]))
    else:
        seq.append(Ins(f"v_mul_hi_u32 {lo(Z)}, {yl}, {s0}"))
        seq.append(Ins(f"v_mad_u64_u32 {A}, {SD}, {yh}, {s0}, {Z}", wr=[SD]))
    seq += [
        Ins(f"v_mad_u64_u32 {B}, {c}, {yl}, {s1}, {A}", wr=[c]),
        Ins(f"v_mad_u64_u32 {E}, {SD}, {yl}, {w0}, {addend}", wr=[SD]),
        Ins(f"v_mov_b32 {lo(A)}, {hi(B)}"),
        Ins(f"v_mul_lo_u32 {lo(F)}, {yl}, {w1}"),
        Ins(f"v_cndmask_b32_e64 {hi(A)}, 0, 1, {c}", rd=[c]),
        Ins(f"v_mad_u64_u32 {F}, {SD}, {yh}, {w0}, {F}", wr=[SD]),
        Ins(f"v_mad_u64_u32 {A}, {SD}, {yh}, {s1}, {A}", wr=[SD]),
        Ins(f"v_mad_u64_u32 {E}, {SD}, {lo(A)}, {st.n0()}, {E}", wr=[SD]),
    ]
    seq += [
        Ins(f"v_mad_u64_u32 {F}, {SD}, {lo(A)}, {st.n1()}, {F}", wr=[SD]),
        Ins(f"v_mad_u64_u32 {F}, {SD}, {hi(A)}, {st.n0()}, {F}", wr=[SD]),
    ]
    if fixup:
        seq.append(fix_seq(E, F))
    return seq


def fix_seq(E, F):
    return Ins(f"v_add_u32 {hi(E)}, {hi(E)}, {lo(F)}")


def reduce_seq(st, dst, src, src_hi, t, u):
    """dst (pair) = src - floor(src / 2^60) * q  in [0, 2q).  t, u: temp VGPRs (32-bit names)."""
    return [
        Ins(f"v_lshrrev_b32 {t}, 28, {src_hi}"),
        Ins(f"v_mad_u64_u32 {dst}, {sp(SGPR_SD)}, {t}, {st.n0()}, {src}", wr=[sp(SGPR_SD)]),
        Ins(f"v_lshlrev_b32 {u}, 28, {t}"),
        Ins(f"v_sub_u32 {hi(dst)}, {hi(dst)}, {u}"),
    ]


def halve_seq(st, dst, src, m, t, c, halves=None):
    """dst = src - m q if src >= m q else src (pairs; any prime q < 2^60, no special form): the
    generic reduction step of InvRound / Round(generic=True).  t: temp pair; c: this stream's mask
    pair; halves: the source's (low, high) 32-bit operands for the selects when src is a tied 64-bit
    operand.  The compare goes first, so its mask is read by the selects 2 instructions later and the
    step needs no s_nop even in a single stream: c = (m q <= src), t = src + (2^64 - m q), select."""
    sl, sh = halves if halves else (lo(src), hi(src))
    return [
        Ins(f"v_cmp_le_u64_e64 {c}, {st.mq(m)}, {src}", wr=[c]),
        Ins(f"v_lshl_add_u64 {t}, {src}, 0, {st.nmq(m)}"),
        Ins(f"v_cndmask_b32_e64 {lo(dst)}, {sl}, {lo(t)}, {c}", rd=[c]),
        Ins(f"v_cndmask_b32_e64 {hi(dst)}, {sh}, {hi(t)}, {c}", rd=[c]),
    ]


def halve_chain(bound):
    """The conditional subtractions that take a value below bound * q to [0, q): (bound / 2) q,
    then (bound / 4) q, ... q, each halving the bound."""
    out, b = [], bound
    while b > 1:
        half = 1
        while 2 * half < b:
            half *= 2
        out.append(half)
        b = half
    return out


def canon_seq(st, dst, r, S, M):
    """dst = r mod q for r < 2q: s = r - q, out = s + (q & sign(s)).  S, M: temp pairs."""
    return [
        Ins(f"v_lshl_add_u64 {S}, {r}, 0, {st.nq()}"),
        Ins(f"v_ashrrev_i32 {lo(M)}, 31, {hi(S)}"),
        Ins(f"v_and_b32 {hi(M)}, {st.qh()}, {lo(M)}"),
        Ins(f"v_and_b32 {lo(M)}, {st.ql()}, {lo(M)}"),
        Ins(f"v_lshl_add_u64 {dst}, {S}, 0, {M}"),
    ]


def emit_statement(struct, st, seq, vmax, comment, run_args):
    seq = pad_hazards(seq)
    body = "\\n\\t".join(i.text for i in seq)
    clob = [f'"v{i}"' for i in range(VBASE, vmax)]
    clob += [f'"s{i}"' for p in sorted(set(SGPR_C + SGPR_RED + [SGPR_SD])) for i in (p, p + 1)]
    clob.append('"memory"')   # keeps the next round's twiddle loads below the statement
    outs = ", ".join(f'[x{k}] "+v"(x[{k}])' for k in range(16))
    ins = ", ".join(f'[{k}] "{c}"({e})' for k, c, e in st.ins)
    nops = sum(1 for i in seq if i.text.startswith("s_nop"))
    valu = sum(1 for i in seq if i.valu)
    return (f"// {comment}, {valu} VALU, {nops} s_nop\n"
            f"template <> struct {struct} {{\n"
            f"    static __device__ __forceinline__ void run({run_args}) {{\n"
            f"        asm volatile(\"{body}\"\n            : {outs}\n            : {ins}\n"
            f"            : {', '.join(clob)});\n    }}\n}};\n")


PIN_BASE = int(os.environ.get("EXACTO_PIN_BASE", "72"))   # first home VGPR of the pinned rounds


def pin_homes_decl():
    """The register variables the pinned statements keep their values in (x[k] = xh_k:xl_k)."""
    decl = ", ".join(f"xl{k} asm(\"v{PIN_BASE + 2 * k}\"), xh{k} asm(\"v{PIN_BASE + 2 * k + 1}\")"
                     for k in range(16))
    return f"#define EXACTO_PIN_DECL register uint32_t {decl};\n"


def emit_pinned(name, st, seq, vmax, comment):
    """A pinned round as a macro over the enclosing kernel's register variables xl0..xh15 (bound to
    the home pairs by EXACTO_PIN_DECL): they are "+v" operands, so hipcc keeps each in its register
    at the statement, and the body addresses them by their physical names; only the temps are
    clobbered.  Macro arguments: tw (const TwPair[15]) and K (AsmK)."""
    seq = pad_hazards(seq)
    body = "\\n\\t".join(i.text for i in seq)
    base = PIN_BASE + 32
    clob = [f'"v{i}"' for i in range(base, vmax)]
    clob += [f'"s{i}"' for p in sorted(set(SGPR_C + SGPR_RED + [SGPR_SD])) for i in (p, p + 1)]
    clob.append('"memory"')
    outs = ", ".join(f'"+v"(xl{k}), "+v"(xh{k})' for k in range(16))
    ins = ", ".join(f'[{k}] "{c}"({e})' for k, c, e in st.ins)
    nops = sum(1 for i in seq if i.text.startswith("s_nop"))
    valu = sum(1 for i in seq if i.valu)
    return (f"// {comment}, {valu} VALU, {nops} s_nop\n"
            f"#define {name}(tw, K) \\\n"
            f"    asm volatile(\"{body}\" \\\n        : {outs} \\\n        : {ins} \\\n"
            f"        : {', '.join(clob)})\n")


class Round(Statement):
    """One forward round (stage bits BHI..LO of a 4-bit window) as one asm statement."""

    def __init__(self, logn, r, approx=True, addx=True, pinned=False, generic=False, qbits=60, bound_in=None,
                 lazy_out=False, perm=None):
        super().__init__()
        self.logn, self.r, self.approx, self.addx, self.pinned = logn, r, approx, addx, pinned
        # perm (pinned only): value k lives in home perm[k] (the lane-pair exchange leaves the values
        # of the 8192-point forward's last round there, LanePairXchg)
        self.perm = perm
        # lazy_out (last round, special primes: the extension transforms that only the asm tensor
        # products read): the final values are left in [0, 2q) after the fold, no canonical step
        self.lazy_out = lazy_out
        # generic: any prime q < 2^60 (the HPS primes): the round-start reduction of X from < 16q to
        # < 2q is three conditional subtractions (8q, 4q, 2q; halve_seq) instead of the special-prime
        # fold, and the final canonical reduction a chain of them down to q.
        # qbits < 60 (generic only, q < 2^qbits): values may grow to 2^64 / 2^qbits q before a
        # reduction, so the round-start reduction is left out while the round's outputs stay below
        # that (bound_in: the inputs' bound in units of q, from fwd_rounds)
        self.generic, self.qbits = generic, qbits
        self.cap = 16 if qbits >= 60 else (1 << (64 - qbits))
        self.c = 3 if approx else 2            # Shoup output bound (units of q)
        self.lo = max(logn - 4 * (r + 1), 0)
        self.bhi = logn - 1 - 4 * r
        self.last = self.lo == 0
        self.uniform_tw = self.lo + 4 >= logn     # thigh == 0: twiddles are block-uniform (SGPR)
        nst = self.bhi - self.lo + 1
        self.bound_in = bound_in if bound_in is not None else (1 if r == 0 else 16)
        # X's bound at the round start: canonical in round 0; reduced to < 2q unless the round's
        # outputs stay below cap q unreduced
        if r == 0:
            self.xbound, self.reduce_x = 1, False
        elif qbits < 60 and self.bound_in + self.c * nst <= self.cap:
            self.xbound, self.reduce_x = self.bound_in, False
        else:
            self.xbound, self.reduce_x = 2, True
        # bound of the round's outputs (units of q): X's bound plus c per stage
        self.bound_last = self.xbound + self.c * nst   # before a final reduction
        self.bound_out = 1 if self.last else self.bound_last

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
        base = PIN_BASE if self.pinned else VBASE
        P = [base + 2 * (self.perm[k] if self.perm else k) for k in range(16)]
        TB = base + 32
        # 10 VGPRs per stream: Z (Z.hi stays 0), A (= D = qh), B (then cq - T), E (T), F (cross chain)
        temps = [dict(Z=TB + 10 * j, A=TB + 10 * j + 2, B=TB + 10 * j + 4, E=TB + 10 * j + 6,
                      F=TB + 10 * j + 8) for j in range(max(W, 2))]
        self.vmax = TB + 10 * len(temps)
        C = SGPR_C
        seq = [Ins("s_nop 1", valu=False)]      # an "s" operand may come straight from a VALU
        if not self.approx:
            for t in temps:
                seq.append(Ins(f"v_mov_b32 {v(t['Z'] + 1)}, 0"))

        st = self.stages()
        nstage = len(st)
        if nstage < 2 and not self.last:
            raise SystemExit("single-stage non-final round not supported")
        first_lb = st[0][0]
        # pinned: the values live in their home pairs P for the whole kernel (register variables
        # bound to them), so every stage reads and writes the homes and nothing goes to tied operands
        xop = {k: (vp(P[k]) if self.pinned else f"%[x{k}]") for k in range(16)}
        in_p = {k: self.pinned for k in range(16)}

        # the generic reductions run as four streams (carry pairs SGPR_RED, temp pairs B and E of
        # the two butterfly temp sets, free outside the butterflies) so that no carry read waits
        red_t = [vp(temps[0]["B"]), vp(temps[1]["B"]), vp(temps[0]["E"]), vp(temps[1]["E"])]
        if self.reduce_x:   # round-start reduction of the first stage's X values into P
            red = [k for k in range(16) if not (k >> first_lb) & 1]
            streams = [[] for _ in range(4 if self.generic else len(temps))]
            for i, k in enumerate(red):
                j = i % len(streams)
                t = temps[j % len(temps)]
                src_hi = v(P[k] + 1) if self.pinned else self.xh(k)
                if self.generic:
                    srch = None if self.pinned else (self.xl(k), self.xh(k))
                    for i2, m in enumerate(halve_chain(self.bound_in)[:-1]):   # down to < 2q
                        first = i2 == 0 and not self.pinned
                        streams[j] += halve_seq(self, vp(P[k]), xop[k] if first else vp(P[k]), m, red_t[j],
                                                sp(SGPR_RED[j]), halves=srch if first else None)
                else:
                    streams[j] += reduce_seq(self, vp(P[k]), xop[k], src_hi, v(t["B"]), v(t["B"] + 1))
                in_p[k] = True
            seq += interleave(streams)

        for si, (lb, bfs) in enumerate(st):
            direct_out = si == nstage - 1 and not self.last and not self.pinned
            for pi in range(0, len(bfs), W):
                streams = []
                for j, (k0, k1, slot) in enumerate(bfs[pi:pi + W]):
                    t = temps[j]
                    c = sp(C[j])
                    T = {n: vp(t[n]) for n in "ZABEF"}
                    if in_p[k1]:
                        yl, yh = v(P[k1]), v(P[k1] + 1)
                    else:
                        yl, yh = self.xl(k1), self.xh(k1)
                    X = vp(P[k0]) if in_p[k0] else xop[k0]
                    o0, o1 = (xop[k0], xop[k1]) if direct_out else (vp(P[k0]), vp(P[k1]))
                    if not direct_out and self.addx:
                        # o0 = X + T straight from the Shoup chain (X is its first mad's addend), and
                        # o1 = (2X + cq) - o0 = X + cq - T (mod 2^64; the true value is < 16q):
                        # one 64-bit add less per butterfly.  2X + cq goes to the E pair before
                        # the chain overwrites X's pair (o0 is usually X's own pair).
                        Zt = T["E"]
                        s = [Ins(f"v_lshl_add_u64 {Zt}, {X}, 1, {self.mq(self.c)}")]
                        s += shoup_seq(self, yl, yh, self.tw(slot, "w0"), self.tw(slot, "w1"),
                                       self.tw(slot, "s0"), self.tw(slot, "s1"), T, c, self.approx,
                                       fixup=False, E=o0, addend=X)
                        s += [
                            Ins(f"v_sub_co_u32_e64 {lo(o1)}, {c}, {lo(Zt)}, {lo(o0)}", wr=[c]),
                            fix_seq(o0, T["F"]),
                            Ins(f"v_subb_co_u32_e64 {hi(o1)}, {c}, {hi(Zt)}, {hi(o0)}, {c}", rd=[c], wr=[c]),
                        ]
                        streams.append(s)
                        in_p[k0] = in_p[k1] = True
                        continue
                    s = shoup_seq(self, yl, yh, self.tw(slot, "w0"), self.tw(slot, "w1"),
                                  self.tw(slot, "s0"), self.tw(slot, "s1"), T, c, self.approx, fixup=False)
                    s += [
                        # cq - T: the low word first, the E.hi fix-up fills the carry's wait states
                        Ins(f"v_sub_co_u32_e64 {v(t['B'])}, {c}, {self.cql(self.c)}, {v(t['E'])}", wr=[c]),
                        fix_seq(T["E"], T["F"]),
                        Ins(f"v_subb_co_u32_e64 {v(t['B'] + 1)}, {c}, {self.cqh(self.c)}, {v(t['E'] + 1)}, {c}",
                            rd=[c], wr=[c]),
                        # o1 first: o0 may be X's own register pair
                        Ins(f"v_lshl_add_u64 {o1}, {T['B']}, 0, {X}"),
                        Ins(f"v_lshl_add_u64 {o0}, {T['E']}, 0, {X}"),
                    ]
                    streams.append(s)
                    if not direct_out:
                        in_p[k0] = in_p[k1] = True
                seq += interleave(streams)

        if self.last:
            # canonical reduction of all 16 values (< 16q) into the tied operands
            streams = [[] for _ in range(4 if self.generic else len(temps))]
            for k in range(16):
                j = k % len(streams)
                t = temps[j % len(temps)]
                R = vp(P[k])
                if self.generic:
                    for m in halve_chain(self.bound_last):
                        streams[j] += halve_seq(self, R, R, m, red_t[j], sp(SGPR_RED[j]))
                    if not self.pinned:
                        streams[j].append(Ins(f"v_lshl_add_u64 {xop[k]}, {R}, 0, 0"))
                    continue
                streams[j] += reduce_seq(self, R, R, v(P[k] + 1), v(t["B"]), v(t["B"] + 1))
                if not self.lazy_out:
                    streams[j] += canon_seq(self, xop[k], R, vp(t["E"]), vp(t["F"]))
                elif xop[k] != R:
                    streams[j].append(Ins(f"v_lshl_add_u64 {xop[k]}, {R}, 0, 0"))
            seq += interleave(streams)
        return seq

    def emit(self):
        seq = self.gen()
        if self.pinned:
            sfx = ("_LP" if self.perm else "") + ("_LZ" if self.lazy_out else "")
            return emit_pinned(f"EXACTO_FWD_PIN_{self.logn}_{self.r}{sfx}", self, seq,
                               self.vmax,
                               f"round {self.r} of the {1 << self.logn}-point forward NTT, pinned homes"
                               f"{' (value k in home PERM_LP[k])' if self.perm else ''}: "
                               f"stage bits {self.bhi}..{self.lo}")
        struct = f"FwdRoundGenAsm<{self.logn}, {self.r}, {self.qbits}>" if self.generic else \
            f"FwdRoundAsm<{self.logn}, {self.r}>"
        return emit_statement(struct, self, seq, self.vmax,
                              f"round {self.r} of the {1 << self.logn}-point forward NTT"
                              f"{f' for any prime below 2^{self.qbits}' if self.generic else ''}: stage bits "
                              f"{self.bhi}..{self.lo}, inputs < {self.bound_in}q, "
                              f"{'round-start reduction' if self.reduce_x else 'no round-start reduction'}",
                              "u64 (&x)[16], const TwPair (&tw)[15], const AsmK& K")


# The lane-pair exchange (LanePairXchg): value 2j of the last round in home j, value 2j + 1 in home 8 + j
PERM_LP = [k // 2 + 8 * (k % 2) for k in range(16)]


class LanePairXchg(Statement):
    """The 8192-point forward's last exchange (element layout LO = 1 -> LO = 0) without LDS.  In the
    LO = 1 layout thread 2s + b holds elements 32 s + 2 k + b (value k); in LO = 0 thread t holds 16 t + k.
    Both are the 32 elements 32 s .. 32 s + 31 spread over the lane pair (2s, 2s + 1), so the exchange is
    a swap of 8 values between adjacent lanes: the even lane keeps its values 0..7 (new values 0, 2, ..,
    14) and takes the odd lane's 0..7 (new 1, 3, .., 15); the odd lane takes the even lane's 8..15
    (new 0, 2, ..) and keeps its own 8..15 (new 1, 3, ..).  Written in place: new value 2j goes to home j,
    2j + 1 to home 8 + j (PERM_LP; the last round and the stores read them there).  Per value pair j and
    32-bit half: T = dpp(home j) (the partner's), home j = even ? home j : dpp(home 8 + j), home 8 + j =
    even ? T : home 8 + j -- a v_mov_b32_dpp, a v_cndmask_b32_dpp and a v_cndmask_b32 with VCC = the
    even lanes; quad_perm [1, 0, 3, 2] swaps adjacent lanes.  48 VALU instead of 16 ds_write_b64 + 16
    ds_read_b64 and two s_barrier."""

    def gen(self):
        P = [PIN_BASE + 2 * k for k in range(16)]
        T = PIN_BASE + 32
        self.vmax = T + 2
        dpp = "quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf"
        seq = [Ins(f"v_and_b32 {v(T)}, 1, %[tid]"),
               Ins(f"v_cmp_eq_u32_e32 vcc, 0, {v(T)}"),
               Ins("s_nop 1", valu=False)]    # VCC and the homes (DPP sources) were written by a VALU
        for j in range(8):
            for h in (0, 1):
                a, b = P[j] + h, P[8 + j] + h
                seq += [Ins(f"v_mov_b32_dpp {v(T + h)}, {v(a)} {dpp}"),
                        Ins(f"v_cndmask_b32_dpp {v(a)}, {v(b)}, {v(a)}, vcc {dpp}"),
                        Ins(f"v_cndmask_b32_e32 {v(b)}, {v(b)}, {v(T + h)}, vcc")]
        return seq

    def emit(self):
        seq = self.gen()
        body = "\\n\\t".join(i.text for i in seq)
        clob = [f'"v{i}"' for i in range(PIN_BASE + 32, self.vmax)] + ['"vcc"']
        outs = ", ".join(f'"+v"(xl{k}), "+v"(xh{k})' for k in range(16))
        valu = sum(1 for i in seq if i.valu)
        return (f"// the 8192-point forward's last exchange within lane pairs (DPP), {valu} VALU\n"
                f"#define EXACTO_XCHG_PIN_LP(TID) \\\n"
                f"    asm volatile(\"{body}\" \\\n        : {outs} \\\n        : [tid] \"v\"(TID) \\\n"
                f"        : {', '.join(clob)})\n")


class InvRound(Statement):
    """One inverse round (Gentleman-Sande, stage bits BLO..BHI ascending) as one asm statement.
    bound_in: every input value < bound_in * q."""

    def __init__(self, logn, r, bound_in, approx=True, generic=False, qbits=60, lazy_out=False):
        super().__init__()
        self.logn, self.r, self.approx = logn, r, approx
        # lazy_out (the last round of the tensor kernels' inverse): the final stage's exact Shoup
        # products are left in [0, 2q) (every consumer of the tensor's output takes them:
        # DESIGN.md §6.4), one 64-bit move instead of the 5-instruction canonical reduction
        self.lazy_out = lazy_out
        # qbits < 60 (generic, q < 2^qbits): sums may reach 2^64 / 2^qbits q before a halving
        self.qbits = qbits
        self.cap = 16 if qbits >= 60 else (1 << (64 - qbits))
        # generic: any prime q < 2^60 (the HPS auxiliary primes): a sum that would pass 16q first
        # halves its larger operand's bound by one conditional subtraction of (bound / 2) q
        # (halve_seq, 4 VALU) instead of the special-prime fold to < 2q (reduce_seq)
        self.generic = generic
        self.tb = 3 if approx else 2             # Shoup output bound (units of q)
        self.lo = min(4 * r, logn - 4)
        self.blo = 4 * r
        self.bhi = min(4 * r + 3, logn - 1)
        self.last = self.bhi == logn - 1
        self.uniform_tw = self.lo + 4 >= logn
        self.bound_in = bound_in
        self.bound_out = None

    def tw(self, slot, part):
        c = "s" if self.uniform_tw else "v"
        expr = {"w0": f"(uint32_t)tw[{slot}].w", "w1": f"(uint32_t)(tw[{slot}].w >> 32)",
                "s0": f"(uint32_t)tw[{slot}].ws", "s1": f"(uint32_t)(tw[{slot}].ws >> 32)"}[part]
        return self._in(f"t{slot}{part}", c, expr)

    def kc(self, name):
        """Final-stage constants (n^-1 and psi_inv_rev[1] * n^-1, Shoup form), block-uniform."""
        return self._in(name, "s", "K." + name)

    def stages(self):
        res, slot = [], 0
        for b in range(self.blo, self.bhi + 1):
            lb = b - self.lo
            half = 1 << lb
            bfs = []
            for g in range(8 >> lb):
                for m in range(half):
                    k0 = g * 2 * half + m
                    bfs.append((k0, k0 + half, None if b == self.logn - 1 else slot + g))
            if b != self.logn - 1:
                slot += 8 >> lb
            res.append((b == self.logn - 1, bfs))
        return res

    def gen(self):
        # pool of VGPR pairs: 16 value homes (values enter in the tied x operands), plus per
        # stream A, B, F, D (and Z when exact) fixed temps and a rotating E
        nfixed = 4 if self.approx else 5
        npairs = 16 + max(W, 2) * (nfixed + 1) + max(W, 2)
        pool = [VBASE + 2 * i for i in range(npairs)]
        self.vmax = VBASE + 2 * npairs
        free = list(pool)

        def alloc():
            return vp(free.pop(0))

        temps = []
        seq = [Ins("s_nop 1", valu=False)]
        for j in range(max(W, 2)):
            t = {n: alloc() for n in ("ABFD" if self.approx else "ZABFD")}
            t["E"] = alloc()
            temps.append(t)
            if not self.approx:
                seq.append(Ins(f"v_mov_b32 {hi(t['Z'])}, 0"))
        loc = {k: None for k in range(16)}      # None: still in the tied operand x[k]
        bnd = {k: self.bound_in for k in range(16)}
        st = self.stages()
        nstage = len(st)
        C = SGPR_C

        def val64(k):
            return f"%[x{k}]" if loc[k] is None else loc[k]

        def halves(k):
            if loc[k] is None:
                return self.xl(k), self.xh(k)
            return lo(loc[k]), hi(loc[k])

        for si, (final, bfs) in enumerate(st):
            direct = si == nstage - 1        # outputs into the tied operands
            for pi in range(0, len(bfs), W):
                streams = []
                # pairs released by this batch's butterflies become allocatable only after the
                # batch: its streams are interleaved, so a pair one stream frees may still be read
                # by that stream after the other stream's instruction that would reuse it
                released = []
                for j, (k0, k1, slot) in enumerate(bfs[pi:pi + W]):
                    t = temps[j]
                    c = sp(C[j])
                    s = []
                    # keep the pair sum and the difference below cap q (16q: 2^64 at q < 2^60)
                    for _ in range(8 if self.generic else 2):
                        if bnd[k0] + bnd[k1] <= self.cap:
                            break
                        kr = k0 if bnd[k0] >= bnd[k1] else k1
                        if self.generic:
                            half = 1
                            while 2 * half < bnd[kr]:
                                half *= 2            # bnd[kr] in (half, 2 half]: subtract half q
                            if loc[kr] is None:   # the first step reads the tied operand
                                dst = alloc()
                                s += halve_seq(self, dst, f"%[x{kr}]", half, t["B"], c,
                                               halves=(self.xl(kr), self.xh(kr)))
                                loc[kr] = dst
                            else:
                                s += halve_seq(self, loc[kr], loc[kr], half, t["B"], c)
                            bnd[kr] = half
                            continue
                        if loc[kr] is None:
                            dst = alloc()
                            s += reduce_seq(self, dst, val64(kr), self.xh(kr), lo(t["B"]), hi(t["B"]))
                            loc[kr] = dst
                        else:
                            s += reduce_seq(self, loc[kr], loc[kr], hi(loc[kr]), lo(t["B"]), hi(t["B"]))
                        bnd[kr] = 2
                    m = bnd[k1]
                    vl, vh = halves(k1)
                    U, V = val64(k0), val64(k1)
                    D = t["D"]
                    # D = (U + m q) - V: the sum U + V goes between the two halves of the
                    # subtraction (U's last read is the first add; V.hi is read after the sum)
                    if final:
                        s0 = loc[k0] if loc[k0] is not None else alloc()
                    elif direct:
                        s0 = f"%[x{k0}]"
                    elif loc[k0] is None:
                        s0 = alloc()
                    else:
                        s0 = loc[k0]
                    s += [
                        Ins(f"v_lshl_add_u64 {D}, {U}, 0, {self.mq(m)}"),
                        Ins(f"v_sub_co_u32_e64 {lo(D)}, {c}, {lo(D)}, {vl}", wr=[c]),
                        Ins(f"v_lshl_add_u64 {s0}, {U}, 0, {V}"),
                        Ins(f"v_subb_co_u32_e64 {hi(D)}, {c}, {hi(D)}, {vh}, {c}", rd=[c], wr=[c]),
                    ]
                    if not final:
                        s += shoup_seq(self, lo(D), hi(D), self.tw(slot, "w0"), self.tw(slot, "w1"),
                                       self.tw(slot, "s0"), self.tw(slot, "s1"), t, c, self.approx)
                        old_v = loc[k1]
                        if direct:
                            s.append(Ins(f"v_lshl_add_u64 %[x{k1}], {t['E']}, 0, 0"))
                            released += [p for p in (loc[k0], old_v) if p is not None]
                            loc[k0] = loc[k1] = None
                        else:
                            loc[k0] = s0
                            loc[k1] = t["E"]                     # rename: E is V's new home
                            t["E"] = old_v if old_v is not None else alloc()
                        bnd[k0] = bnd[k0] + bnd[k1]
                        bnd[k1] = self.tb
                    else:
                        # last stage: x0 = (U+V) n^-1, x1 = D psi_inv_rev[1] n^-1, canonical; two
                        # exact Shoup products through the same temps, S in a spare pair
                        S = s0
                        ex = dict(t)
                        if self.approx:   # exact Shoup here: B doubles as Z (B.hi = 0 first)
                            ex["Z"] = t["B"]
                        for dst, y, w in ((f"%[x{k1}]", D, "l"), (f"%[x{k0}]", S, "n")):
                            if self.approx:
                                s.append(Ins(f"v_mov_b32 {hi(t['B'])}, 0"))
                            wn, sn = ("lw", "ls") if w == "l" else ("ni", "ns")
                            s += shoup_seq(self, lo(y), hi(y), self.kc(wn + "l"), self.kc(wn + "h"),
                                           self.kc(sn + "l"), self.kc(sn + "h"), ex, c, False)
                            if self.lazy_out:
                                s.append(Ins(f"v_lshl_add_u64 {dst}, {ex['E']}, 0, 0"))
                            else:
                                s += canon_seq(self, dst, ex["E"], ex["B"], ex["F"])
                        released += [p for p in {S, loc[k1]} if p is not None]
                        loc[k0] = loc[k1] = None
                        bnd[k0] = bnd[k1] = 2 if self.lazy_out else 1
                    streams.append(s)
                seq += interleave(streams)
                free.extend(int(lo(p)[1:]) for p in released)
        assert all(loc[k] is None for k in range(16))
        self.bound_out = max(bnd.values())
        return seq

    def emit(self):
        seq = self.gen()
        struct = f"InvRoundGenAsm<{self.logn}, {self.r}, {self.qbits}>" if self.generic else \
            f"InvRoundAsm<{self.logn}, {self.r}, true>" if self.lazy_out else f"InvRoundAsm<{self.logn}, {self.r}>"
        return emit_statement(struct, self, seq, self.vmax,
                              f"round {self.r} of the {1 << self.logn}-point inverse NTT"
                              f"{f' for any prime below 2^{self.qbits}' if self.generic else ''}: stage bits "
                              f"{self.blo}..{self.bhi}, inputs < {self.bound_in}q, outputs < "
                              f"{self.bound_out}q",
                              "u64 (&x)[16], const TwPair (&tw)[15], const AsmK& K")


class InvRoundPinned(InvRound):
    """An inverse round whose 16 values stay in fixed home pairs (PIN_BASE + 2k): the sum U + V
    overwrites U's home, the Shoup product of the difference is written straight into V's home (V
    is consumed by then), reductions are in place.  No renaming, so no value-home pool: the
    temps are A, B, F, D, E (and Z exact) per stream after the homes."""

    def gen(self):
        H = [PIN_BASE + 2 * k for k in range(16)]
        names = "ABFDE" if self.approx else "ZABFDE"
        TB = PIN_BASE + 32
        temps = [{n: vp(TB + 2 * (len(names) * j + i)) for i, n in enumerate(names)} for j in range(max(W, 2))]
        self.vmax = TB + 2 * len(names) * max(W, 2)
        seq = [Ins("s_nop 1", valu=False)]
        if not self.approx:
            for t in temps:
                seq.append(Ins(f"v_mov_b32 {hi(t['Z'])}, 0"))
        bnd = {k: self.bound_in for k in range(16)}
        C = SGPR_C
        for final, bfs in self.stages():
            for pi in range(0, len(bfs), W):
                streams = []
                for j, (k0, k1, slot) in enumerate(bfs[pi:pi + W]):
                    t = temps[j]
                    c = sp(C[j])
                    s = []
                    for _ in range(2):
                        if bnd[k0] + bnd[k1] <= 16:
                            break
                        kr = k0 if bnd[k0] >= bnd[k1] else k1
                        s += reduce_seq(self, vp(H[kr]), vp(H[kr]), v(H[kr] + 1), lo(t["B"]), hi(t["B"]))
                        bnd[kr] = 2
                    m = bnd[k1]
                    U, V, D = vp(H[k0]), vp(H[k1]), t["D"]
                    s += [
                        Ins(f"v_lshl_add_u64 {D}, {U}, 0, {self.mq(m)}"),
                        Ins(f"v_sub_co_u32_e64 {lo(D)}, {c}, {lo(D)}, {lo(V)}", wr=[c]),
                        Ins(f"v_lshl_add_u64 {U}, {U}, 0, {V}"),
                        Ins(f"v_subb_co_u32_e64 {hi(D)}, {c}, {hi(D)}, {hi(V)}, {c}", rd=[c], wr=[c]),
                    ]
                    if not final:
                        s += shoup_seq(self, lo(D), hi(D), self.tw(slot, "w0"), self.tw(slot, "w1"),
                                       self.tw(slot, "s0"), self.tw(slot, "s1"), t, c, self.approx, E=V)
                        bnd[k0] = bnd[k0] + bnd[k1]
                        bnd[k1] = self.tb
                    else:
                        ex = dict(t)
                        if self.approx:   # exact Shoup here: B doubles as Z (B.hi = 0 first)
                            ex["Z"] = t["B"]
                        for dst, y, w in ((V, D, "l"), (U, U, "n")):
                            if self.approx:
                                s.append(Ins(f"v_mov_b32 {hi(t['B'])}, 0"))
                            wn, sn = ("lw", "ls") if w == "l" else ("ni", "ns")
                            s += shoup_seq(self, lo(y), hi(y), self.kc(wn + "l"), self.kc(wn + "h"),
                                           self.kc(sn + "l"), self.kc(sn + "h"), ex, c, False)
                            if self.lazy_out:
                                s.append(Ins(f"v_lshl_add_u64 {dst}, {ex['E']}, 0, 0"))
                            else:
                                s += canon_seq(self, dst, ex["E"], ex["B"], ex["F"])
                        bnd[k0] = bnd[k1] = 2 if self.lazy_out else 1
                    streams.append(s)
                seq += interleave(streams)
        self.bound_out = max(bnd.values())
        return seq

    def emit(self):
        seq = self.gen()
        return emit_pinned(f"EXACTO_INV_PIN_{self.logn}_{self.r}{'_LZ' if self.lazy_out else ''}", self, seq, self.vmax,
                           f"round {self.r} of the {1 << self.logn}-point inverse NTT, pinned homes: stage "
                           f"bits {self.blo}..{self.bhi}, inputs < {self.bound_in}q, outputs < {self.bound_out}q")


def inv_rounds_pinned(logn, approx=True):
    out, b = [], INV_BOUND_IN
    for r in range((logn + 3) // 4):
        rd = InvRoundPinned(logn, r, b, approx)
        rd.gen()
        out.append(rd)
        b = rd.bound_out
    return out


def inv_rounds(logn, approx=True, generic=False, qbits=60):
    """The inverse rounds of one transform, each starting at the previous round's output bound."""
    out, b = [], INV_BOUND_IN
    for r in range((logn + 3) // 4):
        rd = InvRound(logn, r, b, approx, generic, qbits)
        rd.gen()
        out.append(rd)
        b = rd.bound_out
    return out


def fwd_rounds(logn, approx=True, addx=True, generic=False, qbits=60):
    """The forward rounds of one transform; with qbits < 60 each starts at the previous round's
    output bound (the 60-bit forms assume < 16q, their round-start reduction's input bound)."""
    out, b = [], None
    for r in range((logn + 3) // 4):
        rd = Round(logn, r, approx, addx, generic=generic, qbits=qbits, bound_in=b if qbits < 60 else None)
        out.append(rd)
        b = rd.bound_out
    return out


class MulPair(Statement):
    """W independent products r_k = a_k * b_k mod q (< 2q) for q = 2^60 - d, d < 2^24, a_k, b_k < 2^60
    (the tensor's variable x variable products).  P = a b = H 2^64 + m0 2^32 + t0 with
    T = a0 b0, M = a0 b1 + a1 b0 + T.hi (< 2^61: a1, b1 < 2^28), H = a1 b1 + M.hi (< 2^57);
    2^64 == 16 d = e and 2^60 == d fold it twice:
      S = (t0, m0 mod 2^28) + (m0 >> 28) d + H.lo e          (< 2^61 + 2^28)
      W = H.hi e + S.hi, value = W 2^32 + S.lo               (W < 2^54)
      r = (S.lo, W.lo mod 2^28) + (W >> 28) d                (< 2^60 + 2^50 < 2q)
    9 slow (8 mads, alignbit) + 6 fast instructions per product instead of the ~26 hipcc emits for
    the same C++ (mulmod_near60)."""

    def __init__(self, w=2, base=None, struct="MulNear60Asm", volatile=True):
        super().__init__()
        self.w = w
        # non-volatile: a pure function of its operands, so the scheduler may move loads across it
        # (an asm volatile statement is a scheduling barrier for every memory access)
        self.volatile = volatile
        self.base = VBASE if base is None else base
        self.struct = struct

    def a(self, k, h): return self._in(f"a{k}{h}", "v", f"(uint32_t)(a{k} >> {32 if h == 'h' else 0})")
    def b(self, k, h): return self._in(f"b{k}{h}", "v", f"(uint32_t)(b{k} >> {32 if h == 'h' else 0})")
    def d(self): return self._in("d", "s", "d")
    def e(self): return self._in("e", "s", "e")

    def gen(self):
        SD = sp(SGPR_SD)
        streams = []
        seq = [Ins("s_nop 1", valu=False)]
        for k in range(self.w):
            base = self.base + 14 * k
            T, Z, M, H, S, Wp = (vp(base + 2 * i) for i in range(6))
            U = v(base + 12)
            R = f"%[r{k}]"
            al, ah, bl, bh = self.a(k, "l"), self.a(k, "h"), self.b(k, "l"), self.b(k, "h")
            seq.append(Ins(f"v_mov_b32 {hi(Z)}, 0"))
            streams.append([
                Ins(f"v_mad_u64_u32 {T}, {SD}, {al}, {bl}, 0", wr=[SD]),
                Ins(f"v_mov_b32 {lo(Z)}, {hi(T)}"),
                Ins(f"v_mad_u64_u32 {M}, {SD}, {al}, {bh}, {Z}", wr=[SD]),
                Ins(f"v_mad_u64_u32 {M}, {SD}, {ah}, {bl}, {M}", wr=[SD]),
                Ins(f"v_mov_b32 {lo(Z)}, {hi(M)}"),
                Ins(f"v_mad_u64_u32 {H}, {SD}, {ah}, {bh}, {Z}", wr=[SD]),
                Ins(f"v_lshrrev_b32 {U}, 28, {lo(M)}"),
                Ins(f"v_and_b32 {hi(T)}, 0x0fffffff, {lo(M)}"),
                Ins(f"v_mad_u64_u32 {S}, {SD}, {U}, {self.d()}, {T}", wr=[SD]),
                Ins(f"v_mad_u64_u32 {S}, {SD}, {lo(H)}, {self.e()}, {S}", wr=[SD]),
                Ins(f"v_mov_b32 {lo(Z)}, {hi(S)}"),
                Ins(f"v_mad_u64_u32 {Wp}, {SD}, {hi(H)}, {self.e()}, {Z}", wr=[SD]),
                Ins(f"v_alignbit_b32 {U}, {hi(Wp)}, {lo(Wp)}, 28"),
                Ins(f"v_and_b32 {hi(S)}, 0x0fffffff, {lo(Wp)}"),
                Ins(f"v_mad_u64_u32 {R}, {SD}, {U}, {self.d()}, {S}", wr=[SD]),
            ])
        self.vmax = self.base + 14 * self.w
        return seq + interleave(streams)

    def emit(self):
        seq = pad_hazards(self.gen())
        body = "\\n\\t".join(i.text for i in seq)
        clob = [f'"v{i}"' for i in range(self.base, self.vmax)] + [f'"s{SGPR_SD}"', f'"s{SGPR_SD + 1}"']
        outs = ", ".join(f'[r{k}] "=&v"(r{k})' for k in range(self.w))
        ins = ", ".join(f'[{k}] "{c}"({e})' for k, c, e in self.ins)
        args = ", ".join([f"u64& r{k}" for k in range(self.w)] + [f"u64 a{k}, u64 b{k}" for k in range(self.w)] +
                         ["uint32_t d", "uint32_t e"])
        valu = sum(1 for i in seq if i.valu)
        nops = sum(1 for i in seq if i.text.startswith("s_nop"))
        return (f"// {self.w} products mod 2^60 - d (< 2q), {valu} VALU, {nops} s_nop\n"
                f"template <> struct {self.struct}<{self.w}> {{\n"
                f"    static __device__ __forceinline__ void run({args}) {{\n"
                f"        asm{' volatile' if self.volatile else ''}(\"{body}\"\n            : {outs}\n            : {ins}\n"
                f"            : {', '.join(clob)});\n    }}\n}};\n")


HEADER = """// GENERATED by tools/gen_ntt_asm.py -- do not edit.
// Hand-scheduled forward / inverse NTT rounds for primes in (2^60 - 2^32, 2^60), and generic-prime
// rounds for any q < 2^60; see the generator's docstring.  Included inside namespace exacto by ntt.hip.
#pragma once

// Emitted forms (measured, DESIGN.md §4): the approximate Shoup quotient (no low-low partial
// product, T < 3q) and, in forward butterflies, X as the Shoup chain's free addend.  The exact
// quotient and the separate X + T add are still modelled by the generator (tools/asm_sim.py checks
// both) but no longer emitted.

struct AsmK {
    uint32_t n0, n1;      // 2^64 - q (n1 = 0xF0000000 for the primes of this path)
    uint32_t ql, qh;      // q
    u64 q, nq;            // q, 2^64 - q
    // inverse last stage: n^-1 and psi_inv_rev[1] * n^-1 with their Shoup companions
    uint32_t nil, nih, nsl, nsh, lwl, lwh, lsl, lsh;
};

__device__ __forceinline__ AsmK make_asmk(u64 q) {
    AsmK K{};
    const u64 nq = (u64)0 - q;
    K.n0 = (uint32_t)nq; K.n1 = (uint32_t)(nq >> 32);
    K.ql = (uint32_t)q; K.qh = (uint32_t)(q >> 32);
    K.q = q; K.nq = nq;
    return K;
}

__device__ __forceinline__ AsmK make_asmk_inv(const PrimeConst& P) {
    AsmK K = make_asmk(P.q);
    K.nil = (uint32_t)P.n_inv; K.nih = (uint32_t)(P.n_inv >> 32);
    K.nsl = (uint32_t)P.n_inv_s; K.nsh = (uint32_t)(P.n_inv_s >> 32);
    K.lwl = (uint32_t)P.last_w; K.lwh = (uint32_t)(P.last_w >> 32);
    K.lsl = (uint32_t)P.last_ws; K.lsh = (uint32_t)(P.last_ws >> 32);
    return K;
}

// ... with the last stage's constants times R = 2^64 mod q: the inverse of Montgomery products
// (every input carries R^-1, which the last stage cancels)
__device__ __forceinline__ AsmK make_asmk_inv_mont(const PrimeConst& P) {
    AsmK K = make_asmk(P.q);
    K.nil = (uint32_t)P.n_inv_r; K.nih = (uint32_t)(P.n_inv_r >> 32);
    K.nsl = (uint32_t)P.n_inv_rs; K.nsh = (uint32_t)(P.n_inv_rs >> 32);
    K.lwl = (uint32_t)P.last_wr; K.lwh = (uint32_t)(P.last_wr >> 32);
    K.lsl = (uint32_t)P.last_wrs; K.lsh = (uint32_t)(P.last_wrs >> 32);
    return K;
}

template <int LOGN, int R> struct FwdRoundAsm;
template <int LOGN, int R, bool LZ = false> struct InvRoundAsm;   // LZ: last round, outputs < 2q
// any prime below 2^QB (the HPS primes; QB < 60: fewer reductions, the values' headroom is larger)
template <int LOGN, int R, int QB = 60> struct InvRoundGenAsm;
template <int LOGN, int R, int QB = 60> struct FwdRoundGenAsm;
template <int W> struct MulNear60Asm;
template <int W> struct MulNear60PinAsm;   // temps below the pinned homes (kernels with EXACTO_PIN_DECL)
template <int W> struct MulNear60PinVAsm;  // ... as asm volatile (ordered with fences and other statements)

"""


def main():
    parts = [HEADER, pin_homes_decl(), "\n", MulPair(2).emit(), "\n", MulPair(1).emit(), "\n",
             MulPair(2, base=PIN_BASE - 28, struct="MulNear60PinAsm", volatile=False).emit(), "\n",
             MulPair(2, base=PIN_BASE - 28, struct="MulNear60PinVAsm").emit(), "\n"]
    approx, addx = True, True
    for logn in (12, 13):
        for r in range((logn + 3) // 4):
            parts.append(Round(logn, r, approx, addx).emit())
            parts.append("\n")
        for rd in inv_rounds(logn, approx):
            parts.append(InvRound(logn, rd.r, rd.bound_in, approx).emit())
            parts.append("\n")
        rd = inv_rounds(logn, approx)[-1]   # the tensor kernels' last round, outputs in [0, 2q)
        parts.append(InvRound(logn, rd.r, rd.bound_in, approx, lazy_out=True).emit())
        parts.append("\n")
        for rd in inv_rounds(logn, approx, generic=True):
            parts.append(InvRound(logn, rd.r, rd.bound_in, approx, generic=True).emit())
            parts.append("\n")
        for r in range((logn + 3) // 4):
            parts.append(Round(logn, r, approx, True, pinned=True).emit())
            parts.append("\n")
        # the extension transforms' last round, outputs in [0, 2q)
        parts.append(Round(logn, (logn + 3) // 4 - 1, approx, True, pinned=True, lazy_out=True).emit())
        parts.append("\n")
        if logn == 13:   # the last round after the lane-pair exchange (EXACTO_FWD13_LP)
            parts.append(LanePairXchg().emit())
            parts.append("\n")
            for lz in (False, True):
                parts.append(Round(13, 3, approx, True, pinned=True, lazy_out=lz, perm=PERM_LP).emit())
                parts.append("\n")
        for rd in inv_rounds_pinned(logn, approx):
            parts.append(InvRoundPinned(logn, rd.r, rd.bound_in, approx).emit())
            parts.append("\n")
        rd = inv_rounds_pinned(logn, approx)[-1]
        parts.append(InvRoundPinned(logn, rd.r, rd.bound_in, approx, lazy_out=True).emit())
        parts.append("\n")
    for logn in GEN_LOGN:   # the generic-prime forward rounds (and n = 1024's inverse rounds)
        for rd in fwd_rounds(logn, approx, addx, generic=True):
            parts.append(rd.emit())
            parts.append("\n")
        if logn not in (12, 13):
            for rd in inv_rounds(logn, approx, generic=True):
                parts.append(InvRound(logn, rd.r, rd.bound_in, approx, generic=True).emit())
                parts.append("\n")
        for qb in GEN_QBITS.get(logn, ()):   # smaller primes: fewer reductions
            for rd in fwd_rounds(logn, approx, addx, generic=True, qbits=qb):
                parts.append(rd.emit())
                parts.append("\n")
            for rd in inv_rounds(logn, approx, generic=True, qbits=qb):
                parts.append(InvRound(logn, rd.r, rd.bound_in, approx, generic=True, qbits=qb).emit())
                parts.append("\n")
    with open(OUT, "w") as f:
        f.write("".join(parts).rstrip("\n") + "\n")
    print("wrote", OUT)


if __name__ == "__main__":
    main()
