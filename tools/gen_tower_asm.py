#!/usr/bin/env python3
"""tools/gen_tower_asm.py — emits lachain_amd/csrc/asm_tower.hpp: Fp12-level gfx950 assembly routines for the
final exponentiation, operating on an Fp12 accumulator that lives in AGPRs a[0:143] for a whole
exponentiation loop.

Why: the compiler-built cyclotomic squaring calls nine Fp2 leaf routines that each clobber
v0..v91, so the 144-word accumulator and the loop's other Fp12 values are shuffled between VGPRs, AGPRs and
scratch around every call (k_final_exp_check: 6.3 KB of scratch per lane, 25 % of wave cycles waiting).  Here
the squaring is ONE call whose operand stays in AGPRs; every temporary is a VGPR the routine owns (v0..v247),
so nothing spills, and the arithmetic is lazy:

  fp4 squaring (a, b) -> (A, B) = (a^2 + xi b^2, 2ab) over Fp2 with double-width products and ONE Montgomery
  reduction per output coefficient: a^2 = ((a0+a1)(a0-a1+p), 2a0 a1), b^2 likewise, (a+b)^2 with a+b reduced,
  A0 = P1 + P3 - P4 + 5p^2, A1 = P2 + P3 + P4, B0 = P5 - P1 - P3 + 5p^2, B1 = P6 - P2 - P4 + 5p^2 (all < 9.5p^2,
  so REDC returns < 2p): 6 x 144 + 4 x 156 MADs instead of 9 full products (1,800 MADs) per fp4.
  Granger-Scott combination z' = 3t -+ 2z in [0, 8p), reduced by three conditional subtractions (4p, 2p, p).

Hazards: every VALU read of an SGPR (carry-in, lane mask) is at least 2 wait states after the VALU write of that
SGPR, and an AGPR read at least 2 after its write (the pass `hazard_fix` inserts s_nop where interleaving of
independent chains does not already provide the distance).  Routine outputs are fully reduced (< p).

Routines:
  lcb_r_fp4sq    (internal) v[0:23] = a, v[24:47] = b (< p), p in v[188:199] -> A, B at FP4_OUT (< 2p)
  lcb_r_cyc_sqr  a[0:143] = f (unitary, components < p) -> a[0:143] = f^2 (Granger-Scott)
  lcb_r_cyc_sqr_n  Fp12 from a memory slot -> count squarings in AGPRs -> memory slot (the only entry point the
                 kernels call: the compiler never holds the AGPR accumulator, so it cannot copy it around)
"""
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gen_asm import P, PL, N, PINV  # noqa: E402

S_PINV = 88
MAD_CARRY = [90, 92, 94, 86]                 # SGPR pairs of interleaved product / REDC chains
LIN_CARRY = [96, 98, 84, 82, 80, 78, 76, 74]  # SGPR pairs of interleaved add / sub / select chains
S_CALL = 26                                  # s[26:27] call target, s[28:29] nested return address
CLOBBER_SGPRS = sorted({S_PINV, 26, 27, 28, 29, 30, 31} | {c + d for c in MAD_CARRY + LIN_CARRY for d in (0, 1)})
VMAX = 248                                   # routines own v0..v247; v248..v255 stay with the compiler

P_REGS = list(range(188, 200))               # p while lcb_r_cyc_sqr runs (read by lcb_r_fp4sq)
SAFE = list(range(200, 248))                 # caller registers lcb_r_fp4sq never writes
FP4_POOL = list(range(172))                  # lcb_r_fp4sq's value registers (v0..v47 = its inputs)
FP4_ACCS = [172, 176, 180, 184]              # its 64-bit MAD accumulator rings (4 aligned blocks)
A_PARK = 144                                 # a[144:167]: one double-width value parked across a product batch

K5P2 = 5 * P * P
K5P2L = [(K5P2 >> (32 * i)) & 0xFFFFFFFF for i in range(2 * N)]


def limbs(x, n=N):
    return [(x >> (32 * i)) & 0xFFFFFFFF for i in range(n)]


# ------------------------------------------------------------------ register allocation
class Pool:
    def __init__(self, regs, accs=()):
        self.free = set(regs)
        self.used_max = set()
        self.accs, self.acc_busy = list(accs), set()

    def take(self, n):
        got = sorted(self.free)[:n]
        if len(got) < n:
            raise RuntimeError(f"out of VGPRs: need {n}, have {len(self.free)}")
        self.free -= set(got)
        self.used_max |= set(got)
        return got

    def take_acc(self):
        """4 consecutive registers starting at an even register (the 64-bit MAD accumulator ring)"""
        for r in self.accs:
            if r not in self.acc_busy:
                self.acc_busy.add(r)
                self.used_max |= {r, r + 1, r + 2, r + 3}
                return r
        raise RuntimeError("no free accumulator block")

    def give_acc(self, r):
        self.acc_busy.remove(r)

    def give(self, regs):
        for r in regs:
            assert r not in self.free, f"double free v{r}"
        self.free |= set(regs)


# ------------------------------------------------------------------ instruction streams
def merge(streams):
    """round-robin interleave of independent instruction lists"""
    out, idx = [], [0] * len(streams)
    while any(idx[k] < len(streams[k]) for k in range(len(streams))):
        for k in range(len(streams)):
            if idx[k] < len(streams[k]):
                out.append(streams[k][idx[k]])
                idx[k] += 1
    return out


def sp(c):
    return f"s[{c}:{c + 1}]"


def add_chain(r, x, y, c, first_carry_in=False):
    """r = x + y over len(r) words; carry out in s[c]"""
    s = [f"v_addc_co_u32_e64 v{r[0]}, {sp(c)}, v{x[0]}, v{y[0]}, {sp(c)}" if first_carry_in else
         f"v_add_co_u32_e64 v{r[0]}, {sp(c)}, v{x[0]}, v{y[0]}"]
    s += [f"v_addc_co_u32_e64 v{r[j]}, {sp(c)}, v{x[j]}, v{y[j]}, {sp(c)}" for j in range(1, len(r))]
    return s


def sub_chain(r, x, y, c):
    """r = x - y over len(r) words; borrow out in s[c]"""
    s = [f"v_sub_co_u32_e64 v{r[0]}, {sp(c)}, v{x[0]}, v{y[0]}"]
    s += [f"v_subb_co_u32_e64 v{r[j]}, {sp(c)}, v{x[j]}, v{y[j]}, {sp(c)}" for j in range(1, len(r))]
    return s


def condsub(r, kp, tmp, c):
    """r <- r - kp if r >= kp (12 words): tmp = r - kp; borrow ? r : tmp"""
    s = sub_chain(tmp, r, kp, c)
    s += [f"v_cndmask_b32_e64 v{r[j]}, v{tmp[j]}, v{r[j]}, {sp(c)}" for j in range(N)]
    return s


def movs_const(r, vals):
    return [f"v_mov_b32 v{r[j]}, 0x{vals[j]:08x}" for j in range(len(r))]


def ring(acc, k):
    return (acc, acc + 1, acc + 3) if k % 2 == 0 else (acc + 2, acc + 3, acc + 1)


def comba(chains):
    """interleaved plain products T = a*b (24 words): chains = [dict(a, b, acc, out, c)].  out[k] is written at
    the end of column k and may alias a[k-11] (k >= 11)."""
    s = []
    for ch in chains:
        s += [f"v_mov_b32 v{ch['acc']}, 0", f"v_mov_b32 v{ch['acc'] + 1}, 0"]
    for k in range(2 * N - 1):
        terms = [(i, k - i) for i in range(max(0, k - (N - 1)), min(k, N - 1) + 1)]
        for n_t, (i, j) in enumerate(terms):
            for ch in chains:
                L, H, C = ring(ch["acc"], k)
                s.append(f"v_mad_u64_u32 v[{L}:{H}], {sp(ch['c'])}, v{ch['a'][i]}, v{ch['b'][j]}, v[{L}:{H}]")
            for ch in chains:
                L, H, C = ring(ch["acc"], k)
                s.append(f"v_addc_co_u32_e64 v{C}, {sp(ch['c'])}, 0, {0 if n_t == 0 else 'v%d' % C}, {sp(ch['c'])}")
        for ch in chains:
            L, H, C = ring(ch["acc"], k)
            s.append(f"v_mov_b32 v{ch['out'][k]}, v{L}")
            if k == 2 * N - 2:
                s.append(f"v_mov_b32 v{ch['out'][2 * N - 1]}, v{H}")
            else:
                L2, H2, C2 = ring(ch["acc"], k + 1)
                s.append(f"v_mov_b32 v{L2}, v{H}")
    return s


def redc(chains, preg):
    """interleaved Montgomery reductions (U + m p) / 2^384 of 24-word U: chains = [dict(u, m, acc, c)];
    the result (< 2p for U < 9.84 p^2) lands in u[12:24]"""
    s = []
    for ch in chains:
        s += [f"v_mov_b32 v{ch['acc']}, 0", f"v_mov_b32 v{ch['acc'] + 1}, 0"]
    for k in range(2 * N):
        for ch in chains:
            L, H, C = ring(ch["acc"], k)
            s.append(f"v_add_co_u32_e64 v{L}, {sp(ch['c'])}, v{L}, v{ch['u'][k]}")
        for ch in chains:
            L, H, C = ring(ch["acc"], k)
            s.append(f"v_addc_co_u32_e64 v{H}, {sp(ch['c'])}, v{H}, 0, {sp(ch['c'])}")
        for ch in chains:
            L, H, C = ring(ch["acc"], k)
            s.append(f"v_addc_co_u32_e64 v{C}, {sp(ch['c'])}, 0, 0, {sp(ch['c'])}")
        terms = [(i, k - i) for i in range(max(0, k - (N - 1)), min(k - 1, N - 1) + 1)]
        if k < N:
            terms.append(("m", k))
        for t in terms:
            if t[0] == "m":
                for ch in chains:
                    L, H, C = ring(ch["acc"], k)
                    s.append(f"v_mul_lo_u32 v{ch['m'][k]}, v{L}, s{S_PINV}")
                xs, y = [ch["m"][k] for ch in chains], preg[0]
            else:
                i, j = t
                xs, y = [ch["m"][i] for ch in chains], preg[j]
            for ch, x in zip(chains, xs):
                L, H, C = ring(ch["acc"], k)
                s.append(f"v_mad_u64_u32 v[{L}:{H}], {sp(ch['c'])}, v{x}, v{y}, v[{L}:{H}]")
            for ch in chains:
                L, H, C = ring(ch["acc"], k)
                s.append(f"v_addc_co_u32_e64 v{C}, {sp(ch['c'])}, 0, v{C}, {sp(ch['c'])}")
        for ch in chains:
            L, H, C = ring(ch["acc"], k)
            if k >= N:
                s.append(f"v_mov_b32 v{ch['u'][k]}, v{L}")     # u[k] was consumed at the start of column k
            if k < 2 * N - 1:
                L2, H2, C2 = ring(ch["acc"], k + 1)
                s.append(f"v_mov_b32 v{L2}, v{H}")
    return s


# ------------------------------------------------------------------ hazard pass
_SREAD_E64 = ("v_addc_co_u32_e64", "v_subb_co_u32_e64", "v_cndmask_b32_e64")


def _sgpr_pairs(txt):
    return [(int(a), int(b)) for a, b in re.findall(r"s\[(\d+):(\d+)\]", txt)]


def hazard_fix(lines):
    """insert s_nop so that (1) a VALU read of an SGPR pair comes >= 2 wait states after a VALU wrote it and
    (2) an AGPR read comes >= 2 wait states after its write.  Wait states = instructions issued in between
    (+ s_nop n counts n + 1)."""
    out = []
    last_sw = {}     # sgpr pair -> position (in wait-state units) of the last VALU write
    last_aw = {}     # agpr -> position of last write
    pos = 0
    for ln in lines:
        mn = ln.split()[0] if ln.strip() else ""
        need = 0
        if mn.startswith("v_"):
            ops = ln[len(mn):].split(",")
            reads = []
            if mn in _SREAD_E64:
                reads = _sgpr_pairs(ops[-1])
            for pr in reads:
                if pr in last_sw:
                    need = max(need, 2 - (pos - last_sw[pr] - 1))
            if mn == "v_accvgpr_read_b32":
                a = int(re.search(r"a(\d+)", ops[1]).group(1))
                if a in last_aw:
                    need = max(need, 2 - (pos - last_aw[a] - 1))
        if need > 0:
            out.append(f"s_nop {need - 1}")
            pos += need
        out.append(ln)
        if mn.startswith("v_"):
            ops = ln[len(mn):].split(",")
            if mn in ("v_mad_u64_u32", "v_add_co_u32_e64", "v_addc_co_u32_e64", "v_sub_co_u32_e64",
                      "v_subb_co_u32_e64"):
                for pr in _sgpr_pairs(ops[1]):
                    last_sw[pr] = pos
            if mn == "v_accvgpr_write_b32":
                last_aw[int(re.search(r"a(\d+)", ops[0]).group(1))] = pos
        if mn.startswith("s_nop"):
            pos += int(ln.split()[1]) + 1
        else:
            pos += 1
    return out


def call(label):
    return [f"s_getpc_b64 s[{S_CALL}:{S_CALL + 1}]",
            f"s_add_u32 s{S_CALL}, s{S_CALL}, {label}@rel32@lo+4",
            f"s_addc_u32 s{S_CALL + 1}, s{S_CALL + 1}, {label}@rel32@hi+12",
            f"s_swappc_b64 s[28:29], s[{S_CALL}:{S_CALL + 1}]"]


# ------------------------------------------------------------------ lcb_r_fp4sq
def gen_fp4():
    pool = Pool(FP4_POOL, FP4_ACCS)
    a0, a1, b0, b1 = [pool.take(N) for _ in range(4)]
    assert a0 == list(range(0, 12)) and b1 == list(range(36, 48))
    Pr = P_REGS
    body = []
    # prep 1: Sa = a0 + a1, Da = a0 - a1 + p, a0x2 = 2 a0, Sb, Db
    Sa, Da, a0x2, Sb, Db = [pool.take(N) for _ in range(5)]
    body += merge([add_chain(Sa, a0, a1, LIN_CARRY[0]),
                   sub_chain(Da, a0, a1, LIN_CARRY[1]) + add_chain(Da, Da, Pr, LIN_CARRY[1]),
                   add_chain(a0x2, a0, a0, LIN_CARRY[2]),
                   add_chain(Sb, b0, b1, LIN_CARRY[3]),
                   sub_chain(Db, b0, b1, LIN_CARRY[4]) + add_chain(Db, Db, Pr, LIN_CARRY[4])])
    # batch 1: P1 = Sa Da, P2 = a0x2 a1, P3 = Sb Db
    chains, outs = [], []
    for t, (x, y) in enumerate([(Sa, Da), (a0x2, a1), (Sb, Db)]):
        fresh = pool.take(N)
        out = fresh[:11] + x + [fresh[11]]
        chains.append(dict(a=x, b=y, acc=pool.take_acc(), out=out, c=MAD_CARRY[t]))
        outs.append(out)
    body += comba(chains)
    for ch in chains:
        pool.give_acc(ch["acc"])
    pool.give(Da + Db)
    P1, P2, P3 = outs
    # X0 = P1 + P3 (in P1), A1' = P3 + P2 (in P3), B1' = K - P2 (in P2)
    K = pool.take(2 * N)
    body += merge([add_chain(P1, P1, P3, LIN_CARRY[0]), movs_const(K, K5P2L)])
    body += merge([add_chain(P3, P3, P2, LIN_CARRY[1]), sub_chain(P2, K, P2, LIN_CARRY[2])])
    X0, A1p, B1p = P1, P3, P2
    pool.give(K)                                  # reloaded for the final sums (register pressure)
    body += [f"v_accvgpr_write_b32 a{A_PARK + j}, v{r}" for j, r in enumerate(X0)]   # parked across batch 2
    pool.give(X0)
    # prep 2: b0x2 = 2 b0, u0 = a0 + b0 mod p, u1 = a1 + b1 mod p
    b0x2, u0, u1, t0, t1 = [pool.take(N) for _ in range(5)]
    body += merge([add_chain(b0x2, b0, b0, LIN_CARRY[0]),
                   add_chain(u0, a0, b0, LIN_CARRY[1]) + condsub(u0, Pr, t0, LIN_CARRY[1]),
                   add_chain(u1, a1, b1, LIN_CARRY[2]) + condsub(u1, Pr, t1, LIN_CARRY[2])])
    pool.give(a0 + a1 + b0)
    # Su = u0 + u1 (in t0), Du = u0 - u1 + p (in t1), u0x2 = 2 u0
    Su, Du = t0, t1
    u0x2 = pool.take(N)
    body += merge([add_chain(Su, u0, u1, LIN_CARRY[0]),
                   sub_chain(Du, u0, u1, LIN_CARRY[1]) + add_chain(Du, Du, Pr, LIN_CARRY[1]),
                   add_chain(u0x2, u0, u0, LIN_CARRY[2])])
    pool.give(u0)
    # batch 2: P4 = b0x2 b1, P5 = Su Du, P6 = u0x2 u1
    chains, outs = [], []
    for t, (x, y) in enumerate([(b0x2, b1), (Su, Du), (u0x2, u1)]):
        fresh = pool.take(N)
        out = fresh[:11] + x + [fresh[11]]
        chains.append(dict(a=x, b=y, acc=pool.take_acc(), out=out, c=MAD_CARRY[t]))
        outs.append(out)
    body += comba(chains)
    for ch in chains:
        pool.give_acc(ch["acc"])
    pool.give(b1 + Du + u1)
    P4, P5, P6 = outs
    # A1 = A1' + P4;  B1 = B1' - P4 + P6;  B0 = P5 + K - X0;  A0 = X0 - P4 + K
    K = pool.take(2 * N)
    X0 = pool.take(2 * N)
    body += merge([movs_const(K, K5P2L), [f"v_accvgpr_read_b32 v{r}, a{A_PARK + j}" for j, r in enumerate(X0)]])
    # one merge: the B0 stream reads X0[j] in the round before the A0 stream overwrites X0[j] (stream order)
    body += merge([add_chain(A1p, A1p, P4, LIN_CARRY[0]),
                   sub_chain(B1p, B1p, P4, LIN_CARRY[1]) + add_chain(B1p, B1p, P6, LIN_CARRY[1]),
                   sub_chain(P5, P5, X0, LIN_CARRY[2]) + add_chain(P5, P5, K, LIN_CARRY[2]),
                   sub_chain(X0, X0, P4, LIN_CARRY[3]) + add_chain(X0, X0, K, LIN_CARRY[3])])
    pool.give(K + P4 + P6)
    A0u, A1u, B0u, B1u = X0, A1p, P5, B1p
    # four reductions, interleaved
    chains = []
    for t, u in enumerate([A0u, A1u, B0u, B1u]):
        chains.append(dict(u=u, m=pool.take(N), acc=pool.take_acc(), c=MAD_CARRY[t]))
    body += redc(chains, Pr)
    outs = [u[N:] for u in (A0u, A1u, B0u, B1u)]
    txt = ["lcb_r_fp4sq:"] + hazard_fix(body + ["s_setpc_b64 s[28:29]"])
    used = pool.used_max
    assert not used & set(P_REGS + SAFE)
    return txt, outs, used


# ------------------------------------------------------------------ lcb_r_cyc_sqr
# AGPR layout of an Fp12 (struct order c0.c0, c0.c1, c0.c2, c1.c0, c1.c1, c1.c2; Fp2 = a, b):
Z = {0: 0, 4: 24, 3: 48, 2: 72, 1: 96, 5: 120}     # z_k -> first AGPR of its 24 words


def agpr_read(vregs, abase):
    return [f"v_accvgpr_read_b32 v{v}, a{abase + j}" for j, v in enumerate(vregs)]


def agpr_write(abase, vregs):
    return [f"v_accvgpr_write_b32 a{abase + j}, v{v}" for j, v in enumerate(vregs)]


def combine_stream(X, zreg_a, sign, P1r, P2r, P4r, tmp, zt, c, out_a):
    """one Fp component: w = 3X - 2z (sign -1) or 3X + 2z (sign +1), X < 2p, z < p (read from AGPR zreg_a into
    zt); w < 8p reduced by conditional subtractions of 4p, 2p, p; written to AGPRs out_a.  tmp, zt: 12 each;
    X is overwritten."""
    s = agpr_read(zt, zreg_a)
    if sign < 0:   # d = 2(X - z + p) + X
        s += sub_chain(tmp, X, zt, c) + add_chain(tmp, tmp, P1r, c)
    else:          # d = 2(X + z) + X
        s += add_chain(tmp, X, zt, c)
    s += add_chain(tmp, tmp, tmp, c) + add_chain(X, tmp, X, c)
    for kp in (P4r, P2r, P1r):
        s += condsub(X, kp, tmp, c)
    s += agpr_write(out_a, X)
    return s


def gen_cyc_sqr(fp4_outs, fp4_used):
    body = []
    body += movs_const(P_REGS, PL) + [f"s_mov_b32 s{S_PINV}, 0x{PINV:08x}"]
    A0, A1, B0, B1 = fp4_outs
    free_after = [r for r in range(200) if r not in set(sum(fp4_outs, [])) and r not in P_REGS]
    P2r, P4r = free_after[:12], free_after[12:24]
    tmps = free_after[24:]

    def consts():
        return merge([movs_const(P2r, limbs(2 * P)), movs_const(P4r, limbs(4 * P))])

    def combos(jobs):
        """jobs: [(X regs, z index, component 0/1, sign, output z index)] -> merged streams"""
        streams = []
        for t, (X, zk, comp, sign, ok) in enumerate(jobs):
            tmp, zt = tmps[24 * t:24 * t + 12], tmps[24 * t + 12:24 * t + 24]
            streams.append(combine_stream(X, Z[zk] + 12 * comp, sign, P_REGS, P2r, P4r, tmp, zt,
                                          LIN_CARRY[t], Z[ok] + 12 * comp))
        return merge(streams)

    # pair (z0, z1) -> z0' = 3A - 2 z0, z1' = 3B + 2 z1
    body += agpr_read(list(range(0, 24)), Z[0]) + agpr_read(list(range(24, 48)), Z[1])
    body += call("lcb_r_fp4sq")
    body += consts()
    body += combos([(A0, 0, 0, -1, 0), (A1, 0, 1, -1, 0), (B0, 1, 0, +1, 1), (B1, 1, 1, +1, 1)])
    # pair (z2, z3) -> (t0, t1) kept in SAFE
    body += agpr_read(list(range(0, 24)), Z[2]) + agpr_read(list(range(24, 48)), Z[3])
    body += call("lcb_r_fp4sq")
    T0a, T0b, T1a, T1b = SAFE[0:12], SAFE[12:24], SAFE[24:36], SAFE[36:48]
    for dst, src in zip((T0a, T0b, T1a, T1b), (A0, A1, B0, B1)):
        body += [f"v_mov_b32 v{d}, v{s_}" for d, s_ in zip(dst, src)]
    # pair (z4, z5) -> (t2, t3) at the fp4 outputs
    body += agpr_read(list(range(0, 24)), Z[4]) + agpr_read(list(range(24, 48)), Z[5])
    body += call("lcb_r_fp4sq")
    body += consts()
    # xi t3 = (t3a - t3b, t3a + t3b) with t3 reduced to [0, p) first -> both in [0, 2p)
    tq, tr = tmps[0:12], tmps[12:24]
    xa, xb = tmps[24:36], tmps[36:48]
    body += merge([condsub(B0, P_REGS, tq, LIN_CARRY[0]), condsub(B1, P_REGS, tr, LIN_CARRY[1])])
    body += merge([sub_chain(xa, B0, B1, LIN_CARRY[0]) + add_chain(xa, xa, P_REGS, LIN_CARRY[0]),
                   add_chain(xb, B0, B1, LIN_CARRY[1])])
    body += [f"v_mov_b32 v{d}, v{s_}" for d, s_ in zip(B0 + B1, xa + xb)]
    # z4' = 3 t0 - 2 z4, z5' = 3 t1 + 2 z5, z2' = 3 xi t3 + 2 z2, z3' = 3 t2 - 2 z3
    body += combos([(T0a, 4, 0, -1, 4), (T0b, 4, 1, -1, 4), (T1a, 5, 0, +1, 5), (T1b, 5, 1, +1, 5)])
    body += combos([(B0, 2, 0, +1, 2), (B1, 2, 1, +1, 2), (A0, 3, 0, -1, 3), (A1, 3, 1, -1, 3)])
    body += ["s_setpc_b64 s[30:31]"]
    return ["lcb_r_cyc_sqr:"] + hazard_fix(body)


# ------------------------------------------------------------------ lcb_r_cyc_sqr_n
# in:  s[20:21] = input slot, s[22:23] = output slot (byte addresses of quad-major SoA Fp12 slots), s19 = n * 16
#      (bytes between word quads, < 2^32), v248 = this lane's byte offset i * 16, s18 = number of squarings (>= 1);
#      s[16:17] walks the quads (64-bit scalar base + 32-bit lane offset: any n < 2^28)
# out: output slot = input^(2^s18); s18 = 0.  Return address saved in s[24:25] across the nested calls.
def gen_cyc_sqr_n():
    b = ["s_mov_b64 s[24:25], s[30:31]", "s_mov_b64 s[16:17], s[20:21]"]
    for g in range(36):     # quad g of this lane at s[16:17] + g * n16 + v248 (64-bit scalar base, 32-bit lane offset)
        b.append(f"global_load_dwordx4 a[{4 * g}:{4 * g + 3}], v248, s[16:17]")
        if g < 35:
            b += ["s_add_u32 s16, s16, s19", "s_addc_u32 s17, s17, 0"]
    b.append("s_waitcnt vmcnt(0)")
    b.append("lcb_cyc_sqr_n_loop:")
    b += ["s_getpc_b64 s[26:27]",
          "s_add_u32 s26, s26, lcb_r_cyc_sqr@rel32@lo+4",
          "s_addc_u32 s27, s27, lcb_r_cyc_sqr@rel32@hi+12",
          "s_swappc_b64 s[30:31], s[26:27]",
          "s_sub_u32 s18, s18, 1",
          "s_cmp_lg_u32 s18, 0",
          "s_cbranch_scc1 lcb_cyc_sqr_n_loop",
          "s_nop 4",                       # AGPR writes by the squaring -> stores of them
          "s_mov_b64 s[16:17], s[22:23]"]
    for g in range(36):
        b.append(f"global_store_dwordx4 v248, a[{4 * g}:{4 * g + 3}], s[16:17]")
        if g < 35:
            b += ["s_add_u32 s16, s16, s19", "s_addc_u32 s17, s17, 0"]
    b.append("s_setpc_b64 s[24:25]")
    return ["lcb_r_cyc_sqr_n:"] + b


# ------------------------------------------------------------------ Fp12 product over the AGPR accumulator (round 5)
# lcb_r_fp12m: a[0:143] <- a[0:143] * M, M an Fp12 in a memory slot.  Karatsuba over Fp6 (t0 = a0 m0, t1 = a1 m1,
# t2 = (a0 + a1)(m0 + m1); r0 = t0 + v t1, r1 = t2 - t0 - t1), each Fp6 product lazily reduced: its six Fp2 products
# (Karatsuba, three 12 x 12 products each) stay double-width (mod 2^768) and every output coefficient is ONE Montgomery
# reduction of its double-width sum plus a multiple of p^2 that makes it nonnegative — 18 products + 6 REDCs per Fp6
# product (3,528 MADs) where the Fp2-level lazy product needs 12 REDCs (4,464).  Double-width Fp2 products go through
# LDS (three per Fp6 product, 144 words per lane); the t0 / t1 halves through a caller-supplied memory slot.
# Entry points: lcb_r_fp12_mul_n (slot x slot -> slot, optional conjugate of the first operand) and lcb_r_pow_z
# (conj(base^|z|): the squaring runs of lcb_r_cyc_sqr and the five products by the base with the accumulator in
# AGPRs throughout).
S_N16, S_M, S_T = 19, 20, 22            # n * 16; s[20:21] M slot; s[22:23] tmp slot
S_A, S_CONJ, S_DST = 56, 65, 60         # s[56:57] first-operand slot; conj flag; s[60:61] destination slot
S_Q0, S_SUM = 62, 64                    # y operand of lcb_r_fp6m: first quad in M; 1 = M[q0..] + M[q0 + 18..]
S_ADDR, S_QT = 66, 68                   # s[66:67] address, s68 quad temp
S_RET6 = 72                             # s[72:73] lcb_r_fp6m return address
V_OFF, V_LDS = 248, 249                 # lane byte offset in slots; lane byte address in LDS (quad g at + g * 1024)
FP12_SGPRS = [16, 17, 18, 24, 25] + list(range(56, 74))

F2_XA, F2_XB, F2_YA, F2_YB = [list(range(12 * i, 12 * i + 12)) for i in range(4)]
F2_SX, F2_SY = list(range(48, 60)), list(range(60, 72))
F2_P0, F2_P1, F2_P2 = list(range(72, 96)), list(range(96, 120)), list(range(120, 144))
F2_ACCS = [144, 148, 152]
F2_RE, F2_IM = F2_P0, F2_P2
PR = list(range(160, 172))
T1, T2, T3 = list(range(172, 196)), list(range(196, 220)), list(range(220, 244))
FP12_VMAX = 244


def pp_limbs(k):
    return limbs(k * P * P, 2 * N)


def gen_fp2dw():
    """lcb_r_fp2dw: (XA + XB i)(YA + YB i), inputs < p, -> RE = XA YA - XB YB, IM = (XA + XB)(YA + YB) - XA YA - XB YB,
    double-width mod 2^768 (RE may be 'negative').  Leaf: v0..v155, returns through s[28:29]."""
    b = merge([add_chain(F2_SX, F2_XA, F2_XB, LIN_CARRY[0]), add_chain(F2_SY, F2_YA, F2_YB, LIN_CARRY[1])])
    b += comba([dict(a=F2_XA, b=F2_YA, acc=F2_ACCS[0], out=F2_P0, c=MAD_CARRY[0]),
                dict(a=F2_XB, b=F2_YB, acc=F2_ACCS[1], out=F2_P1, c=MAD_CARRY[1]),
                dict(a=F2_SX, b=F2_SY, acc=F2_ACCS[2], out=F2_P2, c=MAD_CARRY[2])])
    # the IM stream reads P0[j] in the round before the RE stream overwrites it
    b += merge([sub_chain(F2_P2, F2_P2, F2_P0, LIN_CARRY[0]), sub_chain(F2_P0, F2_P0, F2_P1, LIN_CARRY[1])])
    b += sub_chain(F2_P2, F2_P2, F2_P1, LIN_CARRY[0])
    return ["lcb_r_fp2dw:"] + hazard_fix(b + ["s_setpc_b64 s[28:29]"])


def gen_redc2():
    """lcb_r_redc2: Montgomery reductions of the double-width U1 = v[72:95], U2 = v[120:143] (each < 19.68 p^2, so
    < 3p) and two conditional subtractions -> v[84:95], v[132:143] (< p).  Leaf: m in v0..v23, temps v24..v47,
    accumulators v144..v151; returns through s[28:29].  One copy shared by every reduction of the Fp6 / line products
    keeps their code within the instruction cache."""
    b = redc([dict(u=F2_RE, m=list(range(0, 12)), acc=F2_ACCS[0], c=MAD_CARRY[0]),
              dict(u=F2_IM, m=list(range(12, 24)), acc=F2_ACCS[1], c=MAD_CARRY[1])], PR)
    for _ in range(2):
        b += merge([condsub(F2_RE[N:], PR, list(range(24, 36)), LIN_CARRY[0]),
                    condsub(F2_IM[N:], PR, list(range(36, 48)), LIN_CARRY[1])])
    return ["lcb_r_redc2:"] + hazard_fix(b + ["s_setpc_b64 s[28:29]"])


def call_redc2():
    return [f"s_getpc_b64 s[{S_CALL}:{S_CALL + 1}]", f"s_add_u32 s{S_CALL}, s{S_CALL}, lcb_r_redc2@rel32@lo+4",
            f"s_addc_u32 s{S_CALL + 1}, s{S_CALL + 1}, lcb_r_redc2@rel32@hi+12",
            f"s_swappc_b64 s[28:29], s[{S_CALL}:{S_CALL + 1}]"]


def quad_addr(base, q):
    """s[66:67] = slot base s[base:base+1] + q * n16; q = (sgpr or None, constant)"""
    sg, k = q
    out = [f"s_mov_b32 s{S_QT}, {k}" if sg is None else f"s_add_u32 s{S_QT}, s{sg}, {k}"]
    return out + [f"s_mul_i32 s{S_QT}, s{S_QT}, s{S_N16}", f"s_add_u32 s{S_ADDR}, s{base}, s{S_QT}",
                  f"s_addc_u32 s{S_ADDR + 1}, s{base + 1}, 0"]


def next_quad():
    return [f"s_add_u32 s{S_ADDR}, s{S_ADDR}, s{S_N16}", f"s_addc_u32 s{S_ADDR + 1}, s{S_ADDR + 1}, 0"]


def gload(dst, base, q, kind="v"):
    """len(dst) // 4 consecutive quads from quad q of a slot into contiguous registers dst (v or a)"""
    out = quad_addr(base, q)
    for g in range(len(dst) // 4):
        out.append(f"global_load_dwordx4 {kind}[{dst[4 * g]}:{dst[4 * g] + 3}], v{V_OFF}, s[{S_ADDR}:{S_ADDR + 1}]")
        if g < len(dst) // 4 - 1:
            out += next_quad()
    return out


def gstore(base, q, src, kind="v"):
    out = quad_addr(base, q)
    for g in range(len(src) // 4):
        out.append(f"global_store_dwordx4 v{V_OFF}, {kind}[{src[4 * g]}:{src[4 * g] + 3}], s[{S_ADDR}:{S_ADDR + 1}]")
        if g < len(src) // 4 - 1:
            out += next_quad()
    return out


def lds_write(q, src):
    return [f"ds_write_b128 v{V_LDS}, v[{src[4 * g]}:{src[4 * g] + 3}] offset:{(q + g) * 1024}"
            for g in range(len(src) // 4)]


def lds_read(dst, q):
    return [f"ds_read_b128 v[{dst[4 * g]}:{dst[4 * g] + 3}], v{V_LDS} offset:{(q + g) * 1024}"
            for g in range(len(dst) // 4)]


def modadd(r, x, y, tmp, c):
    return add_chain(r, x, y, c) + condsub(r, PR, tmp, c)


def modsub(r, x, y, tmp, c1, c2):
    """r = x - y mod p (x, y < p): borrow ? r + p : r"""
    s = sub_chain(r, x, y, c1) + add_chain(tmp, r, PR, c2)
    return s + [f"v_cndmask_b32_e64 v{r[j]}, v{r[j]}, v{tmp[j]}, {sp(c1)}" for j in range(N)]


_lbl = [0]


def label(stem):
    _lbl[0] += 1
    return f"lcb_{stem}_{_lbl[0]}"


def fp6_x(k, part, dst):                       # x_k.part of lcb_r_fp6m's x = a[0:71]
    return agpr_read(dst, 24 * k + 12 * part)


def fp6_operands(ks):
    """fp2dw inputs: x = x_k (one index) or x_k1 + x_k2 (two), the same for y (each y_k itself M[q0 + ..] or, when
    s64 = 1, M[q0 + ..] + M[q0 + 18 + ..]), all reduced mod p.  Every load is issued first and the x work (AGPR
    reads and sums) runs while they are in flight."""
    P0 = F2_P0
    q = lambda k, part, hi: (S_Q0, 18 * hi + 6 * k + 3 * part)                      # noqa: E731
    first = [(ks[0], YA_, YB_) for YA_, YB_ in [(F2_YA, F2_YB)]]
    if len(ks) == 2:
        first.append((ks[1], T2[:12], T2[12:]))
    second = [(ks[0], T1[:12], T1[12:])] + ([(ks[1], T3[:12], T3[12:])] if len(ks) == 2 else [])
    s = []
    for k, A, B in first:
        s += gload(A, S_M, q(k, 0, 0)) + gload(B, S_M, q(k, 1, 0))
    skip1, skip2 = label("fp6ld"), label("fp6sum")
    s += [f"s_cmp_eq_u32 s{S_SUM}, 0", f"s_cbranch_scc1 {skip1}"]
    for k, A, B in second:
        s += gload(A, S_M, q(k, 0, 1)) + gload(B, S_M, q(k, 1, 1))
    s += [f"{skip1}:", "s_nop 4"]
    # x (AGPRs) while the loads are in flight
    s += fp6_x(ks[0], 0, F2_XA) + fp6_x(ks[0], 1, F2_XB)
    if len(ks) == 2:
        s += fp6_x(ks[1], 0, F2_SX) + fp6_x(ks[1], 1, P0[:12]) + ["s_nop 1"]
        s += merge([modadd(F2_XA, F2_XA, F2_SX, F2_SY, LIN_CARRY[0]),
                    modadd(F2_XB, F2_XB, P0[:12], P0[12:], LIN_CARRY[1])])
    s += ["s_waitcnt vmcnt(0)", f"s_cmp_eq_u32 s{S_SUM}, 0", f"s_cbranch_scc1 {skip2}"]
    tmps = [P0[:12], P0[12:], F2_P1[:12], F2_P1[12:]]
    streams = []
    for t, ((k, A, B), (_, A2, B2)) in enumerate(zip(first, second)):
        streams.append(modadd(A, A, A2, tmps[2 * t], LIN_CARRY[2 * t]))
        streams.append(modadd(B, B, B2, tmps[2 * t + 1], LIN_CARRY[2 * t + 1]))
    s += merge(streams) + [f"{skip2}:", "s_nop 4"]
    if len(ks) == 2:
        s += merge([modadd(F2_YA, F2_YA, T2[:12], P0[:12], LIN_CARRY[0]),
                    modadd(F2_YB, F2_YB, T2[12:], P0[12:], LIN_CARRY[1])])
    return s + call_fp2dw()


def call_fp2dw():
    return [f"s_getpc_b64 s[{S_CALL}:{S_CALL + 1}]", f"s_add_u32 s{S_CALL}, s{S_CALL}, lcb_r_fp2dw@rel32@lo+4",
            f"s_addc_u32 s{S_CALL + 1}, s{S_CALL + 1}, lcb_r_fp2dw@rel32@hi+12",
            f"s_swappc_b64 s[28:29], s[{S_CALL}:{S_CALL + 1}]"]


def call_ret(label_, ret):
    return [f"s_getpc_b64 s[{S_CALL}:{S_CALL + 1}]", f"s_add_u32 s{S_CALL}, s{S_CALL}, {label_}@rel32@lo+4",
            f"s_addc_u32 s{S_CALL + 1}, s{S_CALL + 1}, {label_}@rel32@hi+12",
            f"s_swappc_b64 s[{ret}:{ret + 1}], s[{S_CALL}:{S_CALL + 1}]"]


# LDS quads of the three double-width diagonal products v_k = x_k y_k: re at 12k, im at 12k + 6
def lds_v(k, part):
    return 12 * k + 6 * part


def fp6_finish(RE, IM, offs, nsub, out_a):
    """RE, IM (+ offs[0], offs[1] multiples of p^2) -> lcb_r_redc2 (reductions + two conditional subtractions) ->
    a[out_a .. out_a + 23]"""
    s = []
    if RE != F2_RE:
        s += mov_regs(F2_RE, RE)
    s += merge([movs_const(T2, pp_limbs(offs[0])), movs_const(T3, pp_limbs(offs[1]))])
    s += merge([add_chain(F2_RE, F2_RE, T2, LIN_CARRY[0]), add_chain(F2_IM, F2_IM, T3, LIN_CARRY[1])])
    return s + call_redc2() + agpr_write(out_a, F2_RE[N:]) + agpr_write(out_a + 12, F2_IM[N:])


def gen_fp6m():
    """lcb_r_fp6m: a[144:215] <- x * y (Fp6, reduced < p); x = a[0:71], y from the M slot at quad s62 (+ quad s62 + 18
    when s64 = 1).  Returns through s[72:73]; clobbers v0..v243, LDS quads 0..35 of the lane."""
    b = []
    for k in range(3):                                               # v_k = x_k y_k -> LDS
        b += fp6_operands([k])
        b += lds_write(lds_v(k, 0), F2_RE) + lds_write(lds_v(k, 1), F2_IM) + ["s_waitcnt lgkmcnt(0)"]
    # c0 = v0 + xi (X12 - v1 - v2).  The sums x1 + x2, y1 + y2 are reduced, so X12 - v1 - v2 is congruent to, not
    # equal to, x1 y2 + x2 y1: as integers re in (-3p^2, 3p^2), im in (-4p^2, 2p^2), and c0 re in (-6p^2, 8p^2),
    # im in (-7p^2, 7p^2): + (6, 7) p^2 -> [0, 14p^2), REDC < 2.43p, two conditional subtractions
    b += fp6_operands([1, 2])
    RE, IM = F2_RE, F2_IM
    for k in (1, 2):
        b += lds_read(T1, lds_v(k, 0)) + lds_read(T2, lds_v(k, 1)) + ["s_waitcnt lgkmcnt(0)"]
        b += merge([sub_chain(RE, RE, T1, LIN_CARRY[0]), sub_chain(IM, IM, T2, LIN_CARRY[1])])
    # xi D = (RE - IM, RE + IM): the T1 stream reads IM[j] in the round before the IM stream overwrites it
    b += merge([sub_chain(T1, RE, IM, LIN_CARRY[0]), add_chain(IM, RE, IM, LIN_CARRY[1])])
    b += lds_read(T2, lds_v(0, 0)) + lds_read(T3, lds_v(0, 1)) + ["s_waitcnt lgkmcnt(0)"]
    b += merge([add_chain(T1, T1, T2, LIN_CARRY[0]), add_chain(IM, IM, T3, LIN_CARRY[1])])
    b += fp6_finish(T1, IM, (6, 7), 2, 144)
    # c1 = X01 - v0 - v1 + xi v2: re in (-6p^2, 4p^2), im in (-5p^2, 5p^2) -> [0, 10p^2), REDC < 2.02p
    b += fp6_operands([0, 1])
    for k in (0, 1):
        b += lds_read(T1, lds_v(k, 0)) + lds_read(T2, lds_v(k, 1)) + ["s_waitcnt lgkmcnt(0)"]
        b += merge([sub_chain(RE, RE, T1, LIN_CARRY[0]), sub_chain(IM, IM, T2, LIN_CARRY[1])])
    b += lds_read(T1, lds_v(2, 0)) + lds_read(T2, lds_v(2, 1)) + ["s_waitcnt lgkmcnt(0)"]
    b += merge([sub_chain(T3, T1, T2, LIN_CARRY[0]), add_chain(T1, T1, T2, LIN_CARRY[1])])
    b += merge([add_chain(RE, RE, T3, LIN_CARRY[0]), add_chain(IM, IM, T1, LIN_CARRY[1])])
    b += fp6_finish(RE, IM, (6, 5), 2, 168)
    # c2 = X02 - v0 - v2 + v1: re, im in (-4p^2, 4p^2) -> [0, 8p^2), REDC < 1.82p
    b += fp6_operands([0, 2])
    for k, op in ((0, sub_chain), (2, sub_chain), (1, add_chain)):
        b += lds_read(T1, lds_v(k, 0)) + lds_read(T2, lds_v(k, 1)) + ["s_waitcnt lgkmcnt(0)"]
        b += merge([op(RE, RE, T1, LIN_CARRY[0]), op(IM, IM, T2, LIN_CARRY[1])])
    b += fp6_finish(RE, IM, (4, 4), 1, 192)
    return ["lcb_r_fp6m:"] + hazard_fix(b + [f"s_setpc_b64 s[{S_RET6}:{S_RET6 + 1}]"])


def gen_fp12m():
    """lcb_r_fp12m: a[0:143] <- a[0:143] * M (components < p in and out); M slot s[20:21], tmp slot s[22:23] (its
    36 quads are overwritten).  Returns through s[30:31]; clobbers v0..v243, a144..a215."""
    X, Y, Z, W = T1[:12], T1[12:], T2[:12], T2[12:]
    b = movs_const(PR, PL) + [f"s_mov_b32 s{S_PINV}, 0x{PINV:08x}"]
    b += [f"s_mov_b32 s{S_Q0}, 0", f"s_mov_b32 s{S_SUM}, 0"] + call_ret("lcb_r_fp6m", S_RET6)   # t0 = a0 m0
    b += ["s_nop 4"] + gstore(S_T, (None, 0), list(range(144, 216)), "a")
    for i in range(6):                                   # a[0:71] <- a1, a[72:143] <- s = a0 + a1
        b += agpr_read(X, 12 * i) + agpr_read(Y, 72 + 12 * i) + ["s_nop 1"]
        b += agpr_write(12 * i, Y) + modadd(X, X, Y, Z, LIN_CARRY[0]) + agpr_write(72 + 12 * i, X)
    b += [f"s_mov_b32 s{S_Q0}, 18"] + call_ret("lcb_r_fp6m", S_RET6)                            # t1 = a1 m1
    b += ["s_nop 4"] + gstore(S_T, (None, 18), list(range(144, 216)), "a")
    for i in range(6):                                   # a[0:71] <- s
        b += agpr_read(X, 72 + 12 * i) + ["s_nop 1"] + agpr_write(12 * i, X)
    b += [f"s_mov_b32 s{S_Q0}, 0", f"s_mov_b32 s{S_SUM}, 1"] + call_ret("lcb_r_fp6m", S_RET6)   # t2 = s (m0 + m1)
    b += ["s_nop 4", "s_waitcnt vmcnt(0)"]
    # r1 = t2 - t0 - t1 -> a[72:143]
    for k in range(3):
        for part in range(2):
            i = 2 * k + part
            b += agpr_read(X, 144 + 12 * i) + gload(Y, S_T, (None, 3 * i)) + gload(Z, S_T, (None, 18 + 3 * i))
            b += ["s_waitcnt vmcnt(0)"] + modsub(X, X, Y, W, LIN_CARRY[0], LIN_CARRY[1])
            b += modsub(X, X, Z, W, LIN_CARRY[2], LIN_CARRY[3]) + agpr_write(72 + 12 * i, X)
    # r0 = t0 + v t1 -> a[0:71]: (v t1)_0 = xi t1_2 = (t1_2a - t1_2b, t1_2a + t1_2b), (v t1)_1 = t1_0, (v t1)_2 = t1_1
    U = T3[:12]
    b += gload(Y, S_T, (None, 18 + 12)) + gload(Z, S_T, (None, 18 + 15)) + ["s_waitcnt vmcnt(0)"]
    b += modsub(U, Y, Z, W, LIN_CARRY[0], LIN_CARRY[1]) + modadd(Y, Y, Z, W, LIN_CARRY[2])      # U = re, Y = im
    for part, V in ((0, U), (1, Y)):
        b += gload(X, S_T, (None, 3 * part)) + ["s_waitcnt vmcnt(0)"] + modadd(X, X, V, W, LIN_CARRY[0])
        b += agpr_write(12 * part, X)
    for k in (1, 2):
        for part in range(2):
            i = 2 * k + part
            b += gload(X, S_T, (None, 3 * i)) + gload(Y, S_T, (None, 18 + 3 * (i - 2))) + ["s_waitcnt vmcnt(0)"]
            b += modadd(X, X, Y, W, LIN_CARRY[0]) + agpr_write(12 * i, X)
    return ["lcb_r_fp12m:"] + hazard_fix(b + ["s_setpc_b64 s[30:31]"])


def conj_c1():
    """a[72:143] <- p - a[72:143] reduced (0 stays 0)"""
    X, Y = T1[:12], T1[12:]
    s = movs_const(PR, PL)
    for i in range(6, 12):
        s += agpr_read(X, 12 * i) + ["s_nop 1"] + sub_chain(Y, PR, X, LIN_CARRY[0])
        s += condsub(Y, PR, X, LIN_CARRY[1]) + agpr_write(12 * i, Y)
    return s


def walk_load(base):
    """a[0:143] <- the 36 quads of the slot at s[base:base+1] (s[16:17] walks)"""
    s = [f"s_mov_b64 s[16:17], s[{base}:{base + 1}]"]
    for g in range(36):
        s.append(f"global_load_dwordx4 a[{4 * g}:{4 * g + 3}], v{V_OFF}, s[16:17]")
        if g < 35:
            s += ["s_add_u32 s16, s16, s19", "s_addc_u32 s17, s17, 0"]
    return s + ["s_waitcnt vmcnt(0)"]


def walk_store(base):
    s = ["s_nop 4", f"s_mov_b64 s[16:17], s[{base}:{base + 1}]"]
    for g in range(36):
        s.append(f"global_store_dwordx4 v{V_OFF}, a[{4 * g}:{4 * g + 3}], s[16:17]")
        if g < 35:
            s += ["s_add_u32 s16, s16, s19", "s_addc_u32 s17, s17, 0"]
    return s


def gen_fp12_mul_n():
    """lcb_r_fp12_mul_n: slot s[60:61] <- (s65 ? conj(A) : A) * M; A slot s[56:57], M slot s[20:21], tmp slot
    s[22:23] (may be the destination or A; not M)"""
    skip = label("mulnc")
    b = ["s_mov_b64 s[24:25], s[30:31]"] + walk_load(S_A)
    b += [f"s_cmp_eq_u32 s{S_CONJ}, 0", f"s_cbranch_scc1 {skip}"] + conj_c1() + [f"{skip}:", "s_nop 4"]
    b += call_ret("lcb_r_fp12m", 30) + walk_store(S_DST) + ["s_setpc_b64 s[24:25]"]
    return ["lcb_r_fp12_mul_n:"] + hazard_fix(b)


def gen_pow_z():
    """lcb_r_pow_z: slot s[60:61] <- conj(B^|z|), B the unitary Fp12 in slot s[20:21] (the same slot may be the
    destination); tmp slot s[22:23].  The runs of squarings between the set bits of |z| (1, 2, 3, 9, 32, 16) are
    lcb_r_cyc_sqr calls, the five products by B lcb_r_fp12m; the accumulator never leaves a[0:143]."""
    b = ["s_mov_b64 s[24:25], s[30:31]"] + walk_load(S_M)
    runs = [1, 2, 3, 9, 32, 16]
    for t, cnt in enumerate(runs):
        loop = label("pzrun")
        b += [f"s_mov_b32 s18, {cnt}", f"{loop}:"] + call_ret("lcb_r_cyc_sqr", 30)
        b += ["s_sub_u32 s18, s18, 1", "s_cmp_lg_u32 s18, 0", f"s_cbranch_scc1 {loop}", "s_nop 4"]
        if t < len(runs) - 1:
            b += call_ret("lcb_r_fp12m", 30) + ["s_nop 4"]
    b += conj_c1() + walk_store(S_DST) + ["s_setpc_b64 s[24:25]"]
    return ["lcb_r_pow_z:"] + hazard_fix(b)


# ------------------------------------------------------------------ the two-pair Miller loop (round 5)
# lcb_r_miller2: f = conj(prod_k l1_k(P1) l2_k(P2)) over two normalised line sets (pairing.hpp miller2_norm_lds), the
# accumulator in a[0:143] from the first line to the last.  A line 1 + b v + c v w (b = B' xP, c = C' yP) is applied
# by lcb_r_line with lazily reduced products: per coefficient position the three double-width Fp2 products (t0 = b X,
# t1 = c Y, S = (b + c)(X + Y)) are combined before reduction — f1_k' = REDC(S - t0 - t1 + f1_k R) and
# f0_k' = REDC(t0_k + f0_k R + t1_{k-1}) — 12 Montgomery reductions per line instead of 18.  A point at infinity is
# stored as (0, 0): b = c = 0 and the line is 1.  The squarings are lcb_r_fp12sq (complex method: two lazily
# reduced Fp6 products through lcb_r_fp6m).
S_P, S_S2, S_PQ, S_SET = 56, 58, 62, 63          # P slot (P1 quads 0..5, P2 6..11); second tmp slot; P quad base; set
V_LS = [244, 246]                                 # working line pointers of the two sets (copies of v[250:253])
L_T, L_PEND, L_T12 = 0, 12, 24                    # LDS quads: parked t, pending f0 sum, t1 of position 2
A_TF1, A_TF0, A_T0 = 144, 168, 192                # AGPRs: new f1_2, new f0_2 (written at the end), parked t0
LINE_B, LINE_C, LINE_BC = T1, T2, T3              # b, c, b + c (< p) across the line's fp2dw calls
K4PP = pp_limbs(4)


def add_hi(U, f):
    """U (24 words, mod 2^768) += f * 2^384"""
    return add_chain(U[N:], U[N:], f, LIN_CARRY[2])


def dw_park_a(abase, RE, IM):
    return agpr_write(abase, RE) + agpr_write(abase + 24, IM)


def dw_from_a(RE, IM, abase):
    return agpr_read(RE, abase) + agpr_read(IM, abase + 24)


def redc_pair(RE, IM, nsub, out):
    """(RE, IM) = (F2_RE, F2_IM) + 4p^2 each -> lcb_r_redc2 -> out(ra, rb)"""
    assert RE == F2_RE and IM == F2_IM
    s = movs_const(list(range(0, 24)), K4PP)
    s += merge([add_chain(RE, RE, list(range(0, 24)), LIN_CARRY[0]), add_chain(IM, IM, list(range(0, 24)), LIN_CARRY[1])])
    return s + call_redc2() + out(RE[N:], IM[N:])


def mov_regs(dst, src):
    return [f"v_mov_b32 v{d}, v{x}" for d, x in zip(dst, src)]


def xi_into(dst_a, dst_b, src_a, src_b, tmp):
    """(dst_a, dst_b) = xi (src_a + src_b u) = (src_a - src_b, src_a + src_b) mod p; sources < p"""
    return merge([modsub(dst_a, src_a, src_b, tmp[:12], LIN_CARRY[0], LIN_CARRY[1]),
                  modadd(dst_b, src_a, src_b, tmp[12:], LIN_CARRY[2])])


def line_operand_y(k, which):
    """fp2dw's y operand (YA, YB) for position k: X = f0_{k-1} / Y = f1_{k-1}, or xi f0_2 / xi f1_2 at k = 0"""
    base = (0 if which == "X" else 72)
    if k > 0:
        return agpr_read(F2_YA, base + 24 * (k - 1)) + agpr_read(F2_YB, base + 24 * (k - 1) + 12)
    return (agpr_read(F2_SX, base + 48) + agpr_read(F2_SY, base + 60) + ["s_nop 1"] +
            xi_into(F2_YA, F2_YB, F2_SX, F2_SY, F2_P0))


def line_operand_xy_sum(k):
    """YA, YB = X + Y (mod p) for position k"""
    s = line_operand_y(k, "X") + mov_regs(list(range(96, 120)), F2_YA + F2_YB)
    s += line_operand_y(k, "Y")
    s += merge([modadd(F2_YA, F2_YA, list(range(96, 108)), F2_P0[:12], LIN_CARRY[0]),
                modadd(F2_YB, F2_YB, list(range(108, 120)), F2_P0[12:], LIN_CARRY[1])])
    return s


def gen_line():
    """lcb_r_line: a[0:143] <- f * (1 + b v + c v w) for the line at the set pointer v[244:245] (s63 = 0) or
    v[246:247] (s63 = 1), b = B' xP, c = C' yP with P at quads s62 .. s62 + 5 of the P slot s[56:57].  PR = p and
    s88 set by the caller.  Returns through s[30:31]."""
    b = []
    other = label("lineset")
    done = label("lineld")
    for half, dst in ((0, LINE_B), (1, LINE_C)):   # b = B' xP, then c = C' yP: products, lcb_r_redc2
        b += [f"s_cmp_eq_u32 s{S_SET}, 0", f"s_cbranch_scc0 {other}_{half}"]
        for t, vp in enumerate(V_LS):
            if t == 1:
                b += [f"{other}_{half}:", "s_nop 4"]
            for g in range(6):
                b.append(f"global_load_dwordx4 v[{48 + 4 * g}:{48 + 4 * g + 3}], v[{vp}:{vp + 1}], "
                         f"off offset:{96 * half + 16 * g}")
            if t == 0:
                b += [f"s_branch {done}_{half}"]
        b += [f"{done}_{half}:", "s_nop 4"]
        b += gload(list(range(24, 36)), S_P, (S_PQ, 3 * half)) + ["s_waitcnt vmcnt(0)"]
        b += comba([dict(a=list(range(48, 60)), b=list(range(24, 36)), acc=F2_ACCS[0], out=F2_RE, c=MAD_CARRY[0]),
                    dict(a=list(range(60, 72)), b=list(range(24, 36)), acc=F2_ACCS[1], out=F2_IM, c=MAD_CARRY[1])])
        b += call_redc2() + mov_regs(dst, F2_RE[N:] + F2_IM[N:])
    b += merge([modadd(LINE_BC[:12], LINE_B[:12], LINE_C[:12], list(range(0, 12)), LIN_CARRY[0]),
                modadd(LINE_BC[12:], LINE_B[12:], LINE_C[12:], list(range(12, 24)), LIN_CARRY[1])])
    RE, IM = F2_RE, F2_IM
    T = list(range(0, 24)), list(range(24, 48))          # temps after a call (fp2dw inputs are dead)

    def call_xy(xregs, yprep):
        return yprep + mov_regs(F2_XA + F2_XB, xregs) + call_fp2dw()

    def sub_lds(q, c0, c1):                               # RE -= LDS[q..q+5], IM -= LDS[q+6..q+11]
        return (lds_read(T[0], q) + lds_read(T[1], q + 6) + ["s_waitcnt lgkmcnt(0)"] +
                merge([sub_chain(RE, RE, T[0], c0), sub_chain(IM, IM, T[1], c1)]))

    def add_lds(q, c0, c1):
        return (lds_read(T[0], q) + lds_read(T[1], q + 6) + ["s_waitcnt lgkmcnt(0)"] +
                merge([add_chain(RE, RE, T[0], c0), add_chain(IM, IM, T[1], c1)]))

    def add_f_hi(abase):                                  # (RE, IM) += (f.a, f.b) * 2^384, f from a[abase..]
        return (agpr_read(T[0][:12], abase) + agpr_read(T[1][:12], abase + 12) + ["s_nop 1"] +
                merge([add_chain(RE[N:], RE[N:], T[0][:12], LIN_CARRY[2]),
                       add_chain(IM[N:], IM[N:], T[1][:12], LIN_CARRY[3])]))

    to_a = lambda abase: (lambda ra, rb: agpr_write(abase, ra) + agpr_write(abase + 12, rb))   # noqa: E731
    # ---- position 2: X = f0_1, Y = f1_1
    b += call_xy(LINE_C, line_operand_y(2, "Y"))                                   # t1_2
    b += lds_write(L_T12, RE) + lds_write(L_T12 + 6, IM)
    b += call_xy(LINE_B, line_operand_y(2, "X"))                                   # t0_2
    b += lds_write(L_T, RE) + lds_write(L_T + 6, IM) + add_f_hi(48)               # + f0_2 R -> pending
    b += lds_write(L_PEND, RE) + lds_write(L_PEND + 6, IM) + ["s_waitcnt lgkmcnt(0)"]
    b += call_xy(LINE_BC, line_operand_xy_sum(2))                                   # S_2
    b += sub_lds(L_T, LIN_CARRY[0], LIN_CARRY[1]) + sub_lds(L_T12, LIN_CARRY[0], LIN_CARRY[1]) + add_f_hi(120)
    b += redc_pair(RE, IM, 2, to_a(A_TF1))                                          # f1_2' (kept aside)
    # ---- position 1: X = f0_0, Y = f1_0
    b += call_xy(LINE_C, line_operand_y(1, "Y"))                                   # t1_1
    b += lds_write(L_T, RE) + lds_write(L_T + 6, IM) + add_lds(L_PEND, LIN_CARRY[0], LIN_CARRY[1])
    b += redc_pair(RE, IM, 2, to_a(A_TF0))                                          # f0_2' (kept aside)
    b += call_xy(LINE_B, line_operand_y(1, "X"))                                   # t0_1
    b += dw_park_a(A_T0, RE, IM) + add_f_hi(24)
    b += lds_write(L_PEND, RE) + lds_write(L_PEND + 6, IM) + ["s_waitcnt lgkmcnt(0)"]
    b += call_xy(LINE_BC, line_operand_xy_sum(1))                                   # S_1
    b += dw_from_a(T[0], T[1], A_T0) + ["s_nop 1"]
    b += merge([sub_chain(RE, RE, T[0], LIN_CARRY[0]), sub_chain(IM, IM, T[1], LIN_CARRY[1])])
    b += sub_lds(L_T, LIN_CARRY[0], LIN_CARRY[1]) + add_f_hi(96)
    b += redc_pair(RE, IM, 2, to_a(96))                                             # f1_1'
    # ---- position 0: X = xi f0_2, Y = xi f1_2 (the originals: f0_2', f1_2' are aside)
    b += call_xy(LINE_C, line_operand_y(0, "Y"))                                   # t1_0
    b += lds_write(L_T, RE) + lds_write(L_T + 6, IM) + add_lds(L_PEND, LIN_CARRY[0], LIN_CARRY[1])
    b += redc_pair(RE, IM, 2, to_a(24))                                             # f0_1'
    b += call_xy(LINE_B, line_operand_y(0, "X"))                                   # t0_0
    b += dw_park_a(A_T0, RE, IM) + add_f_hi(0)
    # + xi t1_2: (re - im, re + im) of the parked double-width t1_2
    b += lds_read(T[0], L_T12) + lds_read(T[1], L_T12 + 6) + ["s_waitcnt lgkmcnt(0)"]
    X2 = list(range(48, 72))
    b += merge([sub_chain(X2, T[0], T[1], LIN_CARRY[0]), add_chain(T[1], T[0], T[1], LIN_CARRY[1])])
    b += merge([add_chain(RE, RE, X2, LIN_CARRY[0]), add_chain(IM, IM, T[1], LIN_CARRY[1])])
    b += redc_pair(RE, IM, 2, to_a(0))                                              # f0_0'
    b += call_xy(LINE_BC, line_operand_xy_sum(0))                                   # S_0
    b += dw_from_a(T[0], T[1], A_T0) + ["s_nop 1"]
    b += merge([sub_chain(RE, RE, T[0], LIN_CARRY[0]), sub_chain(IM, IM, T[1], LIN_CARRY[1])])
    b += sub_lds(L_T, LIN_CARRY[0], LIN_CARRY[1]) + add_f_hi(72)
    b += redc_pair(RE, IM, 2, to_a(72))                                             # f1_0'
    # the positions-2 results into place
    b += ["s_nop 1"] + agpr_read(T[0], A_TF1) + agpr_read(T[1], A_TF0) + ["s_nop 1"]
    b += agpr_write(120, T[0]) + agpr_write(48, T[1])
    return ["lcb_r_line:"] + hazard_fix(b + ["s_setpc_b64 s[30:31]"])


def gen_fp12sq():
    """lcb_r_fp12sq: a[0:143] <- a^2 (f = a + b w, components < p), complex method: t = a b (lcb_r_fp6m, y = b from
    the tmp slot s[22:23] = [a | b]), x = a + v b, u = x (a + b) (y = the slot's sum variant), c0 = u - t - v t,
    c1 = 2t — t kept in a[72:143] once b is consumed, so the slot is written once and only read after.  Returns
    through s[30:31]."""
    X, Y, Z, W = T1[:12], T1[12:], T2[:12], T2[12:]
    b = ["s_nop 4"] + gstore(S_T, (None, 0), list(range(0, 144)), "a") + ["s_waitcnt vmcnt(0)"]   # S1 = [a | b]
    b += [f"s_mov_b64 s[{S_M}:{S_M + 1}], s[{S_T}:{S_T + 1}]", f"s_mov_b32 s{S_Q0}, 18", f"s_mov_b32 s{S_SUM}, 0"]
    b += call_ret("lcb_r_fp6m", S_RET6)                                              # t = a b -> a[144:215]
    b += ["s_nop 4"]
    # x = a + v b -> a[0:71]: (a0 + xi b2, a1 + b0, a2 + b1)
    b += agpr_read(X, 120) + agpr_read(Y, 132) + ["s_nop 1"] + xi_into(Z, W, X, Y, T3)          # xi b2
    for part, V in ((0, Z), (1, W)):
        b += agpr_read(X, 12 * part) + ["s_nop 1"] + modadd(X, X, V, Y, LIN_CARRY[0]) + agpr_write(12 * part, X)
    for i in range(2, 6):
        b += agpr_read(X, 12 * i) + agpr_read(Y, 72 + 12 * (i - 2)) + ["s_nop 1"]
        b += modadd(X, X, Y, Z, LIN_CARRY[0]) + agpr_write(12 * i, X)
    for i in range(6):                                                               # t -> a[72:143] (b consumed)
        b += agpr_read(X, 144 + 12 * i) + ["s_nop 1"] + agpr_write(72 + 12 * i, X)
    b += [f"s_mov_b32 s{S_Q0}, 0", f"s_mov_b32 s{S_SUM}, 1"]
    b += call_ret("lcb_r_fp6m", S_RET6)                                              # u = x (a + b) -> a[144:215]
    b += ["s_nop 4"]
    # c0_k = u_k - t_k - (v t)_k with (v t)_0 = xi t_2, (v t)_1 = t_0, (v t)_2 = t_1; then c1 = 2t
    U3, U4 = T3[:12], T3[12:]
    b += agpr_read(Y, 72 + 48) + agpr_read(Z, 72 + 60) + ["s_nop 1"]
    b += modsub(U3, Y, Z, W, LIN_CARRY[0], LIN_CARRY[1]) + modadd(U4, Y, Z, W, LIN_CARRY[2])  # xi t2 = (U3, U4)
    for i in range(6):                                                               # i = 2k + part
        k, part = divmod(i, 2)
        b += agpr_read(X, 144 + 12 * i) + agpr_read(Z, 72 + 12 * i) + ["s_nop 1"]
        if k == 0:
            V = U3 if part == 0 else U4
        else:
            b += agpr_read(Y, 72 + 12 * (i - 2)) + ["s_nop 1"]
            V = Y
        b += modsub(X, X, Z, W, LIN_CARRY[0], LIN_CARRY[1]) + modsub(X, X, V, W, LIN_CARRY[2], LIN_CARRY[3])
        b += agpr_write(12 * i, X)
    for i in range(6):
        b += agpr_read(X, 72 + 12 * i) + ["s_nop 1"] + modadd(X, X, X, Z, LIN_CARRY[0]) + agpr_write(72 + 12 * i, X)
    return ["lcb_r_fp12sq:"] + hazard_fix(b + ["s_setpc_b64 s[30:31]"])


def gen_miller2():
    """lcb_r_miller2: slot s[60:61] <- conj(prod over the 68 lines of l1_k(P1) l2_k(P2)), squarings before every
    doubling line but the first.  Line sets at the lanes' v[250:251], v[252:253] (68 x 48 words each), P1 / P2 at quads
    0..5 / 6..11 of s[56:57] ((0, 0) for infinity), tmp slots s[22:23], s[58:59]."""
    ONE = limbs((1 << 384) % P)
    b = ["s_waitcnt vmcnt(0) lgkmcnt(0)", "s_mov_b64 s[24:25], s[30:31]"] + movs_const(PR, PL)
    b += [f"s_mov_b32 s{S_PINV}, 0x{PINV:08x}"]
    b += mov_regs([V_LS[0], V_LS[0] + 1, V_LS[1], V_LS[1] + 1], [250, 251, 252, 253])
    b += movs_const(list(range(0, 12)), ONE) + ["v_mov_b32 v12, 0"]
    b += [f"v_accvgpr_write_b32 a{j}, v{j}" for j in range(12)] + [f"v_accvgpr_write_b32 a{j}, v12" for j in range(12, 144)]
    b += [f"s_mov_b32 s{S_QT + 1}, {4 * 48}"]                                      # bytes per line
    i, add_next = 62, False
    for k in range(68):
        if add_next:
            add_next = False
        else:
            if k > 0:
                b += call_ret("lcb_r_fp12sq", 30)
            add_next = bool((Z_ABS_BITS >> i) & 1)
            i -= 1
        for t in range(2):
            b += [f"s_mov_b32 s{S_SET}, {t}", f"s_mov_b32 s{S_PQ}, {6 * t}"] + call_ret("lcb_r_line", 30)
            vp = V_LS[t]
            b += [f"v_add_co_u32_e64 v{vp}, {sp(LIN_CARRY[0])}, v{vp}, s{S_QT + 1}",
                  f"v_addc_co_u32_e64 v{vp + 1}, {sp(LIN_CARRY[0])}, v{vp + 1}, 0, {sp(LIN_CARRY[0])}", "s_nop 2"]
    b += ["s_nop 4"] + conj_c1() + walk_store(S_DST) + ["s_setpc_b64 s[24:25]"]
    return ["lcb_r_miller2:"] + hazard_fix(b)


Z_ABS_BITS = 0xd201000000010000


# ------------------------------------------------------------------ emit
def clobbers_n():
    regs = [f'"v{i}"' for i in range(VMAX)] + [f'"a{i}"' for i in range(A_PARK + 2 * N)]
    regs += [f'"s{s}"' for s in CLOBBER_SGPRS + [16, 17, 24, 25]] + ['"scc"', '"vcc"']
    return ", ".join(regs)


def clobbers(nv=VMAX):
    regs = [f'"v{i}"' for i in range(nv)] + [f'"a{A_PARK + j}"' for j in range(2 * N)]
    regs += [f'"s{s}"' for s in CLOBBER_SGPRS] + ['"scc"', '"vcc"']
    return ", ".join(regs)


def emit():
    fp4_txt, fp4_outs, fp4_used = gen_fp4()
    cyc_txt = gen_cyc_sqr(fp4_outs, fp4_used)
    routines = [gen_cyc_sqr_n(), cyc_txt, fp4_txt, gen_pow_z(), gen_fp12_mul_n(), gen_fp12m(), gen_fp6m(),
                gen_fp2dw(), gen_redc2(), gen_miller2(), gen_fp12sq(), gen_line()]
    lib = "\n".join("  .p2align 8\n" + "\n".join(("  " + l) if not l.endswith(":") else l for l in r)
                    for r in routines)
    esc = lib.replace("\\", "\\\\").replace('"', '\\"')
    o = []
    o.append("// GENERATED by tools/gen_tower_asm.py — do not edit.\n")
    o.append("// gfx950 Fp12-level assembly routines over an AGPR-resident accumulator (see the generator's docstring).\n")
    o.append("#pragma once\n#include <hip/hip_runtime.h>\n#include <stdint.h>\n\n")
    o.append("typedef uint32_t u32;\n\n")
    o.append("#define LCB_ASM_TOWER_LIBRARY(tag) \\\n")
    o.append("extern \"C\" __global__ void __launch_bounds__(64) lcb_asm_tower_library_##tag() { \\\n")
    o.append("    asm volatile(LCB_ASM_TOWER_LIBRARY_TEXT); \\\n}\n\n")
    o.append("#define LCB_ASM_TOWER_LIBRARY_TEXT \\\n    \"  s_endpgm\\n\" \\\n")
    for line in esc.split("\n"):
        o.append(f'    "{line}\\n" \\\n')
    o.append('    ""\n\n')
    o.append(f"""// slot_out <- slot_in^(2^count) for an Fp12 in the cyclotomic subgroup (count >= 1 Granger-Scott squarings in
// AGPRs); slots are quad-major SoA (kcommon.hpp: word quad g of item i at byte (g * n + i) * 16), n16 = n * 16,
// lane_off = i * 16.  Reads / writes memory; clobbers v0..v247, a0..a167.
__device__ __forceinline__ void lcb_asm_cyc_sqr_n(const u32 *slot_in, u32 *slot_out, u32 n16, u32 lane_off, u32 count) {{
    asm volatile("s_getpc_b64 s[{S_CALL}:{S_CALL + 1}]\\n\\t"
        "s_add_u32 s{S_CALL}, s{S_CALL}, lcb_r_cyc_sqr_n@rel32@lo+4\\n\\t"
        "s_addc_u32 s{S_CALL + 1}, s{S_CALL + 1}, lcb_r_cyc_sqr_n@rel32@hi+12\\n\\t"
        "s_swappc_b64 s[30:31], s[{S_CALL}:{S_CALL + 1}]"
        : "+{{s18}}"(count)
        : "{{s[20:21]}}"(slot_in), "{{s[22:23]}}"(slot_out), "{{s19}}"(n16), "{{v248}}"(lane_off)
        : {clobbers_n()}, "memory");
}}
""")
    fp12_clob = ", ".join([f'"v{i}"' for i in range(VMAX)] + [f'"a{i}"' for i in range(216)] +
                          [f'"s{x}"' for x in sorted(set(CLOBBER_SGPRS) | {16, 17, 18, 24, 25, 62, 64, 66, 67, 68,
                                                                              72, 73})] + ['"scc"', '"vcc"'])
    call_seq = lambda lbl: (f'"s_getpc_b64 s[{S_CALL}:{S_CALL + 1}]\\n\\t"\n'
                            f'        "s_add_u32 s{S_CALL}, s{S_CALL}, {lbl}@rel32@lo+4\\n\\t"\n'
                            f'        "s_addc_u32 s{S_CALL + 1}, s{S_CALL + 1}, {lbl}@rel32@hi+12\\n\\t"\n'
                            f'        "s_swappc_b64 s[30:31], s[{S_CALL}:{S_CALL + 1}]"')
    o.append(f"""
// dst <- (conj_a ? conj(a) : a) * m over Fp12 slots (lcb_r_fp12_mul_n: Karatsuba over lazily reduced Fp6 products,
// the accumulator in AGPRs); tmp: a slot the call may overwrite (the destination or a, never m); lds_addr: this
// lane's LDS byte address (36 quads at lds_addr + g * 1024).  Clobbers v0..v247, a0..a215.
__device__ __forceinline__ void lcb_asm_fp12_mul_n(const u32 *a, u32 conj_a, const u32 *m, u32 *tmp, u32 *dst, u32 n16,
                                                   u32 lane_off, u32 lds_addr) {{
    asm volatile({call_seq("lcb_r_fp12_mul_n")}
        :
        : "{{s[56:57]}}"(a), "{{s65}}"(conj_a), "{{s[20:21]}}"(m), "{{s[22:23]}}"(tmp), "{{s[60:61]}}"(dst), "{{s19}}"(n16),
          "{{v248}}"(lane_off), "{{v249}}"(lds_addr)
        : {fp12_clob}, "memory");
}}
// dst <- conj(base^|z|) = base^z for a unitary base (lcb_r_pow_z; dst may be base); tmp: a slot the call may
// overwrite (not base).  Clobbers v0..v247, a0..a215.
__device__ __forceinline__ void lcb_asm_pow_z(const u32 *base, u32 *tmp, u32 *dst, u32 n16, u32 lane_off, u32 lds_addr) {{
    asm volatile({call_seq("lcb_r_pow_z")}
        :
        : "{{s[20:21]}}"(base), "{{s[22:23]}}"(tmp), "{{s[60:61]}}"(dst), "{{s19}}"(n16), "{{v248}}"(lane_off),
          "{{v249}}"(lds_addr)
        : {fp12_clob}, "memory");
}}
""")
    ml_clob = ", ".join([f'"v{i}"' for i in range(VMAX)] + [f'"a{i}"' for i in range(240)] +
                        [f'"s{x}"' for x in sorted(set(CLOBBER_SGPRS) | {16, 17, 18, 20, 21, 24, 25, 62, 63, 64, 66,
                                                                            67, 68, 69, 72, 73})] + ['"scc"', '"vcc"'])
    o.append(f"""// dst <- conj(prod_k l1_k(P1) l2_k(P2)), the 68 normalised lines of two line sets (pairing.hpp miller2_norm_lds,
// the same residues): ls1 / ls2 the lane's line sets (68 x 48 words), pslot a slot holding P1 at quads 0..5 and P2
// at quads 6..11 ((0, 0) for a point at infinity), s1 / s2 two tmp slots, lds_addr the lane's 36 LDS quads.
// Clobbers v0..v247, a0..a239.
__device__ __forceinline__ void lcb_asm_miller2(const u32 *ls1, const u32 *ls2, const u32 *pslot, u32 *s1, u32 *s2,
                                                u32 *dst, u32 n16, u32 lane_off, u32 lds_addr) {{
    asm volatile({call_seq("lcb_r_miller2")}
        :
        : "{{v[250:251]}}"(ls1), "{{v[252:253]}}"(ls2), "{{s[56:57]}}"(pslot), "{{s[22:23]}}"(s1), "{{s[58:59]}}"(s2),
          "{{s[60:61]}}"(dst), "{{s19}}"(n16), "{{v248}}"(lane_off), "{{v249}}"(lds_addr)
        : {ml_clob}, "memory");
}}
""")
    return "".join(o), dict(fp4_outs=fp4_outs, fp4_used=len(fp4_used), n_cyc=len(cyc_txt), n_fp4=len(fp4_txt))


def main():
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lachain_amd", "csrc", "asm_tower.hpp")
    txt, info = emit()
    with open(dst, "w") as f:
        f.write(txt)
    print("wrote", os.path.normpath(dst), {k: v for k, v in info.items() if k != "fp4_outs"})


if __name__ == "__main__":
    main()
