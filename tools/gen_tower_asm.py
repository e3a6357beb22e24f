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
    routines = [gen_cyc_sqr_n(), cyc_txt, fp4_txt]
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
    return "".join(o), dict(fp4_outs=fp4_outs, fp4_used=len(fp4_used), n_cyc=len(cyc_txt), n_fp4=len(fp4_txt))


def main():
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lachain_amd", "csrc", "asm_tower.hpp")
    txt, info = emit()
    with open(dst, "w") as f:
        f.write(txt)
    print("wrote", os.path.normpath(dst), {k: v for k, v in info.items() if k != "fp4_outs"})


if __name__ == "__main__":
    main()
