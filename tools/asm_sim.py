#!/usr/bin/env python3
"""tools/asm_sim.py — single-lane interpreter for the gfx950 leaf routines in lachain_amd/csrc/asm_routines.hpp.

Executes the generated routine text (the subset of VOP2/VOP3/SOP1 instructions tools/gen_asm.py emits) for
one lane with Python integers, so the generator's arithmetic and its register contract (which VGPRs/SGPRs a
routine may write) can be checked on the CPU, without a GPU.  Used by tests/test_asm_routines.py.
"""
import os
import re

M32 = (1 << 32) - 1
HERE = os.path.dirname(os.path.abspath(__file__))
HPP = os.path.join(HERE, "..", "lachain_amd", "csrc", "asm_routines.hpp")


TOWER_HPP = os.path.join(HERE, "..", "lachain_amd", "csrc", "asm_tower.hpp")


def load_library(path=HPP, macro="LCB_ASM_LIBRARY_TEXT"):
    """-> {label: [(mnemonic, [operands])]} parsed from the library text macro."""
    src = open(path).read()
    body = src[src.index("#define " + macro):]
    body = body[:body.index('    ""\n')]
    routines, cur = {}, None
    for raw in re.findall(r'"(.*?)\\n"', body):
        line = raw.strip()
        if not line or line.startswith("."):
            continue
        if line.endswith(":"):
            cur = line[:-1]
            routines[cur] = []
            continue
        if cur is None:
            continue
        mn, _, rest = line.partition(" ")
        ops = [o.strip() for o in rest.split(",")] if rest else []
        routines[cur].append((mn, ops))
    return routines


def _regs(op):
    """'v12' -> ('v', [12]); 'v[36:37]' -> ('v', [36, 37]); 's[90:91]' -> ('s', [90, 91])"""
    m = re.fullmatch(r"([vsa])(\d+)", op)
    if m:
        return m.group(1), [int(m.group(2))]
    m = re.fullmatch(r"([vsa])\[(\d+):(\d+)\]", op)
    if m:
        lo, hi = int(m.group(2)), int(m.group(3))
        return m.group(1), list(range(lo, hi + 1))
    return None, None


class Lane:
    def __init__(self):
        self.v, self.s, self.a = {}, {}, {}
        self.written_v, self.written_s, self.written_a = set(), set(), set()
        self.counts = {}

    def get(self, op):
        kind, rr = _regs(op)
        if kind is None:
            return int(op, 0) & M32
        f = {"v": self.v, "s": self.s, "a": self.a}[kind]
        val = 0
        for k, r in enumerate(rr):
            if r not in f:
                raise KeyError(f"read of undefined {kind}{r}")
            val |= f[r] << (32 * k)
        return val

    def getmask(self, op):  # a lane-mask SGPR pair: this lane's bit
        return self.get(op) & 1

    def put(self, op, val):
        kind, rr = _regs(op)
        f, w = {"v": (self.v, self.written_v), "s": (self.s, self.written_s), "a": (self.a, self.written_a)}[kind]
        if kind == "v" and len(rr) == 2 and rr[0] % 2:
            raise ValueError(f"misaligned 64-bit VGPR pair {op}")
        for k, r in enumerate(rr):
            f[r] = (val >> (32 * k)) & M32
            w.add(r)


def run(routine, lane, routines=None):
    target = None
    for mn, ops in routine:
        g = lane.get
        lane.counts[mn] = lane.counts.get(mn, 0) + 1
        if mn == "v_mad_u64_u32":
            r = g(ops[2]) * g(ops[3]) + g(ops[4])
            lane.put(ops[0], r & ((1 << 64) - 1)); lane.put(ops[1], r >> 64)
        elif mn in ("v_add_co_u32_e64", "v_addc_co_u32_e64"):
            r = g(ops[2]) + g(ops[3]) + (lane.getmask(ops[4]) if mn == "v_addc_co_u32_e64" else 0)
            lane.put(ops[0], r & M32); lane.put(ops[1], r >> 32)
        elif mn in ("v_sub_co_u32_e64", "v_subb_co_u32_e64"):
            r = g(ops[2]) - g(ops[3]) - (lane.getmask(ops[4]) if mn == "v_subb_co_u32_e64" else 0)
            lane.put(ops[0], r & M32); lane.put(ops[1], 1 if r < 0 else 0)
        elif mn == "v_cndmask_b32_e64":
            lane.put(ops[0], g(ops[2]) if lane.getmask(ops[3]) else g(ops[1]))
        elif mn == "v_alignbit_b32":         # ({S0, S1} >> S2[4:0]) low word
            r = ((g(ops[1]) << 32) | g(ops[2])) >> (g(ops[3]) & 31)
            lane.put(ops[0], r & M32)
        elif mn == "v_lshlrev_b32":
            lane.put(ops[0], (g(ops[2]) << (g(ops[1]) & 31)) & M32)
        elif mn == "v_mul_lo_u32":
            lane.put(ops[0], (g(ops[1]) * g(ops[2])) & M32)
        elif mn in ("v_mov_b32", "s_mov_b32", "v_accvgpr_read_b32", "v_accvgpr_write_b32"):
            lane.put(ops[0], g(ops[1]))
        elif mn in ("s_nop", "s_getpc_b64", "s_addc_u32"):
            pass
        elif mn == "s_add_u32":             # call sequence: remember the target label
            target = ops[2].split("@")[0]
        elif mn == "s_swappc_b64":
            run(routines[target], lane, routines)
        elif mn == "s_setpc_b64":
            return
        elif mn == "s_endpgm":
            return
        else:
            raise NotImplementedError(mn)
    raise RuntimeError("routine fell off its end without s_setpc_b64")


def call(routines, label, inputs, agprs=None):
    """inputs: {first VGPR: 12-limb integer}; agprs: {first AGPR: 12-limb integer}.
    Returns (lane, reader(first VGPR) -> integer)."""
    lane = Lane()
    for base, val in inputs.items():
        for j in range(12):
            lane.v[base + j] = (val >> (32 * j)) & M32
    for base, val in (agprs or {}).items():
        for j in range(12):
            lane.a[base + j] = (val >> (32 * j)) & M32
    run(routines[label], lane, routines)

    def read(base):
        return sum(lane.v[base + j] << (32 * j) for j in range(12))
    return lane, read


# ---------------------------------------------------------------- whole-library programs (asm_tower.hpp, round 5)
# Labels, branches, calls with a return stack, SALU, global memory (a dict of 32-bit words keyed by byte address) and
# LDS: enough to run lcb_r_pow_z / lcb_r_fp12_mul_n and their callees for one lane.
def load_program(path=TOWER_HPP, macro="LCB_ASM_TOWER_LIBRARY_TEXT"):
    """-> (instructions [(mnemonic, [operands])], {label: index})"""
    src = open(path).read()
    body = src[src.index("#define " + macro):]
    body = body[:body.index('    ""\n')]
    prog, labels = [], {}
    for raw in re.findall(r'"(.*?)\\n"', body):
        line = raw.strip()
        if not line or line.startswith("."):
            continue
        if line.endswith(":"):
            labels[line[:-1]] = len(prog)
            continue
        mn, _, rest = line.partition(" ")
        ops = [o.strip() for o in rest.split(",")] if rest else []
        prog.append((mn, ops))
    return prog, labels


def _split_off(op):
    """'v[72:75] offset:1024' -> ('v[72:75]', 1024)"""
    m = re.fullmatch(r"(\S+)\s+offset:(\d+)", op)
    return (m.group(1), int(m.group(2))) if m else (op, 0)


class ProgLane(Lane):
    def __init__(self):
        super().__init__()
        self.mem, self.lds, self.scc = {}, {}, 0

    def load(self, addr, n):
        out = 0
        for k in range(n):
            a = addr + 4 * k
            if a not in self.mem:
                raise KeyError(f"load of unwritten memory 0x{a:x}")
            out |= self.mem[a] << (32 * k)
        return out

    def store(self, addr, val, n):
        for k in range(n):
            self.mem[addr + 4 * k] = (val >> (32 * k)) & M32


def run_program(prog, labels, entry, lane, max_steps=50_000_000):
    pc, stack, target = labels[entry], [], None
    g = lane.get
    for _ in range(max_steps):
        mn, ops = prog[pc]
        pc += 1
        lane.counts[mn] = lane.counts.get(mn, 0) + 1
        if mn == "v_mad_u64_u32":
            r = g(ops[2]) * g(ops[3]) + g(ops[4])
            lane.put(ops[0], r & ((1 << 64) - 1)); lane.put(ops[1], r >> 64)
        elif mn in ("v_add_co_u32_e64", "v_addc_co_u32_e64"):
            r = g(ops[2]) + g(ops[3]) + (lane.getmask(ops[4]) if mn == "v_addc_co_u32_e64" else 0)
            lane.put(ops[0], r & M32); lane.put(ops[1], r >> 32)
        elif mn in ("v_sub_co_u32_e64", "v_subb_co_u32_e64"):
            r = g(ops[2]) - g(ops[3]) - (lane.getmask(ops[4]) if mn == "v_subb_co_u32_e64" else 0)
            lane.put(ops[0], r & M32); lane.put(ops[1], 1 if r < 0 else 0)
        elif mn == "v_cndmask_b32_e64":
            lane.put(ops[0], g(ops[2]) if lane.getmask(ops[3]) else g(ops[1]))
        elif mn == "v_mul_lo_u32":
            lane.put(ops[0], (g(ops[1]) * g(ops[2])) & M32)
        elif mn == "v_alignbit_b32":
            lane.put(ops[0], (((g(ops[1]) << 32) | g(ops[2])) >> (g(ops[3]) & 31)) & M32)
        elif mn == "v_lshlrev_b32":
            lane.put(ops[0], (g(ops[2]) << (g(ops[1]) & 31)) & M32)
        elif mn == "s_and_b32":
            r = g(ops[1]) & g(ops[2])
            lane.put(ops[0], r); lane.scc = 1 if r else 0
        elif mn == "s_lshr_b32":
            r = g(ops[1]) >> (g(ops[2]) & 31)
            lane.put(ops[0], r); lane.scc = 1 if r else 0
        elif mn in ("v_mov_b32", "s_mov_b32", "s_mov_b64", "v_accvgpr_read_b32", "v_accvgpr_write_b32"):
            lane.put(ops[0], g(ops[1]))
        elif mn == "s_add_u32":
            if "@" in ops[2]:
                target = ops[2].split("@")[0]
            else:
                r = g(ops[1]) + g(ops[2])
                lane.put(ops[0], r & M32); lane.scc = r >> 32
        elif mn == "s_addc_u32":
            if "@" not in ops[2]:
                r = g(ops[1]) + g(ops[2]) + lane.scc
                lane.put(ops[0], r & M32); lane.scc = r >> 32
        elif mn == "s_sub_u32":
            r = g(ops[1]) - g(ops[2])
            lane.put(ops[0], r & M32); lane.scc = 1 if r < 0 else 0
        elif mn == "s_mul_i32":
            lane.put(ops[0], (g(ops[1]) * g(ops[2])) & M32)
        elif mn == "s_cmp_eq_u32":
            lane.scc = 1 if g(ops[0]) == g(ops[1]) else 0
        elif mn == "s_cmp_lg_u32":
            lane.scc = 1 if g(ops[0]) != g(ops[1]) else 0
        elif mn == "s_branch":
            pc = labels[ops[0]]
        elif mn in ("s_cbranch_scc1", "s_cbranch_scc0"):
            if lane.scc == (1 if mn.endswith("1") else 0):
                pc = labels[ops[0]]
        elif mn in ("s_nop", "s_waitcnt", "s_getpc_b64"):
            pass
        elif mn == "s_swappc_b64":
            stack.append(pc)
            pc = labels[target]
        elif mn == "s_setpc_b64":
            if not stack:
                return
            pc = stack.pop()
        elif mn in ("global_load_dwordx4", "global_store_dwordx4"):
            last, off = _split_off(ops[2])
            if last == "off":                       # 64-bit VGPR address
                addr = g(ops[1] if mn == "global_load_dwordx4" else ops[0]) + off
            else:                                   # SGPR base + 32-bit VGPR offset
                addr = g(last) + g(ops[1] if mn == "global_load_dwordx4" else ops[0]) + off
            if mn == "global_load_dwordx4":
                lane.put(ops[0], lane.load(addr, 4))
            else:
                lane.store(addr, g(ops[1]), 4)
        elif mn in ("ds_write_b128", "ds_read_b128"):
            if mn == "ds_write_b128":
                src, off = _split_off(ops[1])
                a = g(ops[0]) + off
                for k in range(4):
                    lane.lds[a + 4 * k] = (g(src) >> (32 * k)) & M32
            else:
                addr, off = _split_off(ops[1])
                a = g(addr) + off
                lane.put(ops[0], sum(lane.lds[a + 4 * k] << (32 * k) for k in range(4)))
        else:
            raise NotImplementedError(mn)
    raise RuntimeError("step limit")
