"""Static check of the built library for instructions the compiler scheduled inside a whole-wave-mode bracket.

The AMDGPU backend spills SGPRs into lanes of a whole-wave register (v255 here) and copies that register to an AGPR /
scratch and back with EXEC forced to all lanes:  s_or_saveexec_b64 sX, -1 ; <copy of the WWM register> ;
s_mov_b64 exec, sX.  Any other EXEC-dependent instruction scheduled between those two writes runs for all 64 lanes
instead of the lanes of its own region.  VERDICT r4 #2 was exactly that: in one build of k_tpke_rlc_search2b the
copy of `found` out of the `if (cand)` region (v_accvgpr_write_b32 a201, v5) landed inside the bracket that restores
v255 from a199, so the lanes outside the region (j >= len) got a garbage nonzero `found`, the half-wave ballot never
saw exactly two locating lanes and every open group went to single checks.

Usage: python tools/wwm_check.py [lib.so]   (prints every bracket that holds a foreign instruction; exit 1 if any)
"""
import glob
import os
import re
import shutil
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def disassemble(so_path):
    out = []
    with tempfile.TemporaryDirectory() as td:
        so = os.path.join(td, "lib.so")
        shutil.copy(so_path, so)
        subprocess.run([os.path.join(LLVM, "llvm-objdump"), "--offloading", so], cwd=td, check=True,
                       capture_output=True)
        for co in sorted(glob.glob(os.path.join(td, "lib.so.*gfx950"))):
            out.append(subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn", co],
                                      check=True, capture_output=True, text=True).stdout)
    return out


def functions(text):
    """(function name, [instructions]) for every function / kernel of a disassembly"""
    fn, body = None, []
    for line in text.splitlines():
        m = re.match(r"^[0-9a-f]+ <([^>]+)>:", line)
        if m:
            if fn:
                yield fn, body
            fn, body = m.group(1), []
            continue
        ins = line.split("//")[0].strip()
        if ins:
            body.append(ins)
    if fn:
        yield fn, body


def brackets(body):
    """(index of the opening instruction, instructions inside) for every s_or_saveexec_b64 sX, -1 ... s_mov_b64 exec,
    sX of one function"""
    open_reg, inside, at = None, [], 0
    for k, ins in enumerate(body):
        m = re.match(r"s_or_saveexec_b64 (s\[\d+:\d+\]), -1$", ins)
        if m:
            open_reg, inside, at = m.group(1), [], k
            continue
        if open_reg:
            if ins == f"s_mov_b64 exec, {open_reg}":
                yield at, inside
                open_reg = None
            else:
                inside.append(ins)


def lane_registers(body, at, n_inside):
    """the function's SGPR-spill lane VGPRs (v_writelane targets), the registers the bracket opened at `at` saves or
    restores, and the AGPRs / VGPRs the bracket copies them to or from"""
    regs = set()
    for ins in body:                     # the function's SGPR-spill lane VGPRs (targets of v_writelane)
        m = re.match(r"v_writelane_b32 (v\d+),", ins)
        if m:
            regs.add(m.group(1))
    # prologue / epilogue: the bracket saves or restores a register to / from scratch
    for ins in body[at + 1:at + 1 + n_inside]:
        m = re.match(r"(?:scratch|buffer)_(?:store|load)_dword (?:off, )?(v\d+|a\d+)", ins)
        if m:
            regs.add(m.group(1))
    changed = True
    while changed:
        changed = False
        for ins in body[at + 1:at + 1 + n_inside]:
            m = re.match(r"v_accvgpr_(?:write|read)_b32 (\w+), (\w+)$", ins) or re.match(r"v_mov_b32(?:_e32)? (\w+), (\w+)$", ins)
            if m and (m.group(1) in regs) != (m.group(2) in regs):
                regs |= {m.group(1), m.group(2)}
                changed = True
    return regs


def allowed(ins, lanes):
    """copies of the spill-lane register(s), their scratch save / restore and scalar work that does not read EXEC"""
    if ins.startswith(("s_nop", "s_waitcnt")):
        return True
    if ins.startswith("s_") and "exec" not in ins:
        return True
    ops = [o.strip() for o in ins.split(None, 1)[1].split(",")] if " " in ins else []
    if ins.startswith(("v_accvgpr_write_b32", "v_accvgpr_read_b32", "v_mov_b32")) and len(ops) >= 2:
        return ops[0] in lanes and ops[1] in lanes
    if ins.startswith(("scratch_store_dword ", "scratch_load_dword ", "buffer_store_dword ", "buffer_load_dword ")):
        return any(o in lanes for o in ops[:2])
    return False


def check(so_path):
    bad = []
    n = 0
    for text in disassemble(so_path):
        for fn, body in functions(text):
            for at, inside in brackets(body):
                n += 1
                lanes = lane_registers(body, at, len(inside))
                foreign = [i for i in inside if not allowed(i, lanes)]
                if foreign:
                    bad.append((fn, foreign))
    return n, bad


def main():
    so = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "lachain_amd", "liblachain_bls.so")
    n, bad = check(so)
    print(f"{n} whole-wave brackets, {len(bad)} with foreign instructions")
    for fn, foreign in bad:
        print(f"  {fn}: {foreign}")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
