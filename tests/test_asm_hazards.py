"""Static check of the generated inline carry chains (lachain_amd/csrc/asm_routines.hpp, tools/gen_asm.py):
gfx950 needs 2 wait states between a VALU write of a carry (VCC or an SGPR pair) and a VALU read of it as
carry-in / select.  Every chain link must be separated from its producer by other instructions or s_nop."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "lachain_amd", "csrc", "asm_routines.hpp")
CARRY_WRITERS = ("v_add_co_u32", "v_addc_co_u32", "v_sub_co_u32", "v_subb_co_u32")


def inline_bodies():
    text = open(HDR).read()
    for m in re.finditer(r"__device__ __forceinline__ void (lcb_fp\d?_\w+_asm)\(.*?asm volatile\(\"(.*?)\"\n", text, re.S):
        yield m.group(1), m.group(2).split("\\n\\t")


def carry_reg(ins, write):
    ops = [o.strip() for o in ins.split(None, 1)[1].split(",")]
    if ins.startswith("v_cndmask"):
        return None if write else ops[-1]
    if write:
        return ops[1] if ins.startswith(CARRY_WRITERS) else None
    return ops[-1] if ins.startswith(("v_addc_co_u32", "v_subb_co_u32")) else None


def test_inline_chains_respect_carry_hazard():
    names = []
    for name, body in inline_bodies():
        names.append(name)
        last_write = {}
        slots = 0
        for ins in body:
            if ins.startswith("s_nop"):
                slots += int(ins.split()[1]) + 1
                continue
            rd = carry_reg(ins, write=False)
            if rd is not None and rd in last_write:
                assert slots - last_write[rd] >= 2, (name, ins)
            slots += 1
            wr = carry_reg(ins, write=True)
            if wr is not None:
                last_write[wr] = slots
    assert {"lcb_fp_add_asm", "lcb_fp_sub_asm", "lcb_fp2_add_asm", "lcb_fp2_sub_asm", "lcb_fp2_neg_asm",
            "lcb_fp2_mul_xi_asm"} <= set(names)
