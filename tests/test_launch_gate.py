"""Every kernel launch of the library goes through the scratch gate (gate.hpp LCB_LAUNCH_GATED): no
translation unit calls hipLaunchKernelGGL or a triple-chevron launch directly, so no kernel with a private segment can
reach a hardware queue without the gate seeing its reservation.  Static check over the sources (CPU suite)."""
import glob
import os
import re

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lachain_amd", "csrc")


def test_no_ungated_launches():
    bad = []
    for p in sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.hpp")) +
                    glob.glob(os.path.join(CSRC, "*.cpp"))):
        if os.path.basename(p) == "gate.hpp":
            continue
        for i, line in enumerate(open(p), 1):
            code = line.split("//")[0]
            if re.search(r"\bhipLaunchKernelGGL\s*\(", code) or "<<<" in code or re.search(r"\bhipLaunchKernel\s*\(", code):
                bad.append(f"{os.path.basename(p)}:{i}: {line.strip()}")
    assert not bad, "launches outside LCB_LAUNCH_GATED:\n" + "\n".join(bad)


def test_gate_macro_is_the_only_raw_launch():
    src = open(os.path.join(CSRC, "gate.hpp")).read()
    assert src.count("hipLaunchKernelGGL(") == 1
    assert "lcb_gate_enter" in src and "lcb_gate_exit" in src
