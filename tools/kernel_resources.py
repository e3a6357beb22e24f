"""Per-kernel register / spill / scratch figures of the built liblachain_bls.so, from the code-object metadata.

The library's gfx950 code objects are extracted from a copy of the .so (llvm-objdump --offloading) and their AMDGPU
metadata notes read (llvm-readelf --notes): .vgpr_count, .agpr_count, .vgpr_spill_count, .sgpr_spill_count and
.private_segment_fixed_size (scratch per lane) for every kernel.  tests/test_kernel_resources.py gates regressions
with it.  Usage: python tools/kernel_resources.py [path/to/liblachain_bls.so]
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
FIELDS = ("vgpr_count", "agpr_count", "vgpr_spill_count", "sgpr_spill_count", "private_segment_fixed_size",
          "group_segment_fixed_size")


def kernel_resources(so_path=None):
    """{kernel name: {field: int}} for every kernel of the library (the .kd entries, not the asm-library stubs)"""
    so_path = so_path or os.path.join(ROOT, "lachain_amd", "liblachain_bls.so")
    out = {}
    with tempfile.TemporaryDirectory() as td:
        so = os.path.join(td, "lib.so")
        shutil.copy(so_path, so)
        subprocess.run([os.path.join(LLVM, "llvm-objdump"), "--offloading", so], cwd=td, check=True,
                       capture_output=True)
        for co in sorted(glob.glob(os.path.join(td, "lib.so.*gfx950"))):
            notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", co], check=True,
                                   capture_output=True, text=True).stdout
            # one YAML mapping per kernel under amdhsa.kernels; split on the list items
            for blk in re.split(r"\n\s+- \.", notes):
                m = re.search(r"\.name:\s+(\S+)", blk)
                if not m or not re.search(r"\.symbol:\s+\S+\.kd", blk):
                    continue
                rec = {}
                for f in FIELDS:
                    v = re.search(r"(?:^|\.)" + f + r":\s+(\d+)", blk, re.M)
                    rec[f] = int(v.group(1)) if v else 0
                out[m.group(1)] = rec
    return out


def main():
    res = kernel_resources(sys.argv[1] if len(sys.argv) > 1 else None)
    print(f"{'kernel':36s} {'vgpr':>5s} {'agpr':>5s} {'vspill':>7s} {'sspill':>7s} {'scratch':>8s} {'lds':>7s}")
    for k, r in sorted(res.items()):
        print(f"{k:36s} {r['vgpr_count']:5d} {r['agpr_count']:5d} {r['vgpr_spill_count']:7d} "
              f"{r['sgpr_spill_count']:7d} {r['private_segment_fixed_size']:8d} {r['group_segment_fixed_size']:7d}")


if __name__ == "__main__":
    main()
