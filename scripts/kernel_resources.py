#!/usr/bin/env python3
"""Register / LDS / scratch use of every kernel in a built object's gfx950 code object (from
the AMDGPU metadata notes): spills and the VGPR counts that set occupancy, without a GPU.

    python scripts/kernel_resources.py build/obj/k_gemm.hip.o [name-substring ...]
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def main(argv) -> int:
    obj, pats = argv[0], argv[1:]
    with tempfile.TemporaryDirectory() as d:
        fat, co = os.path.join(d, "fat.bin"), os.path.join(d, "gfx950.co")
        subprocess.check_call([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj, os.path.join(d, "x.o")])
        subprocess.check_call([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                               "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={fat}", f"--output={co}"])
        notes = subprocess.check_output([f"{LLVM}/llvm-readelf", "--notes", co], text=True)
    rows = []
    for e in notes.split("  - .agpr_count:")[1:]:
        def g(k):
            m = re.search(r"\." + k + r":\s+(\S+)", e)
            return m.group(1) if m else "?"
        name = g("name")
        if name == "?":
            continue
        dm = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        dm = dm.replace("mpit::(anonymous namespace)::", "")
        dm = dm[: dm.find("(")] if "(" in dm else dm
        if pats and not any(p in dm for p in pats):
            continue
        rows.append((dm, e.split("\n")[0].strip(), g("vgpr_count"), g("vgpr_spill_count"),
                     g("private_segment_fixed_size"), g("group_segment_fixed_size")))
    print("| kernel | agpr | vgpr | vgpr spill | scratch B | static LDS B |")
    print("|---|---|---|---|---|---|")
    for r in sorted(rows):
        print("| `" + r[0] + "` | " + " | ".join(r[1:]) + " |")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
