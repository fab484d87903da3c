"""Per-kernel register / occupancy / spill table of one .hip file (hipcc resource remarks).

    python scripts/kres.py csrc/kernels/gemm.hip [filter]
"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++20", "-Icsrc", "-I/opt/rocm/include",
       "--cuda-device-only", "-Rpass-analysis=kernel-resource-usage", "-c", src, "-o", "/tmp/_kres.o"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark: +(.*?): (.*) \[-Rpass", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2).strip()
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
demangled = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True,
                           text=True).stdout.splitlines()
for r, d in zip(rows, demangled):
    d = re.sub(r"\(.*", "", d.replace("mpit::(anonymous namespace)::", "").replace("void ", ""))
    if flt in d:
        print(f"{d:60s} vgpr={r.get('VGPRs')} agpr={r.get('AGPRs')} occ={r.get('Occupancy [waves/SIMD]')} "
              f"vspill={r.get('VGPRs Spill')} lds={r.get('LDS Size [bytes/block]')}")
