"""Build an A/B variant of the native module with one kernel file replaced (and/or extra hipcc
flags): every other object is reused from build/obj; the variant lands in build/var_<name>/ and
is loaded instead of the in-tree module with MPIT_NATIVE_SO=build/var_<name>/_mpit<ext>.

Usage: python scripts/build_variant.py NAME SOURCE [--replace gemm.hip] [extra hipcc flags...]
(SOURCE stands in for csrc/kernels/<--replace>, default gemm.hip; --no-base skips the in-tree
build first, so two variants can compile at once once build/obj is current)
"""
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpit_amd import _build as B  # noqa: E402


def main():
    name, src = sys.argv[1], os.path.abspath(sys.argv[2])
    flags = sys.argv[3:]
    rep = "gemm.hip"
    if flags[:1] == ["--replace"]:
        rep, flags = flags[1], flags[2:]
    base = "--no-base" not in flags  # --no-base: reuse build/obj as it is (another build made it)
    flags = [f for f in flags if f != "--no-base"]
    if base:
        B.build()  # the in-tree objects the variant reuses
    out = os.path.join(B.ROOT, "build", f"var_{name}")
    os.makedirs(out, exist_ok=True)
    hipcc = os.path.join(B.ROCM, "bin", "hipcc")
    obj = os.path.join(out, "k_" + rep + ".o")
    cmd = [hipcc, f"--offload-arch={B.ARCH}", "-munsafe-fp-atomics"] + B._common_flags() + [f"-I{os.path.join(B.CSRC, 'kernels')}"] + flags + ["-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode:
        raise SystemExit(r.stderr[-4000:])
    objs = [o if os.path.basename(o) != "k_" + rep + ".o" else obj for (_, o, _) in B._jobs()]
    target = os.path.join(out, "_mpit" + B.EXT)
    cmd = [hipcc, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", target] + objs + [
        f"-L{B.ROCM}/lib", "-lamdhip64", "-lrt", "-lpthread", "-ldl", f"-Wl,-rpath,{B.ROCM}/lib"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode:
        raise SystemExit(r.stderr[-4000:])
    print(target)


if __name__ == "__main__":
    main()
