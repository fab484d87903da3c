"""In-tree build of the native module ``mpit_amd/_mpit*.so`` for gfx950.

HIP kernels (``csrc/kernels/*.hip``) are compiled by ``hipcc --offload-arch=gfx950``;
the host runtime (``csrc/core/*.cpp``) and the pybind11 bindings by ``amdclang++`` against
the HIP headers; one shared object links them with libamdhip64. No torch headers are
involved, so a clean build takes well under a minute on 8 cores and cross-compiles on a
machine without a GPU. Objects are rebuilt only when a source or header is newer.

Usage: ``python -m mpit_amd._build [-j N] [--force] [--sanitize address|thread]``

``--sanitize`` builds a host-sanitized variant into ``build/san_<kind>/`` (ASan / TSan on
the host code: the runtime in csrc/core and the host side of the kernel files, the device
code untouched), loaded instead of the in-tree module when ``MPIT_NATIVE_SO`` names it;
scripts/sanitize.sh runs the multi-process suites under both (CPU, MPIT_CPU_ONLY=1).
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(ROOT, "build", "obj")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("MPIT_OFFLOAD_ARCH", "gfx950")
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
TARGET = os.path.join(ROOT, "mpit_amd", "_mpit" + EXT)


def _pybind_include() -> str:
    import pybind11

    return pybind11.get_include()


def _common_flags() -> list[str]:
    return [
        "-O3",
        "-fPIC",
        "-std=c++20",
        "-Wall",
        "-Wno-unused-function",
        "-Wno-unused-variable",
        f"-I{CSRC}",
        f"-I{ROCM}/include",
        "-D__HIP_PLATFORM_AMD__",
    ]


def _headers() -> list[str]:
    return glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True)


def _san_flags(san):
    return [f"-fsanitize={san}", "-fno-omit-frame-pointer", "-g"] if san else []


def _jobs(san=None, build_dir=BUILD) -> list[tuple[str, str, list[str]]]:
    jobs = []
    hipcc = os.path.join(ROCM, "bin", "hipcc")
    clang = os.path.join(ROCM, "llvm", "bin", "clang++")
    if not os.path.exists(clang):
        clang = os.path.join(ROCM, "bin", "amdclang++")
    # hipcc lines: the sanitizer applies to the host compilation only (-Xarch_host before
    # each -fsanitize=), the gfx950 device code is built as usual
    kflags = [f for x in _san_flags(san) for f in (["-Xarch_host", x] if x.startswith("-fsanitize") else [x])]
    for src in sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip"))):
        obj = os.path.join(build_dir, "k_" + os.path.basename(src) + ".o")
        cmd = [hipcc, f"--offload-arch={ARCH}", "-munsafe-fp-atomics"] + _common_flags() + kflags + ["-c", src, "-o", obj]
        jobs.append((src, obj, cmd))
    host_srcs = sorted(glob.glob(os.path.join(CSRC, "core", "*.cpp"))) + [os.path.join(CSRC, "bindings.cpp")]
    for src in host_srcs:
        obj = os.path.join(build_dir, "h_" + os.path.basename(src) + ".o")
        cmd = [clang, "-x", "c++"] + _common_flags() + _san_flags(san) + [
            f"-I{_pybind_include()}",
            f"-I{sysconfig.get_paths()['include']}",
            "-fvisibility=hidden",
            "-c",
            src,
            "-o",
            obj,
        ]
        jobs.append((src, obj, cmd))
    return jobs


_INC = None


def _includes(path: str, seen: set) -> set:
    """Project headers ``path`` includes, transitively (``#include "..."`` resolved against the
    including file's directory, then csrc/)."""
    global _INC
    if _INC is None:
        import re

        _INC = re.compile(r'^\s*#\s*include\s*"([^"]+)"', re.M)
    try:
        with open(path) as f:
            text = f.read()
    except OSError:
        return seen
    for name in _INC.findall(text):
        for base in (os.path.dirname(path), CSRC):
            h = os.path.normpath(os.path.join(base, name))
            if os.path.exists(h):
                if h not in seen:
                    seen.add(h)
                    _includes(h, seen)
                break
    return seen


def _stale(src: str, obj: str, hdr_mtime: float = None) -> bool:
    """An object is stale when its source or any project header it includes (transitively) is
    newer: editing csrc/core/ps.h no longer recompiles the kernel files."""
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    deps = _includes(src, set())
    newest = max([os.path.getmtime(src)] + [os.path.getmtime(h) for h in deps])
    return newest > t


def build(jobs: int = 8, force: bool = False, verbose: bool = False, sanitize: str = None) -> str:
    build_dir = BUILD if not sanitize else os.path.join(ROOT, "build", f"obj_{sanitize}")
    target = TARGET if not sanitize else os.path.join(ROOT, "build", f"san_{sanitize}", "_mpit" + EXT)
    os.makedirs(build_dir, exist_ok=True)
    os.makedirs(os.path.dirname(target), exist_ok=True)
    hdr_mtime = max([os.path.getmtime(h) for h in _headers()] + [0.0])
    all_jobs = _jobs(sanitize, build_dir)
    # a tree shipped without its object files (the GPU box: build/ does not travel) whose
    # module is newer than every source and header is up to date as it is
    if not force and os.path.exists(target) and not all(os.path.exists(o) for (_, o, _) in all_jobs):
        newest_src = max([os.path.getmtime(s) for (s, _, _) in all_jobs] + [hdr_mtime])
        if os.path.getmtime(target) >= newest_src:
            return target
    todo = [(s, o, c) for (s, o, c) in all_jobs if force or _stale(s, o, hdr_mtime)]

    def run(job):
        src, obj, cmd = job
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"compile failed: {src}\n{r.stdout}\n{r.stderr}")
        return src

    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        for src in ex.map(run, todo):
            if verbose:
                print("built", os.path.relpath(src, ROOT), flush=True)
    objs = [o for (_, o, _) in all_jobs]
    newest = max(os.path.getmtime(o) for o in objs)
    if force or todo or not os.path.exists(target) or os.path.getmtime(target) < newest:
        hipcc = os.path.join(ROCM, "bin", "hipcc")
        # sanitized variant: the shared sanitizer runtime comes from LD_PRELOAD (Python is not
        # instrumented), the module only references it
        san = ["-Xarch_host", f"-fsanitize={sanitize}", "-shared-libsan"] if sanitize else []
        # link to a temporary name and rename: a process (or a tree snapshot) that opens the
        # module meanwhile sees the old or the new file, never a half-written one
        tmp = target + ".tmp"
        cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC"] + san + ["-o", tmp] + objs + [
            f"-L{ROCM}/lib",
            "-lamdhip64",
            "-lrt",
            "-lpthread",
            "-ldl",
            f"-Wl,-rpath,{ROCM}/lib",
        ]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, target)
    return target


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", action="store_true")
    ap.add_argument("--sanitize", choices=["address", "thread"], default=None)
    a = ap.parse_args(argv)
    print(build(a.j, a.force, a.v, a.sanitize))
    return 0


if __name__ == "__main__":
    sys.exit(main())
