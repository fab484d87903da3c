#!/usr/bin/env python3
"""One parameterised runner for every GPU-box job (replaces the per-letter gpu_r0*_*.sh files).

    gpurun --timeout 1200 -- python3 scripts/gpu.py <outdir> <step> [<step> ...]

Writes everything under gpurun_out/<outdir>/. Steps run in order, each under its own
``timeout -k 10``; the first failing step (non-zero exit, time limit, abort, segfault) ends
the run with that step's exit code — nothing else touches the GPU after it.

Steps:
  smoke                 __graft_entry__.smoke()                         -> smoke.log
  tier                  pytest -m gpu (whole GPU tier)                  -> pytest_gpu.log
  pytest:<args>[:K=V;K=V] pytest <args> (e.g. pytest:tests/test_overlap.py), extra env -> pytest_<n>.log
  pytestall:<args>[:K=V] the same without -x (a diagnosis run: every test reports)
  bench                 bench.py defaults (fp32 headline + bf16 secondary) -> bench.json
  bench:<args>[:K=V;K=V] bench.py <args> (comma separated), extra env    -> bench_<n>.json
  dbench:<n>:<args>     bench.py on n ranks sharing the box's GPU (rehearsal) -> dbench_<n>.json
  prof:<name>:<args>[:K=V;K=V] rocprofv3 --kernel-trace of bench.py <args> (extra env) + stream table -> streams_<name>.md
  gemmcalls:<name>:<args> per-call GEMM shapes + times of one steady step     -> gemm_calls_<name>.md
  mp:<script>:<n>[:K=V;K=V] tests/mp/<script> on n ranks with extra env   -> mp_<script>_<n>.log
  py:<file>[:args[:K=V;K=V]] python3 <file> <args> with extra env (benchmarks/ probes) -> py_<n>.log
  profpy:<name>:<file>[:args[:K=V;K=V]] rocprofv3 --kernel-trace --stats of python3 <file> -> pp_<name>/
"""
from __future__ import annotations

import os
import shlex
import subprocess
import sys
import time

ROOT = os.environ.get("GRAFT_REPO_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PY = sys.executable


def _run(out: str, name: str, cmd, limit: int, env=None, stdout_file=None) -> int:
    log = os.path.join(out, name)
    e = dict(os.environ)
    e.setdefault("TMPDIR", "/tmp")
    e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    e["PYTHONPATH"] = ROOT + os.pathsep + e.get("PYTHONPATH", "")
    e.update(env or {})
    full = ["timeout", "-k", "10", str(limit)] + cmd
    t0 = time.time()
    print(f"[gpu.py] {name}: {' '.join(shlex.quote(c) for c in cmd)}", flush=True)
    if stdout_file:
        with open(os.path.join(out, stdout_file), "w") as so, open(log, "w") as se:
            rc = subprocess.call(full, stdout=so, stderr=se, env=e, cwd=ROOT)
    else:
        with open(log, "w") as f:
            rc = subprocess.call(full, stdout=f, stderr=subprocess.STDOUT, env=e, cwd=ROOT)
    print(f"[gpu.py] {name}: rc={rc} in {time.time() - t0:.1f}s", flush=True)
    if rc != 0:
        try:
            with open(log) as f:
                print("".join(f.readlines()[-40:]), flush=True)
        except OSError:
            pass
    return rc


def _tail(path: str, n: int = 3) -> str:
    try:
        with open(path) as f:
            return "".join(f.readlines()[-n:]).rstrip()
    except OSError:
        return ""


def main(argv) -> int:
    if len(argv) < 2:
        print(__doc__)
        return 2
    out = os.path.join(ROOT, "gpurun_out", argv[0])
    os.makedirs(out, exist_ok=True)
    # --tb=short: a failure's report never formats the (large, on-GPU) tensor arguments of the
    # frames it crossed, which can take longer than the time limit
    pyt = [PY, "-u", "-m", "pytest", "-x", "-v", "--tb=short", "--timeout", "120", "--timeout-method", "thread"]
    for i, step in enumerate(argv[1:]):
        kind, _, rest = step.partition(":")
        if kind == "smoke":
            rc = _run(out, "smoke.log", [PY, "-u", "-c", "import __graft_entry__ as g; g.smoke()"], 300)
            print(_tail(os.path.join(out, "smoke.log"), 1))
        elif kind == "tier":
            rc = _run(out, "pytest_gpu.log", pyt + ["tests", "-m", "gpu"] + (rest.split(",") if rest else []), 1000)
            print(_tail(os.path.join(out, "pytest_gpu.log"), 2))
        elif kind in ("pytest", "pytestall"):  # pytestall: no -x (every test reports)
            parts = rest.split(":")
            env = dict(kv.split("=", 1) for kv in parts[1].split(";")) if len(parts) > 1 and parts[1] else {}
            base = pyt if kind == "pytest" else [a for a in pyt if a != "-x"]
            rc = _run(out, f"pytest_{i}.log", base + parts[0].split(","), 900, env=env)
            print(_tail(os.path.join(out, f"pytest_{i}.log"), 2))
        elif kind == "bench":
            parts = rest.split(":")
            args = parts[0].split(",") if parts[0] else []
            env = dict(kv.split("=", 1) for kv in parts[1].split(";")) if len(parts) > 1 and parts[1] else {}
            rc = _run(out, f"bench_{i}.err", [PY, "-u", "bench.py"] + args, 600, stdout_file=f"bench_{i}.json", env=env)
            print(_tail(os.path.join(out, f"bench_{i}.json"), 1)[:600])
        elif kind == "dbench":  # bench.py on n ranks of the box's one GPU (a rehearsal, not a scaling run)
            parts = rest.split(":")
            n, args = parts[0], parts[1].split(",") if len(parts) > 1 and parts[1] else []
            port = str(29500 + (os.getpid() + i) % 2000)
            rc = _run(out, f"dbench_{i}.err", [PY, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
                                             "--master-addr=127.0.0.1", f"--master-port={port}", "bench.py",
                                             "--gpus", n] + args, 600, stdout_file=f"dbench_{i}.json")
            print(_tail(os.path.join(out, f"dbench_{i}.json"), 1)[:400])
        elif kind == "prof":
            name, _, args = rest.partition(":")
            args, _, envs = args.partition(":")
            env = dict(kv.split("=", 1) for kv in envs.split(";")) if envs else {}
            d = os.path.join(out, f"prof_{name}")
            rc = _run(out, f"prof_{name}.log", ["rocprofv3", "--kernel-trace", "--stats", "-d", d, "-o", "t",
                                               "--output-format", "csv", "--", PY, "bench.py"]
                      + (args.split(",") if args else []), 600, env=env)
            if rc == 0:
                rc = _run(out, f"streams_{name}.log", [PY, "scripts/stream_summary.py", d,
                                                       os.path.join(out, f"streams_{name}.md"), "cast_batch_kernel", "3"], 300)
                for root, _, files in os.walk(d):
                    for fn in files:
                        p = os.path.join(root, fn)
                        if fn.endswith("kernel_trace.csv") and os.path.getsize(p) > 40 << 20:
                            os.remove(p)
        elif kind == "queues":  # stream -> hardware queue table (kernel + memory-copy trace)
            name, _, args = rest.partition(":")
            d = os.path.join(out, f"q_{name}")
            rc = _run(out, f"q_{name}.log", ["rocprofv3", "--kernel-trace", "--memory-copy-trace", "-d", d, "-o", "t",
                                            "--output-format", "csv", "--", PY, "bench.py"]
                      + (args.split(",") if args else []), 600)
            if rc == 0:
                rc = _run(out, f"q_{name}_table.log", [PY, "scripts/queue_table.py", d,
                                                      os.path.join(out, f"queues_{name}.md"), name], 300)
                for root, _, files in os.walk(d):
                    for fn in files:
                        if fn.endswith("_trace.csv") and os.path.getsize(os.path.join(root, fn)) > 40 << 20:
                            os.remove(os.path.join(root, fn))
        elif kind == "gemmcalls":  # per-call GEMM table (shapes from MPIT_GEMM_LOG, times from the trace)
            name, _, args = rest.partition(":")
            d = os.path.join(out, f"gc_{name}")
            rc = _run(out, f"gc_{name}.log", ["rocprofv3", "--kernel-trace", "-d", d, "-o", "t",
                                             "--output-format", "csv", "--", PY, "bench.py"]
                      + (args.split(",") if args else []), 600, env={"MPIT_GEMM_LOG": "1"})
            if rc == 0:
                rc = _run(out, f"gc_{name}_table.log", [PY, "scripts/gemm_calls.py", os.path.join(out, f"gc_{name}.log"),
                                                       d, os.path.join(out, f"gemm_calls_{name}.md"), name], 300)
                for root, _, files in os.walk(d):
                    for fn in files:
                        if fn.endswith("kernel_trace.csv") and os.path.getsize(os.path.join(root, fn)) > 40 << 20:
                            os.remove(os.path.join(root, fn))
        elif kind == "mp":
            parts = rest.split(":")
            script, n = parts[0], parts[1]
            env = dict(kv.split("=", 1) for kv in parts[2].split(";")) if len(parts) > 2 and parts[2] else {}
            port = str(29500 + (os.getpid() + i) % 2000)
            rc = _run(out, f"mp_{script}_{n}_{i}.log",
                      [PY, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
                       "--master-addr=127.0.0.1", f"--master-port={port}", os.path.join("tests", "mp", script)],
                      500, env=env)
            print(_tail(os.path.join(out, f"mp_{script}_{n}_{i}.log"), 6))
        elif kind == "profpy":  # rocprofv3 kernel trace + stats of python3 <file> (names and times per kernel)
            parts = rest.split(":")
            name, f = parts[0], parts[1]
            args = parts[2] if len(parts) > 2 else ""
            env = dict(kv.split("=", 1) for kv in parts[3].split(";")) if len(parts) > 3 and parts[3] else {}
            d = os.path.join(out, f"pp_{name}")
            rc = _run(out, f"pp_{name}.log", ["rocprofv3", "--kernel-trace", "--stats", "-d", d, "-o", "t",
                                             "--output-format", "csv", "--", PY, "-u", f]
                      + (args.split(",") if args else []), 600, env=env)
            for root, _, files in os.walk(d):
                for fn in files:
                    if fn.endswith("kernel_trace.csv") and os.path.getsize(os.path.join(root, fn)) > 40 << 20:
                        os.remove(os.path.join(root, fn))
            print(_tail(os.path.join(out, f"pp_{name}.log"), 4))
        elif kind == "py":
            parts = rest.split(":")
            f, args = parts[0], parts[1] if len(parts) > 1 else ""
            env = dict(kv.split("=", 1) for kv in parts[2].split(";")) if len(parts) > 2 and parts[2] else {}
            rc = _run(out, f"py_{i}.log", [PY, "-u", f] + (args.split(",") if args else []), 600, env=env)
            print(_tail(os.path.join(out, f"py_{i}.log"), 8))
        else:
            print(f"[gpu.py] unknown step {step!r}")
            return 2
        if rc != 0:
            print(f"[gpu.py] STOP after {step!r} (rc={rc})", flush=True)
            return rc if rc > 0 else 1
    print("[gpu.py] ALL OK", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
