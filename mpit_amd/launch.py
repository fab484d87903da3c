"""Launcher and role topologies (SURVEY §2.10 T1–T6).

Role assignment functions return ``(servers, workers, testers)`` lists of world ranks:

* :func:`even_odd` — asyncsgd/mlaunch.lua:40-46: even ranks serve, odd ranks train;
* :func:`half_half` — asyncsgd/ptest.lua:20-26: first half serve, second half train;
* :func:`master_freq` — BiCNN/plaunch.lua:117-177: rank i serves iff i % freq == 0, with an
  optional dedicated tester first or last (``-testerfirst`` / ``-testerlast``);
* :func:`colocated` — every rank trains and serves one shard (the MI355X default: all 8
  GPUs compute, every worker's push / pull fans out over all 7 xGMI links);
* :func:`dedicated` — the first ``k`` ranks serve (BASELINE "1 pserver + 7 workers").

``python -m mpit_amd.launch --nproc N script.py [args]`` starts N local processes with the
``RANK`` / ``WORLD_SIZE`` / ``LOCAL_RANK`` / ``MASTER_ADDR`` / ``MASTER_PORT`` environment
the runtime reads (the reference used ``mpirun -np N th script.lua``, README.md:30). The
launcher itself never touches the GPU; it forwards signals and returns the first
non-zero exit code (the failure of any rank terminates the others).
"""
from __future__ import annotations

import argparse
import os
import signal
import socket
import subprocess
import sys
import time
from typing import List, Optional, Tuple

Roles = Tuple[List[int], List[int], List[int]]


def even_odd(world: int) -> Roles:
    return [r for r in range(world) if r % 2 == 0], [r for r in range(world) if r % 2 == 1], []


def half_half(world: int) -> Roles:
    h = world // 2
    return list(range(h)), list(range(h, world)), []


def master_freq(world: int, freq: int, tester: str = "first") -> Roles:
    """BiCNN/plaunch.lua:125-163. tester='first': rank 0 tests; rank i >= 1 serves iff
    i % freq == 0, else trains. tester='last': rank i <= world-2 serves iff
    (i+1) % freq == 0, else trains; the last rank tests. The tester is a PS client too
    (it pulls parameters): pass ``testers + workers`` as the client list."""
    if tester == "first":
        servers = [i for i in range(1, world) if i % freq == 0]
        workers = [i for i in range(1, world) if i % freq != 0]
        return servers, workers, [0]
    if tester == "last":
        servers = [i for i in range(world - 1) if (i + 1) % freq == 0]
        workers = [i for i in range(world - 1) if (i + 1) % freq != 0]
        return servers, workers, [world - 1]
    raise ValueError("tester must be 'first' or 'last' (BiCNN/plaunch.lua requires one of them)")


def colocated(world: int) -> Roles:
    return list(range(world)), list(range(world)), []


def dedicated(world: int, nservers: int = 1) -> Roles:
    k = max(1, min(nservers, world - 1)) if world > 1 else 0
    return list(range(k)), list(range(k, world)) if world > 1 else [0], []


TOPOLOGIES = {"even_odd": even_odd, "half_half": half_half, "colocated": colocated}


def roles(name: str, world: int, **kw) -> Roles:
    if name == "master_freq":
        return master_freq(world, kw.get("freq", 2), kw.get("tester", "first"))
    if name == "dedicated":
        return dedicated(world, kw.get("servers", 1))
    return TOPOLOGIES[name](world)


def gpu_for(rank: int, world: int, ngpus: int) -> int:
    """asyncsgd/ptest.lua:44 maps worker ranks to GPUs as (rank % (size/2)) % gpus; on a
    node with one process per GPU the local rank is the device."""
    return rank % max(1, ngpus)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch(nproc: int, argv: List[str], master_port: Optional[int] = None, env_extra=None,
           timeout: Optional[float] = None) -> int:
    port = master_port or _free_port()
    procs = []
    for r in range(nproc):
        env = dict(os.environ)
        env.update({"RANK": str(r), "WORLD_SIZE": str(nproc), "LOCAL_RANK": str(r), "LOCAL_WORLD_SIZE": str(nproc),
                    "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        env["PYTHONPATH"] = root + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
        env.update(env_extra or {})
        procs.append(subprocess.Popen([sys.executable] + argv, env=env, start_new_session=True))

    def kill_all(sig=signal.SIGTERM):
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, sig)
                except ProcessLookupError:
                    pass

    t0 = time.time()
    rc = 0
    try:
        while True:
            alive = 0
            for p in procs:
                c = p.poll()
                if c is None:
                    alive += 1
                elif c != 0 and rc == 0:
                    rc = c
                    kill_all()  # fail fast: one rank died, the job cannot complete
            if alive == 0:
                break
            if timeout is not None and time.time() - t0 > timeout:
                rc = rc or 124
                kill_all(signal.SIGKILL)
                break
            time.sleep(0.05)
    except KeyboardInterrupt:
        kill_all(signal.SIGINT)
        rc = 130
    for p in procs:
        try:
            p.wait(timeout=10)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
    return rc


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="start N local mpit ranks")
    ap.add_argument("--nproc", "-n", "-np", type=int, required=True)
    ap.add_argument("--master-port", type=int, default=None)
    ap.add_argument("--timeout", type=float, default=None)
    ap.add_argument("script")
    ap.add_argument("args", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    return launch(a.nproc, [a.script] + a.args, a.master_port, timeout=a.timeout)


if __name__ == "__main__":
    sys.exit(main())
