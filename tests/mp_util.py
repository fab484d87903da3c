import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run_ranks(script: str, n: int, env=None, timeout=240) -> str:
    """Run tests/mp/<script> on n ranks with torch.distributed.run; return stdout."""
    e = dict(os.environ)
    e.update(env or {})
    e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    e["PYTHONPATH"] = ROOT + os.pathsep + e.get("PYTHONPATH", "")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.join(ROOT, "tests", "mp", script)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=e, cwd=ROOT)
    if r.returncode != 0:
        raise AssertionError(f"{script} x{n} failed ({r.returncode}):\n{r.stdout[-4000:]}\n{r.stderr[-6000:]}")
    return r.stdout
