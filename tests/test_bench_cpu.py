"""bench.py's multi-rank path on CPU (gloo): the headline line, the post-run PS
consistency check and the N>1 secondary fields (dedicated topology, PS ping-pong,
Allreduce) — what the 8-GPU driver run relies on, rehearsed with small shapes."""
import json
import os
import subprocess
import sys

from mp_util import ROOT, free_port


def test_bench_three_ranks_cpu():
    e = dict(os.environ, MPIT_CPU_ONLY="1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    e["PYTHONPATH"] = ROOT + os.pathsep + e.get("PYTHONPATH", "")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=3",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.join(ROOT, "bench.py"), "--gpus", "3",
           "--model", "cnn7", "--batch", "8", "--steps", "2", "--warmup", "1"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=400, env=e, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 3 and out["world"] == 3 and out["dtype"] == "fp32"
    assert out["value"] > 0 and out["config"]["parallelism"] == "async-ps-colocated-3srv-3wrk"
    assert out["ps_check"]["ok"] and out["ps_check"]["workers"] == 3
    sec = out["secondary"]
    assert "error" not in sec, sec
    assert sec["dedicated"]["parallelism"] == "async-ps-dedicated-1srv-2wrk" and sec["dedicated"]["ps_check"]["ok"]
    assert sec["ps_pingpong"]["clients"] == 2 and sec["ps_pingpong"]["aggregate_GBps_bidir"] > 0
    assert sec["allreduce"]["correct"] and sec["allreduce"]["MiB"] == 40.0


def test_bench_preflight_falls_back_to_datapath3_cpu():
    """A broken one-sided (worker, server) path (injected: server 1's pulls to worker 2 arrive
    corrupted) is caught by the pre-timing check; the job switches to the two-sided data plane
    (datapath 3) and runs, reporting why."""
    e = dict(os.environ, MPIT_CPU_ONLY="1", HSA_ENABLE_IPC_MODE_LEGACY="0", MPIT_PS_FAULT="badpull",
             MPIT_PS_FAULT_RANK="1", MPIT_PS_FAULT_CLIENT="2")
    e["PYTHONPATH"] = ROOT + os.pathsep + e.get("PYTHONPATH", "")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=3",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.join(ROOT, "bench.py"), "--gpus", "3",
           "--model", "cnn7", "--batch", "8", "--steps", "2", "--warmup", "1", "--no-secondary"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=400, env=e, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert out["config"]["datapath"] == 3 and out["ps_check"]["ok"], out
    fb = out["preflight"]["fallback"]
    assert fb["from_datapath"] == 2 and "[2, 1]" in fb["reason"], fb


def test_bench_no_peer_access_falls_back_to_datapath3_cpu():
    """A (worker, server) pair without peer access fails the one-sided pre-flight; datapath 3
    maps no peer memory, so its pre-flight passes although the pair is still reported, and
    the job runs there (it used to exit 3 before timing on such a node)."""
    e = dict(os.environ, MPIT_CPU_ONLY="1", HSA_ENABLE_IPC_MODE_LEGACY="0", MPIT_PREFLIGHT_NO_PEER="2:1")
    e["PYTHONPATH"] = ROOT + os.pathsep + e.get("PYTHONPATH", "")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=3",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.join(ROOT, "bench.py"), "--gpus", "3",
           "--model", "cnn7", "--batch", "8", "--steps", "2", "--warmup", "1", "--no-secondary"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=400, env=e, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    pf = out["preflight"]
    assert out["config"]["datapath"] == 3 and pf["ok"] and pf["no_peer"] == [[2, 1]], pf
    assert pf["fallback"]["from_datapath"] == 2 and "unverified" in pf["fallback"], pf
    # opting out ends the run before timing, with the pair named
    r = subprocess.run(cmd[:5] + [f"--master-port={free_port()}"] + cmd[6:] + ["--no-rccl-fallback"],
                       capture_output=True, text=True, timeout=400, env=e, cwd=ROOT)
    assert r.returncode != 0 and "[[2, 1]]" in r.stderr, r.stderr[-2000:]
