"""Probe: host time at the Downpour step boundary (N=1). The trace shows the GPU idle between
the server's apply kernel and the next step's weight cast; this times, on the host, the chain
in between: the PS reply wake-up (pc.wait return), the end of step(), the start of the next
step(), the cast launch (wrappers around PClient.wait and WeightCastPlan.run) and the
stem's forward pieces up to its first GEMM.

    python benchmarks/boundary_probe.py [bf16|fp32] [steps]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def main():
    dt = sys.argv[1] if len(sys.argv) > 1 else "bf16"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    import mpit_amd as mp
    from mpit_amd.train import TrainConfig, Trainer

    mp.Init()
    tr = Trainer(TrainConfig(model="resnet50", batch=256, amp=dt == "bf16"))
    marks = []
    pc = tr.pc
    wait0 = pc.wait

    import resource

    flt = []

    def _minflt():
        return resource.getrusage(getattr(resource, "RUSAGE_THREAD", resource.RUSAGE_SELF)).ru_minflt

    def wait():
        t0 = time.perf_counter()
        wait0()
        marks.append(("wait_in", t0))
        marks.append(("wait_out", time.perf_counter()))
        flt.append(["w", _minflt()])
    pc.wait = wait
    run0 = tr.wcast.run

    def run():
        flt.append(["c", _minflt()])
        marks.append(("cast_call", time.perf_counter()))
        run0()
        marks.append(("cast_done", time.perf_counter()))
    tr.wcast.run = run
    from mpit_amd.ops import conv as C

    fwd0, get0, swp0 = C._StemConvFn.forward, C._StemPackBuf.get.__func__, C.stem_weight_planes

    def fwd(ctx, *a, **k):
        marks.append(("stem_fwd", time.perf_counter()))
        r = fwd0(ctx, *a, **k)
        marks.append(("stem_fwd_done", time.perf_counter()))
        return r

    def get(cls, *a, **k):
        r = get0(cls, *a, **k)
        marks.append(("stem_pack_done", time.perf_counter()))
        return r

    def swp(*a, **k):
        marks.append(("stem_planes", time.perf_counter()))
        return swp0(*a, **k)
    ts0, am0 = C._tile_stats, C.amax_of

    def ts(*a, **k):
        marks.append(("tile_stats", time.perf_counter()))
        r = ts0(*a, **k)
        marks.append(("tile_stats_done", time.perf_counter()))
        return r

    def am(*a, **k):
        marks.append(("amax_of", time.perf_counter()))
        return am0(*a, **k)
    C._tile_stats, C.amax_of = ts, am
    import mpit_amd.train as T
    from mpit_amd.optim import distributed as D

    step0, dp0 = tr._step, D.downpour

    def step_in():
        marks.append(("_step", time.perf_counter()))
        return step0()
    tr._step = step_in

    def dp(*a, **k):
        marks.append(("downpour", time.perf_counter()))
        return dp0(*a, **k)
    D.downpour = dp
    T.dopt.downpour = dp
    armcpu = []
    pusher = tr.opt_config.get("pusher") if getattr(tr, "opt_config", None) else None
    if pusher is not None:
        arm0 = pusher.arm

        def arm(*a, **k):
            c0 = time.thread_time()
            marks.append(("arm", time.perf_counter()))
            r = arm0(*a, **k)
            marks.append(("arm_done", time.perf_counter()))
            armcpu.append([(time.thread_time() - c0) * 1e6])
            return r
        pusher.arm = arm
    fe0 = tr._feval

    def fe(w):
        marks.append(("feval", time.perf_counter()))
        return fe0(w)
    tr._feval = fe
    C._StemConvFn.forward = staticmethod(fwd)
    C._StemPackBuf.get = classmethod(get)
    C.stem_weight_planes = swp
    for _ in range(5):
        tr.step()
    torch.cuda.synchronize()
    from mpit_amd.train import gc_settle

    gc_settle()  # as bench.py's timed region
    import gc

    gcs, gct = [], {}

    def gcb(phase, info):
        if phase == "start":
            gct["t"] = time.perf_counter()
        else:
            gcs.append((info.get("generation"), (time.perf_counter() - gct.get("t", time.perf_counter())) * 1e6))
    gc.callbacks.append(gcb)
    if os.environ.get("PROBE_GC_OFF") == "1":
        gc.disable()
    marks.clear()
    ms0 = torch.cuda.memory_stats()
    for _ in range(steps):
        marks.append(("step_call", time.perf_counter()))
        tr.step()
        marks.append(("step_ret", time.perf_counter()))
    torch.cuda.synchronize()
    # per boundary: wait_out -> step_ret -> step_call -> cast_call -> cast_done
    seq = [n for n, _ in marks]
    t = [x for _, x in marks]
    out = {"wait_blocked_us": [], "wait_out_to_step_ret_us": [], "step_ret_to_next_cast_us": [], "cast_launch_us": []}
    for i, n in enumerate(seq):
        if n == "wait_out":
            out["wait_blocked_us"].append((t[i] - t[i - 1]) * 1e6)
            j = seq.index("step_ret", i)
            out["wait_out_to_step_ret_us"].append((t[j] - t[i]) * 1e6)
            if "cast_call" in seq[j:]:
                k = seq.index("cast_call", j)
                out["step_ret_to_next_cast_us"].append((t[k] - t[j]) * 1e6)
        if n == "step_call":
            for a, b in (("step_call", "_step"), ("_step", "downpour"), ("downpour", "arm"), ("arm", "arm_done"),
                         ("arm_done", "feval"), ("feval", "cast_call")):
                if a in seq[i:] and b in seq[i:]:
                    ia = seq.index(a, i)
                    ib = seq.index(b, ia)
                    out.setdefault(f"{a}->{b}_us", []).append((t[ib] - t[ia]) * 1e6)
        if n == "cast_call":
            out["cast_launch_us"].append((t[i + 1] - t[i]) * 1e6)
            for a, b in (("cast_done", "stem_fwd"), ("stem_fwd", "stem_pack_done"), ("stem_pack_done", "stem_planes"),
                         ("stem_pack_done", "tile_stats"), ("tile_stats", "tile_stats_done"),
                         ("tile_stats_done", "amax_of"), ("amax_of", "stem_planes"), ("stem_planes", "stem_fwd_done")):
                if a in seq[i:] and b in seq[i:]:
                    ia = seq.index(a, i)
                    ib = seq.index(b, ia)
                    out.setdefault(f"{a}->{b}_us", []).append((t[ib] - t[ia]) * 1e6)
    summ = {k: round(sorted(v)[len(v) // 2], 1) for k, v in out.items() if v}
    ms1 = torch.cuda.memory_stats()
    alloc = {k: ms1.get(k, 0) - ms0.get(k, 0) for k in ("num_device_alloc", "num_device_free", "num_alloc_retries",
                                                         "num_sync_all_streams")}
    gc.callbacks.remove(gcb)
    gcsum = {}
    for g, us in gcs:
        c = gcsum.setdefault(f"gen{g}", [0, 0.0])
        c[0] += 1
        c[1] += us
    d = [b[1] - a[1] for a, b in zip(flt, flt[1:]) if a[0] == "w" and b[0] == "c"]
    if d:
        print(json.dumps({"minor_faults_wait_out_to_cast_median": sorted(d)[len(d) // 2], "max": max(d)}), flush=True)
    if armcpu:
        cols = list(zip(*armcpu))
        print(json.dumps({"arm_line_cpu_us_median": [round(sorted(c)[len(c) // 2], 1) for c in cols],
                          "arm_line_cpu_us_max": [round(max(c), 1) for c in cols]}), flush=True)
    print(json.dumps({"gc_per_step": {k: [round(v[0] / steps, 2), round(v[1] / steps, 1)] for k, v in gcsum.items()}}),
          flush=True)
    print(json.dumps({"dtype": dt, "median_us": summ, "allocator_deltas_over_steps": alloc, "steps": steps,
                      "alloc_conf": os.environ.get("PYTORCH_HIP_ALLOC_CONF") or os.environ.get("PYTORCH_CUDA_ALLOC_CONF")}),
          flush=True)
    tr.stop()
    mp.Finalize()


if __name__ == "__main__":
    main()
