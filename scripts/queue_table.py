"""Stream -> hardware-queue table of a rocprofv3 trace (kernel dispatches, and memory copies
when the trace has them): which HIP streams of a rank share a hardware queue.

    python scripts/queue_table.py <trace dir> <out.md> [title] [steady_ms]

rocprofv3 records the queue a dispatch went to (``Queue_Id``) next to the HIP stream it was
launched on (``Stream_Id``). HIP maps streams onto at most GPU_MAX_HW_QUEUES hardware queues
per process; streams that share a queue execute in one FIFO, so an RCCL kernel spinning at
the head of a queue blocks every kernel queued behind it from the other streams of that
queue. The table lists, per (stream, queue) pair, the dispatch count and the most frequent
kernels, and per queue the streams that feed it. ``steady_ms`` (default 300): a second table
restricted to the dispatches that start in the last steady_ms of the trace (the timed steps,
without start-up and the post-run checks), with the host threads that issued them.
"""
from __future__ import annotations

import collections
import csv
import os
import sys


def _rows(d: str, suffix: str):
    for root, _, files in os.walk(d):
        for fn in files:
            if fn.endswith(suffix):
                with open(os.path.join(root, fn)) as f:
                    yield from csv.DictReader(f)


def main(argv) -> int:
    d, out = argv[0], argv[1]
    title = argv[2] if len(argv) > 2 else d
    steady_ms = float(argv[3]) if len(argv) > 3 else 300.0
    pairs = collections.Counter()
    names = collections.defaultdict(collections.Counter)
    busy = collections.Counter()
    rows = list(_rows(d, "kernel_trace.csv"))
    for r in rows:
        key = (r.get("Agent_Id", ""), r["Stream_Id"], r["Queue_Id"])
        pairs[key] += 1
        names[key][r["Kernel_Name"].split("(")[0][:70]] += 1
        busy[key] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    copies = collections.Counter()
    for r in _rows(d, "memory_copy_trace.csv"):
        copies[(r.get("Stream_Id", "?"), r.get("Direction", r.get("Kind", "?")))] += 1
    lines = [f"# Stream -> hardware queue ({title})", "",
             "| agent | stream | queue | dispatches | kernel us | top kernels |", "|---|---|---|---|---|---|"]
    for key in sorted(pairs, key=lambda k: (k[0], int(k[2]) if k[2].isdigit() else 0, k[1])):
        top = ", ".join(f"`{n}` x{c}" for n, c in names[key].most_common(3))
        lines.append(f"| {key[0]} | {key[1]} | {key[2]} | {pairs[key]} | {busy[key] / 1e3:.0f} | {top} |")
    byq = collections.defaultdict(set)
    for a, s, q in pairs:
        byq[(a, q)].add(s)
    lines += ["", "| agent | queue | streams feeding it |", "|---|---|---|"]
    for (a, q), ss in sorted(byq.items()):
        lines.append(f"| {a} | {q} | {', '.join(sorted(ss))} |")
    nq = len({q for _, _, q in pairs})
    lines += ["", f"kernel-dispatching streams: {len({(a, s) for a, s, _ in pairs})}; hardware queues used: {nq}"]
    if rows:
        tend = max(int(r["End_Timestamp"]) for r in rows)
        late = [r for r in rows if tend - int(r["Start_Timestamp"]) < steady_ms * 1e6]
        sp = collections.Counter((r["Stream_Id"], r["Queue_Id"]) for r in late)
        thr = collections.defaultdict(set)
        for r in late:
            thr[(r["Stream_Id"], r["Queue_Id"])].add(r.get("Thread_Id", "?"))
        lines += ["", f"## Last {steady_ms:.0f} ms of the trace (steady steps)", "",
                  "| stream | queue | dispatches | host threads |", "|---|---|---|---|"]
        for (s_, q), c in sorted(sp.items(), key=lambda kv: -kv[1]):
            lines.append(f"| {s_} | {q} | {c} | {', '.join(sorted(thr[(s_, q)]))} |")
        lines += ["", f"streams dispatching in the window: {len({s_ for s_, _ in sp})}; "
                  f"hardware queues: {len({q for _, q in sp})}"]
    if copies:
        lines += ["", "| copy stream | direction | copies |", "|---|---|---|"]
        for (s, k), c in sorted(copies.items()):
            lines.append(f"| {s} | {k} | {c} |")
    with open(out, "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
