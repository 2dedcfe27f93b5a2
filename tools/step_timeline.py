#!/usr/bin/env python3
"""Per-step kernel timeline from a rocprofv3 --kernel-trace CSV of `bench.py` (the overlapped hipGraph replays).

usage: step_timeline.py <run_kernel_trace.csv> [--steps N] [--at F]

Takes N consecutive steps at fraction F of the run (default 20 at 0.5: inside the settle phase's graph replays,
away from the eager stage-timing steps at the end; a step starts at each launch of its first kernel: among the
kernels launched once per step, the one the last step starts with), and prints for each kernel its mean start and end relative to the step's start, in microseconds, and
the mean step length (start to start).  Shows where a chain waits: a kernel whose start lies well after the end of
the kernel feeding it waited for CUs.
"""
import csv
import sys
from collections import defaultdict


def short(name):
    n = name.split("(")[0].replace("void ", "").replace("rrtmgpnn::", "")
    if n.startswith("mlp32_kernel<"):  # the two networks: LW (9 K-steps of inputs) and SW
        return "mlp32_kernel LW" if n.startswith("mlp32_kernel<9,") else "mlp32_kernel SW"
    return n.split("<")[0]


def main():
    path = sys.argv[1]
    last = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 20
    at = float(sys.argv[sys.argv.index("--at") + 1]) if "--at" in sys.argv else 0.5
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if "copyBuffer" in r["Kernel_Name"] or "at::native" in r["Kernel_Name"]:
                continue
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                         r["Kernel_Name"]))
    rows.sort()
    counts = defaultdict(int)
    for _, _, _, full in rows:
        counts[full] += 1
    nstep = min(v for v in counts.values() if v >= 10)  # launched once per step (cloud optics runs twice)
    kernels = [k for k, v in counts.items() if v == nstep]
    # the step's first kernel: among the kernels launched once per step, the one the last step starts with
    firsts = {k: [s for s, _, _, f in rows if f == k] for k in kernels}
    head = min(kernels, key=lambda k: firsts[k][-1])
    i0 = min(int(at * len(firsts[head])), len(firsts[head]) - last - 1)
    starts = firsts[head][i0:i0 + last + 1]
    per = defaultdict(list)
    for i in range(len(starts) - 1):
        t0, t1 = starts[i], starts[i + 1]
        for s, e, n, f in rows:
            if t0 <= s < t1:
                per[(f, n)].append(((s - t0) / 1e3, (e - t0) / 1e3))
    step = sum(b - a for a, b in zip(starts[:-1], starts[1:])) / (len(starts) - 1) / 1e3
    print("mean step %.1f us over %d steps (head: %s)" % (step, len(starts) - 1, short(head)))
    print("%-28s %8s %8s %8s" % ("kernel", "start", "end", "span"))
    for (f, n), v in sorted(per.items(), key=lambda kv: sum(a for a, _ in kv[1]) / len(kv[1])):
        s = sum(a for a, _ in v) / len(v)
        e = sum(b for _, b in v) / len(v)
        print("%-28s %8.1f %8.1f %8.1f" % (n[:28], s, e, e - s))


if __name__ == "__main__":
    main()
