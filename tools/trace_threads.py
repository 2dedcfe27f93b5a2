"""Per host thread breakdown of the steady-state block loops in a rocprofv3 --runtime-trace directory of the Fortran
drop-in (tools/gpu_fortran_prof.sh): the window is the `nloops` loops of `loop_ms` each that end with the last SW
solver kernel; for every thread, the time inside each HIP API function and outside HIP (host work: the staging
memcpys, the Fortran code), and the device's kernel and copy busy time in the window.

usage: trace_threads.py <rocprofv3 output dir> <loop_ms> [nloops=10]
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def rows(d, pat):
    out = []
    for f in glob.glob(os.path.join(d, "**", pat), recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def busy(iv):
    tot, cs, ce = 0, None, None
    for s, e in sorted(iv):
        if ce is None or s > ce:
            if ce is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    return tot + (ce - cs if ce is not None else 0)


def main():
    d, loop_ms = sys.argv[1], float(sys.argv[2])
    nloops = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    api, ker, cpy = rows(d, "*hip_api_trace.csv"), rows(d, "*kernel_trace.csv"), rows(d, "*memory_copy_trace.csv")
    hi = max(int(r["End_Timestamp"]) for r in ker if "sw_2stream" in r["Kernel_Name"])
    lo = hi - int(nloops * loop_ms * 1e6)
    span = (hi - lo) / 1e3
    print("window: last %d loops, %.1f us (%.1f us per loop)" % (nloops, span, span / nloops))
    per = defaultdict(lambda: defaultdict(float))
    for r in api:
        s, e = max(int(r["Start_Timestamp"]), lo), min(int(r["End_Timestamp"]), hi)
        if e > s:
            per[r["Thread_Id"]][r["Function"]] += (e - s) / 1e3
    for tid, fs in sorted(per.items()):
        tot = sum(fs.values())
        top = sorted(fs.items(), key=lambda kv: -kv[1])[:5]
        print("thread %s per loop: host (outside HIP) %.1f us, in HIP %.1f us: %s" % (
            tid, (span - tot) / nloops, tot / nloops, ", ".join("%s %.1f" % (k, v / nloops) for k, v in top)))
    clip = lambda rs: [(max(int(r["Start_Timestamp"]), lo), min(int(r["End_Timestamp"]), hi)) for r in rs
                       if int(r["End_Timestamp"]) > lo and int(r["Start_Timestamp"]) < hi]
    print("device per loop: kernels busy %.1f us, copies busy %.1f us, either %.1f us" % (
        busy(clip(ker)) / 1e3 / nloops, busy(clip(cpy)) / 1e3 / nloops, busy(clip(ker) + clip(cpy)) / 1e3 / nloops))


if __name__ == "__main__":
    main()
