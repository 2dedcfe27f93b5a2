"""Per host thread breakdown of a rocprofv3 --runtime-trace directory: for the last `--loops` seconds' worth of the
trace, the time each thread spends inside each HIP API function, and the device's kernel / copy busy time.

usage: trace_threads.py <rocprofv3 output dir>
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


def main():
    d = sys.argv[1]
    api = rows(d, "*hip_api_trace.csv")
    ker = rows(d, "*kernel_trace.csv")
    cpy = rows(d, "*memory_copy_trace.csv")
    if not api:
        raise SystemExit("no hip_api_trace.csv under " + d)
    t_end = max(int(r["End_Timestamp"]) for r in api)
    # the last half of the trace: the timed block loops (the first loop warms up)
    t0 = min(int(r["Start_Timestamp"]) for r in api)
    lo = t0 + (t_end - t0) // 2
    per = defaultdict(lambda: defaultdict(float))
    for r in api:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if e < lo:
            continue
        per[r["Thread_Id"]][r["Function"]] += (e - max(s, lo)) * 1e-3
    span = (t_end - lo) * 1e-3
    print("window %.1f us" % span)
    for tid, fs in sorted(per.items()):
        tot = sum(fs.values())
        top = sorted(fs.items(), key=lambda kv: -kv[1])[:6]
        print("thread %s: in HIP %.1f us (%.0f%%): %s" % (tid, tot, 100 * tot / span,
                                                        ", ".join("%s %.1f" % kv for kv in top)))

    def busy(rs):
        iv = sorted((max(int(r["Start_Timestamp"]), lo), int(r["End_Timestamp"])) for r in rs
                    if int(r["End_Timestamp"]) > lo)
        tot, cur_s, cur_e = 0, None, None
        for s, e in iv:
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    tot += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        if cur_e is not None:
            tot += cur_e - cur_s
        return tot * 1e-3, len(iv)

    kb, kn = busy(ker)
    cb, cn = busy(cpy)
    print("device: kernels busy %.1f us (%d launches), copies busy %.1f us (%d copies)" % (kb, kn, cb, cn))
    kern = defaultdict(float)
    for r in ker:
        if int(r["End_Timestamp"]) > lo:
            kern[r["Kernel_Name"][:60]] += (int(r["End_Timestamp"]) - max(int(r["Start_Timestamp"]), lo)) * 1e-3
    for k, v in sorted(kern.items(), key=lambda kv: -kv[1])[:8]:
        print("  kernel %-60s %.1f us" % (k, v))


if __name__ == "__main__":
    main()
