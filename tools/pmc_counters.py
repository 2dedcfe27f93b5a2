#!/usr/bin/env python3
"""Per-stage averages of every PMC counter in a rocprofv3 --pmc output directory (stage names as pmc_traffic.py).

usage: pmc_counters.py <pmc_dir> [out.json]
SQ_* cycle counters are in quad-cycles (MI355X_MICROARCH.md, per-instruction table); the derived fractions printed
are WAIT_ANY / WAVE_CYCLES (parked on s_waitcnt), WAIT_INST_ANY / WAVE_CYCLES (issue stalls) and
ACTIVE_INST_VALU / WAVE_CYCLES,
and VALU instructions per wave.
"""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import stage_of  # noqa: E402


def main():
    d = sys.argv[1]
    acc = {}
    files = glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True)
    if not files:
        raise SystemExit("no counter_collection csv under %s" % d)
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                st = stage_of(row.get("Kernel_Name", ""))
                if st is None:
                    continue
                key = (st, row["Counter_Name"])
                s, n = acc.get(key, (0.0, 0))
                acc[key] = (s + float(row["Counter_Value"]), n + 1)
    res = {}
    for (st, c), (s, n) in sorted(acc.items()):
        res.setdefault(st, {})[c] = s / n
    for st, r in res.items():
        wc = r.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
                if c in r:
                    r["frac_" + c[3:].lower()] = round(r[c] / wc, 4)
        if r.get("SQ_INSTS_VALU") and r.get("SQ_WAVES"):
            r["valu_insts_per_wave"] = round(r["SQ_INSTS_VALU"] / r["SQ_WAVES"], 1)
    txt = json.dumps(res, indent=1, sort_keys=True)
    print(txt)
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as fh:
            fh.write(txt)


if __name__ == "__main__":
    main()
