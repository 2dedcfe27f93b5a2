#!/usr/bin/env python3
"""Per-stage averages of every PMC counter in a rocprofv3 --pmc output directory (stage names as pmc_traffic.py).

usage: pmc_counters.py <pmc_dir> [out.json [config]]   (with a config, merged into out.json under that key)
SQ_* cycle counters are in quad-cycles (MI355X_MICROARCH.md, per-instruction table); the derived fractions printed
are WAIT_ANY / WAVE_CYCLES (parked on s_waitcnt), WAIT_INST_ANY / WAVE_CYCLES (issue stalls) and
ACTIVE_INST_VALU / WAVE_CYCLES,
and VALU instructions per wave.

valu_busy = SQ_ACTIVE_INST_VALU * 4 / (kernel cycles * 1024 SIMDs): the fraction of the chip's VALU issue slots
used (one wave64 VALU instruction occupies its SIMD for at least a quad-cycle).  Kernel cycles = SQ_BUSY_CYCLES / 32:
the counter is summed over MI355X's 32 shader engines (8 XCDs x 4); the quotient matches every kernel's measured
duration at 2.1-2.4 GHz.
"""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import stage_of  # noqa: E402


N_SE, N_SIMD = 32, 1024  # MI355X: 8 XCDs x 4 shader engines; 256 CUs x 4 SIMDs


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
        if r.get("SQ_ACTIVE_INST_VALU") and r.get("SQ_BUSY_CYCLES"):
            r["valu_busy"] = round(4.0 * r["SQ_ACTIVE_INST_VALU"] / (r["SQ_BUSY_CYCLES"] / N_SE * N_SIMD), 4)
        if r.get("SQ_INSTS_VALU") and r.get("SQ_WAVES"):
            r["valu_insts_per_wave"] = round(r["SQ_INSTS_VALU"] / r["SQ_WAVES"], 1)
        # MFMA pass: MOPS count multiply-adds / 512 per the counter description, so flops = MOPS * 512;
        # SQ_VALU_MFMA_BUSY_CYCLES sums the matrix pipes' busy cycles over all SIMDs (MI355X_MICROARCH.md), so its
        # share of (kernel cycles x 1024 SIMDs) is the chip's matrix-core utilisation
        if r.get("SQ_INSTS_VALU_MFMA_MOPS_F32") is not None:
            r["mfma_flop"] = r["SQ_INSTS_VALU_MFMA_MOPS_F32"] * 512.0
        if r.get("SQ_VALU_MFMA_BUSY_CYCLES") is not None and r.get("SQ_BUSY_CYCLES"):
            r["mfma_busy"] = round(r["SQ_VALU_MFMA_BUSY_CYCLES"] / (r["SQ_BUSY_CYCLES"] / N_SE * N_SIMD), 4)
            if r.get("SQ_INSTS_MFMA"):
                r["mfma_busy_cycles_per_inst"] = round(r["SQ_VALU_MFMA_BUSY_CYCLES"] / r["SQ_INSTS_MFMA"], 2)
    txt = json.dumps(res, indent=1, sort_keys=True)
    print(txt)
    if len(sys.argv) > 3:
        try:
            with open(sys.argv[2]) as fh:
                allres = json.load(fh)
        except (OSError, ValueError):
            allres = {}
        cfg = allres.setdefault(sys.argv[3], {})
        for st, r in res.items():  # merge: passes of different counter sets add to the same stage entry
            cfg.setdefault(st, {}).update(r)
        allres["_note"] = ("per-launch SQ counters (rocprofv3 --pmc, one pass) by stage; valu_busy = share of the chip's "
                           "VALU issue slots used (tools/pmc_counters.py)")
        with open(sys.argv[2], "w") as fh:
            json.dump(allres, fh, indent=1, sort_keys=True)
    elif len(sys.argv) > 2:
        with open(sys.argv[2], "w") as fh:
            fh.write(txt)


if __name__ == "__main__":
    main()
