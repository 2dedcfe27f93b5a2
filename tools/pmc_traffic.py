#!/usr/bin/env python3
"""Per-launch HBM traffic of each pipeline stage from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE).

usage: pmc_traffic.py <fetch_dir> <write_dir> <config> [out.json]

Both passes are separate runs (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass on gfx950).  Units and
corrections follow /opt/skills/guides/MI355X_MICROARCH.md (HBM section): the counters are in KiB;
FETCH_SIZE on gfx950 reports half the bytes of wide coalesced reads, so it is doubled; WRITE_SIZE is
taken as is.  Averages are over every dispatch of the kernel in the pass.
"""
import csv
import glob
import json
import os
import re
import sys

STAGES = [
    (re.compile(r"sw_2stream(?:_x2|_ck)?_kernel"), "sw_solver"),
    (re.compile(r"lw_noscat_kernel"), "lw_solver"),
    # mlp_pair_kernel<AK, AH1, AH2, BK, BH1, BH2, MODE, ACTS>: MODE 1 LW pair, 4 LW "both", 2 SW pair
    (re.compile(r"mlp_pair_kernel<(?:\s*\d+\s*,){6}\s*[14]\s*,"), "predict_nn_lw"),
    (re.compile(r"mlp_pair_kernel<(?:\s*\d+\s*,){6}\s*2\s*,"), "predict_nn_sw"),
    # mlp32_kernel<KS, AH1, AN2, AH2, AN3, BH1, BN2, BH2, BN3, NGT, MODE, XIN>: MODE 1 LW pair, 4 LW "both", 2 SW pair
    (re.compile(r"mlp32_kernel<(?:\s*\d+\s*,){10}\s*[14]\s*,"), "predict_nn_lw"),
    (re.compile(r"mlp32_kernel<(?:\s*\d+\s*,){10}\s*2\s*,"), "predict_nn_sw"),
    (re.compile(r"cloud_optics_kernel"), "cloud_optics"),
    (re.compile(r"increment_bybnd_kernel"), "increment"),
    (re.compile(r"delta_scale_kernel"), "delta_scale_sw"),
    (re.compile(r"planck_source_kernel"), "planck_source"),
    (re.compile(r"nn_inputs_kernel"), "nn_inputs"),
    (re.compile(r"expand_kernel"), "expand_emis"),
    (re.compile(r"col_dry_kernel"), "get_col_dry"),
    (re.compile(r"sw_boundary_kernel"), "sw_boundary"),
]


def stage_of(kernel):
    for rx, name in STAGES:
        if rx.search(kernel):
            return name
    return None


def read_pass(d, counter):
    acc = {}
    files = glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True)
    if not files:
        raise SystemExit("no counter_collection csv under %s" % d)
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                st = stage_of(row.get("Kernel_Name", ""))
                if st is None:
                    continue
                s, n = acc.get(st, (0.0, 0))
                acc[st] = (s + float(row["Counter_Value"]), n + 1)
    return {k: s / n for k, (s, n) in acc.items()}


def main():
    fetch_dir, write_dir, config = sys.argv[1:4]
    out = sys.argv[4] if len(sys.argv) > 4 else os.path.join(os.path.dirname(__file__), "..", "profiles",
                                                             "pmc_traffic.json")
    fetch = read_pass(fetch_dir, "FETCH_SIZE")
    write = read_pass(write_dir, "WRITE_SIZE")
    res = {}
    for st in sorted(set(fetch) | set(write)):
        fb = 2.0 * 1024.0 * fetch.get(st, 0.0)
        wb = 1024.0 * write.get(st, 0.0)
        res[st] = {"fetch_bytes": round(fb), "write_bytes": round(wb), "hbm_bytes": round(fb + wb),
                   "fetch_size_kib_raw": round(fetch.get(st, 0.0), 1), "write_size_kib_raw": round(write.get(st, 0.0), 1)}
    try:
        with open(out) as fh:
            allres = json.load(fh)
    except (OSError, ValueError):
        allres = {}
    allres[config] = res
    allres["_note"] = ("per-launch averages from rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes); "
                       "fetch doubled per the gfx950 FETCH_SIZE correction; KiB -> bytes")
    with open(out, "w") as fh:
        json.dump(allres, fh, indent=1, sort_keys=True)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
