#!/usr/bin/env python3
"""Publish one profiling run's counter files into profiles/ -- the only writer of profiles/pmc_traffic.json and
profiles/pmc_sq.json (which bench.py reads for its roofline's `traffic`, `valu_busy` and `mfma_busy`).

usage: publish_profiles.py <run_dir> <round> <config> [<config> ...]

<run_dir> is what tools/profile_configs.sh leaves (gpurun_out/ merged back from the GPU box), per config:
<config>/pmc_traffic.txt (tools/pmc_traffic.py's stage table), <config>/pmc_sq.txt and <config>/pmc_mfma.txt
(tools/pmc_counters.py's two passes, merged in that order as profile_configs.sh merges them into pmc_sq.json),
<config>/prof/run_kernel_stats.csv (the bench command's kernel trace), <config>/prof_iso/run_kernel_stats.csv
(--no-overlap) and <config>/bench.json.  (The run-wide pmc_traffic.json / pmc_sq.json are not read: a later box's
merge replaces them.)  For every config given this writes

    profiles/<round>/pmc_traffic_<config>.json, pmc_sq_<config>.json      (that config's counters, as measured)
    profiles/<round>/kernel_stats_<config>.txt, kernel_stats_<config>_iso.txt, bench_<config>_profiled.json

and copies the same counter dictionaries into profiles/pmc_traffic.json / pmc_sq.json under the config, with
"_source": {config: the per-round file}.  tests/test_profiles.py checks that every config entry of the two top-level
files equals the per-round file it names, so a figure quoted from either reproduces from one committed file.
"""
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(ROOT, "profiles")


def _load(path):
    with open(path) as f:
        return json.load(f)


def _dump(obj, path):
    with open(path, "w") as f:
        json.dump(obj, f, indent=1, sort_keys=True)
        f.write("\n")


def main():
    if len(sys.argv) < 4:
        raise SystemExit(__doc__)
    run, rnd, cfgs = sys.argv[1], sys.argv[2], sys.argv[3:]
    out = os.path.join(PROF, rnd)
    os.makedirs(out, exist_ok=True)
    notes = {"pmc_traffic": "per-launch averages from rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes); "
                            "fetch doubled per the gfx950 FETCH_SIZE correction; KiB -> bytes (tools/pmc_traffic.py)",
             "pmc_sq": "per-launch SQ counters (rocprofv3 --pmc, an SQ pass and an MFMA pass) by stage; valu_busy = "
                       "share of the chip's VALU issue slots used (tools/pmc_counters.py)"}
    for kind in ("pmc_traffic", "pmc_sq"):
        top_path = os.path.join(PROF, kind + ".json")
        top = _load(top_path) if os.path.exists(top_path) else {}
        top["_note"] = notes[kind]
        top.pop("_round", None)
        srcs = top.setdefault("_source", {})
        for cfg in cfgs:
            if kind == "pmc_traffic":
                entry = _load(os.path.join(run, cfg, "pmc_traffic.txt"))
            else:
                entry = {}
                for f in ("pmc_sq.txt", "pmc_mfma.txt"):
                    for st, r in _load(os.path.join(run, cfg, f)).items():
                        entry.setdefault(st, {}).update(r)
            rel = os.path.join("profiles", rnd, "%s_%s.json" % (kind, cfg))
            _dump(entry, os.path.join(ROOT, rel))
            top[cfg] = entry
            srcs[cfg] = rel
        _dump(top, top_path)
    summ = os.path.join(ROOT, "tools", "kernel_stats_summary.py")
    for cfg in cfgs:
        for sub, suffix, extra in (("prof", "", ""), ("prof_iso", "_iso", " --no-overlap")):
            csv = os.path.join(run, cfg, sub, "run_kernel_stats.csv")
            if os.path.exists(csv):
                # STEPS: the steps profile_configs.sh ran (its STEPS, default 30)
                cmd = ("rocprofv3 --kernel-trace --stats -- python3 bench.py --config %s --steps %s --warmup 5 "
                       "--no-cpu-baseline --c5-steps 0%s" % (cfg, os.environ.get("STEPS", "30"), extra))
                txt = subprocess.run([sys.executable, summ, csv, cmd], capture_output=True, text=True, check=True).stdout
                with open(os.path.join(out, "kernel_stats_%s%s.txt" % (cfg, suffix)), "w") as f:
                    f.write(txt)
        b = os.path.join(run, cfg, "bench.json")
        if os.path.exists(b):
            shutil.copy(b, os.path.join(out, "bench_%s_profiled.json" % cfg))
    print("published %s into profiles/%s and profiles/pmc_{traffic,sq}.json" % (", ".join(cfgs), rnd))


if __name__ == "__main__":
    main()
