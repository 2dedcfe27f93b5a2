#!/usr/bin/env python3
"""Publish one profiling run's counter files into profiles/ -- the only writer of profiles/pmc_traffic.json and
profiles/pmc_sq.json (which bench.py reads for its roofline's `traffic`, `valu_busy` and `mfma_busy`).

usage: publish_profiles.py <run_dir> <round> <config> [<config> ...]

<run_dir> is what tools/profile_configs.sh leaves (gpurun_out/ merged back from the GPU box): pmc_traffic.json and
pmc_sq.json keyed by config, and per config <config>/prof/run_kernel_stats.csv (the bench command's kernel trace),
<config>/prof_iso/run_kernel_stats.csv (--no-overlap) and <config>/bench.json.  For every config given this writes

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
    for kind in ("pmc_traffic", "pmc_sq"):
        src = _load(os.path.join(run, kind + ".json"))
        top_path = os.path.join(PROF, kind + ".json")
        top = _load(top_path) if os.path.exists(top_path) else {}
        top.setdefault("_note", src.get("_note", ""))
        top.pop("_round", None)
        srcs = top.setdefault("_source", {})
        for cfg in cfgs:
            if cfg not in src:
                raise SystemExit("%s: no %r entry in %s" % (kind, cfg, run))
            rel = os.path.join("profiles", rnd, "%s_%s.json" % (kind, cfg))
            _dump(src[cfg], os.path.join(ROOT, rel))
            top[cfg] = src[cfg]
            srcs[cfg] = rel
        _dump(top, top_path)
    summ = os.path.join(ROOT, "tools", "kernel_stats_summary.py")
    for cfg in cfgs:
        for sub, suffix, extra in (("prof", "", ""), ("prof_iso", "_iso", " --no-overlap")):
            csv = os.path.join(run, cfg, sub, "run_kernel_stats.csv")
            if os.path.exists(csv):
                cmd = ("rocprofv3 --kernel-trace --stats -- python3 bench.py --config %s --steps 30 --warmup 5 "
                       "--no-cpu-baseline%s" % (cfg, extra))
                txt = subprocess.run([sys.executable, summ, csv, cmd], capture_output=True, text=True, check=True).stdout
                with open(os.path.join(out, "kernel_stats_%s%s.txt" % (cfg, suffix)), "w") as f:
                    f.write(txt)
        b = os.path.join(run, cfg, "bench.json")
        if os.path.exists(b):
            shutil.copy(b, os.path.join(out, "bench_%s_profiled.json" % cfg))
    print("published %s into profiles/%s and profiles/pmc_{traffic,sq}.json" % (", ".join(cfgs), rnd))


if __name__ == "__main__":
    main()
