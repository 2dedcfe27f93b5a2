#!/usr/bin/env python3
"""Probe: what does the graph boundary cost per step?  The C3 trace (profiles/r06/timeline_c3_base.txt) shows ~21 us
between the last kernel of one replay and the first of the next.  This captures N consecutive steps -- each with its
own fork and join, exactly the step's launches -- into one hipGraph and times replays of it against replays of the
one-step graph, alternating on one box; ms per step = time / (replays x N).  Fluxes are checked bit for bit.

usage: python tools/graph_batch_probe.py [--config c3] [--batches 1,2,4] [--steps 200] [--reps 3]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rte-rrtmgp-nn_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3", choices=["c3", "c4"])
    ap.add_argument("--batches", default="1,2,4")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import torch
    from rrtmgpnn import data
    from rrtmgpnn.pipeline import ClearSkyStep
    torch.cuda.set_device(0)
    if args.config == "c3":
        prob, clouds = data.rfmip_columns(0, 1800), None
    else:
        prob = data.synthetic_problem(10000, 60, seed=20251015, col0=0)
        clouds = data.allsky_clouds(prob, data.load_cloud_optics("lw"))
    st = ClearSkyStep(prob, device=0, clouds=clouds)
    st.capture()
    graphs = {}
    for n in (int(x) for x in args.batches.split(",")):
        if n == 1:
            graphs[1] = st.graph
            continue
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=st.ctx.stream):
            for _ in range(n):
                st._issue()
        graphs[n] = g
    s = st.ctx.stream

    def run(n, steps):
        reps = max(1, steps // n)
        with torch.cuda.stream(s):
            for _ in range(reps):
                graphs[n].replay()
        return reps * n

    ref = None
    for n in graphs:
        for t in (st.lw_up, st.lw_dn, st.sw_up, st.sw_dn, st.sw_dir):
            t.fill_(float("nan"))
        torch.cuda.synchronize()
        run(n, n)
        torch.cuda.synchronize()
        f = st.fluxes()
        if ref is None:
            ref = f
        same = all(np.array_equal(ref[k].view(np.uint32), f[k].view(np.uint32)) for k in ref)
        print(json.dumps({"batch": n, "bitwise_vs_first": same}), flush=True)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 1.0:  # settle the clocks
        run(1, 50)
        torch.cuda.synchronize()
    res = {n: [] for n in graphs}
    for rep in range(args.reps):
        for n in graphs:
            torch.cuda.synchronize()
            t = time.perf_counter()
            done = run(n, args.steps)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t) / done * 1e3
            res[n].append(ms)
            print(json.dumps({"config": args.config, "rep": rep, "batch": n, "ms_per_step": round(ms, 4)}), flush=True)
    print(json.dumps({"config": args.config, "summary": {n: {"median": round(float(np.median(v)), 4),
                                                              "min": round(min(v), 4)} for n, v in res.items()}}))
    for n, g in graphs.items():
        if n != 1:
            g.reset()
    st.close()


if __name__ == "__main__":
    main()
