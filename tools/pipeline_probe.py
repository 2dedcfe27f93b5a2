#!/usr/bin/env python3
"""Probe: do consecutive column blocks overlap across steps?  (Round 6: the C3 step's timeline has the SW network
alone for its first ~50 us and the LW solver alone for its last ~100 us; a block loop whose next block's SW chain
starts when this block's SW solver ends -- not when its LW solver ends -- fills those phases.)

Modes, each K steps timed after warm-up, alternating over --reps rounds on one box:
  graph      the benchmarked step (ClearSkyStep.replay: one hipGraph, chains forked and joined per step)
  eager      the same launches issued eagerly, forked and joined per step (launch-cost reference for the next two)
  pipe       eager, no per-step join: SW chain on its stream, LW chain on its stream gated on the same step's SW
             network (as in the step), step k+1's SW chain waits only for step k's SW chain (stream order)
  pipe_free  as pipe without the gate (each chain only after its own previous step)
Every mode computes the same fluxes (the probe checks them bit for bit against the graph's)."""
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
    ap.add_argument("--config", default="c3", choices=["c3", "c4", "c5"])
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--modes", default="graph,eager,pipe,pipe_free")
    args = ap.parse_args()
    import torch
    from rrtmgpnn import data
    from rrtmgpnn.pipeline import ClearSkyStep
    dev = torch.device("cuda", 0)
    if args.config == "c3":
        prob, clouds = data.rfmip_columns(0, 1800), None
    else:
        n, nl = (10000, 60) if args.config == "c4" else (125000, 137)
        prob = data.synthetic_problem(n, nl, seed=20251015, col0=0)
        clouds = data.allsky_clouds(prob, data.load_cloud_optics("lw")) if args.config == "c4" else None
    st = ClearSkyStep(prob, device=0, clouds=clouds)
    st.capture()
    torch.cuda.set_stream(st.ctx.stream)
    A, B = st.ctx.stream, st.ctx2.stream
    swn = ("sw_boundary", "cloud_optics_sw", "delta_scale_sw", "predict_nn_sw", "sw_solver")
    lw = [(n, f, a) for n, f, a in st.calls if n not in swn]
    # a separate SW boundary kernel (trees before the fused SW solver entry) goes at the head of the SW stream, so the
    # pipelined SW chain depends on nothing of the LW stream; the fused step forms them inside its SW solver
    sw = [(n, f, ((st.ctx2.h,) + tuple(a[1:])) if n == "sw_boundary" else a) for n, f, a in st.calls if n in swn]
    gate_after = "predict_nn_sw"
    evs = [torch.cuda.Event() for _ in range(4)]

    def issue(calls):
        for n, f, a in calls:
            rc = f(*a)
            if rc:
                raise RuntimeError(n)

    def pipe_step(k, gated):
        for n, f, a in sw:  # SW chain on B
            if f(*a):
                raise RuntimeError(n)
            if n == gate_after and gated:
                evs[k % 4].record(B)
                A.wait_event(evs[k % 4])
        issue(lw)  # LW chain on A

    def run(mode, K):
        if mode == "graph":
            for _ in range(K):
                st.replay()
        elif mode == "eager":
            for _ in range(K):
                st.step()
        elif mode in ("pipe", "pipe_free"):
            B.wait_stream(A)
            for k in range(K):
                pipe_step(k, mode == "pipe")
            A.wait_stream(B)

    modes = args.modes.split(",")
    res = {m: [] for m in modes}
    ref = None
    for m in modes:  # warm + correctness
        for t in (st.lw_up, st.lw_dn, st.sw_up, st.sw_dn, st.sw_dir):
            t.fill_(float("nan"))
        run(m, 20)
        torch.cuda.synchronize()
        f = st.fluxes()
        if ref is None:
            ref = f
        same = all(np.array_equal(ref[k].view(np.uint32), f[k].view(np.uint32)) for k in ref)
        print(json.dumps({"mode": m, "bitwise_vs_first": same}), flush=True)
    t_settle = time.perf_counter()
    while time.perf_counter() - t_settle < 1.0:
        run("graph", 20)
        torch.cuda.synchronize()
    for rep in range(args.reps):
        for m in modes:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            run(m, args.steps)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / args.steps * 1e3
            res[m].append(ms)
            print(json.dumps({"config": args.config, "rep": rep, "mode": m, "ms_per_step": round(ms, 4),
                              "columns_per_s": round(st.ncol / ms * 1e3, 1)}), flush=True)
    print(json.dumps({"config": args.config, "summary": {m: {"median": round(float(np.median(v)), 4),
                                                              "min": round(min(v), 4)} for m, v in res.items()}}))
    torch.cuda.set_stream(torch.cuda.default_stream(dev))
    st.close()


if __name__ == "__main__":
    main()
