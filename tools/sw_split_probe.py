#!/usr/bin/env python3
"""Probe: does the C3 SW solver run faster as several launches over column slices than as one?

At C3 every pass of the checkpointed SW solver streams the whole data set (tau, ssa, the two planes, the checkpoints:
~1.05 GB per launch) at 4.8-5.2 TB/s.  The working set of one pass over half the columns (~250 MB) would fit the
256 MB MALL; a slice's passes 2 and 3 could then re-read from it instead of HBM, at the cost of fewer waves per
launch.  This times rrtmgpnn_sw_solver_2stream over the step's own arrays as 1, 2, 3 and 4 launches of contiguous
column slices (same stream, back to back), alternating, and checks the fluxes equal the single launch's bit for bit.

usage: python tools/sw_split_probe.py [--config c3] [--iters 50] [--rounds 5] [--splits 1,2,3,4]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rte-rrtmgp-nn_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3", choices=["c3", "c5"])
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--splits", default="1,2,3,4")
    args = ap.parse_args()
    import torch
    from rrtmgpnn import _lib, data
    from rrtmgpnn._lib import check
    from rrtmgpnn.pipeline import ClearSkyStep
    torch.cuda.set_device(0)
    prob = data.rfmip_problem() if args.config == "c3" else data.synthetic_problem(125000, 137, seed=20251015)
    st = ClearSkyStep(prob, device=0)
    L = _lib.lib()
    c = st.ctx.h
    ncol, nlay, ng = st.ncol, st.nlay, st.ng_sw
    s = st.ctx.stream
    with torch.cuda.stream(s):
        st.step()
        # the boundary conditions the plain solver entry reads (the fused step forms them inside its solver)
        check(L.rrtmgpnn_sw_boundary_rfmip(c, ng, ncol, st.solar_source.data_ptr(), st.tsi.data_ptr(),
                                           st.sfc_alb.data_ptr(), st.sza.data_ptr(), st.toa.data_ptr(),
                                           st.alb.data_ptr(), st.mu0.data_ptr()), "sw_boundary_rfmip")
    torch.cuda.synchronize()
    F = 4

    def launch(c0, n):
        lay = c0 * nlay * ng * F
        g = c0 * ng * F
        lev = c0 * (nlay + 1) * F
        rc = L.rrtmgpnn_sw_solver_2stream(c, ng, nlay, n, st.top_at_1, st.toa.data_ptr() + g, None,
                                          st.tau_sw.data_ptr() + lay, st.ssa_sw.data_ptr() + lay, None,
                                          st.mu0.data_ptr() + c0 * F, st.alb.data_ptr() + g, st.alb.data_ptr() + g,
                                          st.sw_up.data_ptr() + lev, st.sw_dn.data_ptr() + lev,
                                          st.sw_dir.data_ptr() + lev)
        if rc:
            raise RuntimeError(_lib.lib().rrtmgpnn_last_error())

    def run(k):
        b = [round(i * ncol / k) for i in range(k + 1)]
        for i in range(k):
            launch(b[i], b[i + 1] - b[i])

    splits = [int(x) for x in args.splits.split(",")]
    ref = None
    with torch.cuda.stream(s):
        for k in splits:
            for t in (st.sw_up, st.sw_dn, st.sw_dir):
                t.fill_(float("nan"))
            run(k)
            torch.cuda.synchronize()
            f = [t.cpu().numpy().view(np.uint32).copy() for t in (st.sw_up, st.sw_dn, st.sw_dir)]
            if ref is None:
                ref = f
            print(json.dumps({"splits": k, "bitwise_vs_first": all(np.array_equal(a, b) for a, b in zip(ref, f))}),
                  flush=True)
        res = {k: [] for k in splits}
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for k in splits:  # warm
            for _ in range(5):
                run(k)
        for r in range(args.rounds):
            for k in splits:
                torch.cuda.synchronize()
                e0.record(s)
                for _ in range(args.iters):
                    run(k)
                e1.record(s)
                e1.synchronize()
                res[k].append(e0.elapsed_time(e1) / args.iters)
        for k in splits:
            v = res[k]
            print(json.dumps({"config": args.config, "splits": k, "ms_per_solve_median": round(float(np.median(v)), 4),
                              "min": round(min(v), 4), "all": [round(x, 4) for x in v]}), flush=True)
    torch.cuda.synchronize()
    st.close()


if __name__ == "__main__":
    main()
