"""One stage of the benchmarked step, timed alone across library builds, with its outputs compared bit for bit.

    python tools/kernel_ab.py --config c3 --stage sw_solver variants/a.so variants/b.so ...

The step (bench.py's problem for the config) is built and run once with the default library; then, alternating
between the default and every variant for --rounds rounds, the stage's C call is issued --iters times on the
variant's own context (HIP events around the batch, on that context's stream).  After each variant's first call its
outputs (the call's output arrays: the step's flux / optical-property tensors) are compared with the default's bits.
One line per library: median ms per launch over the rounds, min, and whether the outputs were identical.
"""
import argparse
import ctypes
import os
import statistics
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rte-rrtmgp-nn_amd"))
from rrtmgpnn import _lib, data  # noqa: E402
from rrtmgpnn.pipeline import ClearSkyStep  # noqa: E402

# output tensors of each stage (attribute names on ClearSkyStep)
OUTPUTS = {
    "sw_solver": ["sw_up", "sw_dn", "sw_dir"],
    "lw_solver": ["lw_up", "lw_dn"],
    "predict_nn_lw": ["tau_lw", "lay_src"],
    "predict_nn_sw": ["tau_sw", "ssa_sw"],
}


def problem(config):
    if config == "c3":
        return data.rfmip_columns(0, 1800), None
    ncol, nlay = (10000, 60) if config == "c4" else (125000, 137)
    p = data.synthetic_problem(ncol, nlay, seed=20251015, col0=0)
    return p, (data.allsky_clouds(p, data.load_cloud_optics("lw")) if config == "c4" else None)


def bind(path):
    L = ctypes.CDLL(path)
    for name, (res, argt) in _lib.SIGNATURES.items():
        f = getattr(L, name, None)
        if f is not None:
            f.restype, f.argtypes = res, argt
    h = _lib.c_vp()
    assert L.rrtmgpnn_context_create(0, None, h) == 0
    return L, h


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--stage", default="sw_solver")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--base", default=os.path.join(ROOT, "rte-rrtmgp-nn_amd", "librrtmgpnn.so"),
                    help="the library the others are compared with (default: the in-tree build)")
    ap.add_argument("libs", nargs="*")
    a = ap.parse_args()
    torch.cuda.set_device(0)
    prob, clouds = problem(a.config)
    step = ClearSkyStep(prob, device=0, clouds=clouds, overlap=False)
    step.step()
    torch.cuda.synchronize()
    torch.cuda.set_stream(torch.cuda.default_stream(0))  # the variants' contexts run on the null stream
    calls = {n: (fn, args) for n, fn, args in step.calls}
    libs = [(os.path.basename(a.base), a.base)] + [(os.path.basename(p), p) for p in a.libs]
    handles = [(label, bind(path)) for label, path in libs]
    for stage in a.stage.split(","):  # several stages: each timed in turn, one profiler run covers them all
        fn0, args0 = calls[stage]
        fname = fn0.__name__
        outs = [getattr(step, o) for o in OUTPUTS.get(stage, []) if hasattr(step, o)]
        bound = []
        ref = None
        for label, (L, h) in handles:
            f = getattr(L, fname)
            args = list(args0)
            args[0] = h
            for o in outs:
                o.zero_()
            torch.cuda.synchronize()
            rc = f(*args)
            assert rc == 0, (label, rc, L.rrtmgpnn_last_error())
            torch.cuda.synchronize()
            got = [o.detach().cpu().numpy().copy() for o in outs]
            if ref is None:
                ref = got
                same = "ref"
            else:
                same = "bitwise" if all(np.array_equal(x.view(np.uint32), y.view(np.uint32)) for x, y in zip(got, ref)) \
                    else "DIFFERENT(max %.3g)" % max(float(np.max(np.abs(x - y))) for x, y in zip(got, ref))
            bound.append((label, f, args, same, []))
        for _ in range(a.rounds):
            for label, f, args, same, times in bound:
                f(*args)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    f(*args)
                e1.record()
                e1.synchronize()
                times.append(e0.elapsed_time(e1) / a.iters)
        for label, f, args, same, times in bound:
            print("%-28s %s %s  median %.4f ms  min %.4f ms  %s" % (label, a.config, stage, statistics.median(times),
                                                                     min(times), same), flush=True)


if __name__ == "__main__":
    main()
