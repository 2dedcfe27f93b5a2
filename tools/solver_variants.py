"""Time the LW/SW solver kernels of each variant build (tools/solver_variants.sh) on one config's inputs and
check every variant's fluxes bit for bit against the first variant."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rte-rrtmgp-nn_amd"))
from rrtmgpnn import _lib, data  # noqa: E402
from rrtmgpnn.pipeline import ClearSkyStep  # noqa: E402

B, config, names = sys.argv[1], sys.argv[2], sys.argv[3:]
prob = data.rfmip_problem() if config == "c3" else data.synthetic_problem(10000 if config == "c4" else 125000,
                                                                         60 if config == "c4" else 137)
steps = {"": ClearSkyStep(prob, device=0, fused=False), "fused_": ClearSkyStep(prob, device=0, fused=True)}
calls, outs = {}, {}
for tag, step in steps.items():
    step.step()
    torch.cuda.synchronize()
    for n, fn, a in step.calls:
        if n in ("lw_solver", "sw_solver"):
            calls[tag + n] = (n, a)
    outs[tag + "lw_solver"] = (step.lw_up, step.lw_dn)
    outs[tag + "sw_solver"] = (step.sw_up, step.sw_dn, step.sw_dir)
first = {}
for v in names:
    L = ctypes.CDLL(os.path.join(B, "lib_%s.so" % v))
    for name, (res, args) in _lib.SIGNATURES.items():
        f = getattr(L, name)
        f.restype, f.argtypes = res, args
    h = _lib.c_vp()
    assert L.rrtmgpnn_context_create(0, None, h) == 0
    line = []
    fns = {"lw_solver": L.rrtmgpnn_lw_solver_noscat, "fused_lw_solver": L.rrtmgpnn_lw_solver_noscat_planck,
           "sw_solver": L.rrtmgpnn_sw_solver_2stream, "fused_sw_solver": L.rrtmgpnn_sw_solver_2stream}
    for name, fn in fns.items():
        a = list(calls[name][1])
        a[0] = h
        for t in outs[name]:
            t.fill_(float("nan"))
        rc = fn(*a)
        torch.cuda.synchronize()
        if rc:
            line.append("%s FAILED rc=%d" % (name, rc))
            continue
        res = [t.cpu().numpy().copy() for t in outs[name]]
        if name not in first:
            first[name] = res
            same = "ref"
        else:
            same = "bitwise" if all(np.array_equal(x, y) for x, y in zip(res, first[name])) else "DIFFERS"
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            fn(*a)
        e1.record()
        e1.synchronize()
        line.append("%s %.4f ms (%s)" % (name, e0.elapsed_time(e1) / 20, same))
    print("%-14s" % v, " | ".join(line), flush=True)
