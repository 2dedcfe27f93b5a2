"""Time the LW/SW solver kernels of each ablation build (tools/ablate_solvers.sh) on the C3 inputs."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rte-rrtmgp-nn_amd"))
from rrtmgpnn import _lib, data  # noqa: E402
from rrtmgpnn.pipeline import ClearSkyStep  # noqa: E402

B = sys.argv[1]
step = ClearSkyStep(data.rfmip_problem(), device=0)
step.step()
torch.cuda.synchronize()
calls = {n: a for n, _, a in step.calls}
for v in ["base", "NATIVE_EXP", "NO_REDUCE", "NO_BARRIER"]:
    L = ctypes.CDLL(os.path.join(B, "lib_%s.so" % v))
    for name, (res, args) in _lib.SIGNATURES.items():
        f = getattr(L, name)
        f.restype, f.argtypes = res, args
    h = _lib.c_vp()
    assert L.rrtmgpnn_context_create(0, None, h) == 0
    out = []
    for name, fn in (("lw_solver", L.rrtmgpnn_lw_solver_noscat), ("sw_solver", L.rrtmgpnn_sw_solver_2stream)):
        a = list(calls[name])
        a[0] = h
        fn(*a)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            fn(*a)
        e1.record()
        e1.synchronize()
        out.append("%s %.4f ms" % (name, e0.elapsed_time(e1) / 20))
    print(v, " | ".join(out), flush=True)
