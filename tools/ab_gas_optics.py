"""Time the fused gas-optics entries (rrtmgpnn_gas_optics_{lw,sw}_nn) against the three separate calls they replace,
alternating, in one process (C3 and C4 sizes)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rte-rrtmgp-nn_amd"))
from rrtmgpnn import _lib, data  # noqa: E402
from rrtmgpnn._lib import check  # noqa: E402
from rrtmgpnn.api import context  # noqa: E402
from rrtmgpnn.pipeline import ClearSkyStep  # noqa: E402


def timeit(fns, reps=20):
    for f in fns:
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        for f in fns:
            f()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


for cfg, prob in (("c3", data.rfmip_problem()), ("c4", data.synthetic_problem(10000, 60))):
    # both on the default context (torch's current stream), where the timing events are recorded
    sep = ClearSkyStep(prob, device=0, fused=False, overlap=False, ctx=context(0))
    fus = ClearSkyStep(prob, device=0, fused=True, overlap=False, ctx=context(0))
    call = lambda st, n: (lambda: check(next(f for m, f, a in st.calls if m == n)(*next(a for m, f, a in st.calls if m == n)), n))  # noqa: E731
    for chain, names in (("lw", ("get_col_dry", "nn_inputs_lw", "predict_nn_lw")), ("sw", ("get_col_dry", "nn_inputs_sw", "predict_nn_sw"))):
        a = [call(sep, n) for n in names]
        b = [call(fus, "predict_nn_" + chain)]
        res = {"sep": [], "fused": []}
        for _ in range(3):
            res["sep"].append(timeit(a))
            res["fused"].append(timeit(b))
        print(cfg, chain, "separate %.4f ms  fused %.4f ms" % (min(res["sep"]), min(res["fused"])), flush=True)
