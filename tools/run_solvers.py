"""Run only the fused step's solver kernels (for rocprofv3 counter passes): python3 tools/run_solvers.py [reps] [config]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rte-rrtmgp-nn_amd"))
from rrtmgpnn import data  # noqa: E402
from rrtmgpnn._lib import check  # noqa: E402
from rrtmgpnn.pipeline import ClearSkyStep  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
config = sys.argv[2] if len(sys.argv) > 2 else "c3"
prob = data.rfmip_problem() if config == "c3" else data.synthetic_problem(10000, 60)
step = ClearSkyStep(prob, device=0)
torch.cuda.set_stream(step.ctx.stream)  # the raw calls below run on the step's own streams
step.step()
torch.cuda.synchronize()
for _ in range(reps):
    for name, fn, args in step.calls:
        if name in ("lw_solver", "sw_solver", "predict_nn_lw", "predict_nn_sw"):
            check(fn(*args), name)
torch.cuda.synchronize()
print("ok")
