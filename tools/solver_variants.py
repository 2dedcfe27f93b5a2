"""Time every stage of the fused step (and the unfused LW/SW solvers) for each variant build
(tools/solver_variants.sh), checking each variant's fluxes bit for bit against the first variant."""
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
# c4a: the C4 all-sky step (clouds by the all-sky example's recipe)
prob = data.rfmip_problem() if config == "c3" else data.synthetic_problem(125000 if config == "c5" else 10000,
                                                                         137 if config == "c5" else 60)
clouds = data.allsky_clouds(prob, data.load_cloud_optics("lw")) if config == "c4a" else None
steps = {"": ClearSkyStep(prob, device=0, fused=False, clouds=clouds),
         "f:": ClearSkyStep(prob, device=0, fused=True, clouds=clouds)}
for st in steps.values():
    st.step()
torch.cuda.synchronize()
SHOW = {"": ("lw_solver", "sw_solver"), "f:": ("predict_nn_lw", "lw_solver", "predict_nn_sw", "sw_solver", "nn_inputs_lw")}
first = None


def bind(L):
    for name, (res, args) in _lib.SIGNATURES.items():
        f = getattr(L, name)
        f.restype, f.argtypes = res, args


for v in names:
    # "name@s": variant `name` with the SW solver forced to s g-points per lane (0: the library's choice)
    lib, _, swk = v.partition("@")
    L = ctypes.CDLL(os.path.join(B, "lib_%s.so" % lib))
    bind(L)
    h = _lib.c_vp()
    assert L.rrtmgpnn_context_create(0, None, h) == 0
    if swk or os.environ.get("SW_KERNEL"):
        L.rrtmgpnn_context_set_sw_kernel(h, int(swk or os.environ["SW_KERNEL"]))
    line, res = [], []
    for tag, st in steps.items():
        # the networks are loaded through the variant library too (its packed MLP images)
        calls = []
        for name, fn, a in st.calls:
            a = list(a)
            a[0] = h
            calls.append((name, getattr(L, fn.__name__), a))
        nets = {}
        for m in ("lw_abs", "lw_pfrac", "sw_abs", "sw_ray"):
            hh = _lib.c_vp()
            assert L.rrtmgpnn_network_load(h, data.path(m).encode(), hh) == 0
            nets[m] = hh.value
        keep = []
        for name, fn, a in calls:
            if name.startswith("predict_nn"):
                models = ("lw_abs", "lw_pfrac") if "lw" in name else ("sw_abs", "sw_ray")
                arr = (ctypes.c_void_p * 2)(*[nets[m] for m in models])
                keep.append(arr)
                a[11 if "gas_optics" in fn.__name__ else 7] = arr  # rrtmgpnn_gas_optics_*_nn (fused) or predict_nn_*
            elif name.startswith("nn_inputs"):
                a[8] = ctypes.c_void_p(nets["lw_abs" if "lw" in name else "sw_abs"])
        for t in (st.lw_up, st.lw_dn, st.sw_up, st.sw_dn, st.sw_dir):
            t.fill_(float("nan"))
        for name, fn, a in calls:
            assert fn(*a) == 0, name
        torch.cuda.synchronize()
        res += [t.cpu().numpy().copy() for t in (st.lw_up, st.lw_dn, st.sw_up, st.sw_dn, st.sw_dir)]
        for name, fn, a in calls:
            if name not in SHOW[tag]:
                continue
            best = 1e9
            for _ in range(int(os.environ.get("REPS", "2"))):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(20):
                    fn(*a)
                e1.record()
                e1.synchronize()
                best = min(best, e0.elapsed_time(e1) / 20)
            line.append("%s%s %.4f" % (tag, name, best))
    if first is None:
        first, same = res, "ref"
    else:
        bad = [(i, float(np.nanmax(np.abs(x - y)))) for i, (x, y) in enumerate(zip(res, first))
               if not np.array_equal(x, y)]
        same = "bitwise" if not bad else "DIFFERS " + ",".join("%d:%.2g" % b for b in bad)
    print("%-10s [%s] " % (v, same) + " | ".join(line), flush=True)
