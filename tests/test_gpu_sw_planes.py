"""GPU: the SW solver's workspace-plane fallback.  The large-grid clear-sky instance and the all-sky
instances keep beam-transmittance / exp(-k tau) planes in the context's workspace (up to 3x the checkpoints: 46.4 GB
at the C5 shard).  When that allocation fails, launch_sw_2stream retries with the instances that recompute instead
(the round-4 forms).  RRTMGPNN_SW_NO_PLANES=1 takes that path from the start; a child process run with it must give
the default instances' fluxes bit for bit, for the large clear-sky grid (g = NULL) and for the all-sky (fused
increment) instance with and without g."""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys, numpy as np, torch
sys.path.insert(0, %(pkg)r)
from rrtmgpnn import _lib, data
from rrtmgpnn._lib import check, int_array
from rrtmgpnn.api import context
d = np.load(%(inp)r)
dev = torch.device("cuda", 0)
T = lambda a: torch.as_tensor(np.ascontiguousarray(a), device=dev)
L, c = _lib.lib(), context(0).h
out = {}
for case in ("clear", "inc", "inc_g"):
    ncol, nlay, ngpt = (int(v) for v in d[case + "_shape"])
    tau, ssa = T(d[case + "_tau"]), T(d[case + "_ssa"])
    mu0, toa, alb = T(d[case + "_mu0"]), T(d[case + "_toa"]), T(d[case + "_alb"])
    fl = [torch.full((ncol, nlay + 1), float("nan"), device=dev) for _ in range(3)]
    p = lambda t: t.data_ptr() if t is not None else None
    if case == "clear":
        check(L.rrtmgpnn_sw_solver_2stream(c, ngpt, nlay, ncol, 1, p(toa), None, p(tau), p(ssa), None, p(mu0), p(alb),
                                           p(alb), *[p(f) for f in fl]), case)
    else:
        g = T(d[case + "_g"]) if case == "inc_g" else None
        lims = int_array(d["lims"].ravel())
        ct, cs, cg = T(d[case + "_ctau"]), T(d[case + "_cssa"]), T(d[case + "_cg"])
        check(L.rrtmgpnn_sw_solver_2stream_inc(c, ngpt, nlay, ncol, 1, p(toa), None, p(tau), p(ssa), p(g),
                                               int(d["nband"]), lims, p(ct), p(cs), p(cg), p(mu0), p(alb), p(alb),
                                               *[p(f) for f in fl]), case)
    torch.cuda.synchronize()
    for k, f in zip(("up", "dn", "dir"), fl):
        out[case + "_" + k] = f.cpu().numpy()
np.savez(%(out)r, **out)
"""


def _inputs(path):
    from rrtmgpnn import data
    kd = data.load_kdist("sw")
    ngpt, nband = int(kd["ngpt"]), int(kd["nband"])
    rng = np.random.default_rng(20251018)
    d = {"lims": kd["band_lims_gpt"], "nband": nband}
    # clear sky past the small-grid bound (ncol * ngpt / 2 > 64 * 16 * 256 lanes): the large NN instance
    for case, ncol, nlay in (("clear", 2400, 9), ("inc", 64, 23), ("inc_g", 48, 17)):
        d[case + "_shape"] = np.array([ncol, nlay, ngpt])
        d[case + "_tau"] = (rng.lognormal(-3.0, 2.0, (ncol, nlay, ngpt))).astype(np.float32)
        d[case + "_ssa"] = rng.uniform(0.0, 1.0, (ncol, nlay, ngpt)).astype(np.float32)
        d[case + "_g"] = rng.uniform(0.0, 0.9, (ncol, nlay, ngpt)).astype(np.float32)
        d[case + "_mu0"] = rng.uniform(0.05, 1.0, ncol).astype(np.float32)
        d[case + "_toa"] = rng.uniform(0.0, 10.0, (ncol, ngpt)).astype(np.float32)
        d[case + "_alb"] = rng.uniform(0.0, 0.9, (ncol, ngpt)).astype(np.float32)
        d[case + "_ctau"] = rng.lognormal(-1.0, 1.5, (ncol, nlay, nband)).astype(np.float32)
        d[case + "_cssa"] = rng.uniform(0.5, 1.0, (ncol, nlay, nband)).astype(np.float32)
        d[case + "_cg"] = rng.uniform(0.0, 0.9, (ncol, nlay, nband)).astype(np.float32)
    np.savez(path, **d)


def _run(inp, out, no_planes):
    env = dict(os.environ)
    env.pop("RRTMGPNN_SW_NO_PLANES", None)
    if no_planes:
        env["RRTMGPNN_SW_NO_PLANES"] = "1"
    code = CHILD % {"pkg": os.path.join(ROOT, "rte-rrtmgp-nn_amd"), "inp": inp, "out": out}
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    return dict(np.load(out))


def test_sw_workspace_plane_fallback_is_bitwise(tmp_path):
    inp = str(tmp_path / "in.npz")
    _inputs(inp)
    a = _run(inp, str(tmp_path / "planes.npz"), False)
    b = _run(inp, str(tmp_path / "noplanes.npz"), True)
    assert set(a) == set(b) and len(a) == 9
    for k in a:
        assert np.isfinite(a[k]).all(), k
        np.testing.assert_array_equal(a[k].view(np.uint32), b[k].view(np.uint32), err_msg=k)
