"""GPU: the opt-in tolerance build (librrtmgpnn_fastlibm.so: the solvers' exps on the hardware exponential instead
of glibc's algorithm in double) against the oracle at the north star's bar, <= 1e-3 W/m2 RMS flux error, on every
RFMIP column (C3), on 2000 synthetic all-sky columns (the C4 recipe) and on a strided sample of 500 columns of the
full C5 shard (125 000 x 137, where both solvers are VALU-bound and the build is timed too: DESIGN.md §3).  At C5 the
build misses the bar (sw_up 1.41e-3 W/m2 RMS, round 6): that case is a strict expected failure recording it.  The default library stays bit-identical
(every other -m gpu test); this build trades the last bits for fewer instructions."""
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

FAST = os.path.join(ROOT, "rte-rrtmgp-nn_amd", "librrtmgpnn_fastlibm.so")


@pytest.mark.parametrize("cfg", ["c3", "c4", pytest.param("c5", marks=pytest.mark.xfail(
    strict=True, reason="measured round 6: at 137 layers the SW up flux misses the bar (RMS 1.41e-3 W/m2 on the "
                        "C5 shard sample; DESIGN.md section 3), so the tolerance build is not an option there"))])
def test_fast_libm_build_meets_north_star_tolerance(tmp_path, orc, cfg):
    from rrtmgpnn import data
    assert os.path.exists(FAST), "librrtmgpnn_fastlibm.so missing: make -C rte-rrtmgp-nn_amd"
    out = str(tmp_path / "fast.npz")
    env = dict(os.environ, RRTMGPNN_LIB=FAST)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "flux_dump.py"), cfg, out], env=env,
                       capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stdout + r.stderr
    got = dict(np.load(out))
    m = {k: data.load_model(k) for k in ("lw_abs", "lw_pfrac", "sw_abs", "sw_ray")}
    kl, ks = data.load_kdist("lw"), data.load_kdist("sw")
    if cfg in ("c3", "c5"):
        prob = data.rfmip_problem()
        if cfg == "c5":  # the sampled columns of the shard flux_dump stepped whole
            from conftest import subset
            prob = subset(data.synthetic_problem(125000, 137, seed=20251015), got.pop("idx"))
        lu, ld, _ = orc.clear_sky_lw(prob, [m["lw_abs"], m["lw_pfrac"]], kl)
        su, sd, sr, _ = orc.clear_sky_sw(prob, [m["sw_abs"], m["sw_ray"]], ks)
    else:
        prob = data.synthetic_problem(2000, 60, seed=20251015)
        co_lw, co_sw = data.load_cloud_optics("lw"), data.load_cloud_optics("sw")
        clouds = data.allsky_clouds(prob, co_lw)
        lu, ld, _ = orc.all_sky_lw(prob, [m["lw_abs"], m["lw_pfrac"]], kl, co_lw, clouds)
        su, sd, sr, _ = orc.all_sky_sw(prob, [m["sw_abs"], m["sw_ray"]], ks, co_sw, clouds)
    use = prob["usecol"]
    report = {}
    for k, ref in (("lw_up", lu), ("lw_dn", ld), ("sw_up", su), ("sw_dn", sd), ("sw_dir", sr)):
        g = got[k].astype(np.float64)
        r = ref.astype(np.float64)
        if k.startswith("sw"):
            g, r = g[use], r[use]
        rms = float(np.sqrt(np.mean((g - r) ** 2)))
        report[k] = rms
        assert rms <= 1e-3, "%s: RMS %.3g W/m2 above the north star's 1e-3" % (k, rms)
    print("fast-libm RMS vs oracle (W/m2):", report)
