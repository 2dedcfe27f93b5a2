"""GPU correctness at the sizes bench.py times (BASELINE configs C4 and C5), not just at test sizes.

The benchmarked step runs once over the whole problem -- C4: 10 000 synthetic all-sky columns x 60 layers; C5: one
GPU's shard, 125 000 synthetic columns x 137 layers, whose g-point arrays hold 4.38e9 elements (past 2^32, so every
index and workspace size of the solvers and networks is exercised at full width) -- and a strided sample of columns,
the last column included, is compared bit for bit with the oracle run on those columns alone (columns are
independent, so the sample's fluxes are the full problem's).  Same generators and seeds as bench.py.
"""
import numpy as np
import pytest

from conftest import subset

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a device"
    torch.cuda.set_device(0)
    return torch.device("cuda", 0)


def _sample(ncol, n):
    idx = np.unique(np.concatenate([np.linspace(0, ncol - 1, n).astype(np.int64), [ncol - 1]]))
    return idx


def _check(got, idx, prob_s, lw, sw):
    lu, ld = lw
    su, sd, sr = sw
    np.testing.assert_array_equal(got["lw_up"][idx], lu)
    np.testing.assert_array_equal(got["lw_dn"][idx], ld)
    use = prob_s["usecol"]
    for k, r in (("sw_up", su), ("sw_dn", sd)):
        g = got[k][idx].copy()
        g[~use] = 0.0
        np.testing.assert_array_equal(g, r, err_msg=k)
    np.testing.assert_array_equal(got["sw_dir"][idx][use], sr[use])


def test_c4_full_size_allsky_step_sampled_vs_oracle(dev, orc):
    from rrtmgpnn import data
    from rrtmgpnn.pipeline import ClearSkyStep
    prob = data.synthetic_problem(10000, 60, seed=20251015)
    co_lw, co_sw = data.load_cloud_optics("lw"), data.load_cloud_optics("sw")
    clouds = data.allsky_clouds(prob, co_lw)
    step = ClearSkyStep(prob, device=0, clouds=clouds)
    step.capture()
    step.replay()
    torch.cuda.synchronize()
    got = step.fluxes()
    for v in got.values():
        assert np.isfinite(v).all()
    idx = _sample(prob["ncol"], 400)
    ps = subset(prob, idx)
    cs = tuple(c[idx] for c in clouds)
    m = {k: data.load_model(k) for k in ("lw_abs", "lw_pfrac", "sw_abs", "sw_ray")}
    lu, ld, _ = orc.all_sky_lw(ps, [m["lw_abs"], m["lw_pfrac"]], data.load_kdist("lw"), co_lw, cs)
    su, sd, sr, _ = orc.all_sky_sw(ps, [m["sw_abs"], m["sw_ray"]], data.load_kdist("sw"), co_sw, cs)
    _check(got, idx, ps, (lu, ld), (su, sd, sr))


def test_c5_shard_full_size_step_sampled_vs_oracle(dev, orc):
    from rrtmgpnn import data
    from rrtmgpnn.pipeline import ClearSkyStep
    prob = data.synthetic_problem(125000, 137, seed=20251015)
    assert prob["ncol"] * prob["nlay"] * 256 > 2 ** 32
    step = ClearSkyStep(prob, device=0)
    step.capture()
    step.replay()
    torch.cuda.synchronize()
    got = step.fluxes()
    del step
    torch.cuda.empty_cache()
    for v in got.values():
        assert np.isfinite(v).all()
    idx = _sample(prob["ncol"], 500)
    ps = subset(prob, idx)
    m = {k: data.load_model(k) for k in ("lw_abs", "lw_pfrac", "sw_abs", "sw_ray")}
    lu, ld, _ = orc.clear_sky_lw(ps, [m["lw_abs"], m["lw_pfrac"]], data.load_kdist("lw"))
    su, sd, sr, _ = orc.clear_sky_sw(ps, [m["sw_abs"], m["sw_ray"]], data.load_kdist("sw"))
    _check(got, idx, ps, (lu, ld), (su, sd, sr))
