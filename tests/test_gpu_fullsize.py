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


def test_c5_global_rank_chunked_full_size_sampled_vs_oracle(dev, orc):
    """BASELINE configs[4] as bench.py runs it (--global, and every line's c5_global block): the 1e6 x 137 problem
    split over 3 ranks, rank 1's range [333334, 666667) streamed through pipeline.ChunkedRank in 125 000-column chunks
    -- two full chunks through one captured step and a short last one (83 333 columns) through a second -- run twice
    (the slab refilled with nans in between), then a strided sample of the slab that includes every chunk's first and
    last column compared bit for bit with the oracle on those columns."""
    from concurrent.futures import ThreadPoolExecutor
    from rrtmgpnn import data, shard
    from rrtmgpnn.pipeline import ChunkedRank, ClearSkyStep
    G, CH, NL = 1000000, 125000, 137
    lo, hi = shard.column_range(G, 1, 3)
    chunks = [(c, min(c + CH, hi)) for c in range(lo, hi, CH)]
    assert len(chunks) == 3 and chunks[-1][1] - chunks[-1][0] < CH
    with ThreadPoolExecutor(3) as ex:
        futs = {c: ex.submit(data.synthetic_problem, c[1] - c[0], NL, seed=20251015, col0=c[0]) for c in chunks}
        rank = ChunkedRank(lo, hi, CH, lambda c0, c1: (futs.pop((c0, c1)).result(), None),
                           lambda p, c: ClearSkyStep(p, device=0), use_graph=True)
    rank.first = None
    assert len(rank.steps) == 2
    for rep in range(2):
        for t in rank.flux:
            t.fill_(float("nan"))
        rank.run()
        torch.cuda.synchronize()
    got = dict(zip(("lw_up", "lw_dn", "sw_up", "sw_dn", "sw_dir"), (t.cpu().numpy() for t in rank.flux)))
    del rank
    torch.cuda.empty_cache()
    for v in got.values():
        assert np.isfinite(v).all()
    edges = [c - lo for c0, c1 in chunks for c in (c0, c1 - 1)]
    idx = np.unique(np.concatenate([_sample(hi - lo, 300), edges]))
    # the sampled global columns, generated alone (synthetic_problem is column-addressable)
    parts = [data.synthetic_problem(1, NL, seed=20251015, col0=lo + int(i)) for i in idx]
    ps = _concat(parts)
    m = {k: data.load_model(k) for k in ("lw_abs", "lw_pfrac", "sw_abs", "sw_ray")}
    lu, ld, _ = orc.clear_sky_lw(ps, [m["lw_abs"], m["lw_pfrac"]], data.load_kdist("lw"))
    su, sd, sr, _ = orc.clear_sky_sw(ps, [m["sw_abs"], m["sw_ray"]], data.load_kdist("sw"))
    _check(got, idx, ps, (lu, ld), (su, sd, sr))


def _concat(parts):
    """One problem dict of single-column problems, in order."""
    out = dict(parts[0])
    for k, v in parts[0].items():
        if isinstance(v, np.ndarray) and v.ndim >= 1 and v.shape[0] == 1:
            out[k] = np.concatenate([p[k] for p in parts])
    out["gases"] = {k: np.concatenate([p["gases"][k] for p in parts]) for k in parts[0]["gases"]}
    out["ncol"] = len(parts)
    return out
