"""GPU: the chunked rank path bench.py --global takes when a rank holds more columns than one step's block
(C5 at N < 8: 8, 4 or 2 chunks per rank).  pipeline.ChunkedRank copies each chunk's HBM-resident inputs into the
captured step's buffers, replays the graph and copies the fluxes into the rank's slab; a short last chunk runs through
a step of its own shape.  The slab must equal, bit for bit, one independent ClearSkyStep per chunk -- the last chunk
included -- and stay so over repeated runs (stale buffers or a missed copy would show as a chunk holding another
chunk's fluxes)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a device"
    torch.cuda.set_device(0)
    return torch.device("cuda", 0)


def _problem(config):
    from rrtmgpnn import data

    def problem(c0, c1):
        if config == "rfmip":
            return data.rfmip_columns(c0, c1 - c0), None
        p = data.synthetic_problem(c1 - c0, 60, seed=20251015, col0=c0)
        return p, (data.allsky_clouds(p, data.load_cloud_optics("lw")) if config == "allsky" else None)
    return problem


@pytest.mark.parametrize("config,lo,hi,chunk,graph", [
    ("rfmip", 10, 10 + 3 * 64, 64, True),          # 3 full chunks
    ("rfmip", 1700, 1700 + 3 * 48 + 17, 48, True),  # 3 full + a short last chunk (wraps the 1800 RFMIP columns)
    ("synthetic", 1000, 1000 + 4 * 40, 40, False),  # eager launches, synthetic clear sky
    ("allsky", 0, 3 * 32 + 5, 32, True),            # all-sky step (clouds), ragged last chunk
])
def test_chunked_rank_equals_independent_steps(dev, config, lo, hi, chunk, graph):
    from rrtmgpnn.pipeline import ChunkedRank, ClearSkyStep
    problem = _problem(config)
    rank = ChunkedRank(lo, hi, chunk, problem, lambda p, c: ClearSkyStep(p, device=0, clouds=c), use_graph=graph)
    assert len(rank.chunks) >= 3
    keys = ("lw_up", "lw_dn", "sw_up", "sw_dn", "sw_dir")
    want = []
    for c0, c1 in rank.chunks:
        p, c = problem(c0, c1)
        st = ClearSkyStep(p, device=0, clouds=c)
        st.step()
        torch.cuda.synchronize()
        want.append(st.fluxes())
    for rep in range(3):
        for t in rank.flux:
            t.fill_(float("nan"))
        rank.run()
        torch.cuda.synchronize()
        got = [t.cpu().numpy() for t in rank.flux]
        for (c0, c1), w in zip(rank.chunks, want):
            for k, g in zip(keys, got):
                np.testing.assert_array_equal(g[c0 - lo:c1 - lo], w[k],
                                              err_msg="%s, chunk %d..%d, run %d" % (k, c0, c1, rep))


def test_chunked_rank_after_torn_down_ranks(dev):
    """The round-5 segfault's sequence, on today's code: ranks whose steps were captured several times
    (the removed direct mode held one graph per chunk on each step) are replayed and torn down -- once by close(),
    once left to garbage collection -- and a rank with two step shapes (3 x 48 columns + a short chunk of 17) is then
    built, captured and replayed three times.  Its slab must equal one independent step per chunk bit for bit."""
    import gc
    from rrtmgpnn.pipeline import ChunkedRank, ClearSkyStep
    problem = _problem("rfmip")
    lo, hi, chunk = 1700, 1700 + 3 * 48 + 17, 48
    make = lambda p, c: ClearSkyStep(p, device=0, clouds=c)  # noqa: E731
    for explicit in (True, False):
        old = ChunkedRank(lo, hi, chunk, problem, make, use_graph=True)
        for st in old.steps:
            for _ in range(4):
                st.capture()
        for _ in range(2):
            old.run()
        torch.cuda.synchronize()
        if explicit:
            old.close()
        del old
        gc.collect()
    rank = ChunkedRank(lo, hi, chunk, problem, make, use_graph=True)
    assert len({st.ncol for st in rank.steps}) == 2
    want = []
    for c0, c1 in rank.chunks:
        st = ClearSkyStep(problem(c0, c1)[0], device=0)
        st.step()
        torch.cuda.synchronize()
        want.append(st.fluxes())
        st.close()
    keys = ("lw_up", "lw_dn", "sw_up", "sw_dn", "sw_dir")
    for rep in range(3):
        for t in rank.flux:
            t.fill_(float("nan"))
        rank.run()
        torch.cuda.synchronize()
        got = [t.cpu().numpy() for t in rank.flux]
        for (c0, c1), w in zip(rank.chunks, want):
            for k, g in zip(keys, got):
                np.testing.assert_array_equal(g[c0 - lo:c1 - lo], w[k], err_msg="%s, chunk %d..%d, run %d"
                                              % (k, c0, c1, rep))
    rank.close()
