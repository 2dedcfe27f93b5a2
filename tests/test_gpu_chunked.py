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


def test_pinned_copies_on_a_closed_steps_stream(dev):
    """bench.py's host-resident leg makes non-blocking copies between pinned host tensors and the step's tensors on
    the step's own stream; torch's pinned-memory allocator keeps an event recorded on that stream and queries it when
    the host tensors are freed -- after the step is closed.  Round 6 first destroyed the step's streams in close(),
    and bench.py crashed in that query; streams are now handed back and reused, never destroyed.  The
    sequence must run clean, and a step built afterwards (on a reused stream) must give the first step's fluxes."""
    import gc
    from rrtmgpnn.pipeline import ClearSkyStep
    problem = _problem("rfmip")
    p, _ = problem(0, 96)
    st = ClearSkyStep(p, device=0)
    st.capture()
    torch.cuda.set_stream(st.ctx.stream)
    try:
        st.replay()
        ins, outs = st.io_tensors()
        h_ins = [t.cpu().pin_memory() for t in ins]
        h_outs = [torch.empty(t.shape, dtype=t.dtype, pin_memory=True) for t in outs]
        for _ in range(3):
            for d, h in zip(ins, h_ins):
                d.copy_(h, non_blocking=True)
            st.replay()
            for h, d in zip(h_outs, outs):
                h.copy_(d, non_blocking=True)
        torch.cuda.synchronize()
        want = [h.numpy().copy() for h in h_outs]
    finally:
        torch.cuda.set_stream(torch.cuda.default_stream(dev))
    st.close()
    del st, ins, outs, h_ins, h_outs
    gc.collect()
    torch.cuda.empty_cache()
    again = ClearSkyStep(p, device=0)
    again.capture()
    again.replay()
    torch.cuda.synchronize()
    got = again.io_tensors()[1]
    for w, g in zip(want, got):
        np.testing.assert_array_equal(g.cpu().numpy(), w)
    again.close()


@pytest.mark.parametrize("config", ["rfmip", "allsky"])
def test_block_stream_equals_step(dev, config):
    """ClearSkyStep.run_blocks (the two chains replayed free-running, bench.py's block_stream): after any number of
    blocks the fluxes are the joined step's, bit for bit, and a joined replay afterwards still gives them."""
    from rrtmgpnn.pipeline import ClearSkyStep
    p, c = _problem(config)(100, 100 + 333)
    st = ClearSkyStep(p, device=0, clouds=c)
    st.step()
    torch.cuda.synchronize()
    want = st.fluxes()
    st.capture()
    st.capture_chains()
    keys = ("lw_up", "lw_dn", "sw_up", "sw_dn", "sw_dir")
    for k in (1, 7):
        for name in keys:
            getattr(st, name).fill_(float("nan"))
        st.run_blocks(k)
        torch.cuda.synchronize()
        got = st.fluxes()
        for name in keys:
            np.testing.assert_array_equal(got[name], want[name], err_msg="%s after %d blocks" % (name, k))
    st.replay()
    torch.cuda.synchronize()
    for name, v in st.fluxes().items():
        np.testing.assert_array_equal(v, want[name], err_msg=name)
    st.close()
