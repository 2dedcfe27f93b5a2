"""GPU: the direct beam handed from the SW network to the SW solver (rrtmgpnn_gas_optics_sw_nn_beam, then
rrtmgpnn_sw_solver_2stream on the same context) is bit-identical to the solver forming it itself.

The network kernel walks a column's tiles top first and multiplies the beam down each g-point's layers after a
lane-half swap (kernels_nn32.hip BEAM), the solver reads the checkpoints and the transmittance plane it left
(kernels_sw_ck.hip kBeamIn): every layer count that puts a column into one, two or three 32-row tiles, with chunk
boundaries inside and across tiles, both orientations, the captured step, and the hand-over refused when another
call comes between or the solver call's arrays differ.
"""
import ctypes

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


def _flip(prob):
    out = dict(prob)
    # copies: a flipped (n, 1) array counts as contiguous to numpy but keeps its negative stride, which torch refuses
    for k in ("play", "plev", "tlay", "tlev"):
        out[k] = np.array(prob[k][:, ::-1], order="C", copy=True)
    out["gases"] = {k: np.array(v[:, ::-1], order="C", copy=True) for k, v in prob["gases"].items()}
    out["top_at_1"] = not prob["top_at_1"]
    return out


def _run(prob, beam, graph=False, overlap=True):
    from rrtmgpnn.pipeline import ClearSkyStep
    st = ClearSkyStep(prob, device=0, sw_beam=beam, overlap=overlap)
    if graph:
        st.capture()
        st.replay()
        st.replay()
    else:
        st.step()
        st.step()
    torch.cuda.synchronize()
    out = st.fluxes()
    out["tau_sw"], out["ssa_sw"] = st.tau_sw.cpu().numpy(), st.ssa_sw.cpu().numpy()
    sw_ctx = st.ctx2 if st.overlap else st.ctx
    return out, sw_ctx.sw_beam_handoffs()


def _same(a, b):
    for k in a:
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)


@pytest.mark.parametrize("flip", [False, True])
@pytest.mark.parametrize("ncol", [1, 37, 600])
def test_beam_handoff_rfmip(dev, rfmip, ncol, flip):
    prob = subset(rfmip, np.arange(ncol) * 3 % 1800)
    if flip:
        prob = _flip(prob)
    want, n0 = _run(prob, False)
    got, n1 = _run(prob, True)
    assert n0 == 0 and n1 == 2, (n0, n1)  # both steps handed the beam over
    _same(want, got)


@pytest.mark.parametrize("nlay", [1, 2, 3, 31, 32, 33, 59, 64, 65, 97])
@pytest.mark.parametrize("flip", [False, True])
def test_beam_handoff_layer_counts(dev, nlay, flip):
    from rrtmgpnn import data
    prob = data.synthetic_problem(23, nlay, seed=7, col0=1000)
    if flip:
        prob = _flip(prob)
    want, _ = _run(prob, False)
    got, n = _run(prob, True)
    assert n == 2
    _same(want, got)


def test_beam_handoff_captured_and_serial(dev, rfmip):
    prob = subset(rfmip, np.arange(0, 1800, 4))
    want, _ = _run(prob, False, graph=True)
    got, n = _run(prob, True, graph=True)
    assert n == 2  # the warm-up step and the captured one (whose replays re-run its kernels)
    _same(want, got)
    got2, n2 = _run(prob, True, overlap=False)  # one context: the solver is still the next call after the network
    assert n2 == 2
    _same(want, got2)


def test_beam_handoff_refused(dev, rfmip):
    """A call between the two, or a solver call on other arrays, gets no hand-over -- and the same fluxes."""
    from rrtmgpnn import _lib
    from rrtmgpnn._lib import check
    from rrtmgpnn.pipeline import ClearSkyStep
    prob = subset(rfmip, np.arange(0, 1800, 17))
    st = ClearSkyStep(prob, device=0, sw_beam=True, overlap=False)
    L = _lib.lib()
    net = next(a for n, f, a in st.calls if n == "predict_nn_sw")
    sol = next(a for n, f, a in st.calls if n == "sw_solver")
    outs = []
    for case in ("handed", "between", "other_tau"):
        for t in (st.sw_up, st.sw_dn, st.sw_dir):
            t.zero_()
        check(L.rrtmgpnn_gas_optics_sw_nn_beam(*net), "gas_optics_sw_nn_beam")
        args = list(sol)
        if case == "between":
            st.ctx.mlp_max_cus()  # any entry on the context
        if case == "other_tau":
            torch.cuda.synchronize()
            tau2 = st.tau_sw.clone()
            torch.cuda.synchronize()
            args[7] = tau2.data_ptr()
        before = st.ctx.sw_beam_handoffs()
        check(L.rrtmgpnn_sw_solver_2stream(*args), "sw_solver_2stream")
        torch.cuda.synchronize()
        assert st.ctx.sw_beam_handoffs() - before == (1 if case == "handed" else 0), case
        outs.append([t.cpu().numpy() for t in (st.sw_up, st.sw_dn, st.sw_dir)])
    for o in outs[1:]:
        for a, b in zip(outs[0], o):
            np.testing.assert_array_equal(a, b)


def test_beam_entry_requires_inputs(dev, rfmip):
    from rrtmgpnn import _lib
    from rrtmgpnn.pipeline import ClearSkyStep
    st = ClearSkyStep(subset(rfmip, np.arange(4)), device=0, sw_beam=True, overlap=False)
    net = list(next(a for n, f, a in st.calls if n == "predict_nn_sw"))
    net[-1] = None  # mu0
    assert _lib.lib().rrtmgpnn_gas_optics_sw_nn_beam(*net) != 0
    assert b"mu0" in _lib.lib().rrtmgpnn_last_error()
