"""GPU: the fused entry points are bit-identical to the class layer's call sequence.

* rrtmgpnn_lw_solver_noscat_planck (Planck sources formed in-kernel from pfrac) ==
  compute_planck_source_nn + lw_solver_noscat, and == the oracle, for nmus 1-4 and both orientations;
* rrtmgpnn_sw_solver_2stream with g == NULL == the same call with a zero-filled g;
* the fused ClearSkyStep (the benchmarked step) == the unfused one, bit for bit.
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


def T(a, dev):
    # a copy: a flipped (n, 1) array counts as contiguous to numpy but keeps its negative stride, which torch refuses
    return torch.as_tensor(np.array(a, dtype=np.float32, order="C", copy=True), device=dev)


def _flip(prob):
    out = dict(prob)
    for k in ("play", "plev", "tlay", "tlev"):
        out[k] = np.ascontiguousarray(prob[k][:, ::-1])
    out["gases"] = {k: np.ascontiguousarray(v[:, ::-1]) for k, v in prob["gases"].items()}
    out["top_at_1"] = False
    return out


@pytest.mark.parametrize("nmus", [1, 2, 3, 4])
@pytest.mark.parametrize("top_at_1", [True, False])
def test_fused_lw_solver_matches_oracle(dev, orc, rfmip, nmus, top_at_1):
    from rrtmgpnn import _lib, data
    from rrtmgpnn._lib import check, float_array, int_array
    from rrtmgpnn.api import GAUSS_DS, GAUSS_WTS, context
    prob = subset(rfmip, np.arange(5, 1800, 13))
    if not top_at_1:
        prob = _flip(prob)
    kd = data.load_kdist("lw")
    go = orc.lw_gas_optics(prob, [data.load_model("lw_abs"), data.load_model("lw_pfrac")], kd)
    ncol, nlay, ngpt = go["tau"].shape
    emis = np.repeat(np.asarray(prob["sfc_emis"], np.float32)[:, None], ngpt, axis=1)
    up_o, dn_o = orc.lw_solver(go["tau"], go["lay_source"], go["lev_source"], emis, go["sfc_source"], top_at_1, nmus)
    sfc_lay = 1 if prob["play"][0, 0] > prob["play"][0, nlay - 1] else nlay
    up, dn = torch.empty((ncol, nlay + 1), device=dev), torch.empty((ncol, nlay + 1), device=dev)
    args = [T(go["tau"], dev), T(go["pfrac"], dev), T(prob["tlay"], dev), T(prob["tlev"], dev), T(prob["tsfc"], dev),
            T(kd["totplnk"], dev), T(emis, dev)]
    ctx = context(0)
    check(_lib.lib().rrtmgpnn_lw_solver_noscat_planck(
        ctx.h, ngpt, nlay, ncol, int(top_at_1), nmus, float_array(GAUSS_DS[nmus]), float_array(GAUSS_WTS[nmus]), None,
        args[0].data_ptr(), args[1].data_ptr(), kd["nband"], kd["nPlanckTemp"], args[2].data_ptr(),
        args[3].data_ptr(), args[4].data_ptr(), sfc_lay, int_array(kd["band_lims_gpt"].ravel()),
        float(kd["temp_ref_min"][0]), float(kd["totplnk_delta"]), args[5].data_ptr(), 0, args[6].data_ptr(),
        up.data_ptr(), dn.data_ptr()), "lw_solver_noscat_planck")
    torch.cuda.synchronize()
    np.testing.assert_array_equal(up.cpu().numpy(), up_o)
    np.testing.assert_array_equal(dn.cpu().numpy(), dn_o)


@pytest.mark.parametrize("top_at_1", [True, False])
def test_sw_null_g_equals_zero_g(dev, top_at_1, sw_kernel):
    from rrtmgpnn import _lib
    from rrtmgpnn._lib import check
    from rrtmgpnn.api import context
    rng = np.random.default_rng(11)
    ncol, nlay, ngpt = 41, 37, 224
    tau = T(rng.lognormal(-2, 2, size=(ncol, nlay, ngpt)), dev)
    ssa = T(rng.uniform(0, 1, size=(ncol, nlay, ngpt)), dev)
    zero = torch.zeros_like(tau)
    mu0 = T(rng.uniform(0.05, 1, size=ncol), dev)
    inc = T(rng.uniform(0, 10, size=(ncol, ngpt)), dev)
    ad, af = T(rng.uniform(0, 1, size=(ncol, ngpt)), dev), T(rng.uniform(0, 1, size=(ncol, ngpt)), dev)
    outs = []
    for g in (zero, None):
        o = [torch.empty((ncol, nlay + 1), device=dev) for _ in range(3)]
        check(_lib.lib().rrtmgpnn_sw_solver_2stream(
            context(0).h, ngpt, nlay, ncol, int(top_at_1), inc.data_ptr(), None, tau.data_ptr(), ssa.data_ptr(),
            None if g is None else g.data_ptr(), mu0.data_ptr(), ad.data_ptr(), af.data_ptr(), *[t.data_ptr() for t in o]),
            "sw_solver_2stream")
        torch.cuda.synchronize()
        outs.append([t.cpu().numpy() for t in o])
    for a, b in zip(*outs):
        np.testing.assert_array_equal(a, b)


def test_fused_step_equals_class_sequence(dev, rfmip):
    from rrtmgpnn.pipeline import ClearSkyStep
    prob = subset(rfmip, np.arange(2, 1800, 3))
    res = []
    for fused in (False, True):
        step = ClearSkyStep(prob, device=0, fused=fused)
        step.step()
        torch.cuda.synchronize()
        res.append(step.fluxes())
    for k in res[0]:
        np.testing.assert_array_equal(res[0][k], res[1][k], err_msg=k)


@pytest.mark.parametrize("ncol", [1, 37, 1800])
def test_fused_gas_optics_equals_separate_calls(dev, rfmip, ncol, mlp_kernel):
    """rrtmgpnn_gas_optics_{lw,sw}_nn (network inputs and col_dry formed inside the MLP kernel) == compute_nn_inputs +
    get_col_dry + predict_nn_{lw,sw}, bit for bit; the LW g128 'both' model (no in-kernel instance) takes the
    fallback through the context workspace and matches too."""
    from rrtmgpnn import _lib, data
    from rrtmgpnn._lib import check, ptr_array
    from rrtmgpnn.pipeline import ClearSkyStep
    prob = subset(rfmip, np.arange(ncol) * 7 % 1800)
    st = ClearSkyStep(prob, device=0, fused=False, overlap=False)
    # the step runs on its own streams: torch work on the arrays it hands its raw C calls is ordered on them too
    with torch.cuda.stream(st.ctx.stream):
        L, c, p = _lib.lib(), st.ctx.h, (lambda t: t.data_ptr())
        nl, nc = st.nlay, st.ncol
        for name in ("get_col_dry", "nn_inputs_lw", "predict_nn_lw", "nn_inputs_sw", "predict_nn_sw"):
            fn, args = next((f, a) for n, f, a in st.calls if n == name)
            check(fn(*args), name)
        torch.cuda.synchronize()
        ref = [t.clone() for t in (st.tau_lw, st.lay_src, st.tau_sw, st.ssa_sw)]
        got = [torch.full_like(t, float("nan")) for t in ref]
        check(L.rrtmgpnn_gas_optics_lw_nn(c, nc, nl, st.ng_lw, st.nx_lw, p(st.play), p(st.tlay), p(st.plev),
                                          p(st.gases["h2o"]), st._g_lw, st._nd_lw, st._nets_lw, len(st.lw_nets),
                                          p(got[0]), p(got[1])), "gas_optics_lw_nn")
        check(L.rrtmgpnn_gas_optics_sw_nn(c, nc, nl, st.ng_sw, st.nx_sw, p(st.play), p(st.tlay), p(st.plev),
                                          p(st.gases["h2o"]), st._g_sw, st._nd_sw, st._nets_sw, p(got[2]), p(got[3]), None),
              "gas_optics_sw_nn")
        torch.cuda.synchronize()
        for k, (a, b) in enumerate(zip(ref, got)):
            np.testing.assert_array_equal(a.cpu().numpy(), b.cpu().numpy(), err_msg=str(k))
        # the g128 single-output model (18-64-64-256, no in-kernel instance): nn_inputs + col_dry in the workspace
        from rrtmgpnn._lib import int_array
        hb = _lib.c_vp()
        check(L.rrtmgpnn_network_load(c, data.path("lw_g128_both").encode(), hb), "network_load")
        names = data.rbin.unchars(data.load_model("lw_g128_both")["input_names"])
        g_b = ptr_array([st.gases[n].data_ptr() if (k >= 2 and n in st.gases) else None for k, n in enumerate(names)])
        nd_b = int_array([2] * len(names))
        nets_b = ptr_array([hb.value])
        nx = len(names)
        x = torch.empty((nc, nl, nx), device=dev)
        cd = torch.empty((nc, nl), device=dev)
        out = [torch.full((nc, nl, 128), float("nan"), device=dev) for _ in range(4)]
        check(L.rrtmgpnn_compute_nn_inputs(c, nc, nl, nx, p(st.play), p(st.tlay), g_b, nd_b, hb, p(x)), "nn_inputs")
        check(L.rrtmgpnn_get_col_dry(c, nc, nl, p(st.gases["h2o"]), p(st.plev), p(cd)), "col_dry")
        check(L.rrtmgpnn_predict_nn_lw(c, nc, nl, 128, nx, p(x), p(cd), nets_b, 1, p(out[0]), p(out[1])), "predict")
        check(L.rrtmgpnn_gas_optics_lw_nn(c, nc, nl, 128, nx, p(st.play), p(st.tlay), p(st.plev), p(st.gases["h2o"]),
                                          g_b, nd_b, nets_b, 1, p(out[2]), p(out[3])), "gas_optics_lw_nn both")
        torch.cuda.synchronize()
        np.testing.assert_array_equal(out[0].cpu().numpy(), out[2].cpu().numpy())
        np.testing.assert_array_equal(out[1].cpu().numpy(), out[3].cpu().numpy())
        L.rrtmgpnn_network_destroy(hb)


@pytest.mark.parametrize("allsky", [False, True])
@pytest.mark.parametrize("lw_after", ["", "none", "sw_solver", "nets_first"])
def test_two_stream_overlap_is_bitwise_identical(dev, rfmip, allsky, lw_after):
    """LW and SW chains on two streams (forked at the start, joined at the end; the LW chain started after the SW
    network by default at this size, with both started together, or after the SW solver; or both networks first and
    the SW solver after both networks, on a high-priority stream), eager and as one hipGraph, give the
    single-stream step's fluxes bit for bit."""
    from rrtmgpnn import data
    from rrtmgpnn.pipeline import ClearSkyStep
    prob = subset(rfmip, np.arange(0, 1800, 4))
    clouds = data.allsky_clouds(prob, data.load_cloud_optics("lw")) if allsky else None
    one = ClearSkyStep(prob, device=0, clouds=clouds, overlap=False)
    nets_first = lw_after == "nets_first"
    two = ClearSkyStep(prob, device=0, clouds=clouds, overlap=True,
                       lw_after={"": None, "none": "", "sw_solver": "sw_solver", "nets_first": ""}[lw_after],
                       sw_after={"": None, "nets_first": "predict_nn_lw"}.get(lw_after, ""),
                       sw_priority=-1 if nets_first else 0)
    # default at this size (450 columns): the LW chain after the SW network
    assert two.lw_after == {"": "predict_nn_sw", "none": "", "sw_solver": "sw_solver", "nets_first": ""}[lw_after]
    assert two.sw_after == ("predict_nn_lw" if nets_first else "")
    # the LW network's CU cap is on whenever the LW chain is gated at this size (the default), off when the chains
    # start together, and the step records the cap the context actually holds
    assert (two.lw_net_cus > 0) == bool(two.lw_after)
    assert two.lw_net_cus == two.ctx.mlp_max_cus()
    one.step()
    two.step()
    torch.cuda.synchronize()
    a, b = one.fluxes(), two.fluxes()
    two.capture()
    for t in (two.lw_up, two.lw_dn, two.sw_up, two.sw_dn, two.sw_dir):
        t.fill_(float("nan"))
    for _ in range(3):
        two.replay()
    torch.cuda.synchronize()
    c = two.fluxes()
    for k in a:
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
        np.testing.assert_array_equal(a[k], c[k], err_msg=k)


@pytest.mark.gpu
@pytest.mark.parametrize("allsky", [False, True])
def test_lw_only_step_equals_lw_half(dev, rfmip, allsky):
    """Config C2 (bench.py --config c2): the LW half alone, eager and as a hipGraph, gives the LW fluxes of the full
    LW+SW step bit for bit, and issues no SW launch."""
    from rrtmgpnn import data
    from rrtmgpnn.pipeline import ClearSkyStep
    prob = subset(rfmip, np.arange(0, 1800, 6))
    clouds = data.allsky_clouds(prob, data.load_cloud_optics("lw")) if allsky else None
    full = ClearSkyStep(prob, device=0, clouds=clouds)
    lw = ClearSkyStep(prob, device=0, clouds=clouds, sw=False)
    assert not lw.overlap and all("sw" not in name for name, _, _ in lw.calls)
    full.step()
    lw.step()
    torch.cuda.synchronize()
    a, b = full.fluxes(), lw.fluxes()
    lw.capture()
    lw.lw_up.fill_(float("nan"))
    lw.lw_dn.fill_(float("nan"))
    lw.replay()
    torch.cuda.synchronize()
    c = lw.fluxes()
    for k in ("lw_up", "lw_dn"):
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
        np.testing.assert_array_equal(a[k], c[k], err_msg=k)


def test_captured_graph_pins_context_workspace(dev, rfmip):
    """A hipGraph captured on a context holds the address of its workspace: a later, larger call on the same context
    must fail loudly instead of freeing memory the graph still writes; the graph keeps replaying
    correctly, and unpinning after the graph is gone lets the workspace grow again."""
    from rrtmgpnn._lib import RrtmgpnnError
    from rrtmgpnn.api import Context
    from rrtmgpnn.pipeline import ClearSkyStep
    ctx = Context(0)
    # one stream: the SW solver (the step's workspace user) then runs on ctx
    small = ClearSkyStep(subset(rfmip, np.arange(0, 64)), device=0, ctx=ctx, overlap=False)
    small.capture()
    small.replay()
    torch.cuda.synchronize()
    ref = small.fluxes()
    big = ClearSkyStep(subset(rfmip, np.arange(0, 1800, 2)), device=0, ctx=ctx, overlap=False)
    with pytest.raises(RrtmgpnnError, match="pinned"):
        big.step()
    torch.cuda.synchronize()
    for t in (small.sw_up, small.sw_dn, small.lw_up):
        t.fill_(float("nan"))
    small.replay()
    torch.cuda.synchronize()
    got = small.fluxes()
    for k in ref:
        np.testing.assert_array_equal(got[k], ref[k])
    del small.graph
    ctx.unpin_workspace()
    big.step()
    torch.cuda.synchronize()
    assert np.isfinite(big.fluxes()["sw_dn"]).all()

def test_fused_gas_optics_special_pressures(dev, rfmip, mlp_kernel):
    """log(play) in the fused kernels: the 32x32x2 kernel takes it through the branch-free ref_logf_nb, the separate
    compute_nn_inputs kernel through ref_logf (glibc's branches).  With zero, negative, subnormal, one, huge, inf and
    nan pressures in one column the two give the same tau / pfrac / ssa bits (nan where glibc's logf gives nan)."""
    from rrtmgpnn import _lib
    from rrtmgpnn.pipeline import ClearSkyStep
    from rrtmgpnn._lib import check
    prob = subset(rfmip, np.arange(37) * 11 % 1800)
    st = ClearSkyStep(prob, device=0, fused=False, overlap=False)
    # the step runs on its own streams: torch work on the arrays it hands its raw C calls is ordered on them too
    with torch.cuda.stream(st.ctx.stream):
        special = np.array([0.0, -0.0, 1.0, 1e-40, 1.4e-45, 1.17549435e-38, -5.0, np.inf, -np.inf, np.nan, 3.4e38, 1e-30,
                            0.5, 2.0, 100.0, 1.0000001], np.float32)
        play = st.play.view(st.ncol, st.nlay)
        play[3, :len(special)] = torch.as_tensor(special, device=dev)
        L, c, p = _lib.lib(), st.ctx.h, (lambda t: t.data_ptr())
        nl, nc = st.nlay, st.ncol
        for name in ("get_col_dry", "nn_inputs_lw", "predict_nn_lw", "nn_inputs_sw", "predict_nn_sw"):
            fn, args = next((f, a) for n, f, a in st.calls if n == name)
            check(fn(*args), name)
        torch.cuda.synchronize()
        ref = [t.clone() for t in (st.tau_lw, st.lay_src, st.tau_sw, st.ssa_sw)]
        got = [torch.full_like(t, 7.0) for t in ref]
        check(L.rrtmgpnn_gas_optics_lw_nn(c, nc, nl, st.ng_lw, st.nx_lw, p(st.play), p(st.tlay), p(st.plev),
                                          p(st.gases["h2o"]), st._g_lw, st._nd_lw, st._nets_lw, len(st.lw_nets),
                                          p(got[0]), p(got[1])), "gas_optics_lw_nn")
        check(L.rrtmgpnn_gas_optics_sw_nn(c, nc, nl, st.ng_sw, st.nx_sw, p(st.play), p(st.tlay), p(st.plev),
                                          p(st.gases["h2o"]), st._g_sw, st._nd_sw, st._nets_sw, p(got[2]), p(got[3]), None),
              "gas_optics_sw_nn")
        torch.cuda.synchronize()
        for k, (a, b) in enumerate(zip(ref, got)):
            a, b = a.cpu().numpy(), b.cpu().numpy()
            assert np.isnan(a).any() == np.isnan(b).any(), k
            np.testing.assert_array_equal(a.view(np.uint32)[~np.isnan(a)], b.view(np.uint32)[~np.isnan(b)], err_msg=str(k))
            np.testing.assert_array_equal(np.isnan(a), np.isnan(b), err_msg=str(k))


@pytest.mark.parametrize("nlay", [1, 7, 37, 64, 65, 71, 137])
@pytest.mark.parametrize("top_at_1", [True, False])
@pytest.mark.parametrize("lw_ds", [False, True])
def test_fused_lw_any_nlay(dev, orc, nlay, top_at_1, lw_ds):
    """The one-angle fused LW solver on synthetic columns of 1 to 137 layers (odd and even, shorter and longer than
    its ring of 8 levels and its prefetch depth, the C5 depth) in both orientations, with and without rte_lw's lw_Ds,
    against the oracle."""
    from rrtmgpnn import _lib, data
    from rrtmgpnn._lib import check, float_array, int_array
    from rrtmgpnn.api import GAUSS_DS, GAUSS_WTS, context
    prob = data.synthetic_problem(23, nlay, seed=11)
    if not top_at_1:
        prob = _flip(prob)
    kd = data.load_kdist("lw")
    go = orc.lw_gas_optics(prob, [data.load_model("lw_abs"), data.load_model("lw_pfrac")], kd)
    ncol, _, ngpt = go["tau"].shape
    emis = np.repeat(np.asarray(prob["sfc_emis"], np.float32)[:, None], ngpt, axis=1)
    ds = (np.random.default_rng(nlay).uniform(1.0, 2.5, size=ngpt * ncol).astype(np.float32) if lw_ds else None)
    up_o, dn_o = orc.lw_solver(go["tau"], go["lay_source"], go["lev_source"], emis, go["sfc_source"], top_at_1, 1,
                               lw_Ds=ds)
    sfc_lay = 1 if prob["play"][0, 0] > prob["play"][0, nlay - 1] else nlay
    up, dn = torch.full((ncol, nlay + 1), float("nan"), device=dev), torch.full((ncol, nlay + 1), float("nan"),
                                                                               device=dev)
    args = [T(go["tau"], dev), T(go["pfrac"], dev), T(prob["tlay"], dev), T(prob["tlev"], dev), T(prob["tsfc"], dev),
            T(kd["totplnk"], dev), T(emis, dev)]
    dsd = T(ds, dev) if lw_ds else None
    check(_lib.lib().rrtmgpnn_lw_solver_noscat_planck_gpt(
        context(0).h, ngpt, nlay, ncol, int(top_at_1), 1, float_array(GAUSS_DS[1]), float_array(GAUSS_WTS[1]),
        dsd.data_ptr() if lw_ds else None, None, args[0].data_ptr(), args[1].data_ptr(), kd["nband"],
        kd["nPlanckTemp"], args[2].data_ptr(), args[3].data_ptr(), args[4].data_ptr(), sfc_lay,
        int_array(kd["band_lims_gpt"].ravel()), float(kd["temp_ref_min"][0]), float(kd["totplnk_delta"]),
        args[5].data_ptr(), 0, args[6].data_ptr(), up.data_ptr(), dn.data_ptr(), None, None),
        "lw_solver_noscat_planck_gpt")
    torch.cuda.synchronize()
    np.testing.assert_array_equal(up.cpu().numpy(), up_o)
    np.testing.assert_array_equal(dn.cpu().numpy(), dn_o)


@pytest.mark.parametrize("cap", ["1", "eighth"])
def test_network_cu_cap_is_bitwise(dev, rfmip, cap, mlp_kernel):
    """rrtmgpnn_context_set_mlp_max_cus: the fused gas-optics networks (LW pair, SW pair) on one CU's worth of blocks
    (every wave strides many tiles) or an eighth of the chip give the uncapped outputs bit for bit, for both MFMA
    tilings."""
    from rrtmgpnn import _lib
    from rrtmgpnn._lib import check
    from rrtmgpnn.pipeline import ClearSkyStep
    prob = subset(rfmip, np.arange(0, 1800, 4))
    st = ClearSkyStep(prob, device=0, overlap=False)
    # the step runs on its own streams: torch work on the arrays it hands its raw C calls is ordered on them too
    with torch.cuda.stream(st.ctx.stream):
        assert st.lw_net_cus == 0 and st.ctx.mlp_max_cus() == 0
        calls = [(n, f, a) for n, f, a in st.calls if n in ("predict_nn_lw", "predict_nn_sw")]
        outs = (st.tau_lw, st.lay_src, st.tau_sw, st.ssa_sw)

        def run():
            for t in outs:
                t.fill_(float("nan"))
            for n, f, a in calls:
                check(f(*a), n)
            torch.cuda.synchronize()
            return [t.cpu().numpy().copy() for t in outs]

        ref = run()
        cus = torch.cuda.get_device_properties(0).multi_processor_count
        n = 1 if cap == "1" else max(1, cus // 8)
        st.ctx.set_mlp_max_cus(n)
        assert st.ctx.mlp_max_cus() == n
        got = run()
        st.ctx.set_mlp_max_cus(0)
        for k, (a, b) in enumerate(zip(ref, got)):
            assert np.isfinite(a).all()
            np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32), err_msg=str(k))
        with pytest.raises(ValueError):
            ClearSkyStep(prob, device=0, overlap=False, lw_net_cus=64)


def test_set_stream_inside_a_global_capture(dev, rfmip):
    """rrtmgpnn_context_set_stream called while the NEW stream is being captured into a hipGraph (global capture mode):
    the context's old stream is idle and not capturing, so set_stream synchronises it; the call must succeed, the
    kernel issued next must be captured, and the replay must give the eager result bit for bit."""
    from rrtmgpnn.api import Context
    from rrtmgpnn.pipeline import ClearSkyStep
    prob = subset(rfmip, np.arange(1, 1800, 9))
    # a caller's context on torch's current stream (the legacy null stream), as a class-layer user holds it
    st = ClearSkyStep(prob, device=0, overlap=False, ctx=Context(0))
    st.step()
    torch.cuda.synchronize()
    ref = st.fluxes()
    old = st.ctx.stream
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s, capture_error_mode="global"):
            st.ctx.use_stream(s)  # inside the capture
            st.step()
    st.ctx.use_stream(old)
    for t in (st.lw_up, st.lw_dn, st.sw_up, st.sw_dn, st.sw_dir):
        t.fill_(float("nan"))
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    got = st.fluxes()
    for k in ref:
        np.testing.assert_array_equal(ref[k], got[k], err_msg=k)

