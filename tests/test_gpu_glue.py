"""GPU parity of the gas-optics glue branches the benchmarked step does not take, through the C ABI and the class
layer, against the oracle (bit for bit):

  * gas_optics_int without tlev: rrtmgpnn_interpolate_tlev (rrtmgp/mo_gas_optics_rrtmgp.F90:317-337) and the
    level Planck sources built on it;
  * the optional col_dry= argument (quirk B-3 fixed: honoured) in the LW and SW branches;
  * scalar and 1-D gas concentrations (compute_nn_inputs :724-753) in the class layer and in the fused entries;
  * the single-model ("both") LW network: predict_nn_lw_blas_sp's output_sgemm_lw branch
    (mo_gas_optics_kernels.F90:744-772), in predict_nn_lw and in the fused entry (workspace fallback);
  * the SURVEY 0.4 reference probe (RFMIP column 0) reproduced by the benchmarked GPU step.
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


@pytest.fixture(scope="module")
def models():
    from rrtmgpnn import data
    return {k: data.load_model(k) for k in ("lw_abs", "lw_pfrac", "sw_abs", "sw_ray", "lw_g128_both")}


def T(a, dev):
    return torch.as_tensor(np.ascontiguousarray(a, dtype=np.float32), device=dev)


def _flip(prob):
    out = dict(prob)
    for k in ("play", "plev", "tlay", "tlev"):
        out[k] = np.ascontiguousarray(prob[k][:, ::-1])
    out["gases"] = {k: np.ascontiguousarray(v[:, ::-1]) for k, v in prob["gases"].items()}
    out["top_at_1"] = False
    return out


def _lw_class_layer(dev, prob, gases=None, col_dry=None, tlev=True, nets=("lw_abs", "lw_pfrac")):
    from rrtmgpnn import api, data
    ncol, nlay = prob["ncol"], prob["nlay"]
    kd = api.GasOpticsRRTMGP()
    api.stop_on_err(kd.load("lw"))
    nn = [api.RrtmgpNetwork(0).load_netcdf(data.path(n)) for n in nets]
    gases = prob["gases"] if gases is None else gases
    gc = api.GasConcs()
    api.stop_on_err(gc.init(list(gases)))
    for k, v in gases.items():
        api.stop_on_err(gc.set_vmr(k, float(v) if np.ndim(v) == 0 else T(v, dev)))
    op = api.OpticalProps1scl()
    api.stop_on_err(op.alloc_1scl(ncol, nlay, kd))
    src = api.SourceFuncLW()
    api.stop_on_err(src.alloc(ncol, nlay, kd))
    kw = {"neural_nets": nn}
    if tlev:
        kw["tlev"] = T(prob["tlev"], dev)
    if col_dry is not None:
        kw["col_dry"] = T(col_dry, dev)
    api.stop_on_err(kd.gas_optics(T(prob["play"], dev), T(prob["plev"], dev), T(prob["tlay"], dev),
                                  T(prob["tsfc"], dev), gc, op, src, **kw))
    return op, src


@pytest.mark.parametrize("top_at_1", [True, False])
def test_interpolate_tlev_matches_oracle(dev, orc, rfmip, top_at_1):
    from rrtmgpnn import _lib
    from rrtmgpnn._lib import check
    from rrtmgpnn.api import context
    prob = subset(rfmip, np.arange(0, 1800, 3))
    if not top_at_1:
        prob = _flip(prob)
    ncol, nlay = prob["ncol"], prob["nlay"]
    out = torch.full((ncol, nlay + 1), -1.0, device=dev)
    pa, pv, ta = T(prob["play"], dev), T(prob["plev"], dev), T(prob["tlay"], dev)  # alive until the kernel ran
    check(_lib.lib().rrtmgpnn_interpolate_tlev(context(0).h, ncol, nlay, pa.data_ptr(), pv.data_ptr(), ta.data_ptr(),
                                                 out.data_ptr()), "interpolate_tlev")
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy(), orc.interpolate_tlev(prob["play"], prob["plev"], prob["tlay"]))


@pytest.mark.parametrize("top_at_1", [True, False])
def test_gas_optics_without_tlev_matches_oracle(dev, orc, rfmip, models, top_at_1):
    from rrtmgpnn import data
    prob = subset(rfmip, np.arange(1, 1800, 9))
    if not top_at_1:
        prob = _flip(prob)
    ref = orc.lw_gas_optics(prob, [models["lw_abs"], models["lw_pfrac"]], data.load_kdist("lw"), tlev=False)
    op, src = _lw_class_layer(dev, prob, tlev=False)
    np.testing.assert_array_equal(op.tau.cpu().numpy(), ref["tau"])
    np.testing.assert_array_equal(src.lev_source.cpu().numpy(), ref["lev_source"])
    np.testing.assert_array_equal(src.lay_source.cpu().numpy(), ref["lay_source"])
    np.testing.assert_array_equal(src.sfc_source.cpu().numpy(), ref["sfc_source"])


def test_lw_gas_optics_user_col_dry(dev, orc, rfmip, models, mlp_kernel):
    from rrtmgpnn import data
    prob = subset(rfmip, np.arange(2, 1800, 11))
    rng = np.random.default_rng(5)
    cd = (orc.col_dry(prob["gases"]["h2o"], prob["plev"]) *
          rng.uniform(0.5, 2.0, size=(prob["ncol"], prob["nlay"]))).astype(np.float32)
    ref = orc.lw_gas_optics(prob, [models["lw_abs"], models["lw_pfrac"]], data.load_kdist("lw"), col_dry=cd)
    op, src = _lw_class_layer(dev, prob, col_dry=cd)
    np.testing.assert_array_equal(op.tau.cpu().numpy(), ref["tau"])
    np.testing.assert_array_equal(src.lay_source.cpu().numpy(), ref["lay_source"])


def test_sw_gas_optics_user_col_dry(dev, orc, rfmip, models, mlp_kernel):
    from rrtmgpnn import api, data
    prob = subset(rfmip, np.arange(4, 1800, 13))
    ncol, nlay = prob["ncol"], prob["nlay"]
    rng = np.random.default_rng(6)
    cd = (orc.col_dry(prob["gases"]["h2o"], prob["plev"]) * rng.uniform(0.5, 2.0, size=(ncol, nlay))).astype(np.float32)
    x = orc.nn_inputs(prob["play"], prob["tlay"], prob["gases"], models["sw_abs"]).reshape(-1, 7)
    tau = orc.tau_post(models["sw_abs"], orc.mlp(models["sw_abs"], x), cd)
    ssa = orc.tau_post(models["sw_ray"], orc.mlp(models["sw_ray"], x), cd, tau_abs_to_tot=tau)
    kd = api.GasOpticsRRTMGP()
    api.stop_on_err(kd.load("sw"))
    nets = [api.RrtmgpNetwork(0).load_netcdf(data.path(n)) for n in ("sw_abs", "sw_ray")]
    gc = api.GasConcs()
    names = ["h2o", "o3", "co2", "n2o", "ch4"]
    api.stop_on_err(gc.init(names))
    for k in names:
        api.stop_on_err(gc.set_vmr(k, T(prob["gases"][k], dev)))
    op = api.OpticalProps2str()
    api.stop_on_err(op.alloc_2str(ncol, nlay, kd))
    toa = torch.empty((ncol, kd.get_ngpt()), device=dev)
    api.stop_on_err(kd.gas_optics(T(prob["play"], dev), T(prob["plev"], dev), T(prob["tlay"], dev), gc, op, toa,
                                  col_dry=T(cd, dev), neural_nets=nets))
    np.testing.assert_array_equal(op.tau.cpu().numpy().reshape(-1, 224), tau)
    np.testing.assert_array_equal(op.ssa.cpu().numpy().reshape(-1, 224), ssa)


def _scalar_1d_gases(prob):
    g = dict(prob["gases"])
    g["co2"] = np.float32(4.1e-4)                                                # scalar
    g["ch4"] = np.linspace(1.6e-6, 1.9e-6, prob["nlay"], dtype=np.float32)      # (nlay)
    g["n2o"] = np.float32(3.2e-7)
    return g


def test_class_layer_scalar_and_1d_gases(dev, orc, rfmip, models):
    from rrtmgpnn import data
    prob = subset(rfmip, np.arange(0, 1800, 17))
    g = _scalar_1d_gases(prob)
    ref = orc.lw_gas_optics(dict(prob, gases=g), [models["lw_abs"], models["lw_pfrac"]], data.load_kdist("lw"))
    op, src = _lw_class_layer(dev, prob, gases=g)
    np.testing.assert_array_equal(op.tau.cpu().numpy(), ref["tau"])
    np.testing.assert_array_equal(src.lay_source.cpu().numpy(), ref["lay_source"])


@pytest.mark.parametrize("stream", ["lw", "sw"])
def test_fused_gas_optics_scalar_and_1d_gases(dev, orc, rfmip, models, stream, mlp_kernel):
    """rrtmgpnn_gas_optics_{lw,sw}_nn (the benchmarked entries) with gas_ndims 0 and 1."""
    from rrtmgpnn import _lib, data
    from rrtmgpnn._lib import check, int_array, ptr_array
    from rrtmgpnn.api import context
    prob = subset(rfmip, np.arange(7, 1800, 19))
    ncol, nlay = prob["ncol"], prob["nlay"]
    g = _scalar_1d_gases(prob)
    names = data.rbin.unchars(models[stream + "_abs"]["input_names"])
    keep, ptrs, nds = [], [], []
    for k, n in enumerate(names):
        if k < 2 or n not in g:
            ptrs.append(None)
            nds.append(2)
            continue
        t = T(np.atleast_1d(g[n]), dev)
        keep.append(t)
        ptrs.append(t.data_ptr())
        nds.append(int(np.ndim(g[n])))
    L = _lib.lib()
    h = [_lib.c_vp(), _lib.c_vp()]
    pair = ("lw_abs", "lw_pfrac") if stream == "lw" else ("sw_abs", "sw_ray")
    for i, n in enumerate(pair):
        check(L.rrtmgpnn_network_load(context(0).h, data.path(n).encode(), h[i]), "network_load")
    ng = 256 if stream == "lw" else 224
    o1, o2 = torch.empty((ncol, nlay, ng), device=dev), torch.empty((ncol, nlay, ng), device=dev)
    state = [T(prob["play"], dev), T(prob["tlay"], dev), T(prob["plev"], dev), T(g["h2o"], dev)]
    keep += state  # device arrays must outlive the asynchronous launches
    args = (context(0).h, ncol, nlay, ng, len(names)) + tuple(t.data_ptr() for t in state) + (
        ptr_array(ptrs), int_array(nds), ptr_array([x.value for x in h]))
    x = orc.nn_inputs(prob["play"], prob["tlay"], g, models[pair[0]]).reshape(-1, len(names))
    cd = orc.col_dry(prob["gases"]["h2o"], prob["plev"])
    if stream == "lw":
        check(L.rrtmgpnn_gas_optics_lw_nn(*args, 2, o1.data_ptr(), o2.data_ptr()), "gas_optics_lw_nn")
        r1 = orc.tau_post(models["lw_abs"], orc.mlp(models["lw_abs"], x), cd)
        r2 = orc.mlp(models["lw_pfrac"], x)
        r2 = r2 * r2
    else:
        check(L.rrtmgpnn_gas_optics_sw_nn(*args, o1.data_ptr(), o2.data_ptr(), None), "gas_optics_sw_nn")
        r1 = orc.tau_post(models["sw_abs"], orc.mlp(models["sw_abs"], x), cd)
        r2 = orc.tau_post(models["sw_ray"], orc.mlp(models["sw_ray"], x), cd, tau_abs_to_tot=r1)
    torch.cuda.synchronize()
    for hh in h:
        L.rrtmgpnn_network_destroy(hh)
    np.testing.assert_array_equal(o1.cpu().numpy().reshape(-1, ng), r1)
    np.testing.assert_array_equal(o2.cpu().numpy().reshape(-1, ng), r2)


@pytest.mark.parametrize("fused", [False, True])
def test_both_model_matches_oracle(dev, orc, rfmip, models, fused, mlp_kernel):
    """The g128 single-model network (2*128 outputs): tau and pfrac split as mo_gas_optics_kernels.F90:744-772."""
    from rrtmgpnn import _lib, data
    from rrtmgpnn._lib import check, int_array, ptr_array
    from rrtmgpnn.api import context
    m = models["lw_g128_both"]
    prob = subset(rfmip, np.arange(3, 1800, 23))
    ncol, nlay = prob["ncol"], prob["nlay"]
    names = data.rbin.unchars(m["input_names"])
    x = orc.nn_inputs(prob["play"], prob["tlay"], prob["gases"], m)
    cd = orc.col_dry(prob["gases"]["h2o"], prob["plev"])
    tau_o, pf_o = orc.both_post(m, orc.mlp(m, x.reshape(-1, len(names))), cd)
    L = _lib.lib()
    h = _lib.c_vp()
    check(L.rrtmgpnn_network_load(context(0).h, data.path("lw_g128_both").encode(), h), "network_load")
    tau, pf = torch.empty((ncol, nlay, 128), device=dev), torch.empty((ncol, nlay, 128), device=dev)
    if fused:
        keep, ptrs = [], []
        for k, n in enumerate(names):
            t = T(prob["gases"][n], dev) if k >= 2 and n in prob["gases"] else None
            keep.append(t)
            ptrs.append(t.data_ptr() if t is not None else None)
        state = [T(prob["play"], dev), T(prob["tlay"], dev), T(prob["plev"], dev)]
        check(L.rrtmgpnn_gas_optics_lw_nn(context(0).h, ncol, nlay, 128, len(names), state[0].data_ptr(),
                                          state[1].data_ptr(), state[2].data_ptr(),
                                          keep[2].data_ptr(),  # input 3 is h2o (compute_nn_inputs :709-710)
                                          ptr_array(ptrs), int_array([2] * len(names)), ptr_array([h.value]), 1,
                                          tau.data_ptr(), pf.data_ptr()), "gas_optics_lw_nn(both)")
        torch.cuda.synchronize()
    else:
        xd, cdd = T(x, dev), T(cd, dev)
        check(L.rrtmgpnn_predict_nn_lw(context(0).h, ncol, nlay, 128, len(names), xd.data_ptr(), cdd.data_ptr(),
                                       ptr_array([h.value]), 1, tau.data_ptr(), pf.data_ptr()), "predict_nn_lw(both)")
    torch.cuda.synchronize()
    L.rrtmgpnn_network_destroy(h)
    np.testing.assert_array_equal(tau.cpu().numpy().reshape(-1, 128), tau_o)
    np.testing.assert_array_equal(pf.cpu().numpy().reshape(-1, 128), pf_o)


def test_benchmarked_step_reproduces_reference_probe(dev, rfmip):
    """the reference's own glue + solvers printed LW TOA up 289.75 / surface down 339.35 and, with a flat
    solar_source, SW TOA down 757.35 / TOA up 56.82 / surface down 225.74 for RFMIP column 0 (tests/test_glue_oracle)."""
    from rrtmgpnn import data
    from rrtmgpnn.pipeline import ClearSkyStep
    prob = subset(rfmip, [0, 1, 2, 3])
    step = ClearSkyStep(prob, device=0)
    # the probe's flat solar source, after set_tsi; the step renormalises it to each column's TSI itself
    step.solar_source.copy_(T(data.set_tsi(np.ones(224, np.float32), 1361.0), dev))
    step.step()
    torch.cuda.synchronize()
    f = step.fluxes()
    for got, want in ((f["lw_up"][0, 0], 289.75), (f["lw_dn"][0, -1], 339.35), (f["sw_dn"][0, 0], 757.35),
                      (f["sw_up"][0, 0], 56.82), (f["sw_dn"][0, -1], 225.74)):
        assert abs(float(got) - want) <= 6e-3, (float(got), want)


@pytest.mark.parametrize("which", ["rfmip", "synthetic", "sweep"])
def test_sw_boundary_conditions_match_the_driver(dev, which):
    """rrtmgpnn_sw_boundary_rfmip (the step's per-block SW boundary conditions, rrtmgp_rfmip_sw.F90:403-434) against the
    host's restatement of the same driver lines, bit for bit: toa_flux = solar_source * tsi / def_tsi (data.toa_flux,
    def_tsi summed in g order), the albedo expanded to every g-point, mu0 = merge(cos(sza deg_to_rad), 1, usecol) with
    glibc's cosf (data.ref_cosf).  'sweep': 2 M zenith angles spread over every float exponent of (0, 180) degrees,
    night columns included (usecol false: mu0 = 1)."""
    from rrtmgpnn import _lib, data
    from rrtmgpnn._lib import check
    from rrtmgpnn.api import context
    kd = data.load_kdist("sw")
    if which == "rfmip":
        prob = data.rfmip_problem()
    elif which == "synthetic":
        prob = data.synthetic_problem(3001, 60, seed=5)
    else:
        u = np.arange(np.float32(1e-6).view(np.uint32), np.float32(180.0).view(np.uint32), 541, dtype=np.uint32)
        sza = u.view(np.float32)
        n = sza.size
        rng = np.random.default_rng(3)
        usecol = sza < np.float32(90.0) - np.float32(2.0) * data.spacing(90.0)
        deg_to_rad = np.float32(np.arccos(np.float32(-1.0)) / np.float32(180.0))
        prob = {"ncol": n, "sza": sza, "tsi": rng.uniform(1300, 1400, n).astype(np.float32),
                "sfc_alb": rng.uniform(0, 1, n).astype(np.float32),
                "mu0": np.where(usecol, data.ref_cosf(sza * deg_to_rad), np.float32(1.0)).astype(np.float32)}
    ncol, ngpt = prob["ncol"], int(kd["ngpt"])
    sol = T(data.set_tsi(kd["solar_source"], 1361.0), dev)
    ins = [T(prob[k], dev) for k in ("tsi", "sfc_alb", "sza")]
    toa, alb = (torch.full((ncol, ngpt), float("nan"), device=dev) for _ in range(2))
    mu0 = torch.full((ncol,), float("nan"), device=dev)
    check(_lib.lib().rrtmgpnn_sw_boundary_rfmip(context(0).h, ngpt, ncol, sol.data_ptr(), *[t.data_ptr() for t in ins],
                                                toa.data_ptr(), alb.data_ptr(), mu0.data_ptr()), "sw_boundary_rfmip")
    torch.cuda.synchronize()
    np.testing.assert_array_equal(mu0.cpu().numpy().view(np.uint32), prob["mu0"].view(np.uint32))
    np.testing.assert_array_equal(toa.cpu().numpy().view(np.uint32), data.toa_flux(prob, kd).view(np.uint32))
    np.testing.assert_array_equal(alb.cpu().numpy(), np.repeat(prob["sfc_alb"][:, None], ngpt, axis=1))


@pytest.mark.parametrize("case", ["clear_small", "clear_large", "g", "allsky", "one_column", "one_layer"])
@pytest.mark.parametrize("top_at_1", [True, False])
def test_sw_solver_rfmip_equals_boundary_then_solver(dev, case, top_at_1, sw_kernel):
    """rrtmgpnn_sw_solver_2stream_rfmip (the boundary conditions formed in the checkpointed solver's prologue; the
    other kernels get them from sw_boundary_kernel first) == rrtmgpnn_sw_boundary_rfmip then
    rrtmgpnn_sw_solver_2stream[_inc], bit for bit: the small-grid and large-grid clear-sky instances (g = NULL), a
    non-zero g, the fused cloud increment; night columns (mu0 = 1) among random zenith angles."""
    from rrtmgpnn import _lib, data
    from rrtmgpnn._lib import check, int_array
    from rrtmgpnn.api import context
    L = _lib.lib()
    ks = data.load_kdist("sw")
    ng, nb = int(ks["ngpt"]), int(ks["nband"])
    ncol, nlay = {"clear_small": (300, 40), "clear_large": (3001, 12), "g": (257, 30), "allsky": (190, 33),
                  "one_column": (1, 7), "one_layer": (5, 1)}[case]
    rng = np.random.default_rng(11 + 2 * top_at_1 + len(case))
    t = lambda a: T(a, dev)  # noqa: E731
    tau = t(rng.lognormal(-2, 2, (ncol, nlay, ng)))
    ssa = t(rng.uniform(0, 1, (ncol, nlay, ng)))
    gg = t(rng.uniform(0, 0.8, (ncol, nlay, ng))) if case == "g" else None
    sol = t(data.set_tsi(ks["solar_source"], 1361.0))
    sza = t(np.where(rng.uniform(size=ncol) < 0.15, rng.uniform(90, 180, ncol), rng.uniform(0, 89.9, ncol)))
    tsi = t(rng.uniform(1300, 1400, ncol))
    alb = t(rng.uniform(0, 1, ncol))
    if case == "allsky":
        lims = int_array(ks["band_lims_gpt"].ravel())
        cl = rng.uniform(size=(ncol, nlay, nb)) < 0.4
        s = (ncol, nlay, nb)
        bnd = [t(np.where(cl, rng.lognormal(0, 1, s), 0)), t(np.where(cl, rng.uniform(0.5, 1, s), 0)),
               t(np.where(cl, rng.uniform(0, 0.9, s), 0))]
        bargs = (nb, lims) + tuple(b.data_ptr() for b in bnd)
    else:
        bargs = (0, None, None, None, None)
    f = lambda *s: torch.full(s, float("nan"), device=dev)  # noqa: E731
    toa, albg, mu0 = f(ncol, ng), f(ncol, ng), f(ncol)
    ctx = context(0).h
    gp = gg.data_ptr() if gg is not None else None
    outs = [[f(ncol, nlay + 1) for _ in range(3)] for _ in range(2)]
    check(L.rrtmgpnn_sw_solver_2stream_rfmip(ctx, ng, nlay, ncol, int(top_at_1), sol.data_ptr(), tsi.data_ptr(),
                                             alb.data_ptr(), sza.data_ptr(), tau.data_ptr(), ssa.data_ptr(), gp, *bargs,
                                             toa.data_ptr(), albg.data_ptr(), mu0.data_ptr(),
                                             *[o.data_ptr() for o in outs[0]]), "sw_solver_2stream_rfmip")
    check(L.rrtmgpnn_sw_boundary_rfmip(ctx, ng, ncol, sol.data_ptr(), tsi.data_ptr(), alb.data_ptr(), sza.data_ptr(),
                                       toa.data_ptr(), albg.data_ptr(), mu0.data_ptr()), "sw_boundary_rfmip")
    if case == "allsky":
        check(L.rrtmgpnn_sw_solver_2stream_inc(ctx, ng, nlay, ncol, int(top_at_1), toa.data_ptr(), None, tau.data_ptr(),
                                               ssa.data_ptr(), gp, *bargs, mu0.data_ptr(), albg.data_ptr(),
                                               albg.data_ptr(), *[o.data_ptr() for o in outs[1]]), "sw_solver_2stream_inc")
    else:
        check(L.rrtmgpnn_sw_solver_2stream(ctx, ng, nlay, ncol, int(top_at_1), toa.data_ptr(), None, tau.data_ptr(),
                                           ssa.data_ptr(), gp, mu0.data_ptr(), albg.data_ptr(), albg.data_ptr(),
                                           *[o.data_ptr() for o in outs[1]]), "sw_solver_2stream")
    torch.cuda.synchronize()
    if ncol > 20:
        assert (mu0 == 1).any() and (mu0 < 1).any()
    for a, b, name in zip(outs[0], outs[1], ("up", "dn", "dir")):
        assert not torch.isnan(a).any(), name
        np.testing.assert_array_equal(a.cpu().numpy().view(np.uint32), b.cpu().numpy().view(np.uint32), err_msg=name)
