"""GPU: ty_fluxes_flexible g-point outputs and rte_lw's lw_Ds (rrtmgpnn_lw_solver_noscat_gpt,
rrtmgpnn_lw_solver_noscat_planck_gpt, rrtmgpnn_sw_solver_2stream_gpt) against the oracle, bit for bit.  The oracle's
g-point outputs and lw_Ds path are pinned to the reference's own rte_lw / rte_sw (tests/test_oracle.py)."""
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
    return torch.as_tensor(np.ascontiguousarray(a, dtype=np.float32), device=dev)


def _lw_inputs(orc, rfmip, top_at_1):
    """RFMIP columns (flipped to bottom-first for top_at_1 = False) and their oracle gas optics and sources."""
    from rrtmgpnn import data
    prob = subset(rfmip, np.arange(4, 1800, 41))
    if not top_at_1:
        prob = dict(prob)
        for k in ("play", "plev", "tlay", "tlev"):
            prob[k] = np.ascontiguousarray(prob[k][:, ::-1])
        prob["gases"] = {k: np.ascontiguousarray(v[:, ::-1]) for k, v in prob["gases"].items()}
        prob["top_at_1"] = False
    kd = data.load_kdist("lw")
    go = orc.lw_gas_optics(prob, [data.load_model("lw_abs"), data.load_model("lw_pfrac")], kd)
    return prob, kd, go


@pytest.mark.parametrize("top_at_1", [True, False])
@pytest.mark.parametrize("case", ["nmus1", "nmus2", "nmus3", "lw_ds", "lw_ds_gpt"])
def test_lw_gpt_and_lw_ds_match_oracle(dev, orc, rfmip, top_at_1, case):
    from rrtmgpnn import _lib
    from rrtmgpnn._lib import check, float_array
    from rrtmgpnn.api import GAUSS_DS, GAUSS_WTS, context
    prob, kd, go = _lw_inputs(orc, rfmip, top_at_1)
    ncol, nlay, ngpt = go["tau"].shape
    rng = np.random.default_rng(3)
    emis = rng.uniform(0.8, 1.0, size=(ncol, ngpt)).astype(np.float32)
    nmus = int(case[-1]) if case.startswith("nmus") else 1
    ds = rng.uniform(1.0, 2.5, size=ngpt * ncol).astype(np.float32) if case.startswith("lw_ds") else None
    gpt = case != "lw_ds"
    want = orc.lw_solver(go["tau"], go["lay_source"], go["lev_source"], emis, go["sfc_source"], top_at_1, nmus,
                         lw_Ds=ds, gpt=gpt)
    up, dn = (torch.full((ncol, nlay + 1), float("nan"), device=dev) for _ in range(2))
    gu, gd = ((torch.full((ncol, nlay + 1, ngpt), float("nan"), device=dev) for _ in range(2)) if gpt else (None, None))
    args = [T(a, dev) for a in (go["tau"], go["lay_source"], go["lev_source"], emis, go["sfc_source"])]
    dsd = T(ds, dev) if ds is not None else None
    p = (lambda t: t.data_ptr() if t is not None else None)
    check(_lib.lib().rrtmgpnn_lw_solver_noscat_gpt(
        context(0).h, ngpt, nlay, ncol, int(top_at_1), nmus, float_array(GAUSS_DS[nmus]), float_array(GAUSS_WTS[nmus]),
        p(dsd), None, *[p(a) for a in args], p(up), p(dn), p(gu), p(gd)), "lw_solver_noscat_gpt")
    torch.cuda.synchronize()
    got = [up, dn] + ([gu, gd] if gpt else [])
    for a, b, what in zip(got, want, ("up", "dn", "gpt_up", "gpt_dn")):
        np.testing.assert_array_equal(a.cpu().numpy(), b, err_msg=what)


@pytest.mark.parametrize("top_at_1", [True, False])
@pytest.mark.parametrize("nmus", [1, 3])
def test_lw_planck_gpt_matches_oracle(dev, orc, rfmip, top_at_1, nmus):
    """The fused Planck entry (the Fortran class layer's rte_lw path) with g-point outputs."""
    from rrtmgpnn import _lib
    from rrtmgpnn._lib import check, float_array, int_array
    from rrtmgpnn.api import GAUSS_DS, GAUSS_WTS, context
    prob, kd, go = _lw_inputs(orc, rfmip, top_at_1)
    ncol, nlay, ngpt = go["tau"].shape
    emis = np.repeat(np.asarray(prob["sfc_emis"], np.float32)[:, None], ngpt, axis=1)
    want = orc.lw_solver(go["tau"], go["lay_source"], go["lev_source"], emis, go["sfc_source"], top_at_1, nmus,
                         gpt=True)
    sfc_lay = 1 if prob["play"][0, 0] > prob["play"][0, nlay - 1] else nlay
    out = [torch.empty((ncol, nlay + 1), device=dev) for _ in range(2)]
    gp = [torch.empty((ncol, nlay + 1, ngpt), device=dev) for _ in range(2)]
    a = [T(x, dev) for x in (go["tau"], go["pfrac"], prob["tlay"], prob["tlev"], prob["tsfc"], kd["totplnk"], emis)]
    check(_lib.lib().rrtmgpnn_lw_solver_noscat_planck_gpt(
        context(0).h, ngpt, nlay, ncol, int(top_at_1), nmus, float_array(GAUSS_DS[nmus]), float_array(GAUSS_WTS[nmus]),
        None, None, a[0].data_ptr(), a[1].data_ptr(), kd["nband"], kd["nPlanckTemp"], a[2].data_ptr(),
        a[3].data_ptr(), a[4].data_ptr(), sfc_lay, int_array(kd["band_lims_gpt"].ravel()),
        float(kd["temp_ref_min"][0]), float(kd["totplnk_delta"]), a[5].data_ptr(), 0, a[6].data_ptr(),
        out[0].data_ptr(), out[1].data_ptr(), gp[0].data_ptr(), gp[1].data_ptr()), "lw_solver_noscat_planck_gpt")
    torch.cuda.synchronize()
    for x, y, what in zip(out + gp, want, ("up", "dn", "gpt_up", "gpt_dn")):
        np.testing.assert_array_equal(x.cpu().numpy(), y, err_msg=what)


@pytest.mark.parametrize("top_at_1", [True, False])
@pytest.mark.parametrize("with_g", [False, True])
@pytest.mark.parametrize("ngpt", [224, 223, 222])
def test_sw_gpt_matches_oracle(dev, orc, top_at_1, with_g, ngpt):
    """224: the checkpointed kernel's g-point instance; 222 (even, not a multiple of 4): the same kernel with the
    sequential broadband sums; 223 (odd): the one-g-point-per-lane kernel's g-point instance (sw_solver_2stream saves
    g-point fluxes for any ngpt, rte/kernels/mo_rte_solver_kernels.F90:567-588, 660-684)."""
    from rrtmgpnn import _lib
    from rrtmgpnn._lib import check
    from rrtmgpnn.api import context
    rng = np.random.default_rng(5)
    ncol, nlay = 29, 41
    tau = rng.lognormal(-2, 2, size=(ncol, nlay, ngpt)).astype(np.float32)
    ssa = rng.uniform(0, 1, size=(ncol, nlay, ngpt)).astype(np.float32)
    g = rng.uniform(0, 0.9, size=(ncol, nlay, ngpt)).astype(np.float32) if with_g else np.zeros_like(tau)
    mu0 = rng.uniform(0.05, 1, size=ncol).astype(np.float32)
    inc = rng.uniform(0, 10, size=(ncol, ngpt)).astype(np.float32)
    ad, af = (rng.uniform(0, 1, size=(ncol, ngpt)).astype(np.float32) for _ in range(2))
    want = orc.sw_solver(tau, ssa, g, mu0, inc, ad, af, top_at_1, gpt=True)
    out = [torch.empty((ncol, nlay + 1), device=dev) for _ in range(3)]
    gp = [torch.empty((ncol, nlay + 1, ngpt), device=dev) for _ in range(3)]
    a = [T(x, dev) for x in (inc, tau, ssa, g, mu0, ad, af)]
    check(_lib.lib().rrtmgpnn_sw_solver_2stream_gpt(
        context(0).h, ngpt, nlay, ncol, int(top_at_1), a[0].data_ptr(), None, a[1].data_ptr(), a[2].data_ptr(),
        a[3].data_ptr() if with_g else None, a[4].data_ptr(), a[5].data_ptr(), a[6].data_ptr(),
        *[t.data_ptr() for t in out + gp]), "sw_solver_2stream_gpt")
    torch.cuda.synchronize()
    for x, y, what in zip(out + gp, want, ("up", "dn", "dir", "gpt_up", "gpt_dn", "gpt_dir")):
        np.testing.assert_array_equal(x.cpu().numpy(), y, err_msg=what)


def test_class_layer_flexible_fluxes(dev, orc, rfmip):
    """rte_lw / rte_sw of the Python class layer with FluxesFlexible and lw_Ds: the entries above, with the
    reference's argument checks."""
    from rrtmgpnn import api
    prob, kd, go = _lw_inputs(orc, rfmip, True)
    ncol, nlay, ngpt = go["tau"].shape
    op = api.OpticalProps1scl()
    assert op.init(kd["band_lims_wvn"], kd["band_lims_gpt"]) == ""
    assert op.alloc_1scl(ncol, nlay) == ""
    op.tau = T(go["tau"], dev)
    src = api.SourceFuncLW()
    assert src.alloc(ncol, nlay, op) == ""
    src.lay_source, src.lev_source, src.sfc_source = T(go["lay_source"], dev), T(go["lev_source"], dev), \
        T(go["sfc_source"], dev)
    emis_band = np.repeat(np.asarray(prob["sfc_emis"], np.float32)[:, None], kd["nband"], axis=1)
    emis_gpt = np.repeat(np.asarray(prob["sfc_emis"], np.float32)[:, None], ngpt, axis=1)
    fl = api.FluxesFlexible(flux_up=torch.empty((ncol, nlay + 1), device=dev),
                            flux_dn=torch.empty((ncol, nlay + 1), device=dev),
                            gpt_flux_up=torch.empty((ncol, nlay + 1, ngpt), device=dev),
                            gpt_flux_dn=torch.empty((ncol, nlay + 1, ngpt), device=dev))
    ds = np.random.default_rng(9).uniform(1.0, 2.0, size=(ngpt, ncol)).astype(np.float32)
    assert api.rte_lw(op, True, src, T(emis_band, dev), fl, lw_Ds=T(ds, dev)) == ""
    torch.cuda.synchronize()
    want = orc.lw_solver(go["tau"], go["lay_source"], go["lev_source"], emis_gpt, go["sfc_source"], True, lw_Ds=ds,
                         gpt=True)
    for x, y in zip((fl.flux_up, fl.flux_dn, fl.gpt_flux_up, fl.gpt_flux_dn), want):
        np.testing.assert_array_equal(x.cpu().numpy(), y)
    assert api.rte_lw(op, True, src, T(emis_band, dev), fl, lw_Ds=T(ds[:, :-1], dev)) == \
        "rte_lw: lw_Ds inconsistently sized"
    assert api.rte_lw(op, True, src, T(emis_band, dev), fl, lw_Ds=T(ds * 0.5, dev)) == \
        "rte_lw: one or more values of lw_Ds < 1."
    assert api.rte_lw(op, True, src, T(emis_band, dev), fl, n_gauss_angles=2, lw_Ds=T(ds, dev)) == \
        "rte_lw: providing lw_Ds incompatible with specifying n_gauss_angles"
