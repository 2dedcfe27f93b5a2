"""GPU: the LW scattering solvers through rte_lw on two-stream optical properties,
bit for bit against the oracle (which tests/test_lw_scattering_oracle.py pins to the reference's Fortran):
the rescaled no-scattering solution (default) for 1-4 angles and lw_solver_2stream (use_2stream=True), in both
vertical orientations; plus rte_lw's argument checks for these branches."""
import numpy as np
import pytest

from test_lw_scattering_oracle import _flip, lw_2str_problem

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a device"
    torch.cuda.set_device(0)
    return torch.device("cuda", 0)


def T(a, dev):
    return torch.as_tensor(np.ascontiguousarray(a, dtype=np.float32), device=dev)


def _gpu_lw(p, dev, top_at_1, nmus=None, use_2stream=False, inc=None):
    from rrtmgpnn import api
    kd = p["kd"]
    ncol, nlay, _ = p["tau"].shape
    op = api.OpticalProps2str()
    assert op.init(kd["band_lims_wvn"], kd["band_lims_gpt"]) == ""
    assert op.alloc_2str(ncol, nlay, device=dev) == ""
    op.tau.copy_(T(p["tau"], dev)), op.ssa.copy_(T(p["ssa"], dev)), op.g.copy_(T(p["g"], dev))
    src = api.SourceFuncLW()
    assert src.alloc(ncol, nlay, op, device=dev) == ""
    src.lay_source.copy_(T(p["lay"], dev)), src.lev_source.copy_(T(p["lev"], dev))
    src.sfc_source.copy_(T(p["sfc"], dev))
    f = lambda: torch.empty((ncol, nlay + 1), device=dev)  # noqa: E731
    fl = api.FluxesBroadband(f(), f())
    e = api.rte_lw(op, top_at_1, src, T(p["emis_band"], dev), fl, inc_flux=None if inc is None else T(inc, dev),
                   n_gauss_angles=nmus, use_2stream=use_2stream)
    assert e == "", e
    torch.cuda.synchronize()
    return fl.flux_up.cpu().numpy(), fl.flux_dn.cpu().numpy()


@pytest.fixture(scope="module")
def prob(orc, rfmip):
    return lw_2str_problem(orc, rfmip, ncol=64)


@pytest.mark.parametrize("top_at_1", [True, False])
@pytest.mark.parametrize("nmus", [1, 2, 3, 4])
def test_lw_rescaled_bitwise_vs_oracle(dev, orc, prob, top_at_1, nmus):
    p = prob if top_at_1 else _flip(prob)
    got = _gpu_lw(p, dev, top_at_1, nmus)
    want = orc.lw_solver(p["tau"], p["lay"], p["lev"], p["emis_gpt"], p["sfc"], top_at_1, nmus, ssa=p["ssa"], g=p["g"])
    for x, y, k in zip(got, want, ("up", "dn")):
        np.testing.assert_array_equal(x, y, err_msg=k)


@pytest.mark.parametrize("top_at_1", [True, False])
@pytest.mark.parametrize("with_inc", [False, True])
def test_lw_2stream_bitwise_vs_oracle(dev, orc, prob, top_at_1, with_inc):
    p = prob if top_at_1 else _flip(prob)
    inc = np.random.default_rng(4).uniform(0, 2, p["emis_gpt"].shape).astype(np.float32) if with_inc else None
    got = _gpu_lw(p, dev, top_at_1, use_2stream=True, inc=inc)
    want = orc.lw_solver_2stream(p["tau"], p["ssa"], p["g"], p["lev"], p["emis_gpt"], p["sfc"], top_at_1, inc)
    for x, y, k in zip(got, want, ("up", "dn")):
        np.testing.assert_array_equal(x, y, err_msg=k)


@pytest.mark.parametrize("top_at_1", [True, False])
@pytest.mark.parametrize("mode", ["rescl1", "rescl2", "rescl4", "2stream", "2stream_inc"])
def test_lw_scattering_gpt_bitwise_vs_oracle(dev, orc, prob, top_at_1, mode):
    """FluxesFlexible on two-stream properties (rrtmgpnn_lw_solver_1rescl_gpt / _2stream_gpt through rte_lw): the
    g-point outputs and the broadband fluxes equal the oracle's (pinned to the reference's rte_lw by
    tests/test_lw_scattering_oracle.py), bit for bit."""
    from rrtmgpnn import api
    p = prob if top_at_1 else _flip(prob)
    kd = p["kd"]
    ncol, nlay, ngpt = p["tau"].shape
    two = mode.startswith("2stream")
    nmus = None if two else int(mode[-1])
    inc = np.random.default_rng(6).uniform(0, 2, (ncol, ngpt)).astype(np.float32) if mode.endswith("inc") else None
    op = api.OpticalProps2str()
    assert op.init(kd["band_lims_wvn"], kd["band_lims_gpt"]) == ""
    assert op.alloc_2str(ncol, nlay, device=dev) == ""
    op.tau.copy_(T(p["tau"], dev)), op.ssa.copy_(T(p["ssa"], dev)), op.g.copy_(T(p["g"], dev))
    src = api.SourceFuncLW()
    assert src.alloc(ncol, nlay, op, device=dev) == ""
    src.lay_source.copy_(T(p["lay"], dev)), src.lev_source.copy_(T(p["lev"], dev))
    src.sfc_source.copy_(T(p["sfc"], dev))
    nan = lambda *s: torch.full(s, float("nan"), device=dev)  # noqa: E731
    fl = api.FluxesFlexible(flux_up=nan(ncol, nlay + 1), flux_dn=nan(ncol, nlay + 1),
                            gpt_flux_up=nan(ncol, nlay + 1, ngpt), gpt_flux_dn=nan(ncol, nlay + 1, ngpt))
    e = api.rte_lw(op, top_at_1, src, T(p["emis_band"], dev), fl, inc_flux=None if inc is None else T(inc, dev),
                   n_gauss_angles=nmus, use_2stream=two)
    assert e == "", e
    torch.cuda.synchronize()
    if two:
        want = orc.lw_solver_2stream(p["tau"], p["ssa"], p["g"], p["lev"], p["emis_gpt"], p["sfc"], top_at_1, inc,
                                     gpt=True)
    else:
        want = orc.lw_solver(p["tau"], p["lay"], p["lev"], p["emis_gpt"], p["sfc"], top_at_1, nmus, ssa=p["ssa"],
                             g=p["g"], gpt=True)
    got = (fl.flux_up, fl.flux_dn, fl.gpt_flux_up, fl.gpt_flux_dn)
    for x, y, k in zip(got, want, ("up", "dn", "gpt_up", "gpt_dn")):
        np.testing.assert_array_equal(x.cpu().numpy(), y, err_msg=k)
    # the broadband fluxes are those of the plain entries
    plain = _gpu_lw(p, dev, top_at_1, nmus, use_2stream=two, inc=inc)
    np.testing.assert_array_equal(plain[0], want[0])
    np.testing.assert_array_equal(plain[1], want[1])


def test_lw_scattering_argument_checks(dev, prob):
    from rrtmgpnn import api
    kd = prob["kd"]
    op = api.OpticalProps2str()
    assert op.alloc_2str(2, 3, kd_spec(kd), device=dev) == ""
    src = api.SourceFuncLW()
    assert src.alloc(2, 3, op, device=dev) == ""
    f = lambda: torch.empty((2, 4), device=dev)  # noqa: E731
    fl = api.FluxesBroadband(f(), f())
    emis = torch.ones((2, kd["nband"]), device=dev)
    assert api.rte_lw(op, True, src, emis, fl, n_gauss_angles=2, use_2stream=True) == \
        "rte_lw: using_2stream=true incompatible with specifying n_gauss_angles"
    op.ssa.fill_(2.0)
    assert api.rte_lw(op, True, src, emis, fl, use_2stream=True) == "validate: ssa values out of range"
    one = api.OpticalProps1scl()
    assert one.alloc_1scl(2, 3, kd_spec(kd), device=dev) == ""
    assert api.rte_lw(one, True, src, emis, fl, use_2stream=True) == \
        "rte_lw: can't use two-stream methods with only absorption optical depth"


@pytest.mark.parametrize("kind", ["1scl", "2str"])
def test_rte_lw_jacobian_arguments_as_reference(dev, orc, prob, kind):
    """rte/mo_rte_lw.F90:64, 82-85, 160-163, 252-253 with compute_Jac = .false. (mo_rte_rrtmgp_config.F90:28):
    flux_up_Jac / flux_dn_Jac are accepted on 1scl and on rescaled 2str properties, the fluxes are bit-identical to a
    call without them and the arrays are left untouched; with use_2stream, flux_up_Jac gives the reference's message
    and a lone flux_dn_Jac passes (the reference tests flux_up_Jac twice)."""
    from rrtmgpnn import api
    p, kd = prob, prob["kd"]
    ncol, nlay, _ = p["tau"].shape
    op = api.OpticalProps2str() if kind == "2str" else api.OpticalProps1scl()
    assert op.init(kd["band_lims_wvn"], kd["band_lims_gpt"]) == ""
    if kind == "2str":
        assert op.alloc_2str(ncol, nlay, device=dev) == ""
        op.ssa.copy_(T(p["ssa"], dev)), op.g.copy_(T(p["g"], dev))
    else:
        assert op.alloc_1scl(ncol, nlay, device=dev) == ""
    op.tau.copy_(T(p["tau"], dev))
    src = api.SourceFuncLW()
    assert src.alloc(ncol, nlay, op, device=dev) == ""
    src.lay_source.copy_(T(p["lay"], dev)), src.lev_source.copy_(T(p["lev"], dev))
    src.sfc_source.copy_(T(p["sfc"], dev))
    emis = T(p["emis_band"], dev)
    f = lambda: torch.empty((ncol, nlay + 1), device=dev)  # noqa: E731
    jup, jdn = torch.full((ncol, nlay + 1), -7.0, device=dev), torch.full((ncol, nlay + 1), -7.0, device=dev)
    fl = api.FluxesBroadband(f(), f())
    assert api.rte_lw(op, True, src, emis, fl, flux_up_Jac=jup, flux_dn_Jac=jdn) == ""
    torch.cuda.synchronize()
    if kind == "2str":
        want = orc.lw_solver(p["tau"], p["lay"], p["lev"], p["emis_gpt"], p["sfc"], True, ssa=p["ssa"], g=p["g"])
    else:
        want = orc.lw_solver(p["tau"], p["lay"], p["lev"], p["emis_gpt"], p["sfc"], True)
    np.testing.assert_array_equal(fl.flux_up.cpu().numpy(), want[0])
    np.testing.assert_array_equal(fl.flux_dn.cpu().numpy(), want[1])
    assert bool((jup == -7.0).all()) and bool((jdn == -7.0).all())
    if kind == "2str":
        assert api.rte_lw(op, True, src, emis, fl, use_2stream=True, flux_up_Jac=jup, flux_dn_Jac=jdn) == \
            "rte_lw: can't provide Jacobian of fluxes w.r.t surface temperature with 2-stream"
        assert api.rte_lw(op, True, src, emis, fl, use_2stream=True, flux_dn_Jac=jdn) == ""
        torch.cuda.synchronize()
        assert bool((jdn == -7.0).all())


def kd_spec(kd):
    from rrtmgpnn import api
    s = api.OpticalProps()
    assert s.init(kd["band_lims_wvn"], kd["band_lims_gpt"]) == ""
    return s
