"""GPU: rte_sw on absorption-only (1scl) properties -- apply_BC_factor + sw_solver_noscat (rte/mo_rte_sw.F90:213-222)
-- bit-identical to the oracle, whose spectral beam is pinned to the reference's own kernels (tests/test_oracle.py),
in both orientations, through the C ABI and the Python class layer."""
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


@pytest.mark.parametrize("top_at_1", [True, False])
def test_rte_sw_1scl_matches_oracle(dev, orc, rfmip, top_at_1):
    from rrtmgpnn import api, data
    prob = subset(rfmip, np.arange(0, 1800, 5))
    go = orc.sw_gas_optics(prob, [data.load_model("sw_abs"), data.load_model("sw_ray")])
    tau = go["tau"] if top_at_1 else np.ascontiguousarray(go["tau"][:, ::-1])
    toa = data.toa_flux(prob, data.load_kdist("sw"))
    want = orc.sw_solver_noscat(tau, prob["mu0"], toa, top_at_1)
    ncol, nlay, ngpt = tau.shape
    kd = api.GasOpticsRRTMGP()
    api.stop_on_err(kd.load("sw"))
    op = api.OpticalProps1scl()
    api.stop_on_err(op.alloc_1scl(ncol, nlay, kd))
    op.tau.copy_(T(tau, dev))
    up = torch.full((ncol, nlay + 1), 7.0, device=dev)
    dr = torch.empty((ncol, nlay + 1), device=dev)
    fl = api.FluxesBroadband(flux_up=up, flux_dn_dir=dr)
    alb = T(np.zeros((ncol, ngpt)), dev)
    mu0, inc = T(prob["mu0"], dev), T(toa, dev)
    api.stop_on_err(api.rte_sw(op, top_at_1, mu0, inc, alb, alb, fl))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(dr.cpu().numpy(), want)
    assert float(up.min()) == 7.0 == float(up.max())  # like the reference, the 1scl branch writes the direct flux only
    # no flux_dn_dir to write: an error string, as the class layer's convention
    assert api.rte_sw(op, top_at_1, mu0, inc, alb, alb, api.FluxesBroadband(flux_up=up)) != ""


@pytest.mark.parametrize("top_at_1", [True, False])
def test_rte_sw_1scl_gpt_matches_oracle(dev, orc, rfmip, top_at_1):
    """FluxesFlexible on the 1scl branch: gpt_flux_dn_dir receives the spectral direct beam (the reference's
    apply_BC_factor + sw_solver_noscat, which tests/test_oracle.py pins bit for bit), the broadband direct flux is
    unchanged, and the other g-point arrays are left alone (the reference does not write them)."""
    from rrtmgpnn import api, data
    prob = subset(rfmip, np.arange(2, 1800, 11))
    go = orc.sw_gas_optics(prob, [data.load_model("sw_abs"), data.load_model("sw_ray")])
    tau = go["tau"] if top_at_1 else np.ascontiguousarray(go["tau"][:, ::-1])
    toa = data.toa_flux(prob, data.load_kdist("sw"))
    want, want_g = orc.sw_solver_noscat(tau, prob["mu0"], toa, top_at_1, gpt=True)
    ncol, nlay, ngpt = tau.shape
    kd = api.GasOpticsRRTMGP()
    api.stop_on_err(kd.load("sw"))
    op = api.OpticalProps1scl()
    api.stop_on_err(op.alloc_1scl(ncol, nlay, kd))
    op.tau.copy_(T(tau, dev))
    dr = torch.empty((ncol, nlay + 1), device=dev)
    gdir = torch.full((ncol, nlay + 1, ngpt), float("nan"), device=dev)
    gup = torch.full((ncol, nlay + 1, ngpt), 5.0, device=dev)
    fl = api.FluxesFlexible(flux_dn_dir=dr, gpt_flux_dn_dir=gdir, gpt_flux_up=gup)
    alb = T(np.zeros((ncol, ngpt)), dev)
    mu0, inc = T(prob["mu0"], dev), T(toa, dev)
    api.stop_on_err(api.rte_sw(op, top_at_1, mu0, inc, alb, alb, fl))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(dr.cpu().numpy(), want)
    np.testing.assert_array_equal(gdir.cpu().numpy(), want_g)
    assert float(gup.min()) == 5.0 == float(gup.max())
    bad = api.FluxesFlexible(flux_dn_dir=dr, gpt_flux_dn_dir=gdir[:, :-1])
    assert api.rte_sw(op, top_at_1, mu0, inc, alb, alb, bad) == "rte_sw: g-point flux arrays inconsistently sized"
