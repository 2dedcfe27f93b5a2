"""CPU: the LW scattering solvers of SURVEY.md 8(f) row f-2 -- the rescaled no-scattering solution rte_lw uses
for two-stream optical properties (rte/mo_rte_lw.F90:372-387; lw_solver_noscat with do_rescaling,
rte/kernels/mo_rte_solver_kernels.F90:209-233, lw_transport_1rescl :1729-1795) and lw_solver_2stream (:426-486)
-- restated in oracle/rrtmgpnn_oracle.c and checked bit for bit against the reference's own Fortran compiled
into oracle/_ref, in both vertical orientations and for 1-4 quadrature angles."""
import numpy as np
import pytest

from conftest import subset


def _ref():
    import oracle as O
    try:
        return O.Reference()
    except FileNotFoundError as e:
        pytest.skip(str(e))


def lw_2str_problem(orc, rfmip, ncol=40, seed=1):
    """RFMIP LW gas optics (NN) as a two-stream set, incremented by LW cloud optics (2str, by band) from the
    all-sky recipe: scattering layers between 100 and 900 hPa in 2/3 of the columns."""
    from rrtmgpnn import data
    prob = subset(rfmip, np.arange(ncol) * (rfmip["ncol"] // ncol))
    kd = data.load_kdist("lw")
    go = orc.lw_gas_optics(prob, [data.load_model("lw_abs"), data.load_model("lw_pfrac")], kd)
    co = data.load_cloud_optics("lw")
    clouds = data.allsky_clouds(prob, co)
    cld = orc.cloud_optics(co, *clouds, nstr=2, lut=True, icergh=2)
    z = np.zeros_like(go["tau"])
    tau, ssa, g = orc.increment_bybnd(kd["band_lims_gpt"], (go["tau"], z, z.copy()), cld)
    emis_band = np.repeat(np.asarray(prob["sfc_emis"], np.float32)[:, None], kd["nband"], axis=1)
    emis_gpt = np.repeat(np.asarray(prob["sfc_emis"], np.float32)[:, None], kd["ngpt"], axis=1)
    return dict(kd=kd, tau=tau, ssa=ssa, g=g, lay=go["lay_source"], lev=go["lev_source"], sfc=go["sfc_source"],
                jac=go["sfc_source_Jac"], emis_band=emis_band, emis_gpt=emis_gpt)


def _flip(p):
    q = dict(p)
    for k in ("tau", "ssa", "g", "lay", "lev"):
        q[k] = np.ascontiguousarray(p[k][:, ::-1])
    return q


@pytest.mark.parametrize("top_at_1", [True, False])
@pytest.mark.parametrize("nmus", [1, 2, 3, 4])
def test_lw_rescaled_bitwise_vs_reference(orc, rfmip, top_at_1, nmus):
    ref = _ref()
    p = lw_2str_problem(orc, rfmip)
    assert (p["ssa"] > 0).any()
    if not top_at_1:
        p = _flip(p)
    a = orc.lw_solver(p["tau"], p["lay"], p["lev"], p["emis_gpt"], p["sfc"], top_at_1, nmus, ssa=p["ssa"], g=p["g"])
    b = ref.rte_lw_2str(p["kd"], p["tau"], p["ssa"], p["g"], p["lay"], p["lev"], p["sfc"], p["jac"], p["emis_band"],
                        top_at_1, nmus, use_2stream=False)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)


@pytest.mark.parametrize("top_at_1", [True, False])
def test_lw_2stream_bitwise_vs_reference(orc, rfmip, top_at_1):
    ref = _ref()
    p = lw_2str_problem(orc, rfmip, seed=2)
    if not top_at_1:
        p = _flip(p)
    a = orc.lw_solver_2stream(p["tau"], p["ssa"], p["g"], p["lev"], p["emis_gpt"], p["sfc"], top_at_1)
    b = ref.rte_lw_2str(p["kd"], p["tau"], p["ssa"], p["g"], p["lay"], p["lev"], p["sfc"], p["jac"], p["emis_band"],
                        top_at_1, 1, use_2stream=True)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)


@pytest.mark.parametrize("top_at_1", [True, False])
@pytest.mark.parametrize("mode", ["rescl1", "rescl3", "2stream"])
def test_lw_scattering_gpt_bitwise_vs_reference(orc, rfmip, top_at_1, mode):
    """ty_fluxes_flexible g-point outputs on two-stream properties (rte/mo_rte_lw.F90:357-387): the rescaled
    solution's radiances with one angle (quirk B-5) and angle-summed fluxes with several, lw_solver_2stream's adding
    fluxes -- the restatement == the reference's rte_lw, bit for bit."""
    ref = _ref()
    p = lw_2str_problem(orc, rfmip, seed=3)
    if not top_at_1:
        p = _flip(p)
    if mode == "2stream":
        a = orc.lw_solver_2stream(p["tau"], p["ssa"], p["g"], p["lev"], p["emis_gpt"], p["sfc"], top_at_1, gpt=True)
        nmus = 1
    else:
        nmus = 1 if mode == "rescl1" else 3
        a = orc.lw_solver(p["tau"], p["lay"], p["lev"], p["emis_gpt"], p["sfc"], top_at_1, nmus, ssa=p["ssa"],
                          g=p["g"], gpt=True)
    b = ref.rte_lw_2str_gpt(p["kd"], p["tau"], p["ssa"], p["g"], p["lay"], p["lev"], p["sfc"], p["jac"],
                            p["emis_band"], top_at_1, nmus, use_2stream=mode == "2stream")
    for x, y, what in zip(a, b, ("up", "dn", "gpt_up", "gpt_dn")):
        np.testing.assert_array_equal(x, y, err_msg=what)
    assert np.abs(a[2]).max() > 0


def test_lw_scattering_physics(orc, rfmip):
    """The rescaled solution equals the no-scattering solver where ssa = 0, and the two scattering solvers agree
    on the outgoing LW to ~10 W/m2 (different approximations of the same scattering)."""
    p = lw_2str_problem(orc, rfmip)
    up_n, dn_n = orc.lw_solver(p["tau"], p["lay"], p["lev"], p["emis_gpt"], p["sfc"], True, 1)
    up_r, dn_r = orc.lw_solver(p["tau"], p["lay"], p["lev"], p["emis_gpt"], p["sfc"], True, 1, ssa=p["ssa"], g=p["g"])
    up_2, dn_2 = orc.lw_solver_2stream(p["tau"], p["ssa"], p["g"], p["lev"], p["emis_gpt"], p["sfc"], True)
    clear = ~(p["ssa"] > 0).any(axis=(1, 2))
    np.testing.assert_array_equal(up_r[clear], up_n[clear])
    assert np.abs(up_2[:, 0] - up_r[:, 0]).max() < 15.0
    # (the reference two-stream can give small negative dn near the top for these sources; reproduced, not checked)
    assert np.all(np.isfinite(up_2)) and np.all(np.isfinite(dn_2))
