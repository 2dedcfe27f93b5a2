"""CPU tests: the oracle (C restatement) against the golden fixtures made from the reference, against the
reference library itself when it is built, and against the known-answer properties of SURVEY.md 8c."""
import os

import numpy as np
import pytest

from conftest import subset

GOLD = os.path.join(os.path.dirname(__file__), "golden", "rfmip8_reference.rbin")


@pytest.fixture(scope="module")
def gold():
    from rrtmgpnn import rbin
    return rbin.read(GOLD)


@pytest.fixture(scope="module")
def models():
    from rrtmgpnn import data
    return {k: data.load_model(k) for k in ("lw_abs", "lw_pfrac", "sw_abs", "sw_ray")}


def test_mlp_matches_reference_fixture(orc, gold, models):
    # reference: network_type%output_sgemm_flat + MKL sgemm (neural/mod_network.F90:273-354)
    for m, xk in (("lw_abs", "mlp_lw_x"), ("lw_pfrac", "mlp_lw_x"), ("sw_abs", "mlp_sw_x"), ("sw_ray", "mlp_sw_x")):
        y = orc.mlp(models[m], gold[xk])
        ref = gold["mlp_%s_y" % m]
        # bitwise in practice; allow 1 ulp for BLAS-order differences on other hosts
        np.testing.assert_array_max_ulp(y, ref, maxulp=1)


def test_gas_optics_inputs_reproduce_fixture(orc, gold, rfmip, models):
    from rrtmgpnn import data
    prob = subset(rfmip, gold["cols"])
    go = orc.lw_gas_optics(prob, [models["lw_abs"], models["lw_pfrac"]], data.load_kdist("lw"))
    np.testing.assert_array_equal(go["nn_inputs"].reshape(-1, 18), gold["mlp_lw_x"])
    np.testing.assert_array_equal(go["tau"], gold["lw_tau"])
    np.testing.assert_array_equal(go["lev_source"], gold["lw_lev_source"])


@pytest.mark.parametrize("nmus", [1, 3])
def test_lw_solver_matches_reference_fixture(orc, gold, nmus):
    emis = np.repeat(gold["lw_sfc_emis_band"][:, :1], 256, axis=1)
    up, dn = orc.lw_solver(gold["lw_tau"], gold["lw_lay_source"], gold["lw_lev_source"], emis, gold["lw_sfc_source"],
                           True, nmus)
    np.testing.assert_allclose(up, gold["lw_flux_up_nmu%d" % nmus], rtol=0, atol=1e-4)
    np.testing.assert_allclose(dn, gold["lw_flux_dn_nmu%d" % nmus], rtol=0, atol=1e-4)


def test_lw_solver_bottom_first_reproduces_reference_quirk(orc, gold):
    # rte/kernels/mo_rte_solver_kernels.F90:742-776 hard-codes top-at-1 source indexing (Appendix B-1):
    # the flipped problem does NOT give the same fluxes, and the oracle must reproduce that.
    emis = np.repeat(gold["lw_sfc_emis_band"][:, :1], 256, axis=1)
    up, dn = orc.lw_solver(gold["lw_tau"][:, ::-1], gold["lw_lay_source"][:, ::-1], gold["lw_lev_source"][:, ::-1],
                           emis, gold["lw_sfc_source"], False, 1)
    np.testing.assert_allclose(up, gold["lw_flux_up_flip"], rtol=0, atol=1e-4)
    np.testing.assert_allclose(dn, gold["lw_flux_dn_flip"], rtol=0, atol=1e-4)
    assert abs(up[0, -1] - gold["lw_flux_up_nmu1"][0, 0]) > 0.1  # the quirk is visible (~0.6 W/m2)


@pytest.mark.parametrize("flip", [False, True])
def test_sw_solver_matches_reference_fixture(orc, gold, flip):
    sl = (slice(None), slice(None, None, -1)) if flip else (slice(None), slice(None))
    up, dn, dr = orc.sw_solver(gold["sw_tau"][sl], gold["sw_ssa"][sl], gold["sw_g"][sl], gold["sw_mu0"],
                               gold["sw_toa"], gold["sw_alb"], gold["sw_alb"], top_at_1=not flip)
    suf = "_flip" if flip else ""
    np.testing.assert_allclose(up, gold["sw_flux_up" + suf], rtol=0, atol=1e-4)
    np.testing.assert_allclose(dn, gold["sw_flux_dn" + suf], rtol=0, atol=1e-4)
    np.testing.assert_allclose(dr, gold["sw_flux_dir" + suf], rtol=0, atol=1e-4)


def test_sw_vertical_reversal_invariance(gold):
    # tests/verification.py sw_clear_sky_vr: SW fluxes are orientation invariant in the reference
    np.testing.assert_allclose(gold["sw_flux_up"], gold["sw_flux_up_flip"][:, ::-1], rtol=1e-5, atol=1e-3)
    np.testing.assert_allclose(gold["sw_flux_dn"], gold["sw_flux_dn_flip"][:, ::-1], rtol=1e-5, atol=1e-3)


def test_pfrac_band_sums_known_answer(orc, rfmip, models):
    # KAT: Planck fractions of each band sum to 1 (+-1.5e-3 measured on RFMIP; allow 3e-2)
    from rrtmgpnn import data
    prob = subset(rfmip, np.arange(0, 1800, 45))
    go = orc.lw_gas_optics(prob, [models["lw_abs"], models["lw_pfrac"]], data.load_kdist("lw"))
    s = go["pfrac"].reshape(prob["ncol"], 60, 16, 16).sum(-1)
    assert abs(float(np.median(s)) - 1.0) < 2e-3
    assert np.all(np.abs(s - 1.0) < 3e-2)


def test_oracle_physically_sane(orc, rfmip, models):
    from rrtmgpnn import data
    prob = subset(rfmip, [0])
    up, dn, _ = orc.clear_sky_lw(prob, [models["lw_abs"], models["lw_pfrac"]], data.load_kdist("lw"))
    assert 285 < up[0, 0] < 295 and 335 < dn[0, -1] < 345       # OLR 289.75, surface LW down 339.35
    up, dn, dr, _ = orc.clear_sky_sw(prob, [models["sw_abs"], models["sw_ray"]], data.load_kdist("sw"))
    assert 750 < dn[0, 0] < 765                                   # TOA SW down 757.35


REF_SO = os.path.join(os.path.dirname(os.path.dirname(__file__)), "oracle", "_ref", "librrtmgp_ref.so")


@pytest.mark.skipif(not os.path.exists(REF_SO), reason="reference oracle not built (needs /root/reference)")
def test_oracle_bitwise_vs_reference_full_rfmip(orc, rfmip, models):
    """Whole RFMIP set (1800 columns): oracle == reference Fortran (rte_lw, rte_sw, MLP), bit for bit."""
    import oracle as O
    from rrtmgpnn import data
    ref = O.Reference()
    kd, kds = data.load_kdist("lw"), data.load_kdist("sw")
    prob = subset(rfmip, np.arange(0, 1800, 3))
    up, dn, go = orc.clear_sky_lw(prob, [models["lw_abs"], models["lw_pfrac"]], kd)
    x = go["nn_inputs"].reshape(-1, 18)
    np.testing.assert_array_equal(orc.mlp(models["lw_abs"], x), ref.mlp(models["lw_abs"], x))
    emis_band = np.repeat(prob["sfc_emis"][:, None], 16, axis=1)
    ur, dr_ = ref.rte_lw(kd, go["tau"], go["lay_source"], go["lev_source"], go["sfc_source"], go["sfc_source_Jac"],
                         emis_band, True, 1)
    np.testing.assert_array_equal(up, ur)
    np.testing.assert_array_equal(dn, dr_)
    ups, dns, drs, gs = orc.clear_sky_sw(prob, [models["sw_abs"], models["sw_ray"]], kds)
    toa = data.toa_flux(prob, kds)
    alb = np.repeat(prob["sfc_alb"][:, None], 224, axis=1)
    u2, d2, r2 = ref.rte_sw(kds, gs["tau"], gs["ssa"], gs["g"], prob["mu0"], toa, alb, alb, True)
    m = ~prob["usecol"]
    u2[m] = 0
    d2[m] = 0
    np.testing.assert_array_equal(ups, u2)
    np.testing.assert_array_equal(dns, d2)
    np.testing.assert_array_equal(drs, r2)


@pytest.mark.skipif(not os.path.exists(REF_SO), reason="reference oracle not built (needs /root/reference)")
@pytest.mark.parametrize("top_at_1", [True, False])
def test_sw_noscat_bitwise_vs_reference_kernels(orc, rfmip, models, top_at_1):
    """rte_sw's 1scl branch (rte/mo_rte_sw.F90:213-222): the restatement == the reference's apply_BC_factor +
    sw_solver_noscat kernels, bit for bit, on the NN absorption optical depths of RFMIP columns."""
    import oracle as O
    from rrtmgpnn import data
    ref = O.Reference()
    prob = subset(rfmip, np.arange(0, 1800, 7))
    go = orc.sw_gas_optics(prob, [models["sw_abs"], models["sw_ray"]])
    tau = go["tau"] if top_at_1 else np.ascontiguousarray(go["tau"][:, ::-1])
    toa = data.toa_flux(prob, data.load_kdist("sw"))
    got, got_g = orc.sw_solver_noscat(tau, prob["mu0"], toa, top_at_1, gpt=True)
    want, want_g = ref.sw_noscat(tau, prob["mu0"], toa, top_at_1)
    np.testing.assert_array_equal(got_g, want_g)               # the spectral beam, every column
    np.testing.assert_array_equal(got[0], want[0])             # broadband: the reference's own sum for column 1
    np.testing.assert_array_equal(got, data.seqsum(want_g, axis=-1))  # every column: sum(flux_dir, 1) of its own
    assert np.all(want == want[:1])  # quirk B-11: the reference sums column 1 for every column
    top = 0 if top_at_1 else -1
    assert np.all(got[:, top] > 0) and np.all(np.diff(got, axis=1) * (1 if top_at_1 else -1) <= 0)


@pytest.mark.skipif(not os.path.exists(REF_SO), reason="reference oracle not built (needs /root/reference)")
@pytest.mark.parametrize("top_at_1", [True, False])
def test_gpt_fluxes_and_lw_ds_bitwise_vs_reference(orc, rfmip, models, top_at_1):
    """ty_fluxes_flexible g-point outputs and rte_lw's lw_Ds: the restatement == the reference's rte_lw / rte_sw, bit
    for bit.  LW with one angle returns g-point radiances (quirk B-5), with several the angle-summed fluxes; lw_Ds is
    read in the kernel's (ngpt, ncol) order although rte_lw checks (ncol, ngpt) extents (quirk B-12).  SW g-point down
    fluxes are total (diffuse + direct) and the broadband down flux is summed from them."""
    import oracle as O
    from rrtmgpnn import data
    ref = O.Reference()
    kd, kds = data.load_kdist("lw"), data.load_kdist("sw")
    prob = subset(rfmip, np.arange(1, 1800, 97))
    go = orc.lw_gas_optics(prob, [models["lw_abs"], models["lw_pfrac"]], kd)
    tau, lay, lev = go["tau"], go["lay_source"], go["lev_source"]
    if not top_at_1:
        tau, lay, lev = (np.ascontiguousarray(a[:, ::-1]) for a in (tau, lay, lev))
    ncol, nlay, ngpt = tau.shape
    rng = np.random.default_rng(7)
    emis_band = rng.uniform(0.8, 1.0, size=(ncol, kd["nband"])).astype(np.float32)
    band = np.concatenate([np.full(hi - lo + 1, b) for b, (lo, hi) in enumerate(np.asarray(kd["band_lims_gpt"]).reshape(-1, 2))])
    emis_gpt = np.ascontiguousarray(emis_band[:, band])
    for nmus in (1, 2, 3):
        want = ref.rte_lw_gpt(kd, tau, lay, lev, go["sfc_source"], go["sfc_source_Jac"], emis_band, top_at_1, nmus)
        got = orc.lw_solver(tau, lay, lev, emis_gpt, go["sfc_source"], top_at_1, nmus, gpt=True)
        for a, b, what in zip(got, want, ("up", "dn", "gpt_up", "gpt_dn")):
            np.testing.assert_array_equal(a, b, err_msg="nmus %d %s" % (nmus, what))
    ds = rng.uniform(1.0, 2.5, size=ngpt * ncol).astype(np.float32)
    want = ref.rte_lw_gpt(kd, tau, lay, lev, go["sfc_source"], go["sfc_source_Jac"], emis_band, top_at_1, 1, lw_Ds=ds)
    got = orc.lw_solver(tau, lay, lev, emis_gpt, go["sfc_source"], top_at_1, lw_Ds=ds, gpt=True)
    for a, b, what in zip(got, want, ("up", "dn", "gpt_up", "gpt_dn")):
        np.testing.assert_array_equal(a, b, err_msg="lw_Ds " + what)
    plain = orc.lw_solver(tau, lay, lev, emis_gpt, go["sfc_source"], top_at_1)
    assert not np.array_equal(plain[0], got[0])  # the secants took effect
    gs = orc.sw_gas_optics(prob, [models["sw_abs"], models["sw_ray"]])
    t2, w2, g2 = gs["tau"], gs["ssa"], np.zeros_like(gs["tau"])
    if not top_at_1:
        t2, w2 = (np.ascontiguousarray(a[:, ::-1]) for a in (t2, w2))
    toa = data.toa_flux(prob, kds)
    alb = rng.uniform(0.05, 0.5, size=toa.shape).astype(np.float32)
    mu0 = rng.uniform(0.1, 1.0, size=ncol).astype(np.float32)
    want = ref.rte_sw_gpt(kds, t2, w2, g2, mu0, toa, alb, alb, top_at_1)
    got = orc.sw_solver(t2, w2, g2, mu0, toa, alb, alb, top_at_1, gpt=True)
    for a, b, what in zip(got, want, ("up", "dn", "dir", "gpt_up", "gpt_dn", "gpt_dir")):
        np.testing.assert_array_equal(a, b, err_msg="sw " + what)


def test_sw_g0_identities_sampled():
    """The exact g = 0 rewrites of sw_two_stream's gamma1, gamma2 and alpha1 = alpha2 in the checkpointed SW kernel
    (kernels_sw_ck.hip): every subnormal and every 13th float of [0, 4] against the reference expressions
    (tools/check_sw_identities.py walks every float with |ssa| < 6.8e37)."""
    import numpy as np
    f = np.float32
    hi = int(np.float32(4).view(np.uint32))
    bits = np.concatenate([np.arange(0, 1 << 23, dtype=np.uint32), np.arange(1 << 23, hi, 13, dtype=np.uint32)])
    w = bits.view(np.float32)
    g1_ref = (f(8) - w * (f(5) + f(3) * f(0))) * f(.25)
    g2_ref = f(3) * (w * (f(1) - f(0))) * f(.25)
    a_ref = g1_ref * f(.5) + g2_ref * f(.5)
    g1, g2 = f(2) - w * f(1.25), w * f(.75)
    np.testing.assert_array_equal(g1.view(np.uint32), g1_ref.view(np.uint32))
    np.testing.assert_array_equal(g2.view(np.uint32), g2_ref.view(np.uint32))
    np.testing.assert_array_equal(((g1 + g2) * f(.5)).view(np.uint32), a_ref.view(np.uint32))
