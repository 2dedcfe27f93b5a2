"""GPU: the all-sky building blocks through the class layer, bit for bit against
the oracle (which tests/test_clouds_oracle.py pins to the reference's own Fortran):

* CloudOptics.cloud_optics (ty_cloud_optics, LUT and Pade, 1scl and 2str, each ice roughness);
* increment by band and at the same resolution, every 1scl/2str pairing;
* OpticalProps2str.delta_scale with f = g**2 and with an explicit forward fraction;
* the class-level error messages the reference returns.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a device"
    torch.cuda.set_device(0)
    return torch.device("cuda", 0)


def T(a, dev):
    return torch.as_tensor(np.ascontiguousarray(a, dtype=np.float32), device=dev)


def _clouds(co, ncol=37, nlay=19, seed=3):
    rng = np.random.default_rng(seed)
    lwp = np.where(rng.uniform(size=(ncol, nlay)) < 0.5, rng.uniform(0, 200, (ncol, nlay)), 0).astype(np.float32)
    iwp = np.where(rng.uniform(size=(ncol, nlay)) < 0.5, rng.uniform(0, 200, (ncol, nlay)), 0).astype(np.float32)
    rl = rng.uniform(co["radliq_lwr"][0], co["radliq_upr"][0], (ncol, nlay)).astype(np.float32)
    ri = rng.uniform(co["radice_lwr"][0], co["radice_upr"][0], (ncol, nlay)).astype(np.float32)
    rl[0, 0], ri[0, 0] = co["radliq_upr"][0], co["radice_upr"][0]  # table ends
    rl[0, 1], ri[0, 1] = co["radliq_lwr"][0], co["radice_lwr"][0]
    return lwp, iwp, rl, ri


def _props(api, nstr, spec_wvn, ncol, nlay, dev, gpt=None):
    p = api.OpticalProps1scl() if nstr == 1 else api.OpticalProps2str()
    assert p.init(spec_wvn, gpt) == ""
    e = p.alloc_1scl(ncol, nlay, device=dev) if nstr == 1 else p.alloc_2str(ncol, nlay, device=dev)
    assert e == ""
    return p


def _arrays(p):
    return [p.tau] if p.ssa is None else [p.tau, p.ssa, p.g]


@pytest.mark.parametrize("which", ["lw", "sw"])
@pytest.mark.parametrize("lut", [True, False])
@pytest.mark.parametrize("nstr", [1, 2])
@pytest.mark.parametrize("icergh", [1, 2, 3])
def test_cloud_optics_bitwise_vs_oracle(dev, orc, which, lut, nstr, icergh):
    from rrtmgpnn import api, data
    co = data.load_cloud_optics(which)
    args = _clouds(co)
    c = api.CloudOptics()
    assert c.load(which, use_lut=lut) == ""
    assert c.get_num_ice_roughness_types() == 3
    assert c.set_ice_roughness(icergh) == ""
    ncol, nlay = args[0].shape
    p = _props(api, nstr, co["bnd_limits_wavenumber"], ncol, nlay, dev)
    assert c.cloud_optics(*[T(a, dev) for a in args], p) == ""
    want = orc.cloud_optics(co, *args, nstr=nstr, lut=lut, icergh=icergh)
    for x, y in zip(_arrays(p), want):
        np.testing.assert_array_equal(x.cpu().numpy(), y)


def test_cloud_optics_load_lut_and_pade_match_file_loader(dev):
    """load_lut / load_pade from host arrays == load() of the RBIN file."""
    from rrtmgpnn import api, data
    co = data.load_cloud_optics("sw")
    args = [T(a, dev) for a in _clouds(co, seed=11)]
    outs = []
    for how in ("file_lut", "lut", "file_pade", "pade"):
        c = api.CloudOptics()
        if how.startswith("file"):
            e = c.load("sw", use_lut=how.endswith("lut"))
        elif how == "lut":
            e = c.load_lut(co["bnd_limits_wavenumber"], co["radliq_lwr"][0], co["radliq_upr"][0], co["radice_lwr"][0],
                           co["radice_upr"][0], co["lut_extliq"], co["lut_ssaliq"], co["lut_asyliq"],
                           co["lut_extice"], co["lut_ssaice"], co["lut_asyice"])
        else:
            e = c.load_pade(co["bnd_limits_wavenumber"], *[co["pade_" + k] for k in
                            ("extliq", "ssaliq", "asyliq", "extice", "ssaice", "asyice")],
                            *[co["pade_sizreg_" + k] for k in ("extliq", "ssaliq", "asyliq", "extice", "ssaice",
                                                               "asyice")])
        assert e == ""
        assert c.set_ice_roughness(2) == ""
        p = _props(api, 2, co["bnd_limits_wavenumber"], *args[0].shape, dev)
        assert c.cloud_optics(*args, p) == ""
        outs.append([a.cpu().numpy() for a in _arrays(p)])
    for a, b in ((0, 1), (2, 3)):
        for x, y in zip(outs[a], outs[b]):
            np.testing.assert_array_equal(x, y)


def test_cloud_optics_error_messages(dev):
    from rrtmgpnn import api, data
    co = data.load_cloud_optics("lw")
    c = api.CloudOptics()
    z = torch.zeros((3, 4), device=dev)
    p = _props(api, 1, co["bnd_limits_wavenumber"], 3, 4, dev)
    assert c.cloud_optics(z, z, z, z, p) == "cloud optics: no data has been initialized"
    assert c.set_ice_roughness(1) == "cloud_optics%set_ice_roughness(): can't set before initialization"
    assert c.load("lw") == ""
    assert c.set_ice_roughness(4) == "cloud optics: cloud ice surface roughness flag is out of bounds"
    assert c.cloud_optics(z, torch.zeros((3, 5), device=dev), z, z, p) == "cloud optics: ciwp has wrong extents"
    kd = data.load_kdist("lw")
    q = _props(api, 1, kd["band_lims_wvn"], 3, 4, dev, kd["band_lims_gpt"])
    assert c.cloud_optics(z, z, z, z, q) == "cloud optics: optical properties must be requested by band not g-points"
    api.rte_config_checks(True)
    try:
        bad = torch.full((3, 4), 1000.0, device=dev)
        w = torch.ones((3, 4), device=dev)
        assert c.cloud_optics(w, z, bad, z, p) == "cloud optics: liquid effective radius is out of bounds"
    finally:
        api.rte_config_checks(False)


@pytest.mark.parametrize("nstr_io,nstr_in", [(1, 1), (1, 2), (2, 1), (2, 2)])
def test_increment_bybnd_bitwise_vs_oracle(dev, orc, nstr_io, nstr_in):
    from rrtmgpnn import api, data
    kd = data.load_kdist("sw")
    rng = np.random.default_rng(nstr_io * 10 + nstr_in)
    ncol, nlay, ngpt, nb = 9, 13, kd["ngpt"], kd["nband"]
    io = [rng.lognormal(-2, 2, (ncol, nlay, ngpt)).astype(np.float32)]
    if nstr_io == 2:
        io += [rng.uniform(0, 1, io[0].shape).astype(np.float32), rng.uniform(0, 0.9, io[0].shape).astype(np.float32)]
    inc = [rng.lognormal(-1, 2, (ncol, nlay, nb)).astype(np.float32)]
    if nstr_in == 2:
        inc += [rng.uniform(0, 1, inc[0].shape).astype(np.float32), rng.uniform(0, 0.9, inc[0].shape).astype(np.float32)]
    p_io = _props(api, nstr_io, kd["band_lims_wvn"], ncol, nlay, dev, kd["band_lims_gpt"])
    p_in = _props(api, nstr_in, kd["band_lims_wvn"], ncol, nlay, dev)
    for t, a in zip(_arrays(p_io), io):
        t.copy_(T(a, dev))
    for t, a in zip(_arrays(p_in), inc):
        t.copy_(T(a, dev))
    assert p_in.increment(p_io) == ""
    for x, y in zip(_arrays(p_io), orc.increment_bybnd(kd["band_lims_gpt"], io, inc)):
        np.testing.assert_array_equal(x.cpu().numpy(), y)


@pytest.mark.parametrize("nstr_io,nstr_in", [(1, 1), (1, 2), (2, 1), (2, 2)])
def test_increment_same_resolution(dev, orc, nstr_io, nstr_in):
    """Same g-points: the by-band kernel with one g-point per band is the same arithmetic (oracle check)."""
    from rrtmgpnn import api, data
    kd = data.load_kdist("lw")
    rng = np.random.default_rng(7 + nstr_io * 10 + nstr_in)
    ncol, nlay, ngpt = 5, 11, kd["ngpt"]
    mk = lambda n: [rng.lognormal(-1, 2, (ncol, nlay, ngpt)).astype(np.float32)] + (  # noqa: E731
        [rng.uniform(0, 1, (ncol, nlay, ngpt)).astype(np.float32),
         rng.uniform(0, 0.9, (ncol, nlay, ngpt)).astype(np.float32)] if n == 2 else [])
    io, inc = mk(nstr_io), mk(nstr_in)
    p_io = _props(api, nstr_io, kd["band_lims_wvn"], ncol, nlay, dev, kd["band_lims_gpt"])
    p_in = _props(api, nstr_in, kd["band_lims_wvn"], ncol, nlay, dev, kd["band_lims_gpt"])
    for t, a in zip(_arrays(p_io), io):
        t.copy_(T(a, dev))
    for t, a in zip(_arrays(p_in), inc):
        t.copy_(T(a, dev))
    assert p_in.increment(p_io) == ""
    ident = np.stack([np.arange(1, ngpt + 1)] * 2, axis=1).astype(np.int32)
    for x, y in zip(_arrays(p_io), orc.increment_bybnd(ident, io, inc)):
        np.testing.assert_array_equal(x.cpu().numpy(), y)


def test_increment_rejects_mismatched_bands(dev):
    from rrtmgpnn import api, data
    lw, sw = data.load_kdist("lw"), data.load_kdist("sw")
    a = _props(api, 1, lw["band_lims_wvn"], 2, 3, dev)
    b = _props(api, 1, sw["band_lims_wvn"], 2, 3, dev, sw["band_lims_gpt"])
    assert a.increment(b) == "ty_optical_props%increment: optical properties objects have different band structures"


@pytest.mark.parametrize("with_for", [False, True])
def test_delta_scale_bitwise_vs_oracle(dev, orc, with_for):
    from rrtmgpnn import api, data
    kd = data.load_kdist("sw")
    rng = np.random.default_rng(9)
    shp = (31, 17, kd["ngpt"])
    tau = rng.lognormal(0, 1, shp).astype(np.float32)
    ssa = rng.uniform(0, 1, shp).astype(np.float32)
    g = rng.uniform(0, 0.95, shp).astype(np.float32)
    fwd = rng.uniform(0, 1, shp).astype(np.float32) if with_for else None
    p = _props(api, 2, kd["band_lims_wvn"], shp[0], shp[1], dev, kd["band_lims_gpt"])
    p.tau.copy_(T(tau, dev)), p.ssa.copy_(T(ssa, dev)), p.g.copy_(T(g, dev))
    assert p.delta_scale(None if fwd is None else T(fwd, dev)) == ""
    for x, y in zip(_arrays(p), orc.delta_scale(tau, ssa, g, fwd)):
        np.testing.assert_array_equal(x.cpu().numpy(), y)
    if with_for:
        assert p.delta_scale(T(fwd + 1, dev)) == "delta_scale: values of 'for' out of bounds [0,1]"


# ---------------------------------------------------------------------------------------------
# The C4 all-sky step (examples/all-sky/rrtmgp_allsky.F90:366-446 with NN gas optics) vs the oracle
def _allsky_prob(rfmip, ncol):
    from conftest import subset
    return subset(rfmip, np.arange(ncol) * (rfmip["ncol"] // ncol))


@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("lut", [True, False])
def test_allsky_step_bitwise_vs_oracle(dev, orc, rfmip, fused, lut, sw_kernel):
    from rrtmgpnn import data
    from rrtmgpnn.pipeline import ClearSkyStep
    prob = _allsky_prob(rfmip, 240)
    co_lw, co_sw = data.load_cloud_optics("lw"), data.load_cloud_optics("sw")
    clouds = data.allsky_clouds(prob, co_lw)
    assert (clouds[0] > 0).any() and (clouds[1] > 0).any()
    step = ClearSkyStep(prob, device=0, fused=fused, clouds=clouds, cloud_lut=lut)
    step.step()
    torch.cuda.synchronize()
    got = step.fluxes()
    m = {k: data.load_model(k) for k in ("lw_abs", "lw_pfrac", "sw_abs", "sw_ray")}
    lu, ld, _ = orc.all_sky_lw(prob, [m["lw_abs"], m["lw_pfrac"]], data.load_kdist("lw"), co_lw, clouds, lut=lut)
    su, sd, sr, _ = orc.all_sky_sw(prob, [m["sw_abs"], m["sw_ray"]], data.load_kdist("sw"), co_sw, clouds, lut=lut)
    use = prob["usecol"]
    np.testing.assert_array_equal(got["lw_up"], lu)
    np.testing.assert_array_equal(got["lw_dn"], ld)
    for k, r in (("sw_up", su), ("sw_dn", sd)):
        g = got[k].copy()
        g[~use] = 0.0
        np.testing.assert_array_equal(g, r, err_msg=k)
    np.testing.assert_array_equal(got["sw_dir"][use], sr[use])
    # clouds change the fluxes: cloudy columns differ from the clear-sky step
    clr = ClearSkyStep(prob, device=0)
    clr.step()
    torch.cuda.synchronize()
    cf = clr.fluxes()
    cloudy = (clouds[0] > 0).any(axis=1) | (clouds[1] > 0).any(axis=1)
    assert np.all(np.abs(cf["lw_dn"][cloudy] - got["lw_dn"][cloudy]).max(axis=1) > 0.1)
    np.testing.assert_array_equal(cf["lw_dn"][~cloudy], got["lw_dn"][~cloudy])


def test_allsky_graph_replay_matches_eager(dev, rfmip):
    from rrtmgpnn import data
    from rrtmgpnn.pipeline import ClearSkyStep
    prob = _allsky_prob(rfmip, 300)
    step = ClearSkyStep(prob, device=0, clouds=data.allsky_clouds(prob, data.load_cloud_optics("lw")))
    step.step()
    torch.cuda.synchronize()
    a = step.fluxes()
    step.capture()
    for t in (step.lw_up, step.lw_dn, step.sw_up, step.sw_dn, step.sw_dir):
        t.fill_(float("nan"))
    step.replay()
    torch.cuda.synchronize()
    b = step.fluxes()
    for k in a:
        np.testing.assert_array_equal(a[k], b[k])


@pytest.mark.parametrize("top_at_1", [True, False])
@pytest.mark.parametrize("nmus", [1, 3])
def test_fused_increment_solvers_match_increment_then_solve(dev, rfmip, top_at_1, nmus, sw_kernel):
    """rrtmgpnn_{lw_solver_noscat_planck,sw_solver_2stream}_inc == increment_bybnd followed by the plain solver,
    bit for bit, in both orientations (and for LW with several angles); the inputs are left untouched."""
    from rrtmgpnn import _lib, data
    from rrtmgpnn._lib import float_array, int_array
    from rrtmgpnn.api import GAUSS_DS, GAUSS_WTS, context
    L = _lib.lib()
    rng = np.random.default_rng(5 + nmus + 10 * top_at_1)
    ncol, nlay = 45, 33
    kl, ks = data.load_kdist("lw"), data.load_kdist("sw")
    ctx = context(0).h
    t = lambda a: T(a, dev)  # noqa: E731
    # ---- LW ----
    ng, nb = kl["ngpt"], kl["nband"]
    tau = t(rng.lognormal(-2, 2, (ncol, nlay, ng)))
    pfrac = t(rng.uniform(0, 0.2, (ncol, nlay, ng)))
    tb = t(np.where(rng.uniform(size=(ncol, nlay, nb)) < 0.4, rng.lognormal(0, 1, (ncol, nlay, nb)), 0))
    tlay = t(rng.uniform(200, 300, (ncol, nlay)))
    tlev = t(rng.uniform(200, 300, (ncol, nlay + 1)))
    tsfc = t(rng.uniform(250, 310, ncol))
    emis = t(rng.uniform(0.9, 1, (ncol, ng)))
    lims = int_array(kl["band_lims_gpt"].ravel())
    totplnk = t(kl["totplnk"])
    f = lambda *s: torch.empty(s, device=dev)  # noqa: E731
    up1, dn1, up2, dn2 = f(ncol, nlay + 1), f(ncol, nlay + 1), f(ncol, nlay + 1), f(ncol, nlay + 1)
    tau0 = tau.clone()
    common = (nb, kl["nPlanckTemp"], tlay.data_ptr(), tlev.data_ptr(), tsfc.data_ptr(), nlay if top_at_1 else 1, lims,
              float(kl["temp_ref_min"][0]), float(kl["totplnk_delta"]), totplnk.data_ptr(), 0, emis.data_ptr())
    Ds, W = float_array(GAUSS_DS[nmus]), float_array(GAUSS_WTS[nmus])
    _lib.check(L.rrtmgpnn_lw_solver_noscat_planck_inc(ctx, ng, nlay, ncol, int(top_at_1), nmus, Ds, W, None,
                                                      tau.data_ptr(), tb.data_ptr(), pfrac.data_ptr(), *common,
                                                      up1.data_ptr(), dn1.data_ptr()))
    torch.cuda.synchronize()
    assert torch.equal(tau, tau0)
    _lib.check(L.rrtmgpnn_increment_bybnd(ctx, ncol, nlay, ng, nb, lims, tau.data_ptr(), None, None, tb.data_ptr(),
                                          None, None))
    _lib.check(L.rrtmgpnn_lw_solver_noscat_planck(ctx, ng, nlay, ncol, int(top_at_1), nmus, Ds, W, None,
                                                  tau.data_ptr(), pfrac.data_ptr(), *common, up2.data_ptr(),
                                                  dn2.data_ptr()))
    torch.cuda.synchronize()
    assert torch.equal(up1, up2) and torch.equal(dn1, dn2)
    # ---- SW ----
    ng, nb = ks["ngpt"], ks["nband"]
    tau = t(rng.lognormal(-2, 2, (ncol, nlay, ng)))
    ssa = t(rng.uniform(0, 1, (ncol, nlay, ng)))
    gg = t(rng.uniform(0, 0.8, (ncol, nlay, ng)))
    cl = rng.uniform(size=(ncol, nlay, nb)) < 0.4
    bt = t(np.where(cl, rng.lognormal(0, 1, (ncol, nlay, nb)), 0))
    bw = t(np.where(cl, rng.uniform(0.5, 1, (ncol, nlay, nb)), 0))
    bg = t(np.where(cl, rng.uniform(0, 0.9, (ncol, nlay, nb)), 0))
    mu0 = t(rng.uniform(0.1, 1, ncol))
    inc = t(rng.uniform(0, 5, (ncol, ng)))
    alb = t(rng.uniform(0, 1, (ncol, ng)))
    # the k-distribution's bands (16 g-points each: both g-points of a lane in one band, the kernel's band-pair
    # instance) and a layout with odd band starts (the general instance)
    bl = np.array(ks["band_lims_gpt"], dtype=np.int64).reshape(-1, 2)
    odd = bl.copy()
    odd[0, 1] -= 1
    odd[1, 0] -= 1
    assert (odd[1, 0] - 1) % 2 == 1
    outs = [[f(ncol, nlay + 1) for _ in range(3)] for _ in range(2)]
    for band_lims, with_g in ((b, w) for b in (bl, odd) for w in (True, False)):
        lims = int_array(band_lims.ravel())
        g_in = gg if with_g else None
        saved = [a.clone() for a in (tau, ssa, gg)]
        _lib.check(L.rrtmgpnn_sw_solver_2stream_inc(
            ctx, ng, nlay, ncol, int(top_at_1), inc.data_ptr(), None, tau.data_ptr(), ssa.data_ptr(),
            None if g_in is None else g_in.data_ptr(), nb, lims, bt.data_ptr(), bw.data_ptr(), bg.data_ptr(),
            mu0.data_ptr(), alb.data_ptr(), alb.data_ptr(), *[o.data_ptr() for o in outs[0]]))
        torch.cuda.synchronize()
        assert all(torch.equal(a, b) for a, b in zip(saved, (tau, ssa, gg)))
        t2, s2 = tau.clone(), ssa.clone()
        g2 = gg.clone() if with_g else torch.zeros_like(gg)
        _lib.check(L.rrtmgpnn_increment_bybnd(ctx, ncol, nlay, ng, nb, lims, t2.data_ptr(), s2.data_ptr(),
                                              g2.data_ptr(), bt.data_ptr(), bw.data_ptr(), bg.data_ptr()))
        _lib.check(L.rrtmgpnn_sw_solver_2stream(ctx, ng, nlay, ncol, int(top_at_1), inc.data_ptr(), None,
                                                t2.data_ptr(), s2.data_ptr(), g2.data_ptr(), mu0.data_ptr(),
                                                alb.data_ptr(), alb.data_ptr(), *[o.data_ptr() for o in outs[1]]))
        torch.cuda.synchronize()
        for a, b in zip(*outs):
            assert torch.equal(a, b), "with_g=%s bands=%s" % (with_g, band_lims[:2].tolist())
