"""CPU: the cloud-optics restatement (oracle/rrtmgpnn_oracle.c) against the reference's own
extensions/cloud_optics/mo_cloud_optics.F90 and rte/mo_optical_props.F90 (increment, delta_scale),
compiled from its sources into oracle/_ref -- bit for bit.  SURVEY.md 8(f) row f-1."""
import numpy as np
import pytest


def _ref():
    import oracle as O
    try:
        return O.Reference()
    except FileNotFoundError as e:
        pytest.skip(str(e))


def _clouds(co, ncol=23, nlay=17, seed=3):
    rng = np.random.default_rng(seed)
    lwp = np.where(rng.uniform(size=(ncol, nlay)) < 0.5, rng.uniform(0, 200, (ncol, nlay)), 0).astype(np.float32)
    iwp = np.where(rng.uniform(size=(ncol, nlay)) < 0.5, rng.uniform(0, 200, (ncol, nlay)), 0).astype(np.float32)
    rl = rng.uniform(co["radliq_lwr"][0], co["radliq_upr"][0], (ncol, nlay)).astype(np.float32)
    ri = rng.uniform(co["radice_lwr"][0], co["radice_upr"][0], (ncol, nlay)).astype(np.float32)
    rl[0, 0], ri[0, 0] = co["radliq_upr"][0], co["radice_upr"][0]  # table ends
    rl[0, 1], ri[0, 1] = co["radliq_lwr"][0], co["radice_lwr"][0]
    return lwp, iwp, rl, ri


@pytest.mark.parametrize("which", ["lw", "sw"])
@pytest.mark.parametrize("lut", [True, False])
@pytest.mark.parametrize("nstr", [1, 2])
@pytest.mark.parametrize("icergh", [1, 2, 3])
def test_cloud_optics_bitwise_vs_reference(orc, which, lut, nstr, icergh):
    from rrtmgpnn import data
    ref = _ref()
    co = data.load_cloud_optics(which)
    args = _clouds(co)
    a = orc.cloud_optics(co, *args, nstr=nstr, lut=lut, icergh=icergh)
    b = ref.cloud_optics(co, *args, nstr=nstr, lut=lut, icergh=icergh)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)
    assert np.all(np.isfinite(a[0])) and a[0].max() > 0


@pytest.mark.parametrize("nstr_io,nstr_in", [(1, 1), (1, 2), (2, 1), (2, 2)])
def test_increment_bybnd_bitwise_vs_reference(orc, nstr_io, nstr_in):
    from rrtmgpnn import data
    ref = _ref()
    kd = data.load_kdist("sw")
    rng = np.random.default_rng(nstr_io * 10 + nstr_in)
    ncol, nlay, ngpt, nb = 7, 9, kd["ngpt"], kd["nband"]
    io = [rng.lognormal(-2, 2, (ncol, nlay, ngpt)).astype(np.float32)]
    if nstr_io == 2:
        io += [rng.uniform(0, 1, io[0].shape).astype(np.float32), rng.uniform(0, 0.9, io[0].shape).astype(np.float32)]
    inc = [rng.lognormal(-1, 2, (ncol, nlay, nb)).astype(np.float32)]
    if nstr_in == 2:
        inc += [rng.uniform(0, 1, inc[0].shape).astype(np.float32), rng.uniform(0, 0.9, inc[0].shape).astype(np.float32)]
    a = orc.increment_bybnd(kd["band_lims_gpt"], io, inc)
    b = ref.increment_bybnd(kd, io, inc)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)


@pytest.mark.parametrize("with_for", [False, True])
def test_delta_scale_bitwise_vs_reference(orc, with_for):
    from rrtmgpnn import data
    ref = _ref()
    kd = data.load_kdist("sw")
    rng = np.random.default_rng(9)
    shp = (5, 11, kd["nband"])
    tau = rng.lognormal(0, 1, shp).astype(np.float32)
    ssa = rng.uniform(0, 1, shp).astype(np.float32)
    g = rng.uniform(0, 0.95, shp).astype(np.float32)
    fwd = rng.uniform(0, 1, shp).astype(np.float32) if with_for else None
    for x, y in zip(orc.delta_scale(tau, ssa, g, fwd), ref.delta_scale(kd, tau, ssa, g, fwd)):
        np.testing.assert_array_equal(x, y)


def test_allsky_recipe_matches_example(rfmip):
    """examples/all-sky/rrtmgp_allsky.F90:323-349: cloud layers only between 100 and 900 hPa, 2/3 of columns."""
    from rrtmgpnn import data
    co = data.load_cloud_optics("lw")
    lwp, iwp, rel, rei = data.allsky_clouds(rfmip, co)
    cloudy = (lwp > 0) | (iwp > 0)
    assert not cloudy[2::3].any()                      # mod(icol,3) == 0 (1-based) is clear
    assert cloudy[0::3].any() and cloudy[1::3].any()
    assert np.all(rfmip["play"][cloudy] > 1e4) and np.all(rfmip["play"][cloudy] < 9e4)
    assert set(np.unique(rel)) <= {0.0, 12.0} and set(np.unique(rei)) <= {0.0, 95.0}
