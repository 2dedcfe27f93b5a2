"""CPU tests for row a-20 (heating rates): the oracle's two forms against a line-by-line numpy float32
restatement of the reference's expressions, on the reference's own fluxes (golden fixture) and the RFMIP pressures.

Parity note: neither reference routine is buildable here (extensions/mo_heating_rates.F90 uses modules this fork no
longer has; calc_heating_rate sits in a program that needs netcdf-fortran), so the pin is the expressions themselves,
each operation rounded to float32 in the reference's order."""
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(__file__), "golden", "rfmip8_reference.rbin")
f = np.float32


@pytest.fixture(scope="module")
def case(rfmip):
    from rrtmgpnn import rbin
    g = rbin.read(GOLD)
    cols = np.asarray(g["cols"], dtype=np.int64)
    plev = rfmip["plev"][cols].astype(np.float32)
    return g, plev


def _ks(up, dn, p):
    # extensions/mo_heating_rates.F90:48-52, left to right: ((up(l+1) - up(l) - dn(l+1) + dn(l)) * grav) / (cp_dry * dp)
    grav, cp_dry = f(9.80665), f(1004.64)
    a = ((up[:, 1:] - up[:, :-1]) - dn[:, 1:]) + dn[:, :-1]
    return (a * grav) / (cp_dry * (p[:, 1:] - p[:, :-1]))


def _kday(up, dn, p):
    # rrtmgp_lw_eval_nn_rfmip.F90:639-651: scaling = -(24*3600*grav/1004); hr = scaling * dF / dP
    scaling = -((f(24.0) * f(3600.0) * f(9.80665)) / f(1004.0))
    net = dn - up
    return (scaling * (net[:, 1:] - net[:, :-1])) / (p[:, 1:] - p[:, :-1])


@pytest.mark.parametrize("which", ["lw", "sw"])
def test_oracle_heating_rates_restate_the_reference(orc, case, which):
    g, plev = case
    up = g["lw_flux_up_nmu1" if which == "lw" else "sw_flux_up"].astype(np.float32)
    dn = g["lw_flux_dn_nmu1" if which == "lw" else "sw_flux_dn"].astype(np.float32)
    np.testing.assert_array_equal(orc.heating_rate(up, dn, plev), _ks(up, dn, plev))
    np.testing.assert_array_equal(orc.heating_rate(up, dn, plev, k_day=True), _kday(up, dn, plev))


def test_heating_rate_forms_agree_and_are_physical(orc, case):
    g, plev = case
    up, dn = g["lw_flux_up_nmu1"].astype(np.float32), g["lw_flux_dn_nmu1"].astype(np.float32)
    ks, kd = orc.heating_rate(up, dn, plev), orc.heating_rate(up, dn, plev, k_day=True)
    # the two forms differ by the units and cp (K/day = K/s * 86400 * cp_dry / 1004) and by where they round: the
    # flux differences of ~300 W/m2 values cancel to ~1 W/m2 in different orders (a few 1e-4 relative in float32)
    np.testing.assert_allclose(kd, ks * (86400.0 * 1004.64 / 1004.0), rtol=1e-3, atol=1e-4)
    # clear-sky longwave cools the troposphere (layers below 200 hPa, away from the surface layer) by 0.5-5 K/day
    trop = (0.5 * (plev[:, 1:] + plev[:, :-1]) > 2e4)
    trop[:, -1] = False
    assert np.mean(kd[trop] < 0) > 0.8 and -5.0 < float(np.mean(kd[trop])) < -0.5
    sw_up, sw_dn = g["sw_flux_up"].astype(np.float32), g["sw_flux_dn"].astype(np.float32)
    assert float(np.mean(orc.heating_rate(sw_up, sw_dn, plev, k_day=True))) > 0.0  # shortwave heats


def test_empty_and_single_layer(orc):
    up = np.array([[1.0, 2.0]], np.float32)
    dn = np.array([[5.0, 3.0]], np.float32)
    p = np.array([[100.0, 1100.0]], np.float32)
    np.testing.assert_array_equal(orc.heating_rate(up, dn, p), _ks(up, dn, p))
    assert orc.heating_rate(np.zeros((0, 61), np.float32), np.zeros((0, 61), np.float32),
                            np.zeros((0, 61), np.float32)).shape == (0, 60)
