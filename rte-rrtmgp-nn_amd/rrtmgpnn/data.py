"""Model files, surrogate k-distribution tables and problem generators (host side, numpy).

Arrays are returned in C order with the REVERSED Fortran shape, i.e. the same memory as the
reference's column-major arrays:  Fortran p_lay(nlay, ncol) <-> numpy (ncol, nlay).

`rfmip_problem()` reproduces the RFMIP clear-sky drivers' pre-processing
(examples/rfmip-clear-sky/rrtmgp_rfmip_lw.F90:265-305,385-390 and rrtmgp_rfmip_sw.F90:273-287,
317, 408-434) for a single block of all 1800 columns (100 sites x 18 experiments,
column = site + 100*expt as read_and_block_* reshape them, mo_rfmip_io.F90:74-680).
`synthetic_problem()` builds the larger synthetic configurations (C4, C5 of BASELINE.json).
"""
import functools
import os

import numpy as np

from . import rbin

DATA_DIR = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "data"))

MODEL_FILES = {
    "lw_abs": "nn_lw_g256_abs.rbin",
    "lw_pfrac": "nn_lw_g256_pfrac.rbin",
    "sw_abs": "nn_sw_g224_abs.rbin",
    "sw_ray": "nn_sw_g224_ray.rbin",
    "lw_g128_both": "nn_lw_g128_both.rbin",
}

F32_EPS = np.float32(np.finfo(np.float32).eps)


def path(name):
    return os.path.join(DATA_DIR, MODEL_FILES.get(name, name))


def load_model(name):
    return rbin.read(path(name))


def load_kdist(which):
    """Surrogate k-distribution tables ('lw' -> g256, 'sw' -> g224); see tools/convert_reference_data.py."""
    d = rbin.read(os.path.join(DATA_DIR, "kdist_lw_g256.rbin" if which == "lw" else "kdist_sw_g224.rbin"))
    out = {k: v for k, v in d.items()}
    out["nband"] = int(d["band_lims_gpt"].shape[0])
    out["ngpt"] = int(d["band_lims_gpt"][-1, 1])
    if which == "lw":
        out["nPlanckTemp"] = int(d["totplnk"].shape[1])
        tmin, tmax = np.float32(d["temp_ref_min"][0]), np.float32(d["temp_ref_max"][0])
        # totplnk_delta = (temp_ref_max - temp_ref_min) / (nPlanckTemp - 1)  (mo_gas_optics_rrtmgp.F90:1218)
        out["totplnk_delta"] = np.float32((tmax - tmin) / np.float32(out["nPlanckTemp"] - 1))
    return out


def cloud_optics_path(which):
    return os.path.join(DATA_DIR, "cloud_optics_%s.rbin" % which)


def load_cloud_optics(which):
    """Cloud-optics coefficients (extensions/cloud_optics/rrtmgp-cloud-optics-coeffs-{lw,sw}.nc as RBIN):
    LUT and Pade tables in the file's layout (C order = Fortran arrays reversed)."""
    return rbin.read(cloud_optics_path(which))


def allsky_clouds(problem, co):
    """The all-sky example's cloud recipe (examples/all-sky/rrtmgp_allsky.F90:323-349): clouds where
    100 hPa < p < 900 hPa in columns with mod(icol, 3) /= 0 (1-based icol of the whole problem: a shard starting at
    global column problem["col0"] keeps its columns' clouds); liquid water path 10 g/m2 where T > 263 K, ice
    10 g/m2 where T < 273 K; effective radii at the middle of the tables' ranges.
    Returns clwp, ciwp, rel, rei as (ncol, nlay) float32."""
    play, tlay = np.asarray(problem["play"], np.float32), np.asarray(problem["tlay"], np.float32)
    ncol = play.shape[0]
    col = (int(problem.get("col0", 0)) + np.arange(ncol) + 1) % 3 != 0
    mask = (play > np.float32(100 * 100)) & (play < np.float32(900 * 100)) & col[:, None]
    rel_val = np.float32(0.5) * (np.float32(co["radliq_lwr"][0]) + np.float32(co["radliq_upr"][0]))
    rei_val = np.float32(0.5) * (np.float32(co["radice_lwr"][0]) + np.float32(co["radice_upr"][0]))
    lwp = np.where(mask & (tlay > np.float32(263)), np.float32(10), np.float32(0)).astype(np.float32)
    iwp = np.where(mask & (tlay < np.float32(273)), np.float32(10), np.float32(0)).astype(np.float32)
    rel = np.where(lwp > 0, rel_val, np.float32(0)).astype(np.float32)
    rei = np.where(iwp > 0, rei_val, np.float32(0)).astype(np.float32)
    return lwp, iwp, rel, rei


def spacing(x):
    x = np.float32(x)
    return np.float32(np.nextafter(x, np.float32(np.inf)) - x)


def seqsum(a, axis=-1):
    """float32 sum accumulated strictly in index order, like a Fortran DO loop / SUM (numpy's .sum is pairwise)."""
    return np.take(np.cumsum(np.asarray(a, np.float32), axis=axis, dtype=np.float32), -1, axis=axis)


_fh = float.fromhex
# s_sincosf_data.c: the cosine polynomial (and its negation, quadrants 2-3), the sine polynomial, 2/pi * 2^24 and pi/2
_COSF_C = (tuple(map(_fh, ("0x1p0", "-0x1.ffffffd0c621cp-2", "0x1.55553e1068f19p-5", "-0x1.6c087e89a359dp-10",
                           "0x1.99343027bf8c3p-16"))),
           tuple(map(_fh, ("-0x1p0", "0x1.ffffffd0c621cp-2", "-0x1.55553e1068f19p-5", "0x1.6c087e89a359dp-10",
                           "-0x1.99343027bf8c3p-16"))))
_COSF_S = tuple(map(_fh, ("-0x1.555545995a603p-3", "0x1.1107605230bc4p-7", "-0x1.994eb3774cf24p-13")))
_COSF_HPI_INV, _COSF_HPI = _fh("0x1.45F306DC9C883p+23"), _fh("0x1.921FB54442D18p0")


def ref_cosf(y):
    """cosf as glibc 2.35 evaluates it (sysdeps/ieee754/flt-32/s_cosf.c: a pi/2 reduction and double polynomials,
    rounded once), elementwise for |y| < 120 -- what the reference's driver gets from cos() in working precision when
    built against glibc, as here (rrtmgp_rfmip_sw.F90:431-434).  numpy's own float32 cos rounds differently on a
    quarter of the RFMIP zenith angles.  The device's copy is csrc/libm_ref.hpp ref_cosf; both are checked against
    the host's cosf (tools/check_libm_ref_cosf.c on every float of [-4, 4], tests/test_host.py)."""
    y = np.asarray(y, np.float32)
    if np.any(np.abs(y) >= np.float32(120.0)):
        raise ValueError("ref_cosf: |y| >= 120 is outside the restated path")
    top = (y.view(np.uint32) >> np.uint32(20)) & np.uint32(0x7FF)
    x = y.astype(np.float64)
    small = top < ((0x3F490FDB >> 20) & 0x7FF)  # |y| < pi/4: no reduction, the cosine polynomial
    q = np.where(small, 0, ((x * _COSF_HPI_INV).astype(np.int32) + 0x800000) >> 24)
    xr = np.where(small, x, x - q * _COSF_HPI)
    xr = np.where(small | ((q & 1) == (q & 2) // 2), xr, -xr)  # sign[q & 3] = 1, -1, -1, 1
    n = np.where(small, 1, q ^ 1)
    x2 = xr * xr
    t = (q & 2) != 0
    c = [np.where(t, _COSF_C[1][k], _COSF_C[0][k]) for k in range(5)]
    x4 = x2 * x2
    # sinf_poly, in its order: c = (c0 + x2 c1) + x4 c2, then c + x6 (c3 + x2 c4); s = (x + x3 s1) + x5 (s2 + x2 s3)
    cosp = ((c[0] + x2 * c[1]) + x4 * c[2]) + (x4 * x2) * (c[3] + x2 * c[4])
    x3 = xr * x2
    sinp = (xr + x3 * _COSF_S[0]) + (x3 * x2) * (_COSF_S[1] + x2 * _COSF_S[2])
    out = np.where((n & 1) == 0, sinp, cosp).astype(np.float32)
    return np.where(top < ((0x39800000 >> 20) & 0x7FF), np.float32(1.0), out)  # |y| < 2^-12: 1


def set_tsi(solar_source, tsi):
    """ty_gas_optics_rrtmgp%set_tsi (rrtmgp/mo_gas_optics_rrtmgp.F90:1097-1120), float32."""
    s = np.asarray(solar_source, np.float32)
    norm = np.float32(1.0) / seqsum(s)[()]
    return (s * np.float32(tsi) * norm).astype(np.float32)


LW_GAS_ORDER = ["h2o", "o3", "co2", "n2o", "ch4", "cfc11", "cfc12", "co", "ccl4", "cfc22", "hfc143a",
                "hfc125", "hfc23", "hfc32", "hfc134a", "cf4", "o2", "n2"]


def rfmip_problem(lw_press_clamp=True, fields=None):
    """All 1800 RFMIP clear-sky columns (nlay = 60, top at index 1).

    Returns dict with play (ncol,nlay), plev (ncol,nlay+1), tlay, tlev, tsfc (ncol), gases
    {name: (ncol,nlay)}, sfc_emis (ncol), sfc_alb (ncol), sza, tsi, mu0, usecol, top_at_1.
    `fields`: the input file's fields, by default the committed RBIN conversion; ncio.rfmip_fields(path) reads
    the reference's netCDF file natively instead.
    """
    d = fields if fields is not None else rbin.read(os.path.join(DATA_DIR, "rfmip_clear_sky.rbin"))
    nexp, nsite, nlay = d["temp_layer"].shape
    ncol = nsite * nexp
    site = np.tile(np.arange(nsite), nexp)
    expt = np.repeat(np.arange(nexp), nsite)
    kd = load_kdist("lw")
    pmin = np.float32(kd["press_ref_min"][0])
    play = d["pres_layer"][site].astype(np.float32)
    plev = d["pres_level"][site].astype(np.float32)
    top_at_1 = bool(play[0, 0] < play[0, nlay - 1])
    if lw_press_clamp:  # rrtmgp_rfmip_lw.F90:287  where(p_lay < press_min) p_lay = press_min + spacing(press_min)
        play = np.where(play < pmin, pmin + spacing(pmin), play).astype(np.float32)
    # rrtmgp_rfmip_lw.F90:300-305 / rrtmgp_rfmip_sw.F90:273-278
    if top_at_1:
        plev[:, 0] = pmin + F32_EPS
    else:
        plev[:, nlay] = pmin + F32_EPS
    gases = {"h2o": d["h2o"][expt, site].astype(np.float32), "o3": d["o3"][expt, site].astype(np.float32)}
    for g in LW_GAS_ORDER[2:]:
        gases[g] = np.repeat(d["gm_" + g][expt][:, None], nlay, axis=1).astype(np.float32)
    sza = d["solar_zenith_angle"][site].astype(np.float32)
    # rrtmgp_rfmip_sw.F90:285-287, 432-434
    usecol = sza < np.float32(90.0) - np.float32(2.0) * spacing(90.0)
    deg_to_rad = np.float32(np.arccos(np.float32(-1.0)) / np.float32(180.0))
    mu0 = np.where(usecol, ref_cosf(sza * deg_to_rad), np.float32(1.0)).astype(np.float32)
    return {
        "ncol": ncol, "nlay": nlay, "top_at_1": top_at_1,
        "play": np.ascontiguousarray(play), "plev": np.ascontiguousarray(plev),
        "tlay": d["temp_layer"][expt, site].astype(np.float32),
        "tlev": d["temp_level"][expt, site].astype(np.float32),
        "tsfc": d["surface_temperature"][expt, site].astype(np.float32),
        "gases": gases,
        "sfc_emis": d["surface_emissivity"][site].astype(np.float32),
        "sfc_alb": d["surface_albedo"][site].astype(np.float32),
        "sza": sza, "mu0": mu0, "usecol": usecol,
        "tsi": d["total_solar_irradiance"][site].astype(np.float32),
    }


SYN_BLOCK = 1024  # columns per random stream of synthetic_problem


def _interp_base(base, nlay, pmin):
    """RFMIP profiles (every base column) interpolated linearly in ln(p) onto nlay layers between the column's surface
    pressure and press_ref_min (top at index 0).  Depends on the base column only, so it is computed once per base
    column and indexed by each synthetic column's draw."""
    nl0 = base["nlay"]
    if nlay == nl0:
        return {k: base[k] for k in ("play", "plev", "tlay", "tlev")}, dict(base["gases"])
    psfc = base["plev"][:, nl0].astype(np.float64)
    frac = np.linspace(0.0, 1.0, nlay + 1)[None, :]
    lev = np.exp(np.log(psfc)[:, None] * frac + np.log(np.float64(pmin) * 1.0001) * (1.0 - frac))
    lay = np.sqrt(lev[:, :-1] * lev[:, 1:])
    src_lay = np.log(base["play"].astype(np.float64))
    src_lev = np.log(base["plev"].astype(np.float64))
    src_lev[:, 0] = np.log(np.float64(pmin))
    lnl, lnv = np.log(lay), np.log(lev)

    def interp(src_lnp, vals, dst_lnp):
        out = np.empty(dst_lnp.shape)
        for i in range(dst_lnp.shape[0]):
            out[i] = np.interp(dst_lnp[i], src_lnp[i], vals[i])
        return out

    prof = {"play": lay, "plev": lev, "tlay": interp(src_lay, base["tlay"], lnl),
            "tlev": interp(src_lev, base["tlev"], lnv)}
    prof["plev"][:, 0] = pmin + F32_EPS
    gases = {k: interp(src_lay, v, lnl) for k, v in base["gases"].items()}
    return prof, gases


@functools.lru_cache(maxsize=4)
def _synthetic_base(nlay):
    """(RFMIP base problem, its profiles on nlay layers, their gases, press_ref_min): the same for every column range
    of one synthetic problem, so computed once per nlay (read only by synthetic_problem)."""
    base = rfmip_problem()
    pmin = np.float32(load_kdist("lw")["press_ref_min"][0])
    prof, bgas = _interp_base(base, nlay, pmin)
    return base, prof, bgas, pmin


def synthetic_problem(ncol, nlay=60, seed=20251015, t_sigma=2.0, h2o_sigma=0.2, col0=0):
    """Columns [col0, col0 + ncol) of the synthetic clear-sky problem of BASELINE configs C4/C5.

    Column i takes an RFMIP (site, expt) and its perturbations from the random stream of its block of SYN_BLOCK
    columns (PCG64 seeded by (seed, i // SYN_BLOCK)), so any column range of one global problem -- the rank's shard of
    the 1e6-column C5 problem, or a strided test sample -- is generated alone and is identical to the same columns of
    the whole.  For nlay != 60 the profile is interpolated linearly in ln(p) onto nlay layers between the surface and
    press_ref_min.  T += N(0, t_sigma K) clipped to the NN training range [160, 320.5] K; h2o *= lognormal(0,
    h2o_sigma) clipped to the NN range [xmin^4, xmax^4]; tsfc += N(0, t_sigma K).
    """
    base, prof, bgas, pmin = _synthetic_base(nlay)
    b0, b1 = col0 // SYN_BLOCK, (col0 + ncol + SYN_BLOCK - 1) // SYN_BLOCK
    pick, tn_lay, tn_lev, hf, tn_sfc = [], [], [], [], []
    for b in range(b0, b1):
        rng = np.random.Generator(np.random.PCG64(np.random.SeedSequence([seed, b])))
        pick.append(rng.integers(0, base["ncol"], size=SYN_BLOCK))
        tn_lay.append(rng.normal(0.0, t_sigma, size=(SYN_BLOCK, nlay)))
        tn_lev.append(rng.normal(0.0, t_sigma, size=(SYN_BLOCK, nlay + 1)))
        hf.append(rng.lognormal(0.0, h2o_sigma, size=(SYN_BLOCK, nlay)))
        tn_sfc.append(rng.normal(0.0, t_sigma, size=SYN_BLOCK))
    sl = slice(col0 - b0 * SYN_BLOCK, col0 - b0 * SYN_BLOCK + ncol)
    pick = np.concatenate(pick)[sl]
    cat = lambda xs: np.concatenate(xs)[sl]  # noqa: E731
    tlay = np.clip(prof["tlay"][pick] + cat(tn_lay), 160.0, 320.5)
    tlev = np.clip(prof["tlev"][pick] + cat(tn_lev), 160.0, 320.5)
    gases = {k: v[pick] for k, v in bgas.items()}
    h2o_lo, h2o_hi = 0.0101 ** 4, 0.5077 ** 4
    gases["h2o"] = np.clip(gases["h2o"] * cat(hf), h2o_lo, h2o_hi)
    return {
        "ncol": ncol, "nlay": nlay, "top_at_1": True, "col0": col0,
        "play": np.ascontiguousarray(prof["play"][pick], np.float32),
        "plev": np.ascontiguousarray(prof["plev"][pick], np.float32),
        "tlay": np.ascontiguousarray(tlay, np.float32), "tlev": np.ascontiguousarray(tlev, np.float32),
        "tsfc": np.clip(base["tsfc"][pick] + cat(tn_sfc), 160.0, 340.0).astype(np.float32),
        "gases": {k: np.ascontiguousarray(v, np.float32) for k, v in gases.items()},
        "sfc_emis": base["sfc_emis"][pick].copy(), "sfc_alb": base["sfc_alb"][pick].copy(),
        "sza": base["sza"][pick].copy(), "mu0": base["mu0"][pick].copy(), "usecol": base["usecol"][pick].copy(),
        "tsi": base["tsi"][pick].copy(),
    }


def rfmip_columns(col0, ncol):
    """Columns [col0, col0 + ncol) of the RFMIP set tiled without end (global column i is RFMIP column i % 1800):
    one rank's block when N ranks process N x 1800 columns (bench.py, weak scaling)."""
    base = rfmip_problem()
    idx = (col0 + np.arange(ncol)) % base["ncol"]
    sub = {k: (v[idx] if isinstance(v, np.ndarray) and v.ndim >= 1 and v.shape[0] == base["ncol"] else v)
           for k, v in base.items()}
    sub["gases"] = {k: v[idx] for k, v in base["gases"].items()}
    sub["ncol"] = ncol
    sub["col0"] = col0
    return sub


def toa_flux(problem, kd_sw, tsi_default=1361.0):
    """SW incident flux per (col, gpt): gas_optics_ext's toa_src = solar_source after set_tsi(1361)
    (rrtmgp_rfmip_sw.F90:317; mo_gas_optics_rrtmgp.F90:594-599), renormalised per column to the
    RFMIP TSI (rrtmgp_rfmip_sw.F90:408-427).  Returns (ncol, ngpt) float32."""
    sol = set_tsi(kd_sw["solar_source"], tsi_default)
    ncol = problem["ncol"]
    toa = np.broadcast_to(sol, (ncol, sol.size)).astype(np.float32)
    def_tsi = seqsum(toa, axis=1)
    # toa_flux * total_solar_irradiance / def_tsi, evaluated left to right as the driver does (:423)
    return ((toa * np.asarray(problem["tsi"], np.float32)[:, None]) / def_tsi[:, None]).astype(np.float32)


def write_problem(prob, path, n_gauss_angles=1, clouds=None):
    """Write a problem dict in the Fortran host programs' RBIN input format (rrtmgpnn_rfmip_clear_sky.F90's header;
    also read by oracle/cpu_bench.F90): state arrays, top_at_1, n_gauss_angles, gas_names + vmr_<gas> (every gas
    broadcast to (ncol, nlay)) and, for all-sky, clouds = (clwp, ciwp, rel, rei) as (ncol, nlay) arrays."""
    names = sorted(prob["gases"])
    arrays = {k: np.asarray(prob[k], np.float32) for k in ("play", "plev", "tlay", "tlev", "tsfc", "sfc_emis",
                                                             "sfc_alb", "mu0", "tsi")}
    arrays["usecol"] = np.asarray(prob["usecol"], np.float32)
    arrays["top_at_1"] = np.array([1.0 if prob["top_at_1"] else 0.0], np.float32)
    arrays["n_gauss_angles"] = np.array([n_gauss_angles], np.float32)
    arrays["gas_names"] = rbin.chars(names, 32)
    for g in names:
        arrays["vmr_" + g] = np.broadcast_to(np.asarray(prob["gases"][g], np.float32), prob["play"].shape).copy()
    if clouds is not None:
        for k, a in zip(("clwp", "ciwp", "rel", "rei"), clouds):
            arrays[k] = np.asarray(a, np.float32)
    rbin.write(path, arrays)
    return names
