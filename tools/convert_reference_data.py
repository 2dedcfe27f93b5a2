#!/opt/conda/bin/python3.9
"""Convert the reference's netCDF4/HDF5 data into the framework's RBIN files.

Runs ONLY in the build container (needs h5py, which is in the conda python 3.9
interpreter, and /root/reference).  Its outputs are committed under
`rte-rrtmgp-nn_amd/data/` so neither the GPU box nor the test-suite ever reads
the reference tree.  Everything written here is DATA (weights, inputs, tables).

Outputs
  nn_lw_g256_abs.rbin    neural/data/lw-g256-2018-12-04_absorption_58_58.nc
  nn_lw_g256_pfrac.rbin  neural/data/lw-g256-2018-12-04_planck_frac_16_16.nc
  nn_sw_g224_abs.rbin    neural/data/sw-g224-2018-12-04-absorption_16_16.nc
  nn_sw_g224_ray.rbin    neural/data/sw-g224-2018-12-04-rayleigh_16_16.nc
  nn_lw_g128_both.rbin   neural/data/lw-g128-210809_both_BEST.nc (single "both" model, a-6)
  rfmip_clear_sky.rbin   examples/rfmip-clear-sky/multiple_input4MIPs_radiation_RFMIP_UColorado-RFMIP-1-2_none.nc
  kdist_lw_g256.rbin     SURROGATE LW k-distribution tables (see below)
  kdist_sw_g224.rbin     SURROGATE SW k-distribution tables
  cloud_optics_lw.rbin   extensions/cloud_optics/rrtmgp-cloud-optics-coeffs-lw.nc (LUT + Pade coefficients)
  cloud_optics_sw.rbin   extensions/cloud_optics/rrtmgp-cloud-optics-coeffs-sw.nc

NN model layout follows the reader `neural/mod_network_rrtmgp.F90:58-122`:
  file variable nn_weights_n is C-order (n_in, n_out) = Keras kernel; the
  reference keeps w_transposed(n_out, n_in) (Fortran order) whose memory is the
  same bytes, and evaluates h = W^T x + b.  We store "w<n>" as (n_in, n_out).

RFMIP gas mapping follows `examples/rfmip-clear-sky/mo_rfmip_io.F90:323-358`
(forcing_index = 1, chemical name -> file name) and the "units" scaling of
`mo_rfmip_io.F90:683-698`.

The k-distribution files (rrtmgp-data-{lw-g256,sw-g224}-2018-12-04.nc) are
MISSING from the reference (.MISSING_LARGE_BLOBS).  The NN path only needs from
them: band->g-point limits, totplnk, temp_ref_min/max, press_ref_min and
solar_source.  We build surrogates, shared by the oracle and the GPU build:
  * LW: 16 bands x 16 g-points (confirmed by garand-atmos-1.nc band_lims_gpt);
    band wavenumber limits from extensions/cloud_optics/rrtmgp-cloud-optics-coeffs-lw.nc;
    totplnk(T, band) = band-integrated Planck radiance [W/m2/sr] at
    T = 160..355 K, 1 K steps (196 points), as in upstream RRTMGP.
  * SW: 14 bands x 16 g-points; band limits from ...-coeffs-sw.nc;
    solar_source(g) = band-integrated 5778 K blackbody irradiance at 1 AU,
    split evenly over the 16 g-points of each band.  (The drivers rescale it
    to TSI per column anyway, rrtmgp_rfmip_sw.F90:317,408-427.)
"""
import os
import sys

import h5py
import numpy as np
from scipy.io import netcdf_file

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "rte-rrtmgp-nn_amd", "rrtmgpnn"))
import rbin  # noqa: E402  (rrtmgpnn/rbin.py: numpy-only, no package import)

REF = "/root/reference"
OUT = os.path.join(HERE, "..", "rte-rrtmgp-nn_amd", "data")

ACT = {"linear": 0, "softsign": 1, "relu": 2, "sigmoid": 3, "hard_sigmoid": 4, "tanh": 5, "gaussian": 6}


def _strs(a):
    return [b"".join(r).decode().strip() for r in a]


def convert_nn(src, dst):
    g = h5py.File(os.path.join(REF, "neural", "data", src), "r")
    nl = int(g["nn_dimsize"].shape[0])
    nx = int(g["nn_dim_input"].shape[0])
    dims = [nx] + [int(v) for v in g["nn_dimsize"][()]]
    acts = _strs(g["nn_activation_char"][()])
    names = _strs(g["nn_inputs_char"][()])
    out = {
        "dims": np.array(dims, np.int32),
        "activation": np.array([ACT.get(a, 0) for a in acts], np.int32),
        "input_names": rbin.chars(names),
    }
    for n in range(1, nl + 1):
        w = np.asarray(g["nn_weights_%d" % n][()], np.float32)
        assert w.shape == (dims[n - 1], dims[n]), (src, n, w.shape)
        out["w%d" % n] = w
        out["b%d" % n] = np.asarray(g["nn_bias_%d" % n][()], np.float32)
    out["input_min"] = np.asarray(g["nn_input_coeffs_min"][()], np.float32)
    out["input_max"] = np.asarray(g["nn_input_coeffs_max"][()], np.float32)
    if "nn_output_coeffs_mean" in g:
        out["output_mean"] = np.asarray(g["nn_output_coeffs_mean"][()], np.float32)
        out["output_std"] = np.asarray(g["nn_output_coeffs_std"][()], np.float32)
    rbin.write(os.path.join(OUT, dst), out)
    print(dst, dims, acts)


def convert_rfmip():
    f = h5py.File(os.path.join(REF, "examples", "rfmip-clear-sky",
                               "multiple_input4MIPs_radiation_RFMIP_UColorado-RFMIP-1-2_none.nc"), "r")

    def scale(name):
        return float(f[name].attrs["units"].decode())

    out = {}
    for v in ["pres_layer", "pres_level", "temp_layer", "temp_level", "surface_temperature",
              "surface_emissivity", "surface_albedo", "solar_zenith_angle", "total_solar_irradiance",
              "profile_weight", "lat", "lon"]:
        out[v] = np.asarray(f[v][()], np.float32)
    # h2o / o3: (nexp, ncol, nlay), scaled by the units attribute (mo_rfmip_io.F90:520-560)
    out["h2o"] = (np.asarray(f["water_vapor"][()], np.float32) * np.float32(scale("water_vapor"))).astype(np.float32)
    out["o3"] = (np.asarray(f["ozone"][()], np.float32) * np.float32(scale("ozone"))).astype(np.float32)
    # forcing_index = 1: k-distribution chemical names mapped to RFMIP names (mo_rfmip_io.F90:323-358)
    gas_file = {"co2": "carbon_dioxide", "n2o": "nitrous_oxide", "ch4": "methane", "co": "carbon_monoxide",
                "ccl4": "carbon_tetrachloride", "cfc22": "hcfc22", "o2": "oxygen", "n2": "nitrogen",
                "cfc11": "cfc11", "cfc12": "cfc12", "hfc143a": "hfc143a", "hfc125": "hfc125",
                "hfc23": "hfc23", "hfc32": "hfc32", "hfc134a": "hfc134a", "cf4": "cf4"}
    for chem, fname in gas_file.items():
        v = fname + "_GM"
        # scalar per experiment: value * units (mo_rfmip_io.F90:640-652, scaling_factor * gas_conc_temp_1d)
        vals = np.asarray(f[v][()], np.float32)
        out["gm_" + chem] = (np.float32(scale(v)) * vals).astype(np.float32)
    out["expt_label"] = rbin.chars([s.decode() if isinstance(s, bytes) else str(s) for s in f["expt_label"][()]], 64)
    rbin.write(os.path.join(OUT, "rfmip_clear_sky.rbin"), out)
    print("rfmip", {k: v.shape for k, v in out.items()})


# --- Planck integrals --------------------------------------------------------
H = 6.62607015e-34
C = 2.99792458e8
KB = 1.380649e-23


def planck_wvn(nu_cm, T):
    """Planck radiance per unit wavenumber [W m-2 sr-1 (cm-1)-1]."""
    nu = nu_cm * 100.0
    x = H * C * nu / (KB * T)
    return 2.0 * H * C ** 2 * nu ** 3 / np.expm1(x) * 100.0


def band_integral(lo, hi, T, n=20001):
    nu = np.linspace(lo, hi, n)
    y = planck_wvn(nu, T)
    return np.trapz(y, nu)


def convert_kdist():
    lw = netcdf_file(os.path.join(REF, "extensions/cloud_optics/rrtmgp-cloud-optics-coeffs-lw.nc"), "r", mmap=False)
    sw = netcdf_file(os.path.join(REF, "extensions/cloud_optics/rrtmgp-cloud-optics-coeffs-sw.nc"), "r", mmap=False)
    wl = np.array(lw.variables["bnd_limits_wavenumber"][:], np.float64)  # (16,2)
    ws = np.array(sw.variables["bnd_limits_wavenumber"][:], np.float64)  # (14,2)

    nT = 196
    tmin, tmax = 160.0, 355.0
    temps = np.linspace(tmin, tmax, nT)
    totplnk = np.zeros((wl.shape[0], nT))  # memory = Fortran totplnk(nPlanckTemp, nbnd)
    for b in range(wl.shape[0]):
        for i, T in enumerate(temps):
            totplnk[b, i] = band_integral(wl[b, 0], wl[b, 1], T)
    lims = np.array([[16 * b + 1, 16 * b + 16] for b in range(16)], np.int32)  # Fortran band_lims_gpt(2,nbnd)
    # press_ref_min of the 2018-12-04 g256/g224 files (upstream RRTMGP); consistent with
    # exp(nn_input_coeffs_min(play)) = exp(5.15e-3) in the NN files.
    press_ref_min = 1.00518357
    rbin.write(os.path.join(OUT, "kdist_lw_g256.rbin"), {
        "band_lims_gpt": lims,
        "band_lims_wvn": wl.astype(np.float32),
        "totplnk": totplnk.astype(np.float32),
        "temp_ref_min": np.array([tmin], np.float32),
        "temp_ref_max": np.array([tmax], np.float32),
        "press_ref_min": np.array([press_ref_min], np.float32),
    })
    # SW: 5778 K blackbody, solar disk radiance * pi * (R_sun / AU)^2, 16 equal g-points per band
    rsun, au = 6.957e8, 1.495978707e11
    sol = np.zeros(16 * ws.shape[0])
    for b in range(ws.shape[0]):
        e = np.pi * band_integral(ws[b, 0], ws[b, 1], 5778.0, n=200001) * (rsun / au) ** 2
        sol[16 * b:16 * b + 16] = e / 16.0
    lims = np.array([[16 * b + 1, 16 * b + 16] for b in range(14)], np.int32)
    rbin.write(os.path.join(OUT, "kdist_sw_g224.rbin"), {
        "band_lims_gpt": lims,
        "band_lims_wvn": ws.astype(np.float32),
        "solar_source": sol.astype(np.float32),
        "press_ref_min": np.array([press_ref_min], np.float32),
        "temp_ref_min": np.array([tmin], np.float32),
        "temp_ref_max": np.array([tmax], np.float32),
    })
    print("kdist: sum solar", sol.sum(), " totplnk(300K) sum*pi", totplnk[:, 140].sum() * np.pi,
          " sigma T^4", 5.670374419e-8 * 300.0 ** 4)


def convert_cloud_optics():
    """extensions/cloud_optics/rrtmgp-cloud-optics-coeffs-{lw,sw}.nc (classic netCDF) -> cloud_optics_{lw,sw}.rbin.
    Every variable keeps its file shape (C order = the reference's Fortran arrays reversed) and is stored
    float32, the kind the reference reads it into (examples/all-sky/mo_load_cloud_coefficients.F90)."""
    for which in ("lw", "sw"):
        d = netcdf_file(os.path.join(REF, "extensions/cloud_optics/rrtmgp-cloud-optics-coeffs-%s.nc" % which), "r",
                        mmap=False)
        out = {}
        for name, v in d.variables.items():
            a = np.array(v[:] if v.shape else v.getValue())
            out[name] = np.atleast_1d(a).astype(np.float32)
        rbin.write(os.path.join(OUT, "cloud_optics_%s.rbin" % which), out)


if __name__ == "__main__":
    os.makedirs(OUT, exist_ok=True)
    if sys.argv[1:] == ["cloud"]:
        convert_cloud_optics()
        sys.exit(0)
    convert_cloud_optics()
    convert_nn("lw-g256-2018-12-04_absorption_58_58.nc", "nn_lw_g256_abs.rbin")
    convert_nn("lw-g256-2018-12-04_planck_frac_16_16.nc", "nn_lw_g256_pfrac.rbin")
    convert_nn("sw-g224-2018-12-04-absorption_16_16.nc", "nn_sw_g224_abs.rbin")
    convert_nn("sw-g224-2018-12-04-rayleigh_16_16.nc", "nn_sw_g224_ray.rbin")
    convert_nn("lw-g128-210809_both_64_64_HR_1.10e+00_FRC_8.79e-01.nc", "nn_lw_g128_both.rbin")
    convert_rfmip()
    convert_kdist()
