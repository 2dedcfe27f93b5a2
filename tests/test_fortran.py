"""The Fortran drop-in class layer (rte-rrtmgp-nn_amd/fortran): modules with the reference's names
(mo_gas_optics_rrtmgp, mo_rte_lw, mo_rte_sw, mod_network_rrtmgp, ...) over the C ABI.

CPU: the layer and the example host program build; every C symbol it binds is declared in
include/rrtmgpnn.h; the RBIN reader/writer and ty_gas_concs round-trip data.
GPU: the example RFMIP clear-sky and all-sky host programs (blocked, ragged last block) reproduce the
oracle bit for bit.
"""
import os
import re
import shutil
import subprocess

import numpy as np
import pytest

from conftest import ROOT, subset

FDIR = os.path.join(ROOT, "rte-rrtmgp-nn_amd", "fortran")
FBUILD = os.path.join(FDIR, "build")
EXE = os.path.join(FBUILD, "rrtmgpnn_rfmip_clear_sky")
FC = os.environ.get("FC_RRTMGPNN", "/opt/rocm/lib/llvm/bin/amdflang")

needs_fc = pytest.mark.skipif(not os.path.exists(FC), reason="amdflang not available")


def _make():
    subprocess.run(["make", "-C", os.path.join(ROOT, "rte-rrtmgp-nn_amd")], check=True, capture_output=True)
    r = subprocess.run(["make", "-C", FDIR], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr


def write_problem(prob, path, n_gauss_angles=1):
    from rrtmgpnn import data
    return data.write_problem(prob, path, n_gauss_angles)


@needs_fc
def test_fortran_layer_builds_and_binds_only_header_symbols():
    _make()
    assert os.path.exists(EXE)
    header = open(os.path.join(ROOT, "include", "rrtmgpnn.h")).read()
    declared = set(re.findall(r"\b(rrtmgpnn_\w+)\s*\(", header))
    nm = subprocess.run(["nm", "-u", os.path.join(FBUILD, "librrtmgpnn_fortran.a")], capture_output=True,
                        text=True, check=True).stdout
    bound = set(re.findall(r"\b(rrtmgpnn_\w+)\b", nm))
    assert bound, "the Fortran layer binds no C entry point"
    assert bound <= declared, "bound but not declared: %s" % sorted(bound - declared)


@needs_fc
def test_fortran_rbin_roundtrip_and_gas_concs(tmp_path, rfmip):
    from rrtmgpnn import rbin
    _make()
    exe = str(tmp_path / "rbin_roundtrip")
    lib = os.path.join(ROOT, "rte-rrtmgp-nn_amd")
    subprocess.run([FC, "-O1", "-I", FBUILD, os.path.join(ROOT, "tests", "fortran", "rbin_roundtrip.F90"), "-o", exe,
                    os.path.join(FBUILD, "librrtmgpnn_fortran.a"), "-fopenmp", "-L" + lib, "-lrrtmgpnn",
                    "-Wl,-rpath," + lib],
                   check=True, capture_output=True)
    prob = subset(rfmip, np.arange(0, 1800, 97))
    fin, fout = str(tmp_path / "in.rbin"), str(tmp_path / "out.rbin")
    write_problem(prob, fin)
    subprocess.run([exe, fin, fout], check=True, capture_output=True)
    out = rbin.read(fout)
    np.testing.assert_array_equal(out["play"], prob["play"])
    np.testing.assert_array_equal(out["tsfc"], prob["tsfc"])
    np.testing.assert_array_equal(out["h2o"], prob["gases"]["h2o"])


@pytest.mark.gpu
@needs_fc
@pytest.mark.parametrize("threads,repeat", [(1, 1), (4, 3)])
def test_fortran_rfmip_driver_matches_oracle(tmp_path, orc, rfmip, threads, repeat):
    """The reference-shaped host program, blocked (64 columns, ragged last block), vs the oracle.  threads > 1: the
    blocks run concurrently under OpenMP, each thread with its own device context and stream; repeat > 1: the block
    loop runs again over the device-resident gas concentrations (cached device copies) and the timing line appears."""
    from rrtmgpnn import data, rbin
    if not os.path.exists(EXE):
        _make()
    prob = subset(rfmip, np.arange(0, 1800, 9))
    fin, fout = str(tmp_path / "prob.rbin"), str(tmp_path / "flux.rbin")
    write_problem(prob, fin)
    env = dict(os.environ, OMP_NUM_THREADS=str(threads))
    r = subprocess.run(["timeout", "-k", "10", "300", EXE, fin, fout, data.DATA_DIR, "64", str(repeat)],
                       capture_output=True, text=True, env=env)
    if repeat > 1:
        assert "ms per block loop" in r.stdout and "%d threads" % threads in r.stdout, r.stdout
    assert r.returncode == 0, r.stdout + r.stderr
    got = rbin.read(fout)
    lu, ld, _ = orc.clear_sky_lw(prob, [data.load_model("lw_abs"), data.load_model("lw_pfrac")],
                                 data.load_kdist("lw"))
    su, sd, sr, _ = orc.clear_sky_sw(prob, [data.load_model("sw_abs"), data.load_model("sw_ray")],
                                     data.load_kdist("sw"))
    use = prob["usecol"]
    for k, ref, g in (("lw_up", lu, got["lw_flux_up"]), ("lw_dn", ld, got["lw_flux_dn"]),
                      ("sw_up", su, got["sw_flux_up"]), ("sw_dn", sd, got["sw_flux_dn"]),
                      ("sw_dir", sr[use], got["sw_flux_dir"][use])):
        err = float(np.sqrt(np.mean((g.astype(np.float64) - ref) ** 2)))
        assert err <= 1e-3, "%s: RMS %.3g W/m2" % (k, err)
        np.testing.assert_array_equal(g, ref, err_msg=k + ": not bit-identical")
    # mo_heating_rates%compute_heating_rate on the driver's LW fluxes (row a-20), K/s
    np.testing.assert_array_equal(got["lw_heating_rate"], orc.heating_rate(lu, ld, prob["plev"]))


@pytest.mark.gpu
@needs_fc
@pytest.mark.parametrize("files", ["rbin", "nc"])
def test_fortran_allsky_driver_matches_oracle(tmp_path, orc, rfmip, files):
    """The all-sky host program (cloud_optics, clouds%increment, clouds%delta_scale through the Fortran class
    layer), blocked with a ragged last block, vs the oracle's all-sky pipeline -- bit for bit.  "nc": the models
    and cloud coefficients as netCDF files under the reference's names (load_netcdf, load_cld_lutcoeff through
    the native readers; written here from the RBIN data in the reference's layout)."""
    from ncfixtures import write_arrays_netcdf, write_nn_netcdf
    from rrtmgpnn import data, rbin
    exe = os.path.join(FBUILD, "rrtmgpnn_allsky")
    if not os.path.exists(exe):
        _make()
    prob = subset(rfmip, np.arange(0, 1800, 9))
    fin, fout = str(tmp_path / "prob.rbin"), str(tmp_path / "flux.rbin")
    write_problem(prob, fin)
    ddir, extra = data.DATA_DIR, []
    if files == "nc":
        ddir = str(tmp_path / "data")
        os.makedirs(ddir)
        for k in ("kdist_lw_g256.rbin", "kdist_sw_g224.rbin"):
            shutil.copy(os.path.join(data.DATA_DIR, k), ddir)
        for m, name in (("lw_abs", "lw-g256-2018-12-04_absorption_58_58.nc"),
                        ("lw_pfrac", "lw-g256-2018-12-04_planck_frac_16_16.nc"),
                        ("sw_abs", "sw-g224-2018-12-04-absorption_16_16.nc"),
                        ("sw_ray", "sw-g224-2018-12-04-rayleigh_16_16.nc")):
            write_nn_netcdf(data.load_model(m), os.path.join(ddir, name))
        for w in ("lw", "sw"):
            write_arrays_netcdf(data.load_cloud_optics(w), os.path.join(ddir, "rrtmgp-cloud-optics-coeffs-%s.nc" % w))
        extra = ["nc"]
    r = subprocess.run(["timeout", "-k", "10", "300", exe, fin, fout, ddir, "64"] + extra, capture_output=True,
                       text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    got = rbin.read(fout)
    co_lw, co_sw = data.load_cloud_optics("lw"), data.load_cloud_optics("sw")
    clouds = data.allsky_clouds(prob, co_lw)
    lu, ld, _ = orc.all_sky_lw(prob, [data.load_model("lw_abs"), data.load_model("lw_pfrac")], data.load_kdist("lw"),
                               co_lw, clouds)
    su, sd, sr, _ = orc.all_sky_sw(prob, [data.load_model("sw_abs"), data.load_model("sw_ray")],
                                   data.load_kdist("sw"), co_sw, clouds)
    use = prob["usecol"]
    for k, ref, g in (("lw_up", lu, got["lw_flux_up"]), ("lw_dn", ld, got["lw_flux_dn"]),
                      ("sw_up", su, got["sw_flux_up"]), ("sw_dn", sd, got["sw_flux_dn"]),
                      ("sw_dir", sr[use], got["sw_flux_dir"][use])):
        np.testing.assert_array_equal(g, ref, err_msg=k + ": not bit-identical")


@pytest.mark.gpu
@needs_fc
def test_fortran_device_state_update_host_and_device(tmp_path, orc, rfmip):
    """The device data environment as a reference user sees it (tests/fortran/devstate.F90): after gas_optics,
    update_host() returns tau and the Planck sources (formed from the deferred Planck fraction) bit-identical to the
    oracle's; rte_lw on the device copies equals the oracle; a host write to tau followed by update_device() is what
    the next rte_lw reads (0.5 * tau through the oracle's solver, bit for bit)."""
    from rrtmgpnn import data, rbin
    _make()
    lib = os.path.join(ROOT, "rte-rrtmgp-nn_amd")
    exe = str(tmp_path / "devstate")
    r = subprocess.run([FC, "-O1", "-fopenmp", "-I", FBUILD, os.path.join(ROOT, "tests", "fortran", "devstate.F90"),
                        "-o", exe, os.path.join(FBUILD, "librrtmgpnn_fortran.a"), "-L" + lib, "-lrrtmgpnn",
                        "-Wl,-rpath," + lib], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    prob = subset(rfmip, np.arange(5, 1800, 45))
    fin, fout = str(tmp_path / "in.rbin"), str(tmp_path / "out.rbin")
    write_problem(prob, fin)
    r = subprocess.run(["timeout", "-k", "10", "120", exe, fin, fout, data.DATA_DIR], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    got = rbin.read(fout)
    kd = data.load_kdist("lw")
    go = orc.lw_gas_optics(prob, [data.load_model("lw_abs"), data.load_model("lw_pfrac")], kd)
    np.testing.assert_array_equal(got["tau"], go["tau"])
    np.testing.assert_array_equal(got["lay_source"], go["lay_source"])
    np.testing.assert_array_equal(got["lev_source"], go["lev_source"])
    np.testing.assert_array_equal(got["sfc_source"], go["sfc_source"])
    ngpt = go["tau"].shape[-1]
    emis = np.repeat(np.asarray(prob["sfc_emis"], np.float32)[:, None], ngpt, axis=1)
    for tag, tau in (("a", go["tau"]), ("b", (np.float32(0.5) * go["tau"]).astype(np.float32))):
        up, dn = orc.lw_solver(tau, go["lay_source"], go["lev_source"], emis, go["sfc_source"], prob["top_at_1"])
        np.testing.assert_array_equal(got["flux_up_" + tag], up, err_msg=tag)
        np.testing.assert_array_equal(got["flux_dn_" + tag], dn, err_msg=tag)
    # ty_fluxes_flexible g-point outputs: (c) with lw_Ds, (d) with three angles, on the tau of (b); (e) rte_sw
    tau_b = (np.float32(0.5) * go["tau"]).astype(np.float32)
    ncol = tau_b.shape[0]
    i, g = np.meshgrid(np.arange(1, ncol + 1), np.arange(1, ngpt + 1), indexing="ij")
    ds = (np.float32(1) + np.float32(0.01) * ((7 * i + g) % 100).astype(np.float32)).astype(np.float32)  # (ncol, ngpt)
    np.testing.assert_array_equal(got["lw_ds"], ds.T)  # written with its Fortran extents (ncol, ngpt)
    # the kernel reads the array's memory (Fortran order: icol fastest) as D(igpt, icol) -- quirk B-12
    for tag, kw in (("c", dict(lw_Ds=np.ascontiguousarray(ds.T))), ("d", dict(nmus=3))):
        want = orc.lw_solver(tau_b, go["lay_source"], go["lev_source"], emis, go["sfc_source"], prob["top_at_1"],
                             gpt=True, **kw)
        for k, w in zip(("flux_up_", "flux_dn_", "gpt_up_", "gpt_dn_"), want):
            np.testing.assert_array_equal(got[k + tag], w, err_msg=k + tag)
    t2 = (np.float32(0.1) * go["tau"]).astype(np.float32)
    want = orc.sw_solver(t2, np.full_like(t2, 0.5), np.full_like(t2, 0.3), np.full(ncol, 0.6, np.float32),
                         np.ones((ncol, ngpt), np.float32), np.full((ncol, ngpt), 0.2, np.float32),
                         np.full((ncol, ngpt), 0.2, np.float32), prob["top_at_1"], gpt=True)
    for k, w in zip(("flux_up_e", "flux_dn_e", "flux_dir_e", "gpt_up_e", "gpt_dn_e", "gpt_dir_e"), want):
        np.testing.assert_array_equal(got[k], w, err_msg=k)
    # (f) rescaled and (g) use_2stream rte_lw on those two-stream properties, with g-point fluxes
    w2, g2 = np.full_like(t2, 0.5), np.full_like(t2, 0.3)
    want_f = orc.lw_solver(t2, go["lay_source"], go["lev_source"], emis, go["sfc_source"], prob["top_at_1"], ssa=w2,
                           g=g2, gpt=True)
    want_g = orc.lw_solver_2stream(t2, w2, g2, go["lev_source"], emis, go["sfc_source"], prob["top_at_1"], gpt=True)
    for tag, want in (("f", want_f), ("g", want_g)):
        for k, w in zip(("flux_up_", "flux_dn_", "gpt_up_", "gpt_dn_"), want):
            np.testing.assert_array_equal(got[k + tag], w, err_msg=k + tag)
    # (h) rte_sw on the 1scl tau of (b): broadband and spectral direct beam
    dr, gdr = orc.sw_solver_noscat(tau_b, np.full(ncol, 0.6, np.float32), np.ones((ncol, ngpt), np.float32),
                                   prob["top_at_1"], gpt=True)
    np.testing.assert_array_equal(got["flux_dir_h"], dr)
    np.testing.assert_array_equal(got["gpt_dir_h"], gdr)
    # (i), (j) flux_up_Jac / flux_dn_Jac accepted and untouched (compute_Jac = .false.), fluxes unchanged; the
    # use_2stream messages are checked inside the program (exit status 2 / 3)
    want_j = orc.lw_solver(t2, go["lay_source"], go["lev_source"], emis, go["sfc_source"], prob["top_at_1"], ssa=w2,
                           g=g2)
    for tag, want in (("i", (got["flux_up_b"], got["flux_dn_b"])), ("j", want_j)):
        np.testing.assert_array_equal(got["flux_up_" + tag], want[0], err_msg=tag)
        np.testing.assert_array_equal(got["flux_dn_" + tag], want[1], err_msg=tag)
        for k in ("jac_up_", "jac_dn_"):
            assert (got[k + tag] == np.float32(-7)).all(), k + tag
    # (k), (l) with flux_net associated: rte_lw as (b); rte_sw as (e) but without g-point outputs (whose broadband
    # down flux is summed from the g-point totals, :572-588), so against the oracle's plain solver; net = dn - up
    want_l = orc.sw_solver(t2, np.full_like(t2, 0.5), np.full_like(t2, 0.3), np.full(ncol, 0.6, np.float32),
                           np.ones((ncol, ngpt), np.float32), np.full((ncol, ngpt), 0.2, np.float32),
                           np.full((ncol, ngpt), 0.2, np.float32), prob["top_at_1"])
    for tag, (up, dn) in (("k", (got["flux_up_b"], got["flux_dn_b"])), ("l", want_l[:2])):
        np.testing.assert_array_equal(got["flux_up_" + tag], up, err_msg=tag)
        np.testing.assert_array_equal(got["flux_dn_" + tag], dn, err_msg=tag)
        np.testing.assert_array_equal(got["flux_net_" + tag], dn - up, err_msg=tag)
    np.testing.assert_array_equal(got["flux_dir_l"], want_l[2])


@pytest.mark.gpu
@needs_fc
def test_fortran_vmr_reset_between_parallel_loops(tmp_path, orc, rfmip):
    """4 OpenMP threads, each with its own device context, run gas optics + rte_lw over 4 blocks; between two such
    loops the serial region re-sets h2o and o3 of every block (set_vmr: drop, deallocate, allocate at the same size,
    usually the same address).  The process-wide invalidation of the device data environment (csrc/present.cpp)
    makes loop 2 read the new values in every worker context: both loops are bit-identical to the oracle on their
    own gases (tests/fortran/reset_vmr.F90)."""
    from rrtmgpnn import data, rbin
    _make()
    lib = os.path.join(ROOT, "rte-rrtmgp-nn_amd")
    exe = str(tmp_path / "reset_vmr")
    r = subprocess.run([FC, "-O1", "-fopenmp", "-I", FBUILD, os.path.join(ROOT, "tests", "fortran", "reset_vmr.F90"),
                        "-o", exe, os.path.join(FBUILD, "librrtmgpnn_fortran.a"), "-L" + lib, "-lrrtmgpnn",
                        "-Wl,-rpath," + lib], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    prob = subset(rfmip, np.arange(3, 1800, 9))  # 200 columns: 4 blocks of 50
    fin, fout = str(tmp_path / "in.rbin"), str(tmp_path / "out.rbin")
    write_problem(prob, fin)
    env = dict(os.environ, OMP_NUM_THREADS="4")
    r = subprocess.run(["timeout", "-k", "10", "120", exe, fin, fout, data.DATA_DIR, "50"], capture_output=True,
                       text=True, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    got = rbin.read(fout)
    models, kd = [data.load_model("lw_abs"), data.load_model("lw_pfrac")], data.load_kdist("lw")
    prob2 = dict(prob, gases=dict(prob["gases"]))
    prob2["gases"]["h2o"] = (np.float32(0.5) * np.asarray(prob["gases"]["h2o"], np.float32)).astype(np.float32)
    prob2["gases"]["o3"] = (np.float32(0.25) * np.asarray(prob["gases"]["o3"], np.float32)).astype(np.float32)
    for loop, pr in (("1", prob), ("2", prob2)):
        lu, ld, _ = orc.clear_sky_lw(pr, models, kd)
        np.testing.assert_array_equal(got["flux_up_" + loop], lu, err_msg="loop " + loop)
        np.testing.assert_array_equal(got["flux_dn_" + loop], ld, err_msg="loop " + loop)
    assert not np.array_equal(got["flux_up_1"], got["flux_up_2"])
