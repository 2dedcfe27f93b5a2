"""bench.py's CPU baseline driver (oracle/cpu_bench.F90 -> oracle/_ref/rrtmgp_cpu_bench): the reference's own
rte_lw / rte_sw / network_type sgemm / cloud optics, driven by an OpenMP loop over blocks as the RFMIP drivers do
(examples/rfmip-clear-sky/rrtmgp_rfmip_lw.F90:364-446).  The fluxes it produces must be the oracle's bit for bit
(the oracle is pinned bitwise to the same reference routines, tests/test_oracle.py), so the timed program is known
to compute the benchmarked workload.  CPU only."""
import json
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, subset

EXE = os.path.join(ROOT, "oracle", "_ref", "rrtmgp_cpu_bench")
DATA = os.path.join(ROOT, "rte-rrtmgp-nn_amd", "data")

needs_exe = pytest.mark.skipif(not os.path.exists(EXE), reason="oracle/_ref not built (needs /root/reference)")


def _run(tmp_path, prob, block, threads=4, sw=1, clouds=None):
    from rrtmgpnn import data, rbin
    pin, pout = str(tmp_path / "p.rbin"), str(tmp_path / "f.rbin")
    data.write_problem(prob, pin, clouds=clouds)
    env = dict(os.environ, OMP_STACKSIZE="256M", MKL_THREADING_LAYER="SEQUENTIAL")
    r = subprocess.run([EXE, pin, DATA, str(threads), str(block), str(prob["ncol"]), str(sw), "1", pout],
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["columns"] == prob["ncol"] and line["threads"] == threads and len(line["seconds"]) == 1
    return rbin.read(pout)


@needs_exe
def test_cpu_bench_clear_sky_equals_oracle(tmp_path, rfmip, orc):
    from rrtmgpnn import data
    prob = subset(rfmip, np.arange(0, 1800, 25))  # 72 columns, 2 blocks of 36
    out = _run(tmp_path, prob, 36)
    lw_up, lw_dn, _ = orc.clear_sky_lw(prob, [data.load_model("lw_abs"), data.load_model("lw_pfrac")],
                                       data.load_kdist("lw"))
    sw_up, sw_dn, sw_dir, _ = orc.clear_sky_sw(prob, [data.load_model("sw_abs"), data.load_model("sw_ray")],
                                               data.load_kdist("sw"))
    np.testing.assert_array_equal(out["lw_flux_up"], lw_up)
    np.testing.assert_array_equal(out["lw_flux_dn"], lw_dn)
    m = prob["usecol"]  # the oracle zeroes unused SW columns after the solve (rrtmgp_rfmip_sw.F90 output step)
    np.testing.assert_array_equal(out["sw_flux_up"][m], sw_up[m])
    np.testing.assert_array_equal(out["sw_flux_dn"][m], sw_dn[m])
    np.testing.assert_array_equal(out["sw_flux_dir"], sw_dir)


@needs_exe
def test_cpu_bench_all_sky_equals_oracle(tmp_path, rfmip, orc):
    from rrtmgpnn import data
    prob = subset(rfmip, np.arange(3, 1800, 50))  # 36 columns, one block
    co_lw, co_sw = data.load_cloud_optics("lw"), data.load_cloud_optics("sw")
    clouds = data.allsky_clouds(prob, co_lw)
    out = _run(tmp_path, prob, 36, threads=2, clouds=clouds)
    up, dn, _ = orc.all_sky_lw(prob, [data.load_model("lw_abs"), data.load_model("lw_pfrac")], data.load_kdist("lw"),
                               co_lw, clouds)
    np.testing.assert_array_equal(out["lw_flux_up"], up)
    np.testing.assert_array_equal(out["lw_flux_dn"], dn)
    sup, sdn, sdir, _ = orc.all_sky_sw(prob, [data.load_model("sw_abs"), data.load_model("sw_ray")],
                                       data.load_kdist("sw"), co_sw, clouds)
    m = prob["usecol"]
    np.testing.assert_array_equal(out["sw_flux_up"][m], sup[m])
    np.testing.assert_array_equal(out["sw_flux_dn"][m], sdn[m])
    np.testing.assert_array_equal(out["sw_flux_dir"], sdir)


@needs_exe
def test_cpu_bench_rejects_ragged_blocks(tmp_path, rfmip):
    from rrtmgpnn import data
    prob = subset(rfmip, np.arange(10))
    pin = str(tmp_path / "p.rbin")
    data.write_problem(prob, pin)
    r = subprocess.run([EXE, pin, DATA, "1", "4", "10", "1", "1"], capture_output=True, text=True, timeout=60)
    assert r.returncode != 0 and "evenly" in r.stdout
