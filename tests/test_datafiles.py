"""CPU: the native data-file readers (csrc/datafile.cpp via rrtmgpnn_file_*).

* classic netCDF written here with scipy (every netCDF type, scalars, character arrays, a record dimension,
  text attributes) reads back exactly;
* the reference's own files -- the NN models (netCDF-4/HDF5), the cloud-optics coefficients (classic netCDF)
  and the RFMIP inputs (netCDF-4) -- read natively equal the committed RBIN conversions, and the RFMIP problem
  built from the netCDF file equals the one built from RBIN, bit for bit (skipped where /root/reference is
  absent, e.g. on the GPU box; the GPU side is tests/test_gpu_datafiles.py).
"""
import os

import numpy as np
import pytest

REF = "/root/reference"
needs_ref = pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree not present")
NN = {"lw_abs": "lw-g256-2018-12-04_absorption_58_58.nc", "lw_pfrac": "lw-g256-2018-12-04_planck_frac_16_16.nc",
      "sw_abs": "sw-g224-2018-12-04-absorption_16_16.nc", "sw_ray": "sw-g224-2018-12-04-rayleigh_16_16.nc"}
ACT = ["linear", "softsign", "relu", "sigmoid", "hard_sigmoid", "tanh", "gaussian"]


def test_classic_netcdf_roundtrip(tmp_path):
    from scipy.io import netcdf_file
    from rrtmgpnn import ncio
    p = str(tmp_path / "t.nc")
    rng = np.random.default_rng(0)
    vals = {"f4": rng.normal(size=(3, 5)).astype(np.float32), "f8": rng.normal(size=(7,)),
            "i4": rng.integers(-1000, 1000, (2, 3)).astype(np.int32), "i2": np.array([-3, 4], np.int16),
            "i1": np.array([-1, 2, 3], np.int8)}
    for version in (1, 2):
        with netcdf_file(p, "w", version=version) as f:
            f.title = "native reader test"
            f.createDimension("t", None)  # the record (unlimited) dimension comes first
            f.createDimension("a", 3), f.createDimension("b", 5), f.createDimension("c", 7)
            f.createDimension("d", 2), f.createDimension("e", 3), f.createDimension("s", 8)
            for name, dims in (("f4", ("a", "b")), ("f8", ("c",)), ("i4", ("d", "e")), ("i2", ("d",)),
                               ("i1", ("e",))):
                v = f.createVariable(name, vals[name].dtype, dims)
                v[:] = vals[name]
            v = f.createVariable("names", "c", ("d", "s"))
            v[:] = np.array([list("softsign"), list("linear  ")], "S1")
            v.units = "1.e-6"
            r1 = f.createVariable("rec1", np.float32, ("t", "a"))
            r2 = f.createVariable("rec2", np.int32, ("t",))
            r1[0:4, :] = np.arange(12, dtype=np.float32).reshape(4, 3)
            r2[0:4] = np.arange(4, dtype=np.int32) * 10
        with ncio.DataFile(p) as d:
            np.testing.assert_array_equal(d.read("f4"), vals["f4"])
            np.testing.assert_array_equal(d.read("f8"), vals["f8"].astype(np.float32))
            for k in ("i4", "i2", "i1"):
                np.testing.assert_array_equal(d.read(k), vals[k].astype(np.int32))
            assert d.strings("names") == ["softsign", "linear"]
            assert d.att("names", "units") == "1.e-6" and d.att("", "title") == "native reader test"
            np.testing.assert_array_equal(d.read("rec1"), np.arange(12, dtype=np.float32).reshape(4, 3))
            np.testing.assert_array_equal(d.read("rec2"), np.arange(4, dtype=np.int32) * 10)


def test_classic_netcdf_scalar(tmp_path):
    from scipy.io import netcdf_file
    from rrtmgpnn import ncio
    p = str(tmp_path / "s.nc")
    with netcdf_file(p, "w") as f:
        sc = f.createVariable("radliq_lwr", np.float64, ())
        sc.data[...] = 2.5
    with ncio.DataFile(p) as d:
        assert d.read("radliq_lwr").shape == () and d.read("radliq_lwr") == np.float32(2.5)


def test_reader_errors(tmp_path):
    from rrtmgpnn import _lib, ncio
    bad = tmp_path / "x.bin"
    bad.write_bytes(b"not a data file")
    with pytest.raises(_lib.RrtmgpnnError, match="not an RBIN, netCDF or HDF5 file"):
        ncio.DataFile(str(bad))
    with pytest.raises(_lib.RrtmgpnnError, match="cannot open"):
        ncio.DataFile(str(tmp_path / "missing.nc"))


@needs_ref
@pytest.mark.parametrize("model", sorted(NN))
def test_nn_netcdf4_equals_rbin(model):
    from rrtmgpnn import data, ncio, rbin
    m = data.load_model(model)
    with ncio.DataFile(os.path.join(REF, "neural", "data", NN[model])) as f:
        dims = [f.read("nn_input_coeffs_min").size] + list(f.read("nn_dimsize"))
        np.testing.assert_array_equal(dims, m["dims"])
        assert [ACT.index(a) for a in f.strings("nn_activation_char")] == list(m["activation"])
        assert f.strings("nn_inputs_char") == rbin.unchars(m["input_names"])
        for n in range(1, len(dims)):
            np.testing.assert_array_equal(f.read("nn_weights_%d" % n), m["w%d" % n])
            np.testing.assert_array_equal(f.read("nn_bias_%d" % n), m["b%d" % n])
        np.testing.assert_array_equal(f.read("nn_input_coeffs_min"), m["input_min"])
        np.testing.assert_array_equal(f.read("nn_input_coeffs_max"), m["input_max"])
        if "output_mean" in m:
            np.testing.assert_array_equal(f.read("nn_output_coeffs_mean"), m["output_mean"])
            np.testing.assert_array_equal(f.read("nn_output_coeffs_std"), m["output_std"])
        assert "nn_layers" not in f  # netCDF-4 dimension-only scale: not a variable
        assert f.att("", "emulator_target").startswith("rrtmgp-data-")


@needs_ref
@pytest.mark.parametrize("which", ["lw", "sw"])
def test_cloud_coefficients_classic_netcdf_equal_rbin(which):
    from rrtmgpnn import data, ncio
    co = data.load_cloud_optics(which)
    got = ncio.read(os.path.join(REF, "extensions", "cloud_optics", "rrtmgp-cloud-optics-coeffs-%s.nc" % which))
    assert set(got) == set(co)
    for k, v in co.items():
        np.testing.assert_array_equal(np.atleast_1d(got[k]).astype(np.float32), v, err_msg=k)


@needs_ref
def test_rfmip_problem_from_netcdf_equals_rbin():
    from rrtmgpnn import data, ncio
    nc = os.path.join(REF, "examples", "rfmip-clear-sky",
                      "multiple_input4MIPs_radiation_RFMIP_UColorado-RFMIP-1-2_none.nc")
    a = data.rfmip_problem(fields=ncio.rfmip_fields(nc))
    b = data.rfmip_problem()
    for k in b:
        if k == "gases":
            for g in b[k]:
                np.testing.assert_array_equal(a[k][g], b[k][g], err_msg=g)
        else:
            np.testing.assert_array_equal(a[k], b[k], err_msg=k)
