"""GPU: models and cloud-optics coefficients loaded natively from netCDF (csrc/datafile.cpp) behave exactly like
the RBIN conversions: rrtmgpnn_network_load on a netCDF model file and rrtmgpnn_cloud_optics_load on a classic
netCDF coefficient file give bit-identical results.  The netCDF files are written here from the RBIN data in
the reference's layout (tests/ncfixtures.py), since the reference tree is not on the GPU box."""
import numpy as np
import pytest

from ncfixtures import write_arrays_netcdf, write_nn_netcdf

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a device"
    torch.cuda.set_device(0)
    return torch.device("cuda", 0)


@pytest.mark.parametrize("model", ["lw_abs", "lw_pfrac", "sw_abs", "sw_ray", "lw_g128_both"])
def test_network_from_netcdf_equals_rbin(dev, tmp_path, model):
    from rrtmgpnn import api, data
    m = data.load_model(model)
    nc = write_nn_netcdf(m, str(tmp_path / (model + ".nc")))
    a = api.RrtmgpNetwork().load_netcdf(nc)
    b = api.RrtmgpNetwork().load_netcdf(data.path(model))
    assert a.dims == b.dims and a.activation == b.activation and a.input_names == b.input_names
    np.testing.assert_array_equal(a.coeffs_input_min, b.coeffs_input_min)
    x = torch.rand((4096, a.dims[0]), device=dev)
    ya, yb = a.output_sgemm_flat(x), b.output_sgemm_flat(x)
    torch.cuda.synchronize()
    assert torch.equal(ya, yb)


@pytest.mark.parametrize("which", ["lw", "sw"])
@pytest.mark.parametrize("lut", [True, False])
def test_cloud_optics_from_netcdf_equals_rbin(dev, tmp_path, which, lut):
    from rrtmgpnn import api, data
    co = data.load_cloud_optics(which)
    nc = write_arrays_netcdf(co, str(tmp_path / ("cloud_%s.nc" % which)))
    rng = np.random.default_rng(1)
    ncol, nlay = 17, 9
    lwp = torch.as_tensor(rng.uniform(0, 100, (ncol, nlay)).astype(np.float32), device=dev)
    rel = torch.as_tensor(rng.uniform(co["radliq_lwr"][0], co["radliq_upr"][0], (ncol, nlay)).astype(np.float32),
                          device=dev)
    rei = torch.as_tensor(rng.uniform(co["radice_lwr"][0], co["radice_upr"][0], (ncol, nlay)).astype(np.float32),
                          device=dev)
    outs = []
    for path in (nc, data.cloud_optics_path(which)):
        c = api.CloudOptics()
        assert c._load_path(path, lut) == ""
        p = api.OpticalProps2str()
        assert p.alloc_2str(ncol, nlay, c, device=dev) == ""
        assert c.cloud_optics(lwp, lwp, rel, rei, p) == ""
        outs.append([t.cpu().numpy() for t in (p.tau, p.ssa, p.g)])
    for x, y in zip(*outs):
        np.testing.assert_array_equal(x, y)
