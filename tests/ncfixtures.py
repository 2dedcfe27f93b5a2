"""Classic-netCDF fixtures written with scipy from the committed RBIN conversions, in the reference's file
layout (variable names and dimension order of neural/data/*.nc and rrtmgp-cloud-optics-coeffs-*.nc), so the
native readers can be exercised where the reference tree is absent (the GPU box)."""
import numpy as np
from scipy.io import netcdf_file

ACT = ["linear", "softsign", "relu", "sigmoid", "hard_sigmoid", "tanh", "gaussian"]


def _chars(strings, width=32):
    a = np.full((len(strings), width), b" ", "S1")
    for i, s in enumerate(strings):
        for j, ch in enumerate(s.encode()[:width]):
            a[i, j] = bytes([ch])
    return a


def write_nn_netcdf(m, path):
    """A model dict (rrtmgpnn.data.load_model) as the reference's netCDF model file (mod_network_rrtmgp.F90:58-122)."""
    from rrtmgpnn import rbin
    dims = [int(v) for v in m["dims"]]
    nl = len(dims) - 1
    with netcdf_file(path, "w") as f:
        f.createDimension("nn_layers", nl)
        f.createDimension("nn_dim_input", dims[0])
        f.createDimension("string_len", 32)
        for n in range(1, nl + 1):
            f.createDimension("nn_dim_%d" % n, dims[n])
        v = f.createVariable("nn_dimsize", np.int32, ("nn_layers",))
        v[:] = np.array(dims[1:], np.int32)
        for n in range(1, nl + 1):
            din = "nn_dim_input" if n == 1 else "nn_dim_%d" % (n - 1)
            w = f.createVariable("nn_weights_%d" % n, np.float32, (din, "nn_dim_%d" % n))
            w[:] = m["w%d" % n]
            b = f.createVariable("nn_bias_%d" % n, np.float32, ("nn_dim_%d" % n,))
            b[:] = m["b%d" % n]
        a = f.createVariable("nn_activation_char", "c", ("nn_layers", "string_len"))
        a[:] = _chars([ACT[int(k)] for k in m["activation"]])
        c = f.createVariable("nn_inputs_char", "c", ("nn_dim_input", "string_len"))
        c[:] = _chars(rbin.unchars(m["input_names"]))
        for k, name in (("input_min", "nn_input_coeffs_min"), ("input_max", "nn_input_coeffs_max")):
            v = f.createVariable(name, np.float32, ("nn_dim_input",))
            v[:] = m[k]
        if "output_mean" in m:
            for k, name in (("output_mean", "nn_output_coeffs_mean"), ("output_std", "nn_output_coeffs_std")):
                v = f.createVariable(name, np.float32, ("nn_dim_%d" % nl,))
                v[:] = m[k]
    return path


def write_arrays_netcdf(arrays, path):
    """Arbitrary {name: array} as classic netCDF; scalars for (1,)-shaped entries named like the cloud files'."""
    scalars = {"radliq_lwr", "radliq_upr", "radliq_fac", "radice_lwr", "radice_upr", "radice_fac"}
    with netcdf_file(path, "w") as f:
        for name, a in arrays.items():
            a = np.asarray(a)
            if name in scalars:
                v = f.createVariable(name, np.float64, ())
                v.data[...] = float(a.ravel()[0])
                continue
            dn = []
            for k, n in enumerate(a.shape):
                d = "%s_d%d" % (name, k)
                f.createDimension(d, n)
                dn.append(d)
            v = f.createVariable(name, a.dtype, tuple(dn))
            v[:] = a
    return path
