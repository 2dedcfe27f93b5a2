"""Native data-file reading through the C ABI (rrtmgpnn_file_*, csrc/datafile.cpp): classic netCDF, netCDF-4
(HDF5) and RBIN, all into numpy arrays in file (C) order.  This replaces the netCDF-Fortran reads of the
reference's drivers (neural/mod_network_rrtmgp.F90:58-122, examples/rfmip-clear-sky/mo_rfmip_io.F90,
examples/all-sky/mo_load_cloud_coefficients.F90) -- SURVEY.md 8(f) row f-3.  Host-only: no GPU is touched.
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import check

_DT = {0: np.float32, 1: np.int32, 2: np.uint8}


class DataFile:
    """A data file read whole: `vars` lists the variables, `read(name)` returns an array, `att(var, name)` text."""

    def __init__(self, path):
        L = _lib.lib()
        h = _lib.c_vp()
        check(L.rrtmgpnn_file_open(str(path).encode(), h), "file_open(%s)" % path)
        self.h, self.path = h, str(path)
        n = _lib.c_int()
        check(L.rrtmgpnn_file_nvars(h, n), "file_nvars")
        buf = ctypes.create_string_buffer(256)
        self.vars = []
        for i in range(n.value):
            check(L.rrtmgpnn_file_var_name(h, i, buf, 256), "file_var_name")
            self.vars.append(buf.value.decode())

    def __contains__(self, name):
        return name in self.vars

    def info(self, name):
        dt, nd = _lib.c_int(), _lib.c_int()
        dims = (ctypes.c_longlong * 8)()
        check(_lib.lib().rrtmgpnn_file_var(self.h, name.encode(), dt, nd, dims), "file_var(%s)" % name)
        return dt.value, tuple(int(dims[k]) for k in range(nd.value))

    def read(self, name, dtype=None):
        """The variable as float32 (floating point), int32 (integers) or uint8 (characters); `dtype` converts
        numeric variables (np.float32 / np.int32)."""
        dt, shape = self.info(name)
        if dtype is not None and dt != 2:
            dt = 0 if np.dtype(dtype) == np.float32 else 1
        out = np.empty(shape, _DT[dt])
        check(_lib.lib().rrtmgpnn_file_read(self.h, name.encode(), dt, out.ctypes.data, out.size),
              "file_read(%s)" % name)
        return out

    def strings(self, name):
        """A (n, len) character variable as a list of stripped strings."""
        a = self.read(name)
        return [bytes(r).decode(errors="replace").replace("\0", " ").strip() for r in a.reshape(a.shape[0], -1)]

    def att(self, var, name):
        buf = ctypes.create_string_buffer(1024)
        check(_lib.lib().rrtmgpnn_file_att(self.h, (var or "").encode(), name.encode(), buf, 1024),
              "file_att(%s:%s)" % (var, name))
        return buf.value.decode()

    def close(self):
        if getattr(self, "h", None):
            _lib.lib().rrtmgpnn_file_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def read(path):
    """Every variable of a file as {name: array}."""
    with DataFile(path) as f:
        return {v: f.read(v) for v in f.vars}


# examples/rfmip-clear-sky/mo_rfmip_io.F90:323-358 (forcing_index = 1): chemical name -> RFMIP variable
RFMIP_GASES = {"co2": "carbon_dioxide", "n2o": "nitrous_oxide", "ch4": "methane", "co": "carbon_monoxide",
               "ccl4": "carbon_tetrachloride", "cfc22": "hcfc22", "o2": "oxygen", "n2": "nitrogen",
               "cfc11": "cfc11", "cfc12": "cfc12", "hfc143a": "hfc143a", "hfc125": "hfc125",
               "hfc23": "hfc23", "hfc32": "hfc32", "hfc134a": "hfc134a", "cf4": "cf4"}


def rfmip_fields(path):
    """The RFMIP input file (multiple_input4MIPs_radiation_RFMIP_*.nc) read natively, with the drivers' unit
    scaling (mo_rfmip_io.F90:520-560, 640-652, 683-698: value * real(units attribute)); the same fields the
    RBIN conversion holds (rrtmgpnn.data.rfmip_problem consumes either)."""
    with DataFile(path) as f:
        out = {v: f.read(v, np.float32) for v in
               ("pres_layer", "pres_level", "temp_layer", "temp_level", "surface_temperature", "surface_emissivity",
                "surface_albedo", "solar_zenith_angle", "total_solar_irradiance", "profile_weight", "lat", "lon")}
        scale = lambda v: np.float32(float(f.att(v, "units")))  # noqa: E731
        out["h2o"] = (f.read("water_vapor", np.float32) * scale("water_vapor")).astype(np.float32)
        out["o3"] = (f.read("ozone", np.float32) * scale("ozone")).astype(np.float32)
        for chem, name in RFMIP_GASES.items():
            v = name + "_GM"
            out["gm_" + chem] = (scale(v) * f.read(v, np.float32)).astype(np.float32)
    return out
