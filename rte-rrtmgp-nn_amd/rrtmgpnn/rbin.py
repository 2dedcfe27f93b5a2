"""RBIN: the framework's own container for named float32/int32/char arrays.

Layout (little endian):
    b"RBIN"  u32 version(=1)  u32 count
    repeated `count` times:
        char name[64] (NUL padded)
        u32 dtype      0 = float32, 1 = int32, 2 = uint8 (character data)
        u32 ndim
        u32 dims[ndim] (C / row-major order)
        payload        prod(dims) * itemsize bytes

The same format is parsed by the C++ runtime (csrc/rbin.hpp), the Fortran host
glue (fortran/mo_rrtmgpnn_rbin.F90) and this module.  It replaces netCDF for the
files the reference reads through netcdf-fortran (NN models,
`neural/mod_network_rrtmgp.F90:58-122`; RFMIP inputs,
`examples/rfmip-clear-sky/mo_rfmip_io.F90:74-680`), which is absent here.
This file is importable with any numpy (no torch), so the conversion script can
run under the conda interpreter that has h5py.
"""
import struct

import numpy as np

_DT = {0: np.float32, 1: np.int32, 2: np.uint8}
_CODE = {np.dtype(np.float32): 0, np.dtype(np.int32): 1, np.dtype(np.uint8): 2}


def write(path, arrays):
    """Write an ordered mapping name -> ndarray."""
    with open(path, "wb") as f:
        f.write(b"RBIN")
        f.write(struct.pack("<II", 1, len(arrays)))
        for name, a in arrays.items():
            a = np.ascontiguousarray(a)
            if a.dtype == np.float64:
                a = a.astype(np.float32)
            if a.dtype == np.int64:
                a = a.astype(np.int32)
            code = _CODE[a.dtype]
            nb = name.encode()
            assert len(nb) < 64, name
            f.write(nb + b"\0" * (64 - len(nb)))
            f.write(struct.pack("<II", code, a.ndim))
            f.write(struct.pack("<%dI" % a.ndim, *a.shape))
            f.write(a.astype(a.dtype.newbyteorder("<")).tobytes())


def read(path):
    """Read an RBIN file into a dict name -> ndarray (insertion ordered)."""
    out = {}
    with open(path, "rb") as f:
        buf = f.read()
    if buf[:4] != b"RBIN":
        raise ValueError("%s: not an RBIN file" % path)
    ver, count = struct.unpack_from("<II", buf, 4)
    if ver != 1:
        raise ValueError("%s: unsupported RBIN version %d" % (path, ver))
    off = 12
    for _ in range(count):
        name = buf[off:off + 64].split(b"\0")[0].decode()
        off += 64
        code, ndim = struct.unpack_from("<II", buf, off)
        off += 8
        dims = struct.unpack_from("<%dI" % ndim, buf, off)
        off += 4 * ndim
        dt = np.dtype(_DT[code]).newbyteorder("<")
        n = int(np.prod(dims)) if ndim else 1
        a = np.frombuffer(buf, dtype=dt, count=n, offset=off).reshape(dims).copy()
        off += n * dt.itemsize
        out[name] = a
    return out


def chars(names, width=32):
    """Fortran-style fixed-width, space-padded character array (n, width) uint8."""
    a = np.full((len(names), width), ord(" "), dtype=np.uint8)
    for i, s in enumerate(names):
        b = s.encode()[:width]
        a[i, :len(b)] = np.frombuffer(b, dtype=np.uint8)
    return a


def unchars(a):
    return [bytes(r).decode().strip() for r in np.asarray(a, dtype=np.uint8)]
