"""ctypes binding of librrtmgpnn.so (the C ABI declared in include/rrtmgpnn.h).

The shared library is built in-tree (rte-rrtmgp-nn_amd/librrtmgpnn.so, `make -C rte-rrtmgp-nn_amd`).
There is deliberately NO fallback: if the HIP library cannot be loaded the product path
raises, so a test can never pass on a silent CPU implementation.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# RRTMGPNN_LIB: another build of the same library (tools/solver_variants.sh variants under a profiler)
LIB_PATH = os.environ.get("RRTMGPNN_LIB") or os.path.normpath(os.path.join(_HERE, "..", "librrtmgpnn.so"))

c_int, c_float, c_ll, c_vp, c_char_p = ctypes.c_int, ctypes.c_float, ctypes.c_longlong, ctypes.c_void_p, ctypes.c_char_p
P = ctypes.POINTER

# name -> (restype, argtypes); mirrors include/rrtmgpnn.h one-to-one.
SIGNATURES = {
    "rrtmgpnn_version": (c_int, []),
    "rrtmgpnn_last_error": (c_char_p, []),
    "rrtmgpnn_context_create": (c_int, [c_int, c_vp, P(c_vp)]),
    "rrtmgpnn_context_destroy": (c_int, [c_vp]),
    "rrtmgpnn_context_set_stream": (c_int, [c_vp, c_vp]),
    "rrtmgpnn_context_set_sw_kernel": (c_int, [c_vp, c_int]),
    "rrtmgpnn_context_set_mlp_kernel": (c_int, [c_vp, c_int]),
    "rrtmgpnn_context_set_mlp_max_cus": (c_int, [c_vp, c_int]),
    "rrtmgpnn_context_get_mlp_max_cus": (c_int, [c_vp, ctypes.POINTER(c_int)]),
    "rrtmgpnn_context_unpin_workspace": (c_int, [c_vp]),
    "rrtmgpnn_sw_solver_noscat": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp]),
    "rrtmgpnn_context_stream": (c_vp, [c_vp]),
    "rrtmgpnn_context_synchronize": (c_int, [c_vp]),
    "rrtmgpnn_malloc": (c_int, [c_vp, c_ll, P(c_vp)]),
    "rrtmgpnn_free": (c_int, [c_vp, c_vp]),
    "rrtmgpnn_memcpy_h2d": (c_int, [c_vp, c_vp, c_vp, c_ll]),
    "rrtmgpnn_memcpy_d2h": (c_int, [c_vp, c_vp, c_vp, c_ll]),
    "rrtmgpnn_context_create_owned": (c_int, [c_int, P(c_vp)]),
    "rrtmgpnn_present": (c_int, [c_vp, c_vp, c_ll, c_int, P(c_vp)]),
    "rrtmgpnn_present_update_host": (c_int, [c_vp, c_vp]),
    "rrtmgpnn_present_update_device": (c_int, [c_vp, c_vp]),
    "rrtmgpnn_present_delete": (c_int, [c_vp, c_vp]),
    "rrtmgpnn_stage_h2d": (c_int, [c_vp, c_vp, c_ll, P(c_vp)]),
    "rrtmgpnn_scratch": (c_int, [c_vp, c_ll, P(c_vp)]),
    "rrtmgpnn_release": (c_int, [c_vp, c_vp]),
    "rrtmgpnn_copy_d2h": (c_int, [c_vp, c_vp, c_vp, c_ll]),
    "rrtmgpnn_copy_h2d": (c_int, [c_vp, c_vp, c_vp, c_ll]),
    "rrtmgpnn_copy_d2d": (c_int, [c_vp, c_vp, c_vp, c_ll]),
    "rrtmgpnn_memset_async": (c_int, [c_vp, c_vp, c_int, c_ll]),
    "rrtmgpnn_network_load": (c_int, [c_vp, c_char_p, P(c_vp)]),
    "rrtmgpnn_network_create": (c_int, [c_vp, c_int, P(c_int), P(c_int), P(c_vp), P(c_vp), c_vp, c_vp, c_vp, c_vp,
                                        c_char_p, P(c_vp)]),
    "rrtmgpnn_network_destroy": (c_int, [c_vp]),
    "rrtmgpnn_network_get_dims": (c_int, [c_vp, P(c_int), P(c_int)]),
    "rrtmgpnn_network_get_input_name": (c_int, [c_vp, c_int, c_char_p, c_int]),
    "rrtmgpnn_network_get_input_scaling": (c_int, [c_vp, c_vp, c_vp]),
    "rrtmgpnn_compute_nn_inputs": (c_int, [c_vp, c_int, c_int, c_int, c_vp, c_vp, P(c_vp), P(c_int), c_vp, c_vp]),
    "rrtmgpnn_get_col_dry": (c_int, [c_vp, c_int, c_int, c_vp, c_vp, c_vp]),
    "rrtmgpnn_interpolate_tlev": (c_int, [c_vp, c_int, c_int, c_vp, c_vp, c_vp, c_vp]),
    "rrtmgpnn_predict_nn_lw": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_vp, c_vp, P(c_vp), c_int, c_vp, c_vp]),
    "rrtmgpnn_predict_nn_sw": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_vp, c_vp, P(c_vp), c_vp, c_vp, c_vp]),
    "rrtmgpnn_gas_optics_lw_nn": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp, P(c_vp), P(c_int),
                                          P(c_vp), c_int, c_vp, c_vp]),
    "rrtmgpnn_gas_optics_sw_nn": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp, P(c_vp), P(c_int),
                                          P(c_vp), c_vp, c_vp, c_vp]),
    "rrtmgpnn_network_forward": (c_int, [c_vp, c_vp, c_ll, c_vp, c_vp]),
    "rrtmgpnn_compute_planck_source_nn": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_int,
                                                  P(c_int), c_float, c_float, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "rrtmgpnn_lw_solver_noscat": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_int, P(c_float), P(c_float), c_vp, c_vp,
                                          c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "rrtmgpnn_lw_solver_noscat_planck": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_int, P(c_float), P(c_float),
                                                 c_vp, c_vp, c_vp, c_int, c_int, c_vp, c_vp, c_vp, c_int, P(c_int),
                                                 c_float, c_float, c_vp, c_int, c_vp, c_vp, c_vp]),
    "rrtmgpnn_lw_solver_noscat_planck_inc": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_int, P(c_float),
                                                     P(c_float), c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_vp, c_vp,
                                                     c_vp, c_int, P(c_int), c_float, c_float, c_vp, c_int, c_vp,
                                                     c_vp, c_vp]),
    "rrtmgpnn_sw_solver_2stream_inc": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp,
                                               c_int, P(c_int), c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                               c_vp]),
    "rrtmgpnn_lw_solver_1rescl": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_int, P(c_float), P(c_float)]
                                  + [c_vp] * 10),
    "rrtmgpnn_lw_solver_2stream": (c_int, [c_vp, c_int, c_int, c_int, c_int] + [c_vp] * 9),
    "rrtmgpnn_sw_solver_2stream": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                           c_vp, c_vp, c_vp, c_vp, c_vp]),
    "rrtmgpnn_lw_solver_noscat_gpt": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_int, P(c_float), P(c_float)]
                                      + [c_vp] * 11),
    "rrtmgpnn_lw_solver_noscat_planck_gpt": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_int, P(c_float),
                                                     P(c_float), c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_vp, c_vp,
                                                     c_vp, c_int, P(c_int), c_float, c_float, c_vp, c_int, c_vp,
                                                     c_vp, c_vp, c_vp, c_vp]),
    "rrtmgpnn_sw_solver_2stream_gpt": (c_int, [c_vp, c_int, c_int, c_int, c_int] + [c_vp] * 14),
    "rrtmgpnn_lw_solver_1rescl_gpt": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_int, P(c_float), P(c_float)]
                                      + [c_vp] * 12),
    "rrtmgpnn_lw_solver_2stream_gpt": (c_int, [c_vp, c_int, c_int, c_int, c_int] + [c_vp] * 11),
    "rrtmgpnn_sw_solver_noscat_gpt": (c_int, [c_vp, c_int, c_int, c_int, c_int] + [c_vp] * 5),
    "rrtmgpnn_expand_band_to_gpt": (c_int, [c_vp, c_int, c_int, c_int, P(c_int), c_vp, c_vp]),
    "rrtmgpnn_compute_heating_rate": (c_int, [c_vp, c_int, c_int, c_vp, c_vp, c_vp, c_vp]),
    "rrtmgpnn_calc_heating_rate_k_day": (c_int, [c_vp, c_int, c_int, c_vp, c_vp, c_vp, c_vp]),
    "rrtmgpnn_cloud_optics_create_lut": (c_int, [c_vp, c_int, P(c_float), c_int, c_int, c_int, c_float, c_float,
                                                 c_float, c_float, P(c_float), P(c_float), P(c_float), P(c_float),
                                                 P(c_float), P(c_float), P(c_vp)]),
    "rrtmgpnn_cloud_optics_create_pade": (c_int, [c_vp, c_int, P(c_float), c_int, c_int, c_int, c_int]
                                          + [P(c_float)] * 12 + [P(c_vp)]),
    "rrtmgpnn_cloud_optics_load": (c_int, [c_vp, c_char_p, c_int, P(c_vp)]),
    "rrtmgpnn_cloud_optics_set_ice_roughness": (c_int, [c_vp, c_int]),
    "rrtmgpnn_cloud_optics_get": (c_int, [c_vp, P(c_int), P(c_int), P(c_float)]),
    "rrtmgpnn_cloud_optics_destroy": (c_int, [c_vp]),
    "rrtmgpnn_cloud_optics_compute": (c_int, [c_vp, c_vp, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "rrtmgpnn_increment_bybnd": (c_int, [c_vp, c_int, c_int, c_int, c_int, P(c_int), c_vp, c_vp, c_vp, c_vp, c_vp,
                                         c_vp]),
    "rrtmgpnn_increment": (c_int, [c_vp, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "rrtmgpnn_delta_scale_2str": (c_int, [c_vp, c_ll, c_vp, c_vp, c_vp, c_vp]),
    "rrtmgpnn_sw_boundary_rfmip": (c_int, [c_vp, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "rrtmgpnn_sw_solver_2stream_rfmip": (c_int, [c_vp, c_int, c_int, c_int, c_int] + [c_vp] * 7
                                         + [c_int, P(c_int)] + [c_vp] * 9),
    "rrtmgpnn_file_open": (c_int, [c_char_p, P(c_vp)]),
    "rrtmgpnn_file_close": (c_int, [c_vp]),
    "rrtmgpnn_file_nvars": (c_int, [c_vp, P(c_int)]),
    "rrtmgpnn_file_var_name": (c_int, [c_vp, c_int, c_char_p, c_int]),
    "rrtmgpnn_file_var": (c_int, [c_vp, c_char_p, P(c_int), P(c_int), P(c_ll)]),
    "rrtmgpnn_file_read": (c_int, [c_vp, c_char_p, c_int, c_vp, c_ll]),
    "rrtmgpnn_file_att": (c_int, [c_vp, c_char_p, c_char_p, c_char_p, c_int]),
}


class RrtmgpnnError(RuntimeError):
    pass


_lib = None


def lib():
    """Load (once) and return the ctypes handle; raises if the HIP library is missing."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RrtmgpnnError("librrtmgpnn.so not found at %s: build it with `make -C rte-rrtmgp-nn_amd` "
                                "(no CPU fallback exists by design)" % LIB_PATH)
        h = ctypes.CDLL(LIB_PATH)
        # an RRTMGPNN_LIB override (A/B runs against builds of older trees) may lack newer entry points; the
        # shipped library must export every one (tests/test_host.py checks include/rrtmgpnn.h against it)
        lenient = bool(os.environ.get("RRTMGPNN_LIB"))
        for name, (res, args) in SIGNATURES.items():
            if lenient and not hasattr(h, name):
                continue
            f = getattr(h, name)
            f.restype = res
            f.argtypes = args
        _lib = h
    return _lib


_hip = None


def _hip_runtime():
    """The process's HIP runtime (torch's libamdhip64.so.7, which librrtmgpnn.so also binds by soname)."""
    global _hip
    if _hip is None:
        h = ctypes.CDLL("libamdhip64.so.7")
        h.hipStreamCreateWithPriority.restype = c_int
        h.hipStreamCreateWithPriority.argtypes = [P(c_vp), ctypes.c_uint, c_int]
        h.hipSetDevice.restype = c_int
        h.hipSetDevice.argtypes = [c_int]
        _hip = h
    return _hip


_free_streams = {}  # (device, priority) -> handles released by their last owner


def stream_acquire(device, priority=0):
    """A non-blocking HIP stream held by one owner at a time (ClearSkyStep), not one of torch's pooled streams, which
    torch hands to every caller round-robin: a stream a closed owner released, or a new one.  Streams are never
    destroyed: events recorded on a stream (torch's pinned-memory allocator keeps such events and queries them after
    their tensors are freed) reference its queue, and a destroyed stream's queue is freed memory -- bench.py crashed in
    exactly that way when close() destroyed the step's streams (round 6)."""
    key = (int(device), int(priority))
    if _free_streams.get(key):
        return _free_streams[key].pop()
    h = _hip_runtime()
    s = c_vp()
    rc = h.hipSetDevice(int(device)) or h.hipStreamCreateWithPriority(ctypes.byref(s), 1, int(priority))
    if rc:
        raise RrtmgpnnError("hipStreamCreateWithPriority failed (hip error %d)" % rc)
    return s.value


def stream_release(handle, device, priority=0):
    """Give a stream back once its owner's work on it is complete (the next owner's work is ordered after it anyway:
    the stream is in-order)."""
    if handle:
        _free_streams.setdefault((int(device), int(priority)), []).append(handle)


def check(rc, what=""):
    if rc != 0:
        msg = lib().rrtmgpnn_last_error().decode(errors="replace")
        raise RrtmgpnnError("%s failed (code %d): %s" % (what or "rrtmgpnn call", rc, msg))


def int_array(vals):
    return (c_int * len(vals))(*[int(v) for v in vals])


def float_array(vals):
    return (c_float * len(vals))(*[float(v) for v in vals])


def ptr_array(ptrs):
    return (c_vp * len(ptrs))(*[p if p else None for p in ptrs])
