"""rrtmgpnn -- MI355X-native RTE+RRTMGP-NN hot path (host-side Python mirror of the reference API).

Submodules:
  rbin      RBIN container I/O (numpy only)
  data      model files, surrogate k-distribution tables, RFMIP / synthetic problem builders
  _lib      ctypes binding of librrtmgpnn.so (include/rrtmgpnn.h); raises if the library is missing
  api       mirror of the reference's class layer: rrtmgp_network_type, ty_gas_concs,
            ty_optical_props_1scl/2str, ty_source_func_lw, ty_fluxes_broadband,
            ty_gas_optics_rrtmgp%gas_optics, rte_lw, rte_sw  (torch device tensors)
  pipeline  fused clear-sky LW+SW step used by bench.py and the multi-GPU driver
"""
__all__ = ["rbin", "data"]
