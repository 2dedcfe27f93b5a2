#!/usr/bin/env python3
"""Calibrate rocprofv3's FETCH_SIZE / WRITE_SIZE at the solvers' access widths (tools/pmc_calib.hip).

usage: pmc_calib.py run <lib.so>                  (the GPU program: run it under rocprofv3 --pmc FETCH_SIZE, then WRITE_SIZE)
       pmc_calib.py parse <fetch_dir> <write_dir> [out.json]
       pmc_calib.py valu <lib.so>                 (fma_kernel<float/double>: run under rocprofv3 --pmc SQ_* counters;
                                                   prints the hipEvent times and v_fma rates)
Prints, per calibration kernel, counter bytes (KiB * 1024, no correction) / true bytes moved.  Buffers exceed the
256 MiB Infinity Cache so the counted traffic is HBM traffic (MI355X_MICROARCH.md, HBM and L3 sections).
"""
import csv
import ctypes
import glob
import json
import os
import re
import sys

GiB = 1 << 30
NGPT, NLEV, NCOL = 224, 61, 10000  # the C4 SW workspace plane


def run(lib):
    import torch
    L = ctypes.CDLL(lib)
    buf = torch.zeros(GiB // 4, dtype=torch.float32, device="cuda")
    out = torch.zeros(1, dtype=torch.float32, device="cuda")
    col = torch.zeros(NGPT * NLEV * NCOL, dtype=torch.float32, device="cuda")
    vp = ctypes.c_void_p
    for w in (4, 8, 16):
        assert L.calib_read(w, vp(buf.data_ptr()), ctypes.c_size_t(GiB), vp(out.data_ptr())) == 0
        torch.cuda.synchronize()
        assert L.calib_write(w, vp(buf.data_ptr()), ctypes.c_size_t(GiB)) == 0
        torch.cuda.synchronize()
    for w in (4, 8):
        for st in (0, 1):
            assert L.calib_column(w, st, vp(col.data_ptr()), NGPT, NLEV, NCOL, vp(out.data_ptr())) == 0
            torch.cuda.synchronize()


def true_bytes(kernel):
    if "column_kernel" in kernel:
        return 4 * NGPT * NLEV * NCOL
    return GiB


def read_pass(d, counter):
    acc = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                k = re.sub(r"\(.*", "", row["Kernel_Name"]).replace("void ", "")
                s, n = acc.get(k, (0.0, 0))
                acc[k] = (s + float(row["Counter_Value"]), n + 1)
    return {k: s / n for k, (s, n) in acc.items()}


def parse(fdir, wdir, out=None):
    fetch, write = read_pass(fdir, "FETCH_SIZE"), read_pass(wdir, "WRITE_SIZE")
    res = {}
    for k in sorted(set(fetch) | set(write)):
        tb = true_bytes(k)
        store = "write_kernel" in k or "true>" in k
        c = (write if store else fetch).get(k)
        if c is None:
            continue
        res[k] = {"counter": "WRITE_SIZE" if store else "FETCH_SIZE", "true_bytes": tb,
                  "counter_bytes": round(1024.0 * c), "ratio": round(1024.0 * c / tb, 4)}
    txt = json.dumps(res, indent=1)
    print(txt)
    if out:
        with open(out, "w") as fh:
            fh.write(txt)


FMA_BLOCKS, FMA_NIT = 256 * 16, 4096


def valu(lib):
    import torch
    L = ctypes.CDLL(lib)
    L.calib_fma.restype = ctypes.c_float
    out = torch.zeros(2, dtype=torch.float64, device="cuda")
    res = {}
    for kind, name, per in ((0, "v_fma_f32", 1), (1, "v_fma_f64", 1), (2, "v_pk_fma_f32", 2)):
        L.calib_fma(kind, ctypes.c_void_p(out.data_ptr()), FMA_BLOCKS, 16)  # warm
        ms = L.calib_fma(kind, ctypes.c_void_p(out.data_ptr()), FMA_BLOCKS, FMA_NIT)
        waves = FMA_BLOCKS * 4
        insts = 8 * FMA_NIT * waves
        res[name] = {"ms": round(ms, 4), "wave_insts": insts, "cycles_per_inst_per_simd_at_2.4GHz":
                     round(ms * 1e-3 * 2.4e9 * 1024 / insts, 2),
                     "tflops": round(2 * 64 * per * insts / (ms * 1e-3) / 1e12, 1)}
    print(json.dumps(res))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2])
    elif sys.argv[1] == "valu":
        valu(sys.argv[2])
    else:
        parse(*sys.argv[2:])
