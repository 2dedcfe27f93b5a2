#!/usr/bin/env python3
"""Exhaustive float32 check of the exact rewrites the SW solvers use for g = 0 (the NN path's g is identically zero,
mo_gas_optics_rrtmgp.F90:560-567), against sw_two_stream's own expressions (rte/kernels/mo_rte_solver_kernels.F90:
1366-1480, as the oracle writes them, oracle/rrtmgpnn_oracle.c):

  gamma1 = (8 - w*(5 + 3g)) * .25       ->  2 - w*1.25
  gamma2 = 3*(w*(1 - g)) * .25          ->  w*.75
  alpha1 = gamma1*gamma4 + gamma2*gamma3 and alpha2 = gamma1*gamma3 + gamma2*gamma4, with gamma3 = gamma4 = .5
                                        ->  (gamma1 + gamma2) * .5

for every float32 w with |w| < 6.8e37 (all their bit patterns; NaNs compared as NaNs).  Each is one rounding of the
same real value where the reference rounds a power-of-two multiple of it, so they agree except possibly in the
subnormal range, which this walks too.  Beyond 6.8e37 the reference's w*5 (or 3*w) overflows to inf while the rewrite
stays finite: those w are reported separately (an ssa is a ratio in [0, 1]).  numpy float32 arithmetic is IEEE single precision with round-to-nearest-even, as the device's is.

    python tools/check_sw_identities.py          (about a minute on one core)
"""
import sys

import numpy as np


def check(chunk_bits=1 << 26):
    f = np.float32
    bad = {"gamma1": 0, "gamma2": 0, "alpha": 0}
    overflow = 0
    with np.errstate(all="ignore"):
        for start in range(0, 1 << 32, chunk_bits):
            w = np.arange(start, start + chunk_bits, dtype=np.uint64).astype(np.uint32).view(np.float32)
            g = f(0)
            g1_ref = (f(8) - w * (f(5) + f(3) * g)) * f(.25)
            g2_ref = f(3) * (w * (f(1) - g)) * f(.25)
            g3 = (f(2) - f(3) * f(0.6) * g) * f(.25)  # any mu0: g = 0 makes it exactly .5
            g4 = f(1) - g3
            a1_ref = g1_ref * g4 + g2_ref * g3
            a2_ref = g1_ref * g3 + g2_ref * g4
            g1 = f(2) - w * f(1.25)
            g2 = w * f(.75)
            a = (g1 + g2) * f(.5)

            inr = np.abs(w) < f(6.8e37)
            overflow += int((~inr & ~np.isnan(w)).sum())

            def ne(x, y):
                return inr & ~((x.view(np.uint32) == y.view(np.uint32)) | (np.isnan(x) & np.isnan(y)))
            bad["gamma1"] += int(ne(g1, g1_ref).sum())
            bad["gamma2"] += int(ne(g2, g2_ref).sum())
            bad["alpha"] += int((ne(a, a1_ref) | ne(a, a2_ref)).sum())
    return bad, overflow


if __name__ == "__main__":
    res, overflow = check()
    print("mismatches for |w| < 6.8e37:", res, "(floats beyond, not compared: %d)" % overflow)
    sys.exit(1 if any(res.values()) else 0)
