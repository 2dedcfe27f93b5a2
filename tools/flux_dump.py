#!/usr/bin/env python3
"""Run the benchmarked step once and save its broadband fluxes: python tools/flux_dump.py <c3|c4|c5> <out.npz>.

The library is the one RRTMGPNN_LIB names (default: the in-tree bitwise build), so the opt-in tolerance build
(librrtmgpnn_fastlibm.so) can be compared with the oracle in a separate process (tests/test_gpu_tolerance.py).
c5: the full C5 shard (125 000 synthetic columns x 137 layers) is stepped and a strided sample of 500 columns saved,
with their indices ("idx")."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rte-rrtmgp-nn_amd"))
from rrtmgpnn import data  # noqa: E402
from rrtmgpnn.pipeline import ClearSkyStep  # noqa: E402


def c5_sample(ncol=125000, n=500):
    """The C5 shard columns flux_dump saves (every shard column's first and last among them)."""
    return np.unique(np.concatenate([np.linspace(0, ncol - 1, n).astype(np.int64), [ncol - 1]]))


def problem(cfg):
    if cfg == "c3":
        return data.rfmip_problem(), None
    if cfg == "c5":
        return data.synthetic_problem(125000, 137, seed=20251015), None
    prob = data.synthetic_problem(2000, 60, seed=20251015)
    return prob, data.allsky_clouds(prob, data.load_cloud_optics("lw"))


def main():
    cfg, out = sys.argv[1], sys.argv[2]
    prob, clouds = problem(cfg)
    torch.cuda.set_device(0)
    step = ClearSkyStep(prob, device=0, clouds=clouds)
    step.step()
    torch.cuda.synchronize()
    f = step.fluxes()
    if cfg == "c5":
        idx = c5_sample(prob["ncol"])
        f = dict({k: v[idx] for k, v in f.items()}, idx=idx)
    np.savez(out, **f)
    step.close()


if __name__ == "__main__":
    main()
