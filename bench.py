#!/usr/bin/env python3
"""bench.py -- clear-sky LW+SW fluxes (RTE+RRTMGP-NN hot path) on 1..N MI355X.

Metric (BASELINE.json): atmospheric columns/s for LW+SW clear-sky fluxes.  Workload at N=1:
configs[2] "RFMIP clear-sky LW+SW, 1800 columns x 60 layers, NN gas optics both streams"
(the real RFMIP inputs shipped with the reference + the reference's NN weights).  A step is
gas_optics(LW, NN) + rte_lw + gas_optics(SW, NN) + rte_sw over the block, inputs resident in HBM.

Multi-GPU: `python bench.py --gpus N` starts its own N rank processes (torch.distributed.run, rendezvous
on 127.0.0.1) before touching the GPU, and the driver's `python -m torch.distributed.run --nproc-per-node
N bench.py --gpus N` runs the same ranks directly (WORLD_SIZE must then equal N).  One process per
GPU.  The job is one global problem partitioned by rrtmgpnn.shard.column_range (the gloo-tested
partition): by default N x the config's block (weak scaling, N x 1800 RFMIP columns at C3, each rank
a 1800-column block); with --global the config's fixed global size (C5: 1e6 synthetic columns x 137
layers, strong scaling), each rank streaming its range through the step in chunks of at most
125 000 columns.  No collective in the data path; barrier + synchronize around the timed region, max
over ranks.  After timing, the broadband fluxes are all-gathered once with shard.gather_columns over
RCCL (the final flux reduction the north star names), timed as "gather_ms" and folded into
"end_to_end" (all columns / (timed steps + gather)), never into `value`; every rank then checks the
gathered array against every rank's own slab ("gather_check"; a failure exits non-zero).

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "rte-rrtmgp-nn_amd"))

METRIC = "atmospheric columns/sec (LW+SW clear-sky fluxes), 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0       # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
FP32_MFMA_PEAK_TFS = 157.3  # MI355X_MICROARCH.md: FP32 matrix 157.3 TFLOP/s (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--settle-s", type=float, default=1.0,
                    help="untimed steps for this many seconds before the warmup steps (the GPU's clocks ramp up over "
                         "the first ~0.1 s of steps: 20 steps after 5 warmup steps ran 0.53 ms/step at C3 where "
                         "steady state is 0.44-0.45); reported as settle_s / settle_steps")
    ap.add_argument("--config", default="c3", choices=["c1", "c2", "c3", "c4", "c5"],
                    help="c3: RFMIP 1800x60 LW+SW (default, the metric's config); c1: the first 100 RFMIP columns, LW "
                         "only (BASELINE configs[0], the reference's CPU case); c2: the 1800 columns, LW only "
                         "(BASELINE configs[1], metric in LW columns/s); c4: 10000x60 synthetic all-sky; "
                         "c5: 125000x137 synthetic clear-sky per GPU")
    ap.add_argument("--global", dest="global_cols", nargs="?", type=int, const=-1, default=0,
                    help="partition one global problem of this many columns over the ranks (strong scaling; "
                         "without a value the config's global size: C5 1e6 columns); default: N x the config's block")
    ap.add_argument("--no-graph", action="store_true", help="launch eagerly instead of replaying a hipGraph")
    ap.add_argument("--no-overlap", action="store_true", help="issue the SW chain on the same stream as LW")
    ap.add_argument("--lw-after", default="", help="start the LW chain after this SW-chain call (e.g. predict_nn_sw; none: chains start together; default: the library pipeline's choice)")
    ap.add_argument("--sw-after", default="", help="the SW solver waits for this LW-chain call (predict_nn_lw: both "
                    "networks first, then the solvers side by side; none: no wait; default: the library pipeline's "
                    "choice)")
    ap.add_argument("--sw-priority", type=int, default=0, help="priority of the SW chain's stream (-1: high)")
    ap.add_argument("--sw-net-cus", type=int, default=0, help="the SW network's blocks on at most this many CUs (0: all)")
    ap.add_argument("--lw-net-cus", type=int, default=None,
                    help="the LW network's blocks on at most this many CUs (0: all; default: the library pipeline's "
                         "choice: 3/8 of the CUs at small grids, where the LW chain follows the SW network)")
    ap.add_argument("--unfused", action="store_true",
                    help="issue the class layer's exact call sequence (Planck sources and g materialised in HBM)")
    ap.add_argument("--sw-kernel", type=int, default=0, choices=[0, 1, 2, 3],
                    help="SW solver: 0 the library's choice, 1 / 2 g-points per lane, 3 checkpointed passes "
                         "(rrtmgpnn_context_set_sw_kernel)")
    ap.add_argument("--fortran", action="store_true",
                    help="time the Fortran drop-in instead: rrtmgpnn_rfmip_clear_sky's block loop on the C3 columns "
                         "(host arrays in and out, as a reference driver calls it)")
    ap.add_argument("--fortran-block", type=int, default=1800, help="--fortran: columns per block")
    ap.add_argument("--fortran-threads", type=int, default=1, help="--fortran: OpenMP threads over blocks")
    ap.add_argument("--c5-steps", type=int, default=3,
                    help="timed steps of the c5_global block every line carries (BASELINE configs[4]: 1e6 synthetic "
                         "columns x 137 layers split over the ranks, streamed in 125 000-column chunks); 0: skip it")
    ap.add_argument("--c5-warmup", type=int, default=1, help="untimed steps of the c5_global block")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="target CPU-baseline work")
    ap.add_argument("--cpu-kind", default="auto", choices=["auto", "reference", "port"],
                    help="auto: the reference's own Fortran (oracle/_ref) when built, else the C restatement")
    ap.add_argument("--cpu-bind", default="none", choices=["none", "close", "spread"],
                    help="OpenMP thread placement of the CPU baseline (OMP_PROC_BIND with OMP_PLACES=cores; none: "
                         "unbound, the default: on the GPU box 'close' put all 16 threads on 2 places, 10x slower)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    ap.add_argument("--sq-json", default=os.path.join(ROOT, "profiles", "pmc_sq.json"),
                    help="committed SQ counters per config/stage (tools/profile_configs.sh): valu_busy")
    return ap.parse_args()


# Algorithmic work per unit.  FLOPs count 2*n_in*n_out per sample and layer.
def mlp_flops(dims):
    return 2 * sum(dims[i] * dims[i + 1] for i in range(len(dims) - 1))


def stage_work(name, step):
    """(kind, amount per launch[, kind2, amount2]): 'flop' for MFMA stages, 'byte' for HBM stages (algorithmic:
    every array the stage must read once and write once)."""
    ncol, nlay = step.ncol, step.nlay
    N = ncol * nlay
    glw, gsw = step.ng_lw, step.ng_sw
    f4 = 4
    nsw_out = 2 if step.fused else 3  # tau, ssa (+ g when it is materialised)
    # all-sky, fused: the solvers also read the band-resolved cloud properties (1 LW, 3 SW arrays of nb x L)
    cld_lw = step.nb_lw * nlay * f4 if (step.allsky and step.fused) else 0
    cld_sw = 3 * step.nb_sw * nlay * f4 if (step.allsky and step.fused) else 0
    if name == "predict_nn_lw":
        from rrtmgpnn import data
        fl = sum(mlp_flops([int(v) for v in data.load_model(m)["dims"]]) for m in ("lw_abs", "lw_pfrac"))
        return "flop", fl * N, "bytes", N * (step.nx_lw + 1 + 2 * glw) * f4
    if name == "predict_nn_sw":
        from rrtmgpnn import data
        fl = sum(mlp_flops([int(v) for v in data.load_model(m)["dims"]]) for m in ("sw_abs", "sw_ray"))
        return "flop", fl * N, "bytes", N * (step.nx_sw + 1 + nsw_out * gsw) * f4
    if name == "lw_solver":
        if step.fused:
            # tau, pfrac (G x L) + emis (G) + tlay, tlev, tsfc read; flux up/dn written (124 880 B/col at L=60)
            return "byte", ncol * ((2 * glw * nlay + glw + 2 * nlay + 2) * f4 + 2 * (nlay + 1) * f4 + cld_lw), None, None
        # tau, lay (G x L) + lev (G x (L+1)) + emis, sfc (G) read; flux up/dn (L+1) written
        return "byte", ncol * ((2 * glw * nlay + glw * (nlay + 1) + 2 * glw) * f4 + 2 * (nlay + 1) * f4), None, None
    if name == "sw_solver":
        # tau, ssa (, g) (G x L) + toa, alb_dir, alb_dif (G) + mu0 read; up/dn/dir written
        return "byte", ncol * ((nsw_out * gsw * nlay + 3 * gsw + 1) * f4 + 3 * (nlay + 1) * f4 + cld_sw), None, None
    if name in ("cloud_optics_lw", "cloud_optics_sw"):
        # lwp, iwp, rel, rei read; 1 (LW 1scl) or 3 (SW 2str) by-band arrays written
        nb = step.nb_lw if name.endswith("lw") else step.nb_sw
        return "byte", N * (4 + (1 if name.endswith("lw") else 3) * nb) * f4, None, None
    if name == "delta_scale_sw":
        return "byte", N * 6 * step.nb_sw * f4, None, None
    if name == "increment_lw":
        return "byte", N * (2 * glw + step.nb_lw) * f4, None, None
    if name == "increment_sw":
        return "byte", N * (6 * gsw + 3 * step.nb_sw) * f4, None, None
    if name == "sw_boundary":
        # tsi, albedo, sza (+ the g-point source) read; toa and the per-g albedo (G) and mu0 written
        return "byte", ncol * (3 + 2 * gsw + 1) * f4 + gsw * f4, None, None
    if name == "planck_source":
        # pfrac read, lay (in place) + lev + sfc + sfcJac written
        return "byte", ncol * ((glw * nlay + glw * nlay + glw * (nlay + 1) + 2 * glw) * f4), None, None
    return "byte", 0, None, None


def fortran_bench(args):
    """--fortran: the Fortran drop-in measured through its own host program.  rrtmgpnn_rfmip_clear_sky
    (rte-rrtmgp-nn_amd/fortran, shaped like examples/rfmip-clear-sky/rrtmgp_rfmip_{lw,sw}.F90) runs its block loop
    --steps + 1 times over the 1800 C3 columns -- per block gas_optics -> rte_lw and gas_optics -> rte_sw through the
    reference's interfaces, state arrays copied in and fluxes copied out every call, optical properties and sources
    device-resident in between -- and reports the mean of the last --steps loops (system_clock)."""
    import re
    import subprocess
    import tempfile
    from rrtmgpnn import data
    exe = os.path.join(ROOT, "rte-rrtmgp-nn_amd", "fortran", "build", "rrtmgpnn_rfmip_clear_sky")
    prob = data.rfmip_columns(0, 1800)
    env = dict(os.environ, OMP_NUM_THREADS=str(args.fortran_threads))
    with tempfile.TemporaryDirectory() as td:
        pin, pout = os.path.join(td, "p.rbin"), os.path.join(td, "f.rbin")
        data.write_problem(prob, pin)
        r = subprocess.run([exe, pin, pout, data.DATA_DIR, str(args.fortran_block), str(args.steps + 1)],
                           capture_output=True, text=True, env=env, timeout=600)
    m = re.search(r"timing:\s*([0-9.]+) ms per block loop", r.stdout)
    if r.returncode != 0 or not m:
        raise SystemExit("bench --fortran: host program failed: " + (r.stdout + r.stderr)[-600:])
    ms = float(m.group(1))
    nblocks = (1800 + args.fortran_block - 1) // args.fortran_block
    print(json.dumps({
        "metric": METRIC, "value": round(1800 / (ms * 1e-3), 1), "unit": "columns/s", "n_gpus": 1,
        "steps": args.steps, "warmup": 1, "ms_per_step": round(ms, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32",
        "data": "real RFMIP inputs (reference's RFMIP file) + the reference's trained NN weights; surrogate k-dist tables",
        "config": {"workload": "C3 through the Fortran drop-in: rrtmgpnn_rfmip_clear_sky's block loop (gas_optics + "
                               "rte_lw, gas_optics + rte_sw per block; host arrays in, fluxes out)",
                   "global_columns": 1800, "nlay": 60, "block_size": args.fortran_block, "blocks": nblocks,
                   "threads": args.fortran_threads, "parallelism": "OpenMP over blocks, a device context per thread"},
        "column_layers_per_s": round(1800 * 60 / (ms * 1e-3), 1)}), flush=True)


def result_stream():
    """The stream for the result line alone: the process's fd 1 is pointed at stderr from here on, so whatever a
    library writes to stdout (gloo's connection notes under a launcher, runtime chatter) cannot mix with the one line
    the caller parses.  Returns a stream on the original stdout."""
    sys.stdout.flush()
    out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    return out


def main():
    args = parse()
    if args.fortran:
        fortran_bench(args)
        return
    import torch
    import torch.distributed as dist
    from rrtmgpnn import shard

    # --gpus N: under an outer launcher (torch.distributed.run) this process is one rank and WORLD_SIZE must equal
    # N; without one, N > 1 starts N rank processes here, before any GPU call in this process (a child process,
    # never an exec), and exits with their status -- rank 0 prints the line.  N = 1 runs in this process.
    try:
        plan = shard.launch_plan(args.gpus, os.environ)
    except ValueError as e:
        sys.stderr.write("bench.py: %s\n" % e)
        sys.exit(2)
    if plan == "spawn":
        sys.exit(shard.spawn_ranks(args.gpus, os.path.abspath(__file__), sys.argv[1:], torch.cuda.device_count()))

    result = result_stream()  # a rank (or the single process): only its result line reaches stdout
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    # one process per GPU; with more ranks than GPUs (rehearsing the N-rank path on a smaller box) ranks share
    # devices round-robin, and RRTMGPNN_DIST_BACKEND=gloo replaces RCCL, which refuses two ranks on one GPU
    ndev = max(1, torch.cuda.device_count())
    local = int(os.environ.get("LOCAL_RANK", "0")) % ndev
    backend = os.environ.get("RRTMGPNN_DIST_BACKEND", "nccl")
    if world > 1:
        kw = {"device_id": torch.device("cuda", local)} if backend == "nccl" else {}
        dist.init_process_group(backend, init_method="env://", world_size=world, rank=rank, **kw)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from rrtmgpnn import data
    from rrtmgpnn import _lib
    from rrtmgpnn.pipeline import ChunkedRank, ClearSkyStep

    # ---- the global problem and this rank's part of it (shard.column_range) ----
    metric = METRIC
    block = {"c1": 100, "c2": 1800, "c3": 1800, "c4": 10000, "c5": 125000}[args.config]
    nlay_cfg = 137 if args.config == "c5" else 60
    if args.global_cols:
        global_cols = 1000000 if (args.global_cols < 0 and args.config == "c5") else (
            args.global_cols if args.global_cols > 0 else block * world)
        scaling = "strong"
    else:
        global_cols = block * world
        scaling = "weak"
    lo, hi = shard.column_range(global_cols, rank, world)

    def problem(c0, c1):
        """Columns [c0, c1) of the global problem (and their clouds at C4)."""
        if args.config in ("c1", "c2", "c3"):
            return data.rfmip_columns(c0, c1 - c0), None
        p = data.synthetic_problem(c1 - c0, nlay_cfg, seed=20251015, col0=c0)
        return p, (data.allsky_clouds(p, data.load_cloud_optics("lw")) if args.config == "c4" else None)

    if args.config == "c1":
        workload = "C1: RFMIP clear-sky LW only, 100 columns x 60 layers x 256 g-points, NN gas optics (g256)"
        data_desc = "real RFMIP inputs (reference's RFMIP file) + the reference's trained NN weights; surrogate k-dist tables"
        metric = "atmospheric columns/sec (LW clear-sky fluxes), 1 MI355X"
    elif args.config == "c2":
        workload = "C2: RFMIP clear-sky LW only, 1800 columns x 60 layers x 256 g-points, NN gas optics (g256)"
        data_desc = "real RFMIP inputs (reference's RFMIP file) + the reference's trained NN weights; surrogate k-dist tables"
        metric = "atmospheric columns/sec (LW clear-sky fluxes), 1 MI355X"
    elif args.config == "c3":
        workload = "C3: RFMIP clear-sky LW+SW, 1800 columns x 60 layers, NN gas optics (g256 LW + g224 SW)"
        data_desc = "real RFMIP inputs (reference's RFMIP file) + the reference's trained NN weights; surrogate k-dist tables"
    elif args.config == "c4":
        workload = ("C4: all-sky LW+SW, 10000 synthetic columns x 60 layers, NN gas optics + cloud_optics (LUT, ice "
                    "roughness 2; LW 1scl increment, SW delta-scaled 2str increment)")
        data_desc = ("synthetic columns drawn from RFMIP profiles (PCG64 streams seeded by (20251015, column block)); "
                     "clouds by the all-sky example's recipe (rrtmgp_allsky.F90:329-350); the reference's cloud-optics "
                     "coefficients")
    else:
        workload = ("C5: 1e6 synthetic columns x 137 layers clear-sky LW+SW, column-sharded" if scaling == "strong"
                    else "C5 shard: 125000 synthetic columns x 137 layers per GPU, clear-sky LW+SW")
        data_desc = ("synthetic columns interpolated from RFMIP profiles (PCG64 streams seeded by (20251015, column "
                     "block))")
    if args.sw_kernel:
        from rrtmgpnn import api
        api.set_sw_kernel_default(args.sw_kernel)
    lw_after = None if not args.lw_after else ("" if args.lw_after == "none" else args.lw_after)
    sw_after = None if not args.sw_after else ("" if args.sw_after == "none" else args.sw_after)
    use_graph = not args.no_graph
    # the rank's columns in chunks of at most one block (pipeline.ChunkedRank): with more than one chunk every chunk's
    # inputs are resident in HBM and copied into the step's buffers before its replay, its fluxes copied into the
    # rank's slab after it (device to device, inside the timed region); tests/test_gpu_chunked.py checks the slab
    rank_run = ChunkedRank(lo, hi, block, problem,
                           lambda p, c: ClearSkyStep(p, device=local, fused=not args.unfused, clouds=c,
                                                     overlap=not args.no_overlap, sw=args.config not in ("c1", "c2"),
                                                     lw_after=lw_after, sw_after=sw_after,
                                                     sw_priority=args.sw_priority, lw_net_cus=args.lw_net_cus,
                                                     sw_net_cus=args.sw_net_cus),
                           use_graph=use_graph)
    step = rank_run.step
    prob, clouds = rank_run.first
    ncol, nlay = step.ncol, step.nlay
    # everything below runs on the step's own stream (its graph replays, the chunk copies, the host-resident copies),
    # not on the legacy null stream
    torch.cuda.set_stream(step.ctx.stream)
    run_one = step.replay if use_graph else step.step
    run = rank_run.run

    def warm_and_time():
        """W untimed warmup steps, then exactly K steps bracketed by barrier + synchronize; max over ranks (s)."""
        for _ in range(args.warmup):
            run()
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            run()
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el

    # unsettled: the first W + K steps of the process, exactly as the driver's command would time them without the
    # settle phase (reported beside `value` as ms_per_step_unsettled, for comparison with rounds 1-2)
    elapsed_unsettled = warm_and_time() if args.settle_s > 0 else None
    # settle: untimed steps until the GPU runs at its steady clocks (reported in the line), then the warmup steps
    settle_steps, ts0 = 0, time.perf_counter()
    while time.perf_counter() - ts0 < args.settle_s:
        for _ in range(8):
            run()
        settle_steps += 8
        torch.cuda.synchronize(dev)
    settle_s = time.perf_counter() - ts0
    elapsed = warm_and_time()
    ms_per_step = elapsed / args.steps * 1e3
    total_cols = global_cols * args.steps
    value = total_cols / elapsed

    # ---- block stream (never `value`): the step's block streamed K times with its two chains free-running
    # (ClearSkyStep.run_blocks: block b+1's SW chain beside block b's LW chain, no per-block join) -- the rate of a
    # stream of independent blocks, the reference driver's block loop (rrtmgp_rfmip_lw.F90:364-446), whose OpenMP
    # threads also run blocks side by side.  `value` keeps the joined step ----
    block_stream = None
    if step.overlap and step.sw and rank_run.single and use_graph:
        step.capture_chains()
        nb = max(args.steps, 50)
        for _ in range(3):
            step.run_blocks(max(1, args.warmup))
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        step.run_blocks(nb)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        el_b = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([el_b], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el_b = float(t.item())
        block_stream = {"value": round(global_cols * nb / el_b, 1), "unit": "columns/s", "blocks": nb,
                        "ms_per_block": round(el_b / nb * 1e3, 4),
                        "vs_joined_step": round((el_b / nb) / (elapsed / args.steps), 4),
                        "note": "the step's block streamed `blocks` times per rank, LW and SW chains as two hipGraphs "
                                "replayed free-running on their streams (block b+1's SW chain beside block b's LW "
                                "chain); same fluxes bit for bit (tests/test_gpu_chunked.py); not `value`"}

    # ---- host-resident variant: pinned H2D of every input, the step, D2H of the fluxes (never `value`; one chunk) ----
    ins, outs = step.io_tensors()
    run = run_one
    h_ins = [t.cpu().pin_memory() for t in ins]
    h_outs = [torch.empty(t.shape, dtype=t.dtype, pin_memory=True) for t in outs]
    io_bytes = sum(t.numel() * 4 for t in ins) + sum(t.numel() * 4 for t in outs)

    def run_io():
        for d, h in zip(ins, h_ins):
            d.copy_(h, non_blocking=True)
        run()
        for h, d in zip(h_outs, outs):
            h.copy_(d, non_blocking=True)

    run_io()
    torch.cuda.synchronize(dev)
    io_steps = max(3, min(20, args.steps))
    t0 = time.perf_counter()
    for _ in range(io_steps):
        run_io()
    torch.cuda.synchronize(dev)
    io_ms = (time.perf_counter() - t0) / io_steps * 1e3
    pcie = {"value": round(ncol / (io_ms * 1e-3), 1), "unit": "columns/s", "ms_per_step": round(io_ms, 4),
            "bytes_per_step": io_bytes, "note": "per GPU; pinned host buffers, H2D inputs + step + D2H fluxes"}

    # ---- per-stage kernel times: HIP events around every launch of `reps` whole steps issued eagerly, each launch on
    # the stream it runs on.  stages_ms (the rooflines): the launches serialised -- each kernel has the chip to
    # itself, in its place in the step (after the kernel that produced its inputs), as in the graph replays of
    # `bench.py --no-overlap`, whose rocprofv3 --kernel-trace averages they match.  stages_overlapped_ms: the step's
    # own concurrency (LW and SW chains overlapped, as the timed region runs); there the events also hold the time a
    # launch waits for CUs the other chain occupies ----
    reps = max(3, min(20, args.steps))

    def time_stages(serial):
        # serialised: every kernel on the whole chip, the LW network's CU cap (rrtmgpnn_context_set_mlp_max_cus, an
        # overlap measure) lifted for the measurement
        if serial and step.lw_net_cus:
            _lib.check(step.L.rrtmgpnn_context_set_mlp_max_cus(step.ctx.h, 0), "context_set_mlp_max_cus")
        if serial and getattr(step, "sw_net_cus", 0):
            _lib.check(step.L.rrtmgpnn_context_set_mlp_max_cus(step.ctx2.h, 0), "context_set_mlp_max_cus")
        step.step()  # warm the eager path
        torch.cuda.synchronize(dev)
        timing = {}
        prev = None  # serial: every launch waits for the one before it, across steps too
        for _ in range(reps):
            if serial:
                for name, fn, cargs in step.calls:
                    s = step.stream_for(name)
                    if prev is not None:
                        s.wait_event(prev)
                    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    ev0.record(s)
                    fn(*cargs)
                    ev1.record(s)
                    timing.setdefault(name, []).append((ev0, ev1))
                    prev = ev1
            else:
                step.step(timing)
        torch.cuda.synchronize(dev)
        if serial and step.lw_net_cus:
            _lib.check(step.L.rrtmgpnn_context_set_mlp_max_cus(step.ctx.h, step.lw_net_cus), "context_set_mlp_max_cus")
        if serial and getattr(step, "sw_net_cus", 0):
            _lib.check(step.L.rrtmgpnn_context_set_mlp_max_cus(step.ctx2.h, step.sw_net_cus), "context_set_mlp_max_cus")
        return {name: sum(a.elapsed_time(b) for a, b in pairs) / len(pairs) for name, pairs in timing.items()}

    stages = time_stages(True)
    stages_ov = time_stages(False) if step.overlap else None
    # dominant kernel and its roofline
    best = None
    for name, ms in stages.items():
        kind, amount, _, _ = stage_work(name, step)
        if amount <= 0:
            continue
        if best is None or ms > stages[best[0]]:
            best = (name, kind, amount)
    roof = None
    stage_roofs = {}
    try:  # share of the chip's VALU issue slots each stage used, from the committed SQ counter pass
        with open(args.sq_json) as f:
            sq = json.load(f).get(args.config, {})
    except (OSError, ValueError):
        sq = {}
    for name, ms in stages.items():
        kind, amount, k2, a2 = stage_work(name, step)
        if amount <= 0:
            continue
        if kind == "flop":
            ach = amount / (ms * 1e-3) / 1e12
            stage_roofs[name] = {"bound": "mfma", "achieved_tflops": round(ach, 2),
                                 "frac": round(ach / FP32_MFMA_PEAK_TFS, 4),
                                 "algorithmic_gbs": round(a2 / (ms * 1e-3) / 1e9, 1)}
        else:
            ach = amount / (ms * 1e-3) / 1e9
            stage_roofs[name] = {"bound": "hbm", "achieved_gbs": round(ach, 1), "frac": round(ach / HBM_PEAK_GBS, 4)}
        if sq.get(name, {}).get("valu_busy") is not None:
            stage_roofs[name]["valu_busy"] = sq[name]["valu_busy"]
        if kind == "flop" and sq.get(name, {}).get("mfma_busy") is not None:
            stage_roofs[name]["mfma_busy"] = sq[name]["mfma_busy"]  # rocprof matrix-core utilisation (pmc_counters.py)
            if sq[name].get("mfma_flop"):
                stage_roofs[name]["mfma_flop_counter"] = sq[name]["mfma_flop"]
    if best is not None:
        name, kind, amount = best
        ms = stages[name]
        traffic = None
        try:
            with open(args.traffic_json) as f:
                tj = json.load(f)
            tk = tj.get(args.config, {}).get(name)
            if isinstance(tk, dict):
                tk = tk.get("hbm_bytes")
            if tk is not None:
                traffic = tk
        except (OSError, ValueError):
            pass
        if kind == "flop":
            ach = amount / (ms * 1e-3) / 1e12
            roof = {"kernel": name, "bound": "mfma", "achieved": round(ach, 3), "peak": FP32_MFMA_PEAK_TFS,
                    "unit": "TFLOP/s", "frac": round(ach / FP32_MFMA_PEAK_TFS, 4), "traffic": traffic,
                    "algorithmic_per_launch": amount, "avg_launch_ms": round(ms, 4)}
        else:
            ach = amount / (ms * 1e-3) / 1e9
            roof = {"kernel": name, "bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic, "algorithmic_per_launch": amount,
                    "avg_launch_ms": round(ms, 4),
                    "timing": "HIP events around each launch, whole steps with the launches serialised (the kernel "
                              "alone on the chip; rocprofv3 trace of bench.py --no-overlap)"}
            if traffic:
                roof["actual_gbs"] = round(traffic / (ms * 1e-3) / 1e9, 1)  # PMC bytes / launch time
        if roof is not None and sq.get(name, {}).get("valu_busy") is not None:
            roof["valu_busy"] = sq[name]["valu_busy"]  # the solvers' binding limit: VALU issue

    # ---- final flux all-gather over RCCL (outside the timed region): shard.gather_columns, the partition's
    # tested exchange, of the rank's (ncol, 5, nlev) flux slab into the global (global_cols, 5, nlev) array ----
    gather_ms = None
    end_to_end = None
    gather_check = None
    if world > 1:
        local_slab = torch.stack(list(rank_run.flux), dim=1)
        torch.cuda.synchronize(dev)
        dist.barrier()
        g0 = time.perf_counter()
        full = shard.gather_columns(local_slab, global_cols, world)
        torch.cuda.synchronize(dev)
        gather_ms = (time.perf_counter() - g0) * 1e3
        t = torch.tensor([gather_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        gather_ms = float(t.item())
        assert full.shape[0] == global_cols
        # every rank checks the gathered array: its own slab in place bit for bit, every rank's slab in place by an
        # exact checksum of its bits, finite fluxes; the verdict is reduced over ranks
        chk = shard.verify_gather(full, local_slab, global_cols, rank, world)
        ok = torch.tensor([1 if chk["ok"] else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        gather_check = dict(chk, ok=bool(ok.item()), ranks_checked=world,
                            note="rank 0's view; ok is the minimum over ranks of (own slab bitwise, every slab's "
                                 "checksum in place, finite)")
        del full
        if not gather_check["ok"]:
            sys.stderr.write("bench.py: flux all-gather check failed on some rank: %s\n" % chk)
        end_to_end = {"value": round(total_cols / (elapsed + gather_ms * 1e-3), 1), "unit": "columns/s",
                      "note": "all ranks' columns over the timed steps plus one final flux all-gather"}

    config = {"workload": workload, "global_columns": global_cols, "ncol_per_gpu": hi - lo,
              "chunk_columns": ncol, "nlay": nlay, "ngpt_lw": step.ng_lw,
              "ngpt_sw": step.ng_sw if step.sw else None,
              "parallelism": "column-sharded (shard.column_range), 1 process per GPU",
              "launch": ("hipGraph replay" if use_graph else "eager") +
                        (", LW and SW chains on two streams" if step.overlap else "") +
                        (", the LW chain after %s" % step.lw_after if step.lw_after else "") +
                        (" (LW network on %d CUs)" % step.lw_net_cus if step.lw_net_cus else "") +
                        (", the SW solver after %s" % step.sw_after if step.sw_after else "") +
                        (", SW stream priority %d" % step.sw_priority if step.sw_priority else ""),
              "kernels": ("class-layer sequence" if not step.fused else
                          "fused Planck-in-LW-solver, g=0 elided" +
                          (", cloud increments fused into both solvers" if step.allsky else ""))}
    step_sw = step.sw
    # the main line's steps, workspaces and chunk inputs are released before c5_global allocates its own (at C5 each
    # holds ~116 GB of the device's 288: both at once can exceed HBM)
    torch.cuda.set_stream(torch.cuda.default_stream(dev))
    rank_run.close()
    del rank_run, step, ins, outs, h_ins, h_outs, run, run_one
    torch.cuda.empty_cache()

    # ---- BASELINE configs[4] as stated: 1e6 x 137 columns over the ranks (strong scaling), in every line ----
    c5g = None
    if args.config == "c5" and scaling == "strong" and global_cols == C5_GLOBAL_COLS:
        c5g = {"same_as_main": True, "note": "this line's own workload is configs[4]: see value / ms_per_step / "
                                             "gather_ms / gather_check"}
    elif args.c5_steps > 0:
        c5g = c5_global(args, world, rank, dev)

    # ---- CPU baseline: C restatement (oracle, bit-identical to the reference's RTE/MLP) on host cores ----
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(prob, clouds, args.cpu_seconds, args.cpu_kind, sw=step_sw, bind=args.cpu_bind)

    if rank == 0:
        out = {
            "metric": metric, "value": round(value, 1), "unit": "columns/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "settle_s": round(settle_s, 3) if args.settle_s > 0 else 0.0,
            "settle_steps": settle_steps, "ms_per_step": round(ms_per_step, 4),
            "ms_per_step_unsettled": (None if elapsed_unsettled is None else
                                      round(elapsed_unsettled / args.steps * 1e3, 4)),
            "value_unsettled": (None if elapsed_unsettled is None else
                                round(total_cols / elapsed_unsettled, 1)),
            "higher_is_better": True,
            "scaling": scaling, "vs_baseline": None, "dtype": "f32", "data": data_desc,
            "config": config,
            "column_layers_per_s": round(value * nlay, 1),
            "roofline": roof,
            "cpu_baseline": cpu,
            "stages_ms": {k: round(v, 4) for k, v in stages.items()},
            "stages_overlapped_ms": None if stages_ov is None else {k: round(v, 4) for k, v in stages_ov.items()},
            "stage_roofline": stage_roofs,
            "gather_ms": None if gather_ms is None else round(gather_ms, 3),
            "gather_check": gather_check,
            "end_to_end": end_to_end,
            "host_resident": pcie,
            "block_stream": block_stream,
            "c5_global": c5g,
        }
        if world > 1:
            out["ranks"] = {"launcher": ("bench.py --gpus %d (torch.distributed.run child)" % world
                                         if os.environ.get("RRTMGPNN_VISIBLE_DEVICES") else "outer launcher"),
                            "world_size": world, "visible_devices": ndev, "backend": backend,
                            "ranks_per_device": -(-world // ndev)}
        print(json.dumps(out), file=result, flush=True)
    if world > 1:
        dist.destroy_process_group()
        if not gather_check["ok"] or (c5g and c5g.get("gather_check") and not c5g["gather_check"]["ok"]):
            sys.exit(1)


C5_GLOBAL_COLS, C5_CHUNK, C5_NLAY = 1000000, 125000, 137


def c5_global(args, world, rank, dev):
    """BASELINE.json configs[4] exactly as stated -- 1e6 synthetic columns x 137 layers, clear-sky LW+SW, column-sharded
    over the ranks -- measured beside the line's own workload, so that the driver's `--gpus N` runs (N = 1, 2, 4, 8)
    record it: each rank takes its shard.column_range of the 1e6 columns and streams it through one step in chunks of
    at most 125 000 columns (pipeline.ChunkedRank: 8 chunks at N = 1, one at N = 8; every chunk's inputs resident in
    HBM, copied into the step's buffers inside the timed region).  The reference's own decomposition is the OpenMP
    loop over column blocks of examples/rfmip-clear-sky/rrtmgp_rfmip_lw.F90:364-446; the ranks replace the threads.
    `--c5-warmup` untimed steps, then `--c5-steps` steps bracketed by barrier + synchronize, max over ranks; then the
    final broadband flux all-gather (2.76 GB of (ncol, 5, 138) slabs) over RCCL, timed and checked as the main line's.
    Synthetic columns: data.synthetic_problem (PCG64 streams seeded by (20251015, column block)), generated on host
    threads, chunk by chunk."""
    import torch
    import torch.distributed as dist
    from concurrent.futures import ThreadPoolExecutor
    from rrtmgpnn import data, shard
    from rrtmgpnn.pipeline import ChunkedRank, ClearSkyStep
    G, CH, NL = C5_GLOBAL_COLS, C5_CHUNK, C5_NLAY
    lo, hi = shard.column_range(G, rank, world)
    torch.cuda.synchronize(dev)
    free0 = torch.cuda.mem_get_info(dev)[0]
    chunks = shard.chunk_ranges(lo, hi, CH)
    t0 = time.perf_counter()
    with ThreadPoolExecutor(max(1, min(8, len(chunks)))) as ex:
        futs = {c: ex.submit(data.synthetic_problem, c[1] - c[0], NL, seed=20251015, col0=c[0]) for c in chunks}
        rr = ChunkedRank(lo, hi, CH, lambda c0, c1: (futs.pop((c0, c1)).result(), None),
                         lambda p, c: ClearSkyStep(p, device=dev.index), use_graph=not args.no_graph)
    rr.first = None  # the first chunk's host arrays are not needed here
    setup_s = time.perf_counter() - t0
    torch.cuda.set_stream(rr.step.ctx.stream)
    for _ in range(args.c5_warmup):
        rr.run()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.c5_steps):
        rr.run()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    free1 = torch.cuda.mem_get_info(dev)[0]  # steps, workspaces and chunk inputs in place
    slab = torch.stack(list(rr.flux), dim=1)  # (ncol, 5, nlev): lw_up, lw_dn, sw_up, sw_dn, sw_dir
    finite = bool(torch.isfinite(slab).all().item())
    slab_bytes = slab.numel() * 4
    gather_ms, check = None, {"ok": finite, "finite": finite,
                              "note": "one rank: its slab is the global array, no exchange"}
    if world > 1:
        torch.cuda.synchronize(dev)
        dist.barrier()
        g0 = time.perf_counter()
        full = shard.gather_columns(slab, G, world)
        torch.cuda.synchronize(dev)
        gather_ms = (time.perf_counter() - g0) * 1e3
        t = torch.tensor([gather_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        gather_ms = float(t.item())
        chk = shard.verify_gather(full, slab, G, rank, world)
        ok = torch.tensor([1 if chk["ok"] else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        check = dict(chk, ok=bool(ok.item()), ranks_checked=world, gathered_bytes=full.numel() * 4,
                     note="rank 0's view; ok is the minimum over ranks")
        del full
        if not check["ok"]:
            sys.stderr.write("bench.py: c5_global flux all-gather check failed on some rank: %s\n" % chk)
    steps = args.c5_steps
    res = {"workload": "C5 (BASELINE configs[4]): 1e6 synthetic columns x 137 layers, clear-sky LW+SW, column-sharded "
                       "over the ranks (shard.column_range), each rank streaming its range in chunks of <= 125000",
           "global_columns": G, "nlay": NL, "n_gpus": world, "ncol_per_rank": hi - lo, "chunks_per_rank": len(chunks),
           "chunk_columns": CH, "steps": steps, "warmup": args.c5_warmup, "scaling": "strong",
           "ms_per_step": round(el / steps * 1e3, 3), "value": round(G * steps / el, 1), "unit": "columns/s",
           "column_layers_per_s": round(G * steps / el * NL, 1),
           "gather_ms": None if gather_ms is None else round(gather_ms, 3), "gather_check": check,
           "end_to_end": {"value": round(G * steps / (el + (gather_ms or 0.0) * 1e-3), 1), "unit": "columns/s",
                          "note": "the timed steps plus one final flux all-gather"},
           "setup_s": round(setup_s, 1),
           # this block's device memory on the rank: torch's allocator peak (steps, chunk inputs, flux slab, gathered
           # array) plus the library's own buffers (network images, workspaces: rrtmgpnn_context_workspace_bytes)
           "hbm_gb_per_rank": {"steps_and_inputs": round((free0 - free1) / 1e9, 2),
                               "flux_slab": round(slab_bytes / 1e9, 3),
                               "note": "device memory this block held on the rank after its steps ran (hipMemGetInfo "
                                       "before and after: the steps' arrays, the library's workspaces, every chunk's "
                                       "resident inputs); plus the flux slab and, at N > 1, the gathered array"},
           "data": "synthetic columns interpolated from RFMIP profiles (PCG64 streams seeded by (20251015, column "
                   "block)), generated per chunk on host threads (setup_s, outside the timed region)"}
    torch.cuda.set_stream(torch.cuda.default_stream(dev))
    rr.close()
    del rr, slab
    torch.cuda.empty_cache()
    return res


def _subset(prob, idx):
    sub = {k: (v[idx] if isinstance(v, np.ndarray) and v.ndim >= 1 and v.shape[0] == prob["ncol"] else v)
           for k, v in prob.items()}
    sub["gases"] = {k: (v[idx] if np.ndim(v) == 2 else v) for k, v in prob["gases"].items()}
    sub["ncol"] = len(idx)
    return sub


def _cpu_block(ncol):
    """Columns per block: the reference RFMIP example's 36 (examples/rfmip-clear-sky/Makefile:7) when it divides the
    sample, else the largest divisor <= 36 (the driver needs whole blocks, rrtmgp_rfmip_lw.F90:213)."""
    return max(d for d in range(1, min(36, ncol) + 1) if ncol % d == 0)


def cpu_baseline(prob, clouds, target_s, kind="auto", sw=True, reps=7, bind="none"):
    """CPU path on the host cores over a bounded sample of the same workload (rank 0, N=1 only).

    kind "reference" (default when oracle/_ref is built): oracle/_ref/rrtmgp_cpu_bench (oracle/cpu_bench.F90), the
    reference's own rte_lw / rte_sw / network_type%output_sgemm_flat (MKL sgemm, sequential) / ty_cloud_optics,
    compiled from its sources and driven as examples/rfmip-clear-sky/rrtmgp_rfmip_lw.F90:364-446 drives them: an
    OpenMP loop over blocks of 36 columns, per-thread objects allocated once.  The NN glue (compute_nn_inputs,
    get_col_dry, output scaling, compute_Planck_source_nn) is the C restatement's (its reference modules need
    netcdf-fortran).  Blocks cycle through up to 3 600 columns of the workload; `reps` timed runs, the median
    reported (tests/test_cpu_bench.py checks the program's fluxes against the oracle bit for bit).

    Threads: `value` is measured on the CPU share the GPU box gives one GPU's job -- OMP_NUM_THREADS, which the box
    sets to 16 (its rules size every worker pool to that share), capped by the process's affinity mask; the line
    records both (`cpu_allotment`, with the cgroup CPU quota).  Threads are unbound by default: OMP_PROC_BIND=close
    with OMP_PLACES=cores put all 16 threads on the 2 places the runtime found on the GPU box (4.97 k columns/s
    against 49 k unbound, profiles/r04/cpu_bind_close.json); the median of `reps` runs is the value.  `thread_sweep` adds measured 1- and
    8-thread points, and `extrapolated` scales the measured value linearly to nproc / 8 logical CPUs (one GPU's
    share of the node's CPUs) and to all nproc: the blocks are independent, so linear scaling is an upper bound on
    the CPU path there, not a measurement.
    kind "port": the C restatement alone, OpenMP over columns (when oracle/_ref is absent)."""
    import statistics
    import subprocess
    import tempfile
    from rrtmgpnn import data
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = os.cpu_count() or 1
    omp_env = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = min(omp_env or 16, affinity)
    allot = {"omp_num_threads_env": omp_env or None, "affinity_cpus": affinity, "nproc": os.cpu_count(),
             "bind": bind}
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            allot["cgroup_cpu_max"] = f.read().strip()
    except OSError:
        pass
    bind_env = {} if bind == "none" else {"OMP_PROC_BIND": bind, "OMP_PLACES": "cores"}
    exe = os.path.join(ROOT, "oracle", "_ref", "rrtmgp_cpu_bench")
    what = "%s gas optics%s + RTE" % ("LW+SW" if sw else "LW",
                                      " + cloud optics/increment/delta-scale" if clouds is not None else "")
    if kind in ("auto", "reference") and os.path.exists(exe):
        ncol = prob["ncol"]
        nsamp = ncol if ncol <= 3600 else 3600
        sub = prob if nsamp == ncol else _subset(prob, np.arange(nsamp))
        cl = None if clouds is None else tuple(np.asarray(c)[:nsamp] for c in clouds)
        block = _cpu_block(nsamp)
        with tempfile.TemporaryDirectory() as td:
            path = os.path.join(td, "problem.rbin")
            data.write_problem(sub, path, clouds=cl)

            def run(nthr, ncols, nreps):
                env = dict(os.environ, OMP_NUM_THREADS=str(nthr), OMP_STACKSIZE="256M",
                           MKL_THREADING_LAYER="SEQUENTIAL", **bind_env)
                if bind == "none":
                    env.pop("OMP_PROC_BIND", None)
                    env.pop("OMP_PLACES", None)
                r = subprocess.run([exe, path, data.DATA_DIR, str(nthr), str(block), str(ncols), str(int(sw)),
                                    str(nreps)], capture_output=True, text=True, env=env, timeout=600)
                if r.returncode != 0:
                    raise RuntimeError("rrtmgp_cpu_bench failed: " + (r.stdout + r.stderr)[-400:])
                return json.loads(r.stdout.strip().splitlines()[-1])

            def measure(nthr, seconds, nreps):
                n0 = max(nsamp, 8 * nthr * block)  # every thread busy for the calibration run too
                cal = run(nthr, n0, 1)  # after the program's own untimed warm-up pass
                per_rep = seconds / (nreps + 1)
                n = max(nsamp, int(round(n0 * per_rep / max(cal["seconds"][0], 1e-4) / block)) * block)
                return run(nthr, n, nreps)

            try:
                load0, wall0 = os.getloadavg(), time.time()
                res = measure(threads, target_s, reps)
                load1 = os.getloadavg()
                sweep = {}
                for t in sorted({1, min(8, threads)} - {threads}):
                    r = measure(t, max(2.0, target_s / 5), 3)
                    sweep[str(t)] = round(r["columns"] / statistics.median(r["seconds"]), 1)
            except (RuntimeError, ValueError, subprocess.TimeoutExpired) as e:
                return {"value": None, "unit": "columns/s", "cores": threads, "kind": "reference",
                        "sample": "failed: %s" % e}
        secs = res["seconds"]
        med = statistics.median(secs)
        value = res["columns"] / med
        sweep[str(threads)] = round(value, 1)
        nproc = int(res["nproc"])
        per_thread = value / threads
        # the CPUs the job may use: its cgroup quota (cpu.max "quota period") caps it below the affinity mask on the
        # GPU box (16 of 256), so the per-GPU share of nproc / 8 = 32 threads cannot be measured there
        quota = None
        try:
            q, per = allot.get("cgroup_cpu_max", "").split()
            quota = None if q == "max" else round(int(q) / int(per), 2)
        except ValueError:
            pass
        ss = sorted(secs)
        return {"value": round(value, 1), "unit": "columns/s", "cores": threads, "kind": "reference",
                "nproc": nproc, "runs_s": [round(t, 4) for t in secs],
                # each run's start (s after the first timed run's) and the host's load averages around the
                # measurement, so a slow run can be tied to other tenants' load on the box
                "runs_start_s": [round(t, 3) for t in res.get("starts", [])],
                "host_loadavg": {"before": [round(x, 2) for x in load0], "after": [round(x, 2) for x in load1],
                                 "wall_start_unix": round(wall0, 1)},
                "spread": round((max(secs) - min(secs)) / med, 4),
                # without the fastest and the slowest run (other tenants' load on the host shows up as single outliers)
                "spread_trimmed": round((ss[-2] - ss[1]) / med, 4) if len(ss) >= 5 else None,
                "quota_cpus": quota,
                "thread_sweep": sweep, "cpu_allotment": allot,
                "extrapolated": {
                    "node_share_per_gpu": {"threads": max(1, nproc // 8),
                                           "value": round(per_thread * max(1, nproc // 8), 1)},
                    "node": {"threads": nproc, "value": round(per_thread * nproc, 1)},
                    "note": "not measured: linear in threads from the %d-thread value (an upper bound, the blocks are "
                            "independent), to nproc/8 and nproc logical CPUs; the measured %d threads are the CPU "
                            "share the GPU box allots this job (OMP_NUM_THREADS%s)"
                            % (threads, threads, ", cgroup quota %s CPUs" % quota if quota else "")},
                "sample": ("%d columns per run (blocks of %d cycling through %d columns of the workload), %s, median "
                           "of %d runs: the reference's Fortran rte_lw/rte_sw + network_type sgemm MLP (MKL, "
                           "sequential)%s compiled from its sources, OpenMP over blocks on %d threads (%s) "
                           "(oracle/cpu_bench.F90, as rrtmgp_rfmip_lw.F90:364-446); NN glue from the C restatement"
                           % (res["columns"], block, nsamp, what, len(secs),
                              " + ty_cloud_optics" if clouds is not None else "", threads,
                              "unbound" if bind == "none" else "OMP_PROC_BIND=%s, OMP_PLACES=cores" % bind))}
    # the C restatement alone (bit-identical to the reference on the solvers and MLP), OpenMP over columns
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    try:
        import oracle as O
        orc = O.Oracle()
    except Exception as e:  # oracle library not built
        return {"value": None, "unit": "columns/s", "cores": 0, "kind": "port", "sample": "unavailable: %s" % e}
    orc.set_threads(threads)
    models_lw = [data.load_model("lw_abs"), data.load_model("lw_pfrac")]
    models_sw = [data.load_model("sw_abs"), data.load_model("sw_ray")]
    kd, kds = data.load_kdist("lw"), data.load_kdist("sw")
    co_lw, co_sw = (data.load_cloud_optics(w) for w in ("lw", "sw")) if clouds is not None else (None, None)
    n = min(prob["ncol"], 3600)
    sub = _subset(prob, np.arange(n))
    cl = None if clouds is None else tuple(np.asarray(c)[:n] for c in clouds)
    secs = []
    for _ in range(reps):
        t0 = time.perf_counter()
        if cl is not None:
            orc.all_sky_lw(sub, models_lw, kd, co_lw, cl)
            orc.all_sky_sw(sub, models_sw, kds, co_sw, cl)
        else:
            orc.clear_sky_lw(sub, models_lw, kd)
            if sw:
                orc.clear_sky_sw(sub, models_sw, kds)
        secs.append(time.perf_counter() - t0)
    med = float(np.median(secs))
    return {"value": round(n / med, 1), "unit": "columns/s", "cores": threads, "kind": "port",
            "runs_s": [round(t, 4) for t in secs],
            "sample": "%d columns of the workload (%s), median of %d runs: C restatement (oracle), OpenMP over columns"
                      % (n, what, reps)}


if __name__ == "__main__":
    main()
