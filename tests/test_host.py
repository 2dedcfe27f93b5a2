"""CPU tests of the host side: data files, problem builders, the C-ABI library's exports, and the
column sharding used by the multi-GPU driver (gloo, world_size 2)."""
import os
import re
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_rbin_roundtrip(tmp_path):
    from rrtmgpnn import rbin
    a = {"x": np.arange(12, dtype=np.float32).reshape(3, 4), "i": np.array([1, 2], np.int32),
         "c": rbin.chars(["h2o", "o3"])}
    p = str(tmp_path / "t.rbin")
    rbin.write(p, a)
    b = rbin.read(p)
    for k in a:
        np.testing.assert_array_equal(a[k], b[k])
    assert rbin.unchars(b["c"]) == ["h2o", "o3"]


def test_models_have_reference_shapes():
    from rrtmgpnn import data
    shapes = {"lw_abs": [18, 58, 58, 256], "lw_pfrac": [18, 16, 16, 256], "sw_abs": [7, 16, 16, 224],
              "sw_ray": [7, 16, 16, 224], "lw_g128_both": [18, 64, 64, 256]}
    for k, dims in shapes.items():
        m = data.load_model(k)
        assert list(m["dims"]) == dims
        assert list(m["activation"]) == [1, 1, 0]  # softsign, softsign, linear
        for n in range(3):
            assert m["w%d" % (n + 1)].shape == (dims[n], dims[n + 1])
    assert "output_mean" not in data.load_model("lw_pfrac")


def test_surrogate_planck_table_integrates_to_sigma_t4():
    from rrtmgpnn import data
    kd = data.load_kdist("lw")
    T = 300.0
    i = int(round((T - 160.0) / float(kd["totplnk_delta"])))
    total = np.pi * kd["totplnk"][:, i].sum()
    assert abs(total / (5.670374419e-8 * T ** 4) - 1.0) < 2e-3  # bands cover 10-3250 cm-1
    assert kd["nPlanckTemp"] == 196 and kd["ngpt"] == 256 and kd["nband"] == 16
    kds = data.load_kdist("sw")
    assert kds["ngpt"] == 224 and kds["nband"] == 14


def test_rfmip_problem_matches_driver_preprocessing(rfmip):
    from rrtmgpnn import data
    p = rfmip
    assert p["ncol"] == 1800 and p["nlay"] == 60 and p["top_at_1"]
    pmin = np.float32(data.load_kdist("lw")["press_ref_min"][0])
    assert np.all(p["plev"][:, 0] == pmin + data.F32_EPS)            # rrtmgp_rfmip_lw.F90:300-305
    assert np.all(p["play"] >= pmin)                                  # :287
    assert np.all((p["mu0"] > 0) & (p["mu0"] <= 1))
    assert p["usecol"].sum() == 918
    toa = data.toa_flux(p, data.load_kdist("sw"))
    np.testing.assert_allclose(toa.sum(1), p["tsi"], rtol=1e-5)         # rrtmgp_rfmip_sw.F90:408-427


def test_synthetic_problem_ranges():
    from rrtmgpnn import data
    s = data.synthetic_problem(300, 137, seed=3)
    assert s["play"].shape == (300, 137) and s["plev"].shape == (300, 138)
    assert np.all(np.diff(s["plev"], axis=1) > 0)
    assert s["tlay"].min() >= 160 and s["tlay"].max() <= 320.5
    s2 = data.synthetic_problem(300, 137, seed=3)
    np.testing.assert_array_equal(s["tlay"], s2["tlay"])  # seeded


def _header_symbols():
    with open(os.path.join(ROOT, "include", "rrtmgpnn.h")) as f:
        txt = f.read()
    return sorted(set(re.findall(r"\b(rrtmgpnn_[a-z0-9_]+)\s*\(", txt)))


def test_c_abi_exports_every_header_symbol():
    import ctypes
    from rrtmgpnn import _lib
    h = ctypes.CDLL(_lib.LIB_PATH)
    syms = _header_symbols()
    assert len(syms) >= 25
    missing = [s for s in syms if not hasattr(h, s)]
    assert not missing, missing
    assert set(syms) == set(_lib.SIGNATURES), "ctypes table out of sync with include/rrtmgpnn.h"


def test_c_abi_errors_are_reported_not_crashed():
    from rrtmgpnn import _lib
    L = _lib.lib()
    assert L.rrtmgpnn_version() == 1
    h = _lib.c_vp()
    rc = L.rrtmgpnn_context_create(-1, None, h)
    assert rc != 0 and L.rrtmgpnn_last_error()
    assert L.rrtmgpnn_lw_solver_noscat(None, 256, 60, 1, 1, 1, None, None, None, None, None, None, None, None, None,
                                       None) != 0
    assert b"null context" in L.rrtmgpnn_last_error()
    assert L.rrtmgpnn_context_set_sw_kernel(None, 4) != 0 and b"sw kernel mode" in L.rrtmgpnn_last_error()
    assert L.rrtmgpnn_context_set_sw_kernel(None, 0) == 0
    assert L.rrtmgpnn_context_set_mlp_max_cus(None, 192) != 0 and b"null context" in L.rrtmgpnn_last_error()


def _shard_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    from rrtmgpnn import shard
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    ncol = 1001
    lo, hi = shard.column_range(ncol, rank, world)
    # flux-like slabs (ncol_local, 5 quantities, nlev): per-rank values from a seeded generator
    g = torch.Generator().manual_seed(100 + rank)
    local = torch.rand((hi - lo, 5, 61), generator=g) * 400.0
    local[:, 0, 0] = torch.arange(lo, hi, dtype=torch.float32)
    full = shard.gather_columns(local, ncol, world)
    chk = shard.verify_gather(full, local, ncol, rank, world)
    # a gathered array with two of the other rank's columns swapped must fail the checksum on this rank
    bad = full.clone()
    o_lo, o_hi = shard.column_range(ncol, 1 - rank, world)
    bad[[o_lo, o_lo + 1]] = bad[[o_lo + 1, o_lo]]
    chk_bad = shard.verify_gather(bad, local, ncol, rank, world)
    # real fluxes: each rank computes its half of 12 RFMIP columns (the oracle's clear-sky LW+SW, as a rank's step
    # would) and the gathered (12, 5, 61) array must equal the whole problem's fluxes computed in one piece.  12 / 2
    # shards are equal, so gather_columns sends the slab as it is into the one preallocated output
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from rrtmgpnn import data
    orc = O.Oracle()
    ms_lw = [data.load_model("lw_abs"), data.load_model("lw_pfrac")]
    ms_sw = [data.load_model("sw_abs"), data.load_model("sw_ray")]
    kd, kds = data.load_kdist("lw"), data.load_kdist("sw")

    def fluxes(p):
        lu, ld, _ = orc.clear_sky_lw(p, ms_lw, kd)
        su, sd, sr, _ = orc.clear_sky_sw(p, ms_sw, kds)
        return torch.from_numpy(np.stack([lu, ld, su, sd, sr], axis=1).astype(np.float32))

    n2 = 12
    a, b = shard.column_range(n2, rank, world)
    whole = data.rfmip_columns(0, n2)
    mine = fluxes(data.rfmip_columns(a, b - a))
    got = shard.gather_columns(mine, n2, world)
    real_ok = bool(torch.equal(got, fluxes(whole))) and shard.verify_gather(got, mine, n2, rank, world)["ok"]
    q.put((rank, lo, hi, bool(torch.equal(full[:, 0, 0], torch.arange(ncol, dtype=torch.float32))), chk["ok"],
           chk_bad["ok"], chk_bad["own_slab_bitwise"], real_ok, tuple(got.shape)))
    dist.destroy_process_group()


def test_column_sharding_gloo_world2():
    import socket

    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_shard_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert res[0][1] == 0 and res[0][2] == res[1][1] and res[1][2] == 1001
    assert res[0][3] and res[1][3]
    assert res[0][4] and res[1][4]              # the gather check passes on the true gather
    assert not res[0][5] and not res[1][5]      # ... and catches another rank's misplaced columns
    assert res[0][6] and res[1][6]              # (the rank's own slab was untouched)
    assert res[0][7] and res[1][7]              # real fluxes gathered equal the whole problem's, bit for bit
    assert res[0][8] == res[1][8] == (12, 5, 61)


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_c5_global_chunk_plan(world):
    """bench.py's c5_global (BASELINE configs[4], 1e6 columns x 137 layers) at the driver's N = 1, 2, 4, 8: every rank
    streams equal 125 000-column chunks, so each rank captures ONE step shape (no second, short-chunk step), and the
    ranks' flux slabs are equal, so the final gather sends each slab as it is into one preallocated output."""
    sys.path.insert(0, ROOT)
    import bench
    from rrtmgpnn import shard
    plan = shard.chunk_plan(bench.C5_GLOBAL_COLS, world, bench.C5_CHUNK)
    assert len(plan) == world
    assert all(sizes == [125000] * (8 // world) for _, sizes in plan)
    assert {n for _, sizes in plan for n in sizes} == {125000}
    assert bench.C5_GLOBAL_COLS % world == 0
    # the chunker itself: ragged ranges end in one short chunk, empty ranges are one empty chunk
    assert shard.chunk_ranges(0, 300001, 125000) == [(0, 125000), (125000, 250000), (250000, 300001)]
    assert shard.chunk_ranges(5, 5, 10) == [(5, 5)]
    assert [len(s) for _, s in shard.chunk_plan(bench.C5_GLOBAL_COLS, 3, bench.C5_CHUNK)] == [3, 3, 3]


def test_bench_launch_plan():
    """bench.py --gpus N: one rank in-process at N = 1, self-launch at N > 1, the outer launcher's world must be N."""
    from rrtmgpnn import shard
    assert shard.launch_plan(1, {}) == "single"
    assert shard.launch_plan(8, {}) == "spawn"
    assert shard.launch_plan(4, {"WORLD_SIZE": "4"}) == "rank"
    assert shard.launch_plan(1, {"WORLD_SIZE": "1"}) == "rank"
    with pytest.raises(ValueError):
        shard.launch_plan(8, {"WORLD_SIZE": "2"})
    with pytest.raises(ValueError):
        shard.launch_plan(0, {})
    cmd = shard.launch_command(8, "/x/bench.py", ["--gpus", "8", "--steps", "20"], 29500)
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--master-addr=127.0.0.1" in cmd and "--nnodes=1" in cmd
    assert cmd[-5:] == ["/x/bench.py", "--gpus", "8", "--steps", "20"]


def test_bench_rejects_gpus_world_mismatch():
    import subprocess
    import sys
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2 and "disagrees" in r.stderr


def test_spawn_ranks_starts_n_processes(tmp_path, capsys):
    """spawn_ranks runs the script as N torch.distributed.run ranks (no GPU: the script only reports its env); of the
    ranks' stdout only JSON lines reach stdout (rank 0's result line), the rest goes to stderr."""
    from rrtmgpnn import shard
    out = tmp_path / "ranks"
    out.mkdir()
    script = tmp_path / "rank.py"
    script.write_text("import os, sys\n"
                      "open(os.path.join(sys.argv[1], os.environ['RANK']), 'w').write("
                      "'%s %s %s %s' % (os.environ['WORLD_SIZE'], os.environ['LOCAL_RANK'], "
                      "os.environ.get('RRTMGPNN_DIST_BACKEND'), sys.argv[2]))\n"
                      "print('[chatter] rank', os.environ['RANK'], flush=True)\n"
                      "if os.environ['RANK'] == '0': print('{\"rank\": 0}', flush=True)\n")
    env_backup = os.environ.pop("RRTMGPNN_DIST_BACKEND", None)
    try:
        rc = shard.spawn_ranks(2, str(script), [str(out), "--gpus"], visible_devices=1)
    finally:
        if env_backup is not None:
            os.environ["RRTMGPNN_DIST_BACKEND"] = env_backup
    assert rc == 0
    got = sorted((p.name, p.read_text()) for p in out.iterdir())
    assert got == [("0", "2 0 gloo --gpus"), ("1", "2 1 gloo --gpus")]
    cap = capsys.readouterr()
    assert cap.out.strip() == '{"rank": 0}'
    assert "[chatter] rank 0" in cap.err and "[chatter] rank 1" in cap.err


def test_bench_result_stream_keeps_stdout_to_the_line():
    """Under an outer launcher a rank's libraries may write to stdout (gloo's '[Gloo] Rank 0 is connected ...');
    bench.result_stream() points fd 1 at stderr, so the caller reads only the result line."""
    import subprocess
    import sys
    code = ("import os, sys; sys.path.insert(0, %r); import bench\n"
            "r = bench.result_stream()\n"
            "print('[Gloo] chatter', flush=True); os.write(1, b'raw fd write\\n')\n"
            "r.write('{\"ok\": 1}\\n'); r.flush()\n") % ROOT
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    assert p.stdout == '{"ok": 1}\n'
    assert "[Gloo] chatter" in p.stderr and "raw fd write" in p.stderr


def test_synthetic_problem_column_ranges_are_slices_of_the_whole():
    """bench.py builds each rank's shard (and each chunk of it) as a column range of one global synthetic problem:
    a range generated alone must equal the same columns of the whole, at 60 and 137 layers."""
    from rrtmgpnn import data
    for nlay in (60, 137):
        whole = data.synthetic_problem(2500, nlay, seed=7)
        part = data.synthetic_problem(900, nlay, seed=7, col0=1100)
        for k in ("play", "plev", "tlay", "tlev", "tsfc", "mu0", "sfc_alb", "tsi"):
            np.testing.assert_array_equal(part[k], whole[k][1100:2000], err_msg=k)
        for g in whole["gases"]:
            np.testing.assert_array_equal(part["gases"][g], whole["gases"][g][1100:2000], err_msg=g)
    co = data.load_cloud_optics("lw")
    whole = data.synthetic_problem(300, 60, seed=7)
    part = data.synthetic_problem(100, 60, seed=7, col0=101)
    for a, b in zip(data.allsky_clouds(part, co), data.allsky_clouds(whole, co)):
        np.testing.assert_array_equal(a, b[101:201])
    r = data.rfmip_columns(3500, 200)
    full = data.rfmip_problem()
    np.testing.assert_array_equal(r["tlay"], full["tlay"][(3500 + np.arange(200)) % 1800])


@pytest.mark.parametrize("allsky", [False, True])
@pytest.mark.parametrize("lw_after", ["", "predict_nn_sw", "sw_solver", "cloud_optics_sw"])
def test_issue_order_keeps_each_chain_in_order(allsky, lw_after):
    """The step's issue order (pipeline.issue_order) keeps every chain in FUSED_ORDER's relative order -- each chain
    runs on one stream in issue order, so a call issued ahead of its producer would read the previous step's data --
    and with an LW gate the SW-chain calls up to the gate come first."""
    from rrtmgpnn.pipeline import FUSED_ORDER, SW_CHAIN, issue_order
    names = ["sw_boundary", "predict_nn_lw", "lw_solver", "predict_nn_sw", "sw_solver"]
    if allsky:
        names = names[:1] + ["cloud_optics_lw"] + names[1:3] + ["cloud_optics_sw", "delta_scale_sw"] + names[3:]
    elif lw_after == "cloud_optics_sw":
        with pytest.raises(ValueError):
            issue_order([(n, None, ()) for n in names], True, lw_after)
        return
    calls = [(n, None, ()) for n in reversed(names)]  # any construction order
    out = [n for n, _, _ in issue_order(calls, True, lw_after)]
    assert sorted(out) == sorted(names)
    for chain in (SW_CHAIN, set(names) - SW_CHAIN):
        got = [n for n in out if n in chain]
        assert got == sorted(got, key=FUSED_ORDER.index)
    assert out[0] == "sw_boundary"  # the head of the SW chain
    if lw_after:
        cut = out.index(lw_after)
        assert all(n in SW_CHAIN for n in out[:cut + 1])
        assert [n for n in out[:cut + 1]] == [n for n in sorted(names, key=FUSED_ORDER.index)
                                              if n in SW_CHAIN][:cut + 1]


def test_ref_cosf_is_glibc_cosf():
    """mu0 = cos(sza * deg_to_rad) as the reference driver forms it with glibc's cosf (rrtmgp_rfmip_sw.F90:431-434):
    data.ref_cosf (the host restatement the problem builders use; the device's is libm_ref.hpp ref_cosf) equals the
    host libm's cosf on a sample of every exponent of [-4, 4] and on every RFMIP zenith angle.  numpy's float32 cos,
    which built mu0 before round 6, rounds differently on some of them (tools/check_libm_ref_cosf.c: every float)."""
    import ctypes
    from rrtmgpnn import data
    libm = ctypes.CDLL("libm.so.6")
    libm.cosf.restype, libm.cosf.argtypes = ctypes.c_float, [ctypes.c_float]
    u = np.arange(0, np.float32(4.0).view(np.uint32), 4099, dtype=np.uint32)
    d2r = np.float32(np.arccos(np.float32(-1.0)) / np.float32(180.0))
    sza = np.asarray(data.rfmip_problem()["sza"], np.float32)
    x = np.concatenate([u.view(np.float32), -u.view(np.float32), (sza * d2r).astype(np.float32)])
    want = np.array([libm.cosf(float(v)) for v in x], np.float32)
    np.testing.assert_array_equal(data.ref_cosf(x).view(np.uint32), want.view(np.uint32))
    assert (np.cos(x, dtype=np.float32) != want).any()  # numpy's own cos is not the reference's
