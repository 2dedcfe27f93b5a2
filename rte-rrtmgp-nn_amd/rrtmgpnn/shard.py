"""Column sharding across GPUs (one process per GPU, torch.distributed: RCCL on GPUs, gloo on CPU).

Columns are independent in every hot-path routine (no reference routine couples columns), so a
contiguous column range per rank is the whole decomposition.  The only exchange is the final
all-gather of broadband flux slabs (north star), done once per job, not per step.
launch_plan / spawn_ranks let `bench.py --gpus N` start its own N ranks; verify_gather checks the
gathered array against every rank's own slab.
"""
import os
import socket
import subprocess
import sys

import torch
import torch.distributed as dist


def column_range(ncol, rank, world):
    """Contiguous [lo, hi) column range of `rank`; the first ncol % world ranks get one extra column."""
    base, extra = divmod(ncol, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def launch_plan(gpus, env):
    """How a `bench.py --gpus N` process runs, from N and its environment:
    "single": N == 1 and no outer launcher (the one-rank path, unchanged);
    "rank": under an outer launcher (WORLD_SIZE set) whose world size equals N -- this process is one rank;
    "spawn": N > 1 and no launcher -- start N rank processes (spawn_ranks) before touching the GPU.
    Raises ValueError when an outer launcher's WORLD_SIZE disagrees with N (the line would report the wrong N)."""
    if gpus < 1:
        raise ValueError("--gpus must be >= 1 (got %d)" % gpus)
    ws = env.get("WORLD_SIZE")
    if ws is not None and ws != "":
        if int(ws) != gpus:
            raise ValueError("--gpus %d disagrees with the launcher's WORLD_SIZE=%s" % (gpus, ws))
        return "rank"
    return "single" if gpus == 1 else "spawn"


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_command(n, script, argv, port):
    """The torch.distributed.run command that starts n ranks of `script` on this node (rendezvous on 127.0.0.1)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % n,
            "--master-addr=127.0.0.1", "--master-port=%d" % port, script] + list(argv)


def spawn_ranks(n, script, argv, visible_devices):
    """Start n rank processes of `script` with `argv` and wait for them; returns the launcher's exit code.
    Call before any GPU work in this process (it starts children and never execs).  With fewer visible devices
    than ranks (rehearsing the N-rank path on a smaller box) the ranks share devices round-robin, and the flux
    gather uses gloo (RCCL refuses two ranks on one GPU) unless RRTMGPNN_DIST_BACKEND says otherwise."""
    env = dict(os.environ)
    if visible_devices < n:
        env.setdefault("RRTMGPNN_DIST_BACKEND", "gloo")
    env["RRTMGPNN_VISIBLE_DEVICES"] = str(visible_devices)
    # the ranks' stdout is filtered: JSON lines (rank 0's result line) pass to stdout, everything else (gloo and
    # launcher chatter) goes to stderr, so the caller still reads one JSON line
    p = subprocess.Popen(launch_command(n, script, argv, free_port()), env=env, stdout=subprocess.PIPE, text=True)
    for line in p.stdout:
        (sys.stdout if line.lstrip().startswith("{") else sys.stderr).write(line)
        sys.stdout.flush()
    return p.wait()


def slab_checksum(x):
    """Exact, order-sensitive checksum of a tensor's bits (int64): sum over elements of bits(x_i) * (i mod 65521 + 1).
    Two slabs agree bit for bit when, and (with overwhelming probability) only when, their checksums agree."""
    b = x.contiguous().view(-1).view(torch.int32).to(torch.int64)
    w = torch.arange(b.numel(), dtype=torch.int64, device=b.device) % 65521 + 1
    return int((b * w).sum().item())


def verify_gather(full, local, ncol, rank, world):
    """Check a gathered (ncol, ...) array on this rank against every rank's own slab: each rank all-gathers the
    checksum of the slab it computed, then checks that the columns [lo_r, hi_r) of ITS gathered copy carry rank r's
    checksum for every r, and that its own slab sits in place bit for bit and holds finite values.  Returns
    {"ok", "own_slab_bitwise", "all_slabs_checksum", "finite"} for this rank (callers reduce "ok" over ranks)."""
    lo, hi = column_range(ncol, rank, world)
    own = bool(torch.equal(full[lo:hi], local))
    mine = torch.tensor([slab_checksum(local)], dtype=torch.int64, device=local.device)
    sums = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(sums, mine)
    placed = True
    for r in range(world):
        a, b = column_range(ncol, r, world)
        placed &= slab_checksum(full[a:b]) == int(sums[r].item())
    finite = bool(torch.isfinite(local).all().item())
    return {"ok": own and placed and finite, "own_slab_bitwise": own, "all_slabs_checksum": placed,
            "finite": finite}


def gather_columns(local, ncol, world):
    """All-gather per-rank (ncol_local, ...) slabs into the full (ncol, ...) array on every rank, with one
    all_gather_into_tensor into one preallocated output.  When world divides ncol (every driver case: 1e6 and
    N x 1800 columns over 1, 2, 4, 8 ranks) the shards are equal, the rank's slab is sent as it is and the output IS
    the global array: one (ncol, ...) allocation per rank.  Otherwise shards differ by one column: they are padded to
    equal size for the collective and the padded output is compacted (one more copy)."""
    per = -(-ncol // world)
    inp = local.contiguous()
    if inp.shape[0] != per:
        inp = torch.zeros((per,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
        inp[:local.shape[0]] = local
    out = torch.empty((world * per,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(out, inp)
    if world * per == ncol:
        return out
    parts = []
    for r in range(world):
        lo, hi = column_range(ncol, r, world)
        parts.append(out[r * per:r * per + hi - lo])
    return torch.cat(parts, dim=0)


def chunk_ranges(lo, hi, chunk):
    """The chunks pipeline.ChunkedRank streams the column range [lo, hi) through: [(c0, c1)], at most `chunk`
    columns each, the last one possibly short (it then runs through a second step of its own shape)."""
    return [(c, min(c + chunk, hi)) for c in range(lo, hi, chunk)] or [(lo, lo)]


def chunk_plan(ncol, world, chunk):
    """Every rank's chunk sizes for a global problem of ncol columns: [(rank, [c1 - c0 for each chunk])]."""
    plan = []
    for r in range(world):
        lo, hi = column_range(ncol, r, world)
        plan.append((r, [c1 - c0 for c0, c1 in chunk_ranges(lo, hi, chunk)]))
    return plan
