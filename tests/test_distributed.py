"""The bench's multi-rank path on CPU: world_size 2 over gloo (127.0.0.1).

bench.py --gpus N runs one process per GPU; each rank extracts its own
contig shard (weak scaling) and torch.distributed is used only for the
barrier and the max/sum reductions.  These tests run that orchestration with
the gloo backend: rendezvous, the reductions bench.py reports from, and that
rank shards are distinct, deterministic workloads.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out):
    os.environ.update({'RANK': str(rank), 'LOCAL_RANK': str(rank), 'WORLD_SIZE': str(world),
                       'MASTER_ADDR': '127.0.0.1', 'MASTER_PORT': str(port)})
    import bench
    from magot_amd import synth
    dist, r, local, n = bench.dist_setup(world)
    assert (r, local, n) == (rank, rank, world)
    assert dist.get_backend() == 'gloo'
    bench.barrier(dist)
    # per-rank "elapsed" and "bases": bench reports max(elapsed), sum(bases)
    elapsed = 0.5 + rank
    bases = 1000.0 * (rank + 1)
    mx = bench.allreduce_max(dist, elapsed)
    sm = bench.allreduce_sum(dist, bases)
    w = synth.make('small', seed=bench.shard_seed('small', rank), genome_bases=200_000, n_tx=50)
    digest = int(np.bitwise_xor.reduce(w.genome[:4096].astype(np.uint64) * 2654435761))
    out.put((rank, mx, sm, digest, int(w.cds_bases)))
    bench.barrier(dist)
    dist.destroy_process_group()


def test_bench_two_ranks_gloo():
    world = 2
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    assert all(r[1] == pytest.approx(1.5) for r in res)      # max over ranks
    assert all(r[2] == pytest.approx(3000.0) for r in res)   # sum over ranks
    assert res[0][3] != res[1][3]                             # distinct shards
    assert res[0][4] > 0 and res[1][4] > 0


def test_shard_seed_deterministic():
    import bench
    from magot_amd import synth
    assert bench.shard_seed('C3', 0) == synth.SEED_BASE + 3
    assert bench.shard_seed('C3', 7) == synth.SEED_BASE + 3 + 7000
    a = synth.make('small', seed=bench.shard_seed('small', 1), genome_bases=100_000, n_tx=20)
    b = synth.make('small', seed=bench.shard_seed('small', 1), genome_bases=100_000, n_tx=20)
    assert np.array_equal(a.genome, b.genome) and np.array_equal(a.ex_start, b.ex_start)


# ---------------------------------------------------------------------------
# C4 (strong) orchestration: magot_amd/shard.py
# ---------------------------------------------------------------------------

def test_lpt_contigs_balance_and_cover():
    from magot_amd import shard
    rng = np.random.default_rng(5)
    w = rng.lognormal(0, 1, size=64)
    owner, load = shard.lpt_contigs(w, 8)
    assert owner.min() >= 0 and owner.max() < 8
    assert np.allclose(np.bincount(owner, weights=w, minlength=8), load)
    # LPT bound: makespan <= 4/3 OPT, OPT >= max(mean, largest)
    assert load.max() <= 4.0 / 3.0 * max(load.mean(), w.max()) + 1e-9


def test_record_shards_partition_records():
    from magot_amd import shard
    rng = np.random.default_rng(6)
    tx_contig = rng.integers(0, 20, size=5000)
    tx_bases = rng.integers(50, 3000, size=5000)
    owner, shards, load = shard.record_shards(tx_contig, tx_bases, 20, 4)
    allrec = np.sort(np.concatenate(shards))
    assert np.array_equal(allrec, np.arange(5000))
    for r, sh in enumerate(shards):
        assert np.all(owner[tx_contig[sh]] == r)           # whole contigs per rank
        assert np.all(np.diff(sh) > 0)                      # global order kept


def test_reassemble_round_trip():
    from magot_amd import shard
    rng = np.random.default_rng(7)
    lens = rng.integers(0, 50, size=300)
    off = np.zeros(301, dtype=np.int64)
    np.cumsum(lens, out=off[1:])
    data = rng.integers(0, 255, size=int(off[-1])).astype(np.uint8)
    shards = [np.arange(0, 300, 3), np.arange(1, 300, 3), np.arange(2, 300, 3)]
    parts, offs = [], []
    for sh in shards:
        lo = np.zeros(len(sh) + 1, dtype=np.int64)
        np.cumsum(lens[sh], out=lo[1:])
        parts.append(np.concatenate([data[off[i]:off[i + 1]] for i in sh]))
        offs.append(lo)
    out, goff = shard.reassemble(shards, parts, offs)
    assert np.array_equal(out, data) and np.array_equal(goff, off)


def _gather_worker(rank, world, port, q):
    os.environ.update({'RANK': str(rank), 'WORLD_SIZE': str(world),
                       'MASTER_ADDR': '127.0.0.1', 'MASTER_PORT': str(port)})
    import torch
    import torch.distributed as dist
    from magot_amd import shard
    dist.init_process_group('gloo', rank=rank, world_size=world)
    n = 10 + 7 * rank
    t = torch.arange(n + 5, dtype=torch.int64).to(torch.uint8) + rank
    got = shard.gather_bytes(dist, rank, world, t, n)
    if rank == 0:
        q.put([g.tolist() for g in got])
    dist.barrier()
    dist.destroy_process_group()


def test_gather_bytes_two_ranks_gloo():
    world = 2
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        n = 10 + 7 * r
        assert got[r] == [(i + r) & 0xFF for i in range(n)]
