"""The bench's multi-rank path on CPU: world_size 2 over gloo (127.0.0.1).

bench.py --gpus N runs one process per GPU (started by bench itself, or by
torchrun); by default the N ranks share ONE job (C4: genome broadcast,
records sharded in genome order, outputs returned per rank or gathered to
rank 0).  These tests run that orchestration with the gloo backend:
rank launching and failure propagation, rendezvous, the reductions bench.py
reports from, the record sharding on C3's own tables, the byte gather and
the reassembly into global record order.
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
    dist, r, local, n = bench.dist_setup()
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


def test_tables_without_genome_match_full_workload():
    """Ranks > 0 of a shared job make only the record tables
    (synth.make(genome=False)): the same contigs, records and intervals as
    rank 0's full workload, for every configuration shape."""
    from magot_amd import synth
    for cfg, kw in (('small', {}), ('C2', {'genome_bases': 400_000, 'n_tx': 300}),
                    ('C3', {'genome_bases': 2_000_000, 'n_tx': 400})):
        full = synth.make(cfg, **kw)
        tab = synth.make(cfg, genome=False, **kw)
        assert tab.genome is None and full.genome is not None
        for k in ('contig_len', 'tx_contig', 'tx_strand', 'ex_count', 'ex_start', 'ex_len'):
            assert np.array_equal(getattr(full, k), getattr(tab, k)), (cfg, k)
        a, b = full.plan_tables(), tab.plan_tables()
        assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def _values_worker(rank, world, port, q):
    os.environ.update({'RANK': str(rank), 'LOCAL_RANK': str(rank), 'WORLD_SIZE': str(world),
                       'MASTER_ADDR': '127.0.0.1', 'MASTER_PORT': str(port)})
    import bench
    dist, r, local, n = bench.dist_setup()
    vals = bench.all_values(dist, 10.0 * (rank + 1))
    q.put((rank, vals))
    dist.barrier()
    dist.destroy_process_group()


def test_all_values_two_ranks_gloo():
    """The per-rank host figures of the line (RSS, set-up) gathered from every rank."""
    world = 2
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_values_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][1] == res[1][1] == [10.0, 20.0]


def test_dist_setup_one_rank_forced_gloo(tmp_path):
    """--dist: a process group of one rank (gloo here; nccl = RCCL on a GPU box)."""
    import subprocess
    code = ('import os, sys; sys.path.insert(0, %r); import bench; '
            'os.environ.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", '
            'MASTER_ADDR="127.0.0.1", MASTER_PORT=str(bench._free_port())); '
            'd, r, l, n = bench.dist_setup(force=True); '
            'assert d is not None and n == 1 and d.get_world_size() == 1; '
            'assert bench.all_values(d, 3.5) == [3.5]; '
            'assert bench.allreduce_max(d, 2.0) == 2.0; '
            'print(d.get_backend()); d.destroy_process_group()' % ROOT)
    env = dict(os.environ)
    env.pop('WORLD_SIZE', None)
    r = subprocess.run([sys.executable, '-c', code], env=env, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip().splitlines()[-1] == 'gloo'


def test_dist_setup_under_torchrun_two_ranks(tmp_path):
    """The driver's launch exactly: ``python -m torch.distributed.run --nnodes=1
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port P``.  Each rank's
    bench.dist_setup joins the elastic agent's store through the explicit
    tcp:// URL (TORCHELASTIC_USE_AGENT_STORE), then a reduction, the
    per-rank value gather and a barrier run over gloo."""
    import subprocess
    probe = tmp_path / 'probe.py'
    probe.write_text(
        'import os, sys\nsys.path.insert(0, %r)\nimport bench\n'
        'd, r, l, n = bench.dist_setup()\n'
        'assert n == 2 and d.get_world_size() == 2 and d.get_rank() == r\n'
        'assert os.environ.get("TORCHELASTIC_USE_AGENT_STORE") == "True"\n'
        'assert bench.allreduce_sum(d, r + 1.0) == 3.0\n'
        'assert bench.all_values(d, 10.0 * (r + 1)) == [10.0, 20.0]\n'
        'bench.barrier(d)\n'
        'print("rank%%d %%s ok" %% (r, d.get_backend()), flush=True)\n'
        'd.destroy_process_group()\n' % ROOT)
    env = dict(os.environ)
    for k in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_ADDR', 'MASTER_PORT'):
        env.pop(k, None)
    r = subprocess.run([sys.executable, '-m', 'torch.distributed.run', '--nnodes=1',
                        '--nproc-per-node', '2', '--master-addr', '127.0.0.1',
                        '--master-port', str(_free_port()), str(probe)],
                       env=env, capture_output=True, text=True, timeout=180, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    assert 'rank0 gloo ok' in r.stdout and 'rank1 gloo ok' in r.stdout, r.stdout


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
    tx_start = rng.integers(0, 10**6, size=5000)
    shards, load, spans = shard.record_shards(tx_contig, tx_bases, 20, 4, tx_start=tx_start)
    allrec = np.sort(np.concatenate(shards))
    assert np.array_equal(allrec, np.arange(5000))
    for r, sh in enumerate(shards):
        assert np.all(np.diff(sh) > 0)                      # global order kept
        assert load[r] == tx_bases[sh].sum()
        # one genome range per rank: (contig, start) of its records is contiguous
        key = tx_contig * 10**7 + tx_start
        lo, hi = key[sh].min(), key[sh].max()
        others = np.setdiff1d(np.arange(5000), sh)
        assert not np.any((key[others] > lo) & (key[others] < hi))
    assert shard.imbalance(load) < 0.01
    for c in range(20):
        ranks = [r for r in range(4) if np.any(tx_contig[shards[r]] == c)]
        assert (spans[c, 0], spans[c, 1]) == (min(ranks), max(ranks))


def test_record_shards_c3_balance():
    """C3's own tables (seed 20261018): its largest contig holds 23 % of the
    CDS bases, so contig-granular LPT was 86 % imbalanced at 8 ranks; the
    genome-order ranges split it and stay far below 5 % at 2, 4 and 8."""
    from magot_amd import shard, synth
    w = synth.make('C3')
    assert synth.SEED_BASE + 3 == 20261018
    first = np.zeros(w.n_tx + 1, dtype=np.int64)
    np.cumsum(w.ex_count, out=first[1:])
    tx_bases = np.add.reduceat(w.ex_len, first[:-1])
    per_contig = np.bincount(w.tx_contig, weights=tx_bases)
    assert per_contig.max() / per_contig.sum() > 0.2            # the oversized contig
    for n in (2, 4, 8):
        shards, load, spans = shard.record_shards(w.tx_contig, tx_bases, len(w.contig_len), n,
                                                  tx_start=w.ex_start[first[:-1]])
        assert shard.imbalance(load) < 0.05, (n, shard.imbalance(load))
        assert sum(len(s) for s in shards) == w.n_tx
        assert load.sum() == w.cds_bases
        assert np.any(spans[:, 0] != spans[:, 1])               # a contig spans ranks
        del shards


def test_reassemble_split_contig_global_order():
    """Per-rank outputs of a sharded job (oracle extraction of each shard)
    put back together equal the single-job output, with contigs split."""
    from magot_amd import shard, synth
    from oracle import cds_oracle
    w = synth.make('small', seed=11, genome_bases=300_000, n_tx=400)
    first = np.zeros(w.n_tx + 1, dtype=np.int64)
    np.cumsum(w.ex_count, out=first[1:])
    tx_bases = np.add.reduceat(w.ex_len, first[:-1])
    shards, load, spans = shard.record_shards(w.tx_contig, tx_bases, len(w.contig_len), 5,
                                              tx_start=w.ex_start[first[:-1]])
    assert np.any(spans[:, 0] != spans[:, 1])
    for protein in (False, True):
        full, foff, _ = cds_oracle.extract_workload(w, protein)
        parts, offs = [], []
        for sh in shards:
            out, off, st = cds_oracle.extract_workload(w, protein, tx_subset=sh)
            assert not st.any()
            parts.append(out)
            offs.append(off)
        got, goff = shard.reassemble(shards, parts, offs)
        assert np.array_equal(got, full) and np.array_equal(goff, foff)


def test_genome_ordered_shards_reassemble_to_global_order():
    """Ranks extract their shards in genome order (shard.genome_order); the
    reassembly, which follows the order each rank's records were given in,
    still yields the single-job output in global record order."""
    from magot_amd import shard, synth
    from oracle import cds_oracle
    w = synth.make('small', seed=13, genome_bases=300_000, n_tx=300)
    first = np.zeros(w.n_tx + 1, dtype=np.int64)
    np.cumsum(w.ex_count, out=first[1:])
    tx_bases = np.add.reduceat(w.ex_len, first[:-1])
    tx_start = w.ex_start[first[:-1]]
    shards, _, _ = shard.record_shards(w.tx_contig, tx_bases, len(w.contig_len), 3,
                                       tx_start=tx_start)
    ordered = [shard.genome_order(sh, w.tx_contig, tx_start) for sh in shards]
    for sh, od in zip(shards, ordered):
        assert np.array_equal(np.sort(od), sh)                 # the same records
        key = w.tx_contig[od] * 10**9 + tx_start[od]
        assert np.all(np.diff(key) >= 0)                       # in genome order
    assert any(not np.array_equal(a, b) for a, b in zip(shards, ordered))
    for protein in (False, True):
        full, foff, _ = cds_oracle.extract_workload(w, protein)
        parts, offs = [], []
        for od in ordered:
            out, off, st = cds_oracle.extract_workload(w, protein, tx_subset=od)
            parts.append(out)
            offs.append(off)
        got, goff = shard.reassemble(ordered, parts, offs)
        assert np.array_equal(got, full) and np.array_equal(goff, foff)


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


def test_six_frame_blocks_reassemble_to_single_gpu_layout():
    """C5 over N ranks: each rank's six-frame output is its records' blocks of
    six 16-byte padded streams (magot_orf6_sizes over its own records); one
    segment per record puts them back into exactly the layout a single-GPU
    job writes (magot_orf6_sizes over the global record order), stream by
    stream (j = 6 * record + 2 * frame + strand)."""
    from magot_amd import engine, shard
    rng = np.random.default_rng(17)
    n = 700
    rec_len = rng.integers(0, 400, size=n)
    rec_len[:5] = [0, 1, 2, 3, 5]                       # None streams and short frames
    noff = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(rec_len, out=noff[1:])
    gsoff, gslen = engine.orf6_sizes(noff)
    # the single-GPU output: stream j filled with a byte derived from j
    glob = np.zeros(int(gsoff[-1]), dtype=np.uint8)
    for j in range(6 * n):
        glob[int(gsoff[j]):int(gsoff[j]) + int(gslen[j])] = (j * 37 + 11) & 0xFF
    tx_contig = np.sort(rng.integers(0, 6, size=n))
    shards, _, _ = shard.record_shards(tx_contig, rec_len + 1, 6, 4,
                                       tx_start=rng.integers(0, 10**6, size=n))
    parts, offs = [], []
    for sh in shards:
        lo = np.zeros(len(sh) + 1, dtype=np.int64)
        np.cumsum(rec_len[sh], out=lo[1:])
        soff, slen = engine.orf6_sizes(lo)
        part = np.zeros(int(soff[-1]), dtype=np.uint8)
        for i, t in enumerate(sh):
            for k in range(6):
                j = 6 * int(t) + k
                part[int(soff[6 * i + k]):int(soff[6 * i + k]) + int(slen[6 * i + k])] = \
                    (j * 37 + 11) & 0xFF
        parts.append(part)
        offs.append(shard.six_frame_blocks(soff, slen))
    got, goff = shard.reassemble(shards, parts, offs)
    assert np.array_equal(goff, gsoff[0::6].astype(np.int64))
    assert np.array_equal(got, glob)


def test_reassembly_tables_rank_major():
    from magot_amd import shard
    shards = [np.array([1, 3]), np.array([0, 2, 4])]
    offs = [np.array([0, 5, 6]), np.array([0, 2, 2, 9])]
    src, dst, goff = shard.reassembly_tables(shards, offs, cap=16)
    assert goff.tolist() == [0, 2, 7, 7, 8, 15]
    assert dst.tolist() == goff.tolist()
    assert src.tolist() == [16, 0, 18, 5, 18]
    with pytest.raises(ValueError):
        shard.reassembly_tables(shards, [offs[0], offs[1][:-1]], cap=16)
    # (starts, lengths) places: rank 1 lays its records out as 4, 0, 2
    pl = [(np.array([0, 5]), np.array([5, 1])), (np.array([7, 9, 0]), np.array([2, 0, 7]))]
    src2, dst2, goff2 = shard.reassembly_tables(shards, pl, cap=16)
    assert dst2.tolist() == goff.tolist() and src2.tolist() == [23, 0, 25, 5, 16]
    # six-frame blocks: a record's six padded streams
    st, ln = shard.six_frame_blocks(np.array([32, 48, 64, 96, 112, 128, 0, 0, 0, 0, 0, 16, 144]),
                                    np.array([10, 16, 20, 1, 0, 16, 0, 0, 0, 0, 0, 3]))
    assert st.tolist() == [32, 0] and ln.tolist() == [16 + 16 + 32 + 16 + 0 + 16, 16]


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
    offs = shard.gather_offsets(dist, rank, world, np.arange(3 + rank) * (rank + 2))
    if rank == 0:
        q.put(([g.tolist() for g in got], [o.tolist() for o in offs]))
    else:
        assert offs is None
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
    got, offs = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        n = 10 + 7 * r
        assert got[r] == [(i + r) & 0xFF for i in range(n)]
        assert offs[r] == [i * (r + 2) for i in range(3 + r)]


# ---------------------------------------------------------------------------
# bench.py launching its own ranks (python bench.py --gpus N, no torchrun)
# ---------------------------------------------------------------------------

_CHILD = r"""
import json, os, sys
sys.path.insert(0, %(root)r)
import bench
dist, rank, local, world = bench.dist_setup()
assert (rank, local) == (int(os.environ['RANK']), int(os.environ['LOCAL_RANK']))
assert dist.get_backend() == 'gloo'
fail = int(sys.argv[1]) if len(sys.argv) > 1 else -1
if rank == fail:
    sys.exit(3)
bench.barrier(dist)
s = bench.allreduce_sum(dist, float(rank + 1))
if rank == 0:
    print(json.dumps({'n_gpus': world, 'sum': s}), flush=True)
dist.destroy_process_group()
"""


def _launch(tmp_path, n, argv):
    import subprocess
    child = tmp_path / 'child.py'
    child.write_text(_CHILD % {'root': ROOT})
    code = ('import sys; sys.path.insert(0, %r); import bench; '
            'sys.exit(bench.spawn_ranks(%d, %r, script=%r))' % (ROOT, n, argv, str(child)))
    env = dict(os.environ, MAGOT_DIST_BACKEND='gloo')
    env.pop('WORLD_SIZE', None)
    return subprocess.run([sys.executable, '-c', code], env=env, capture_output=True,
                          text=True, timeout=180)


def test_spawn_ranks_two_gloo(tmp_path):
    import json
    r = _launch(tmp_path, 2, [])
    assert r.returncode == 0, r.stderr
    # gloo itself prints "[Gloo] Rank 0 is connected ..." on stdout
    lines = [x for x in r.stdout.splitlines() if x.startswith('{')]
    assert len(lines) == 1                                   # rank 0's line only
    assert json.loads(lines[0]) == {'n_gpus': 2, 'sum': 3.0}


def test_spawn_ranks_failure_propagates(tmp_path):
    # rank 1 exits 3 while rank 0 waits in a barrier: the launcher reports
    # 3 and terminates rank 0 instead of hanging
    r = _launch(tmp_path, 2, ['1'])
    assert r.returncode == 3
    assert '{' not in r.stdout


def test_bench_refuses_more_ranks_than_devices(tmp_path):
    import subprocess
    env = dict(os.environ)
    env.pop('WORLD_SIZE', None)
    env.pop('MAGOT_DIST_BACKEND', None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), '--gpus', '2'],
                       env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 2 and 'device(s) visible' in r.stderr
