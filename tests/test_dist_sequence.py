"""The multi-GPU job's collective calls at N = 8, on CPU, against a mocked
``torch.distributed``.

RCCL needs what gloo forgives: every rank issues the same collectives in the
same order, a gather's or all_gather's buffers have the same size on every
rank, and the process group is bound to the rank's device.  These tests run
bench.py's start-up (``dist_setup``) and its output return
(``gather_outputs``: size exchanges, padded gathers, offset gathers,
reductions) in eight threads over an in-memory fake of the collectives that
records every call, then check:
  * the ``init_process_group`` arguments of every rank (explicit tcp:// URL
    on 127.0.0.1, rank, world size, ``device_id`` = the rank's GPU) and that
    the device is bound before the group exists;
  * one identical call sequence on all ranks (op, dtype, shape), every
    gather / all_gather with equal-sized buffers, nothing but
    nccl-supported collectives;
  * rank 0's reassembled output equal to the job's global record order.
"""
import ctypes
import os
import sys
import threading
import types

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

WORLD = 8
NCCL_OPS = {'all_gather', 'gather', 'all_reduce', 'broadcast', 'barrier',
            'broadcast_object_list', 'all_gather_object'}


class FakeGroup(object):
    """The shared state of WORLD ranks in threads: every collective meets at a
    barrier, exchanges through slots, and is recorded per rank."""

    def __init__(self, world):
        self.world = world
        self.bar = threading.Barrier(world, timeout=60)
        self.slots = [None] * world
        self.calls = [[] for _ in range(world)]
        self.init_kwargs = [None] * world


class FakeDist(object):
    ReduceOp = types.SimpleNamespace(MAX='max', SUM='sum')

    def __init__(self, group, rank, backend='nccl'):
        self.g, self.rank, self.backend = group, rank, backend

    # -- bookkeeping ------------------------------------------------------------
    def _rec(self, name, *tensors, **extra):
        sig = tuple((str(t.dtype), tuple(t.shape)) for t in tensors)
        self.g.calls[self.rank].append((name, sig, tuple(sorted(extra.items()))))

    def _exchange(self, value):
        self.g.slots[self.rank] = value
        self.g.bar.wait()
        got = list(self.g.slots)
        self.g.bar.wait()
        return got

    # -- the torch.distributed surface bench.py and shard.py use -----------------
    def init_process_group(self, **kw):
        self.g.init_kwargs[self.rank] = kw
        self._exchange(None)

    def get_backend(self):
        return self.backend

    def get_world_size(self):
        return self.g.world

    def barrier(self):
        self._rec('barrier')
        self._exchange(None)

    def all_gather(self, out, t):
        self._rec('all_gather', t, *out)
        for o in out:
            assert o.shape == t.shape and o.dtype == t.dtype, 'all_gather: unequal buffers'
        got = self._exchange(t.clone())
        for o, v in zip(out, got):
            assert v.shape == t.shape, 'all_gather: ranks disagree on the size'
            o.copy_(v)

    def gather(self, t, gather_list=None, dst=0):
        self._rec('gather', t, dst=dst)
        got = self._exchange(t.clone())
        assert all(v.shape == t.shape and v.dtype == t.dtype for v in got), \
            'gather: ranks disagree on the size'
        if self.rank == dst:
            assert len(gather_list) == self.g.world
            for o, v in zip(gather_list, got):
                assert o.shape == v.shape
                o.copy_(v)
        else:
            assert gather_list is None

    def all_reduce(self, t, op=None):
        self._rec('all_reduce', t, op=op)
        got = self._exchange(t.clone())
        stack = torch.stack(got)
        t.copy_(stack.max(0).values if op == 'max' else stack.sum(0))

    def broadcast(self, t, src=0):
        self._rec('broadcast', t, src=src)
        got = self._exchange(t.clone())
        t.copy_(got[src])

    def all_gather_object(self, out, obj):
        self._rec('all_gather_object')
        got = self._exchange(obj)
        out[:] = got

    def broadcast_object_list(self, lst, src=0):
        self._rec('broadcast_object_list')
        got = self._exchange(list(lst))
        lst[:] = got[src]


def _run_ranks(fn):
    group = FakeGroup(WORLD)
    errors = [None] * WORLD
    results = [None] * WORLD

    def body(r):
        try:
            results[r] = fn(FakeDist(group, r), r)
        except BaseException as e:          # noqa: B902 -- reported below
            errors[r] = e
            group.bar.abort()

    th = [threading.Thread(target=body, args=(r,)) for r in range(WORLD)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    for e in errors:
        if e is not None and not isinstance(e, threading.BrokenBarrierError):
            raise e
    assert not any(errors), errors
    return group, results


def test_dist_init_kwargs_eight_ranks():
    import bench
    env = {'MASTER_ADDR': '127.0.0.1', 'MASTER_PORT': '29511'}
    for r in range(WORLD):
        kw = bench.dist_init_kwargs('nccl', r, WORLD, r, env=env)
        assert kw['init_method'] == 'tcp://127.0.0.1:29511'
        assert (kw['rank'], kw['world_size'], kw['backend']) == (r, WORLD, 'nccl')
        assert kw['device_id'] == torch.device('cuda', r)
    # no name to resolve without MASTER_ADDR; gloo gets no device binding
    kw = bench.dist_init_kwargs('gloo', 3, WORLD, None, env={'MASTER_PORT': '1'})
    assert kw['init_method'] == 'tcp://127.0.0.1:1' and 'device_id' not in kw


def test_dist_setup_binds_device_before_the_group(monkeypatch, tmp_path):
    """dist_setup on eight ranks (mocked): the device is selected and its
    context made before init_process_group, which gets the tcp:// URL and
    device_id; RCCL's init log goes to one file per rank."""
    import bench
    import torch.distributed as tdist
    order = []

    def fake_bind(local):
        order.append(('bind', local))
        return local

    monkeypatch.setattr(bench, 'bind_device', fake_bind)
    monkeypatch.delenv('MAGOT_DIST_BACKEND', raising=False)
    monkeypatch.setenv('TMPDIR', str(tmp_path))
    for k in ('NCCL_DEBUG_SUBSYS', 'NCCL_DEBUG_FILE'):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv('NCCL_DEBUG', 'VERSION')      # the pool's boxes preset it
    seen = []

    def fake_init(**kw):
        order.append(('init', kw['rank']))
        seen.append((kw, os.environ.get('NCCL_DEBUG_FILE'), os.environ.get('NCCL_DEBUG')))

    monkeypatch.setattr(tdist, 'init_process_group', fake_init)
    for r in range(WORLD):
        monkeypatch.setenv('WORLD_SIZE', str(WORLD))
        monkeypatch.setenv('RANK', str(r))
        monkeypatch.setenv('LOCAL_RANK', str(r))
        monkeypatch.setenv('MASTER_ADDR', '127.0.0.1')
        monkeypatch.setenv('MASTER_PORT', '29600')
        monkeypatch.delenv('NCCL_DEBUG_FILE', raising=False)
        d, rank, local, world = bench.dist_setup()
        assert (rank, local, world) == (r, r, WORLD) and d is tdist
    assert order == [x for r in range(WORLD) for x in (('bind', r), ('init', r))]
    files = set()
    for r, (kw, f, level) in enumerate(seen):
        assert kw['backend'] == 'nccl' and kw['device_id'] == torch.device('cuda', r)
        assert kw['init_method'] == 'tcp://127.0.0.1:29600'
        assert (kw['rank'], kw['world_size']) == (r, WORLD)
        assert level == 'INFO' and f.endswith('rank%d.log' % r) and str(tmp_path) in f
        files.add(f)
    assert len(files) == WORLD


def test_rccl_init_summary_keeps_the_init_lines(tmp_path):
    import bench
    p = tmp_path / 'rank0.log'
    p.write_text('h:1:1 [0] NCCL INFO Kernel version: 6.18\n'
                 'h:1:1 [0] NCCL INFO RCCL version : 2.26.6-HEAD:64f48b6\n'
                 'h:1:2 [0] NCCL INFO ncclCommInitRankConfig_impl comm 0x1 rank 0 nranks 8 '
                 'cudaDev 0 busId a4000 commId 0x2 - Init COMPLETE\n'
                 'h:1:2 [0] NCCL INFO something else\n')
    s = bench.rccl_init_summary(str(p))
    assert len(s['lines']) == 2 and 'Init COMPLETE' in s['lines'][1]
    assert bench.rccl_init_summary(str(tmp_path / 'none.log'))['lines'] == []


class FakePlan(object):
    """One rank's extraction plan as gather_outputs sees it: outputs in the
    rank's own (genome) order, copied into the Gather's send buffer."""

    def __init__(self, nuc, noff, pep, poff):
        from magot_amd import engine
        self.nuc, self.noff, self.pep, self.poff = nuc, noff, pep, poff
        self.nuc_bytes, self.pep_bytes = len(nuc), len(pep)
        self.outputs = engine.OUT_NUC | engine.OUT_PEP

    def fetch_to(self, a, b):
        assert a is None and b is None
        return self.noff, self.poff

    def copy_outputs(self, a, b):
        src = self.nuc if a is not None else self.pep
        if len(src):
            ctypes.memmove(a if a is not None else b, src.ctypes.data, len(src))


@pytest.mark.parametrize('with_empty_rank', [False, True])
def test_gather_outputs_collective_sequence_eight_ranks(monkeypatch, with_empty_rank):
    import bench
    from magot_amd import shard
    rng = np.random.default_rng(8)
    n = 400
    nlen = rng.integers(0, 300, size=n)
    plen = nlen // 3
    tx_contig = np.sort(rng.integers(0, 5, size=n))
    tx_start = rng.integers(0, 10**6, size=n)
    weights = nlen + 1
    if with_empty_rank:
        weights = weights.copy()
        weights[:] = 1
        weights[0] = 10**9          # one record outweighs the rest: empty ranks
    shards, _, _ = shard.record_shards(tx_contig, weights, 5, WORLD, tx_start=tx_start)
    shards = [shard.genome_order(sh, tx_contig, tx_start) for sh in shards]
    if with_empty_rank:
        assert any(len(sh) == 0 for sh in shards)
    goff = np.zeros(n + 1, np.int64)
    np.cumsum(nlen, out=goff[1:])
    gpoff = np.zeros(n + 1, np.int64)
    np.cumsum(plen, out=gpoff[1:])
    gnuc = rng.integers(0, 256, size=int(goff[-1])).astype(np.uint8)
    gpep = rng.integers(0, 256, size=int(gpoff[-1])).astype(np.uint8)

    def part(sh, off, data, lens):
        lo = np.zeros(len(sh) + 1, np.int64)
        np.cumsum(lens[sh], out=lo[1:])
        buf = np.concatenate([data[off[i]:off[i + 1]] for i in sh]) if len(sh) else \
            np.zeros(0, np.uint8)
        return np.ascontiguousarray(buf, np.uint8), lo

    plans = []
    for sh in shards:
        nb, no = part(sh, goff, gnuc, nlen)
        pb, po = part(sh, gpoff, gpep, plen)
        plans.append(FakePlan(nb, no.astype(np.uint64), pb, po.astype(np.uint64)))

    monkeypatch.setattr(shard, 'OUTPUT_DEVICE', 'cpu')
    monkeypatch.setattr(shard, 'collective_device', lambda d: 'cpu')
    monkeypatch.setattr(torch.cuda, 'synchronize', lambda *a, **k: None)

    captured = []

    def host_reassemble(shards_, offs, gathered, cap, ctx=None):
        src_off, _, go = shard.reassembly_tables(shards_, offs, cap)
        flat = gathered.numpy()
        lens = go[1:] - go[:-1]
        idx = np.repeat(src_off.astype(np.int64) - go[:-1], lens) + np.arange(int(go[-1]))
        captured.append((flat[idx].copy(), go))
        return torch.from_numpy(captured[-1][0]), go

    monkeypatch.setattr(shard, 'reassemble_device', host_reassemble)
    args = types.SimpleNamespace(no_verify=True)
    w = types.SimpleNamespace(n_tx=n)

    def rank_fn(d, r):
        return bench.gather_outputs(args, d, r, WORLD, w, plans[r], None, shards, None)

    group, results = _run_ranks(rank_fn)
    # one call sequence on every rank, the same buffer shapes, nccl's ops only
    ops0 = [(op, sig, ex) for op, sig, ex in group.calls[0]]
    assert ops0, 'no collectives recorded'
    for r in range(1, WORLD):
        assert group.calls[r] == ops0, 'rank %d issued a different collective sequence' % r
    assert {op for op, _, _ in ops0} <= NCCL_OPS
    kinds = [op for op, _, _ in ops0]
    assert kinds.count('gather') == 2 + 4          # two outputs + (starts, lengths) x 2
    # rank 0 put every record back in global record order
    assert results[0]['reassembly'].startswith('magot_copy_segments')
    assert results[0]['bytes'] == len(gnuc) + len(gpep)
    assert len(captured) == 2
    assert np.array_equal(captured[0][0], gnuc) and np.array_equal(captured[0][1], goff)
    assert np.array_equal(captured[1][0], gpep) and np.array_equal(captured[1][1], gpoff)
