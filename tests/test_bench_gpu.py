"""bench.py end to end on the GPU at test size: the one-rank job and the
multi-rank C4 path that ``python bench.py --gpus N`` launches itself (two
ranks rehearsed on one card with MAGOT_DIST_BACKEND=gloo; the RCCL path is the
same code with the nccl backend, one GPU per rank; RCCL refuses two ranks on
one device, so MAGOT_COLLECTIVE_TENSORS=cuda rehearses its device-tensor
collectives through gloo).  Each rank checks its own
shard against the C oracle, and rank 0 checks the outputs gathered from every
rank in global record order."""

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _failure(r):
    """A failed child's exit, with a signal named (a native crash: bench.py's
    fault handler has printed every thread's stack into the stderr tail)."""
    import signal
    what = 'exit status %d' % r.returncode
    if r.returncode < 0:
        try:
            what = 'killed by %s' % signal.Signals(-r.returncode).name
        except ValueError:
            what = 'killed by signal %d' % -r.returncode
    return '%s; stderr tail:\n%s' % (what, r.stderr[-6000:])


def _bench(args, env_extra=None):
    env = dict(os.environ)
    for k in ('WORLD_SIZE', 'MAGOT_DIST_BACKEND', 'MAGOT_COLLECTIVE_TENSORS'):
        env.pop(k, None)
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py')] + args, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, _failure(r)
    lines = [x for x in r.stdout.splitlines() if x.startswith('{')]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


COMMON = ['--steps', '5', '--warmup', '1', '--settle-ms', '5', '--no-cpu-baseline']


def test_bench_one_rank():
    d = _bench(['--config', 'small'] + COMMON)
    assert d['n_gpus'] == 1 and d['scaling'] == 'strong'
    assert d['parity'].startswith('bit-exact'), d['parity']
    assert d['value'] > 0 and d['roofline']['kernel_ms'] > 0
    assert d['phases_s']['outputs_d2h_pinned'] > 0
    # kernel time from events around exactly the K timed launches
    tl = d['roofline']['timed_launches']
    assert tl['count'] == 5 and tl['first'] == 1 + d['settle']['launches'] + 1
    assert d['roofline']['kernel_ms'] <= d['ms_per_step'] * 1.05
    probe = d['box_state']['probe_before']
    assert probe['store_gbs'] > 100 and probe['copy_gbs'] > 100


@pytest.mark.parametrize('tensors', ['cpu', 'cuda'])
def test_bench_spawns_two_ranks_strong(tensors):
    """The C4 job over two ranks; 'cuda': the genome broadcast, the size
    exchanges and the output gather take device tensors, as under nccl."""
    d = _bench(['--gpus', '2', '--config', 'small'] + COMMON,
               {'MAGOT_DIST_BACKEND': 'gloo', 'MAGOT_COLLECTIVE_TENSORS': tensors})
    assert d['outputs_gather']['collective_tensors'] == tensors
    assert d['n_gpus'] == 2 and d['scaling'] == 'strong'
    assert d['parity'].startswith('bit-exact'), d['parity']
    assert d['outputs_gather']['parity'].startswith('bit-exact'), d['outputs_gather']
    assert d['load_imbalance'] < 0.05
    assert d['genome_broadcast_s'] is not None
    assert d['config']['parallelism'].startswith('contig-sharded x2')


def test_bench_torchrun_two_ranks_strong():
    """The driver's own launch (``python -m torch.distributed.run --nnodes=1
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port P bench.py
    --gpus 2``): the ranks join torchrun's agent store through bench's tcp://
    URL; gloo with device tensors, both ranks on this card."""
    sys.path.insert(0, ROOT)
    import bench
    env = dict(os.environ)
    for k in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_ADDR', 'MASTER_PORT'):
        env.pop(k, None)
    env.update({'MAGOT_DIST_BACKEND': 'gloo', 'MAGOT_COLLECTIVE_TENSORS': 'cuda'})
    r = subprocess.run([sys.executable, '-m', 'torch.distributed.run', '--nnodes=1',
                        '--nproc-per-node', '2', '--master-addr', '127.0.0.1',
                        '--master-port', str(bench._free_port()),
                        os.path.join(ROOT, 'bench.py'), '--gpus', '2', '--config', 'small'] +
                       COMMON, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, _failure(r)
    lines = [x for x in r.stdout.splitlines() if x.startswith('{')]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d['n_gpus'] == 2 and d['scaling'] == 'strong'
    assert d['parity'].startswith('bit-exact'), d['parity']
    assert d['outputs_gather']['parity'].startswith('bit-exact'), d['outputs_gather']


def test_bench_spawns_two_ranks_weak():
    d = _bench(['--gpus', '2', '--config', 'small', '--mode', 'weak'] + COMMON,
               {'MAGOT_DIST_BACKEND': 'gloo'})
    assert d['n_gpus'] == 2 and d['scaling'] == 'weak'
    assert d['parity'].startswith('bit-exact'), d['parity']


def test_bench_spawns_eight_ranks_strong():
    """The world-8 job end to end (eight gloo ranks sharing this card, device
    tensors handed to the collectives as under nccl): the 8-way sharding, the wire broadcast of the genome, every rank's shard
    checked, the 8-part gather and the reassembly in global record order."""
    d = _bench(['--gpus', '8', '--config', 'small'] + COMMON,
               {'MAGOT_DIST_BACKEND': 'gloo', 'MAGOT_COLLECTIVE_TENSORS': 'cuda'})
    assert d['n_gpus'] == 8 and d['outputs_gather']['collective_tensors'] == 'cuda'
    assert d['parity'].startswith('bit-exact'), d['parity']
    g = d['outputs_gather']
    assert g['parity'].startswith('bit-exact') and 'global record order' in g['parity'], g
    assert d['genome_broadcast_bytes'] < 0.35 * d['genome_arena_bytes']
    assert d['host']['peak_rss_gib_max_rank'] > 0
    assert len(d['host']['peak_rss_gib_per_rank']) == 8
    assert len(d['roofline']['kernel_ms_per_rank']) == 8
    assert max(d['roofline']['kernel_ms_per_rank']) == d['roofline']['kernel_ms']


@pytest.mark.parametrize('tensors', ['cpu', 'cuda'])
def test_bench_six_frame_job_two_ranks(tensors):
    """The C5 job over two ranks: six-frame streams gathered and put back into
    the single-GPU layout, all six frames of every record checked; with
    device tensors handed to the collectives, as under nccl."""
    d = _bench(['--gpus', '2', '--config', 'small5'] + COMMON,
               {'MAGOT_DIST_BACKEND': 'gloo', 'MAGOT_COLLECTIVE_TENSORS': tensors})
    assert d['outputs_gather']['collective_tensors'] == tensors
    assert d['roofline']['kernel'] == 'orf6_kernel'
    assert d['parity'].startswith('bit-exact'), d['parity']
    g = d['outputs_gather']
    assert g['outputs'] == ['six-frame residues']
    assert g['parity'].startswith('bit-exact') and 'six frames' in g['parity'], g


@pytest.mark.parametrize('config', ['small', 'small5'])
def test_bench_dist_one_rank_rccl(config):
    """The multi-GPU job's collective path through RCCL itself (nccl backend,
    a process group of one rank on this card): the genome broadcast out of
    the wire image and the replica rebuilt from it, the output gather into
    the rank-major buffer, the reassembly on the device, the float64
    reductions -- checked bit-exact in global record order."""
    d = _bench(['--dist', '--config', config] + COMMON)
    assert d['config']['backend'] == 'nccl', d['config']
    assert d['n_gpus'] == 1
    g = d['outputs_gather']
    assert g['backend'] == 'nccl' and g['collective_tensors'] == 'cuda'
    assert g['parity'].startswith('bit-exact') and 'global record order' in g['parity'], g
    assert d['parity'] == g['parity']
    # the 2-bit replica image (+ meta), not the 1-byte-per-base arena
    assert d['genome_broadcast_bytes'] < 0.35 * d['genome_arena_bytes'], d['genome_replica']
    assert d['roofline']['kernel'] == ('orf6_kernel' if config == 'small5' else 'extract_kernel')
    # RCCL's own init record travels in the line (NCCL_DEBUG=INFO, INIT, per rank)
    lines = d['rccl_init'][0]['lines']
    assert any('Init COMPLETE' in x and 'nranks 1' in x for x in lines), d['rccl_init']
