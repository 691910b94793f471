"""The multi-GPU job's data path at full size, rehearsed on one GPU
(BASELINE configs[3] "C4" and configs[4] "C5 over 8 GPUs").

For N = 2, 4 and 8: the real C3 (C5) tables are sharded with
``shard.record_shards`` exactly as ``bench.py --gpus N`` shards them, every
rank's shard is planned and run on this GPU (the tile size each shard's plan
picks: 3-slot tiles for one GPU's share of the 8-GPU C3 job), the per-rank
outputs are laid out rank-major as the RCCL gather leaves them on rank 0, put
back into global record order by ``shard.reassemble_device``
(magot_copy_segments) and compared byte for byte with the C oracle over the
WHOLE job: C3's nucleotides and peptides, all six frames of every C5 record.
"""

import os

import numpy as np
import pytest
import torch

from magot_amd import _lib, engine, shard, synth

pytestmark = [pytest.mark.gpu, pytest.mark.slow]


@pytest.fixture(scope='module', autouse=True)
def _device():
    if _lib.lib().magot_device_count() <= 0:
        pytest.fail('no HIP device visible for a gpu test')


def _threads():
    return int(os.environ.get('OMP_NUM_THREADS', '0')) or min(16, os.cpu_count() or 1)


_cache = {}


def _job(config):
    """Workload, its packed genome and the oracle's whole-job output (one
    configuration held at a time)."""
    from oracle import cds_oracle
    if config not in _cache:
        for k in list(_cache):
            _cache.pop(k)[1].close()
        w = synth.make(config)
        dev = engine.DeviceGenome(w.contigs())
        ref, roff, st = cds_oracle.extract_workload(w, False)
        assert not st.any()
        pref = cds_oracle.extract_workload(w, True)[0] if config == 'C3' else None
        _cache[config] = (w, dev, ref, roff, pref)
    return _cache[config]


def pep_matches(pep, poff, pref):
    """Device peptides (untrimmed frame 0) == oracle peptides (one leading 'X'
    trimmed per record, genome.py:819-821)."""
    starts = poff[:-1].astype(np.int64)
    lens = (poff[1:] - poff[:-1]).astype(np.int64)
    first = np.zeros(len(starts), dtype=bool)
    first[lens > 0] = pep[starts[lens > 0]] == ord('X')
    keep = np.ones(len(pep), dtype=bool)
    keep[starts[first]] = False
    return np.array_equal(pep[keep], pref)


def _shards(w, n):
    first = np.zeros(w.n_tx + 1, dtype=np.int64)
    np.cumsum(w.ex_count, out=first[1:])
    tx_bases = np.add.reduceat(w.ex_len, first[:-1])
    shards, load, spans = shard.record_shards(w.tx_contig, tx_bases, len(w.contig_len), n,
                                              tx_start=w.ex_start[first[:-1]])
    assert shard.imbalance(load) < 0.05
    assert sorted(np.concatenate(shards).tolist()) == list(range(w.n_tx))
    return shards


def _rank_major(parts, sizes):
    """The rank-major receive buffer of a gather (16-byte aligned slots)."""
    cap = (max(max(sizes), 1) + 15) & ~15
    buf = torch.zeros(len(parts) * cap, dtype=torch.uint8, device='cuda')
    torch.cuda.synchronize()  # the library's stream does not wait for torch's fill
    for r, fill in enumerate(parts):
        if sizes[r]:
            fill(buf[r * cap:].data_ptr())
    torch.cuda.synchronize()
    return buf, cap


@pytest.mark.parametrize('n', [2, 4, 8])
def test_c4_shards_reassembled_vs_c_oracle(n):
    w, dev, ref, roff, pref = _job('C3')
    shards = _shards(w, n)
    plans = []
    try:
        for sh in shards:
            ex, tx = w.plan_tables(tx_subset=sh)
            p = engine.ExtractionPlan(dev, ex, tx)
            p.execute()
            plans.append(p)
        offs = [p.fetch_to(None, None) for p in plans]
        nbuf, ncap = _rank_major([lambda a, p=p: p.copy_outputs(a, None) for p in plans],
                                 [p.nuc_bytes for p in plans])
        nuc, goff = shard.reassemble_device(shards, [o[0].astype(np.int64) for o in offs], nbuf,
                                            ncap)
        assert np.array_equal(goff, roff)
        got = nuc.cpu().numpy()
        if not np.array_equal(got, ref):
            bad = int(np.nonzero(got != ref)[0][0])
            raise AssertionError('N=%d: nucleotide byte %d (record %d) differs'
                                 % (n, bad, int(np.searchsorted(roff, bad, 'right') - 1)))
        del nbuf, nuc
        pbuf, pcap = _rank_major([lambda a, p=p: p.copy_outputs(None, a) for p in plans],
                                 [p.pep_bytes for p in plans])
        pep, pgoff = shard.reassemble_device(shards, [o[1].astype(np.int64) for o in offs], pbuf,
                                             pcap)
        assert pep_matches(pep.cpu().numpy(), pgoff, pref)
    finally:
        for p in plans:
            p.close()


@pytest.mark.parametrize('n', [2, 4, 8])
def test_c5_shards_reassembled_six_frames_vs_c_oracle(n):
    from oracle import cds_oracle
    w, dev, ref, roff, _ = _job('C5')
    shards = _shards(w, n)
    plans, o6s = [], []
    try:
        for sh in shards:
            ex, tx = w.plan_tables(tx_subset=sh)
            p = engine.ExtractionPlan(dev, ex, tx, engine.OUT_NUC)
            o = engine.Orf6Plan(p)
            o.execute()
            plans.append(p)
            o6s.append(o)
        offs = []
        for o in o6s:
            soff, slen = o.fetch_to(None)
            offs.append(shard.six_frame_blocks(soff, slen))  # blocks in the plan's walk order
        buf, cap = _rank_major([o.copy_outputs for o in o6s], [o.total for o in o6s])
        for o in o6s:
            o.close()
        o6s = []
        for p in plans:
            p.close()
        plans = []
        out, goff = shard.reassemble_device(shards, offs, buf, cap)
        soff, slen = engine.orf6_sizes(roff)
        assert np.array_equal(goff, soff[0::6].astype(np.int64))
        host = out.cpu().numpy()
        del buf, out
        assert cds_oracle.orf6_compare(ref, roff, host, soff, slen, threads=_threads()) == (0, -1)
    finally:
        for o in o6s:
            o.close()
        for p in plans:
            p.close()
