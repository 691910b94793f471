"""Genome-ordered extraction plans (MAGOT_OUT_GENOME_ORDER): the records are
laid out in the device buffers by genome coordinate, and every delivery path
(magot_plan_fetch, magot_plan_copy_outputs, magot_fasta_text_*) still returns
record order -- byte for byte what the record-order plan returns, which the
rest of the GPU suite pins to the oracle (the C3 case here checks against the
C oracle directly).  Needs an MI355X: ``pytest -m gpu``."""

import ctypes

import numpy as np
import pytest
import torch

from magot_amd import _lib, engine, synth
from magot_amd import genome as G

pytestmark = pytest.mark.gpu

ORDER = engine.OUT_GENOME_ORDER
BOTH = engine.OUT_NUC | engine.OUT_PEP


@pytest.fixture(autouse=True, params=['auto', '6'])
def tile_size(request, monkeypatch):
    """Both extraction tile sizes (see test_gpu_parity.tile_size)."""
    if request.param == 'auto':
        monkeypatch.delenv('MAGOT_EXTRACT_LANE_CHUNKS', raising=False)
    else:
        monkeypatch.setenv('MAGOT_EXTRACT_LANE_CHUNKS', request.param)
    return request.param


@pytest.fixture(scope='module', autouse=True)
def _device():
    if _lib.lib().magot_device_count() <= 0:
        pytest.fail('no HIP device visible for a gpu test')


def _run(dev, ex, tx, outputs):
    p = engine.ExtractionPlan(dev, ex, tx, outputs)
    p.execute()
    return p, p.fetch()


def _device_bytes(plan, ptr, n):
    """n bytes of a plan's device buffer at address ptr, to the host."""
    if not n:
        return np.zeros(0, dtype=np.uint8)
    out = torch.empty(n, dtype=torch.uint8, device='cuda')
    torch.cuda.synchronize()
    engine.copy_segments(ptr, n, out.data_ptr(), [0], [0, n], ctx=plan.ctx)
    return out.cpu().numpy()


def _first_keys(w, ex, tx):
    """Each record's genome key: packed position of its first non-empty
    interval (contigs packed in index order), -1 for records without one."""
    base = np.concatenate([[0], np.cumsum(np.asarray(w.contig_len, dtype=np.int64))])
    key = np.full(len(tx), -1, dtype=np.int64)
    for r, (b, k, _) in enumerate(tx.tolist()):
        for e in range(b, b + k):
            if ex['len'][e]:
                key[r] = base[ex['contig'][e]] + (int(ex['start_rc'][e]) & ((1 << 63) - 1))
                break
    return key


def _same_as_record_order(dev, ex, tx, outputs=BOTH):
    base, want = _run(dev, ex, tx, outputs)
    plan, got = _run(dev, ex, tx, outputs | ORDER)
    try:
        for a, b in zip(got, want):
            assert (a is None and b is None) or np.array_equal(a, b)
        assert plan.nuc_bytes == base.nuc_bytes and plan.pep_bytes == base.pep_bytes
        # every record sits at its layout place, in a permutation of the buffer
        ns, ps = plan.layout()
        noff, poff = want[1].astype(np.int64), want[3].astype(np.int64)
        nlen, plen = np.diff(noff), np.diff(poff)
        for start, lens, total in ((ns, nlen, plan.nuc_bytes), (ps, plen, plan.pep_bytes)):
            st = start.astype(np.int64)
            keep = lens > 0
            order = np.argsort(st[keep], kind='stable')
            s, l = st[keep][order], lens[keep][order]
            assert np.array_equal(s, np.concatenate([[0], np.cumsum(l)[:-1]]) if len(s) else s)
            assert (l.sum() if len(l) else 0) == total
        # record-order plans report their prefix offsets as the layout
        bns, bps = base.layout()
        assert np.array_equal(bns, want[1][:-1]) and np.array_equal(bps, want[3][:-1])
        # the device buffers hold each record at its place
        nptr, pptr = _device_outputs(plan)
        for ptr_, total, start, off, ref in ((nptr, plan.nuc_bytes, ns.astype(np.int64), noff, want[0]),
                                             (pptr, plan.pep_bytes, ps.astype(np.int64), poff, want[2])):
            if ref is None or not total:
                continue
            raw = _device_bytes(plan, ptr_, total)
            for r in range(0, len(off) - 1, max(1, (len(off) - 1) // 300)):
                assert np.array_equal(raw[start[r]:start[r] + off[r + 1] - off[r]],
                                      ref[off[r]:off[r + 1]])
        # copy_outputs puts record order into caller device memory
        for which, total, ref in ((0, plan.nuc_bytes, want[0]), (1, plan.pep_bytes, want[2])):
            if ref is None or not total:
                continue
            buf = torch.full((total + 64,), 0xEE, dtype=torch.uint8, device='cuda')
            torch.cuda.synchronize()
            plan.copy_outputs(buf.data_ptr() if which == 0 else None,
                              buf.data_ptr() if which == 1 else None)
            host = buf.cpu().numpy()
            assert np.array_equal(host[:total], ref)
            assert (host[total:] == 0xEE).all()  # nothing written past the end
        return plan.layout()
    finally:
        plan.close()
        base.close()


def _device_outputs(plan):
    """The plan's device output buffers (magot_plan_device_outputs)."""
    n, p = ctypes.c_void_p(), ctypes.c_void_p()
    _lib.check(_lib.lib().magot_plan_device_outputs(plan.handle, ctypes.byref(n),
                                                    ctypes.byref(p)), 'magot_plan_device_outputs')
    return n.value, p.value


@pytest.mark.parametrize('config', ['small', 'C2'])
def test_genome_order_matches_record_order(config):
    w = synth.make(config)
    dev = engine.DeviceGenome(w.contigs())
    try:
        ex, tx = w.plan_tables()
        ns, _ = _same_as_record_order(dev, ex, tx)
        # the layout really is in genome order: places ascend with the first
        # interval's genome position (ties keep record order)
        key = _first_keys(w, ex, tx)
        has = key >= 0
        by_key = np.argsort(key[has], kind='stable')
        assert (np.diff(ns[has][by_key].astype(np.int64)) >= 0).all()
        assert not np.array_equal(by_key, np.arange(has.sum()))  # GFF order differs
        _same_as_record_order(dev, ex, tx, engine.OUT_NUC)
        _same_as_record_order(dev, ex, tx, engine.OUT_PEP)
    finally:
        dev.close()


def _edge_tables(w):
    """Records with no intervals, empty intervals, 1-2 bases (no codon), both
    strands, identical starts and records given in reverse genome order."""
    rng = np.random.default_rng(5)
    n_contigs = len(w.contig_len)
    rows, recs = [], []
    for r in range(400):
        k = int(rng.integers(0, 4))
        recs.append((len(rows), k))
        c = int(rng.integers(0, n_contigs))
        clen = int(w.contig_len[c])
        for j in range(k):
            kind = rng.integers(0, 6)
            ln = 0 if kind == 0 else (int(rng.integers(1, 3)) if kind == 1
                                      else int(rng.integers(3, 900)))
            ln = min(ln, clen)
            st = (400 - r) * 37 % max(1, clen - ln) if kind != 2 else 0
            rc = int(rng.integers(0, 2)) << 63
            rows.append((st | rc, c, ln))
    ex = np.array(rows, dtype=_lib.EXON_DTYPE)
    tx = np.array([(b, k, 0) for b, k in recs], dtype=_lib.TX_DTYPE)
    return ex, tx


@pytest.mark.parametrize('batch', ['1', '37', '4096'])
def test_genome_order_fetch_in_bounded_batches(monkeypatch, batch):
    """magot_plan_fetch of a genome-ordered plan reassembles through a bounded
    scratch, batch by batch of records (MAGOT_FETCH_BATCH_BYTES; a record
    longer than the batch is a batch of its own, odd batch starts keep the
    copy's 16-byte alignment): byte for byte the record-order fetch."""
    monkeypatch.setenv('MAGOT_FETCH_BATCH_BYTES', batch)
    w = synth.make('small')
    dev = engine.DeviceGenome(w.contigs())
    try:
        ex, tx = w.plan_tables()
        base, want = _run(dev, ex, tx, BOTH)
        plan, got = _run(dev, ex, tx, BOTH | ORDER)
        try:
            for a, b in zip(got, want):
                assert np.array_equal(a, b)
        finally:
            plan.close()
            base.close()
        ex2, tx2 = _edge_tables(w)
        _same_as_record_order(dev, ex2, tx2)
    finally:
        dev.close()


def test_genome_order_edge_records():
    w = synth.make('small')
    dev = engine.DeviceGenome(w.contigs())
    try:
        ex, tx = _edge_tables(w)
        _same_as_record_order(dev, ex, tx)
        # no records at all, and one record
        _same_as_record_order(dev, ex[:0], tx[:0])
        _same_as_record_order(dev, ex[:tx['n_exons'][0]], tx[:1])
    finally:
        dev.close()


def test_genome_order_refusals():
    w = synth.make('small')
    dev = engine.DeviceGenome(w.contigs())
    try:
        ex, tx = w.plan_tables()
        p = engine.ExtractionPlan(dev, ex, tx, engine.OUT_NUC | ORDER)
        with pytest.raises(_lib.MagotError, match='GENOME_ORDER'):
            engine.Orf6Plan(p)
        p.execute()
        buf = torch.zeros(p.nuc_bytes + 64, dtype=torch.uint8, device='cuda')
        torch.cuda.synchronize()
        with pytest.raises(_lib.MagotError, match='16-byte'):
            p.copy_outputs(buf.data_ptr() + 1, None)
        p.close()
        with pytest.raises(_lib.MagotError, match='unknown output flags'):
            engine.ExtractionPlan(dev, ex, tx, engine.OUT_NUC | 8)
    finally:
        dev.close()


@pytest.mark.parametrize('seq_type', ['nucleotide', 'protein'])
def test_genome_order_fasta_text(seq_type):
    """The device FASTA text of a genome-ordered plan is the record-order text."""
    w = synth.make('small')
    fasta, gff = w.fasta_text(), w.gff3_text()
    gs = G.GenomeSequence(fasta)
    names = list(gs)
    dev = engine.DeviceGenome([(n, gs[n]) for n in names])
    plan = engine.GffPlan.build(G.ensure_file(gff).read(), names, [len(gs[n]) for n in names],
                                protein=seq_type == 'protein', order='py2')
    assert plan is not None
    out = engine.OUT_PEP if seq_type == 'protein' else engine.OUT_NUC
    texts = []
    try:
        for flags in (out, out | ORDER):
            ex = engine.ExtractionPlan(dev, plan.exons, plan.txs, flags)
            text = engine.FastaText(plan, ex)
            ex.execute()
            text.execute()
            texts.append(text.fetch().tobytes())
            text.close()
            ex.close()
    finally:
        plan.close()
        dev.close()
    assert texts[0] == texts[1] and len(texts[0]) > 1000


@pytest.mark.slow
def test_genome_order_c3_vs_c_oracle():
    """The benchmark's C3 job laid out in genome order, fetched and compared
    with the C oracle over every byte (nucleotides and trimmed peptides)."""
    from oracle import cds_oracle
    from test_gpu_sharded import pep_matches
    w = synth.make('C3')
    dev = engine.DeviceGenome(w.contigs())
    try:
        ex, tx = w.plan_tables()
        p, (nuc, noff, pep, poff) = _run(dev, ex, tx, BOTH | ORDER)
        p.close()
        ref, roff, st = cds_oracle.extract_workload(w, False)
        assert np.array_equal(noff.astype(np.int64), roff)
        assert np.array_equal(nuc, ref)
        del ref
        pref = cds_oracle.extract_workload(w, True)[0]
        assert pep_matches(pep, poff, pref)
    finally:
        dev.close()
