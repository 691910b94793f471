"""Genome placement and output reassembly on the GPU:

* the device packer (magot_genome_load, devpack.hip) against its host twin
  (MAGOT_PACK_HOST, pack.cpp): byte-equal arenas and host tables, over every
  byte value, runs across contigs / 32-byte groups / the 64 MiB staging
  chunks, empty contigs, FASTA line layout, and the C5 genome;
* the wire replica (magot_genome_wire_ranges + magot_genome_attach_wire):
  only the forward plane, runs and directory are transferred, the mirror is
  rebuilt, and the attached arena equals the packed one byte for byte;
* the compact replica image (magot_genome_wire_export / _import: 2-bit
  codes, soft-mask runs, exception runs): the genome rebuilt from it equals
  the packed arena byte for byte, over every byte value, case patterns that
  stress the mask runs and directories, edge genomes and C3 / C5;
* magot_copy_segments against numpy, aligned and unaligned.
"""

import numpy as np
import pytest
import torch

from magot_amd import _lib, engine, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module', autouse=True)
def _device():
    if _lib.lib().magot_device_count() <= 0:
        pytest.fail('no HIP device visible for a gpu test')


def _arena(g):
    buf = torch.empty(g.device_bytes, dtype=torch.uint8, device='cuda')
    g.copy_arena(buf.data_ptr())
    torch.cuda.synchronize()
    return buf.cpu().numpy()


def _defined(g, arena):
    """The arena bytes the layout defines: both nibble planes + 16 bytes of
    slack, the runs (with their sentinel) and the directory -- not the
    256-byte alignment padding between the pieces, which nothing writes."""
    (o0, l0), (o1, l1) = g.wire_ranges()
    assert o0 == 0
    runs = (g.n_exception_runs + 1) * 16
    o_dir = o1 + ((runs + 255) & ~255)
    extent = 64 + g.total_bases
    dir_bytes = 4 * (((extent + 64 + 4095) >> 12) + 2)
    assert o_dir + dir_bytes <= o1 + l1
    return np.concatenate([arena[o0:o0 + 2 * l0 + 16], arena[o1:o1 + runs],
                           arena[o_dir:o_dir + dir_bytes]])


def _assert_same_pack(contigs):
    dg = engine.DeviceGenome(contigs, pack='device')
    hg = engine.DeviceGenome(contigs, pack='host')
    try:
        assert dg.export() == hg.export()  # layout, runs, directory, contig table
        assert dg.device_bytes == hg.device_bytes
        a, b = _arena(dg), _arena(hg)
        da, db = _defined(dg, a), _defined(hg, b)
        if not np.array_equal(da, db):
            bad = int(np.nonzero(da != db)[0][0])
            raise AssertionError('arenas differ at defined byte %d: %r vs %r'
                                 % (bad, da[bad:bad + 8], db[bad:bad + 8]))
        return dg.n_exception_runs
    finally:
        dg.close()
        hg.close()


def test_device_pack_every_byte_value():
    """Every byte GenomeSequence keeps (all but CR/LF, genome.py:875) in runs
    of varying length, runs touching each other, crossing 32-byte groups and
    contig boundaries, zero-length contigs between them."""
    rng = np.random.default_rng(5)
    values = [b for b in range(256) if b not in (10, 13)]
    parts = []
    for k, b in enumerate(values * 3):
        parts.append(rng.choice(np.frombuffer(b'ACGTacgt', np.uint8), int(rng.integers(0, 40))))
        parts.append(np.full(1 + (k * 7) % 45, b, dtype=np.uint8))
    seq = np.concatenate(parts).tobytes()
    cuts = sorted(rng.choice(len(seq), 12, replace=False).tolist())
    contigs, last = [], 0
    for i, c in enumerate(cuts + [len(seq)]):
        contigs.append(('c%d' % i, seq[last:c]))
        if i % 4 == 1:
            contigs.append(('empty%d' % i, b''))
        last = c
    assert _assert_same_pack(contigs) > 700


@pytest.mark.parametrize('shape', ['empty', 'one_base', 'all_N', 'exc_at_ends'])
def test_device_pack_edge_genomes(shape):
    contigs = {
        'empty': [],
        'one_base': [('a', b'n')],
        'all_N': [('a', b'N' * 100_000), ('b', b'N' * 33)],
        'exc_at_ends': [('a', b'RACGTY'), ('b', b'YY' + b'ACGT' * 40 + b'-'), ('c', b'')],
    }[shape]
    _assert_same_pack(contigs)


def test_device_pack_crosses_staging_chunks():
    """A 210 Mb genome: runs cross the 64 MiB pinned staging chunks."""
    rng = np.random.default_rng(9)
    G = 210_000_000
    g = np.frombuffer(b'ACGT', np.uint8)[rng.integers(0, 4, size=G, dtype=np.uint8)]
    for c in range(1, 4):  # an N run straddling each chunk boundary
        p = c * (64 << 20)
        g[p - 1000:p + 1000] = ord('N')
        g[p - 3000] = ord('Y')
    g[rng.integers(0, G, 5000)] = ord('R')
    contigs = [('a', g[:G // 3].tobytes()), ('b', g[G // 3:].tobytes())]
    assert _assert_same_pack(contigs) > 4000


def test_device_pack_fasta_line_layout():
    """magot_genome_load_fasta streams the file's lines (newlines dropped) to
    the device packer: same arena as the host packer over the same contigs."""
    w = synth.make('small', seed=4, genome_bases=300_000, n_tx=10, iupac_rate=1e-3)
    text = w.fasta_text(width=61).encode('latin-1')
    fg = engine.FastaGenome.load(text)
    hg = engine.DeviceGenome(w.contigs(), pack='host')
    try:
        assert fg.names == w.contig_names
        m1, m2 = fg.export(), hg.export()
        assert m1 == m2
        assert np.array_equal(_defined(fg, _arena(fg)), _defined(hg, _arena(hg)))
    finally:
        fg.close()
        hg.close()


@pytest.mark.slow
def test_device_pack_c5_genome():
    """BASELINE configs[4]'s 3 Gb genome, device vs host packer."""
    w = synth.make('C5')
    _assert_same_pack(w.contigs())


def _wire_replica(g):
    """What a receiving rank holds: the wire ranges copied into fresh memory
    (the rest poisoned), attached with the mirror rebuilt."""
    meta, nbytes = g.export()
    src = torch.empty(nbytes, dtype=torch.uint8, device='cuda')
    g.copy_arena(src.data_ptr())
    dst = torch.full((nbytes,), 0xAB, dtype=torch.uint8, device='cuda')
    moved = 0
    for off, ln in g.wire_ranges():
        dst[off:off + ln].copy_(src[off:off + ln])
        moved += ln
    torch.cuda.synchronize()
    rep = engine.DeviceGenome.attach(meta, dst.data_ptr(), g.names, g.lengths, keepalive=dst,
                                     wire=True)
    return rep, moved


def test_wire_replica_equals_packed_arena():
    w = synth.make('small', seed=12, genome_bases=2_000_000, n_tx=800, iupac_rate=1e-3)
    g = engine.DeviceGenome(w.contigs())
    rep, moved = _wire_replica(g)
    try:
        a, b = _arena(g), _arena(rep)
        assert np.array_equal(_defined(g, a), _defined(rep, b))
        (o0, l0), (o1, l1) = g.wire_ranges()
        assert moved == l0 + l1 and o1 >= 2 * l0 + 16  # the mirror plane is not sent
        # and the replica extracts the same bytes
        ex, tx = w.plan_tables()
        outs = []
        for gen in (g, rep):
            plan = engine.ExtractionPlan(gen, ex, tx)
            outs.append(plan.run())
            plan.close()
        for x, y in zip(outs[0], outs[1]):
            assert np.array_equal(x, y)
    finally:
        rep.close()
        g.close()


@pytest.mark.slow
def test_wire_replica_c3_genome():
    w = synth.make('C3')
    g = engine.DeviceGenome(w.contigs())
    rep, moved = _wire_replica(g)
    try:
        assert np.array_equal(_defined(g, _arena(g)), _defined(rep, _arena(rep)))
        assert moved < 0.51 * g.device_bytes
    finally:
        rep.close()
        g.close()


def _image_replica(g, poison=0xAB):
    """What a receiving rank builds: the image written into fresh (poisoned)
    device memory, a genome imported from it, the image freed."""
    meta, _ = g.export()
    n = g.wire_size()
    buf = torch.full((n + 64,), poison, dtype=torch.uint8, device='cuda')
    torch.cuda.synchronize()
    assert g.wire_export(buf.data_ptr(), n) == n
    rep = engine.DeviceGenome.from_wire(meta, buf.data_ptr(), n, g.names, g.lengths)
    del buf
    torch.cuda.synchronize()
    return rep, n


def _assert_image_round_trip(contigs, max_frac=None):
    g = engine.DeviceGenome(contigs)
    rep, n = _image_replica(g)
    try:
        assert rep.export() == g.export()
        a, b = _defined(g, _arena(g)), _defined(rep, _arena(rep))
        if not np.array_equal(a, b):
            bad = int(np.nonzero(a != b)[0][0])
            raise AssertionError('rebuilt arena differs at defined byte %d: %r vs %r'
                                 % (bad, b[bad:bad + 8], a[bad:bad + 8]))
        if max_frac is not None:
            assert n < max_frac * g.device_bytes, (n, g.device_bytes)
        return g.device_bytes, n
    finally:
        rep.close()
        g.close()


def _case_genome(kind, rng):
    acgt = np.frombuffer(b'ACGTacgt', np.uint8)
    if kind == 'alternating_case':   # a mask run every other base: the densest run list
        s = np.frombuffer(b'ACGT', np.uint8)[rng.integers(0, 4, 300_000)].copy()
        s[1::2] |= 0x20
        return [('a', s.tobytes()), ('b', s[:77].tobytes())]
    if kind == 'all_lower':          # one mask run across many directory blocks
        return [('a', b'acgt' * 50_000), ('b', b'ttt'), ('c', b'a' * 8191)]
    if kind == 'mixed':              # mask runs cut by exceptions (n, N, IUPAC, '-')
        parts = []
        for _ in range(4000):
            k = int(rng.integers(0, 5))
            ln = int(rng.integers(1, 70))
            if k == 0:
                parts.append(rng.choice(acgt[4:], ln))
            elif k == 1:
                parts.append(rng.choice(acgt[:4], ln))
            else:
                parts.append(np.full(ln, rng.choice(np.frombuffer(b'nNRy-x*', np.uint8)),
                                     dtype=np.uint8))
        s = np.concatenate(parts).tobytes()
        return [('a', s[:len(s) // 3]), ('e', b''), ('b', s[len(s) // 3:])]
    raise ValueError(kind)


@pytest.mark.parametrize('kind', ['alternating_case', 'all_lower', 'mixed'])
def test_image_round_trip_case_patterns(kind):
    _assert_image_round_trip(_case_genome(kind, np.random.default_rng(41)))


def test_image_round_trip_every_byte_value():
    rng = np.random.default_rng(5)
    values = [b for b in range(256) if b not in (10, 13)]
    parts = []
    for k, b in enumerate(values * 3):
        parts.append(rng.choice(np.frombuffer(b'ACGTacgt', np.uint8), int(rng.integers(0, 40))))
        parts.append(np.full(1 + (k * 7) % 45, b, dtype=np.uint8))
    seq = np.concatenate(parts).tobytes()
    _assert_image_round_trip([('a', seq[:5000]), ('b', seq[5000:])])


@pytest.mark.parametrize('shape', ['empty', 'one_base', 'all_N', 'exc_at_ends'])
def test_image_round_trip_edge_genomes(shape):
    contigs = {
        'empty': [],
        'one_base': [('a', b'n')],
        'all_N': [('a', b'N' * 100_000), ('b', b'N' * 33)],
        'exc_at_ends': [('a', b'RACGTY'), ('b', b'YY' + b'acgt' * 40 + b'-'), ('c', b'')],
    }[shape]
    _assert_image_round_trip(contigs)


def test_image_round_trip_fasta_loaded():
    """A genome read and packed from FASTA text (magot_genome_load_fasta) replicates
    through its image like one packed from contigs."""
    w = synth.make('small', seed=4, genome_bases=300_000, n_tx=10, iupac_rate=1e-3)
    fg = engine.FastaGenome.load(w.fasta_text(width=61).encode('latin-1'))
    rep, n = _image_replica(fg)
    try:
        assert rep.export() == fg.export()
        assert np.array_equal(_defined(fg, _arena(fg)), _defined(rep, _arena(rep)))
    finally:
        rep.close()
        fg.close()


def test_image_replica_extracts_the_same_bytes():
    w = synth.make('small', seed=12, genome_bases=2_000_000, n_tx=800, iupac_rate=1e-3)
    g = engine.DeviceGenome(w.contigs())
    rep, n = _image_replica(g)
    try:
        assert n < 0.3 * g.device_bytes
        ex, tx = w.plan_tables()
        outs = []
        for gen in (g, rep):
            plan = engine.ExtractionPlan(gen, ex, tx)
            outs.append(plan.run())
            plan.close()
        for x, y in zip(outs[0], outs[1]):
            assert np.array_equal(x, y)
    finally:
        rep.close()
        g.close()


def test_image_refused_for_another_genome():
    a = engine.DeviceGenome([('a', b'ACGTacgtNN' * 1000)])
    b = engine.DeviceGenome([('a', b'ACGTacgtNN' * 1001)])
    try:
        meta_b, _ = b.export()
        n = a.wire_size()
        buf = torch.empty(n, dtype=torch.uint8, device='cuda')
        a.wire_export(buf.data_ptr(), n)
        with pytest.raises(engine.MagotError):
            engine.DeviceGenome.from_wire(meta_b, buf.data_ptr(), n, b.names, b.lengths)
        with pytest.raises(engine.MagotError):   # too small a buffer for the export
            a.wire_export(buf.data_ptr(), n - 1)
        meta_a, _ = a.export()
        with pytest.raises(engine.MagotError):   # the caller's contig table disagrees
            engine.DeviceGenome.from_wire(meta_a, buf.data_ptr(), n, ['a', 'b'], [10000, 5])
    finally:
        a.close()
        b.close()


@pytest.mark.slow
@pytest.mark.parametrize('config', ['C3', 'C5'])
def test_image_round_trip_full_size(config):
    """The images a C4 / C5 job broadcasts: 0.27 B per base of the arena's 1 B."""
    w = synth.make(config)
    arena, n = _assert_image_round_trip(w.contigs(), max_frac=0.3)
    print('%s: image %d bytes of a %d-byte arena (%.3f)' % (config, n, arena, n / arena))


@pytest.mark.parametrize('aligned', [False, True])
def test_copy_segments_vs_numpy(aligned):
    rng = np.random.default_rng(21 + aligned)
    n = 5000
    lens = rng.integers(0, 300, n)
    lens[rng.integers(0, n, 50)] = rng.integers(1000, 5000, 50)  # a few long segments
    if aligned:
        lens = (lens + 15) & ~15
    src_bytes = int(lens.sum()) + 3 * n + 64
    src = rng.integers(0, 256, src_bytes, dtype=np.uint8)
    perm = rng.permutation(n)
    # source places: a shuffled packing of the segments (aligned if asked)
    src_off = np.zeros(n, dtype=np.uint64)
    at = 0
    for i in perm:
        src_off[i] = at
        at += int(lens[i]) + (0 if aligned else int(rng.integers(0, 3)))
    assert at <= src_bytes
    dst_off = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(lens, out=dst_off[1:])
    want = np.concatenate([src[int(src_off[i]):int(src_off[i]) + int(lens[i])] for i in range(n)])
    d_src = torch.from_numpy(src).cuda()
    d_dst = torch.full((int(dst_off[-1]) + 64,), 0xEE, dtype=torch.uint8, device='cuda')
    torch.cuda.synchronize()
    engine.copy_segments(d_src.data_ptr(), src_bytes, d_dst.data_ptr(), src_off, dst_off)
    got = d_dst.cpu().numpy()
    assert np.array_equal(got[:int(dst_off[-1])], want)
    assert (got[int(dst_off[-1]):] == 0xEE).all()  # nothing written past the end
    # a segment reaching past the source is refused before any launch
    bad = src_off.copy()
    i = int(np.argmax(lens))
    bad[i] = src_bytes - int(lens[i]) + 1
    with pytest.raises(engine.MagotError):
        engine.copy_segments(d_src.data_ptr(), src_bytes, d_dst.data_ptr(), bad, dst_off)
