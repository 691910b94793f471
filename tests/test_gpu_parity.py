"""Parity of the HIP path (through the C ABI) with the reference goldens and the
CPU oracle.  Needs an MI355X: ``pytest -m gpu``."""

import contextlib
import hashlib
import io
import json
import os

import numpy as np
import pytest

import goldlib
from magot_amd import engine, synth
from magot_amd import genome as G
from oracle import magot_oracle as mo

pytestmark = pytest.mark.gpu


def _json(name):
    with open(os.path.join(goldlib.HERE, name)) as fh:
        return json.load(fh)


def _padded_end(soff, slen, j):
    """End of stream j's 16-byte padded span (its padding bytes are zero)."""
    return int(soff[j]) + ((int(slen[j]) + 15) & ~15)


def _sha(s):
    if isinstance(s, str):
        s = s.encode('latin-1')
    return hashlib.sha256(s).hexdigest()


@pytest.fixture(autouse=True, params=['auto', '6'])
def tile_size(request, monkeypatch):
    """Every test under both extraction tile sizes: 'auto' (test-size plans
    take the small 3-slot tile, full-size ones the large tile) and the large
    6-slot tile forced (magot_plan_create reads MAGOT_EXTRACT_LANE_CHUNKS)."""
    if request.param == 'auto':
        monkeypatch.delenv('MAGOT_EXTRACT_LANE_CHUNKS', raising=False)
    else:
        monkeypatch.setenv('MAGOT_EXTRACT_LANE_CHUNKS', request.param)
    return request.param


@pytest.fixture(scope='module', autouse=True)
def _device():
    from magot_amd import _lib
    if _lib.lib().magot_device_count() <= 0:
        pytest.fail('no HIP device visible for a gpu test')


# ---------------------------------------------------------------------------
# Sequence ops (genome.py:784-851) vs known-answer vectors from the reference
# ---------------------------------------------------------------------------

def test_revcomp_kat_batch():
    recs = _json('kat.json')
    got = engine.revcomp_batch([r['seq'] for r in recs])
    assert got == [r['revcomp'] for r in recs]


def test_translate_kat_batch():
    recs = _json('kat.json')
    seqs, frames, strands, want, trims = [], [], [], [], []
    for r in recs:
        for key, exp in r['translate'].items():
            if isinstance(exp, dict):
                continue
            seqs.append(r['seq'])
            frames.append(int(key[0]))
            strands.append(key[1])
            trims.append(bool(int(key[2])))
            want.append(exp)
    got = engine.translate_batch(seqs, frames, strands)
    for s, f, st, t, g, w in zip(seqs, frames, strands, trims, got, want):
        if g is not None and t and g[:1] == 'X':
            g = g[1:]
        assert g == w, (s, f, st, t)


def test_single_sequence_abi_kat():
    """magot_translate / magot_revcomp (single-sequence C entry points)
    against the reference's KATs: frames 0-4, both strands, trimX on/off,
    -1 where translate() returns None."""
    import ctypes
    from magot_amd import _lib
    L = _lib.lib()
    ctx = _lib.default_context()
    for r in _json('kat.json'):
        seq = r['seq'].encode('latin-1')
        buf = (ctypes.c_uint8 * max(len(seq), 1)).from_buffer_copy(seq or b'\0')
        out = (ctypes.c_uint8 * max(len(seq), 1))()
        _lib.check(L.magot_revcomp(ctx.handle, buf, len(seq), out), 'magot_revcomp')
        assert bytes(out)[:len(seq)].decode('latin-1') == r['revcomp']
        for key, want in r['translate'].items():
            if isinstance(want, dict):
                continue
            f, st, trim = int(key[0]), key[1], int(key[2])
            n = ctypes.c_int64()
            # out sized as the header states, (len + 2) / 3, plus guard bytes
            cap = (len(seq) + 2) // 3
            tout = (ctypes.c_uint8 * (cap + 8))(*([0xEE] * (cap + 8)))
            _lib.check(L.magot_translate(ctx.handle, buf, len(seq), f, ord(st), trim, tout,
                                         ctypes.byref(n)), 'magot_translate')
            got = None if n.value < 0 else bytes(tout)[:n.value].decode('latin-1')
            assert got == want, (r['seq'], key)
            assert n.value <= cap and bytes(tout)[max(n.value, 0):] == b'\xee' * (
                cap + 8 - max(n.value, 0)), (r['seq'], key)  # nothing past the result
    # frame 1 of a length with len % 3 == 2: (len + 1) / 3 residues before the trim
    for seq, f, trim, want in [(b'GATGA', 1, 0, 'X*'), (b'GATGA', 1, 1, '*'),
                               (b'GGATGAAAA', 2, 0, 'XE')]:
        cap = (len(seq) + 2) // 3
        tout = (ctypes.c_uint8 * (cap + 4))(*([0xEE] * (cap + 4)))
        n = ctypes.c_int64()
        _lib.check(L.magot_translate(ctx.handle, seq, len(seq), f, ord('+'), trim, tout,
                                     ctypes.byref(n)), 'magot_translate')
        assert bytes(tout)[:n.value].decode() == want and bytes(tout)[n.value:] == \
            b'\xee' * (cap + 4 - n.value)


def test_sequence_api_kat():
    S = G.Sequence('ATGGCCTTTAAACCCGGGTAG')
    assert S.translate() == 'MAFKPG*'
    assert S.translate(strand='-') == 'LPGFKGH'
    assert S.translate(frame=1) == 'GL*TRV'
    assert S.translate(frame=2, strand='-') == 'PGLKA'
    assert G.Sequence('NNNATGNNN').translate() == 'MX'
    assert G.Sequence('AT').translate() is None
    assert G.Sequence('ATGC').translate(frame=1) == ''
    assert G.Sequence('ACGTRYacgtn-*.').reverse_compliment() == 'nn-nacgtnnACGT'
    assert isinstance(S.reverse_compliment(), G.Sequence)
    for r in _json('kat.json')[:14]:
        for key, exp in r['orfs'].items():
            longest, atg = bool(int(key[0])), bool(int(key[1]))
            if isinstance(exp, dict):
                with pytest.raises(Exception) as ei:
                    G.Sequence(r['seq']).get_orfs(longest=longest, from_atg=atg)
                assert type(ei.value).__name__ == exp['exc']
            else:
                assert G.Sequence(r['seq']).get_orfs(longest=longest, from_atg=atg) == exp


def test_custom_library():
    lib = dict(G.Sequence._STANDARD)
    lib['ATG'] = 'Z'
    assert G.Sequence('ATGATG').translate(library=lib) == 'ZZ'


# ---------------------------------------------------------------------------
# get_fasta: edge cases, the reference's fixtures, its test-suite cksums
# ---------------------------------------------------------------------------

def test_edge_cases_gpu(capsys):
    for case in _json('edge_cases.json'):
        capsys.readouterr()
        res = exc = None
        try:
            g = G.Genome(case['fasta'])
            g.read_gff(case['gff'])
            res = g.annotations.get_fasta('gene', seq_type=case['seq_type'],
                                          longest=case['longest'], genomic=case['genomic'])
        except Exception as e:  # noqa: BLE001
            exc = type(e).__name__
        out = capsys.readouterr().out
        tag = (case['case'], case['seq_type'], case['longest'], case['genomic'])
        assert exc == case['exc'], tag
        assert res == case['result'], tag
        assert out == case['stdout'], tag


def test_get_seq_single_interval():
    g = G.Genome('>c1\nACGTACGTAAccggttNNRYacgtACGTAAATTTGGGCCC\n')
    g.read_gff('c1\tt\tgene\t1\t40\t.\t+\t.\tID=g\n'
               'c1\tt\tmRNA\t1\t40\t.\t+\t.\tID=t;Parent=g\n'
               'c1\tt\tCDS\t10\t20\t.\t-\t0\tID=c;Parent=t\n')
    s = g.annotations.CDS['c'].get_seq()
    assert s == 'nnNNaaccggT' and isinstance(s, G.Sequence)


@pytest.mark.parametrize('seq_type', ['nucleotide', 'protein'])
def test_get_fasta_children_from_two_genomes(seq_type):
    """A record whose children belong to annotation sets of two Genomes (CDS
    objects grafted from one set into another keep their own
    annotation_set, so get_seq reads their own genome, genome.py:603-608):
    one launch per genome, joined per record; against the oracle's object
    model built the same way."""
    fa1 = 'ACGTACGTAAccggttNNRYacgtACGTAAATTTGGGCCC'
    fa2 = {'c1': 'TTTTGGGGCCCCAAAATGATGATGCCCGGGAAATTT', 'c9': 'ATGCCCtagGGA'}
    g1 = G.Genome('>c1\n%s\n' % fa1)
    g1.read_gff('c1\tt\tgene\t1\t40\t.\t+\t.\tID=g\n'
                'c1\tt\tmRNA\t1\t40\t.\t+\t.\tID=t;Parent=g\n'
                'c1\tt\tCDS\t1\t6\t.\t+\t0\tID=a1;Parent=t\n'
                'c1\tt\tCDS\t10\t20\t.\t+\t0\tID=a2;Parent=t\n')
    g2 = G.Genome('>c1\n%s\n>c9\n%s\n' % (fa2['c1'], fa2['c9']))
    g2.read_gff('c1\tt\tgene\t1\t30\t.\t+\t.\tID=h\n'
                'c1\tt\tmRNA\t1\t30\t.\t+\t.\tID=u;Parent=h\n'
                'c1\tt\tCDS\t22\t27\t.\t+\t0\tID=b1;Parent=u\n'
                'c9\tt\tCDS\t1\t9\t.\t+\t0\tID=b2;Parent=u\n')
    s1 = g1.annotations
    for cid in ('b1', 'b2'):
        s1.CDS[cid] = g2.annotations.CDS[cid]
        s1.mRNA['t'].child_list.append(cid)
    got = s1.mRNA['t'].get_fasta(seq_type=seq_type)

    o1 = mo.OracleSet(mo.OracleGenome({'c1': fa1}))
    o2 = mo.OracleSet(mo.OracleGenome(fa2))
    kids = [('a1', 'c1', (1, 6), o1), ('a2', 'c1', (10, 20), o1), ('b1', 'c1', (22, 27), o2),
            ('b2', 'c9', (1, 9), o2)]
    for cid, sid, co, owner in kids:
        o1.CDS[cid] = mo.OBase(cid, sid, co, 'CDS', 't', '+', {}, owner)
    o1.mRNA = {'t': mo.OParent('t', 'c1', 'mRNA', [k[0] for k in kids], 'g', '+', o1, {})}
    want = mo.get_fasta(o1.mRNA['t'], o1, seq_type)
    assert got == want and want.count('\n') == 1


def _gff2fasta(fasta, gff, **kw):
    order = kw.pop('order', 'insertion')
    g = G.Genome(fasta)
    g.read_gff(gff)
    return g.annotations.get_fasta('gene', order=order, **kw) + '\n'


@pytest.mark.parametrize('key', ['obiroi/nucleotide/insertion', 'obiroi/protein/insertion',
                                 'obiroi/nucleotide/py2', 'obiroi/protein/py2',
                                 'obiroi/longest/insertion', 'obiroi/genomic/insertion'])
def test_obiroi_gpu(key):
    want = _json('fixtures.json')[key]
    _, kind, order = key.split('/')
    kw = {'order': order}
    if kind == 'protein':
        kw['seq_type'] = 'protein'
    if kind == 'longest':
        kw['longest'] = True
    if kind == 'genomic':
        kw['genomic'] = True
    buf = io.StringIO()
    try:
        with contextlib.redirect_stdout(buf):
            out = _gff2fasta(goldlib.path('O.biroi_refseqGenomeSubset.fasta'),
                             goldlib.path('O.biroi_NCBIrefseq_gff3Subset.gff'), **kw)
        exc = None
    except Exception as e:  # noqa: BLE001
        out, exc = None, type(e).__name__
    assert exc == want['exc']
    assert _sha(buf.getvalue()) == want['stdout_sha256']
    if out is not None:
        assert _sha(out) == want['sha256']
        crc, n = goldlib.posix_cksum(out)
        assert '%d %d' % (crc, n) == want['cksum']


@pytest.fixture(scope='module')
def c14_path(tmp_path_factory):
    p = tmp_path_factory.mktemp('c14') / 'C14.fasta'
    p.write_bytes(goldlib.rebuild_c14().encode('latin-1'))
    return str(p)


@pytest.mark.parametrize('ann', ['StandardGTF.gtf', 'transcriptlessGTF.gtf', 'minimalGFF3.gff'])
def test_c14_annotations_gpu(c14_path, ann):
    table = _json('fixtures.json')
    for seq_type in ('nucleotide', 'protein'):
        for order in ('insertion', 'py2'):
            out = _gff2fasta(c14_path, goldlib.path(ann), seq_type=seq_type, order=order)
            assert _sha(out) == table['c14/%s/%s/%s' % (ann, seq_type, order)]['sha256'], \
                (ann, seq_type, order)


def _cli(argv):
    from magot_amd import genome_tools

    class _Out(object):
        def __init__(self):
            self.buffer = io.BytesIO()

        def write(self, s):
            self.buffer.write(s.encode('latin-1'))

        def flush(self):
            pass

    out = _Out()
    with contextlib.redirect_stdout(out):
        genome_tools.main(argv)
    return out.buffer.getvalue()


def test_reference_test_suite_lines_12_13_14(c14_path):
    """test_data/test_suite.py:12-14 through the drop-in CLI, byte for byte."""
    data = _cli(['gff2fasta', c14_path, goldlib.path('StandardGTF.gtf')])
    assert goldlib.posix_cksum(data) == (2836090577, 690750)
    data = _cli(['gff2fasta', c14_path, goldlib.path('StandardGTF.gtf'), 'seq_type=protein'])
    assert goldlib.posix_cksum(data) == (111942461, 233762)
    data = _cli(['cds2pep', goldlib.path('CDSannotations.cds')])
    assert goldlib.posix_cksum(data) == (111942461, 233762)


@pytest.mark.parametrize('ann', ['StandardGTF.gtf', 'transcriptlessGTF.gtf', 'minimalGFF3.gff'])
@pytest.mark.parametrize('seq_type', ['nucleotide', 'protein'])
def test_cli_native_planner_equals_object_path(c14_path, ann, seq_type):
    """gff2fasta through the native planner (default) and through the Python
    object path (native=False) write identical bytes."""
    base = ['gff2fasta', c14_path, goldlib.path(ann), 'seq_type=' + seq_type]
    assert _cli(base) == _cli(base + ['native=False'])


def test_cli_native_planner_synthetic(tmp_path):
    w = synth.make('small', seed=31, genome_bases=2_000_000, n_tx=1000, iupac_rate=1e-3)
    fa, gf = tmp_path / 'g.fa', tmp_path / 'a.gff3'
    fa.write_text(w.fasta_text())
    gf.write_text(w.gff3_text())
    for seq_type in ('nucleotide', 'protein'):
        base = ['gff2fasta', str(fa), str(gf), 'seq_type=' + seq_type]
        native = _cli(base)
        assert native == _cli(base + ['native=False'])
        want = mo.gff2fasta(str(fa), str(gf), seq_type=seq_type, order='py2')
        assert native == want.encode('latin-1')


def test_synth_small_gpu():
    want = _json('synth_small.json')
    w = synth.make('small')
    fa = w.fasta_text()
    for fmt, text in (('gff3', w.gff3_text()), ('gtf', w.gtf_text())):
        for seq_type in ('nucleotide', 'protein'):
            out = _gff2fasta(fa, text, seq_type=seq_type)
            assert _sha(out) == want['%s/%s' % (fmt, seq_type)]['sha256'], (fmt, seq_type)


# ---------------------------------------------------------------------------
# Direct plan tables vs the C oracle (random shapes, ragged edges, full size)
# ---------------------------------------------------------------------------

def gpu_extract(w, outputs=engine.OUT_NUC | engine.OUT_PEP):
    dev = engine.DeviceGenome(w.contigs())
    ex, tx = w.plan_tables()
    plan = engine.ExtractionPlan(dev, ex, tx, outputs)
    nuc, noff, pep, poff = plan.run()
    plan.close()
    dev.close()
    return nuc, noff, pep, poff


def trimmed(pep, poff):
    """Apply trimX (drop one leading 'X' per record) to the untrimmed output."""
    starts = poff[:-1].astype(np.int64)
    lens = (poff[1:] - poff[:-1]).astype(np.int64)
    first = np.zeros(len(starts), dtype=bool)
    nonempty = lens > 0
    first[nonempty] = pep[starts[nonempty]] == ord('X')
    keep = np.ones(len(pep), dtype=bool)
    keep[starts[first]] = False
    lens -= first
    off = np.zeros(len(lens) + 1, dtype=np.int64)
    np.cumsum(lens, out=off[1:])
    return pep[keep], off


def check_against_oracle(w):
    from oracle import cds_oracle
    nuc, noff, pep, poff = gpu_extract(w)
    ref, roff, st = cds_oracle.extract_workload(w, False)
    assert not st.any()
    assert np.array_equal(noff.astype(np.int64), roff)
    if not np.array_equal(nuc, ref):
        bad = int(np.nonzero(nuc != ref)[0][0])
        t = int(np.searchsorted(roff, bad, side='right') - 1)
        raise AssertionError('nucleotide mismatch at byte %d (record %d): %r vs %r' % (
            bad, t, nuc[max(0, bad - 8):bad + 8].tobytes(), ref[max(0, bad - 8):bad + 8].tobytes()))
    pref, proff, pst = cds_oracle.extract_workload(w, True)
    got, goff = trimmed(pep, poff)
    ok = pst == 0
    assert np.array_equal(goff[1:][ok] - goff[:-1][ok], proff[1:][ok] - proff[:-1][ok])
    assert np.array_equal(got, pref)


@pytest.mark.parametrize('seed', [1, 2, 3])
def test_random_workloads_vs_c_oracle(seed):
    w = synth.make('small', seed=seed, genome_bases=3_000_000, n_tx=1500, iupac_rate=1e-3)
    check_against_oracle(w)


def test_tiny_exons_and_lds_overflow_vs_c_oracle():
    """1-12 base exons: many exons per 16-byte chunk and > 512 exons per tile
    (the kernel's global-memory search path)."""
    rng = np.random.default_rng(99)
    w = synth.make('small', seed=5, genome_bases=400_000, n_tx=400, iupac_rate=5e-3)
    w.ex_len = rng.integers(1, 13, size=w.n_exons).astype(np.int64)
    check_against_oracle(w)


def test_c2_full_size_nucleotide_only():
    """BASELINE configs[1] at its stated size: 100 Mb, 50k single-exon CDS."""
    from oracle import cds_oracle
    w = synth.make('C2')
    assert w.n_tx == 50_000 and int(w.contig_len.sum()) == 100_000_000
    nuc, noff, pep, poff = gpu_extract(w, engine.OUT_NUC)
    ref, roff, st = cds_oracle.extract_workload(w, False)
    assert pep is None
    assert np.array_equal(nuc, ref)


@pytest.mark.slow
def test_c3_full_size_vs_c_oracle():
    """The headline workload (1 Gb genome, 500k transcripts), byte for byte."""
    w = synth.make('C3')
    check_against_oracle(w)


@pytest.mark.slow
def test_c3_full_size_small_tiles_vs_c_oracle(monkeypatch, tile_size):
    """C3 at full size cut into the small 3-slot tiles (the size one GPU's
    share of the multi-GPU job takes), byte for byte."""
    if tile_size != 'auto':
        pytest.skip('one run is enough')
    monkeypatch.setenv('MAGOT_EXTRACT_LANE_CHUNKS', '3')
    w = synth.make('C3')
    check_against_oracle(w)


@pytest.mark.slow
def test_c5_full_size_six_frames_vs_c_oracle():
    """BASELINE configs[4] at its stated size (3 Gb genome, 2M transcripts):
    the fused gather + six-frame kernel, ALL six frames of ALL records against
    the C oracle's translate(frame, strand) (genome.py:795-851)."""
    from oracle import cds_oracle
    w = synth.make('C5')
    dev = engine.DeviceGenome(w.contigs())
    ex, tx = w.plan_tables()
    plan = engine.ExtractionPlan(dev, ex, tx, engine.OUT_NUC)
    o6 = engine.Orf6Plan(plan)
    o6.execute()
    out, soff, slen = o6.fetch()
    o6.close()
    plan.close()
    dev.close()
    ref, roff, st = cds_oracle.extract_workload(w, False)
    assert not st.any()
    threads = int(os.environ.get('OMP_NUM_THREADS', '0')) or min(16, os.cpu_count() or 1)
    assert cds_oracle.orf6_compare(ref, roff, out, soff, slen, threads=threads) == (0, -1)


@pytest.mark.parametrize('seed', [7, 8])
def test_huge_exons_vs_c_oracle(seed):
    """Records far larger than a tile: 15 % of the exons 20-300 kb (clamped at
    the contig ends as Python slices are), so one record spans dozens of
    extraction tiles and orf6 windows, its peptide and six streams continue
    across every tile boundary; extraction and all six frames against the C
    oracle."""
    from oracle import cds_oracle
    rng = np.random.default_rng(seed)
    w = synth.make('small', seed=seed, genome_bases=3_000_000, n_tx=150, iupac_rate=1e-3)
    big = rng.random(w.n_exons) < 0.15
    w.ex_len = np.where(big, rng.integers(20_000, 300_000, size=w.n_exons), w.ex_len)
    check_against_oracle(w)
    dev = engine.DeviceGenome(w.contigs())
    ex, tx = w.plan_tables()
    plan = engine.ExtractionPlan(dev, ex, tx, engine.OUT_NUC)
    o6 = engine.Orf6Plan(plan)
    o6.execute()
    out, soff, slen = o6.fetch()
    o6.close()
    plan.close()
    dev.close()
    ref, roff, st = cds_oracle.extract_workload(w, False)
    assert not st.any() and int(roff[-1]) > 10 * 5072
    assert cds_oracle.orf6_compare(ref, roff, out, soff, slen, threads=4) == (0, -1)


@pytest.mark.parametrize('paths', ['1', '2', '3'])
def test_forced_general_paths_vs_c_oracle(monkeypatch, paths):
    """MAGOT_DEBUG_PATHS routes every chunk (1), every residue chunk (2) or
    both (3) through the general per-segment / per-residue code."""
    monkeypatch.setenv('MAGOT_DEBUG_PATHS', paths)
    w = synth.make('small', seed=11, genome_bases=2_000_000, n_tx=800, iupac_rate=1e-3)
    check_against_oracle(w)


def test_sorted_record_order_vs_c_oracle():
    w = synth.make('small', seed=12, genome_bases=3_000_000, n_tx=1500, iupac_rate=1e-3,
                   order='sorted')
    check_against_oracle(w)


def _recase(w, rng, lo, hi):
    """Soft-mask runs of U[lo, hi] bases (alternating case) over the plain
    bases of w's genome; exception bytes are left as they are."""
    g = w.genome
    n = len(g)
    runs = rng.integers(lo, hi + 1, size=n // lo + 2)
    ends = np.cumsum(runs)
    lower = np.zeros(n, dtype=bool)
    lower_run = np.searchsorted(ends, np.arange(n), side='right') & 1
    lower[:] = lower_run.astype(bool)
    plain = np.isin(g, np.frombuffer(b'ACGTacgt', dtype=np.uint8))
    up = g & 0xDF
    w.genome = np.where(plain, np.where(lower, up | 0x20, up), g).astype(np.uint8)
    return w


@pytest.mark.parametrize('runs', [(1, 40), (10, 30), (150, 600)])
def test_dense_soft_mask_runs_vs_c_oracle(runs):
    """Soft-mask runs of 1-600 bases (case changes inside chunks, at chunk
    edges and across interval joins), intervals of 1-400 bases, both
    strands, N runs and IUPAC bytes."""
    rng = np.random.default_rng(runs[0] * 7 + runs[1])
    w = synth.make('small', seed=21, genome_bases=2_000_000, n_tx=900, iupac_rate=2e-3)
    w.ex_len = rng.integers(1, 401, size=w.n_exons).astype(np.int64)
    check_against_oracle(_recase(w, rng, *runs))


def test_degenerate_intervals_vs_c_oracle():
    """Zero-length intervals, records shorter than one codon, 1-2 base
    exons mixed with long ones, and intervals clamped at contig ends."""
    rng = np.random.default_rng(13)
    w = synth.make('small', seed=13, genome_bases=1_000_000, n_tx=600, iupac_rate=2e-3)
    n = w.n_exons
    pick = rng.random(n)
    w.ex_len = np.where(pick < 0.08, 0, np.where(pick < 0.16, rng.integers(1, 3, size=n),
                                                  w.ex_len)).astype(np.int64)
    # last interval of the first 20 records runs past its contig end (slice clamp)
    last = np.cumsum(w.ex_count)[:20] - 1
    clen = w.contig_len[w.tx_contig[:20]]
    w.ex_start = w.ex_start.copy()
    w.ex_start[last] = np.maximum(clen - 3, w.ex_start[last])
    w.ex_len[last] = 10
    check_against_oracle(w)


@pytest.mark.parametrize('shape', ['no_records', 'all_empty', 'one_base_each'])
def test_empty_and_tiny_plans(shape):
    """Plans with no record, with records whose intervals are all empty, and
    with one-base records: extraction, translation and the six-frame plan
    return empty or exact outputs without launching out of range."""
    w = synth.make('small', seed=3, genome_bases=200_000, n_tx=50)
    dev = engine.DeviceGenome(w.contigs())
    ex, tx = w.plan_tables()
    if shape == 'no_records':
        ex, tx = ex[:0], tx[:0]
    elif shape == 'all_empty':
        ex['len'] = 0
    else:
        ex['len'] = np.minimum(ex['len'], 1)
        tx['n_exons'] = np.minimum(tx['n_exons'], 1)
        ex = ex[tx['exon_begin'].astype(np.int64)]
        tx['exon_begin'] = np.arange(len(tx))
    plan = engine.ExtractionPlan(dev, ex, tx, engine.OUT_NUC | engine.OUT_PEP)
    nuc, noff, pep, poff = plan.run()
    lens = ex['len'].astype(np.int64)
    assert len(noff) == len(tx) + 1 and int(noff[-1]) == int(lens.sum())
    assert int(poff[-1]) == 0  # no record reaches one codon
    if shape == 'one_base_each':
        seqs = [s for _, s in w.contigs()]
        for r in range(len(tx)):
            st = int(ex['start_rc'][r]) & ((1 << 63) - 1)
            b = seqs[int(ex['contig'][r])][st:st + int(ex['len'][r])]
            if int(ex['start_rc'][r]) >> 63:
                b = mo_revcomp(b)
            assert nuc[int(noff[r]):int(noff[r + 1])].tobytes() == b
    o6 = engine.Orf6Plan(plan)
    o6.execute()
    out, soff, slen = o6.fetch()
    assert len(soff) == 6 * len(tx) + 1 and not slen.any()
    o6.close()
    plan.close()
    dev.close()


def mo_revcomp(b):
    from oracle import magot_oracle as mo
    return mo.reverse_complement(b.decode('latin-1')).encode('latin-1')


# ---------------------------------------------------------------------------
# Six-frame translation (Sequence.get_orfs, genome.py:824-851): orf6_kernel
# ---------------------------------------------------------------------------

def _oracle_six(s):
    return [mo.translate(s, frame=f, strand=st) for f in (0, 1, 2) for st in ('-', '+')]


def test_orf6_batch_vs_oracle():
    rng = np.random.default_rng(41)
    alphabet = np.frombuffer(b'ACGTACGTACGTacgtNnRY-*', dtype=np.uint8)
    seqs = []
    for L in list(range(0, 24)) + [int(x) for x in rng.integers(24, 3000, size=300)]:
        seqs.append(alphabet[rng.integers(0, len(alphabet), size=L)].tobytes().decode('latin-1'))
    got = engine.orf6_batch(seqs)
    for s, six in zip(seqs, got):
        assert six == _oracle_six(s), s[:40]


def test_orf6_batch_tile_shapes_vs_oracle():
    """Tile edge cases of the input-stationary kernel: hundreds of tiny
    records in one tile (several record batches), records longer than a tile
    (chunks owned by different tiles, both strands), and a record ending
    exactly at the end of the batch."""
    rng = np.random.default_rng(47)
    alphabet = np.frombuffer(b'ACGTACGTACGTacgtNnRY', dtype=np.uint8)
    lens = [int(x) for x in rng.integers(0, 12, size=900)]
    lens += [3968, 3967, 3969, 7936, 12_345, 20_001] + [int(x) for x in rng.integers(0, 9000, 40)]
    lens += [int(x) for x in rng.integers(0, 7, size=500)]
    seqs = [alphabet[rng.integers(0, len(alphabet), size=L)].tobytes().decode('latin-1')
            for L in lens]
    got = engine.orf6_batch(seqs)
    for i, (s, six) in enumerate(zip(seqs, got)):
        assert six == _oracle_six(s), (i, len(s))


@pytest.mark.parametrize('walk', ['genome', 'record'])
def test_orf6_over_extraction_plan_vs_oracle(monkeypatch, walk):
    """C5 shape at small size: gather + six-frame translation, all in HBM;
    the kernel's walk in genome order (default) and in record order
    (MAGOT_ORF6_ORDER=record)."""
    if walk == 'record':
        monkeypatch.setenv('MAGOT_ORF6_ORDER', 'record')
    else:
        monkeypatch.delenv('MAGOT_ORF6_ORDER', raising=False)
    w = synth.make('small', seed=43, genome_bases=1_000_000, n_tx=400, iupac_rate=2e-3)
    dev = engine.DeviceGenome(w.contigs())
    ex, tx = w.plan_tables()
    plan = engine.ExtractionPlan(dev, ex, tx, engine.OUT_NUC)
    nuc, noff, _, _ = plan.run()
    o6 = engine.Orf6Plan(plan)
    o6.execute()
    out, soff, slen = o6.fetch()
    # the plan's layout: each record's six streams one 16-byte aligned block,
    # the blocks tiling [0, total) (in walk order by default, record order
    # under MAGOT_ORF6_ORDER=record)
    from magot_amd import shard
    st, ln = shard.six_frame_blocks(soff, slen)
    order = np.argsort(st, kind='stable')
    assert (st % 16 == 0).all() and int(soff[-1]) == o6.total
    assert np.array_equal(np.cumsum(ln[order])[:-1], st[order][1:]) and st[order][0] == 0
    assert int(st[order][-1] + ln[order][-1]) == o6.total
    if walk == 'record':
        ref_soff, _ = engine.orf6_sizes(noff)
        assert np.array_equal(soff, ref_soff)
    raw = out.tobytes().decode('latin-1')
    for r in range(len(tx)):
        s = nuc[int(noff[r]):int(noff[r + 1])].tobytes().decode('latin-1')
        want = _oracle_six(s)
        for k in range(6):
            j = 6 * r + k
            assert int(soff[j]) % 16 == 0
            assert not out[int(soff[j] + slen[j]):_padded_end(soff, slen, j)].any()  # zero padding
            t = raw[int(soff[j]):int(soff[j] + slen[j])]
            if k < 2 and t[:1] == 'X':
                t = t[1:]
            if want[k] is None:
                assert t == ''
            else:
                assert t == want[k], (r, k)
    o6.close()
    plan.close()
    dev.close()


def test_orf6_flag_in_upper_lanes_vs_oracle():
    """Windows whose only exception-flagged interval is staged by lanes 32-63
    (or 96-127): the wave-wide test of the flags once dropped those lanes and
    decoded the N runs as 'A' (found by the full-size C5 check)."""
    from oracle import cds_oracle
    from test_orf6_plan import orf6_windows, upper_lane_workload, upper_only
    w = upper_lane_workload()
    assert upper_only(orf6_windows(w)) >= 20
    dev = engine.DeviceGenome(w.contigs())
    ex, tx = w.plan_tables()
    plan = engine.ExtractionPlan(dev, ex, tx, engine.OUT_NUC)
    o6 = engine.Orf6Plan(plan)
    o6.execute()
    out, soff, slen = o6.fetch()
    ref, roff, st = cds_oracle.extract_workload(w, False)
    assert not st.any()
    assert cds_oracle.orf6_compare(ref, roff, out, soff, slen, threads=4) == (0, -1)
    o6.close()
    plan.close()
    dev.close()


def test_orf6_fused_gather_tiny_intervals_vs_oracle():
    """The fused gather over 1-6 base intervals on both strands (many
    intervals per 16-base vector, windows shortened to the interval cap) and
    long records spanning several tiles."""
    rng = np.random.default_rng(53)
    w = synth.make('small', seed=53, genome_bases=300_000, n_tx=10, iupac_rate=5e-3)
    dev = engine.DeviceGenome(w.contigs())
    lens = [len(s) for _, s in w.contigs()]
    rows, txs = [], []
    for t in range(700):
        n = int(rng.integers(1, 40)) if t % 50 else 3000  # a few records of ~10 kb
        b = len(rows)
        for _ in range(n):
            c = int(rng.integers(0, len(lens)))
            ln = int(rng.integers(0, 7)) if t % 3 else int(rng.integers(1, 9))
            st = int(rng.integers(0, lens[c] - ln))
            rows.append(((st | (1 << 63)) if rng.integers(0, 2) else st, c, ln))
        txs.append((b, n, 0))
    ex = np.array(rows, dtype=engine.EXON_DTYPE)
    tx = np.array(txs, dtype=engine.TX_DTYPE)
    plan = engine.ExtractionPlan(dev, ex, tx, engine.OUT_NUC)
    nuc, noff, _, _ = plan.run()
    o6 = engine.Orf6Plan(plan)
    o6.execute()
    out, soff, slen = o6.fetch()
    raw = out.tobytes().decode('latin-1')
    for r in range(len(tx)):
        s = nuc[int(noff[r]):int(noff[r + 1])].tobytes().decode('latin-1')
        want = _oracle_six(s)
        for k in range(6):
            j = 6 * r + k
            assert not out[int(soff[j] + slen[j]):_padded_end(soff, slen, j)].any()
            t = raw[int(soff[j]):int(soff[j] + slen[j])]
            if k < 2 and t[:1] == 'X':
                t = t[1:]
            assert t == (want[k] or ''), (r, k)
    o6.close()
    plan.close()
    dev.close()


def test_orf6_intervals_at_plane_edges_vs_oracle():
    """Six frames of records whose intervals touch the first and last bases of
    the genome plane on both strands ('-' intervals are read backwards from
    the forward planes, so their windows run to the plane's two ends), with
    exceptions right at the edges; single- and multi-interval records."""
    rng = np.random.default_rng(77)
    acgt = np.frombuffer(b'ACGTacgt', np.uint8)
    first = b'NR' + rng.choice(acgt, 500).tobytes() + b'YN'
    mid = rng.choice(acgt, 3000).tobytes()
    last = rng.choice(acgt, 700).tobytes() + b'KMn'
    contigs = [('a', first), ('b', mid), ('c', last)]
    text = [c.decode('latin-1') for _, c in contigs]
    dev = engine.DeviceGenome(contigs)
    rows, txs, want = [], [], []
    for t in range(300):
        n = 1 + t % 4
        minus = bool(t % 2)
        b = len(rows)
        segs = []
        for k in range(n):
            c = 0 if (t + k) % 3 == 0 else 2
            L = len(contigs[c][1])
            ln = int(rng.integers(1, 60)) if t % 5 else int(rng.integers(100, L))
            st = 0 if (t // 2) % 2 == 0 else L - ln  # at the contig's first / last base
            rows.append(((st | (1 << 63)) if minus else st, c, ln))
            seg = text[c][st:st + ln]
            segs.append(mo.reverse_complement(seg) if minus else seg)
        txs.append((b, n, 0))
        want.append(''.join(segs))
    ex = np.array(rows, dtype=engine.EXON_DTYPE)
    tx = np.array(txs, dtype=engine.TX_DTYPE)
    plan = engine.ExtractionPlan(dev, ex, tx, engine.OUT_NUC)
    nuc, noff, _, _ = plan.run()
    for r, s in enumerate(want):
        assert nuc[int(noff[r]):int(noff[r + 1])].tobytes().decode('latin-1') == s, r
    o6 = engine.Orf6Plan(plan)
    o6.execute()
    out, soff, slen = o6.fetch()
    raw = out.tobytes().decode('latin-1')
    for r, s in enumerate(want):
        six = _oracle_six(s)
        for k in range(6):
            j = 6 * r + k
            got = raw[int(soff[j]):int(soff[j] + slen[j])]
            if k < 2 and got[:1] == 'X':
                got = got[1:]
            assert got == (six[k] or ''), (r, k, s)
    o6.close()
    plan.close()
    dev.close()


def test_every_byte_class_both_strands_vs_oracle():
    """Every printable byte GenomeSequence keeps (genome.py:875) inside CDS
    intervals on both strands: the literal classes the kernels decode from
    the nibble (N n - R Y K M; forward strand) and the run-list path (every
    other byte; reverse strand maps all of them to n N -)."""
    rng = np.random.default_rng(71)
    printable = bytes(range(33, 127)) + b' '
    contig = bytearray(rng.choice(np.frombuffer(b'ACGTacgt', np.uint8), 60_000).tobytes())
    for k in range(0, 60_000, 400):  # a run of one byte class every 400 bases
        b = printable[(k // 400) % len(printable)]
        contig[k:k + 1 + (k // 400) % 37] = bytes([b]) * (1 + (k // 400) % 37)
    contig = bytes(contig)
    dev = engine.DeviceGenome([('c0', contig)])
    rows, txs = [], []
    for t in range(600):
        n = int(rng.integers(1, 6))
        b = len(rows)
        minus = bool(rng.integers(0, 2))
        for _ in range(n):
            ln = int(rng.integers(1, 300))
            st = int(rng.integers(0, len(contig) - ln))
            rows.append(((st | (1 << 63)) if minus else st, 0, ln))
        txs.append((b, n, 0))
    ex = np.array(rows, dtype=engine.EXON_DTYPE)
    tx = np.array(txs, dtype=engine.TX_DTYPE)
    plan = engine.ExtractionPlan(dev, ex, tx)
    nuc, noff, pep, poff = plan.run()
    text = contig.decode('latin-1')
    for r, (b, n, _) in enumerate(txs):
        segs = []
        for sr, _c, ln in rows[b:b + n]:
            st = sr & ~(1 << 63)
            s = text[st:st + ln]
            segs.append(mo.reverse_complement(s) if sr >> 63 else s)
        want = ''.join(segs)
        assert nuc[int(noff[r]):int(noff[r + 1])].tobytes().decode('latin-1') == want, r
        got = pep[int(poff[r]):int(poff[r + 1])].tobytes().decode('latin-1')
        assert got == (mo.translate(want, trimX=False) or ''), r
    plan.close()
    dev.close()


@pytest.mark.parametrize('max_len', [20, 70, 400])
def test_reverse_forward_segments_vs_oracle(max_len):
    """extract_kernel's reverse-forward path (v19): '-' intervals without
    exceptions read the forward plane descending and are reverse-complemented
    in registers; '-' intervals over N runs or IUPAC bytes read the mirror;
    chunks whose two segments differ in strand or in path take the mirror for
    their '-' segment.  Per-interval random strands inside records, short
    intervals (two- and three-segment chunks), soft-masked runs, contig
    starts and ends, several contigs."""
    rng = np.random.default_rng(max_len)
    contigs = []
    for k, n in enumerate((30_000, 777, 45_001, 64)):
        b = rng.choice(np.frombuffer(b'ACGTacgt', np.uint8), n)
        for j in range(0, n, 900):  # sparse N runs and IUPAC bytes
            if rng.random() < 0.3:
                b[j:j + int(rng.integers(1, 40))] = ord('N')
            if rng.random() < 0.2:
                b[min(j + 300, n - 1)] = rng.choice(np.frombuffer(b'RYKMSWn-', np.uint8))
        contigs.append(('c%d' % k, b.tobytes()))
    dev = engine.DeviceGenome(contigs)
    rows, txs = [], []
    for t in range(900):
        ci = int(rng.integers(0, len(contigs)))
        clen = len(contigs[ci][1])
        n = int(rng.integers(1, 9))
        b = len(rows)
        for _ in range(n):
            ln = int(rng.integers(1, min(max_len, clen) + 1))
            u = rng.random()
            st = 0 if u < 0.05 else clen - ln if u < 0.1 else int(rng.integers(0, clen - ln + 1))
            minus = bool(rng.integers(0, 2))
            rows.append(((st | (1 << 63)) if minus else st, ci, ln))
        txs.append((b, n, 0))
    ex = np.array(rows, dtype=engine.EXON_DTYPE)
    tx = np.array(txs, dtype=engine.TX_DTYPE)
    plan = engine.ExtractionPlan(dev, ex, tx)
    nuc, noff, pep, poff = plan.run()
    for r, (b, n, _) in enumerate(txs):
        segs = []
        for sr, ci, ln in rows[b:b + n]:
            st = sr & ~(1 << 63)
            s = contigs[ci][1][st:st + ln].decode('latin-1')
            segs.append(mo.reverse_complement(s) if sr >> 63 else s)
        want = ''.join(segs)
        assert nuc[int(noff[r]):int(noff[r + 1])].tobytes().decode('latin-1') == want, r
        got = pep[int(poff[r]):int(poff[r + 1])].tobytes().decode('latin-1')
        assert got == (mo.translate(want, trimX=False) or ''), r
    plan.close()
    dev.close()


def test_orf6_fused_code_plane_boundaries_vs_oracle():
    """The fused gather's 2-bit fast path at its edges: intervals of 14-20
    bases put the second (and third) interval exactly at the 16th-18th
    position of a vector, on both strands, over a genome dense in IUPAC
    bytes and N runs (the exception plane and the per-interval flags), plus
    long intervals that cross many vectors."""
    rng = np.random.default_rng(61)
    w = synth.make('small', seed=61, genome_bases=400_000, n_tx=10, iupac_rate=2e-2)
    dev = engine.DeviceGenome(w.contigs())
    lens = [len(s) for _, s in w.contigs()]
    rows, txs = [], []
    for t in range(900):
        n = int(rng.integers(1, 14))
        b = len(rows)
        for _ in range(n):
            c = int(rng.integers(0, len(lens)))
            ln = int(rng.integers(14, 21)) if t % 4 else int(rng.integers(40, 400))
            st = int(rng.integers(0, lens[c] - ln))
            rows.append(((st | (1 << 63)) if rng.integers(0, 2) else st, c, ln))
        txs.append((b, n, 0))
    ex = np.array(rows, dtype=engine.EXON_DTYPE)
    tx = np.array(txs, dtype=engine.TX_DTYPE)
    plan = engine.ExtractionPlan(dev, ex, tx, engine.OUT_NUC)
    nuc, noff, _, _ = plan.run()
    contigs = [s for _, s in w.contigs()]
    for r, (b, n, _) in enumerate(txs):  # the records, gathered in Python (genome.py:603-614)
        segs = []
        for sr, c, ln in rows[b:b + n]:
            s = contigs[c][sr & ~(1 << 63):(sr & ~(1 << 63)) + ln].decode('latin-1')
            segs.append(mo.reverse_complement(s) if sr >> 63 else s)
        assert nuc[int(noff[r]):int(noff[r + 1])].tobytes().decode('latin-1') == ''.join(segs)
    o6 = engine.Orf6Plan(plan)
    o6.execute()
    out, soff, slen = o6.fetch()
    raw = out.tobytes().decode('latin-1')
    for r in range(len(tx)):
        s = nuc[int(noff[r]):int(noff[r + 1])].tobytes().decode('latin-1')
        want = _oracle_six(s)
        for k in range(6):
            j = 6 * r + k
            t = raw[int(soff[j]):int(soff[j] + slen[j])]
            if k < 2 and t[:1] == 'X':
                t = t[1:]
            assert t == (want[k] or ''), (r, k)
    o6.close()
    plan.close()
    dev.close()


# ---------------------------------------------------------------------------
# FASTA text assembly on device (magot_fasta_text_*)
# ---------------------------------------------------------------------------

def _device_text(fasta, gff, seq_type, order='py2'):
    gs = G.GenomeSequence(fasta)
    names = list(gs)
    dev = engine.DeviceGenome([(n, gs[n]) for n in names])
    plan = engine.GffPlan.build(G.ensure_file(gff).read(), names, [len(gs[n]) for n in names],
                                protein=seq_type == 'protein', order=order)
    assert plan is not None
    ex = engine.ExtractionPlan(dev, plan.exons, plan.txs,
                               engine.OUT_PEP if seq_type == 'protein' else engine.OUT_NUC)
    text = engine.FastaText(plan, ex)
    ex.execute()
    text.execute()
    got = text.fetch().tobytes()
    text.execute()  # idempotent re-run on the same buffers
    again = text.fetch().tobytes()
    host = plan.render(*ex.fetch())
    assert text.time(2) > 0
    text.close()
    ex.close()
    plan.close()
    assert got == again
    return got, host


@pytest.mark.parametrize('seq_type', ['nucleotide', 'protein'])
def test_device_text_assembly_vs_oracle(seq_type):
    """Blank gene records, renamed IDs, X-trimmed peptides, minus strands."""
    fasta = ('>c1\n' + 'NNNACGTTGCAACGGATCCATGNNNAAA' * 40 + '\n>c2\n' +
             'GGGAAATTTCCCRYACGT' * 30 + '\n')
    rows = []
    for g in range(30):
        c = 'c1' if g % 3 else 'c2'
        lo = 1 + 17 * g
        rows.append('%s\tx\tgene\t%d\t%d\t.\t+\t.\tID=g%d' % (c, lo, lo + 200, g))
        if g % 4 == 1:
            continue  # gene without CDS: a blank record
        s = '+-'[g % 2]
        rows.append('%s\tx\tmRNA\t%d\t%d\t.\t%s\t.\tID=m%d;Parent=g%d' % (c, lo, lo + 200, s, g, g))
        for k in range(1 + g % 3):
            rows.append('%s\tx\tCDS\t%d\t%d\t.\t%s\t0\tID=cds%d;Parent=m%d'
                        % (c, lo + 40 * k, lo + 40 * k + 30, s, g, g))
    gff = '\n'.join(rows) + '\n'
    got, host = _device_text(fasta, gff, seq_type)
    assert got == host
    want = mo.gff2fasta(fasta, gff, seq_type=seq_type, order='py2')  # with the CLI's '\n'
    assert got + b'\n' == want.encode('latin-1')
    if seq_type == 'protein':
        assert b'\n>' in got


def test_device_text_assembly_obiroi():
    got, host = _device_text(goldlib.path('O.biroi_refseqGenomeSubset.fasta'),
                             goldlib.path('O.biroi_NCBIrefseq_gff3Subset.gff'), 'protein')
    assert got == host
    want = _json('fixtures.json')['obiroi/protein/py2']
    assert _sha(got + b'\n') == want['sha256']  # fixture: get_fasta + '\n'


@pytest.mark.parametrize('seq_type', ['nucleotide', 'protein'])
def test_device_text_assembly_tiny_units(seq_type):
    """Many units per 16-byte chunk and per 16-unit group: CDS of 1-40 bases,
    blank genes, long IDs, both strands -- every partial-chunk and group-edge
    case of text_copy_kernel against the host render and the oracle.  (Protein
    CDS keep 3+ bases: shorter records take the reference's None path, which
    the native planner hands to the object path.)"""
    rng = np.random.default_rng(11)
    lo_len = 0 if seq_type == 'nucleotide' else 2
    fasta = '>c1\n' + ''.join(rng.choice(list('ACGTacgtN'), 20000)) + '\n'
    rows = []
    for g in range(700):
        lo = 1 + int(rng.integers(0, 19000))
        gid = 'g%d' % g + ('x' * int(rng.integers(0, 40)) if g % 5 == 0 else '')
        rows.append('c1\tx\tgene\t%d\t%d\t.\t+\t.\tID=%s' % (lo, lo + 900, gid))
        if g % 3 == 0:
            continue  # blank record
        s = '+-'[int(rng.integers(0, 2))]
        rows.append('c1\tx\tmRNA\t%d\t%d\t.\t%s\t.\tID=m%d;Parent=%s' % (lo, lo + 900, s, g, gid))
        for k in range(1 + int(rng.integers(0, 3))):
            a = lo + 60 * k
            rows.append('c1\tx\tCDS\t%d\t%d\t.\t%s\t0\tID=cds%d_%d;Parent=m%d'
                        % (a, a + int(rng.integers(lo_len, 40)), s, g, k, g))
    gff = '\n'.join(rows) + '\n'
    got, host = _device_text(fasta, gff, seq_type)
    assert got == host
    want = mo.gff2fasta(fasta, gff, seq_type=seq_type, order='py2')
    assert got + b'\n' == want.encode('latin-1')
