"""Native gff2fasta planner (magot_gff_plan, csrc/gffplan.cpp) on CPU.

The planner is host code: it parses the GFF with read_gff's rules, orders the
gene records and lowers get_fasta to interval / record tables plus a text
skeleton.  Here the record payloads are computed from those tables by the
oracle (never by the product), and the rendered text must equal the oracle's
gff2fasta output byte for byte (and hence the reference's goldens).  Inputs
that take a reference diagnostic path must be declined (None) so that the
object path, which reproduces the diagnostics, runs instead.
"""

import numpy as np
import pytest

import goldlib
from magot_amd import engine, synth
from magot_amd import genome as G
from oracle import magot_oracle as mo


def _payloads(plan, seqs):
    """Record bytes for the plan's tables (oracle; untrimmed peptides)."""
    nuc, pep, noff, poff = [], [], [0], [0]
    ex, tx = plan.exons, plan.txs
    for t in range(len(tx)):
        b, n = int(tx['exon_begin'][t]), int(tx['n_exons'][t])
        parts = []
        for e in range(b, b + n):
            st = int(ex['start_rc'][e])
            rc = bool(st >> 63)
            st &= (1 << 63) - 1
            s = seqs[int(ex['contig'][e])][st:st + int(ex['len'][e])]
            parts.append(mo.reverse_complement(s) if rc else s)
        s = ''.join(parts)
        nuc.append(s)
        noff.append(noff[-1] + len(s))
        p = mo.translate(s, trimX=False) if len(s) > 2 else ''
        pep.append(p)
        poff.append(poff[-1] + len(p))
    enc = lambda parts: np.frombuffer((''.join(parts) + ' ').encode('latin-1'), np.uint8)
    return enc(nuc), np.array(noff, np.uint64), enc(pep), np.array(poff, np.uint64)


def native_gff2fasta(fasta, gff, seq_type='nucleotide', order='insertion', longest=False,
                     genomic=False, from_exons=False):
    gs = G.GenomeSequence(fasta)
    names = list(gs)
    plan = engine.GffPlan.build(G.ensure_file(gff).read(), names, [len(gs[n]) for n in names],
                                protein=seq_type == 'protein', order=order, longest=longest,
                                genomic=genomic, from_exons=from_exons)
    if plan is None:
        return None
    text = plan.render(*_payloads(plan, [gs[n] for n in names]))
    plan.close()
    return text.decode('latin-1') + '\n'


CASES = [
    ('obiroi', 'O.biroi_refseqGenomeSubset.fasta', 'O.biroi_NCBIrefseq_gff3Subset.gff'),
    ('c14-gtf', None, 'StandardGTF.gtf'),
    ('c14-transcriptless', None, 'transcriptlessGTF.gtf'),
    ('c14-minimal-gff3', None, 'minimalGFF3.gff'),
]


@pytest.fixture(scope='module')
def c14():
    return goldlib.rebuild_c14()


@pytest.mark.parametrize('name,fa,gff', CASES)
@pytest.mark.parametrize('seq_type', ['nucleotide', 'protein'])
@pytest.mark.parametrize('order', ['insertion', 'py2'])
def test_native_plan_matches_oracle(c14, name, fa, gff, seq_type, order):
    fasta = c14 if fa is None else goldlib.path(fa)
    got = native_gff2fasta(fasta, goldlib.path(gff), seq_type, order)
    if got is None:
        # declined: the reference takes a diagnostic path on this input
        out = []
        try:
            mo.gff2fasta(fasta, goldlib.path(gff), seq_type=seq_type, order=order, out=out)
            diag = bool(out)
        except Exception:
            diag = True
        assert diag, 'native planner declined an input without diagnostics'
        return
    want = mo.gff2fasta(fasta, goldlib.path(gff), seq_type=seq_type, order=order)
    assert got == want


def test_native_plan_reproduces_test_suite_goldens(c14):
    """test_data/test_suite.py:12-13 cksums through the native planner."""
    nuc = native_gff2fasta(c14, goldlib.path('StandardGTF.gtf'), 'nucleotide', 'py2')
    pep = native_gff2fasta(c14, goldlib.path('StandardGTF.gtf'), 'protein', 'py2')
    assert goldlib.posix_cksum(nuc.encode('latin-1')) == (2836090577, 690750)
    assert goldlib.posix_cksum(pep.encode('latin-1')) == (111942461, 233762)


@pytest.mark.parametrize('fmt', ['gff3', 'gff3-ncbi', 'gtf'])
def test_native_plan_synthetic(fmt):
    w = synth.make('small', seed=21, genome_bases=400_000, n_tx=300, iupac_rate=1e-3)
    fasta = w.fasta_text()
    gff = {'gff3': w.gff3_text, 'gff3-ncbi': lambda: w.gff3_text(ids='ncbi'),
           'gtf': w.gtf_text}[fmt]()
    for seq_type in ('nucleotide', 'protein'):
        got = native_gff2fasta(fasta, gff, seq_type, 'py2')
        assert got is not None
        assert got == mo.gff2fasta(fasta, gff, seq_type=seq_type, order='py2')


@pytest.mark.parametrize('gff', [
    # orphan parent (print + None in read_gff)
    'c1\tx\tCDS\t1\t9\t.\t+\t0\tID=c1;Parent=nope\n',
    # invalid strand on a CDS (print + TypeError in get_fasta)
    'c1\tx\tgene\t1\t9\t.\t+\t.\tID=g1\nc1\tx\tmRNA\t1\t9\t.\t+\t.\tID=m1;Parent=g1\n'
    'c1\tx\tCDS\t1\t9\t.\t?\t0\tID=c1;Parent=m1\n',
    # missing seqid
    'zz\tx\tgene\t1\t9\t.\t+\t.\tID=g1\nzz\tx\tmRNA\t1\t9\t.\t+\t.\tID=m1;Parent=g1\n'
    'zz\tx\tCDS\t1\t9\t.\t+\t0\tID=c1;Parent=m1\n',
    # non-integer coordinate (ValueError)
    'c1\tx\tgene\t1\tten\t.\t+\t.\tID=g1\n',
    # mixed Base / Parent children
    'c1\tx\tgene\t1\t9\t.\t+\t.\tID=g1\nc1\tx\tCDS\t1\t9\t.\t+\t0\tID=c1;Parent=g1\n'
    'c1\tx\tmRNA\t1\t9\t.\t+\t.\tID=m1;Parent=g1\n',
])
def test_native_plan_declines_diagnostic_paths(gff):
    gs = G.GenomeSequence('>c1\nACGTACGTACGT\n')
    assert engine.GffPlan.build(gff, list(gs), [12], protein=True) is None


def test_native_plan_dedupe_and_join_shapes():
    """Duplicate IDs (ID2, ID-3), genes without CDS (blank records), nested
    parents and '-' strand ordering by the last child's strand."""
    fasta = '>c1\n' + 'ACGTTGCAAC' * 30 + '\n>c2\n' + 'GGGAAATTTCCC' * 20 + '\n'
    gff = ''.join([
        'c1\tx\tgene\t1\t300\t.\t+\t.\tID=g1\n',
        'c1\tx\tmRNA\t1\t300\t.\t+\t.\tID=m1;Parent=g1\n',
        'c1\tx\tCDS\t10\t40\t.\t+\t0\tID=cds;Parent=m1\n',
        'c1\tx\tCDS\t50\t90\t.\t+\t0\tID=cds;Parent=m1\n',
        'c1\tx\tCDS\t100\t140\t.\t-\t0\tID=cds;Parent=m1\n',
        'c1\tx\tmRNA\t1\t300\t.\t-\t.\tID=m2;Parent=g1\n',
        'c1\tx\tCDS\t200\t260\t.\t-\t0\tID=m2c;Parent=m2\n',
        'c1\tx\tCDS\t150\t180\t.\t-\t0\tID=m2d;Parent=m2\n',
        'c1\tx\tCDS\t150\t180\t.\t-\t0\tID=m2e;Parent=m2\n',
        'c2\tx\tgene\t1\t200\t.\t+\t.\tID=g2\n',
        'c2\tx\tgene\t1\t200\t.\t+\t.\tID=g3\n',
        'c2\tx\tmRNA\t5\t150\t.\t+\t.\tID=m3;Parent=g3\n',
        'c2\tx\tCDS\t5\t150\t.\t+\t0\tID=m3c;Parent=m3\n',
        'c2\tx\tCDS\t230\t260\t.\t+\t0\tID=past;Parent=m3\n',
    ])
    for seq_type in ('nucleotide', 'protein'):
        for order in ('insertion', 'py2'):
            got = native_gff2fasta(fasta, gff, seq_type, order)
            assert got is not None
            assert got == mo.gff2fasta(fasta, gff, seq_type=seq_type, order=order)


def _dup_heavy_gff():
    """Shared CDS IDs in runs, an ID repeated out of run order, CRLF lines,
    comments and ignored exons: the ordered pass's rename prediction and the
    chunk split both have to hold."""
    rows = []
    for g in range(40):
        lo = 1 + 30 * (g % 9)
        rows.append('c1\tx\tgene\t%d\t%d\t.\t%s\t.\tID=g%d' % (lo, lo + 25, '+-'[g % 2], g))
        rows.append('c1\tx\tmRNA\t%d\t%d\t.\t%s\t.\tID=m%d;Parent=g%d' % (lo, lo + 25, '+-'[g % 2], g, g))
        if g % 5 == 0:
            rows.append('# a comment line')
        for k in range(1 + g % 4):
            rows.append('c1\tx\texon\t%d\t%d\t.\t+\t.\tID=e%d;Parent=m%d' % (lo + k, lo + k + 4, g, g))
            cid = 'shared' if g % 7 == 3 else 'cds%d' % (g // 2)
            rows.append('c1\tx\tCDS\t%d\t%d\t.\t%s\t0\tID=%s;Parent=m%d'
                        % (lo + 5 * k, lo + 5 * k + 4, '+-'[g % 2], cid, g))
    text = ''
    for i, r in enumerate(rows):
        text += r + ('\r\n' if i % 11 == 0 else '\n')
    return text


@pytest.mark.parametrize('chunks', [1, 2, 7, 64])
def test_native_plan_chunked_parse(monkeypatch, chunks):
    """The parallel parse and lowering passes over forced splits give the oracle's
    output (renamed IDs across chunk boundaries included)."""
    monkeypatch.setenv('MAGOT_GFF_CHUNKS', str(chunks))
    fasta = '>c1\n' + 'ACGTTGCAACGGAT' * 30 + '\n'
    gff = _dup_heavy_gff()
    for seq_type in ('nucleotide', 'protein'):
        for order in ('insertion', 'py2'):
            got = native_gff2fasta(fasta, gff, seq_type, order)
            assert got is not None
            assert got == mo.gff2fasta(fasta, gff, seq_type=seq_type, order=order)


@pytest.mark.parametrize('fmt', ['gff3', 'gtf'])
def test_native_plan_chunked_synthetic(monkeypatch, fmt):
    monkeypatch.setenv('MAGOT_GFF_CHUNKS', '13')
    w = synth.make('small', seed=5, genome_bases=300_000, n_tx=200, iupac_rate=1e-3)
    fasta = w.fasta_text()
    gff = w.gff3_text() if fmt == 'gff3' else w.gtf_text()
    got = native_gff2fasta(fasta, gff, 'protein', 'py2')
    assert got is not None
    assert got == mo.gff2fasta(fasta, gff, seq_type='protein', order='py2')


def test_native_plan_chunked_declines(monkeypatch):
    """A diagnostic line found by a later chunk still declines the input."""
    monkeypatch.setenv('MAGOT_GFF_CHUNKS', '5')
    gs = G.GenomeSequence('>c1\n' + 'ACGT' * 100 + '\n')
    good = ''.join('c1\tx\tgene\t1\t9\t.\t+\t.\tID=g%d\n' % i for i in range(50))
    assert engine.GffPlan.build(good, list(gs), [400], protein=True) is not None
    bad = good + 'c1\tx\tgene\t1\tten\t.\t+\t.\tID=gz\n'
    assert engine.GffPlan.build(bad, list(gs), [400], protein=True) is None


# ---------------------------------------------------------------------------
# get_fasta(longest=True) and get_fasta(genomic=True) through the native
# planner (genome.py:680-682, 711-724), on the randomised inputs whose
# reference outputs tests/golden/fuzz*.json hold (renamed IDs, reversed and
# past-end coordinates, mixed strands, UTR / exon children, GTF hierarchies)
# ---------------------------------------------------------------------------

def _fuzz_inputs():
    import json
    import os
    out = []
    for name in ('fuzz.json', 'fuzz2.json'):
        for rec in json.load(open(os.path.join(goldlib.HERE, name))):
            out.append((rec['fasta'], rec['gff']))
    return out


FUZZ_INPUTS = _fuzz_inputs()


def _oracle_or_diag(fasta, gff, **kw):
    import io
    out = io.StringIO()  # the oracle's diagnostic prints
    try:
        text = mo.gff2fasta(fasta, gff, out=out, **kw)
    except Exception:
        return None, True
    return text, bool(out.getvalue())


@pytest.mark.parametrize('i', range(len(FUZZ_INPUTS)))
def test_native_longest_and_genomic_match_oracle(i):
    fasta, gff = FUZZ_INPUTS[i]
    calls = [dict(seq_type='nucleotide', longest=True), dict(seq_type='protein', longest=True),
             dict(seq_type='nucleotide', genomic=True), dict(seq_type='protein', genomic=True),
             dict(seq_type='protein', genomic=True, longest=True),
             dict(seq_type='nucleotide', from_exons=True), dict(seq_type='protein', from_exons=True),
             dict(seq_type='nucleotide', from_exons=True, genomic=True)]
    for kw in calls:
        for order in ('insertion', 'py2'):
            got = native_gff2fasta(fasta, gff, order=order, **kw)
            want, diag = _oracle_or_diag(fasta, gff, order=order, **kw)
            if got is None:
                assert diag, ('declined without a diagnostic path', kw, order)
                continue
            assert not diag, ('planned an input with a diagnostic path', kw, order)
            assert got == want, (kw, order)


def test_native_longest_and_genomic_plan_most_inputs():
    """The native planner serves most of those calls (the rest hit a
    reference diagnostic path and go to the object path)."""
    planned = 0
    for fasta, gff in FUZZ_INPUTS:
        for kw in (dict(longest=True), dict(genomic=True)):
            planned += native_gff2fasta(fasta, gff, 'nucleotide', 'py2', **kw) is not None
    assert planned >= len(FUZZ_INPUTS) // 2, planned


def test_native_longest_synthetic():
    """Genes with 1-4 transcripts of random CDS sets on both strands, some of
    equal length (a tie: the later transcript wins), genes without
    transcripts, in GFF3 and in both record orders."""
    rng = np.random.default_rng(33)
    contig = ''.join(rng.choice(list('ACGTacgtN'), 60_000))
    fasta = '>c1\n' + contig + '\n'
    rows = []
    for g in range(150):
        lo = int(rng.integers(1, 55_000))
        st = '+-'[int(rng.integers(0, 2))]
        rows.append('c1\tx\tgene\t%d\t%d\t.\t%s\t.\tID=g%d' % (lo, lo + 4000, st, g))
        shared = None
        for m in range(int(rng.integers(0, 5))):
            rows.append('c1\tx\tmRNA\t%d\t%d\t.\t%s\t.\tID=g%d.m%d;Parent=g%d'
                        % (lo, lo + 4000, st, g, m, g))
            if shared is not None and rng.random() < 0.3:
                cds = shared  # same intervals: same length, a tie
            else:
                cds = sorted({(int(a), int(a) + int(rng.integers(3, 300)))
                              for a in rng.integers(lo, lo + 3500, size=int(rng.integers(1, 6)))})
            shared = cds
            for k, (a, b) in enumerate(cds):
                rows.append('c1\tx\tCDS\t%d\t%d\t.\t%s\t0\tID=cds.g%d.m%d;Parent=g%d.m%d'
                            % (a, b, st, g, m, g, m))
    gff = '\n'.join(rows) + '\n'
    for order in ('py2', 'insertion'):
        for seq_type in ('nucleotide', 'protein'):
            got = native_gff2fasta(fasta, gff, seq_type, order, longest=True)
            want, diag = _oracle_or_diag(fasta, gff, seq_type=seq_type, order=order, longest=True)
            assert (got is None) == diag, seq_type  # protein: records below one codon
            if got is not None:
                assert got == want, seq_type
        gen = native_gff2fasta(fasta, gff.replace('\tID=g7\n', '\tID=g7\n'), 'protein', order,
                               genomic=True)
        want, diag = _oracle_or_diag(fasta, gff, seq_type='protein', order=order, genomic=True)
        assert (gen is None) == diag  # genes without transcripts: get_coords() is None
        if gen is not None:
            assert gen == want


def test_native_longest_protein_picks_by_trimmed_length():
    """Two transcripts whose CDS are 12 bases each: four codons, but the
    first one's leading codon holds an N, so trimX drops its 'X' and the
    second (4 residues against 3) is the longest; swapped, the later one
    wins the tie (genome.py:720-724)."""
    seq = 'NAAATGGCCTTT' + 'ATGAAACCCGGG'
    fasta = '>c1\n' + seq + '\n'
    head = 'c1\tx\tgene\t1\t24\t.\t+\t.\tID=g1\n'
    def tx(name, a, b):
        return ('c1\tx\tmRNA\t%d\t%d\t.\t+\t.\tID=%s;Parent=g1\n' % (a, b, name) +
                'c1\tx\tCDS\t%d\t%d\t.\t+\t0\tID=%s.c;Parent=%s\n' % (a, b, name, name))
    for gff in (head + tx('m1', 1, 12) + tx('m2', 13, 24), head + tx('m2', 13, 24) + tx('m1', 1, 12),
                head + tx('m1', 13, 24) + tx('m2', 13, 24)):
        gs = G.GenomeSequence(fasta)
        plan = engine.GffPlan.build(gff, list(gs), [24], protein=True, longest=True)
        assert plan is not None and plan.n_select == 1
        plan.close()
        for order in ('insertion', 'py2'):
            got = native_gff2fasta(fasta, gff, 'protein', order, longest=True)
            assert got == mo.gff2fasta(fasta, gff, seq_type='protein', order=order, longest=True)


def test_native_from_exons_replace_and_substring_ignore():
    """from_exons="True" (genome_tools.py:326-327): "\texon\t" becomes "\tCDS\t"
    anywhere in the line (the source column too, non-overlapping, left to
    right), then every type that is a substring of "CDS" ("", C, D, S, CD,
    DS, CDS) is ignored; other types stay (genomic spans over what remains)."""
    fasta = '>c1\n' + 'ACGTTGCA' * 40 + '\n'
    rows = ['c1\tx\tgene\t1\t300\t.\t+\t.\tID=g1',
            'c1\texon\tmRNA\t5\t200\t.\t+\t.\tID=m1;Parent=g1',
            'c1\tx\texon\t5\t50\t.\t+\t.\tID=e1;Parent=m1',
            'c1\tx\tCD\t60\t70\t.\t+\t.\tID=x1;Parent=m1',
            'c1\tx\tregion\t80\t90\t.\t+\t.\tID=r1;Parent=m1',
            'c1\tx\tgene\t100\t250\t.\t-\t.\tID=g2',
            'c1\texon\tmRNA\t100\t250\t.\t-\t.\tID=m2;Parent=g2',
            'c1\tx\tUTR\t100\t120\t.\t-\t.\tID=u2;Parent=m2']
    gff = '\n'.join(rows) + '\n'
    planned = 0
    for kw in (dict(), dict(genomic=True), dict(longest=True)):
        for seq_type in ('nucleotide', 'protein'):
            got = native_gff2fasta(fasta, gff, seq_type, 'insertion', from_exons=True, **kw)
            want, diag = _oracle_or_diag(fasta, gff, seq_type=seq_type, order='insertion',
                                         from_exons=True, **kw)
            assert (got is None) == diag, (kw, seq_type)
            if got is not None:
                assert got == want, (kw, seq_type)
                planned += 1
    assert planned >= 2  # genomic and longest hit the reference's TypeError / ValueError on g2


@pytest.mark.parametrize('fmt', ['gff3', 'gtf'])
def test_native_plan_many_contigs(fmt):
    """150 contigs, each with one gene: the planner's seqid table grows past its
    initial 64 slots (rehash), and for GTF the hierarchy IDs outnumber the
    lines the ID table was reserved for."""
    import random
    rng = random.Random(7)
    fasta, gff = [], []
    for i in range(150):
        seq = ''.join(rng.choice('ACGT') for _ in range(90))
        fasta.append('>chr%d\n%s\n' % (i, seq))
        s = '+-'[i % 2]
        if fmt == 'gff3':
            gff.append('chr%d\tx\tgene\t1\t60\t.\t%s\t.\tID=g%d\n' % (i, s, i))
            gff.append('chr%d\tx\tmRNA\t1\t60\t.\t%s\t.\tID=m%d;Parent=g%d\n' % (i, s, i, i))
            gff.append('chr%d\tx\tCDS\t4\t30\t.\t%s\t0\tID=c%d;Parent=m%d\n' % (i, s, i, i))
            gff.append('chr%d\tx\tCDS\t34\t57\t.\t%s\t0\tID=c%d;Parent=m%d\n' % (i, s, i, i))
        else:
            for lo, hi in ((4, 30), (34, 57)):
                gff.append('chr%d\tx\tCDS\t%d\t%d\t.\t%s\t0\tgene_id "g%d"; transcript_id "t%d";\n'
                           % (i, lo, hi, s, i, i))
    fasta, gff = ''.join(fasta), ''.join(gff)
    for seq_type in ('nucleotide', 'protein'):
        got = native_gff2fasta(fasta, gff, seq_type, 'py2')
        assert got is not None
        assert got == mo.gff2fasta(fasta, gff, seq_type=seq_type, order='py2')


def _tables_text(plan, seqs):
    return (plan.exons.tobytes(), plan.txs.tobytes(), plan.render(*_payloads(plan, seqs)))


@pytest.mark.parametrize('fmt', ['gff3', 'gtf'])
@pytest.mark.parametrize('kw', [{}, {'protein': True, 'order': 'py2'},
                                {'genomic': True}, {'protein': True, 'longest': True}])
def test_two_step_read_then_lower_equals_one_call(fmt, kw):
    """gff2fasta reads the GFF (magot_gff_read) while the genome loads and
    lowers it against the loaded contigs afterwards (magot_gff_lower): the
    same tables and text as magot_gff_plan in one call."""
    w = synth.make('small', seed=23, genome_bases=300_000, n_tx=200, iupac_rate=1e-3)
    gs = G.GenomeSequence(w.fasta_text())
    names = list(gs)
    lens = [len(gs[n]) for n in names]
    gff = w.gff3_text() if fmt == 'gff3' else w.gtf_text()
    one = engine.GffPlan.build(gff, names, lens, **kw)
    rd = engine.GffRead.read(gff)
    two = rd.lower(names, lens, **kw)
    assert rd.handle is None                      # the plan took the handle over
    seqs = [gs[n] for n in names]
    assert _tables_text(one, seqs) == _tables_text(two, seqs)
    assert (one.protein, one.n_select) == (two.protein, two.n_select)
    one.close()
    two.close()
    with pytest.raises(engine.MagotError):        # one lowering per read
        rd.lower(names, lens)


def test_two_step_declines_like_one_call():
    gs = G.GenomeSequence('>c1\nACGTACGTACGT\n')
    # read_gff itself declines (orphan parent) ...
    assert engine.GffRead.read('c1\tx\tCDS\t1\t9\t.\t+\t0\tID=c1;Parent=nope\n') is None
    # ... or only the lowering does (a seqid the genome lacks)
    rd = engine.GffRead.read('zz\tx\tgene\t1\t9\t.\t+\t.\tID=g1\nzz\tx\tmRNA\t1\t9\t.\t+\t.\t'
                             'ID=m1;Parent=g1\nzz\tx\tCDS\t1\t9\t.\t+\t0\tID=c1;Parent=m1\n')
    assert rd is not None
    assert rd.lower(list(gs), [12], protein=True) is None
    assert rd.handle is None


def test_two_step_abi_state_errors():
    import ctypes
    from magot_amd import _lib
    L = _lib.lib()
    h = ctypes.c_void_p()
    text = b'c1\tx\tgene\t1\t9\t.\t+\t.\tID=g1\n'
    assert L.magot_gff_read(text, len(text), 0, ctypes.byref(h)) == 0
    names = (ctypes.c_char_p * 1)(b'c1')
    lens = np.array([12], dtype=np.uint64)
    ne, nt = ctypes.c_uint64(), ctypes.c_uint64()
    args = (names, lens.ctypes.data_as(_lib._u64p), 1, b'gene', 0, ctypes.byref(ne),
            ctypes.byref(nt))
    assert L.magot_gff_lower(h, *args) == 0
    assert L.magot_gff_lower(h, *args) == _lib.ERR_STATE      # lowered already
    L.magot_gffplan_destroy(h)
    assert L.magot_gff_lower(None, *args) == _lib.ERR_ARG
