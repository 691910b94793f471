"""Pin the CPU oracle against the reference's goldens (CPU only).

* test_data/test_suite.py:12,13,14 cksums (rebuilt C14, Python-2 order)
* golden vectors generated from the reference itself (make_golden.py)
"""

import hashlib
import json
import os

import numpy as np
import pytest

import goldlib
from oracle import magot_oracle as mo

GOLDEN = goldlib.HERE


def _json(name):
    with open(os.path.join(GOLDEN, name)) as fh:
        return json.load(fh)


def _sha(s):
    return hashlib.sha256(s.encode('latin-1')).hexdigest()


def _cks(s):
    crc, n = goldlib.posix_cksum(s)
    return '%d %d' % (crc, n)


def test_cksum_matches_coreutils_vector():
    # coreutils: printf '' | cksum -> 4294967295 0 ; printf 'a' | cksum -> 1220704766 1
    assert goldlib.posix_cksum(b'') == (4294967295, 0)
    assert goldlib.posix_cksum(b'a') == (1220704766, 1)


def test_cds_annotations_file_is_golden_12():
    with open(goldlib.path('CDSannotations.cds'), 'rb') as fh:
        data = fh.read()
    assert _cks(data.decode('latin-1')) == '2836090577 690750'   # test_suite.py:12


@pytest.fixture(scope='module')
def c14():
    return goldlib.rebuild_c14()


def test_suite_line12_gff2fasta(c14):
    out = mo.gff2fasta(c14, goldlib.path('StandardGTF.gtf'), order='py2')
    assert _cks(out) == '2836090577 690750'


def test_suite_line13_gff2fasta_protein(c14):
    out = mo.gff2fasta(c14, goldlib.path('StandardGTF.gtf'), seq_type='protein', order='py2')
    assert _cks(out) == '111942461 233762'


def test_suite_line14_cds2pep():
    out = mo.cds2pep(goldlib.path('CDSannotations.cds'))
    assert _cks(out) == '111942461 233762'


def test_py2_order_reproduces_golden_record_order():
    import re
    order = []
    seen = set()
    with open(goldlib.path('StandardGTF.gtf')) as fh:
        for line in fh:
            g = re.search(r'gene_id "([^"]+)"', line).group(1)
            if g not in seen:
                seen.add(g)
                order.append(g)
    with open(goldlib.path('CDSannotations.cds')) as fh:
        gold = [l[1:].rstrip('\n').rsplit('.t', 1)[0] for l in fh if l.startswith('>')]
    assert mo.py2_order_after_deepcopy(order) == gold
    assert mo.py2_dict_order(order) != gold      # one build is not enough (deepcopy)


def test_kat_vectors():
    for rec in _json('kat.json'):
        s = rec['seq']
        assert mo.reverse_complement(s) == rec['revcomp'], s
        for key, want in rec['translate'].items():
            frame, strand, trim = int(key[0]), key[1], bool(int(key[2]))
            if isinstance(want, dict):
                with pytest.raises(Exception) as ei:
                    mo.translate(s, frame=frame, strand=strand, trimX=trim)
                assert type(ei.value).__name__ == want['exc']
            else:
                assert mo.translate(s, frame=frame, strand=strand, trimX=trim) == want, (s, key)
        for key, want in rec['orfs'].items():
            longest, atg = bool(int(key[0])), bool(int(key[1]))
            if isinstance(want, dict):
                with pytest.raises(Exception) as ei:
                    mo.get_orfs(s, longest=longest, from_atg=atg)
                assert type(ei.value).__name__ == want['exc']
            else:
                assert mo.get_orfs(s, longest=longest, from_atg=atg) == want, (s, key)


def test_edge_cases(capsys):
    for case in _json('edge_cases.json'):
        capsys.readouterr()
        res = exc = None
        try:
            aset = mo.load(case['fasta'], case['gff'])
            res = aset.get_fasta('gene', seq_type=case['seq_type'], longest=case['longest'],
                                 genomic=case['genomic'])
        except Exception as e:  # noqa: BLE001
            exc = type(e).__name__
        out = capsys.readouterr().out
        tag = (case['case'], case['seq_type'], case['longest'], case['genomic'])
        # read_gff returning None makes Genome.read_gff raise AttributeError
        if case['exc'] == 'AttributeError' and exc == 'AttributeError':
            pass
        else:
            assert exc == case['exc'], tag
            assert res == case['result'], tag
        assert out == case['stdout'], tag


@pytest.mark.parametrize('key', ['obiroi/nucleotide/insertion', 'obiroi/protein/insertion',
                                 'obiroi/nucleotide/py2', 'obiroi/protein/py2',
                                 'obiroi/longest/insertion', 'obiroi/genomic/insertion'])
def test_obiroi(key):
    want = _json('fixtures.json')[key]
    _, kind, order = key.split('/')
    kw = {'order': order}
    if kind == 'protein':
        kw['seq_type'] = 'protein'
    if kind == 'longest':
        kw['longest'] = True
    if kind == 'genomic':
        kw['genomic'] = True
    try:
        out = mo.gff2fasta(goldlib.path('O.biroi_refseqGenomeSubset.fasta'),
                           goldlib.path('O.biroi_NCBIrefseq_gff3Subset.gff'), **kw)
        exc = None
    except Exception as e:  # noqa: BLE001
        out, exc = None, type(e).__name__
    assert exc == want['exc']
    if out is not None:
        assert _cks(out) == want['cksum']
        assert _sha(out) == want['sha256']


@pytest.mark.parametrize('ann', ['transcriptlessGTF.gtf', 'minimalGFF3.gff'])
def test_c14_other_annotations(c14, ann):
    table = _json('fixtures.json')
    for seq_type in ('nucleotide', 'protein'):
        for order in ('insertion', 'py2'):
            out = mo.gff2fasta(c14, goldlib.path(ann), seq_type=seq_type, order=order)
            assert _sha(out) == table['c14/%s/%s/%s' % (ann, seq_type, order)]['sha256']


def test_synth_small_matches_reference():
    from magot_amd import synth
    want = _json('synth_small.json')
    w = synth.make('small')
    fa = w.fasta_text()
    assert _sha(fa) == want['fasta_sha256'], 'synthetic generator drifted'
    for fmt, text in (('gff3', w.gff3_text()), ('gtf', w.gtf_text())):
        assert _sha(text) == want['%s_sha256' % fmt]
        for seq_type in ('nucleotide', 'protein'):
            out = mo.gff2fasta(fa, text, seq_type=seq_type)
            assert _sha(out) == want['%s/%s' % (fmt, seq_type)]['sha256']


def test_c_oracle_matches_python_oracle():
    from oracle import cds_oracle
    from magot_amd import synth
    w = synth.make('small', seed=7, genome_bases=200_000, n_tx=120)
    fa, gff = w.fasta_text(), w.gff3_text()
    for protein in (False, True):
        out, off, st = cds_oracle.extract_workload(w, protein)
        assert not st.any()
        text = mo.gff2fasta(fa, gff, seq_type='protein' if protein else 'nucleotide')
        seqs = text.split('\n')[1::2]
        got = [out[off[i]:off[i + 1]].tobytes().decode('latin-1') for i in range(w.n_tx)]
        assert got == seqs


def test_c_oracle_six_frames_vs_reference_kats():
    """oracle_orf6_compare's translate(frame, strand) (cds_oracle.c) against
    the reference's own outputs in kat.json (frames 0-2, both strands, with
    and without trimX), laid out as the device streams are: frame 0
    untrimmed, frames 1/2 without their junk codon (= trimmed)."""
    from oracle import cds_oracle
    kats = _json('kat.json')
    seqs = [k['seq'] for k in kats]
    buf = np.frombuffer(''.join(seqs).encode('latin-1'), dtype=np.uint8)
    off = np.zeros(len(seqs) + 1, dtype=np.int64)
    np.cumsum([len(x) for x in seqs], out=off[1:])
    streams = []
    for k in kats:
        for f in (0, 1, 2):
            for st in ('-', '+'):
                v = k['translate']['%d%s%d' % (f, st, 0 if f == 0 else 1)]
                streams.append(v or '')
    slen = np.array([len(x) for x in streams], dtype=np.uint64)
    soff = np.zeros(len(streams) + 1, dtype=np.uint64)
    np.cumsum(slen, out=soff[1:])
    dev = np.frombuffer(''.join(streams).encode('latin-1') + b'\0', dtype=np.uint8)
    assert cds_oracle.orf6_compare(buf, off, dev, soff, slen, threads=2) == (0, -1)
    # a flipped residue is caught, in the right stream
    j = next(i for i, x in enumerate(streams) if x)
    bad = dev.copy()
    bad[int(soff[j]) + len(streams[j]) - 1] ^= 0x20
    assert cds_oracle.orf6_compare(buf, off, bad, soff, slen)[1] == j
