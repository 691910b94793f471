"""Host-layer tests (CPU): the drop-in's parser, annotation walk, error
semantics, record order and rendering, with the device executor replaced by
an oracle-backed stand-in.  The GPU path itself is tested in test_gpu_*.py;
here only ``_Batch.run`` (the one call that reaches libmagot) is swapped.
"""

import hashlib
import json
import os
import re

import pytest

import goldlib
from magot_amd import genome as G
from magot_amd import py2order
from oracle import magot_oracle as mo


class _FakeDevice(object):
    def __init__(self, seqdict):
        self.names = list(seqdict)
        self.index = {n: i for i, n in enumerate(self.names)}
        self.seqs = [seqdict[n] for n in self.names]


def _oracle_run(self):
    res = []
    for j, kind in enumerate(self.kinds):
        b, n = self.tx_begin[j], self.tx_n[j]
        parts = []
        for e in range(b, b + n):
            st = self.ex_start[e]
            rc = bool(st >> 63)
            st &= (1 << 63) - 1
            dev = self.genomes[self.ex_gid[e]][1]
            s = dev.seqs[self.ex_contig[e]][st:st + self.ex_len[e]]
            parts.append(mo.reverse_complement(s) if rc else s)
        s = ''.join(parts)
        res.append(s if kind == 'nuc' else mo.translate(s))
    self.results = res


@pytest.fixture
def host_only(monkeypatch):
    monkeypatch.setattr(G, '_device_genome_for', _FakeDevice)
    monkeypatch.setattr(G._Batch, 'run', _oracle_run)


def _json(name):
    with open(os.path.join(goldlib.HERE, name)) as fh:
        return json.load(fh)


def _sha(s):
    return hashlib.sha256(s.encode('latin-1')).hexdigest()


def gff2fasta(fasta, gff, **kw):
    order = kw.pop('order', 'insertion')
    g = G.Genome(fasta)
    g.read_gff(gff)
    return g.annotations.get_fasta('gene', order=order, **kw) + '\n'


def test_genome_sequence_parse_matches_oracle():
    text = '>a b\r\nACGT\nac\r\n>e\n>a b\nTT\n\n>z\nNN RYk\n'
    assert dict(G.GenomeSequence(text)) == mo.read_fasta(text)
    assert dict(G.GenomeSequence(text, truncate_names=True)) == \
        mo.read_fasta(text, truncate_names=True)
    pre = 'ACG\n>x\nTT\n'
    assert dict(G.GenomeSequence(pre)) == mo.read_fasta(pre)
    fa = goldlib.path('O.biroi_refseqGenomeSubset.fasta')
    assert dict(G.GenomeSequence(fa)) == mo.read_fasta(fa)


def _shape(aset, getter):
    out = {}
    for name, table in sorted(vars(aset).items()):
        if type(table) is not dict:
            continue
        rows = []
        for k, obj in table.items():
            rows.append((k, 'child_list' in vars(obj), obj.ID, obj.seqid, getattr(obj, 'coords', None),
                         obj.strand, obj.parent, list(getattr(obj, 'child_list', [])),
                         sorted((a, str(b)) for a, b in vars(obj).items()
                                if a not in ('annotation_set',))))
        out[name] = rows
    return out


@pytest.mark.parametrize('ann', ['O.biroi_NCBIrefseq_gff3Subset.gff', 'StandardGTF.gtf',
                                 'transcriptlessGTF.gtf', 'minimalGFF3.gff'])
def test_read_gff_builds_the_reference_graph(ann):
    mine = G.read_gff(goldlib.path(ann))
    ref = mo.read_gff(goldlib.path(ann))
    assert _shape(mine, None) == _shape(ref, None)


def test_getitem_last_sorted_attribute_wins():
    a = G.AnnotationSet()
    a.zeta = {'x': 1}
    a.CDS['x'] = 2
    assert a['x'] == 1          # 'zeta' sorts after 'CDS'
    with pytest.raises(KeyError):
        a['missing']
    a.gene['gene'] = 3
    assert a['gene'] == 3       # no __dict__ entry in the Python-2 dir()


def test_py2order_matches_oracle_model():
    keys = ['g%d' % i for i in range(3000)] + ['', 'a', 'ab', 'Chromosome14-CDS2']
    assert py2order.dict_order(keys) == mo.py2_dict_order(keys)
    assert py2order.order_after_copies(keys, 1) == mo.py2_order_after_deepcopy(keys)


def test_edge_cases_host(host_only, capsys):
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


@pytest.mark.parametrize('key', ['obiroi/nucleotide/insertion', 'obiroi/protein/insertion',
                                 'obiroi/nucleotide/py2', 'obiroi/protein/py2',
                                 'obiroi/longest/insertion', 'obiroi/genomic/insertion'])
def test_obiroi_host(host_only, key):
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
        out, exc = gff2fasta(goldlib.path('O.biroi_refseqGenomeSubset.fasta'),
                             goldlib.path('O.biroi_NCBIrefseq_gff3Subset.gff'), **kw), None
    except Exception as e:  # noqa: BLE001
        out, exc = None, type(e).__name__
    assert exc == want['exc']
    if out is not None:
        assert _sha(out) == want['sha256']


def test_c14_suite_lines_12_13_host(host_only):
    c14 = goldlib.rebuild_c14()
    out = gff2fasta(c14, goldlib.path('StandardGTF.gtf'), order='py2')
    assert goldlib.posix_cksum(out) == (2836090577, 690750)
    out = gff2fasta(c14, goldlib.path('StandardGTF.gtf'), order='py2', seq_type='protein')
    assert goldlib.posix_cksum(out) == (111942461, 233762)


def test_batch_tables_match_synth_plan_tables(host_only):
    """The walker's interval tables equal the ones bench.py builds directly."""
    from magot_amd import synth
    w = synth.make('small', seed=11, genome_bases=300_000, n_tx=150)
    g = G.Genome(w.fasta_text())
    g.read_gff(w.gff3_text())
    batch = G._Batch()
    for k in g.annotations.gene:
        g.annotations.gene[k]._plan_fasta(batch, 'nucleotide', False, False, 'ID')
    ex, tx = w.plan_tables()
    assert batch.tx_n == tx['n_exons'].tolist()
    assert batch.ex_len == ex['len'].tolist()
    assert batch.ex_start == ex['start_rc'].tolist()
    assert batch.ex_contig == ex['contig'].tolist()


def test_cli_argument_parsing():
    from magot_amd import genome_tools
    name, args, kw = genome_tools.parse_argv(['gff2fasta', 'a.fa', 'b.gtf', 'seq_type=protein',
                                             'longest=True'])
    assert name == 'gff2fasta' and args == ['a.fa', 'b.gtf']
    assert kw == {'seq_type': 'protein', 'longest': 'True'}


def test_no_device_fails_loudly(monkeypatch):
    """Without a usable device the product path raises MagotError -- it never
    falls back to a CPU path or degrades into the reference's diagnostics."""
    from magot_amd import _lib

    def no_device(*a, **k):
        raise _lib.MagotError('no HIP device visible')
    monkeypatch.setattr(G.engine, 'DeviceGenome', no_device)
    g = G.Genome('>c1\nACGTACGTAC\n')
    g.read_gff('c1\tx\tgene\t1\t9\t.\t+\t.\tID=g1\n'
               'c1\tx\tmRNA\t1\t9\t.\t+\t.\tID=m1;Parent=g1\n'
               'c1\tx\tCDS\t1\t9\t.\t+\t0\tID=c1;Parent=m1\n')
    with pytest.raises(_lib.MagotError):
        g.annotations.get_fasta('gene')
