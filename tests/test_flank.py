"""Native extract_upstream_downstream planner (magot_flank_plan, csrc/gffplan.cpp)
on CPU.

The planner scans the GFF with the rules of genome_tools.py:457-480 and lowers
every printed window to a single-interval record plus a text skeleton.  Here
the windows' bytes come from the plan's tables through the oracle (never the
product), the skeleton is rendered on the host, and the text must equal the
oracle's, which tests/test_loci.py pins to the reference's own stdout
(tests/golden/loci.json).  Inputs on which the reference raises must be
declined (None): the line loop in genome_tools reproduces the exception.
"""

import json
import os

import pytest

import goldlib
from magot_amd import engine
from oracle import magot_oracle as mo
from test_gffplan import _payloads

GOLD = json.load(open(os.path.join(goldlib.HERE, 'loci.json')))


def native_flank(fasta, gff, n, stream, feature_type='gene', namefrom='ID', truncate='True'):
    seqs = mo.read_fasta(fasta, truncate_names=truncate == 'True')
    names = list(seqs)
    with open(gff, 'rb') as fh:
        text = fh.read()
    plan = engine.GffPlan.flank(text, names, [len(seqs[x]) for x in names], n, stream,
                                feature_type=feature_type, namefrom=namefrom)
    if plan is None:
        return None
    try:
        out = plan.render(*_payloads(plan, [seqs[x] for x in names]))
    finally:
        plan.close()
    return out.decode('latin-1') + '\n'


def _oracle(fasta, gff, n, stream, ft='gene', nf='ID', tr='True'):
    try:
        return mo.extract_upstream_downstream(fasta, gff, n, stream, ft, nf, tr), None
    except Exception as e:  # noqa: BLE001
        return None, type(e).__name__


@pytest.fixture(scope='module')
def small(tmp_path_factory):
    d = tmp_path_factory.mktemp('flank')
    fa, gff = d / 'loci.fa', d / 'loci.gff'
    fa.write_text(GOLD['_inputs']['genome'])
    gff.write_text(GOLD['_inputs']['gff'])
    return str(fa), str(gff)


def _paths(tag, small):
    if tag == 'small':
        return small
    return (goldlib.path('O.biroi_refseqGenomeSubset.fasta'),
            goldlib.path('O.biroi_NCBIrefseq_gff3Subset.gff'))


@pytest.mark.parametrize('key', sorted(k for k in GOLD if k.startswith('updown/')))
def test_native_flank_matches_reference_cases(small, key):
    _, tag, stream, n, ft, nf, tr = key.split('/')
    fa, gff = _paths(tag, small)
    want, exc = _oracle(fa, gff, n, stream, ft, nf, tr)
    got = native_flank(fa, gff, n, stream, ft, nf, tr)
    if exc is not None:
        assert got is None
    else:
        assert got == want


@pytest.mark.parametrize('stream', ['up', 'down'])
@pytest.mark.parametrize('n', ['0', '1', '1000', '20000'])
@pytest.mark.parametrize('ft,nf', [('gene', 'ID'), ('mRNA', 'Parent'), ('CDS', 'Name'),
                                   ('exon', 'gene')])
def test_native_flank_obiroi(stream, n, ft, nf):
    fa, gff = _paths('obiroi', None)
    want, exc = _oracle(fa, gff, n, stream, ft, nf)
    assert exc is None
    assert native_flank(fa, gff, n, stream, ft, nf) == want


@pytest.mark.parametrize('chunks', [2, 7, 64])
def test_native_flank_chunked(monkeypatch, chunks):
    """Forced chunk splits: the 'seq<k>' names and the window a later chunk's
    odd-strand line repeats cross chunk boundaries."""
    fa, gff = _paths('obiroi', None)
    want, _ = _oracle(fa, gff, '500', 'up', 'CDS', 'nothing')
    monkeypatch.setenv('MAGOT_GFF_CHUNKS', str(chunks))
    assert native_flank(fa, gff, '500', 'up', 'CDS', 'nothing') == want


FASTA = '>c1 first contig\n' + 'ACGTTGCAACGGATCC' * 8 + '\n>c2\n' + 'TTAGGCAT' * 6 + '\n'


@pytest.mark.parametrize('gff,args', [
    # odd strands repeat the previous window (named after their own line)
    ('c1\tt\tgene\t40\t50\t.\t+\t.\tID=a\nc1\tt\tgene\t60\t70\t.\t.\t.\tID=b\n'
     'c1\tt\tgene\t80\t90\t.\t?\t.\tName=z\n', ('5', 'up')),
    # a line with six tabs: its strand field is the last one, '+\\n'
    ('c1\tt\tgene\t40\t50\t.\t-\t.\tID=a\nc1\tt\tgene\t60\t70\t.\t+\n', ('5', 'down')),
    # windows clipped at contig ends are dropped; coordinate 0 wraps to the end
    ('c1\tt\tgene\t1\t9\t.\t+\t.\tID=a\nc1\tt\tgene\t0\t9\t.\t+\t.\tID=b\n'
     'c2\tt\tgene\t40\t48\t.\t+\t.\tID=c\nc2\tt\tgene\t2\t47\t.\t-\t.\tID=d\n', ('4', 'up')),
    ('c1\tt\tgene\t1\t9\t.\t+\t.\tID=a\nc1\tt\tgene\t0\t9\t.\t+\t.\tID=b\n'
     'c2\tt\tgene\t40\t48\t.\t+\t.\tID=c\nc2\tt\tgene\t2\t47\t.\t-\t.\tID=d\n', ('4', 'down')),
    # names: the last matching attribute, text between the first two '=',
    # '\\r' dropped, ' ID' is not 'ID'; CRLF lines, comments, swapped coordinates
    ('#c1\tt\tgene\t5\t9\t.\t+\t.\tID=hidden\r\n'
     'c1\tt\tgene\t30\t20\t.\t+\t.\tID=x=y;Name=n; ID=no;ID=last\r\n'
     'c2\tt\tgene\t20\t30\t.\t-\t.\tName=q\r\n', ('6', 'up')),
    # zero-length windows print; negative lengths never do
    ('c1\tt\tgene\t40\t50\t.\t+\t.\tID=a\nc2\tt\tgene\t10\t12\t.\t-\t.\n', ('0', 'up')),
    ('c1\tt\tgene\t40\t50\t.\t+\t.\tID=a\n', ('-3', 'down')),
    # other feature types and no matching lines at all
    ('c1\tt\tmRNA\t40\t50\t.\t+\t.\tID=a\n', ('5', 'up')),
    ('', ('5', 'up')),
    # an unknown seqid on an odd-strand line is never looked up
    ('c1\tt\tgene\t40\t50\t.\t+\t.\tID=a\nnope\tt\tgene\t60\t70\t.\t.\t.\tID=b\n', ('5', 'up')),
    # stream neither up nor down: no line matches, or UnboundLocalError
    ('', ('5', 'sideways')),
])
def test_native_flank_edges(tmp_path, gff, args):
    fa, gf = tmp_path / 'g.fa', tmp_path / 'a.gff'
    fa.write_text(FASTA)
    gf.write_bytes(gff.encode('latin-1'))
    want, exc = _oracle(str(fa), str(gf), *args)
    assert exc is None, exc
    assert native_flank(str(fa), str(gf), *args) == want


@pytest.mark.parametrize('gff,args', [
    ('c1\tt\tgene\t40\t50\t.\t.\t.\tID=a\n', ('5', 'up')),              # UnboundLocalError
    ('c1\tt\tgene\t40\t50\t.\t+\t.\tID=a\n', ('5', 'sideways')),        # UnboundLocalError
    ('nope\tt\tgene\t40\t50\t.\t+\t.\tID=a\n', ('5', 'up')),            # KeyError
    ('c1\tt\tgene\t4x\t50\t.\t+\t.\tID=a\n', ('5', 'up')),              # ValueError
    ('c1\tt\tgene\t40\t50\t.\t+\t.\tID;Name=a\n', ('5', 'up')),         # IndexError
    ('c1\tt\tgene\t40\t50\t.\t+\t.\tID=a\n', ('five', 'up')),           # ValueError
])
def test_native_flank_declines_error_paths(tmp_path, gff, args):
    fa, gf = tmp_path / 'g.fa', tmp_path / 'a.gff'
    fa.write_text(FASTA)
    gf.write_text(gff)
    _, exc = _oracle(str(fa), str(gf), *args)
    assert exc is not None
    assert native_flank(str(fa), str(gf), *args) is None


EDGES = json.load(open(os.path.join(goldlib.HERE, 'flank_edges.json')))


def _edge_files(tmp_path, case):
    fa, gf = tmp_path / 'g.fa', tmp_path / 'a.gff'
    fa.write_text(EDGES['genome'])
    gf.write_bytes(case['gff'].encode('latin-1'))
    return str(fa), str(gf), (case['sequence_length'], case['stream'], case['feature_type'],
                              case['namefrom'])


@pytest.mark.parametrize('k', range(len(EDGES['cases'])))
def test_flank_edges_match_reference(tmp_path, k):
    """tests/golden/flank_edges.json: the REFERENCE's stdout / exception on the
    edge cases (make_golden.py --only-flank-edges).  The oracle reproduces
    them; the native planner renders the same text or declines exactly where
    the reference raises."""
    case = EDGES['cases'][k]
    fa, gf, args = _edge_files(tmp_path, case)
    want, exc = _oracle(fa, gf, *args)
    assert exc == case['exc']
    if exc is None:
        assert want == case['stdout']
        assert native_flank(fa, gf, *args) == case['stdout']
    else:
        assert native_flank(fa, gf, *args) is None


# ---------------------------------------------------------------------------
# GPU: the drop-in CLI function on the native path (windows gathered by the
# extraction kernel, text assembled on the device) against the oracle
# ---------------------------------------------------------------------------

def _cli(*args, **kw):
    import contextlib
    import io

    from magot_amd import genome_tools
    buf = io.BytesIO()
    out = io.TextIOWrapper(buf, encoding='latin-1', write_through=True)
    with contextlib.redirect_stdout(out):
        genome_tools.extract_upstream_downstream(*args, **kw)
    out.flush()
    return buf.getvalue().decode('latin-1')


@pytest.mark.gpu
@pytest.mark.parametrize('stream', ['up', 'down'])
@pytest.mark.parametrize('n,ft,nf,tr', [('1000', 'gene', 'ID', 'True'),
                                        ('0', 'mRNA', 'Parent', 'True'),
                                        ('50', 'CDS', 'nothing', 'False'),
                                        ('20000', 'exon', 'gene', 'True')])
def test_gpu_flank_native_path(monkeypatch, stream, n, ft, nf, tr):
    from magot_amd import genome_tools
    calls = []
    real = genome_tools._flank_native

    def spy(*a, **k):
        r = real(*a, **k)
        calls.append(r is not None)
        return r

    monkeypatch.setattr(genome_tools, '_flank_native', spy)
    fa, gff = _paths('obiroi', None)
    want, exc = _oracle(fa, gff, n, stream, ft, nf, tr)
    assert exc is None
    assert _cli(fa, gff, n, stream, ft, nf, tr) == want
    assert calls == [True]  # served natively
    assert _cli(fa, gff, n, stream, ft, nf, tr, native='False') == want


@pytest.mark.gpu
def test_gpu_flank_edges_and_declines(tmp_path):
    fa, gf = tmp_path / 'g.fa', tmp_path / 'a.gff'
    fa.write_text(FASTA)
    gf.write_text('c1\tt\tgene\t1\t9\t.\t+\t.\tID=a\nc1\tt\tgene\t0\t9\t.\t+\t.\tID=b\n'
                  'c2\tt\tgene\t40\t48\t.\t+\t.\tID=c\nc2\tt\tgene\t2\t47\t.\t-\t.\n'
                  'c1\tt\tgene\t60\t70\t.\t.\t.\tID=r\n')
    for stream in ('up', 'down'):
        for n in ('0', '4', '30'):
            want, exc = _oracle(str(fa), str(gf), n, stream)
            assert exc is None
            assert _cli(str(fa), str(gf), n, stream) == want
    gf.write_text('c1\tt\tgene\t40\t50\t.\t.\t.\tID=a\n')
    with pytest.raises(UnboundLocalError):
        _cli(str(fa), str(gf), '5', 'up')


@pytest.mark.gpu
@pytest.mark.parametrize('k', range(len(EDGES['cases'])))
def test_gpu_flank_edges_match_reference(tmp_path, k):
    case = EDGES['cases'][k]
    fa, gf, args = _edge_files(tmp_path, case)
    try:
        text, exc = _cli(fa, gf, *args), None
    except Exception as e:  # noqa: BLE001
        text, exc = None, type(e).__name__
    assert exc == case['exc']
    if exc is None:
        assert text == case['stdout']


FUZZ = json.load(open(os.path.join(goldlib.HERE, 'flank_fuzz.json')))


@pytest.mark.parametrize('k', range(len(FUZZ['cases'])))
def test_flank_fuzz_matches_reference(tmp_path, k):
    """tests/golden/flank_fuzz.json: the REFERENCE on 150 random GFFs (every
    strand form, coordinates at and past the contig ends, names with '=', CRLF,
    six-tab lines; make_golden.py _flank_case).  The oracle reproduces them;
    the native planner renders the same text or declines where the
    reference raises."""
    case = FUZZ['cases'][k]
    fa, gf, args = _fuzz_files(tmp_path, case)
    want, exc = _oracle(fa, gf, *args)
    assert exc == case['exc']
    if exc is None:
        assert want == case['stdout']
        assert native_flank(fa, gf, *args) == case['stdout']
    else:
        assert native_flank(fa, gf, *args) is None


def _fuzz_files(tmp_path, case):
    fa, gf = tmp_path / 'g.fa', tmp_path / 'a.gff'
    fa.write_text(FUZZ['genome'])
    gf.write_bytes(case['gff'].encode('latin-1'))
    return str(fa), str(gf), (case['sequence_length'], case['stream'], case['feature_type'],
                              case['namefrom'])


@pytest.mark.gpu
@pytest.mark.parametrize('k', range(len(FUZZ['cases'])))
def test_gpu_flank_fuzz_matches_reference(tmp_path, k):
    """The reference's random cases through the drop-in CLI function."""
    case = FUZZ['cases'][k]
    fa, gf, args = _fuzz_files(tmp_path, case)
    try:
        text, exc = _cli(fa, gf, *args), None
    except Exception as e:  # noqa: BLE001
        text, exc = None, type(e).__name__
    assert exc == case['exc']
    if exc is None:
        assert text == case['stdout']
