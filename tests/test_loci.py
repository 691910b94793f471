"""Locus extraction: genome_tools.extract_upstream_downstream
(genome_tools.py:457-480) and coords2fasta (:656-661).

tests/golden/loci.json holds the REFERENCE's own stdout / exception for every
case (tests/golden/make_golden.py).  CPU: the oracle restatement reproduces
them.  GPU (marked): the drop-in CLI functions, which gather every window with
one extraction-kernel launch, reproduce them byte for byte.
"""
import contextlib
import hashlib
import io
import json
import os

import pytest

import goldlib
from oracle import magot_oracle as mo

GOLD = json.load(open(os.path.join(goldlib.HERE, 'loci.json')))


def _sha(s):
    return hashlib.sha256(s.encode('latin-1')).hexdigest()


@pytest.fixture(scope='module')
def small(tmp_path_factory):
    d = tmp_path_factory.mktemp('loci')
    fa, gff = d / 'loci.fa', d / 'loci.gff'
    fa.write_text(GOLD['_inputs']['genome'])
    gff.write_text(GOLD['_inputs']['gff'])
    return str(fa), str(gff)


def _updown_cases():
    for key in sorted(GOLD):
        if key.startswith('updown/'):
            yield key


def _coords_cases():
    for key in sorted(GOLD):
        if key.startswith('coords/'):
            yield key


def _paths(tag, small):
    if tag == 'small':
        return small
    return (goldlib.path('O.biroi_refseqGenomeSubset.fasta'),
            goldlib.path('O.biroi_NCBIrefseq_gff3Subset.gff'))


@pytest.mark.parametrize('key', list(_updown_cases()))
def test_oracle_updown_matches_reference(small, key):
    _, tag, stream, n, ft, nf, tr = key.split('/')
    fa, gff = _paths(tag, small)
    want = GOLD[key]
    try:
        text = mo.extract_upstream_downstream(fa, gff, n, stream, ft, nf, tr)
        exc = None
    except Exception as e:  # noqa: BLE001
        text, exc = '', type(e).__name__
    assert exc == want['exc']
    assert _sha(text) == want['stdout_sha256']


@pytest.mark.parametrize('key', list(_coords_cases()))
def test_oracle_coords2fasta_matches_reference(small, key):
    _, seqid, a, b, tr = key.split('/')
    text, exc = mo.coords2fasta(small[0], seqid, a, b, tr)
    assert (type(exc).__name__ if exc else None) == GOLD[key]['exc']
    assert text == GOLD[key]['stdout']


def _run_cli(fn, *args):
    buf = io.BytesIO()
    out = io.TextIOWrapper(buf, encoding='latin-1', write_through=True)
    exc = None
    with contextlib.redirect_stdout(out):
        try:
            fn(*args)
        except Exception as e:  # noqa: BLE001
            exc = type(e).__name__
    out.flush()
    return buf.getvalue().decode('latin-1'), exc


@pytest.mark.gpu
@pytest.mark.parametrize('key', list(_updown_cases()))
def test_gpu_updown_matches_reference(small, key):
    from magot_amd import genome_tools
    _, tag, stream, n, ft, nf, tr = key.split('/')
    fa, gff = _paths(tag, small)
    text, exc = _run_cli(genome_tools.extract_upstream_downstream, fa, gff, n, stream, ft, nf, tr)
    assert exc == GOLD[key]['exc']
    if exc is None:
        assert _sha(text) == GOLD[key]['stdout_sha256']


@pytest.mark.gpu
@pytest.mark.parametrize('key', list(_coords_cases()))
def test_gpu_coords2fasta_matches_reference(small, key):
    from magot_amd import genome_tools
    _, seqid, a, b, tr = key.split('/')
    text, exc = _run_cli(genome_tools.coords2fasta, small[0], seqid, a, b, tr)
    assert exc == GOLD[key]['exc']
    assert text == GOLD[key]['stdout']


# ---------------------------------------------------------------------------
# dna2orfs (genome_tools.py:145-180): broken in the reference -- str.translate
# takes no keyword arguments -- pinned by tests/golden/orfs.json.
# ---------------------------------------------------------------------------

def test_dna2orfs_matches_reference_failure(tmp_path):
    import json
    from magot_amd import genome_tools
    gold = json.load(open(os.path.join(os.path.dirname(__file__), 'golden', 'orfs.json')))
    fa = tmp_path / 'orfs.fa'
    fa.write_text(gold['_inputs']['small'])
    for key, want in gold.items():
        if not key.startswith('small/'):
            continue
        _, atg, lg = key.split('/')
        dst = tmp_path / 'out.txt'
        dst.write_text('stale')
        with pytest.raises(TypeError):
            genome_tools.dna2orfs(str(fa), str(dst), from_atg=atg, longest=lg)
        assert want['exc'] == 'TypeError' and want['bytes'] == 0
        assert dst.read_text() == ''  # created (truncated) before the failure
        text, exc = mo.dna2orfs(str(fa), atg, lg)
        assert text == '' and isinstance(exc, TypeError)
    empty = tmp_path / 'empty.fa'
    empty.write_text('')
    genome_tools.dna2orfs(str(empty), str(tmp_path / 'o2.txt'))  # no contig: no error
    assert (tmp_path / 'o2.txt').read_text() == ''


def test_get_cds_peptides_matches_reference_failure(tmp_path):
    """genome_tools.py:283-322 calls the undefined Genome.read_gff3: the
    reference raises AttributeError after reading the genome and before it
    opens the output file; so does the drop-in (no output file)."""
    from magot_amd import genome_tools
    fa = tmp_path / 'g.fa'
    fa.write_text('>c1\nATGAAATAG\n')
    dst = tmp_path / 'out.fa'
    with pytest.raises(AttributeError):
        genome_tools.get_CDS_peptides(str(fa), 'unused.gff', str(dst))
    assert not dst.exists()
