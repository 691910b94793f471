"""Randomised gff2fasta cases against the REFERENCE (tests/golden/fuzz.json,
fuzz3.json and fuzz2.json,
made by tests/golden/make_golden.py from the reference's own Genome /
read_gff / get_fasta): small genomes with lower case, N and IUPAC bytes, and
GFF3 / GTF files with renamed duplicate IDs, reversed, zero and past-end
coordinates, '.', '-' and mixed strands, duplicate coordinates, UTR and exon
children, comment and short lines.  Every case is run as nucleotide, protein,
longest, and in both record orders.

CPU: the oracle reproduces every call.  GPU (marked): the drop-in CLI, on its
native planner path and on the object path, reproduces every call's stdout
(diagnostic prints, then the FASTA text) and exception.
"""
import contextlib
import hashlib
import io
import json
import os

import pytest

import goldlib
from oracle import magot_oracle as mo

# fuzz3.json: 200 more cases of the same generator, another seed
CASES = json.load(open(os.path.join(goldlib.HERE, 'fuzz.json'))) + \
    json.load(open(os.path.join(goldlib.HERE, 'fuzz3.json')))
# genomic=True, longest protein and from_exons=True (exon features as CDS)
# (fuzz4.json: 120 more of them, another seed)
CASES2 = json.load(open(os.path.join(goldlib.HERE, 'fuzz2.json'))) + \
    json.load(open(os.path.join(goldlib.HERE, 'fuzz4.json')))


def _sha(s):
    return hashlib.sha256(s.encode('latin-1')).hexdigest()


def _keys():
    for i, rec in enumerate(CASES):
        for call in sorted(rec['calls']):
            yield i, call


def _run(fn, *a, **kw):
    b = io.BytesIO()
    out = io.TextIOWrapper(b, encoding='latin-1', write_through=True)
    exc = None
    with contextlib.redirect_stdout(out):
        try:
            fn(*a, **kw)
        except Exception as e:  # noqa: BLE001
            exc = type(e).__name__
    out.flush()
    return b.getvalue().decode('latin-1'), exc


def _check(full, exc, want):
    assert exc == want['exc']
    assert full.startswith(want['stdout'])
    if exc is None:
        assert _sha(full[len(want['stdout']):]) == want['sha256']
    else:
        assert full == want['stdout']


@pytest.mark.parametrize('i', range(len(CASES)))
def test_oracle_matches_reference(i):
    rec = CASES[i]
    for call, want in sorted(rec['calls'].items()):
        seq_type, longest, order = call.split('/')

        def run():
            sys_out = mo.gff2fasta(rec['fasta'], rec['gff'], seq_type=seq_type,
                                   longest=longest == '1', order=order)
            import sys
            sys.stdout.write(sys_out)
        full, exc = _run(run)
        _check(full, exc, want)


@pytest.mark.gpu
@pytest.mark.parametrize('native', ['True', 'False'])
@pytest.mark.parametrize('i', range(len(CASES)))
def test_gpu_gff2fasta_matches_reference(i, native):
    from magot_amd import genome_tools
    rec = CASES[i]
    for call, want in sorted(rec['calls'].items()):
        seq_type, longest, order = call.split('/')
        full, exc = _run(genome_tools.gff2fasta, rec['fasta'], rec['gff'], seq_type=seq_type,
                         longest=str(longest == '1'), order=order, native=native)
        _check(full, exc, want)


def _call2(key):
    seq_type, longest, genomic, from_exons, order = key.split('/')
    return seq_type, longest == '1', genomic == '1', from_exons == '1', order


@pytest.mark.parametrize('i', range(len(CASES2)))
def test_oracle_options_match_reference(i):
    rec = CASES2[i]
    for call, want in sorted(rec['calls'].items()):
        seq_type, longest, genomic, from_exons, order = _call2(call)

        def run():
            sys_out = mo.gff2fasta(rec['fasta'], rec['gff'], seq_type=seq_type, longest=longest,
                                   genomic=genomic, order=order, from_exons=from_exons)
            import sys
            sys.stdout.write(sys_out)
        full, exc = _run(run)
        _check(full, exc, want)


@pytest.mark.gpu
@pytest.mark.parametrize('i', range(len(CASES2)))
def test_gpu_gff2fasta_options_match_reference(i):
    from magot_amd import genome_tools
    rec = CASES2[i]
    for call, want in sorted(rec['calls'].items()):
        seq_type, longest, genomic, from_exons, order = _call2(call)
        full, exc = _run(genome_tools.gff2fasta, rec['fasta'], rec['gff'],
                         from_exons=str(from_exons), seq_type=seq_type, longest=str(longest),
                         genomic=str(genomic), order=order)
        _check(full, exc, want)
