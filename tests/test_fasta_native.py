"""Native FASTA reader (magot_fasta_read, csrc/fasta.cpp) vs the Python
GenomeSequence (genome.py:854-877 semantics), host only."""
import numpy as np
import pytest

import goldlib
from magot_amd import engine
from magot_amd import genome as G

CASES = [
    '>a b\r\nACGT\nac\r\n>e\n>a b\nTT\n\n>z\nNN RYk\n',
    'ACG\n>x\nTT\n',
    '>x\nAAA\n>y\n\n>x\nCC\n',
    '>x\nAAA\n>y\nGG\n>x\n\n',
    '>only header',
    '',
    '\n\n>q\r\n\r\nA>B\n>r\n>\nCCC\n',
    '>t1 desc one\nACGT\n>t2\tdesc\nTTTT\n',
]


@pytest.mark.parametrize('text', CASES)
@pytest.mark.parametrize('trunc', [False, True])
def test_fasta_read_matches_python_reader(text, trunc):
    try:
        want = dict(G.GenomeSequence(text, truncate_names=trunc))
    except IndexError:
        want = None
    got = engine.fasta_read(text, truncate_names=trunc)
    if got is None:
        assert want is None or trunc  # declined: Python reader takes it
        return
    assert want is not None
    assert [(k, v.decode('latin-1')) for k, v in got] == list(want.items())


def test_fasta_read_fixtures():
    for name in ('O.biroi_refseqGenomeSubset.fasta',):
        text = open(goldlib.path(name), 'rb').read()
        got = engine.fasta_read(text)
        want = G.GenomeSequence(goldlib.path(name))
        assert [(k, v.decode('latin-1')) for k, v in got] == list(want.items())
    c14 = goldlib.rebuild_c14()
    got = engine.fasta_read(c14, truncate_names=True)
    want = G.GenomeSequence(c14, truncate_names=True)
    assert [(k, v.decode('latin-1')) for k, v in got] == list(want.items())


def test_fasta_read_random():
    rng = np.random.default_rng(3)
    for _ in range(50):
        parts = []
        for _ in range(rng.integers(0, 6)):
            parts.append('>' + ''.join(rng.choice(list('abc \t1'), size=rng.integers(0, 6))) + '\n')
            for _ in range(rng.integers(0, 4)):
                parts.append(''.join(rng.choice(list('ACGTn>\r'), size=rng.integers(0, 9))) + '\n')
        text = ''.join(parts)
        for trunc in (False, True):
            try:
                want = list(G.GenomeSequence(text, truncate_names=trunc).items())
            except IndexError:
                want = None
            got = engine.fasta_read(text, truncate_names=trunc)
            if got is None:
                continue
            assert want is not None
            assert [(k, v.decode('latin-1')) for k, v in got] == want, repr(text)
