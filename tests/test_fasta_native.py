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


LAYOUT_CASES = [
    '>a\n' + 'ACGTACGTAC\n' * 5 + 'ACG\n',          # uniform lines, short last line
    '>a\r\n' + 'ACGTACGTAC\r\n' * 5 + 'ACG\r\n',    # CRLF
    '>a\n' + 'ACGTacgtNN\n' * 4,                    # exact multiple of the width
    '>a\nACGT\nAC',                                 # no final newline
    '>a\nACGT\nACGT\n\n>b\nAC\n',                   # blank last line
    '>a\nACGT\n\nACGT\n',                           # blank middle line
    '>a\nACG\nACGTT\nA\n',                          # a longer later line
    '>a\nAC\rG\nACGT\n',                            # CR inside a line
    '>a\nACGT\n\r\nACGT\n',                         # a line holding only CR
    '>a\nACGT\rACGT\r',                             # CR-only line ends
    '>a\r\nACGT\r\nACGT\nAC\r\n',                   # mixed terminators
    '>a\nACGT\nACG\nACGT\n',                        # a short middle line
    '>a\nACGT\nACGTA',                              # long unterminated last line
    '>a\nA\nC\nG\n>a\nTT\nT\n',                     # width 1, repeated name
]


@pytest.mark.parametrize('text', LAYOUT_CASES)
def test_fasta_read_line_layouts(text):
    """Fixed-width records are packed from the text in place (line layout);
    anything else is stripped -- both must give GenomeSequence's bytes."""
    want = dict(G.GenomeSequence(text))
    got = engine.fasta_read(text)
    assert [(k, v.decode('latin-1')) for k, v in got] == list(want.items())


def test_fasta_read_layout_across_chunks():
    """A record larger than the scanner's 8 MiB chunks, with one bad line
    terminator far from the start (forces the strip path) and without."""
    rng = np.random.default_rng(11)
    seq = rng.choice(np.frombuffer(b'ACGTacgtN', np.uint8), size=20_000_003)
    w = 61
    lines = [seq[i:i + w].tobytes() for i in range(0, len(seq), w)]
    body = b'\n'.join(lines) + b'\n'
    cut = body.index(b'\n', 15_000_000)
    for text in (b'>big\n' + body + b'>s\nAC\n',
                 b'>big\n' + body[:cut] + b'\r' + body[cut:] + b'>s\nAC\n',   # CRLF once
                 b'>big\n' + body[:cut] + b'\nT' + body[cut:] + b'>s\nAC\n'):  # width broken
        got = engine.fasta_read(text)
        assert got[0][0] == 'big'
        assert got[0][1] == text.split(b'\n', 1)[1].split(b'\n>s')[0].replace(b'\n', b'').replace(b'\r', b'')
