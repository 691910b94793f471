"""Sequence.translate with any codon library and any integer frame
(genome.py:795-822), against tests/golden/translate_lib.json (generated from
the reference by tests/golden/make_golden.py): keys that are not ACGT
triplets ('NNN', IUPAC, 1-/2-character junk-codon keys), multi-character,
empty and non-string values, lower-case keys, frames -6..6, both strands,
trimX on and off -- results, None, and the reference's IndexError/TypeError.

CPU: the oracle restatement, and the product's host logic
(_translate_general) with the two device calls stood in for by numpy and the
oracle.  GPU: the product end to end through the C ABI."""
import json
import os

import numpy as np
import pytest

import goldlib
from oracle import magot_oracle as mo


def _cases():
    with open(os.path.join(goldlib.HERE, 'translate_lib.json')) as fh:
        d = json.load(fh)
    std = mo.STANDARD_CODE
    libs = {}
    for name, (base, extra) in d['libs'].items():
        lib = dict(std) if base == 'standard' else {}
        lib.update(extra)
        libs[name] = lib
    return libs, d['cases']


def _run(fn, c, lib):
    try:
        return fn(c['seq'], lib, c['frame'], c['strand'], c['trim']), None
    except Exception as e:  # noqa: BLE001
        return None, type(e).__name__


def _check(fn):
    libs, cases = _cases()
    bad = []
    for c in cases:
        got, exc = _run(fn, c, libs[c['lib']])
        if exc != c['exc'] or (exc is None and got != c['out']):
            bad.append((c, got, exc))
    assert not bad, '%d of %d differ, first: %r' % (len(bad), len(cases), bad[0])
    return len(cases)


def test_oracle_translate_any_library_any_frame():
    n = _check(lambda s, lib, f, st, t: mo.translate(s, library=lib, frame=f, strand=st, trimX=t))
    assert n > 10000


def test_general_path_host_logic(monkeypatch):
    from magot_amd import engine
    from magot_amd import genome as G

    def symbols(seq, cls, K, lut, ctx=None):
        b = np.frombuffer(seq.encode('latin-1'), dtype=np.uint8)
        c = cls[b].astype(np.int64).reshape(-1, 3)
        return lut[c[:, 0] + K * c[:, 1] + K * K * c[:, 2]].tolist()

    monkeypatch.setattr(engine, 'codon_symbols', symbols)
    monkeypatch.setattr(engine, 'revcomp_batch', lambda seqs, ctx=None:
                        [mo.reverse_complement(s) for s in seqs])

    def product(s, lib, f, st, t):
        return G._translate_general(s, lib, f, st, t)
    _check(product)


@pytest.mark.gpu
def test_sequence_translate_any_library_gpu():
    from magot_amd import _lib
    from magot_amd.genome import Sequence
    if _lib.lib().magot_device_count() <= 0:
        pytest.fail('no HIP device visible for a gpu test')
    _check(lambda s, lib, f, st, t: Sequence(s).translate(library=lib, frame=f, strand=st,
                                                          trimX=t))
