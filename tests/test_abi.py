"""The C-ABI library builds, loads and exports what include/magot.h declares
(CPU: no compute calls need a device here)."""

import ctypes
import os
import re

import numpy as np
import pytest

from magot_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    with open(os.path.join(ROOT, 'include', 'magot.h')) as fh:
        text = fh.read()
    return sorted(set(re.findall(r'\b(magot_[a-z0-9_]+)\s*\(', text)))


def test_library_is_built_and_loads():
    assert os.path.exists(_lib.LIB_PATH), 'run python -m magot_amd.build'
    assert _lib.lib().magot_abi_version() == 1


def test_every_declared_symbol_is_exported():
    L = ctypes.CDLL(_lib.LIB_PATH)
    declared = _declared()
    assert len(declared) >= 20
    for name in declared:
        assert hasattr(L, name), name
    assert sorted(_lib.EXPORTS) == declared


def test_struct_layouts_match_header():
    assert _lib.EXON_DTYPE.itemsize == 16
    assert _lib.TX_DTYPE.itemsize == 16


def test_translate_sizes_host_function():
    off = np.array([0, 0, 2, 5, 9, 20], dtype=np.uint64)
    frames = np.array([0, 0, 0, 1, 2], dtype=np.int32)
    poff = np.empty(6, dtype=np.uint64)
    cod = np.empty(5, dtype=np.int64)
    _lib.check(_lib.lib().magot_translate_sizes(_lib.ptr(off), 5, _lib.ptr(frames), _lib.ptr(poff),
                                                _lib.ptr(cod)), 'sizes')
    # lengths 0,2,3,4,11: None, None, 1 codon, frame1 len4 -> junk only, frame2 len11
    assert cod.tolist() == [-1, -1, 1, 1, 3]
    assert poff.tolist() == [0, 0, 0, 1, 2, 5]


def test_orf6_sizes_host_function():
    """Six-frame stream sizes (genome.py:809-818 frame quirk) and placement:
    16-byte-aligned, non-overlapping spans covering [0, total), each record's
    three '-' streams (j = 6r + 2f) before its three '+' streams."""
    lens = [0, 2, 3, 4, 5, 17, 48, 100]
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    n = len(lens)
    soff = np.empty(6 * n + 1, dtype=np.uint64)
    slen = np.empty(6 * n, dtype=np.uint64)
    none = np.empty(6 * n, dtype=np.uint8)
    _lib.check(_lib.lib().magot_orf6_sizes(_lib.ptr(off), n, _lib.ptr(soff), _lib.ptr(slen),
                                           _lib.ptr(none)), 'sizes')
    pos = 0
    for r, L in enumerate(lens):
        for st in (0, 1):
            for f in range(3):
                j = 6 * r + 2 * f + st
                want = (L - 2 * f) // 3 if L > 2 + f and L >= 2 * f + 3 else 0
                assert slen[j] == want, (L, f)
                assert none[j] == (1 if L <= 2 + f else 0)
                assert soff[j] == pos
                pos += (want + 15) & ~15
    assert soff[6 * n] == pos


def test_errors_are_reported_not_swallowed():
    L = _lib.lib()
    rc = L.magot_ctx_create(0, None)
    assert rc != 0
    assert L.magot_last_error()


def test_product_fails_loudly_without_device():
    if _lib.lib().magot_device_count() > 0:
        pytest.skip('a device is visible')
    from magot_amd.genome import Sequence
    with pytest.raises(_lib.MagotError):
        Sequence('ATGAAA').translate()
