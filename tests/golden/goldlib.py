"""Helpers over the golden fixtures (test infrastructure).

* ``posix_cksum``: the POSIX ``cksum`` CRC the reference's test driver
  compares (test_data/test_suite.py:22-27).
* ``rebuild_c14``: the reference's goldens need test_data/C14.fasta, which is
  not shipped.  Its CDS bases are fully determined by the checked-in golden
  output CDSannotations.cds (= stdout of ``gff2fasta C14.fasta
  StandardGTF.gtf``, test_suite.py:12) laid back onto the StandardGTF.gtf
  intervals; every other base is 'N'.
"""

import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
C14_LENGTH = 8589052


def path(name):
    return os.path.join(HERE, name)


def _crc_table():
    tab = []
    for i in range(256):
        c = i << 24
        for _ in range(8):
            c = ((c << 1) ^ 0x04C11DB7) if c & 0x80000000 else (c << 1)
        tab.append(c & 0xFFFFFFFF)
    return tab


_TAB = _crc_table()


def posix_cksum(data):
    """(crc, size) exactly as coreutils ``cksum`` prints them."""
    if isinstance(data, str):
        data = data.encode('latin-1')
    crc = 0
    tab = _TAB
    for b in data:
        crc = ((crc << 8) & 0xFFFFFFFF) ^ tab[(crc >> 24) ^ b]
    n = len(data)
    size = n
    while n:
        crc = ((crc << 8) & 0xFFFFFFFF) ^ tab[(crc >> 24) ^ (n & 0xFF)]
        n >>= 8
    return (~crc) & 0xFFFFFFFF, size


_COMP = {'a': 't', 't': 'a', 'g': 'c', 'c': 'g', 'A': 'T', 'T': 'A', 'G': 'C', 'C': 'G',
         'n': 'n', 'N': 'N'}


def rebuild_c14():
    """FASTA text of Chromosome14 reconstructed from the committed fixtures."""
    recs = {}
    name = None
    with open(path('CDSannotations.cds'), 'rb') as fh:
        for line in fh.read().decode('latin-1').split('\n'):
            if line.startswith('>'):
                name = line[1:]
                recs[name] = []
            elif name is not None:
                recs[name].append(line)
    recs = {k: ''.join(v) for k, v in recs.items()}
    tx = {}
    with open(path('StandardGTF.gtf'), 'rb') as fh:
        for line in fh.read().decode('latin-1').split('\n'):
            f = line.split('\t')
            if len(f) != 9:
                continue
            tid = re.search(r'transcript_id "([^"]+)"', f[8]).group(1)
            tx.setdefault(tid, []).append((int(f[3]), int(f[4]), f[6]))
    g = bytearray(b'N' * C14_LENGTH)
    for tid, ivs in tx.items():
        seq = recs[tid]
        if ivs[-1][2] == '-':
            seq = ''.join(_COMP[c] for c in reversed(seq))
        p = 0
        for s, e in sorted(set((a, b) for a, b, _ in ivs)):
            g[s - 1:e] = seq[p:p + (e - s + 1)].encode('latin-1')
            p += e - s + 1
        assert p == len(seq), tid
    return '>Chromosome14\n' + g.decode('latin-1') + '\n'
