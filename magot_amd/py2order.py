"""Python 2.7 dict iteration order for str keys.

The reference is a Python 2.7 program: ``AnnotationSet.get_fasta`` emits
records in the iteration order of a plain dict (genome.py:580), i.e. CPython
2.7's open-addressing slot order, after ``read_gff`` has rebuilt every dict
once more through ``copy.deepcopy`` (genome.py:415).  Its own goldens
(test_data/test_suite.py:12-13) are in that order.  This module computes it
from the insertion sequence so the drop-in can reproduce those files byte for
byte (``order="py2"``).

Model (CPython 2.7, 64-bit, no -R):
  * string_hash: x = c0 << 7; x = (1000003 * x) ^ c per char; x ^= len;
    -1 maps to -2; "" hashes to 0.
  * lookdict probing: i = h & mask, then i = 5*i + perturb + 1, perturb >>= 5.
  * after inserting a NEW key, if fill*3 >= (mask+1)*2 the table is rebuilt
    at the smallest power of two > (used>50000 ? 2 : 4) * used (min 8),
    re-inserting entries in old slot order.
"""

_MASK64 = 0xFFFFFFFFFFFFFFFF


def str_hash(key):
    if len(key) == 0:
        return 0
    h = (ord(key[0]) << 7) & _MASK64
    for ch in key:
        h = ((h * 1000003) & _MASK64) ^ ord(ch)
    h ^= len(key)
    if h == _MASK64:
        h = _MASK64 - 1
    return h


class _SlotTable(object):
    __slots__ = ('slots', 'used')

    def __init__(self, size=8):
        self.slots = [None] * size
        self.used = 0

    def _place(self, key, h):
        slots = self.slots
        mask = len(slots) - 1
        i = h & mask
        perturb = h
        while True:
            cur = slots[i & mask]
            if cur is None:
                slots[i & mask] = key
                return True
            if cur == key:
                return False
            i = (i * 5 + perturb + 1) & _MASK64
            perturb >>= 5

    def insert(self, key):
        if not self._place(key, str_hash(key)):
            return
        self.used += 1
        if self.used * 3 >= len(self.slots) * 2:
            want = (2 if self.used > 50000 else 4) * self.used
            size = 8
            while size <= want:
                size <<= 1
            old = self.slots
            self.slots = [None] * size
            for k in old:
                if k is not None:
                    self._place(k, str_hash(k))

    def order(self):
        return [k for k in self.slots if k is not None]


def dict_order(keys):
    """Iteration order of a Py2 dict built by inserting ``keys`` in order."""
    t = _SlotTable()
    for k in keys:
        t.insert(k)
    return t.order()


def order_after_copies(keys, copies=1):
    """Insertion, then ``copies`` rebuilds (deepcopy re-inserts in iteration order)."""
    out = dict_order(keys)
    for _ in range(copies):
        out = dict_order(out)
    return out
