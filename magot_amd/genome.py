"""Drop-in MI355X implementation of MAGOT's ``genome`` module extraction path.

Public names and signatures follow the reference (``genome.py``):
``Genome``, ``GenomeSequence``, ``AnnotationSet``, ``BaseAnnotation``,
``ParentAnnotation``, ``Sequence``, ``read_gff``, ``ensure_file``.

How a call is executed
----------------------
``AnnotationSet.get_fasta`` / ``ParentAnnotation.get_fasta`` walk the
annotation graph with exactly the reference's control flow (child order,
duplicate-coordinate collapse, order taken from the LAST child's strand,
diagnostics printed to stdout at the same points, the same exceptions raised
at the same points) but, instead of slicing strings, they record every
record's interval list into one batch and return a deferred string.  The
batch becomes one device plan (``engine.ExtractionPlan``); a single launch of
the fused HIP kernel gathers, reverse-complements and translates every record
from the 2-bit genome in HBM; the deferred strings are then rendered from the
device output.  Errors of the reference never depend on sequence content, so
all of them are raised during the walk, before the GPU runs.

Record order: insertion order by default (Python 3); ``order="py2"``
reproduces the CPython 2.7 dict order the reference's own goldens use
(``py2order``).
"""

import os
import sys

import numpy as np

from . import engine
from .py2order import order_after_copies

verbose = True

DEFAULT_ORDER = 'insertion'

# genome.py:612-613 (the string continues across a backslash-newline, keeping
# the next line's indentation)
_MSG_GETSEQ = ("either base_annotation has not annotation_set, or annotation_set has no genome, "
               "or genome has no            genome sequence, or genome sequence has no matching "
               "seqid, or coords are out of range on that seqid")
_MSG_MIXED = "ParentAnnotation has both ParentAnnotation and BaseAnnotation children!"
_MSG_ORPHAN = ("It seems that this line has a parent attribute but that that parent doesn't have "
               "a line itself nor\n                    does this line have a defline attribute "
               "that specifies a parent type. I'm afraid this function can't currently\n"
               "                    deal with that.")


def _emit(*items):
    """Python-2 ``print`` of each item on its own line."""
    for it in items:
        sys.stdout.write(str(it) + '\n')


# ---------------------------------------------------------------------------
# I/O (magot_smallfuncs.py:32-43)
# ---------------------------------------------------------------------------

class _Lines(object):
    """Line iterator over bytes decoded latin-1, split on '\\n' only (the
    Python 2 file iteration the reference relies on)."""

    def __init__(self, text):
        self.text = text

    def __iter__(self):
        t = self.text
        n = len(t)
        i = 0
        while i < n:
            j = t.find('\n', i)
            if j < 0:
                yield t[i:]
                return
            yield t[i:j + 1]
            i = j + 1

    def read(self):
        return self.text


def _read_source(potential_file):
    if hasattr(potential_file, 'read'):
        data = potential_file.read()
    else:
        try:
            with open(potential_file, 'rb') as fh:
                data = fh.read()
        except (OSError, ValueError):
            data = potential_file
    if isinstance(data, (bytes, bytearray)):
        data = bytes(data).decode('latin-1')
    return data


def read_bytes(potential_file):
    """ensure_file's content as raw bytes (latin-1 for text), for native parsers."""
    if hasattr(potential_file, 'read'):
        data = potential_file.read()
    else:
        try:
            with open(potential_file, 'rb') as fh:
                return fh.read()
        except (OSError, ValueError):
            data = potential_file
    return data if isinstance(data, (bytes, bytearray)) else data.encode('latin-1')


def read_buffer(potential_file):
    """Like read_bytes, but a file on disk is memory-mapped (read-only, no
    copy): the native parsers read the page cache directly."""
    if isinstance(potential_file, str) and os.path.isfile(potential_file):
        import mmap
        with open(potential_file, 'rb') as fh:
            if os.fstat(fh.fileno()).st_size == 0:
                return b''
            return mmap.mmap(fh.fileno(), 0, access=mmap.ACCESS_READ)
    return read_bytes(potential_file)


def ensure_file(potential_file):
    """magot_smallfuncs.py:32-43: a path is opened; a string that cannot be
    opened is itself the content; a file object passes through."""
    if potential_file is None:
        return None
    return _Lines(_read_source(potential_file))


# ---------------------------------------------------------------------------
# Sequence (genome.py:781-851)
# ---------------------------------------------------------------------------

_ACGT = 'ACGT'


def _ascii_upper(t):
    """str.upper() of a Python 2 byte string: only a-z change."""
    return t.translate(_UPPER)


_UPPER = {c: c - 32 for c in range(ord('a'), ord('z') + 1)}


def _matchable(key):
    """Can ``key`` equal a triplet the reference's loop builds (1-3 upper-cased
    characters, genome.py:810-812)?"""
    return isinstance(key, str) and 1 <= len(key) <= 3 and _ascii_upper(key) == key


def _library_lut(library):
    """64-entry residue table (index c0 + 4*c1 + 16*c2) for a codon library
    that the standard translation kernel can run: every matchable key an ACGT
    triplet with a one-character value.  None for the standard code; False
    when the library needs the extended-alphabet path (_translate_general)."""
    if library is None or library is Sequence._STANDARD:
        return None
    lut = bytearray(b'X' * 64)
    for key, val in library.items():
        if not _matchable(key):
            continue
        if len(key) != 3 or any(c not in _ACGT for c in key):
            return False
        if not (isinstance(val, str) and len(val) == 1 and ord(val) < 256):
            return False
        x = _ACGT.index(key[0]) + 4 * _ACGT.index(key[1]) + 16 * _ACGT.index(key[2])
        lut[x] = ord(val)
    return bytes(lut)


def _lookup(library, triplet):
    """``library[triplet]``, 'X' on KeyError (genome.py:813-816)."""
    try:
        return library[triplet]
    except KeyError:
        return 'X'


def _same_items(a, b):
    """Two snapshots of a library's items, values compared as the symbol
    table distinguishes them (identity, or same type and equal)."""
    return len(a) == len(b) and all(
        ka == kb and (va is vb or (type(va) is type(vb) and va == vb))
        for (ka, va), (kb, vb) in zip(a, b))


_LIBRARY_TABLES = []  # [(id, items snapshot, tables)], most recent last


def _library_tables(library):
    """(chars, class256, K, values, symbol lut) of a codon library for
    magot_codon_symbols: the extended alphabet (ACGT, the other characters of
    matchable 3-character keys, 'other'), the byte -> class map, and for every
    class triplet the index of its value in ``values`` (one entry per distinct
    value).  Cached per library object while its items are unchanged, so
    get_orfs' six translate() calls build it once."""
    items = list(library.items())
    for i, (lid, snap, tables) in enumerate(_LIBRARY_TABLES):
        if lid == id(library) and _same_items(snap, items):
            _LIBRARY_TABLES.append(_LIBRARY_TABLES.pop(i))
            return tables
    chars = list(_ACGT)
    for key in library.keys():
        if _matchable(key) and len(key) == 3:
            for c in key:
                if c not in chars:
                    chars.append(c)
    K = len(chars) + 1
    if K ** 3 > 32768:
        raise NotImplementedError('codon library keys use more than 31 distinct characters')
    cls = np.full(256, K - 1, dtype=np.uint8)
    for i, c in enumerate(chars):
        if ord(c) < 256:
            cls[ord(c)] = i
    for b in range(ord('a'), ord('z') + 1):
        cls[b] = cls[b - 32]
    values, lut = [], np.zeros(K ** 3, dtype=np.uint8)
    seen = {}  # (type, value) -> index, for hashable values
    for x in range(K ** 3):
        c0, c1, c2 = x % K, (x // K) % K, x // (K * K)
        if K - 1 in (c0, c1, c2):
            v = 'X'                                    # no key holds this character
        else:
            v = _lookup(library, chars[c0] + chars[c1] + chars[c2])
        try:
            key = (type(v), v)
            j = seen.get(key)
        except TypeError:                              # unhashable value: linear scan
            key = None
            j = next((i for i, u in enumerate(values)
                      if u is v or (type(u) is type(v) and u == v)), None)
        if j is None:
            if len(values) == 256:
                raise NotImplementedError('codon library has more than 256 distinct values')
            values.append(v)
            j = len(values) - 1
            if key is not None:
                seen[key] = j
        lut[x] = j
    tables = (chars, cls, K, values, lut)
    _LIBRARY_TABLES.append((id(library), items, tables))
    del _LIBRARY_TABLES[:-8]
    return tables


def _translate_general(s, library, frame, strand, trimX):
    """Sequence.translate (genome.py:795-822) for any library and any integer
    frame.  The characters the loop visits -- positions frame .. len-1, a
    negative position p reading seq[p] -- are laid out as one string V; its
    first codon (1-3 characters: emitted where (p + frame) % 3 == 2) is looked
    up here, every full codon after it on the GPU (magot_codon_symbols, an
    extended-alphabet codon table), and the symbols mapped to the library's
    values."""
    n = len(s)
    seq = s if strand == '+' else engine.revcomp_batch([s])[0]
    if not (len(seq) > (2 + frame)):
        return None
    if not isinstance(frame, int):
        raise TypeError('range() integer start argument expected, got %s.' % type(frame).__name__)
    if frame < 0:
        if -frame > n:
            raise IndexError('string index out of range')
        V = seq[frame:] + seq
    else:
        V = seq[frame:]
    J = (2 - 2 * frame) % 3 + 1        # first emission at V position J - 1
    first = _lookup(library, _ascii_upper(V[:J]))
    body = V[J:]
    m = len(body) // 3
    chars, cls, K, values, lut = _library_tables(library)
    sym = engine.codon_symbols(V[J:J + 3 * m], cls, K, lut)
    if not isinstance(first, str):
        raise TypeError('can only concatenate str (not "%s") to str' % type(first).__name__)
    for j in sorted(set(sym), key=sym.index):   # the first non-string value in order
        if not isinstance(values[j], str):
            raise TypeError('can only concatenate str (not "%s") to str'
                            % type(values[j]).__name__)
    if all(isinstance(v, str) and len(v) == 1 and ord(v) < 256 for v in values):
        table = bytes(ord(v) for v in values) + bytes(256 - len(values))
        newseq = first + bytes(sym).translate(table).decode('latin-1')
    else:
        newseq = first + ''.join([values[j] for j in sym])
    if trimX:
        if newseq[0] == 'X':
            newseq = newseq[1:]
    return newseq


class Sequence(str):
    """DNA sequence (genome.py:781-851); every operation runs on the GPU."""

    # genome.py:795-802 (standard genetic code), TCAG-ordered
    _STANDARD = None

    def reverse_compliment(self):
        """genome.py:784-793."""
        return Sequence(engine.revcomp_batch([str(self)])[0])

    def translate(self, library=None, frame=0, strand='+', trimX=True):
        """genome.py:795-822.  ``library=None`` is the reference's default
        (standard) table.  Libraries of one-character values over ACGT
        triplets and frames >= 0 run the batch translation kernel; any other
        library (keys such as 'NNN' or 1-2 character keys matching the junk
        codon, multi-character or non-string values) or a negative frame runs
        _translate_general (extended-alphabet codon kernel)."""
        if strand not in ('+', '-'):
            raise UnboundLocalError("local variable 'seq' referenced before assignment")
        lut = _library_lut(library)
        if lut is False or not isinstance(frame, int) or frame < 0:
            lib = Sequence._STANDARD if library is None else library
            return _translate_general(str(self), lib, frame, strand, trimX)
        res = engine.translate_batch([str(self)], [frame], [strand], lut64=lut)[0]
        return _trim(res, trimX)

    def get_orfs(self, longest=False, strand='both', from_atg=False):
        """genome.py:824-851; the ``strand`` argument is shadowed (genome.py:830)."""
        peps = engine.orf6_batch([str(self)])[0]  # six-frame kernel, loop order kept
        return _orfs_from_translations(peps, longest, from_atg)


def _trim(res, trimX):
    if res is None:
        return None
    if trimX and res[0] == 'X':
        res = res[1:]
    return res


def _orfs_from_translations(peps, longest, from_atg):
    orfs = []
    cands = []
    best = 0
    for t in peps:
        if not t:
            continue
        for orf in t.split('*'):
            out = 'M' + ''.join(orf.split('M')[1:]) if from_atg else orf
            if longest:
                if len(out) > best:
                    cands.append(out)
                    best = len(out)
            else:
                orfs.append(out)
    if longest:
        return cands[-1]
    return orfs


def _standard_dict():
    aa = 'FFLLSSSSYY**CC*WLLLLPPPPHHQQRRRRIIIMTTTTNNKKSSRRVVVVAAAADDEEGGGG'
    t = 'TCAG'
    return {a + b + c: aa[16 * i + 4 * j + k]
            for i, a in enumerate(t) for j, b in enumerate(t) for k, c in enumerate(t)}


Sequence._STANDARD = _standard_dict()


# ---------------------------------------------------------------------------
# GenomeSequence (genome.py:854-877)
# ---------------------------------------------------------------------------

class GenomeSequence(dict):
    """seqid -> sequence (latin-1 ``str``).  The packed HBM copy used by the
    extraction kernels is built on first use and dropped on mutation."""

    def __init__(self, genome_sequence=None, truncate_names=False):
        dict.__init__(self)
        self._device = None
        if genome_sequence is None:
            return
        text = _read_source(genome_sequence)
        name = ''
        n = len(text)
        pos = 0
        # A record starts at every line whose first byte is '>'.
        while pos < n:
            if text[pos] == '>':
                eol = text.find('\n', pos)
                if eol < 0:
                    eol = n
                head = text[pos + 1:eol].replace('\r', '')
                if truncate_names is True:
                    head = head.split()[0]
                name = head
                pos = eol + 1
                continue
            nxt = text.find('\n>', pos)
            end = n if nxt < 0 else nxt + 1
            seq = text[pos:end].replace('\r', '').replace('\n', '')
            if seq != '':          # empty records are dropped (genome.py:870, 876)
                self[name] = seq
            pos = end

    # mutations invalidate the HBM copy
    def __setitem__(self, k, v):
        self._device = None
        dict.__setitem__(self, k, v)

    def __delitem__(self, k):
        self._device = None
        dict.__delitem__(self, k)

    def update(self, *a, **kw):
        self._device = None
        dict.update(self, *a, **kw)

    def device(self):
        """The engine.DeviceGenome of this dict (packed once, cached)."""
        if self._device is None:
            self._device = engine.device_genome(list(self.items()))
        return self._device


def _device_genome_for(seqdict):
    if isinstance(seqdict, GenomeSequence):
        return seqdict.device()
    return engine.device_genome(list(seqdict.items()))


# ---------------------------------------------------------------------------
# Deferred output strings
# ---------------------------------------------------------------------------

class _Rec(object):
    """A record's sequence: result of batch job ``job``."""
    __slots__ = ('job',)

    def __init__(self, job):
        self.job = job


class _Cat(object):
    __slots__ = ('parts',)

    def __init__(self, parts):
        self.parts = parts


class _Join(object):
    __slots__ = ('items',)

    def __init__(self, items):
        self.items = items


class _Longest(object):
    __slots__ = ('items',)

    def __init__(self, items):
        self.items = items


def _join(items):
    """'\\n'.join(items) with the reference's TypeError on None."""
    for i, it in enumerate(items):
        if it is None:
            raise TypeError('sequence item %d: expected str instance, NoneType found' % i)
    if not items:
        return ''
    if len(items) == 1:
        return items[0]
    return _Join(items)


class _Batch(object):
    """Interval lists of every record of one get_fasta call."""

    def __init__(self):
        self.genomes = []      # [(GenomeSequence, device genome)], in first-use order
        self.ex_gid = []       # genome of each interval
        self.ex_start = []
        self.ex_contig = []
        self.ex_len = []
        self.tx_begin = []
        self.tx_n = []
        self.kinds = []        # 'nuc' | 'pep'
        self.results = None

    def bind(self, seqdict):
        """(device genome, genome id) of a GenomeSequence.  One call usually
        sees one genome; annotations of several (their annotation sets bound
        to different Genomes) are gathered per genome in run()."""
        for gid, (sd, dev) in enumerate(self.genomes):
            if sd is seqdict:
                return dev, gid
        dev = _device_genome_for(seqdict)
        self.genomes.append((seqdict, dev))
        return dev, len(self.genomes) - 1

    def add(self, exons, kind):
        """exons: list of (contig_index, start, length, rc, genome id)."""
        self.tx_begin.append(len(self.ex_start))
        self.tx_n.append(len(exons))
        for ci, st, ln, rc, gid in exons:
            self.ex_start.append(st | (1 << 63) if rc else st)
            self.ex_contig.append(ci)
            self.ex_len.append(ln)
            self.ex_gid.append(gid)
        self.kinds.append(kind)
        return len(self.kinds) - 1

    def _run_genomes(self, ex, tx):
        """Records over several genomes: each genome's intervals gathered as
        one-interval pieces in one launch per genome, joined per record, and
        the protein records translated in one translate_batch launch."""
        gid = np.array(self.ex_gid, dtype=np.int64)
        piece = [None] * len(ex)
        for k, (_, dev) in enumerate(self.genomes):
            idx = np.nonzero(gid == k)[0]
            if len(idx) == 0:
                continue
            sub_tx = np.zeros(len(idx), dtype=engine.TX_DTYPE)
            sub_tx['exon_begin'] = np.arange(len(idx), dtype=np.uint64)
            sub_tx['n_exons'] = 1
            nuc, noff, _, _ = engine.extract_records(dev, ex[idx], sub_tx, engine.OUT_NUC)
            raw = nuc.tobytes().decode('latin-1') if nuc is not None else ''
            for j, e in enumerate(idx.tolist()):
                piece[e] = raw[int(noff[j]):int(noff[j + 1])]
        recs = []
        for b, n in zip(self.tx_begin, self.tx_n):
            recs.append(''.join(piece[b:b + n]))
        pep_ids = [i for i, k in enumerate(self.kinds) if k == 'pep']
        res = list(recs)
        if pep_ids:
            peps = engine.translate_batch([recs[i] for i in pep_ids], [0] * len(pep_ids),
                                          ['+'] * len(pep_ids))
            for i, t in zip(pep_ids, peps):
                res[i] = t or ''
        return res

    def run(self):
        n = len(self.kinds)
        if n == 0:
            self.results = []
            return
        ex = np.empty(len(self.ex_start), dtype=engine.EXON_DTYPE)
        ex['start_rc'] = np.array(self.ex_start, dtype=np.uint64)
        ex['contig'] = np.array(self.ex_contig, dtype=np.uint32)
        ex['len'] = np.array(self.ex_len, dtype=np.uint32)
        tx = np.zeros(n, dtype=engine.TX_DTYPE)
        tx['exon_begin'] = np.array(self.tx_begin, dtype=np.uint64)
        tx['n_exons'] = np.array(self.tx_n, dtype=np.uint32)
        if not self.genomes:      # no record has an interval: every sequence is empty
            res = [''] * n
        elif len(self.genomes) > 1:
            res = self._run_genomes(ex, tx)
        else:
            outputs = 0
            if 'nuc' in self.kinds:
                outputs |= engine.OUT_NUC
            if 'pep' in self.kinds:
                outputs |= engine.OUT_PEP
            genome = self.genomes[0][1] if self.genomes else None
            nuc, noff, pep, poff = engine.extract_records(genome, ex, tx, outputs)
            nraw = nuc.tobytes().decode('latin-1') if nuc is not None else ''
            praw = pep.tobytes().decode('latin-1') if pep is not None else ''
            noff = noff.tolist()
            poff = poff.tolist()
            res = []
            for i, kind in enumerate(self.kinds):
                if kind == 'nuc':
                    res.append(nraw[noff[i]:noff[i + 1]])
                else:
                    res.append(praw[poff[i]:poff[i + 1]])
        for i, kind in enumerate(self.kinds):
            if kind == 'pep' and res[i] and res[i][0] == 'X':  # trimX (genome.py:819-821)
                res[i] = res[i][1:]
        self.results = res

    def render(self, node):
        if self.results is None:
            self.run()
        return self._render(node)

    def _render(self, node):
        if isinstance(node, str):
            return node
        if isinstance(node, _Rec):
            return self.results[node.job]
        if isinstance(node, _Cat):
            return ''.join(self._render(p) for p in node.parts)
        if isinstance(node, _Join):
            return '\n'.join(self._render(p) for p in node.items)
        if isinstance(node, _Longest):
            by_len = {}
            for it in node.items:
                s = self._render(it)
                by_len[len(''.join(s.split('\n')[1:]))] = s
            return by_len[max(list(by_len))]
        if node is None:
            return None
        raise TypeError('bad deferred node %r' % (node,))


def _slice_interval(contig, a, b):
    """(start, length) of ``contig[a:b]`` (Python slice rules, step 1)."""
    start, stop, _ = slice(a, b).indices(len(contig))
    return start, max(0, stop - start)


# ---------------------------------------------------------------------------
# Annotation model (genome.py:524-778)
# ---------------------------------------------------------------------------

class AnnotationSet(object):
    """genome.py:524-583.  One dict per feature type as an instance attribute;
    ``aset[ID]`` searches them all."""

    def __init__(self, genome=None):
        self.gene = {}
        self.transcript = {}
        self.CDS = {}
        self.UTR = {}
        self.genome = genome

    def __getitem__(self, item):
        """genome.py:536-544: attributes in sorted (``dir``) order, the LAST
        dict holding ``item`` wins; KeyError when none does.  Python 2's
        ``dir`` of an old-style instance has no ``__dict__`` entry."""
        hit = _MISSING
        for name in sorted(self.__dict__):
            val = self.__dict__[name]
            if type(val) is dict:
                try:
                    hit = val[item]
                except (KeyError, TypeError):
                    pass
        if hit is _MISSING:
            raise KeyError(item)
        return hit

    def read_gff(self, gff, *args, **kwargs):
        """genome.py:546-548."""
        kwargs['annotation_set_to_modify'] = self
        read_gff(gff, *args, **kwargs)

    def read_exonerate(self, exonerate_output):
        """genome.py:569-570."""
        read_exonerate(exonerate_output, annotation_set_to_modify=self)

    def read_blast_csv(self, blast_csv, hierarchy=['match', 'match_part'], source='blast',
                       find_truncated_locname=False):
        """genome.py:572-573."""
        read_blast_csv(blast_csv, annotation_set_to_modify=self, hierarchy=hierarchy,
                       source=source, find_truncated_locname=find_truncated_locname)

    def read_cegma_gff(self, cegma_gff):
        """genome.py:575-576."""
        read_cegma_gff(cegma_gff, annotation_set_to_modify=self)

    def get_fasta(self, feature, seq_type='nucleotide', longest=False, genomic=False, order=None):
        """genome.py:578-582, batched: one device launch for every record.

        ``order``: 'insertion' (default) or 'py2' (CPython 2.7 dict order,
        as the reference's goldens)."""
        table = getattr(self, feature)
        keys = list(table)
        if (order or DEFAULT_ORDER) == 'py2':
            keys = order_after_copies(keys, self.__dict__.get('_magot_copies', 0))
        elif (order or DEFAULT_ORDER) != 'insertion':
            raise ValueError("order must be 'insertion' or 'py2'")
        batch = _Batch()
        nodes = []
        for k in keys:
            obj = table[k]
            if not isinstance(obj, ParentAnnotation):
                raise AttributeError("%s instance has no attribute 'get_fasta'"
                                     % type(obj).__name__)
            nodes.append(obj._plan_fasta(batch, seq_type, longest, genomic, 'ID'))
        return batch.render(_join(nodes))


_MISSING = object()


class BaseAnnotation(object):
    """genome.py:586-645 (extraction part)."""

    def __init__(self, ID, seqid, coords, feature_type, parent=None, strand='.',
                 other_attributes={}, annotation_set=None):
        self.ID = ID
        self.seqid = seqid
        self.coords = coords
        self.feature_type = feature_type
        self.annotation_set = annotation_set
        for attribute in other_attributes:
            setattr(self, attribute, other_attributes[attribute])
        self.parent = parent
        self.strand = strand

    def get_coords(self):
        return self.coords

    def _plan_seq(self, batch):
        """genome.py:603-614 as an interval (contig, start, len, rc) or None
        (after the reference's diagnostics)."""
        try:
            if self.strand == '+' or self.strand == '.':
                rc = False
            elif self.strand == '-':
                rc = True
            else:
                _emit(self.ID + ' has invalid strand value "' + self.strand + '"')
                return None
            seqs = self.annotation_set.genome.genome_sequence
            contig = seqs[self.seqid]
            start, length = _slice_interval(contig, self.coords[0] - 1, self.coords[1])
            dev, gid = batch.bind(seqs)
            return (dev.index[self.seqid], start, length, rc, gid)
        except (NotImplementedError, engine.MagotError):
            raise  # device / build failures are not reference semantics: fail loudly
        except Exception:
            _emit(_MSG_GETSEQ, self.seqid)
        return None

    def get_seq(self):
        """genome.py:603-614 -- one interval, gathered on the GPU."""
        batch = _Batch()
        iv = self._plan_seq(batch)
        if iv is None:
            return None
        job = batch.add([iv], 'nuc')
        return Sequence(batch.render(_Rec(job)))


class ParentAnnotation(object):
    """genome.py:649-731 (extraction part)."""

    def __init__(self, ID, seqid, feature_type, child_list=[], parent=None, strand='.',
                 annotation_set=None, other_attributes={}):
        self.ID = ID
        self.seqid = seqid
        self.feature_type = feature_type
        self.child_list = list(child_list)
        self.parent = parent
        self.annotation_set = annotation_set
        self.strand = strand
        for attribute in other_attributes:
            setattr(self, attribute, other_attributes[attribute])

    def get_coords(self):
        """genome.py:663-675."""
        if len(self.child_list) > 0 and self.annotation_set is not None:
            pts = []
            for child in self.child_list:
                obj = self.annotation_set[child]
                if isinstance(obj, ParentAnnotation):
                    pts = pts + list(obj.get_coords())
                elif isinstance(obj, BaseAnnotation):
                    pts = pts + list(obj.coords)
                else:
                    _emit("for some reason you have children in ParentAnnotation " + self.ID +
                          " which are neither                     ParentAnnotation objects nor "
                          "BaseAnnotation object. Get your act together")
            return (min(pts), max(pts))
        return None

    def get_fasta(self, seq_type='nucleotide', longest=False, genomic=False, name_from='ID'):
        """genome.py:677-731 -- the records of this feature, extracted on the GPU."""
        batch = _Batch()
        node = self._plan_fasta(batch, seq_type, longest, genomic, name_from)
        return batch.render(node)

    def _plan_fasta(self, batch, seq_type, longest, genomic, name_from):
        aset = self.annotation_set
        if genomic == True:  # noqa: E712 (reference compares with ==)
            if aset.genome is not None:
                span = self.get_coords()
                seqs = aset.genome.genome_sequence
                contig = seqs[self.seqid]
                head = '>' + self.ID + '\n'
                start, length = _slice_interval(contig, span[0] - 1, span[1])
                dev, gid = batch.bind(seqs)
                job = batch.add([(dev.index[self.seqid], start, length, False, gid)], 'nuc')
                return _Cat([head, _Rec(job), '\n'])
            return None
        if not (len(self.child_list) > 0 and aset is not None):
            return ''
        if aset.genome is None:
            return ''
        records = []
        first = aset[self.child_list[0]]
        if type(first).__name__ == 'BaseAnnotation' or isinstance(first, BaseAnnotation):
            by_coords = {}
            for child in self.child_list:
                obj = aset[child]
                try:
                    if not isinstance(obj, BaseAnnotation):
                        raise AttributeError('get_seq')
                    iv = obj._plan_seq(batch)
                    by_coords[obj.coords] = iv
                except AttributeError:
                    _emit(_MSG_MIXED, self.ID)
                strand = obj.strand
            keys = sorted(by_coords)
            if strand == '-':
                keys.reverse()
            parts = [by_coords[k] for k in keys]
            for i, p in enumerate(parts):
                if p is None:
                    raise TypeError('sequence item %d: expected str instance, NoneType found' % i)
            total = sum(p[2] for p in parts)
            if seq_type == 'nucleotide':
                seq = _Rec(batch.add(parts, 'nuc'))
            elif seq_type == 'protein':
                if not total > 2:      # translate() returns None (genome.py:810)
                    _ = '>' + self.__dict__[name_from] + '\n'
                    raise TypeError('can only concatenate str (not "NoneType") to str')
                seq = _Rec(batch.add(parts, 'pep'))
            else:
                _emit(seq_type + ' is not valid seq_type. Please specify "protein" or '
                      '"nucleotide".')
                raise UnboundLocalError("local variable 'new_seq' referenced before assignment")
            records.append(_Cat(['>' + self.__dict__[name_from] + '\n', seq]))
        else:
            for child in self.child_list:
                obj = aset[child]
                try:
                    if not isinstance(obj, ParentAnnotation):
                        raise AttributeError('get_fasta')
                    sub = obj._plan_fasta(batch, seq_type, False, False, name_from)
                    if sub != '':
                        records.append(sub)
                except AttributeError:
                    _emit(_MSG_MIXED, self.ID)
        if longest == True:  # noqa: E712
            if not records:
                raise ValueError('max() arg is an empty sequence')
            return _Longest(records)
        return _join(records)


# ---------------------------------------------------------------------------
# GFF3 / GTF reader (genome.py:242-415)
# ---------------------------------------------------------------------------

_PRESETS = ('augustus', 'RepeatMasker', 'CEGMA')


def read_gff(gff, annotation_set_to_modify=None, base_features=['CDS', 'match_part', 'similarity',
                                                                  'region'],
             features_to_ignore=['exon'], gff_version='auto', parents_hierarchy=[],
             features_to_replace=[], IDfield='ID', parent_field='Parent', presets=None):
    """genome.py:242-415.  Same acceptance rule (first char not '#', exactly 8
    tabs), version sniffing on the first accepted line, ID synthesis and
    de-duplication, parent creation/linking and Base/Parent typing."""
    if presets == 'augustus':
        features_to_ignore = ['gene', 'transcript', 'stop_codon', 'terminal', 'internal',
                              'initial', 'intron', 'start_codon', 'single']
        parent_field = None
        parents_hierarchy = ['transcript_id', 'gene_id']
        IDfield = None
    elif presets == 'RepeatMasker':
        parent_field = None
        IDfield = 'Target'
    elif presets == 'CEGMA':
        # genome.py:265-266: the preset text indexes a list with a tuple
        raise TypeError('list indices must be integers, not tuple')
    version = gff_version
    lines = ensure_file(gff)
    swaps = [('\n', ''), ('\r', '')]
    for pair in features_to_replace:
        swaps.append(('\t' + pair[0] + '\t', '\t' + pair[1] + '\t'))
    aset = AnnotationSet() if annotation_set_to_modify is None else annotation_set_to_modify
    renamed = {}
    for raw in lines:
        if raw[0] == '#' or raw.count('\t') != 8:
            continue
        line = raw
        for old, new in swaps:
            line = line.replace(old, new)
        cols = line.split('\t')
        tags_text = cols[8]
        if version == 'auto':
            if '=' in tags_text:
                version = 3
            else:
                version = 2
                if IDfield is not None and parents_hierarchy == [] and \
                        (' ' + IDfield + ' ') not in (' ' + tags_text.replace(';', ' ')):
                    IDfield = None
                    parent_field = None
                    if 'gene_id' in tags_text and 'transcript_id' in tags_text:
                        parents_hierarchy = ['transcript_id', 'gene_id']
                    elif 'gene_id' in tags_text:
                        parents_hierarchy = ['gene_id']
        seqid = cols[0]
        extra = {'source': cols[1]}
        ftype = cols[2]
        if ftype in features_to_ignore:
            continue
        lo, hi = int(cols[3]), int(cols[4])
        coords = (lo, hi) if lo <= hi else (hi, lo)
        try:
            extra['score'] = float(cols[5])
        except ValueError:
            pass
        strand = cols[6]
        if cols[7] in ('0', '1', '2'):
            extra['phase'] = int(cols[7])
        tags = {}
        for item in tags_text.split(';'):
            if item == '':
                continue
            if parent_field == '':
                tags[''] = item
            elif version == 2:
                words = item.split()
                if '"' in item:
                    tags[words[0]] = item.split('"')[1]
                elif len(words) > 1:
                    tags[words[0]] = words[1]
                else:
                    _emit(item)
                    return None
            elif version == 3:
                kv = item.split('=')
                tags[kv[0]] = kv[1]
        parent = None
        if parent_field is not None:
            parent = tags.get(parent_field)
        elif parents_hierarchy != []:
            for key in parents_hierarchy:
                if key in tags:
                    parent = tags[key]
                    break
        if IDfield is not None:
            if IDfield in tags:
                ID = tags[IDfield]
            elif parent is not None:
                ID = parent + '-' + ftype
            else:
                ID = None
        elif parent is not None:
            ID = parent + '-' + ftype
        else:
            ID = seqid + '-' + ftype + cols[3]
        # de-duplicate against every feature type; the new name is not re-checked
        try:
            aset[ID]
            if ID in renamed:
                renamed[ID] += 1
                ID = ID + '-' + str(renamed[ID])
            else:
                renamed[ID] = 2
                ID = ID + '2'
        except KeyError:
            pass
        if parent is not None:
            child = ID
            depth = len(parents_hierarchy)
            for level, key in enumerate(parents_hierarchy):
                if key not in tags:
                    continue
                pid = tags[key]
                ptype = key.split('_')[0]
                grand = None
                if level != depth - 1:
                    for up in parents_hierarchy[level + 1:]:
                        if up in tags:
                            grand = tags[up]
                table = aset.__dict__.setdefault(ptype, {})
                if pid in table:
                    if child not in table[pid].child_list:
                        table[pid].child_list.append(child)
                else:
                    table[pid] = ParentAnnotation(pid, seqid, ptype, child_list=[child],
                                                  parent=grand, strand=strand,
                                                  annotation_set=aset)
                child = pid
            try:
                holder = aset[parent]
            except KeyError:
                _emit(_MSG_ORPHAN, ID, parent)
                return None
            if ID not in holder.child_list:
                holder.child_list.append(ID)
        for key in tags:
            if key not in (IDfield, parent_field):
                extra[key] = tags[key]
        table = aset.__dict__.setdefault(ftype, {})
        if ftype in base_features:
            table[ID] = BaseAnnotation(ID, seqid, coords, ftype, parent, strand, extra, aset)
        else:
            table[ID] = ParentAnnotation(ID, seqid, ftype, [], parent, strand, aset, extra)
    if annotation_set_to_modify is None:
        # genome.py:415 returns copy.deepcopy(annotation_set): same content;
        # under Python 2 the copy re-inserts every dict (py2order).
        aset.__dict__['_magot_copies'] = aset.__dict__.get('_magot_copies', 0) + 1
        return aset


# ---------------------------------------------------------------------------
# Aligner outputs as match / match_part annotations (genome.py:32-121,
# 418-499): the inputs of genome_tools blast_csv2fasta / exonerate2fasta,
# which extract them through the same get_fasta path.
# ---------------------------------------------------------------------------

def vulgar2gff(vulgarlist, feature_types=['match', 'match_part'], source='exonerate'):
    """genome.py:32-86: one exonerate vulgar record -> GFF lines (a match
    line, then a match_part line per run of M/S/G/F operations).  Reference
    quirks kept: the match_part bounds are min/max over the coordinate
    STRINGS (lexicographic), and a '-' target keeps its start and moves its
    end up by one."""
    qname = vulgarlist[0] + '-against-' + vulgarlist[4]
    tname = vulgarlist[4]
    tstart = vulgarlist[5]
    tend = vulgarlist[6]
    tstrand = vulgarlist[7]
    score = vulgarlist[8]
    trips = vulgarlist[9:]
    addfeat = False
    idnum = 1
    if tstrand == '+':
        tpos = int(tstart) + 1
    else:
        tpos = int(tstart)
        tend = str(int(tend) + 1)
    lines = ['\t'.join([tname, source, feature_types[0], str(tpos), tend, score, tstrand, '.',
                        'ID=' + qname])]
    head = coords = None
    for i in range(len(trips)):
        field = trips[i]
        if i % 3 == 0:
            if field in ('M', 'S', 'G', 'F'):
                if not addfeat:
                    addfeat = True
                    head = [tname, source, feature_types[1]]
                    coords = [str(tpos)]
            elif addfeat:
                lines.append('\t'.join(head + [min(coords), max(coords), '.', tstrand, '.',
                                               'ID=' + qname + '_' + feature_types[1] + str(idnum) +
                                               ';Parent=' + qname]))
                idnum += 1
                addfeat = False
        if i % 3 == 2:
            if tstrand == '+':
                tpos += int(field)
            elif tstrand == '-':
                tpos -= int(field)
            if addfeat:
                if tstrand == '+':
                    coords.append(str(tpos - 1))
                elif tstrand == '-':
                    coords.append(str(tpos + 1))
    if addfeat:
        lines.append('\t'.join(head + [min(coords), max(coords), '.', tstrand, '.',
                                       'ID=' + qname + '_' + feature_types[1] + str(idnum) +
                                       ';Parent=' + qname]))
    return '\n'.join(lines)


def read_exonerate(exonerate_output, annotation_set_to_modify=None):
    """genome.py:88-121: the Query / Target header lines name the next vulgar
    record (':[revcomp]' / '[revcomp]' stripped from the target, one trailing
    space dropped); a repeated query-target pair gets a numbered query name.
    The GFF goes through read_gff into the set (no copy)."""
    aset = AnnotationSet() if annotation_set_to_modify is None else annotation_set_to_modify
    gfflines = []
    seen = {}
    qname = ''
    tname = ''
    for raw in ensure_file(exonerate_output):
        line = raw.replace('\r', '').replace('\n', '')
        if line[:16] == '         Query: ':
            qname = line[16:]
        elif line[:16] == '        Target: ':
            tname = line[16:].replace(':[revcomp]', '').replace('[revcomp]', '')
            if tname[-1] == ' ':
                tname = tname[:-1]
        elif line[:8] == 'vulgar: ':
            vl = line[8:].split()
            vl[0] = qname
            vl[4] = tname
            key = vl[0] + '-against-' + vl[4]
            if key in seen:
                vl[0] = vl[0] + str(seen[key])
                seen[key] = seen[key] + 1
            else:
                seen[key] = 1
            gfflines.append(vulgar2gff(vl))
    read_gff('\n'.join(gfflines), annotation_set_to_modify=aset)
    if annotation_set_to_modify is None:
        return aset


def read_cegma_gff(cegma_gff, annotation_set_to_modify=None):
    """genome.py:418-422 (the CEGMA preset raises, see read_gff)."""
    aset = read_gff(cegma_gff, annotation_set_to_modify=annotation_set_to_modify, presets='CEGMA')
    if annotation_set_to_modify is None:
        return aset


def read_blast_csv(blast_csv, annotation_set_to_modify=None, hierarchy=['match', 'match_part'],
                   source='blast', find_truncated_locname=False):
    """genome.py:425-499: BLAST -outfmt 10 rows (more than 8 fields) ->
    one base feature (hierarchy[-1]) per row under a chain of parents named
    ID + '-' + parent type.  Subject coordinates give the strand (start <
    end: '+', else '-').  A repeated query ID becomes ID-1, ID-2, ..."""
    rows = ensure_file(blast_csv)
    aset = AnnotationSet() if annotation_set_to_modify is None else annotation_set_to_modify
    gen = {}
    feature_type = hierarchy[-1]
    chain = hierarchy[:-1]
    chain.reverse()
    if feature_type not in aset.__dict__:
        setattr(aset, feature_type, {})
    if find_truncated_locname:
        if aset.genome is None:
            _emit('"warning: find_truncated_locname" was set to true, but annotation set has no '
                  'associated genome object so this cannot be done')
            find_truncated_locname = False
        else:
            genome_seqids = aset.genome.get_seqids()
    for raw in rows:
        line = raw.replace('\r', '').replace('\n', '')
        fields = line.split(',')
        if len(fields) > 8:
            seqid = fields[1]
            if find_truncated_locname and seqid not in genome_seqids:
                for full in genome_seqids:
                    if seqid == full.split()[0]:
                        seqid = full
                        break
            tstart = int(fields[8])
            tend = int(fields[9])
            if tstart < tend:
                coords, strand = (tstart, tend), '+'
            else:
                coords, strand = (tend, tstart), '-'
            score = fields[11]
            base = fields[0]
            table = getattr(aset, feature_type)
            if base in table:
                ID = base + '-' + str(gen[base])
                gen[base] = gen[base] + 1
                while ID in table:
                    ID = base + '-' + str(gen[base])
                    gen[base] = gen[base] + 1
            else:
                ID = base
                gen[base] = 1
            extra = {'evalue': fields[10], 'score': score}
            parent = ID + '-' + chain[0]
            child = ID
            for level in range(len(chain)):
                ptype = chain[level]
                if ptype not in aset.__dict__:
                    setattr(aset, ptype, {})
                up = ID + '-' + chain[level + 1] if level != len(chain) - 1 else None
                aset.__dict__[ptype][ID + '-' + ptype] = ParentAnnotation(
                    ID + '-' + ptype, seqid, ptype, [child], up, strand, aset, other_attributes={})
                child = ID + '-' + ptype
            getattr(aset, feature_type)[ID] = BaseAnnotation(ID, seqid, coords, feature_type,
                                                             parent, strand, extra, aset)
    if annotation_set_to_modify is None:
        return aset


# ---------------------------------------------------------------------------
# Genome facade (genome.py:880-978)
# ---------------------------------------------------------------------------

class Genome(object):
    """genome.py:880-978 (sequence + annotations)."""

    def __init__(self, genome_sequence=None, annotations=None, varients=None,
                 annotation_format='annotation_set', truncate_names=False):
        if genome_sequence.__class__.__name__ == 'GenomeSequence' or genome_sequence is None:
            self.genome_sequence = genome_sequence
        else:
            self.genome_sequence = GenomeSequence(genome_sequence, truncate_names=truncate_names)
        if annotations is not None:
            # genome.py:889 compares against the misspelt "AnotationSet", so an
            # AnnotationSet object with the default format is never attached.
            if annotations.__class__.__name__ == 'AnotationSet' and \
                    annotation_format == 'annotation_set':
                self.annotations = annotations
                self.annotations.genome = self
            elif annotation_format == 'gff3':
                self.annotations = read_gff(annotations)
                self.annotations.genome = self
            elif annotation_format == 'cegma_gff':
                self.annotations = read_cegma_gff(annotations)
                self.annotations.genome = self
            elif annotation_format == 'blast_csv':
                self.annotations = read_blast_csv(annotations)
                self.annotations.genome = self
            elif annotation_format == 'exonerate_output':
                self.annotations = read_exonerate(annotations)
                self.annotations.genome = self
        else:
            self.annotations = annotations

    def get_scaffold_fasta(self, seqid):
        return '>' + seqid + '\n' + self.genome_sequence[seqid]

    def get_genome_fasta(self, remove_spaces=False):
        out = []
        for seqid in self.genome_sequence:
            head = seqid.split()[0] if remove_spaces else seqid
            out.append('>' + head + '\n' + self.genome_sequence[seqid])
        return '\n'.join(out)

    def get_seqids(self, from_annotations=False):
        ids = []
        if self.genome_sequence is not None:
            ids.extend(self.genome_sequence)
        if self.annotations is not None and from_annotations:
            raise NotImplementedError('from_annotations is outside the extraction path')
        return ids

    def read_exonerate(self, exonerate_output):
        """genome.py:950-955."""
        if self.annotations is not None:
            self.annotations.read_exonerate(exonerate_output)
        else:
            self.annotations = read_exonerate(exonerate_output)
            self.annotations.genome = self

    def read_blast_csv(self, blast_csv, hierarchy=['match', 'match_part'], source='blast',
                       find_truncated_locname=False):
        """genome.py:957-961."""
        if self.annotations is None:
            self.annotations = AnnotationSet()
            self.annotations.genome = self
        self.annotations.read_blast_csv(blast_csv, hierarchy=hierarchy, source=source,
                                        find_truncated_locname=find_truncated_locname)

    def read_cegma_gff(self, cegma_gff):
        """genome.py:963-968."""
        if self.annotations is not None:
            self.annotations.read_cegma_gff(cegma_gff)
        else:
            self.annotations = read_cegma_gff(cegma_gff)
            self.annotations.genome = self

    def read_gff(self, gff, *args, **kwargs):
        """genome.py:970-975."""
        if self.annotations is not None:
            self.annotations.read_gff(gff, *args, **kwargs)
        else:
            self.annotations = read_gff(gff, *args, **kwargs)
            self.annotations.genome = self


__all__ = ['Genome', 'GenomeSequence', 'AnnotationSet', 'BaseAnnotation', 'ParentAnnotation',
           'Sequence', 'read_gff', 'read_exonerate', 'read_blast_csv', 'read_cegma_gff',
           'vulgar2gff', 'ensure_file', 'DEFAULT_ORDER']
