"""Device-level objects over the C ABI: packed genome, extraction plan, and the
raw-sequence batch ops.  Everything here runs on the GPU through libmagot.so;
there is no host compute path."""

import ctypes
import os

import numpy as np

from . import _lib
from ._lib import (EXON_DTYPE, TX_DTYPE, OUT_NUC, OUT_PEP, OUT_GENOME_ORDER, MagotError, check,
                   ptr)


def _as_bytes(s):
    if isinstance(s, (bytes, bytearray, memoryview)):
        return bytes(s)
    return s.encode('latin-1')


def _text_view(s):
    """A uint8 view of text for the native parsers without copying: bytes,
    bytearray, mmap (genome.read_buffer) or numpy; str is encoded."""
    if isinstance(s, str):
        s = s.encode('latin-1')
    if isinstance(s, np.ndarray):
        return np.ascontiguousarray(s).view(np.uint8).reshape(-1)
    return np.frombuffer(s, dtype=np.uint8)


def _text_ptr(view):
    return view.ctypes.data if len(view) else None


class DeviceGenome(object):
    """A GenomeSequence packed into HBM (magot_genome_load).

    ``contigs`` is a list of (name, sequence) pairs; sequences are ``str``
    (latin-1, one char per byte), ``bytes`` or uint8 numpy arrays.
    """

    def __init__(self, contigs, ctx=None, pack='device'):
        """``pack``: 'device' (default: raw bytes streamed to HBM once, packed
        by kernels) or 'host' (pack.cpp, then the plane uploaded)."""
        if pack not in ('device', 'host'):
            raise ValueError(pack)
        self.ctx = ctx or _lib.default_context()
        names = []
        bufs = []
        for name, seq in contigs:
            names.append(name)
            if isinstance(seq, np.ndarray):  # a uint8 view (no copy)
                bufs.append(np.ascontiguousarray(seq).view(np.uint8).reshape(-1))
            else:
                bufs.append(np.frombuffer(_as_bytes(seq), dtype=np.uint8))
        n = len(bufs)
        self.names = names
        self.index = {nm: i for i, nm in enumerate(names)}
        self.lengths = np.array([len(b) for b in bufs], dtype=np.uint64)
        ptrs = (ctypes.POINTER(ctypes.c_uint8) * max(n, 1))()
        for i, b in enumerate(bufs):
            if len(b):
                ptrs[i] = b.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))
        lens = np.ascontiguousarray(self.lengths)
        h = ctypes.c_void_p()
        L = _lib.lib()
        flags = _lib.PACK_HOST if pack == 'host' else 0
        check(L.magot_genome_load_ex(self.ctx.handle, ptrs, lens.ctypes.data_as(_lib._u64p), n,
                                     flags, ctypes.byref(h)), 'magot_genome_load')
        self.handle = h
        self._keepalive = None
        self._stats()

    def _check_contigs(self):
        """The caller's contig lengths against the genome's own table (a
        replica built from a meta blob of another genome is refused)."""
        n = ctypes.c_uint32()
        nl = ctypes.c_uint64()
        L = _lib.lib()
        check(L.magot_genome_contigs(self.handle, ctypes.byref(n), None, None, 0,
                                     ctypes.byref(nl)), 'magot_genome_contigs')
        lens = np.zeros(max(n.value, 1), dtype=np.uint64)
        check(L.magot_genome_contigs(self.handle, ctypes.byref(n), ptr(lens), None, 0,
                                     ctypes.byref(nl)), 'magot_genome_contigs')
        if n.value != len(self.names) or not np.array_equal(lens[:n.value], self.lengths):
            self.close()
            raise MagotError('genome replica: %d contigs in the meta blob, %d names / lengths '
                             'given, or their lengths differ' % (n.value, len(self.names)))

    def _stats(self):
        tb, nr, db = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        check(_lib.lib().magot_genome_stats(self.handle, ctypes.byref(tb), ctypes.byref(nr),
                                            ctypes.byref(db)), 'magot_genome_stats')
        self.total_bases = tb.value
        self.n_exception_runs = nr.value
        self.device_bytes = db.value

    # -- replication (magot_genome_export / copy_arena / attach) -------------
    def export(self):
        """(meta bytes, arena size in bytes) of the packed genome."""
        L = _lib.lib()
        n, ab = ctypes.c_uint64(), ctypes.c_uint64()
        check(L.magot_genome_export(self.handle, None, 0, ctypes.byref(n), ctypes.byref(ab)),
              'magot_genome_export')
        meta = np.empty(n.value, dtype=np.uint8)
        check(L.magot_genome_export(self.handle, ptr(meta), n.value, ctypes.byref(n),
                                    ctypes.byref(ab)), 'magot_genome_export')
        return meta.tobytes(), ab.value

    def wire_ranges(self):
        """[(offset, length)] of the arena a replica must receive (the forward
        plane, then runs + directory); the mirror is rebuilt on attach."""
        off = np.zeros(2, dtype=np.uint64)
        ln = np.zeros(2, dtype=np.uint64)
        n = ctypes.c_uint32()
        check(_lib.lib().magot_genome_wire_ranges(self.handle, off.ctypes.data_as(_lib._u64p),
                                                  ln.ctypes.data_as(_lib._u64p), ctypes.byref(n)),
              'magot_genome_wire_ranges')
        return [(int(off[k]), int(ln[k])) for k in range(n.value)]

    def wire_size(self):
        """Bytes of the compact replica image (magot_genome_wire_export)."""
        n = ctypes.c_uint64()
        check(_lib.lib().magot_genome_wire_export(self.handle, None, 0, ctypes.byref(n)),
              'magot_genome_wire_export')
        return n.value

    def wire_export(self, dst_dev_ptr, cap):
        """Write the compact replica image (2-bit codes, soft-mask runs,
        exception runs) into caller device memory of ``cap`` bytes; returns
        its size."""
        n = ctypes.c_uint64()
        check(_lib.lib().magot_genome_wire_export(self.handle, ctypes.c_void_p(dst_dev_ptr),
                                                  int(cap), ctypes.byref(n)),
              'magot_genome_wire_export')
        return n.value

    @classmethod
    def from_wire(cls, meta, wire_dev_ptr, wire_bytes, names, lengths, ctx=None):
        """A genome rebuilt on this device from a replica image in device
        memory (magot_genome_wire_import); it owns its arena, and the image
        can be freed afterwards."""
        self = cls.__new__(cls)
        self.ctx = ctx or _lib.default_context()
        self.names = list(names)
        self.index = {nm: i for i, nm in enumerate(self.names)}
        self.lengths = np.asarray(lengths, dtype=np.uint64)
        self._keepalive = None
        m = np.frombuffer(meta, dtype=np.uint8)
        h = ctypes.c_void_p()
        check(_lib.lib().magot_genome_wire_import(self.ctx.handle, ptr(m), len(m),
                                                  ctypes.c_void_p(wire_dev_ptr), int(wire_bytes),
                                                  ctypes.byref(h)), 'magot_genome_wire_import')
        self.handle = h
        self._check_contigs()
        self._stats()
        return self

    def copy_arena(self, dst_dev_ptr):
        """D2D copy of the packed arena to caller device memory (an address)."""
        check(_lib.lib().magot_genome_copy_arena(self.handle, ctypes.c_void_p(dst_dev_ptr)),
              'magot_genome_copy_arena')

    @classmethod
    def attach(cls, meta, arena_dev_ptr, names, lengths, ctx=None, keepalive=None, wire=False):
        """A genome over caller device memory that holds a broadcast arena.
        ``keepalive`` (e.g. the tensor owning the memory) lives as long as this.
        ``wire=True``: the memory holds only the wire ranges; the mirror plane
        is rebuilt on this device (magot_genome_attach_wire)."""
        self = cls.__new__(cls)
        self.ctx = ctx or _lib.default_context()
        self.names = list(names)
        self.index = {nm: i for i, nm in enumerate(self.names)}
        self.lengths = np.asarray(lengths, dtype=np.uint64)
        self._keepalive = keepalive
        m = np.frombuffer(meta, dtype=np.uint8)
        h = ctypes.c_void_p()
        fn = _lib.lib().magot_genome_attach_wire if wire else _lib.lib().magot_genome_attach
        check(fn(self.ctx.handle, ptr(m), len(m), ctypes.c_void_p(arena_dev_ptr), ctypes.byref(h)),
              'magot_genome_attach')
        self.handle = h
        self._check_contigs()
        self._stats()
        return self

    def close(self):
        if getattr(self, 'handle', None):
            _lib.lib().magot_genome_destroy(self.handle)
            self.handle = None
        self._keepalive = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# One device plane addresses < 4 Gbases (32-bit window offsets, extract.hip);
# a larger genome is packed as several planes (PartitionedGenome).  The C side
# refuses a plane whose packed span (kOrigin=64 pad bases + bases + 256) reaches
# 0xFFFFFFF0 (magot_genome_load), so the part size is clamped below that.
PLANE_LIMIT = 0xFFFFFFF0 - 64 - 256 - 1
PART_BASES = min(int(os.environ.get('MAGOT_GENOME_PART_BASES', '3500000000')), PLANE_LIMIT)


def plan_parts(lengths, limit=None):
    """Contigs (in order) -> part index per contig: consecutive contigs share
    a part while its bases stay <= limit.  A contig above the limit cannot be
    packed (MagotError)."""
    limit = PART_BASES if limit is None else limit
    part = np.zeros(len(lengths), dtype=np.int64)
    k, acc = 0, 0
    for i, n in enumerate(int(x) for x in lengths):
        if n > limit:
            raise MagotError('contig %d has %d bases: above the %d-base device plane' %
                             (i, n, limit))
        if acc and acc + n > limit:
            k, acc = k + 1, 0
        part[i] = k
        acc += n
    return part


class PartitionedGenome(object):
    """A genome above one device plane: contigs cut into parts (plan_parts),
    each packed into its own HBM arena.  Extraction over it runs one plan per
    part (extract_records)."""

    def __init__(self, contigs, ctx=None, limit=None):
        contigs = list(contigs)
        self.ctx = ctx or _lib.default_context()
        self.names = [n for n, _ in contigs]
        self.index = {nm: i for i, nm in enumerate(self.names)}
        self.lengths = np.array([len(s) for _, s in contigs], dtype=np.uint64)
        self.part_of = plan_parts(self.lengths, limit)
        n_parts = int(self.part_of.max()) + 1 if len(contigs) else 0
        self.local = np.zeros(len(contigs), dtype=np.int64)
        self.parts = []
        for k in range(n_parts):
            idx = np.nonzero(self.part_of == k)[0]
            self.local[idx] = np.arange(len(idx))
            self.parts.append(DeviceGenome([contigs[i] for i in idx], ctx=self.ctx))
        self.total_bases = int(self.lengths.sum())

    def close(self):
        for g in self.parts:
            g.close()
        self.parts = []


def device_genome(contigs, ctx=None):
    """DeviceGenome, or PartitionedGenome above PART_BASES bases."""
    contigs = list(contigs)
    if sum(len(s) for _, s in contigs) > PART_BASES:
        return PartitionedGenome(contigs, ctx=ctx)
    return DeviceGenome(contigs, ctx=ctx)


def extract_records(genome, exons, txs, outputs=OUT_NUC | OUT_PEP):
    """ExtractionPlan(genome, exons, txs, outputs).run() over either genome
    kind.  On a PartitionedGenome: one plan (one launch) per part; a record
    whose intervals lie in two parts is gathered as one-interval pieces in
    their parts, joined, and translated in one translate_batch launch."""
    if not isinstance(genome, PartitionedGenome):
        plan = ExtractionPlan(genome, exons, txs, outputs)
        try:
            return plan.run()
        finally:
            plan.close()
    exons = np.ascontiguousarray(exons, dtype=EXON_DTYPE)
    txs = np.ascontiguousarray(txs, dtype=TX_DTYPE)
    T = len(txs)
    begin = txs['exon_begin'].astype(np.int64)
    count = txs['n_exons'].astype(np.int64)
    ex_part = genome.part_of[exons['contig'].astype(np.int64)] if len(exons) else \
        np.zeros(0, np.int64)
    rec_part = np.zeros(T, dtype=np.int64)
    cross = np.zeros(T, dtype=bool)
    for t in np.nonzero(count > 0)[0]:
        ps = ex_part[begin[t]:begin[t] + count[t]]
        rec_part[t] = ps[0]
        cross[t] = bool((ps != ps[0]).any())
    rec_len = np.zeros(T, dtype=np.int64)
    if len(exons):
        cs = np.concatenate([[0], np.cumsum(exons['len'].astype(np.int64))])
        rec_len = cs[begin + count] - cs[begin]
    noff = np.zeros(T + 1, dtype=np.uint64)
    np.cumsum(rec_len, out=noff[1:])
    want_pep = bool(outputs & OUT_PEP)
    pep_len = rec_len // 3
    poff = np.zeros(T + 1, dtype=np.uint64)
    np.cumsum(pep_len, out=poff[1:])
    nuc = np.empty(int(noff[-1]), dtype=np.uint8) if outputs & OUT_NUC or cross.any() else None
    pep = np.empty(int(poff[-1]), dtype=np.uint8) if want_pep else None
    for k, part in enumerate(genome.parts):
        whole = np.nonzero((rec_part == k) & ~cross)[0]
        pieces = [e for t in np.nonzero(cross)[0]
                  for e in range(begin[t], begin[t] + count[t]) if ex_part[e] == k]
        if len(whole) == 0 and not pieces:
            continue
        sub_ex = [exons[begin[t]:begin[t] + count[t]] for t in whole] + \
            [exons[e:e + 1] for e in pieces]
        sub_ex = np.concatenate(sub_ex) if sub_ex else np.zeros(0, EXON_DTYPE)
        sub_ex['contig'] = genome.local[sub_ex['contig'].astype(np.int64)]
        cnt = np.concatenate([count[whole], np.ones(len(pieces), np.int64)])
        sub_tx = np.zeros(len(cnt), dtype=TX_DTYPE)
        sub_tx['n_exons'] = cnt
        sub_tx['exon_begin'] = np.cumsum(cnt) - cnt
        sub_out = outputs | (OUT_NUC if pieces else 0)
        n_k, no_k, p_k, po_k = extract_records(part, sub_ex, sub_tx, sub_out)
        for i, t in enumerate(whole):
            if nuc is not None and n_k is not None:
                nuc[int(noff[t]):int(noff[t + 1])] = n_k[int(no_k[i]):int(no_k[i + 1])]
            if want_pep:
                pep[int(poff[t]):int(poff[t + 1])] = p_k[int(po_k[i]):int(po_k[i + 1])]
        piece_bytes = {}
        for j, e in enumerate(pieces):
            i = len(whole) + j
            piece_bytes[e] = n_k[int(no_k[i]):int(no_k[i + 1])]
        for t in np.nonzero(cross)[0]:
            o = int(noff[t])
            for e in range(begin[t], begin[t] + count[t]):
                ln = int(exons['len'][e])
                if e in piece_bytes:
                    nuc[o:o + ln] = piece_bytes[e]
                o += ln
    if want_pep and cross.any():
        ids = np.nonzero(cross)[0]
        seqs = [nuc[int(noff[t]):int(noff[t + 1])].tobytes().decode('latin-1') for t in ids]
        peps = translate_batch(seqs, [0] * len(seqs), ['+'] * len(seqs))
        for t, pstr in zip(ids, peps):
            pep[int(poff[t]):int(poff[t + 1])] = np.frombuffer(
                (pstr or '').encode('latin-1'), dtype=np.uint8)
    if not outputs & OUT_NUC:
        nuc = None
    return nuc, noff, pep, poff


def _fasta_index(L, tp, size, truncate_names):
    """(count, lengths, NUL-separated name bytes) of a FASTA text, or None."""
    n = ctypes.c_uint32()
    nl = ctypes.c_uint64()
    rc = L.magot_fasta_read(tp, size, int(bool(truncate_names)), ctypes.byref(n), None,
                            None, 0, ctypes.byref(nl), None, 0)
    if rc == _lib.ERR_UNSUPPORTED:
        return None
    check(rc, 'magot_fasta_read')
    lens = np.zeros(max(n.value, 1), dtype=np.uint64)
    names = np.zeros(max(nl.value, 1), dtype=np.uint8)
    check(L.magot_fasta_read(tp, size, int(bool(truncate_names)), ctypes.byref(n),
                             ptr(lens), ptr(names), nl.value, ctypes.byref(nl), None, 0),
          'magot_fasta_read')
    return n, lens, names, nl


def fasta_contigs(text, truncate_names=False):
    """(names, lengths) of the contigs the native reader (magot_fasta_read)
    finds in a FASTA text, without copying any sequence; None when a header
    needs the Python reader.  Host only."""
    L = _lib.lib()
    data = _text_view(text)
    idx = _fasta_index(L, _text_ptr(data), len(data), truncate_names)
    if idx is None:
        return None
    n, lens, names, nl = idx
    nms = names[:nl.value].tobytes().split(b'\0')[:n.value]
    return [x.decode('latin-1') for x in nms], [int(x) for x in lens[:n.value]]


def fasta_read(text, truncate_names=False):
    """Native GenomeSequence reader (magot_fasta_read): [(name, bytes)], or None
    when a header needs the Python reader.  Host only."""
    L = _lib.lib()
    data = _text_view(text)
    tp = _text_ptr(data)
    idx = _fasta_index(L, tp, len(data), truncate_names)
    if idx is None:
        return None
    n, lens, names, nl = idx
    seqs = np.zeros(max(int(lens[:n.value].sum()), 1), dtype=np.uint8)
    check(L.magot_fasta_read(tp, len(data), int(bool(truncate_names)), ctypes.byref(n),
                             ptr(lens), ptr(names), nl.value, ctypes.byref(nl), ptr(seqs),
                             len(seqs)), 'magot_fasta_read')
    nms = names[:nl.value].tobytes().split(b'\0')[:n.value]
    out, o = [], 0
    for i in range(n.value):
        out.append((nms[i].decode('latin-1'), seqs[o:o + int(lens[i])].tobytes()))
        o += int(lens[i])
    return out


class FastaGenome(DeviceGenome):
    """A FASTA file read and packed natively (magot_genome_load_fasta): the
    batch path's GenomeSequence, without Python strings.  ``None`` from
    ``load`` when a header needs the Python reader."""

    @classmethod
    def load(cls, text, truncate_names=False, ctx=None):
        L = _lib.lib()
        self = cls.__new__(cls)
        self.ctx = ctx or _lib.default_context()
        self._keepalive = None
        data = _text_view(text)
        h = ctypes.c_void_p()
        rc = L.magot_genome_load_fasta(self.ctx.handle, _text_ptr(data), len(data),
                                       int(bool(truncate_names)), ctypes.byref(h))
        if rc == _lib.ERR_UNSUPPORTED:
            return None
        check(rc, 'magot_genome_load_fasta')
        self.handle = h
        n = ctypes.c_uint32()
        nl = ctypes.c_uint64()
        check(L.magot_genome_contigs(h, ctypes.byref(n), None, None, 0, ctypes.byref(nl)),
              'magot_genome_contigs')
        lens = np.zeros(max(n.value, 1), dtype=np.uint64)
        names = np.zeros(max(nl.value, 1), dtype=np.uint8)
        check(L.magot_genome_contigs(h, ctypes.byref(n), ptr(lens), ptr(names), nl.value,
                                     ctypes.byref(nl)), 'magot_genome_contigs')
        self.names = [x.decode('latin-1') for x in names[:nl.value].tobytes().split(b'\0')[:n.value]]
        self.index = {nm: i for i, nm in enumerate(self.names)}
        self.lengths = lens[:n.value]
        self._stats()
        return self


class ExtractionPlan(object):
    """Interval table -> device plan (magot_plan_create).

    ``exons``: structured array of EXON_DTYPE in output order; ``txs``:
    structured array of TX_DTYPE tiling it.  ``outputs``: OUT_NUC | OUT_PEP,
    optionally | OUT_GENOME_ORDER (records laid out in genome order on the
    device; fetch / copy_outputs still return record order, ``layout()`` gives
    each record's place in the device buffers).
    """

    def __init__(self, genome, exons, txs, outputs=OUT_NUC | OUT_PEP):
        self.genome = genome
        self.ctx = genome.ctx
        exons = np.ascontiguousarray(exons, dtype=EXON_DTYPE)
        txs = np.ascontiguousarray(txs, dtype=TX_DTYPE)
        self.n_exons = len(exons)
        self.n_tx = len(txs)
        self.outputs = outputs
        h = ctypes.c_void_p()
        nb, pb = ctypes.c_uint64(), ctypes.c_uint64()
        check(_lib.lib().magot_plan_create(self.ctx.handle, genome.handle, ptr(exons),
                                           self.n_exons, ptr(txs), self.n_tx, outputs,
                                           ctypes.byref(h), ctypes.byref(nb), ctypes.byref(pb)),
              'magot_plan_create')
        self.handle = h
        self.nuc_bytes = nb.value
        self.pep_bytes = pb.value

    def execute(self):
        check(_lib.lib().magot_plan_execute(self.ctx.handle, self.handle), 'magot_plan_execute')

    def sync(self):
        self.ctx.sync()

    def fetch(self):
        """Returns (nuc uint8[B] or None, nuc_off uint64[T+1], pep uint8[P] or None,
        pep_off uint64[T+1])."""
        nuc = np.empty(self.nuc_bytes, dtype=np.uint8) if self.outputs & OUT_NUC else None
        pep = np.empty(self.pep_bytes, dtype=np.uint8) if self.outputs & OUT_PEP else None
        noff = np.empty(self.n_tx + 1, dtype=np.uint64)
        poff = np.empty(self.n_tx + 1, dtype=np.uint64)
        check(_lib.lib().magot_plan_fetch(self.ctx.handle, self.handle,
                                          ptr(nuc) if nuc is not None and len(nuc) else None,
                                          ptr(noff),
                                          ptr(pep) if pep is not None and len(pep) else None,
                                          ptr(poff)), 'magot_plan_fetch')
        return nuc, noff, pep, poff

    def run(self):
        self.execute()
        return self.fetch()

    def layout(self):
        """(nuc_start uint64[T], pep_start uint64[T]): each record's start in
        the device buffers (magot_plan_layout)."""
        ns = np.empty(self.n_tx, dtype=np.uint64)
        ps = np.empty(self.n_tx, dtype=np.uint64)
        check(_lib.lib().magot_plan_layout(self.handle, ptr(ns) if self.n_tx else None,
                                           ptr(ps) if self.n_tx else None), 'magot_plan_layout')
        return ns, ps

    def copy_outputs(self, nuc_dev_ptr=None, pep_dev_ptr=None):
        """D2D copy of the outputs into caller device memory (addresses)."""
        check(_lib.lib().magot_plan_copy_outputs(
            self.ctx.handle, self.handle,
            ctypes.c_void_p(nuc_dev_ptr) if nuc_dev_ptr else None,
            ctypes.c_void_p(pep_dev_ptr) if pep_dev_ptr else None), 'magot_plan_copy_outputs')

    def fetch_to(self, nuc_addr=None, pep_addr=None):
        """D2H of the outputs straight into caller host memory given by address
        (e.g. pinned buffers); returns (nuc_off, pep_off)."""
        noff = np.empty(self.n_tx + 1, dtype=np.uint64)
        poff = np.empty(self.n_tx + 1, dtype=np.uint64)
        check(_lib.lib().magot_plan_fetch(self.ctx.handle, self.handle,
                                          ctypes.c_void_p(nuc_addr) if nuc_addr else None,
                                          ptr(noff),
                                          ctypes.c_void_p(pep_addr) if pep_addr else None,
                                          ptr(poff)), 'magot_plan_fetch')
        return noff, poff

    def time(self, iters):
        """Mean duration of `iters` isolated launches (an event pair each)."""
        ms = ctypes.c_double()
        check(_lib.lib().magot_plan_time(self.ctx.handle, self.handle, int(iters),
                                         ctypes.byref(ms)), 'magot_plan_time')
        return ms.value

    def time_b2b(self, iters):
        """Per-launch time of `iters` back-to-back launches (one event pair)."""
        ms = ctypes.c_double()
        check(_lib.lib().magot_plan_time_b2b(self.ctx.handle, self.handle, int(iters),
                                             ctypes.byref(ms)), 'magot_plan_time_b2b')
        return ms.value

    @property
    def algorithmic_bytes(self):
        return int(_lib.lib().magot_plan_algorithmic_bytes(self.handle))

    def close(self):
        if getattr(self, 'handle', None):
            _lib.lib().magot_plan_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class GffPlan(object):
    """Native gff2fasta planner (magot_gff_plan): GFF text -> interval and
    record tables + FASTA skeleton.  ``GffPlan.build`` returns None when the
    input takes one of the reference's diagnostic paths (the caller then uses
    the object path).  Host-only: no device needed to plan or render."""

    def __init__(self, handle, n_exons, n_tx, protein):
        self.handle = handle
        self.protein = protein
        # the plan's own tables, viewed in place (C3: 72 MB not copied);
        # close() turns the views into copies before the plan goes
        ep, tp = ctypes.c_void_p(), ctypes.c_void_p()
        check(_lib.lib().magot_gffplan_table_views(handle, ctypes.byref(ep), ctypes.byref(tp)),
              'magot_gffplan_table_views')
        self.exons = _view(ep.value, n_exons, EXON_DTYPE)
        self.txs = _view(tp.value, n_tx, TX_DTYPE)
        self._views = True
        n = ctypes.c_uint64()
        check(_lib.lib().magot_gffplan_selections(handle, ctypes.byref(n)),
              'magot_gffplan_selections')
        # longest=True protein choices, made by render() from the peptides
        # (no device text assembly for such a plan)
        self.n_select = n.value

    @classmethod
    def build(cls, gff, names, lengths, feature='gene', protein=False, order='insertion',
              longest=False, genomic=False, from_exons=False):
        """``longest`` / ``genomic``: get_fasta's options (genome.py:677-724).
        genomic=True is never translated (a nucleotide plan whatever
        ``protein`` says).  longest=True over protein candidates is chosen at
        render time (``n_select`` > 0), from the trimmed peptide lengths."""
        L = _lib.lib()
        text = _text_view(gff)
        n = len(names)
        arr = (ctypes.c_char_p * max(n, 1))(*[_as_bytes(x) for x in names])
        lens = np.ascontiguousarray(np.asarray(lengths, dtype=np.uint64))
        flags = (_lib.GFF_PROTEIN if protein else 0) | \
            (_lib.GFF_ORDER_PY2 if order == 'py2' else 0) | \
            (_lib.GFF_LONGEST if longest else 0) | (_lib.GFF_GENOMIC if genomic else 0) | \
            (_lib.GFF_FROM_EXONS if from_exons else 0)
        h = ctypes.c_void_p()
        ne, nt = ctypes.c_uint64(), ctypes.c_uint64()
        rc = L.magot_gff_plan(_text_ptr(text), len(text), arr, lens.ctypes.data_as(_lib._u64p), n,
                              _as_bytes(feature), flags, ctypes.byref(h), ctypes.byref(ne),
                              ctypes.byref(nt))
        if rc == _lib.ERR_UNSUPPORTED:
            return None
        check(rc, 'magot_gff_plan')
        return cls(h, ne.value, nt.value, protein and not genomic)

    @staticmethod
    def flags(protein=False, order='insertion', longest=False, genomic=False, from_exons=False):
        return (_lib.GFF_PROTEIN if protein else 0) | \
            (_lib.GFF_ORDER_PY2 if order == 'py2' else 0) | \
            (_lib.GFF_LONGEST if longest else 0) | (_lib.GFF_GENOMIC if genomic else 0) | \
            (_lib.GFF_FROM_EXONS if from_exons else 0)

    @classmethod
    def flank(cls, gff, names, lengths, sequence_length, stream, feature_type='gene',
              namefrom='ID'):
        """extract_upstream_downstream's windows (genome_tools.py:457-480,
        magot_flank_plan) as a nucleotide plan: one single-interval record per
        printed window, the same skeleton shape as gff2fasta.  None when the
        reference would raise (the caller's line loop reproduces it).
        ``sequence_length`` and ``stream`` are the reference's strings."""
        L = _lib.lib()
        text = _text_view(gff)
        n = len(names)
        arr = (ctypes.c_char_p * max(n, 1))(*[_as_bytes(x) for x in names])
        lens = np.ascontiguousarray(np.asarray(lengths, dtype=np.uint64))
        h = ctypes.c_void_p()
        ne, nt = ctypes.c_uint64(), ctypes.c_uint64()
        rc = L.magot_flank_plan(_text_ptr(text), len(text), arr, lens.ctypes.data_as(_lib._u64p),
                                n, _as_bytes(feature_type), _as_bytes(namefrom),
                                _as_bytes(str(sequence_length)), _as_bytes(stream),
                                ctypes.byref(h), ctypes.byref(ne), ctypes.byref(nt))
        if rc == _lib.ERR_UNSUPPORTED:
            return None
        check(rc, 'magot_flank_plan')
        return cls(h, ne.value, nt.value, False)

    def render(self, nuc, noff, pep, poff):
        """The FASTA text (bytes) around the fetched record payloads."""
        L = _lib.lib()
        size = ctypes.c_uint64()
        args = (ptr(nuc), ptr(noff), ptr(pep), ptr(poff))
        check(L.magot_gffplan_render(self.handle, *args, None, 0, ctypes.byref(size)),
              'magot_gffplan_render')
        out = np.empty(size.value, dtype=np.uint8)
        check(L.magot_gffplan_render(self.handle, *args, ptr(out), size.value,
                                     ctypes.byref(size)), 'magot_gffplan_render')
        return out.tobytes()

    def close(self):
        if self.handle:
            if self._views:
                # the views die with the plan: anyone still holding the
                # attributes keeps valid copies
                self.exons, self.txs = self.exons.copy(), self.txs.copy()
                self._views = False
            _lib.lib().magot_gffplan_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _view(addr, n, dtype):
    """n rows of `dtype` at host address `addr` (not owned; empty when n == 0)."""
    dtype = np.dtype(dtype)
    if not n:
        return np.zeros(0, dtype=dtype)
    buf = (ctypes.c_uint8 * (n * dtype.itemsize)).from_address(addr)
    return np.frombuffer(buf, dtype=dtype, count=n)


class GffRead(object):
    """read_gff done natively (magot_gff_read) before the genome's contigs are
    known; ``lower`` turns it into a GffPlan against them (magot_gff_lower).
    gff2fasta reads the GFF this way while another thread loads the FASTA.
    ``read`` returns None when the input takes a diagnostic path."""

    def __init__(self, handle, text, from_exons):
        self.handle = handle
        self._text = text  # the plan reads views of it until lower() returns
        self.from_exons = from_exons

    @classmethod
    def read(cls, gff, from_exons=False):
        L = _lib.lib()
        text = _text_view(gff)
        h = ctypes.c_void_p()
        rc = L.magot_gff_read(_text_ptr(text), len(text),
                              GffPlan.flags(from_exons=from_exons), ctypes.byref(h))
        if rc == _lib.ERR_UNSUPPORTED:
            if h.value:
                L.magot_gffplan_destroy(h)
            return None
        check(rc, 'magot_gff_read')
        return cls(h, text, from_exons)

    def lower(self, names, lengths, feature='gene', protein=False, order='insertion',
              longest=False, genomic=False):
        """The GffPlan (this object gives its handle up), or None when the
        lowering takes a diagnostic path (the handle is freed)."""
        if not self.handle:
            raise MagotError('GffRead.lower: already lowered or closed')
        L = _lib.lib()
        n = len(names)
        arr = (ctypes.c_char_p * max(n, 1))(*[_as_bytes(x) for x in names])
        lens = np.ascontiguousarray(np.asarray(lengths, dtype=np.uint64))
        flags = GffPlan.flags(protein, order, longest, genomic, self.from_exons)
        ne, nt = ctypes.c_uint64(), ctypes.c_uint64()
        h, self.handle = self.handle, None
        try:
            rc = L.magot_gff_lower(h, arr, lens.ctypes.data_as(_lib._u64p), n, _as_bytes(feature),
                                   flags, ctypes.byref(ne), ctypes.byref(nt))
            if rc == _lib.ERR_UNSUPPORTED:
                return None
            check(rc, 'magot_gff_lower')
            plan = GffPlan(h, ne.value, nt.value, protein and not genomic)
            h = None
            return plan
        finally:
            self._text = None
            if h is not None:
                L.magot_gffplan_destroy(h)

    def close(self):
        if self.handle:
            _lib.lib().magot_gffplan_destroy(self.handle)
            self.handle = None
        self._text = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class FastaText(object):
    """The gff2fasta text assembled on device (magot_fasta_text_*): the
    GffPlan skeleton filled with an ExtractionPlan's payloads in one device
    buffer, fetched with a single D2H."""

    def __init__(self, gffplan, extraction):
        L = _lib.lib()
        self.ctx = extraction.ctx
        self._keep = (gffplan, extraction)
        h = ctypes.c_void_p()
        cap = ctypes.c_uint64()
        check(L.magot_fasta_text_create(self.ctx.handle, gffplan.handle, extraction.handle,
                                        ctypes.byref(h), ctypes.byref(cap)),
              'magot_fasta_text_create')
        self.handle = h
        self.max_bytes = cap.value

    def execute(self):
        check(_lib.lib().magot_fasta_text_execute(self.ctx.handle, self.handle),
              'magot_fasta_text_execute')

    def fetch(self):
        """The text as a bytes-like numpy array (no trailing newline)."""
        L = _lib.lib()
        out = np.empty(max(self.max_bytes, 1), dtype=np.uint8)
        n = ctypes.c_uint64()
        check(L.magot_fasta_text_fetch(self.ctx.handle, self.handle, ptr(out), self.max_bytes,
                                       ctypes.byref(n)), 'magot_fasta_text_fetch')
        return out[:n.value]

    def time(self, iters):
        ms = ctypes.c_double()
        check(_lib.lib().magot_fasta_text_time(self.ctx.handle, self.handle, int(iters),
                                               ctypes.byref(ms)), 'magot_fasta_text_time')
        return ms.value

    def close(self):
        if getattr(self, 'handle', None):
            _lib.lib().magot_fasta_text_destroy(self.handle)
            self.handle = None
        self._keep = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _concat(seqs):
    parts = [_as_bytes(s) for s in seqs]
    off = np.zeros(len(parts) + 1, dtype=np.uint64)
    if parts:
        np.cumsum([len(p) for p in parts], out=off[1:])
    buf = np.frombuffer(b''.join(parts), dtype=np.uint8) if parts else np.zeros(0, np.uint8)
    return buf, off


def revcomp_batch(seqs, ctx=None):
    """Sequence.reverse_compliment (genome.py:784-793) over a list of strings."""
    ctx = ctx or _lib.default_context()
    buf, off = _concat(seqs)
    out = np.empty(max(len(buf), 1), dtype=np.uint8)
    check(_lib.lib().magot_revcomp_batch(ctx.handle, ptr(buf) if len(buf) else None, ptr(off),
                                         len(seqs), ptr(out)), 'magot_revcomp_batch')
    raw = out.tobytes()
    return [raw[int(off[i]):int(off[i + 1])].decode('latin-1') for i in range(len(seqs))]


def orf6_batch(seqs, lut64=None, ctx=None):
    """The six translations Sequence.get_orfs splits (genome.py:824-851), per
    input: a list of 6 values in the reference's loop order (frame 0,1,2 x
    strand '-','+'), each the trimmed ``translate()`` result or None."""
    ctx = ctx or _lib.default_context()
    n = len(seqs)
    buf, off = _concat(seqs)
    soff = np.empty(6 * n + 1, dtype=np.uint64)
    slen = np.empty(max(6 * n, 1), dtype=np.uint64)
    none = np.empty(max(6 * n, 1), dtype=np.uint8)
    L = _lib.lib()
    check(L.magot_orf6_sizes(ptr(off), n, ptr(soff), ptr(slen), ptr(none)), 'magot_orf6_sizes')
    total = int(soff[6 * n])
    out = np.empty(max(total, 1), dtype=np.uint8)
    lut = np.frombuffer(bytes(lut64), dtype=np.uint8).copy() if lut64 is not None else None
    check(L.magot_orf6_batch(ctx.handle, ptr(buf) if len(buf) else None, ptr(off), n, ptr(lut),
                             ptr(soff), ptr(out)), 'magot_orf6_batch')
    raw = out[:total].tobytes().decode('latin-1')
    res = []
    for r in range(n):
        six = []
        for j in range(6 * r, 6 * r + 6):
            if none[j]:
                six.append(None)
                continue
            t = raw[int(soff[j]):int(soff[j] + slen[j])]
            if (j % 6) < 2 and t[:1] == 'X':  # frame 0: trimX (genome.py:819-821)
                t = t[1:]
            six.append(t)
        res.append(six)
    return res


class Orf6Plan(object):
    """Six-frame translation of an ExtractionPlan's records, in HBM
    (magot_plan_orf6): BASELINE configs[4] (C5).  The kernel gathers the
    records from the packed genome itself (the plan's nucleotide output is
    neither needed nor read)."""

    def __init__(self, plan, lut64=None):
        self.plan = plan
        self.ctx = plan.ctx
        lut = np.frombuffer(bytes(lut64), dtype=np.uint8).copy() if lut64 is not None else None
        h = ctypes.c_void_p()
        tot = ctypes.c_uint64()
        check(_lib.lib().magot_plan_orf6(self.ctx.handle, plan.handle, ptr(lut), ctypes.byref(h),
                                         ctypes.byref(tot)), 'magot_plan_orf6')
        self.handle = h
        self.total = tot.value

    def execute(self):
        check(_lib.lib().magot_orf6_execute(self.ctx.handle, self.handle), 'magot_orf6_execute')

    def fetch(self):
        """(padded residue bytes, stream offsets 6n+1 (16-aligned), real stream lengths 6n)."""
        out = np.empty(max(self.total, 1), dtype=np.uint8)
        soff = np.empty(6 * self.plan.n_tx + 1, dtype=np.uint64)
        slen = np.empty(max(6 * self.plan.n_tx, 1), dtype=np.uint64)
        check(_lib.lib().magot_orf6_fetch(self.ctx.handle, self.handle, ptr(out), ptr(soff),
                                          ptr(slen)), 'magot_orf6_fetch')
        return out[:self.total], soff, slen[:6 * self.plan.n_tx]

    def fetch_to(self, out_addr):
        """D2H of the padded residue bytes into caller host memory (an address,
        e.g. a pinned buffer of ``total`` bytes); returns (stream_off, stream_len)."""
        soff = np.empty(6 * self.plan.n_tx + 1, dtype=np.uint64)
        slen = np.empty(max(6 * self.plan.n_tx, 1), dtype=np.uint64)
        check(_lib.lib().magot_orf6_fetch(self.ctx.handle, self.handle,
                                          ctypes.c_void_p(out_addr) if out_addr else None,
                                          ptr(soff), ptr(slen)), 'magot_orf6_fetch')
        return soff, slen[:6 * self.plan.n_tx]

    def copy_outputs(self, dst_dev_ptr):
        """D2D copy of the padded residue bytes (``total``) into caller device
        memory (an address), e.g. the buffer an output gather sends."""
        check(_lib.lib().magot_orf6_copy_outputs(self.ctx.handle, self.handle,
                                                 ctypes.c_void_p(dst_dev_ptr)),
              'magot_orf6_copy_outputs')

    def time(self, iters):
        ms = ctypes.c_double()
        check(_lib.lib().magot_orf6_time(self.ctx.handle, self.handle, int(iters),
                                         ctypes.byref(ms)), 'magot_orf6_time')
        return ms.value

    def time_b2b(self, iters):
        ms = ctypes.c_double()
        check(_lib.lib().magot_orf6_time_b2b(self.ctx.handle, self.handle, int(iters),
                                             ctypes.byref(ms)), 'magot_orf6_time_b2b')
        return ms.value

    def close(self):
        if getattr(self, 'handle', None):
            _lib.lib().magot_orf6_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def copy_segments(src_dev_ptr, src_bytes, dst_dev_ptr, src_off, dst_off, ctx=None):
    """dst[dst_off[i]:dst_off[i+1]] = src[src_off[i]:...] on the device
    (magot_copy_segments; addresses of device memory, src_bytes the source's
    size, host offset tables)."""
    ctx = ctx or _lib.default_context()
    so = np.ascontiguousarray(src_off, dtype=np.uint64)
    do = np.ascontiguousarray(dst_off, dtype=np.uint64)
    if len(do) != len(so) + 1:
        raise ValueError('dst_off needs len(src_off) + 1 entries')
    check(_lib.lib().magot_copy_segments(ctx.handle, ctypes.c_void_p(src_dev_ptr), int(src_bytes),
                                         ctypes.c_void_p(dst_dev_ptr), ptr(so), ptr(do), len(so)),
          'magot_copy_segments')


def orf6_sizes(rec_off):
    """(stream_off 6n+1, stream_len 6n) of the six-frame layout over records
    with nucleotide offsets ``rec_off`` (n+1): magot_orf6_sizes."""
    off = np.ascontiguousarray(rec_off, dtype=np.uint64)
    n = len(off) - 1
    soff = np.empty(6 * n + 1, dtype=np.uint64)
    slen = np.empty(max(6 * n, 1), dtype=np.uint64)
    check(_lib.lib().magot_orf6_sizes(ptr(off), n, ptr(soff), ptr(slen), None), 'magot_orf6_sizes')
    return soff, slen[:6 * n]


def codon_symbols(seq, class256, n_classes, lut, ctx=None):
    """One symbol per full codon of ``seq`` (str/bytes, length a multiple of 3)
    over an extended alphabet (magot_codon_symbols): a list of ints."""
    ctx = ctx or _lib.default_context()
    buf = np.frombuffer(_as_bytes(seq), dtype=np.uint8)
    m = len(buf) // 3
    out = np.empty(max(m, 1), dtype=np.uint8)
    cls = np.ascontiguousarray(class256, dtype=np.uint8)
    lt = np.ascontiguousarray(lut, dtype=np.uint8)
    check(_lib.lib().magot_codon_symbols(ctx.handle, ptr(buf) if m else None, m, ptr(cls),
                                         int(n_classes), ptr(lt), ptr(out)),
          'magot_codon_symbols')
    return out[:m].tolist()


def translate_batch(seqs, frames, strands, lut64=None, ctx=None):
    """Untrimmed Sequence.translate (genome.py:795-822) residues per input, or None
    where the reference returns None.  The caller applies trimX."""
    ctx = ctx or _lib.default_context()
    n = len(seqs)
    buf, off = _concat(seqs)
    fr = np.ascontiguousarray(frames, dtype=np.int32)
    st = np.frombuffer(''.join(strands).encode('latin-1'), dtype=np.uint8).copy() if n else \
        np.zeros(0, np.uint8)
    poff = np.empty(n + 1, dtype=np.uint64)
    codons = np.empty(max(n, 1), dtype=np.int64)
    L = _lib.lib()
    check(L.magot_translate_sizes(ptr(off), n, ptr(fr), ptr(poff), ptr(codons)),
          'magot_translate_sizes')
    total = int(poff[n])
    out = np.empty(max(total, 1), dtype=np.uint8)
    lut = None
    if lut64 is not None:
        lut = np.frombuffer(bytes(lut64), dtype=np.uint8).copy()
    check(L.magot_translate_batch(ctx.handle, ptr(buf) if len(buf) else None, ptr(off), n,
                                  ptr(fr), ptr(st), ptr(lut), ptr(poff), ptr(out)),
          'magot_translate_batch')
    raw = out.tobytes()
    res = []
    for i in range(n):
        if codons[i] < 0:
            res.append(None)
        else:
            res.append(raw[int(poff[i]):int(poff[i + 1])].decode('latin-1'))
    return res


__all__ = ['DeviceGenome', 'ExtractionPlan', 'revcomp_batch', 'translate_batch', 'codon_symbols',
           'OUT_NUC',
           'OUT_PEP', 'MagotError', 'GffPlan', 'orf6_batch', 'Orf6Plan', 'fasta_read',
           'FastaGenome', 'PartitionedGenome', 'device_genome', 'extract_records', 'plan_parts',
           'copy_segments', 'orf6_sizes']
