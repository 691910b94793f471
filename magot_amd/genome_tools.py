"""Command-line tools on the extraction path (genome_tools.py of the reference).

    python -m magot_amd.genome_tools gff2fasta <fasta> <gff> [seq_type=protein]
           [longest=True] [genomic=True] [from_exons=True] [order=py2|insertion]
           [native=False]
    python -m magot_amd.genome_tools cds2pep <cds.fasta>
    python -m magot_amd.genome_tools extract_upstream_downstream <fasta> <gff> <length> up|down
           [feature_type=gene] [namefrom=ID] [truncate_names=True] [native=False]
    python -m magot_amd.genome_tools coords2fasta <fasta> <seqid> <start> <stop> [truncate_names=False]
    python -m magot_amd.genome_tools blast_csv2fasta <fasta> <blast.csv> [order=py2|insertion]
    python -m magot_amd.genome_tools exonerate2fasta <fasta> <exonerate.txt> [order=py2|insertion]
    python -m magot_amd.genome_tools get_seq_from_fasta <fasta> <seq_name> [truncate_names=False]

Arguments follow the reference's CLI convention (genome_tools.py:25-45):
positional values, then ``key=value`` pairs, all strings.  The reference
``eval``s the assembled call; here values are parsed as Python literals
(``True``/``False``/numbers) and never executed.

Record order defaults to ``py2`` so the bytes written match the reference's
own goldens (test_data/test_suite.py:12-13); ``order=insertion`` gives the
Python-3 order.
"""

import ast
import ctypes
import json
import os
import sys
import time

import numpy as np

from . import engine
from . import genome


class _Clock(object):
    """Wall-clock phases of one CLI call, from the call's start: with
    MAGOT_CLI_TIMING=1 one JSON line on stderr (``{"cli_phases_s": ...}``);
    otherwise nothing is recorded.  ``at(name)`` stamps the time since the
    start (any thread); ``lap(name)`` the time since the previous lap."""

    def __init__(self):
        self.on = os.environ.get('MAGOT_CLI_TIMING') == '1'
        self.t0 = self.last = time.perf_counter()
        self.laps, self.stamps = {}, {}
        self.release_thread = None

    def lap(self, name):
        if self.on:
            t = time.perf_counter()
            self.laps[name] = self.laps.get(name, 0.0) + t - self.last
            self.last = t

    def at(self, name):
        if self.on:
            self.stamps[name] = time.perf_counter() - self.t0

    def emit(self):
        if self.on:
            sys.stderr.write(json.dumps({'cli_phases_s': self.laps, 'cli_stamps_s': self.stamps,
                                         'cli_total_s': time.perf_counter() - self.t0}) + '\n')
            sys.stderr.flush()


class _Release(object):
    """What one CLI call closes when it is done, in order.  ``later()``
    closes it on a background thread and returns that thread: once the
    text is in the caller's hands, freeing the device buffers and the
    planner's host tables (C3: ~0.12 s) need not delay it.  The thread is
    not a daemon, so an interpreter that exits first still waits for it."""

    def __init__(self):
        self.objs = []

    def add(self, obj):
        if obj is not None:
            self.objs.append(obj)
        return obj

    def now(self):
        objs, self.objs = self.objs, []
        for obj in objs:
            obj.close()

    def later(self):
        import threading
        th = threading.Thread(target=self.now, name='magot-release')
        th.start()
        return th


def _literal(text):
    try:
        return ast.literal_eval(text)
    except (ValueError, SyntaxError):
        return text


def _write(text):
    out = getattr(sys.stdout, 'buffer', None)
    if out is not None:
        sys.stdout.flush()
        out.write(text.encode('latin-1'))
        out.flush()
    else:
        sys.stdout.write(text)


def _write_bytes(*parts):
    out = getattr(sys.stdout, 'buffer', None)
    if out is not None:
        sys.stdout.flush()
        for p in parts:
            out.write(p)
        out.flush()
    else:
        sys.stdout.write(''.join(bytes(p).decode('latin-1') for p in parts))


def gff2fasta(genome_sequence, gff, from_exons='False', seq_type='nucleotide', longest='False',
              genomic='False', order='py2', native='True'):
    """genome_tools.py:324-330.

    The native planner (magot_gff_plan: read_gff + get_fasta lowering in C++)
    and one kernel launch serve every combination of from_exons, genomic and
    longest; inputs that take one of the reference's diagnostic paths use the
    object path (``native=False`` forces it)."""
    lg, gm = _literal(longest), _literal(genomic)
    if (native == 'True' and isinstance(lg, bool) and isinstance(gm, bool) and
            seq_type in ('nucleotide', 'protein')):
        clock = _Clock()
        text, parsed = _gff2fasta_native(genome_sequence, gff, seq_type, order,
                                         longest=lg is True, genomic=gm is True,
                                         from_exons=from_exons == 'True', clock=clock)
        if text is not None:
            _write_bytes(text, b'\n')
            clock.lap('write')
            clock.emit()
            return
        if parsed is not None:
            genome_sequence = parsed  # read once: the object path reuses it
    g = genome.Genome(genome_sequence)
    if from_exons == 'True':
        # reference quirk kept: a str features_to_ignore is a substring test
        g.read_gff(gff, features_to_ignore='CDS', features_to_replace=[('exon', 'CDS')])
    else:
        g.read_gff(gff)
    text = g.annotations.get_fasta('gene', seq_type=seq_type, longest=_literal(longest),
                                   genomic=_literal(genomic), order=order)
    _write(text + '\n')


def _gff2fasta_native(genome_sequence, gff, seq_type, order, longest=False, genomic=False,
                      from_exons=False, clock=None):
    """(text, parsed): the gff2fasta text (bytes) via the native planner, the
    extraction kernel and device text assembly, or (None, GenomeSequence or
    None) when it declines -- the GenomeSequence already parsed, for the
    object path to reuse."""
    if order not in ('py2', 'insertion'):
        raise ValueError("order must be 'insertion' or 'py2'")
    protein = seq_type == 'protein'
    clock = clock or _Clock()

    # The FASTA is read and packed natively (Python reader for unusual
    # headers) on another thread, which starts the device first; this thread
    # reads the GFF meanwhile (read_gff needs no genome), then lowers it
    # against the loaded genome's contigs.  Both native calls release the GIL.
    from concurrent.futures import ThreadPoolExecutor
    fa = genome.read_buffer(genome_sequence)
    clock.lap('fasta_map')

    def load(text):
        clock.at('load_thread_start')
        from . import _lib
        ctx = _lib.default_context()          # device start-up
        clock.at('device_context_ready')
        g = engine.FastaGenome.load(text, ctx=ctx)
        clock.at('genome_on_device')
        return g

    with ThreadPoolExecutor(1) as pool:
        loading = pool.submit(load, fa)
        try:
            read = engine.GffRead.read(genome.read_buffer(gff), from_exons=from_exons)
            clock.lap('gff_read')
        except BaseException:
            # the genome may already be on the device: free it before raising
            try:
                loaded = loading.result()
            except Exception:
                loaded = None
            if loaded is not None:
                loaded.close()
            raise
        try:
            dev = loading.result()
        except BaseException:
            if read is not None:
                read.close()
            raise
        clock.lap('wait_genome')
    owned = dev  # the FastaGenome this call loaded (closed on every return)
    if read is None:  # read_gff takes a diagnostic path: the object path
        if dev is not None:
            dev.close()
        return None, None

    def plan_gff(names, lengths):
        # lowers the one read (None when the lowering takes a diagnostic path)
        return read.lower(names, lengths, protein=protein, order=order, longest=longest,
                          genomic=genomic)

    release = _Release()
    try:
        plan = None
        if dev is not None:
            plan = plan_gff(dev.names, dev.lengths)
            clock.lap('gff_lower')
            if plan is None:
                return None, None
        return _gff2fasta_run(genome_sequence, dev, plan, plan_gff, clock, release)
    finally:
        release.add(read)
        release.add(owned)
        clock.release_thread = release.later()
        clock.lap('close')


def _gff2fasta_run(genome_sequence, dev, plan, plan_gff, clock, release):
    seqs = None
    if dev is None:
        seqs = genome.GenomeSequence(genome_sequence)
        if sum(len(v) for v in seqs.values()) > engine.PART_BASES:
            # several device planes: the object path extracts per plane;
            # decided before anything is packed
            return None, seqs
        dev = seqs.device()
        plan = plan_gff(dev.names, [int(x) for x in dev.lengths])
        if plan is None:
            return None, seqs
    try:
        # records laid out in genome order on the device (neighbouring loci in
        # neighbouring tiles share genome lines: the kernel the bench line
        # times); the device text assembly reads each record at its place, so
        # the text is the record-order text.  longest=True over peptides
        # fetches the payloads for a host render: record order there.
        out = engine.OUT_PEP if plan.protein else engine.OUT_NUC
        ex = engine.ExtractionPlan(dev, plan.exons, plan.txs,
                                   out if plan.n_select else out | engine.OUT_GENOME_ORDER)
        clock.lap('plan_create')
        if plan.n_select:
            # longest=True over peptides: the render picks from the trimmed
            # lengths, on the host
            try:
                return plan.render(*ex.run()), None
            finally:
                ex.close()
        text = engine.FastaText(plan, ex)
        clock.lap('text_create')
        try:
            ex.execute()
            text.execute()  # records + headers + joiners in one device buffer
            ex.sync()
            clock.lap('kernel_and_text_assembly')
            out = text.fetch()
            clock.lap('text_d2h')
            return out, None
        finally:
            release.add(text)
            release.add(ex)
    finally:
        release.add(plan)


def _cds_translate(seq, seg_off):
    """(pep offsets, codon counts, residues) of the segments' frame-0 '+'
    translations (magot_translate_batch, one launch)."""
    from . import _lib
    n = len(seg_off) - 1
    fr = np.zeros(n, np.int32)
    st = np.full(n, ord('+'), np.uint8)
    poff = np.empty(n + 1, dtype=np.uint64)
    codons = np.empty(max(n, 1), dtype=np.int64)
    L = _lib.lib()
    _lib.check(L.magot_translate_sizes(_lib.ptr(seg_off), n, _lib.ptr(fr), _lib.ptr(poff),
                                       _lib.ptr(codons)), 'magot_translate_sizes')
    out = np.empty(max(int(poff[n]), 1), dtype=np.uint8)
    _lib.check(L.magot_translate_batch(_lib.default_context().handle,
                                       _lib.ptr(seq) if len(seq) else None, _lib.ptr(seg_off), n,
                                       _lib.ptr(fr), _lib.ptr(st), None, _lib.ptr(poff),
                                       _lib.ptr(out)), 'magot_translate_batch')
    return poff, codons, out


def _cds2pep_native(data):
    """cds2pep's stdout for a file's bytes: magot_cds_scan (no per-line
    Python), one translation batch, magot_cds_render; None when the line loop
    must run (an empty line's IndexError, a CR inside a line)."""
    from . import _lib
    L = _lib.lib()
    d = engine._text_view(data)
    tp = engine._text_ptr(d)
    n_seg, nb = ctypes.c_uint64(), ctypes.c_uint64()
    rc = L.magot_cds_scan(tp, len(d), ctypes.byref(n_seg), ctypes.byref(nb), None, None, None,
                          None, 0)
    if rc == _lib.ERR_UNSUPPORTED:
        return None
    _lib.check(rc, 'magot_cds_scan')
    n = n_seg.value
    seg_off = np.empty(n + 1, np.uint64)
    hdr_off = np.empty(max(n - 1, 1), np.uint64)
    hdr_len = np.empty(max(n - 1, 1), np.uint64)
    seq = np.empty(max(nb.value, 1), np.uint8)
    _lib.check(L.magot_cds_scan(tp, len(d), ctypes.byref(n_seg), ctypes.byref(nb),
                                _lib.ptr(seg_off), _lib.ptr(hdr_off), _lib.ptr(hdr_len),
                                _lib.ptr(seq), len(seq)), 'magot_cds_scan')
    poff, codons, pep = _cds_translate(seq[:nb.value], seg_off)
    size = ctypes.c_uint64()
    args = (tp, n, _lib.ptr(seg_off), _lib.ptr(hdr_off), _lib.ptr(hdr_len), _lib.ptr(pep),
            _lib.ptr(poff), _lib.ptr(codons))
    _lib.check(L.magot_cds_render(*args, None, 0, ctypes.byref(size)), 'magot_cds_render')
    out = np.empty(max(size.value, 1), np.uint8)
    _lib.check(L.magot_cds_render(*args, _lib.ptr(out), size.value, ctypes.byref(size)),
               'magot_cds_render')
    return out[:size.value]


def cds2pep(fasta_file, native='True'):
    """genome_tools.py:664-675: headers echoed, each record translated; all
    records go to the GPU as one batch.  A file path is scanned natively
    (``native=False`` forces the line loop, which also reproduces the
    reference's IndexError on an empty line)."""
    if not hasattr(fasta_file, 'read'):
        with open(fasta_file, 'rb'):  # the reference open()s the path (:666): a missing file raises
            pass
        if native == 'True' and isinstance(fasta_file, str):
            text = _cds2pep_native(genome.read_buffer(fasta_file))
            if text is not None:
                _write_bytes(text)
                return
    events = []       # ('line', text) | ('pep', job index)
    seqs = []
    failure = None
    work = []
    for raw in genome.ensure_file(fasta_file):
        line = raw.replace('\n', '').replace('\r', '')
        try:
            first = line[0]
        except IndexError as e:
            failure = e
            break
        if first == '>':
            cur = ''.join(work)
            if cur != '':
                events.append(('pep', len(seqs)))
                seqs.append(cur)
                work = []
            events.append(('line', line))
        else:
            work.append(line)
    if failure is None:
        events.append(('pep', len(seqs)))
        seqs.append(''.join(work))
    peps = engine.translate_batch(seqs, [0] * len(seqs), ['+'] * len(seqs)) if seqs else []
    out = []
    for kind, val in events:
        if kind == 'line':
            out.append(val)
        else:
            p = peps[val]
            if p is not None and p[:1] == 'X':
                p = p[1:]
            out.append(str(p))
    _write(''.join(s + '\n' for s in out))
    if failure is not None:
        raise failure


def _gather(seqs, intervals):
    """Bytes of (contig index, start, length, rc) intervals: one kernel launch."""
    if not intervals:
        return []
    ex = np.zeros(len(intervals), dtype=engine.EXON_DTYPE)
    for i, (c, st, ln, rc) in enumerate(intervals):
        ex[i] = ((st | (1 << 63)) if rc else st, c, ln)
    tx = np.zeros(len(intervals), dtype=engine.TX_DTYPE)
    tx['exon_begin'] = np.arange(len(intervals))
    tx['n_exons'] = 1
    nuc, noff, _, _ = engine.extract_records(seqs.device(), ex, tx, engine.OUT_NUC)
    raw = nuc.tobytes().decode('latin-1')
    return [raw[int(noff[i]):int(noff[i + 1])] for i in range(len(intervals))]


def extract_upstream_downstream(genome_sequence, gff, sequence_length, stream,
                                feature_type='gene', namefrom='ID', truncate_names='True',
                                native='True'):
    """genome_tools.py:457-480: the `sequence_length` bases up- or downstream of
    every `feature_type` line, strand-aware.  Reference quirks kept: 'down' on
    '+' and 'up' on '-' are reverse complemented; a strand other than '+'/'-'
    reuses the previous line's sequence (or raises UnboundLocalError); only
    full-length windows print.

    Natively (magot_flank_plan: the GFF scanned in C++, the windows gathered
    by the extraction kernel, the FASTA text assembled on the device) unless
    the input would take one of the reference's error paths, which the line
    loop below reproduces (``native=False`` forces it)."""
    truncate = _literal(truncate_names)
    if native == 'True' and isinstance(truncate, bool):
        text = _flank_native(genome_sequence, gff, sequence_length, stream, feature_type,
                             namefrom, truncate)
        if text is not None:
            _write_bytes(text, b'\n')
            return
    seqs = genome.GenomeSequence(genome_sequence, truncate_names=truncate)
    index = {name: i for i, name in enumerate(seqs)}
    current = None
    items = []
    with open(gff, 'rb') as fh:
        lines = fh.read().decode('latin-1').split('\n')
    lines = [ln + '\n' for ln in lines[:-1]] + ([lines[-1]] if lines[-1] else [])
    for line in lines:
        if line.count('\t') > 5 and line[0] != '#':
            fields = line.split('\t')
            if fields[2] == feature_type:
                name = None
                coords = sorted([int(fields[3]), int(fields[4])])
                for attribute in fields[-1].split(';'):
                    if namefrom == attribute.split('=')[0]:
                        name = attribute.split('=')[1].replace('\r', '').replace('\n', '')
                if name is None:
                    name = 'seq' + str(len(items))
                # evaluation order of the reference: the contig (KeyError),
                # then int(sequence_length) (ValueError)
                if stream == 'up' and fields[6] == '+' or stream == 'down' and fields[6] == '-':
                    stop = coords[0] - 1
                    contig = seqs[fields[0]]
                    n = int(sequence_length)
                    st, ln = genome._slice_interval(contig, stop - n, stop)
                    current = (index[fields[0]], st, ln, False)
                elif stream == 'down' and fields[6] == '+' or stream == 'up' and fields[6] == '-':
                    start = coords[1]
                    contig = seqs[fields[0]]
                    n = int(sequence_length)
                    st, ln = genome._slice_interval(contig, start, start + n)
                    current = (index[fields[0]], st, ln, True)
                if current is None:
                    raise UnboundLocalError(
                        "local variable 'sequence' referenced before assignment")
                if current[2] == int(sequence_length):
                    items.append((name, current))
    texts = _gather(seqs, [iv for _, iv in items])
    _write('\n'.join('>' + name + '\n' + t for (name, _), t in zip(items, texts)) + '\n')


def _flank_native(genome_sequence, gff, sequence_length, stream, feature_type, namefrom,
                  truncate):
    """extract_upstream_downstream's text (bytes, no final newline) via
    magot_flank_plan, one extraction launch and device text assembly; None
    when the FASTA needs the Python reader or the input takes an error path."""
    dev = engine.FastaGenome.load(genome.read_buffer(genome_sequence), truncate_names=truncate)
    if dev is None:
        return None
    plan = engine.GffPlan.flank(genome.read_buffer(gff), dev.names,
                                [int(x) for x in dev.lengths], sequence_length, stream,
                                feature_type=feature_type, namefrom=namefrom)
    if plan is None:
        return None
    try:
        if len(plan.txs) == 0:
            return b''
        ex = engine.ExtractionPlan(dev, plan.exons, plan.txs, engine.OUT_NUC)
        text = engine.FastaText(plan, ex)
        try:
            ex.execute()
            text.execute()
            return text.fetch()
        finally:
            text.close()
            ex.close()
    finally:
        plan.close()


def coords2fasta(fasta_file, seqid, start, stop, truncate_names='False'):
    """genome_tools.py:656-661: header, then contig[start-1:stop] (Python slice
    rules) gathered on the GPU.  The FASTA is read and packed natively
    (magot_genome_load_fasta) unless a header needs the Python reader."""
    _write('>' + seqid + ':' + start + '-' + stop + '\n')
    truncate = _literal(truncate_names)
    dev = None
    if isinstance(truncate, bool):
        dev = engine.FastaGenome.load(genome.read_buffer(fasta_file), truncate_names=truncate)
    if dev is None:
        seqs = genome.Genome(fasta_file, truncate_names=truncate).genome_sequence
        contig = seqs[seqid]
        st, ln = genome._slice_interval(contig, int(start) - 1, int(stop))
        index = {name: i for i, name in enumerate(seqs)}
        _write(_gather(seqs, [(index[seqid], st, ln, False)])[0] + '\n')
        return
    c = dev.index[seqid]  # KeyError, as genome_sequence[seqid]
    a, b = slice(int(start) - 1, int(stop)).indices(int(dev.lengths[c]))[:2]
    _write_bytes(_gather_device(dev, [(c, a, max(0, b - a), False)])[0], b'\n')


def _gather_device(dev, intervals):
    """Bytes of (contig index, start, length, rc) intervals on a device
    genome: one kernel launch."""
    ex = np.zeros(len(intervals), dtype=engine.EXON_DTYPE)
    for i, (c, st, ln, rc) in enumerate(intervals):
        ex[i] = ((st | (1 << 63)) if rc else st, c, ln)
    tx = np.zeros(len(intervals), dtype=engine.TX_DTYPE)
    tx['exon_begin'] = np.arange(len(intervals))
    tx['n_exons'] = 1
    nuc, noff, _, _ = engine.extract_records(dev, ex, tx, engine.OUT_NUC)
    return [nuc[int(noff[i]):int(noff[i + 1])].tobytes() for i in range(len(intervals))]


def _match_fasta(g, order):
    """genome_tools.py:268-271 / 277-280: every match record's get_fasta(),
    joined with newlines and printed; all records gathered in one launch
    (AnnotationSet.get_fasta('match') is that same join).  The match dict is
    built by insertion, never copied: Python-2 order after zero copies."""
    if 'match' not in g.annotations.__dict__:
        raise AttributeError("AnnotationSet instance has no attribute 'match'")
    _write(g.annotations.get_fasta('match', order=order) + '\n')


def blast_csv2fasta(genome_sequence, blast_csv, order='py2'):
    """genome_tools.py:265-271: BLAST -outfmt 10 hits -> subject sequences
    (reverse-complemented where the subject runs backwards)."""
    g = genome.Genome(genome_sequence)
    g.read_blast_csv(blast_csv)
    _match_fasta(g, order)


def exonerate2fasta(genome_sequence, exonerate_file, order='py2'):
    """genome_tools.py:274-280: exonerate vulgar alignments -> the target
    sequence of each alignment's aligned blocks, spliced."""
    g = genome.Genome(genome_sequence)
    g.read_exonerate(exonerate_file)
    _match_fasta(g, order)


def get_seq_from_fasta(genome_sequence, seq_name, truncate_names='False'):
    """genome_tools.py:483-485: one contig as FASTA (host only: a whole
    contig is a copy, not a gather)."""
    g = genome.Genome(genome_sequence, truncate_names=_literal(truncate_names))
    _write(g.get_scaffold_fasta(seq_name) + '\n')


TOOLS = {'gff2fasta': gff2fasta, 'cds2pep': cds2pep,
         'extract_upstream_downstream': extract_upstream_downstream,
         'coords2fasta': coords2fasta,
         'blast_csv2fasta': blast_csv2fasta, 'exonerate2fasta': exonerate2fasta,
         'get_seq_from_fasta': get_seq_from_fasta}


def parse_argv(argv):
    """['tool', 'pos', 'k=v', ...] -> (tool, positional, keywords) as the
    reference's main() assembles them (genome_tools.py:35-44: only the text
    between the first and second '=' is the value)."""
    name = argv[0]
    args, kw = [], {}
    for a in argv[1:]:
        if '=' in a:
            parts = a.split('=')
            kw[parts[0]] = parts[1]
        else:
            args.append(a)
    return name, args, kw


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    if not argv or argv[0] in ('-h', '-help', '--help', 'help'):
        sys.stdout.write(__doc__)
        return 0
    name, args, kw = parse_argv(argv)
    if name not in TOOLS:
        sys.stderr.write('unknown tool %r (extraction path tools: %s)\n'
                         % (name, ', '.join(sorted(TOOLS))))
        return 2
    TOOLS[name](*args, **kw)
    return 0


if __name__ == '__main__':
    sys.exit(main())
