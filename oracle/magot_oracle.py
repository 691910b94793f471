"""CPU ORACLE for the MAGOT extraction path -- TEST INFRASTRUCTURE ONLY.

This module is a from-scratch Python 3 restatement of the semantics of the
reference's CDS extraction path (``/root/reference/genome.py``, Python 2.7).
It exists to CHECK the MI355X product (``magot_amd``); it is never imported by
the product.  Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may use it.

Pinning ("Oracle and parity"):
  * ``test_data/test_suite.py:12,13,14`` cksums reproduced on the C14 genome
    rebuilt from the reference's own fixtures (``tests/golden/c14.py``);
  * O.biroi outputs captured from the lib2to3 copy of the reference in the
    build container (``tests/golden/make_golden.py``), both record orders;
  * SURVEY Appendix A known-answer vectors (``tests/golden/kat.json``).

Every function cites the reference lines it restates.  Semantics are those of
the Python-2 reference (e.g. ``AnnotationSet.__getitem__`` does not see
``__dict__``), not of a Python-3 port of it.
"""

import copy
import sys

# ---------------------------------------------------------------------------
# Sequence arithmetic (genome.py:781-851)
# ---------------------------------------------------------------------------

# genome.py:787 -- every byte outside this map becomes lowercase 'n'
_RC_MAP = {'a': 't', 't': 'a', 'g': 'c', 'c': 'g', 'A': 'T', 'T': 'A',
           'G': 'C', 'C': 'G', 'n': 'n', 'N': 'N', '-': '-'}

# genome.py:795-802 -- the standard code, written here as (first base row,
# second base column, third base) walk TCAG x TCAG x TCAG.
_AA_BY_TCAG = ('FFLLSSSSYY**CC*W'
               'LLLLPPPPHHQQRRRR'
               'IIIMTTTTNNKKSSRR'
               'VVVVAAAADDEEGGGG')


def _standard_library():
    order = 'TCAG'
    lib = {}
    n = 0
    for a in order:
        for b in order:
            for c in order:
                lib[a + b + c] = _AA_BY_TCAG[n]
                n += 1
    return lib


STANDARD_CODE = _standard_library()


def reverse_complement(s):
    """genome.py:784-793 (Sequence.reverse_compliment)."""
    return ''.join(_RC_MAP.get(ch, 'n') for ch in reversed(s))


def translate(s, library=None, frame=0, strand='+', trimX=True):
    """genome.py:795-822 (Sequence.translate).

    Returns None when ``len(seq) <= 2 + frame`` (genome.py:810).  Residue
    positions run over ``range(frame, len)`` and a codon is emitted whenever
    ``(pos + frame) % 3 == 2`` -- so frames 1 and 2 start with a 1- or 2-char
    junk codon (genome.py:811-818).  Unknown triplets become 'X'; one leading
    'X' is dropped when trimX (genome.py:819-821).
    """
    if library is None:
        library = STANDARD_CODE
    if strand == '+':
        seq = s
    elif strand == '-':
        seq = reverse_complement(s)
    else:
        # genome.py:806-809 leave ``seq`` unbound: UnboundLocalError
        raise UnboundLocalError("local variable 'seq' referenced before assignment")
    if not len(seq) > (2 + frame):
        return None
    out = []
    trip = ''
    for pos in range(frame, len(s)):
        trip += seq[pos].upper()
        if (pos + frame) % 3 == 2:
            out.append(library.get(trip, 'X'))
            trip = ''
    pep = ''.join(out)
    if trimX and pep[0] == 'X':
        pep = pep[1:]
    return pep


def get_orfs(s, longest=False, strand='both', from_atg=False):
    """genome.py:824-851 (Sequence.get_orfs); the ``strand`` argument is
    shadowed by the loop variable (genome.py:830) and therefore ignored."""
    orfs = []
    cands = []
    best = 0
    for frame in (0, 1, 2):
        for st in ('-', '+'):
            t = translate(s, frame=frame, strand=st)
            if not t:
                continue
            for orf in t.split('*'):
                if from_atg:
                    out = 'M' + ''.join(orf.split('M')[1:])
                else:
                    out = orf
                if longest:
                    if len(out) > best:
                        cands.append(out)
                        best = len(out)
                else:
                    orfs.append(out)
    if longest:
        return cands[-1]
    return orfs


# ---------------------------------------------------------------------------
# Input helpers (magot_smallfuncs.py:32-43)
# ---------------------------------------------------------------------------

def _lines(src):
    """magot_smallfuncs.ensure_file: a path is opened, anything that fails to
    open is treated as literal content.  Lines split on '\\n' only (Python-2
    file iteration), bytes decoded latin-1 so every byte survives."""
    if src is None:
        return None
    if hasattr(src, 'read'):
        data = src.read()
    else:
        try:
            with open(src, 'rb') as fh:
                data = fh.read()
        except (OSError, ValueError, TypeError):
            data = src
    if isinstance(data, bytes):
        data = data.decode('latin-1')
    return _split_keep_nl(data)


def _split_keep_nl(text):
    out = []
    start = 0
    n = len(text)
    while start < n:
        j = text.find('\n', start)
        if j < 0:
            out.append(text[start:])
            break
        out.append(text[start:j + 1])
        start = j + 1
    return out


# ---------------------------------------------------------------------------
# Genome store (genome.py:854-877)
# ---------------------------------------------------------------------------

def read_fasta(src, truncate_names=False):
    """genome.py:856-877 (GenomeSequence.__init__): dict seqid -> str."""
    out = {}
    lines = _lines(src)
    if lines is None:
        return out
    name = ''
    parts = []
    for line in lines:
        if line[0] == '>':
            head = line[1:].replace('\r', '').replace('\n', '')
            if truncate_names is True:
                head = head.split()[0]
            seq = ''.join(parts)
            if seq != '':
                out[name] = seq
            parts = []
            name = head
        else:
            parts.append(line.replace('\r', '').replace('\n', ''))
    seq = ''.join(parts)
    if seq != '':
        out[name] = seq
    return out


# ---------------------------------------------------------------------------
# Annotation model (genome.py:524-778)
# ---------------------------------------------------------------------------

_GETSEQ_FAIL = ("either base_annotation has not annotation_set, or annotation_set has "
                "no genome, or genome has no            genome sequence, or genome "
                "sequence has no matching seqid, or coords are out of range on that seqid")
_MIXED = "ParentAnnotation has both ParentAnnotation and BaseAnnotation children!"
_NO_PARENT = ("It seems that this line has a parent attribute but that that parent doesn't "
              "have a line itself nor\n                    does this line have a defline "
              "attribute that specifies a parent type. I'm afraid this function can't "
              "currently\n                    deal with that.")


class OracleGenome(object):
    def __init__(self, seqs):
        self.genome_sequence = seqs


class OracleSet(object):
    """genome.py:524-545.  Feature-type dicts live in the instance __dict__."""

    def __init__(self, genome=None):
        self.gene = {}
        self.transcript = {}
        self.CDS = {}
        self.UTR = {}
        self.genome = genome

    def lookup(self, item):
        """genome.py:536-544: scan attributes in sorted (``dir``) order, keep
        the LAST dict that holds ``item``; KeyError when none does.  Python 2
        old-style ``dir`` lists no ``__dict__``, so only instance attributes
        holding dicts take part."""
        hit = None
        found = False
        for name in sorted(self.__dict__):
            val = self.__dict__[name]
            if type(val) is dict:
                try:
                    hit = val[item]
                    found = True
                except (KeyError, TypeError):
                    pass
        if not found:
            raise KeyError(item)
        return hit

    def get_fasta(self, feature, seq_type='nucleotide', longest=False, genomic=False,
                  order=None, out=None):
        """genome.py:578-582.  ``order`` may give an explicit key order (the
        Python-2 dict-order emulation); default is insertion order."""
        d = getattr(self, feature)
        keys = list(d) if order is None else order
        return '\n'.join(get_fasta(d[k], self, seq_type, longest, genomic, out=out)
                         for k in keys)


class OBase(object):
    """genome.py:586-598 (BaseAnnotation)."""

    def __init__(self, ID, seqid, coords, feature_type, parent, strand, attrs, aset):
        self.ID = ID
        self.seqid = seqid
        self.coords = coords
        self.feature_type = feature_type
        self.annotation_set = aset
        for k in attrs:
            setattr(self, k, attrs[k])
        self.parent = parent
        self.strand = strand


class OParent(object):
    """genome.py:652-661 (ParentAnnotation)."""

    def __init__(self, ID, seqid, feature_type, child_list, parent, strand, aset, attrs):
        self.ID = ID
        self.seqid = seqid
        self.feature_type = feature_type
        self.child_list = list(child_list)
        self.parent = parent
        self.annotation_set = aset
        self.strand = strand
        for k in attrs:
            setattr(self, k, attrs[k])


def _say(out, text):
    (out or sys.stdout).write(str(text) + '\n')


def get_seq(obj, out=None):
    """genome.py:603-614 (BaseAnnotation.get_seq)."""
    try:
        if obj.strand == '+' or obj.strand == '.':
            contig = obj.annotation_set.genome.genome_sequence[obj.seqid]
            return contig[obj.coords[0] - 1:obj.coords[1]]
        elif obj.strand == '-':
            contig = obj.annotation_set.genome.genome_sequence[obj.seqid]
            return reverse_complement(contig[obj.coords[0] - 1:obj.coords[1]])
        else:
            _say(out, obj.ID + ' has invalid strand value "' + obj.strand + '"')
    except Exception:
        _say(out, _GETSEQ_FAIL)
        _say(out, obj.seqid)
    return None


def get_coords(obj):
    """genome.py:600-601 / 663-675."""
    if isinstance(obj, OBase):
        return obj.coords
    if len(obj.child_list) > 0 and obj.annotation_set is not None:
        pts = []
        for child in obj.child_list:
            c = obj.annotation_set.lookup(child)
            if isinstance(c, OParent):
                pts = pts + list(get_coords(c))
            elif isinstance(c, OBase):
                pts = pts + list(c.coords)
        return (min(pts), max(pts))
    return None


def get_fasta(obj, aset, seq_type='nucleotide', longest=False, genomic=False,
              name_from='ID', out=None):
    """genome.py:677-731 (ParentAnnotation.get_fasta)."""
    if not isinstance(obj, OParent):
        raise AttributeError("BaseAnnotation instance has no attribute 'get_fasta'")
    if genomic is True:
        if obj.annotation_set.genome is not None:
            span = get_coords(obj)
            contig = obj.annotation_set.genome.genome_sequence[obj.seqid]
            return '>' + obj.ID + '\n' + contig[span[0] - 1:span[1]] + '\n'
        return None
    if not (len(obj.child_list) > 0 and obj.annotation_set is not None):
        return ''
    s = obj.annotation_set
    if s.genome is None:
        return ''
    records = []
    first = s.lookup(obj.child_list[0])
    if isinstance(first, OBase):
        by_coords = {}
        strand = None
        for child in obj.child_list:
            c = s.lookup(child)
            try:
                key = c.coords
                by_coords[key] = get_seq(c, out) if isinstance(c, OBase) else _no_get_seq()
            except AttributeError:
                _say(out, _MIXED)
                _say(out, obj.ID)
            strand = c.strand
        keys = sorted(by_coords)
        if strand == '-':
            keys.reverse()
        parts = [by_coords[k] for k in keys]
        if seq_type == 'nucleotide':
            seq = ''.join(parts)
        elif seq_type == 'protein':
            seq = translate(''.join(parts))
        else:
            _say(out, seq_type + ' is not valid seq_type. Please specify "protein" or "nucleotide".')
            raise UnboundLocalError("local variable 'new_seq' referenced before assignment")
        records.append('>' + obj.__dict__[name_from] + '\n' + seq)
    else:
        for child in obj.child_list:
            c = s.lookup(child)
            try:
                sub = get_fasta(c, s, seq_type=seq_type, name_from=name_from, out=out)
                if sub != '':
                    records.append(sub)
            except AttributeError:
                _say(out, _MIXED)
                _say(out, obj.ID)
    if longest is True:
        by_len = {}
        for rec in records:
            by_len[len(''.join(rec.split('\n')[1:]))] = rec
        return by_len[max(list(by_len))]
    return '\n'.join(records)


def _no_get_seq():
    raise AttributeError("ParentAnnotation instance has no attribute 'get_seq'")


# ---------------------------------------------------------------------------
# GFF3 / GTF walker (genome.py:242-415)
# ---------------------------------------------------------------------------

def read_gff(src, base_features=('CDS', 'match_part', 'similarity', 'region'),
             features_to_ignore=('exon',), gff_version='auto', parents_hierarchy=(),
             features_to_replace=(), IDfield='ID', parent_field='Parent', out=None, into=None):
    """genome.py:242-415 (module read_gff), presets omitted (not on the path).

    Returns an OracleSet, or None where the reference returns None.  ``into``
    is annotation_set_to_modify: that set is filled in place and returned
    (no deep copy, genome.py:413-415).
    """
    base_features = list(base_features)
    features_to_ignore = list(features_to_ignore) if not isinstance(features_to_ignore, str) \
        else features_to_ignore
    parents_hierarchy = list(parents_hierarchy)
    repl = {'\n': '', '\r': ''}
    for pair in features_to_replace:
        repl['\t' + pair[0] + '\t'] = '\t' + pair[1] + '\t'
    version = gff_version
    aset = OracleSet() if into is None else into
    renames = {}
    for raw in _lines(src):
        if raw[0] == '#' or raw.count('\t') != 8:
            continue
        line = raw
        for k in repl:
            line = line.replace(k, repl[k])
        f = line.split('\t')
        # version sniffing on the first accepted line (genome.py:288-300)
        if version == 'auto':
            if '=' in f[8]:
                version = 3
            else:
                version = 2
                if IDfield is not None:
                    if (' ' + IDfield + ' ') not in (' ' + f[8].replace(';', ' ')) \
                            and parents_hierarchy == []:
                        IDfield = None
                        parent_field = None
                        if 'gene_id' in f[8] and 'transcript_id' in f[8]:
                            parents_hierarchy = ['transcript_id', 'gene_id']
                        elif 'gene_id' in f[8]:
                            parents_hierarchy = ['gene_id']
        seqid = f[0]
        attrs = {'source': f[1]}
        ftype = f[2]
        if ftype in features_to_ignore:
            continue
        coords = tuple(sorted((int(f[3]), int(f[4]))))
        try:
            attrs['score'] = float(f[5])
        except ValueError:
            pass
        strand = f[6]
        if f[7] in ('0', '1', '2'):
            attrs['phase'] = int(f[7])
        tags = {}
        for fld in f[8].split(';'):
            if fld == '':
                continue
            if parent_field == '':
                tags[''] = fld
            elif version == 2:
                if '"' in fld:
                    tags[fld.split()[0]] = fld.split('"')[1]
                else:
                    try:
                        tags[fld.split()[0]] = fld.split()[1]
                    except Exception:
                        _say(out, fld)
                        return None
            elif version == 3:
                tags[fld.split('=')[0]] = fld.split('=')[1]
        parent = None
        if parent_field is not None:
            if parent_field in tags:
                parent = tags[parent_field]
        elif parents_hierarchy != []:
            for pt in parents_hierarchy:
                if pt in tags:
                    parent = tags[pt]
                    break
        # ID synthesis (genome.py:344-353)
        ID = None
        if IDfield is not None:
            try:
                ID = tags[IDfield]
            except KeyError:
                if parent is not None:
                    ID = parent + '-' + ftype
        elif parent is not None:
            ID = parent + '-' + ftype
        else:
            ID = seqid + '-' + ftype + f[3]
        # dedupe (genome.py:355-364): the renamed ID is not re-checked
        try:
            aset.lookup(ID)
            if ID in renames:
                renames[ID] += 1
                ID = ID + '-' + str(renames[ID])
            else:
                renames[ID] = 2
                ID = ID + '2'
        except KeyError:
            pass
        # parents (genome.py:366-399)
        if parent is not None:
            child = ID
            for i, pf in enumerate(parents_hierarchy):
                if pf in tags:
                    pid = tags[pf]
                    ptype = pf.split('_')[0]
                    pparent = None
                    if i != len(parents_hierarchy) - 1:
                        for ppf in parents_hierarchy[i + 1:]:
                            if ppf in tags:
                                pparent = tags[ppf]
                    if ptype not in aset.__dict__:
                        aset.__dict__[ptype] = {}
                    tbl = aset.__dict__[ptype]
                    if pid in tbl:
                        if child not in tbl[pid].child_list:
                            tbl[pid].child_list.append(child)
                    else:
                        tbl[pid] = OParent(pid, seqid, ptype, [child], pparent, strand, aset, {})
                    child = pid
            try:
                p = aset.lookup(parent)
                if ID not in p.child_list:
                    p.child_list.append(ID)
            except KeyError:
                _say(out, _NO_PARENT)
                _say(out, ID)
                _say(out, parent)
                return None
        for k in tags:
            if k not in (IDfield, parent_field):
                attrs[k] = tags[k]
        if ftype not in aset.__dict__:
            aset.__dict__[ftype] = {}
        if ftype in base_features:
            aset.__dict__[ftype][ID] = OBase(ID, seqid, coords, ftype, parent, strand, attrs, aset)
        else:
            aset.__dict__[ftype][ID] = OParent(ID, seqid, ftype, [], parent, strand, aset, attrs)
    return copy.deepcopy(aset) if into is None else aset


def load(fasta, gff, truncate_names=False, **kw):
    """Genome(fasta) + Genome.read_gff(gff) (genome.py:883-887, 970-975)."""
    g = OracleGenome(read_fasta(fasta, truncate_names=truncate_names))
    aset = read_gff(gff, **kw)
    aset.genome = g
    return aset


# ---------------------------------------------------------------------------
# Python 2.7 dict iteration order (CPython 2.7
# Objects/dictobject.c + Objects/stringobject.c string_hash)
# ---------------------------------------------------------------------------

_M64 = (1 << 64) - 1


def py2_str_hash(s):
    if not s:
        return 0
    x = (ord(s[0]) << 7) & _M64
    for ch in s:
        x = ((1000003 * x) & _M64) ^ ord(ch)
    x ^= len(s)
    if x == _M64:          # -1 is reserved
        x = _M64 - 1
    return x


def _py2_insert(table, key, h):
    mask = len(table) - 1
    i = h & mask
    perturb = h
    while True:
        k = table[i & mask]
        if k is None:
            table[i & mask] = key
            return True
        if k == key:
            return False
        i = (5 * i + perturb + 1) & _M64
        perturb >>= 5


def py2_dict_order(keys):
    """Slot order of a Python 2.7 dict into which ``keys`` were inserted."""
    table = [None] * 8
    used = 0
    for k in keys:
        if _py2_insert(table, k, py2_str_hash(k)):
            used += 1
            if used * 3 >= len(table) * 2:
                need = (2 if used > 50000 else 4) * used
                size = 8
                while size <= need:
                    size <<= 1
                old = table
                table = [None] * size
                for k2 in old:
                    if k2 is not None:
                        _py2_insert(table, k2, py2_str_hash(k2))
    return [k for k in table if k is not None]


def py2_order_after_deepcopy(keys):
    """read_gff's ``copy.deepcopy`` (genome.py:415) re-inserts in iteration order."""
    return py2_dict_order(py2_dict_order(keys))


def gff2fasta(fasta, gff, seq_type='nucleotide', longest=False, genomic=False, order='insertion',
              out=None, from_exons=False):
    """genome_tools.py:324-330: the text ``print`` writes.  from_exons reads
    with features_to_ignore="CDS" (a string: substring test, as :327 passes
    it) and exon -> CDS replaced."""
    kw = {'features_to_ignore': 'CDS', 'features_to_replace': [('exon', 'CDS')]} if from_exons else {}
    aset = load(fasta, gff, out=out, **kw)
    keys = None
    if order == 'py2':
        keys = py2_order_after_deepcopy(list(aset.gene))
    return aset.get_fasta('gene', seq_type=seq_type, longest=longest, genomic=genomic,
                          order=keys, out=out) + '\n'


def cds2pep(fasta, out=None):
    """genome_tools.py:664-675: header lines echoed, each record translated.
    With ``out`` (a text stream) every line is written as the reference
    prints it, so a blank line's IndexError (:668, ``line[0]``) leaves the
    lines before it; without, the text is returned."""
    outl = []
    sink = (lambda t: out.write(t + '\n')) if out is not None else outl.append
    work = ''
    for raw in _lines(fasta):
        line = raw.replace('\n', '').replace('\r', '')
        if line[0] == '>':
            if work != '':
                sink(str(translate(work)))
                work = ''
            sink(line)
        else:
            work = work + line
    sink(str(translate(work)))
    return '\n'.join(outl) + '\n' if out is None else None


# ---------------------------------------------------------------------------
# Locus extraction: genome_tools.py:457-480 and :656-661
# ---------------------------------------------------------------------------

def extract_upstream_downstream(genome_sequence, gff_path, sequence_length, stream,
                                feature_type='gene', namefrom='ID', truncate_names='True',
                                out=None):
    """genome_tools.py:457-480.  Returns the printed text; exceptions propagate
    after whatever the reference would have printed (nothing: it prints once,
    at the end)."""
    seqs = read_fasta(genome_sequence, truncate_names=truncate_names == 'True')
    output_seqs = []
    sequence = None
    bound = False
    with open(gff_path, 'rb') as fh:
        text = fh.read().decode('latin-1')
    for line in _split_keep_nl(text):
        if line.count('\t') > 5 and line[0] != '#':
            fields = line.split('\t')
            if fields[2] == feature_type:
                name = None
                coords = [int(fields[3]), int(fields[4])]
                coords.sort()
                for attribute in fields[-1].split(';'):
                    if namefrom == attribute.split('=')[0]:
                        name = attribute.split('=')[1].replace('\r', '').replace('\n', '')
                if name is None:
                    name = 'seq' + str(len(output_seqs))
                # int(sequence_length) where the reference evaluates it: in a
                # branch, then in the comparison (after the unbound check)
                if stream == 'up' and fields[6] == '+' or stream == 'down' and fields[6] == '-':
                    stop = coords[0] - 1
                    sequence = seqs[fields[0]][stop - int(sequence_length):stop]
                    bound = True
                elif stream == 'down' and fields[6] == '+' or stream == 'up' and fields[6] == '-':
                    start = coords[1]
                    sequence = reverse_complement(
                        seqs[fields[0]][start:start + int(sequence_length)])
                    bound = True
                if not bound:
                    raise UnboundLocalError("local variable 'sequence' referenced before "
                                            "assignment")
                if len(sequence) == int(sequence_length):
                    output_seqs.append('>' + name + '\n' + sequence)
    return '\n'.join(output_seqs) + '\n'


def coords2fasta(fasta_file, seqid, start, stop, truncate_names='False', out=None):
    """genome_tools.py:656-661: (text printed, exception or None)."""
    text = '>' + seqid + ':' + start + '-' + stop + '\n'
    try:
        seq = read_fasta(fasta_file, truncate_names=truncate_names == 'True')[seqid][
            int(start) - 1:int(stop)]
    except Exception as e:  # noqa: BLE001 -- the header is printed before the lookup
        return text, e
    return text + seq + '\n', None



# ---------------------------------------------------------------------------
# Aligner outputs (genome.py:32-121, 425-499) and their extraction tools
# (genome_tools.py:265-280, 483-485)
# ---------------------------------------------------------------------------

def vulgar2gff(v, feature_types=('match', 'match_part'), source='exonerate'):
    """genome.py:32-86.  v = vulgar fields: query, qstart, qend, qstrand,
    target, tstart, tend, tstrand, score, then (op, query len, target len)
    triplets.  The target cursor starts at tstart+1 ('+') or tstart ('-',
    whose end also moves up by one); it advances by each target length, and
    every run of M/S/G/F ops is one match_part whose bounds are the min and
    max of its cursor positions compared as strings."""
    qname = v[0] + '-against-' + v[4]
    tname, tstart, tend, tstrand, score = v[4], v[5], v[6], v[7], v[8]
    if tstrand == '+':
        cur = int(tstart) + 1
    else:
        cur = int(tstart)
        tend = str(int(tend) + 1)
    out = [tname + '\t' + source + '\t' + feature_types[0] + '\t' + str(cur) + '\t' + tend +
           '\t' + score + '\t' + tstrand + '\t.\tID=' + qname]
    part = None      # cursor positions (strings) of the open match_part
    n = 0

    def close():
        out.append('\t'.join([tname, source, feature_types[1], min(part), max(part), '.',
                              tstrand, '.', 'ID=%s_%s%d;Parent=%s' % (qname, feature_types[1],
                                                                     n + 1, qname)]))

    trips = v[9:]
    for i, f in enumerate(trips):
        if i % 3 == 0:
            if f in ('M', 'S', 'G', 'F'):
                if part is None:
                    part = [str(cur)]
            elif part is not None:
                close()
                n += 1
                part = None
        elif i % 3 == 2:
            step = int(f)
            if tstrand == '+':
                cur += step
                if part is not None:
                    part.append(str(cur - 1))
            elif tstrand == '-':
                cur -= step
                if part is not None:
                    part.append(str(cur + 1))
    if part is not None:
        close()
    return '\n'.join(out)


def read_exonerate(src, into=None):
    """genome.py:88-121."""
    aset = OracleSet() if into is None else into
    q = t = ''
    seen = {}
    gff = []
    for raw in _lines(src):
        line = raw.replace('\r', '').replace('\n', '')
        if line.startswith('         Query: '):
            q = line[16:]
        elif line.startswith('        Target: '):
            t = line[16:].replace(':[revcomp]', '').replace('[revcomp]', '')
            if t[-1] == ' ':
                t = t[:-1]
        elif line.startswith('vulgar: '):
            v = line[8:].split()
            v[0], v[4] = q, t
            k = q + '-against-' + t
            if k in seen:
                v[0] = q + str(seen[k])
                seen[k] += 1
            else:
                seen[k] = 1
            gff.append(vulgar2gff(v))
    read_gff('\n'.join(gff), into=aset)
    return aset


def read_blast_csv(src, into=None, hierarchy=('match', 'match_part'), source='blast',
                   find_truncated_locname=False, out=None):
    """genome.py:425-499 (fields: 0 query, 1 subject, 8/9 subject start/end,
    10 evalue, 11 score)."""
    aset = OracleSet() if into is None else into
    base = hierarchy[-1]
    parents = list(hierarchy[:-1])[::-1]
    if base not in aset.__dict__:
        aset.__dict__[base] = {}
    names = None
    if find_truncated_locname:
        if aset.genome is None:
            _say(out, '"warning: find_truncated_locname" was set to true, but annotation set '
                      'has no associated genome object so this cannot be done')
        else:
            names = list(aset.genome.genome_sequence)
    counters = {}
    for raw in _lines(src):
        f = raw.replace('\r', '').replace('\n', '').split(',')
        if len(f) <= 8:
            continue
        sid = f[1]
        if names is not None and sid not in names:
            sid = next((n for n in names if n.split()[0] == sid), sid)
        a, b = int(f[8]), int(f[9])
        coords, strand = ((a, b), '+') if a < b else ((b, a), '-')
        score, qid = f[11], f[0]
        tbl = aset.__dict__[base]
        if qid in tbl:
            while True:
                ID = qid + '-' + str(counters[qid])
                counters[qid] += 1
                if ID not in tbl:
                    break
        else:
            ID = qid
            counters[qid] = 1
        attrs = {'evalue': f[10], 'score': score}
        child = ID
        for i, pt in enumerate(parents):
            up = ID + '-' + parents[i + 1] if i < len(parents) - 1 else None
            aset.__dict__.setdefault(pt, {})[ID + '-' + pt] = OParent(
                ID + '-' + pt, sid, pt, [child], up, strand, aset, {})
            child = ID + '-' + pt
        tbl[ID] = OBase(ID, sid, coords, base, ID + '-' + parents[0], strand, attrs, aset)
    return aset


def _match_tool(aset, order, out=None):
    d = getattr(aset, 'match')  # AttributeError without any match (the reference's loop)
    keys = py2_dict_order(list(d)) if order == 'py2' else list(d)
    return '\n'.join(get_fasta(d[k], aset, out=out) for k in keys) + '\n'


def blast_csv2fasta(fasta, blast_csv, order='insertion', out=None):
    """genome_tools.py:265-271 -> stdout text (record order: the match dict's,
    insertion or Python 2 after zero copies)."""
    aset = OracleSet(OracleGenome(read_fasta(fasta)))
    read_blast_csv(blast_csv, into=aset, out=out)
    return _match_tool(aset, order, out)


def exonerate2fasta(fasta, exonerate_output, order='insertion', out=None):
    """genome_tools.py:274-280 -> stdout text."""
    aset = OracleSet(OracleGenome(read_fasta(fasta)))
    read_exonerate(exonerate_output, into=aset)
    return _match_tool(aset, order, out)


def get_seq_from_fasta(fasta, seq_name, truncate_names='False'):
    """genome_tools.py:483-485 -> stdout text."""
    seqs = read_fasta(fasta, truncate_names=truncate_names == 'True')
    return '>' + seq_name + '\n' + seqs[seq_name] + '\n'
