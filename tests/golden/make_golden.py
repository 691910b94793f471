"""Regenerate the golden vectors in tests/golden/*.json from the REFERENCE.

Runs only in the build container (never on the GPU box): it needs the
reference at /root/reference.  The reference is Python 2.7; importing it under
Python 3.10 fails with an ordinary SyntaxError, so this script makes a
mechanical lib2to3 copy in /tmp/magot_py3 (outside the repository) and imports
that.  On this path the only Python-2/3 difference is dict iteration order,
handled by re-ordering the gene dict with the Python-2 order model
(oracle.magot_oracle.py2_order_after_deepcopy), which is itself pinned by
test_data/test_suite.py:12-13 (see tests/test_oracle.py).

Outputs (data only: inputs, expected outputs, hashes):
  kat.json        Sequence.reverse_compliment / translate / get_orfs vectors
  edge_cases.json get_fasta edge cases incl. stdout/exception
  fixtures.json   hashes of whole-file gff2fasta outputs on the shipped data
  synth_small.json hashes of gff2fasta on the seeded small synthetic
  loci.json       extract_upstream_downstream / coords2fasta outputs (stdout)
  flank_edges.json extract_upstream_downstream on the native flank planner's edge cases
  flank_fuzz.json  extract_upstream_downstream on random GFFs
  coords_fuzz.json coords2fasta on random windows of the O.biroi contigs
  matches.json    blast_csv2fasta / exonerate2fasta / get_seq_from_fasta outputs
  blast_fuzz.json blast_csv2fasta on random BLAST tables
  fuzz.json       random small GFF3/GTF cases through gff2fasta's path
  fuzz3.json      200 more of them (another seed)
  fuzz4.json      120 more cases of fuzz2.json's generator (another seed)
  translate_lib.json Sequence.translate with non-standard libraries, frames -6..6

Usage:  python tests/golden/make_golden.py [--only-translate-lib | --only-flank-edges |
                                           --only-fuzz3 | --only-cds2pep2 |
                                           --only-blast-fuzz | --only-coords-fuzz |
                                           --only-synth]
"""

import contextlib
import hashlib
import io
import json
import os
import random
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

import goldlib  # noqa: E402
from oracle import magot_oracle as mo  # noqa: E402

REF = '/root/reference'
PY3 = '/tmp/magot_py3'
REF_FILES = ['genome.py', 'genome_tools.py', 'genome_tools_config.py', 'magot_smallfuncs.py',
             'magot_variants.py', 'annotation_funcs.py']


def reference_module():
    if not os.path.exists(os.path.join(PY3, 'genome.py')):
        os.makedirs(PY3, exist_ok=True)
        for f in REF_FILES:
            shutil.copy(os.path.join(REF, f), PY3)
            os.chmod(os.path.join(PY3, f), 0o644)
        subprocess.check_call([sys.executable, '-m', 'lib2to3', '-w', '-n'] +
                              [os.path.join(PY3, f) for f in REF_FILES],
                              stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    sys.path.insert(0, PY3)
    import genome as refgenome
    return refgenome


def sha(s):
    if isinstance(s, str):
        s = s.encode('latin-1')
    return hashlib.sha256(s).hexdigest()


def call(fn):
    """(result, exception name, captured stdout)."""
    buf = io.StringIO()
    res = None
    exc = None
    with contextlib.redirect_stdout(buf):
        try:
            res = fn()
        except Exception as e:  # noqa: BLE001
            exc = type(e).__name__
    return res, exc, buf.getvalue()


# ---------------------------------------------------------------------------

KAT_STRINGS = ['ATGGCCTTTAAACCCGGGTAG', 'NNNATGNNN', 'ATGRYKatgu', 'AT', 'ATGC',
               'ACGTRYacgtn-*.', 'ATGAAAMTAGCCCATGGGTAA', 'ATGAAAATGTAGCCCATGGGTAA', '', 'A',
               'ATG', 'atgaaatag', 'XATGCCC', 'ATGCCCGGGTTTAAACCC' * 3]


def make_kat(ref):
    rnd = random.Random(1015)
    alpha = 'ACGTACGTACGTacgtNnRYKMSW-.* U'
    strs = list(KAT_STRINGS)
    for n in list(range(0, 12)) + [17, 30, 31, 32, 33, 47, 48, 49, 64, 100]:
        for _ in range(3):
            strs.append(''.join(rnd.choice(alpha) for _ in range(n)))
    out = []
    for s in strs:
        S = ref.Sequence(s)
        rec = {'seq': s, 'revcomp': S.reverse_compliment(), 'translate': {}, 'orfs': {}}
        for frame in range(5):
            for strand in '+-':
                for trim in (True, False):
                    r, e, _ = call(lambda: S.translate(frame=frame, strand=strand, trimX=trim))
                    rec['translate']['%d%s%d' % (frame, strand, int(trim))] = \
                        {'exc': e} if e else r
        for longest in (False, True):
            for atg in (False, True):
                r, e, _ = call(lambda: S.get_orfs(longest=longest, from_atg=atg))
                rec['orfs']['%d%d' % (int(longest), int(atg))] = {'exc': e} if e else r
        out.append(rec)
    return out


# Codon libraries beyond the standard table (Sequence.translate's `library`,
# genome.py:795-818): keys that are not ACGT triplets ('NNN', IUPAC, the 1-
# and 2-character junk codons of frames 1/2), multi-character, empty and
# non-string values, lower-case keys that never match; frames -6..6.
TRANSLATE_LIBS = {
    'std+junk': ('standard', {'NNN': 'Z', 'A': 'a', 'AC': 'b', 'RYK': 'r', 'N-.': '#',
                              'ATGC': 'never'}),
    'multi': ('standard', {'ATG': 'Met', 'TAA': '', 'TAG': 'Stop', 'TGA': '*', 'GCC': 'XA'}),
    'sparse': (None, {'ATG': 'M', 'AAA': 'K', 'NNN': 'n', 'atg': 'lower', 'T': 'j'}),
    'intval': (None, {'ATG': 5, 'CCC': 'P'}),
    'empties': (None, {'ATG': '', 'CCC': '', 'GGG': 'G', 'TTT': ''}),
    'X-lead': ('standard', {'ATG': 'XM', 'GCC': 'X'}),
}


def translate_library(name, std):
    base, extra = TRANSLATE_LIBS[name]
    lib = dict(std) if base == 'standard' else {}
    lib.update(extra)
    return lib


def make_translate_lib(ref):
    std = ref.Sequence.translate.__defaults__[0]
    rnd = random.Random(1017)
    alpha = 'ACGTACGTACGTacgtNnRYKMSW-.*'
    strs = list(KAT_STRINGS)
    for n in (0, 1, 2, 3, 4, 5, 6, 7, 8, 11, 13, 20, 31, 40):
        for _ in range(2):
            strs.append(''.join(rnd.choice(alpha) for _ in range(n)))
    out = []
    for name in sorted(TRANSLATE_LIBS):
        lib = translate_library(name, std)
        for s in strs:
            S = ref.Sequence(s)
            for frame in range(-6, 7):
                for strand in '+-':
                    for trim in (True, False):
                        r, e, _ = call(lambda: S.translate(library=lib, frame=frame,
                                                           strand=strand, trimX=trim))
                        out.append({'lib': name, 'seq': s, 'frame': frame, 'strand': strand,
                                    'trim': trim, 'out': None if e else r, 'exc': e})
    return {'libs': {k: [v[0], v[1]] for k, v in TRANSLATE_LIBS.items()}, 'cases': out}


# ---------------------------------------------------------------------------

EDGE_GENOME = '>c1\nACGTACGTAAccggttNNRYacgtACGTAAATTTGGGCCC\n>c2 desc\nGGGAAATTTCCCgggaaatttccc\n'


def _gtf_line(seqid, start, end, strand, tid, gid, ftype='CDS'):
    return '%s\tt\t%s\t%d\t%d\t.\t%s\t0\ttranscript_id "%s"; gene_id "%s";\n' % (
        seqid, ftype, start, end, strand, tid, gid)


def _gff3(seqid, ftype, start, end, strand, attrs):
    return '%s\tt\t%s\t%d\t%d\t.\t%s\t.\t%s\n' % (seqid, ftype, start, end, strand, attrs)


def edge_case_inputs():
    g3h = _gff3('c1', 'gene', 1, 40, '+', 'ID=g') + _gff3('c1', 'mRNA', 1, 40, '+', 'ID=t;Parent=g')

    def cds(*ivs):
        return ''.join(_gff3(sid, 'CDS', a, b, s, 'ID=c;Parent=t') for sid, a, b, s in ivs)

    cases = {
        'dup_coords': g3h + cds(('c1', 1, 6, '+'), ('c1', 1, 6, '+'), ('c1', 10, 20, '+')),
        'minus_iupac': g3h + cds(('c1', 1, 6, '-'), ('c1', 10, 20, '-')),
        'mixed_strand': g3h + cds(('c1', 1, 6, '-'), ('c1', 10, 20, '+')),
        'mixed_strand_rev': g3h + cds(('c1', 1, 6, '+'), ('c1', 10, 20, '-')),
        'dot_strand': g3h + cds(('c1', 1, 6, '.')),
        'past_end': g3h + cds(('c1', 35, 99, '+')),
        'past_end_minus': g3h + cds(('c1', 35, 99, '-')),
        'start_zero': g3h + cds(('c1', 0, 5, '+')),
        'start_zero_past_end': g3h + cds(('c1', 0, 50, '+')),
        'reversed_coords': g3h + cds(('c1', 6, 1, '+')),
        'protein_n_codons': g3h + cds(('c1', 15, 20, '+'), ('c1', 1, 9, '+')),
        'protein_short': g3h + cds(('c1', 1, 2, '+')),
        'protein_len3_minus': g3h + cds(('c1', 18, 20, '-')),
        'bad_strand': g3h + cds(('c1', 1, 6, '?')),
        'missing_seqid': g3h + cds(('cX', 1, 6, '+')),
        'desc_seqid': _gff3('c2 desc', 'gene', 1, 9, '+', 'ID=g') +
        _gff3('c2 desc', 'mRNA', 1, 9, '+', 'ID=t;Parent=g') +
        _gff3('c2 desc', 'CDS', 1, 9, '+', 'ID=c;Parent=t'),
        'nine_tabs': g3h + cds(('c1', 1, 6, '+')).replace('\n', '\textra\n'),
        'gene_no_cds': g3h + _gff3('c1', 'gene', 1, 5, '+', 'ID=g2') + cds(('c1', 1, 6, '+')),
        'utr_after_cds': g3h + cds(('c1', 1, 6, '+')) +
        _gff3('c1', 'UTR', 7, 9, '+', 'ID=u;Parent=t'),
        'utr_first': g3h + _gff3('c1', 'UTR', 7, 9, '+', 'ID=u;Parent=t') + cds(('c1', 1, 6, '+')),
        'two_mrna': g3h + cds(('c1', 1, 9, '+')) + _gff3('c1', 'mRNA', 1, 40, '-', 'ID=t2;Parent=g') +
        _gff3('c1', 'CDS', 4, 30, '-', 'ID=c2;Parent=t2'),
        'child_before_parent': _gff3('c1', 'CDS', 1, 6, '+', 'ID=c;Parent=t') + g3h,
        'comment_lines': '#c\n' + g3h + '##x\n' + cds(('c1', 1, 12, '+')),
        'gtf_two_genes': _gtf_line('c1', 1, 9, '+', 't1', 'g1') + _gtf_line('c1', 12, 20, '+', 't1', 'g1') +
        _gtf_line('c2 desc', 1, 12, '-', 't2', 'g2'),
        'gtf_gene_only': 'c1\tt\tCDS\t1\t9\t.\t-\t0\tgene_id "gA";\nc1\tt\tCDS\t20\t30\t.\t-\t0\tgene_id "gA";\n',
        'exon_ignored': g3h + _gff3('c1', 'exon', 1, 40, '+', 'ID=e;Parent=t') + cds(('c1', 2, 13, '+')),
    }
    return cases


EDGE_CALLS = [('nucleotide', False, False), ('protein', False, False), ('nucleotide', True, False),
              ('nucleotide', False, True), ('protein', True, False)]


def make_edges(ref):
    out = []
    for name, gff in sorted(edge_case_inputs().items()):
        for seq_type, longest, genomic in EDGE_CALLS:
            def run():
                g = ref.Genome(EDGE_GENOME)
                g.read_gff(gff)
                return g.annotations.get_fasta('gene', seq_type=seq_type, longest=longest,
                                               genomic=genomic)
            r, e, so = call(run)
            out.append({'case': name, 'fasta': EDGE_GENOME, 'gff': gff, 'seq_type': seq_type,
                        'longest': longest, 'genomic': genomic, 'result': r, 'exc': e,
                        'stdout': so})
    return out


# ---------------------------------------------------------------------------

def ref_gff2fasta(ref, fasta, gff, seq_type='nucleotide', longest=False, genomic=False,
                  order='insertion', from_exons=False):
    def run():
        g = ref.Genome(fasta)
        if from_exons:  # genome_tools.py:327
            g.read_gff(gff, features_to_ignore="CDS", features_to_replace=[('exon', 'CDS')])
        else:
            g.read_gff(gff)
        if order == 'py2':
            keys = mo.py2_order_after_deepcopy(list(g.annotations.gene))
            g.annotations.gene = {k: g.annotations.gene[k] for k in keys}
        return g.annotations.get_fasta('gene', seq_type=seq_type, longest=longest,
                                       genomic=genomic) + '\n'
    return call(run)


def digest(res, exc, so):
    d = {'exc': exc, 'stdout_sha256': sha(so)}
    if res is not None:
        crc, size = goldlib.posix_cksum(res)
        d.update({'cksum': '%d %d' % (crc, size), 'sha256': sha(res)})
    return d


def make_fixture_hashes(ref):
    out = {}
    fa = goldlib.path('O.biroi_refseqGenomeSubset.fasta')
    gff = goldlib.path('O.biroi_NCBIrefseq_gff3Subset.gff')
    for seq_type in ('nucleotide', 'protein'):
        for order in ('insertion', 'py2'):
            out['obiroi/%s/%s' % (seq_type, order)] = digest(
                *ref_gff2fasta(ref, fa, gff, seq_type, order=order))
    out['obiroi/genomic/insertion'] = digest(*ref_gff2fasta(ref, fa, gff, genomic=True))
    out['obiroi/longest/insertion'] = digest(*ref_gff2fasta(ref, fa, gff, longest=True))
    c14 = goldlib.rebuild_c14()
    for ann in ('StandardGTF.gtf', 'transcriptlessGTF.gtf', 'minimalGFF3.gff'):
        for seq_type in ('nucleotide', 'protein'):
            for order in ('insertion', 'py2'):
                out['c14/%s/%s/%s' % (ann, seq_type, order)] = digest(
                    *ref_gff2fasta(ref, c14, goldlib.path(ann), seq_type, order=order))
    return out


def make_synth(ref):
    from magot_amd import synth
    w = synth.make('small')
    fa = w.fasta_text()
    out = {'fasta_sha256': sha(fa)}
    for fmt, text in (('gff3', w.gff3_text()), ('gtf', w.gtf_text())):
        out['%s_sha256' % fmt] = sha(text)
        for seq_type in ('nucleotide', 'protein'):
            out['%s/%s' % (fmt, seq_type)] = digest(*ref_gff2fasta(ref, fa, text, seq_type))
    return out


LOCUS_GENOME = ('>c1 first contig\nACGTACGTAAccggttNNRYacgtACGTAAATTTGGGCCCAATTGGCC\n'
                '>c2\nGGGAAATTTCCCgggaaatttcccAAACCCGGGTTT\n')
LOCUS_GFF = ''.join([
    'c1\tt\tgene\t10\t20\t.\t+\t.\tID=g1;Name=alpha\n',
    'c1\tt\tgene\t3\t8\t.\t-\t.\tID=g2\n',
    'c1\tt\tgene\t30\t40\t.\t-\t.\tName=gamma\n',
    '#c1\tt\tgene\t1\t5\t.\t+\t.\tID=hidden\n',
    'c2\tt\tgene\t20\t12\t.\t+\t.\tID=g4\n',
    'c2\tt\tmRNA\t12\t20\t.\t+\t.\tID=m4;Parent=g4\n',
    'c2\tt\tgene\t2\t5\t.\t+\t.\tID=g5\n',
])


FLANK_GENOME = '>c1 first contig\n' + 'ACGTTGCAACGGATCC' * 8 + '\n>c2\n' + 'TTAGGCAT' * 6 + '\n'
FLANK_CASES = [
    # (gff text, sequence_length, stream, feature_type, namefrom)
    ('c1\tt\tgene\t40\t50\t.\t+\t.\tID=a\nc1\tt\tgene\t60\t70\t.\t.\t.\tID=b\n'
     'c1\tt\tgene\t80\t90\t.\t?\t.\tName=z\n', '5', 'up', 'gene', 'ID'),
    ('c1\tt\tgene\t40\t50\t.\t-\t.\tID=a\nc1\tt\tgene\t60\t70\t.\t+\n', '5', 'down',
     'gene', 'ID'),
    ('c1\tt\tgene\t1\t9\t.\t+\t.\tID=a\nc1\tt\tgene\t0\t9\t.\t+\t.\tID=b\n'
     'c2\tt\tgene\t40\t48\t.\t+\t.\tID=c\nc2\tt\tgene\t2\t47\t.\t-\t.\tID=d\n', '4', 'up',
     'gene', 'ID'),
    ('c1\tt\tgene\t1\t9\t.\t+\t.\tID=a\nc1\tt\tgene\t0\t9\t.\t+\t.\tID=b\n'
     'c2\tt\tgene\t40\t48\t.\t+\t.\tID=c\nc2\tt\tgene\t2\t47\t.\t-\t.\tID=d\n', '4', 'down',
     'gene', 'ID'),
    ('#c1\tt\tgene\t5\t9\t.\t+\t.\tID=hidden\r\n'
     'c1\tt\tgene\t30\t20\t.\t+\t.\tID=x=y;Name=n; ID=no;ID=last\r\n'
     'c2\tt\tgene\t20\t30\t.\t-\t.\tName=q\r\n', '6', 'up', 'gene', 'ID'),
    ('c1\tt\tgene\t40\t50\t.\t+\t.\tID=a\nc2\tt\tgene\t10\t12\t.\t-\t.\n', '0', 'up',
     'gene', 'ID'),
    ('c1\tt\tgene\t40\t50\t.\t+\t.\tID=a\n', '-3', 'down', 'gene', 'ID'),
    ('c1\tt\tmRNA\t40\t50\t.\t+\t.\tID=a\n', '5', 'up', 'gene', 'ID'),
    ('', '5', 'up', 'gene', 'ID'),
    ('c1\tt\tgene\t40\t50\t.\t+\t.\tID=a\nnope\tt\tgene\t60\t70\t.\t.\t.\tID=b\n', '5',
     'up', 'gene', 'ID'),
    ('', '5', 'sideways', 'gene', 'ID'),
    ('c1\tt\tgene\t40\t50\t.\t+\t.\tName=a;Name=b=c;gene=g\n', '7', 'down', 'gene', 'Name'),
    ('c1\tt\tgene\t40\t50\t.\t+\t.\tID=a;\n', '5', 'up', 'gene', ''),
    ('c1\tt\tgene\t40\t50\t.\t.\t.\tID=a\n', '5', 'up', 'gene', 'ID'),
    ('c1\tt\tgene\t40\t50\t.\t+\t.\tID=a\n', '5', 'sideways', 'gene', 'ID'),
    ('nope\tt\tgene\t40\t50\t.\t+\t.\tID=a\n', '5', 'up', 'gene', 'ID'),
    ('c1\tt\tgene\t4x\t50\t.\t+\t.\tID=a\n', '5', 'up', 'gene', 'ID'),
    ('c1\tt\tgene\t40\t50\t.\t+\t.\tID;Name=a\n', '5', 'up', 'gene', 'ID'),
    ('c1\tt\tgene\t40\t50\t.\t+\t.\tID=a\n', 'five', 'up', 'gene', 'ID'),
    ('c1\tt\tgene\t40\t50\t.\t+\t.\tID=a\n', 'five', 'sideways', 'gene', 'ID'),
    ('nope\tt\tgene\t40\t50\t.\t+\t.\tID=a\n', 'five', 'up', 'gene', 'ID'),
]


def make_flank_edges(ref):
    """The reference's extract_upstream_downstream (:457-480) on the edge cases
    of the native flank planner (tests/test_flank.py): stdout and exception.
    No case ends a line with a lone '\\r' (Python 3's universal newlines would
    split there, Python 2's file iteration does not)."""
    sys.path.insert(0, PY3)
    import genome_tools as rt
    import tempfile
    cases = []
    with tempfile.TemporaryDirectory() as td:
        fa_path = os.path.join(td, 'g.fa')
        with open(fa_path, 'w') as fh:
            fh.write(FLANK_GENOME)
        for k, (gff, n, stream, ft, nf) in enumerate(FLANK_CASES):
            gff_path = os.path.join(td, 'a%d.gff' % k)
            with open(gff_path, 'w', newline='') as fh:
                fh.write(gff)
            _, exc, so = call(lambda: rt.extract_upstream_downstream(fa_path, gff_path, n, stream,
                                                                    ft, nf, 'True'))
            cases.append({'gff': gff, 'sequence_length': n, 'stream': stream,
                          'feature_type': ft, 'namefrom': nf, 'stdout': so, 'exc': exc})
    return {'genome': FLANK_GENOME, 'cases': cases}


def _flank_case(rnd):
    """A random GFF and call for extract_upstream_downstream: the feature type
    or others, every strand form, coordinates at and past the contig ends (0,
    negative, swapped), names present, repeated, absent or holding '=', CRLF
    and comment lines, lines with six tabs; lengths from 0 up and negative."""
    rows = []
    for _ in range(rnd.randint(0, 14)):
        if rnd.random() < 0.08:
            rows.append('#c1\tt\tgene\t1\t5\t.\t+\t.\tID=x')
            continue
        seqid = 'c1 first contig' if rnd.random() < 0.03 else rnd.choice(['c1', 'c2'])
        ftype = rnd.choice(['gene', 'gene', 'gene', 'mRNA', 'CDS'])
        a, b = rnd.randint(-5, 140), rnd.randint(-5, 140)
        strand = rnd.choice(['.', '?']) if rnd.random() < 0.1 else rnd.choice(['+', '-'])
        attrs = rnd.choice(['ID=g%d' % rnd.randint(0, 9),
                            'ID=g%d;Name=n%d' % (rnd.randint(0, 9), rnd.randint(0, 9)),
                            'Name=q', 'ID=a=b', 'x=1;ID=z;ID=w', ''])
        cols = [seqid, 't', ftype, str(a), str(b), '.', strand]
        if rnd.random() >= 0.1:
            cols += ['.', attrs]
        rows.append('\t'.join(cols))
    gff = ''.join(r + ('\r\n' if rnd.random() < 0.2 else '\n') for r in rows)
    n = rnd.choice(['0', '1', '4', '9', '30', '-2'])
    stream = 'both' if rnd.random() < 0.05 else rnd.choice(['up', 'down'])
    return gff, n, stream, rnd.choice(['gene', 'gene', 'mRNA']), rnd.choice(['ID', 'Name', 'x', ''])


def make_flank_fuzz(ref, n=150):
    """The reference's extract_upstream_downstream on random GFFs
    (_flank_case) over FLANK_GENOME: stdout and exception (tests/test_flank.py)."""
    sys.path.insert(0, PY3)
    import genome_tools as rt
    import tempfile
    rnd = random.Random(20261022)
    cases = []
    with tempfile.TemporaryDirectory() as td:
        fa_path = os.path.join(td, 'g.fa')
        with open(fa_path, 'w') as fh:
            fh.write(FLANK_GENOME)
        for k in range(n):
            gff, sl, stream, ft, nf = _flank_case(rnd)
            gff_path = os.path.join(td, 'a%d.gff' % k)
            with open(gff_path, 'w', newline='') as fh:
                fh.write(gff)
            _, exc, so = call(lambda: rt.extract_upstream_downstream(fa_path, gff_path, sl, stream,
                                                                    ft, nf, 'True'))
            cases.append({'gff': gff, 'sequence_length': sl, 'stream': stream,
                          'feature_type': ft, 'namefrom': nf, 'stdout': so, 'exc': exc})
    return {'genome': FLANK_GENOME, 'cases': cases}


def make_coords_fuzz(ref, n=60):
    """The reference's coords2fasta (:656-661) on random windows of the
    O.biroi contigs (starts at or below 0, stops past the end, reversed and
    empty windows, a malformed number, a missing contig): stdout digest and
    exception (tests/test_loci.py)."""
    sys.path.insert(0, PY3)
    import genome_tools as rt
    rnd = random.Random(20261023)
    fa = goldlib.path('O.biroi_refseqGenomeSubset.fasta')
    cases = []
    for _ in range(n):
        tr = rnd.choice(['True', 'False'])
        seqs = mo.read_fasta(fa, truncate_names=tr == 'True')
        name = rnd.choice(sorted(seqs) + ['absent'])
        L = len(seqs.get(name, 'x' * 1000))
        pick = lambda: str(rnd.choice([rnd.randint(-L - 10, L + 10), 0, 1, L, L + 1, -1]))
        a, b = pick(), pick()
        if rnd.random() < 0.05:
            b = '12x'
        _, exc, so = call(lambda: rt.coords2fasta(fa, name, a, b, tr))
        cases.append({'seqid': name, 'start': a, 'stop': b, 'truncate_names': tr, 'exc': exc,
                      'stdout_sha256': sha(so), 'stdout_head': so[:200]})
    return cases


def make_locus(ref):
    """genome_tools.extract_upstream_downstream (:457-480) and coords2fasta
    (:656-661) of the reference, stdout captured (the shapes SURVEY 8(f)4)."""
    sys.path.insert(0, PY3)
    import genome_tools as rt
    import tempfile
    out = {}
    with tempfile.TemporaryDirectory() as td:
        gff_path = os.path.join(td, 'loci.gff')
        with open(gff_path, 'w') as fh:
            fh.write(LOCUS_GFF)
        fa_path = os.path.join(td, 'loci.fa')
        with open(fa_path, 'w') as fh:
            fh.write(LOCUS_GENOME)
        ob_fa = goldlib.path('O.biroi_refseqGenomeSubset.fasta')
        ob_gff = goldlib.path('O.biroi_NCBIrefseq_gff3Subset.gff')
        runs = []
        for stream in ('up', 'down'):
            for n in ('3', '6', '12'):
                for ft in ('gene', 'mRNA'):
                    for nf in ('ID', 'Name'):
                        runs.append(('small', fa_path, gff_path, n, stream, ft, nf, 'True'))
            for n in ('50', '300'):
                for ft in ('gene', 'CDS'):
                    runs.append(('obiroi', ob_fa, ob_gff, n, stream, ft, 'ID', 'True'))
        runs.append(('obiroi-untruncated', ob_fa, ob_gff, '50', 'up', 'gene', 'ID', 'False'))
        for tag, fa, gff, n, stream, ft, nf, tr in runs:
            key = 'updown/%s/%s/%s/%s/%s/%s' % (tag, stream, n, ft, nf, tr)
            res, exc, so = call(lambda: rt.extract_upstream_downstream(fa, gff, n, stream, ft, nf, tr))
            d = digest(None, exc, so)
            if len(so) < 400:
                d['stdout'] = so
            out[key] = d
        for seqid, a, b, tr in [('c1', '1', '10'), ('c1', '0', '5'), ('c1', '40', '99'),
                                ('c2', '5', '3'), ('c1 first contig', '2', '4'), ('c1', '2', '4'),
                                ('zz', '1', '2')] and [(x[0], x[1], x[2], t) for x in
                                                       [('c1', '1', '10'), ('c1', '0', '5'),
                                                        ('c1', '40', '99'), ('c2', '5', '3'),
                                                        ('c1 first contig', '2', '4'),
                                                        ('c1', '2', '4'), ('zz', '1', '2')]
                                                       for t in ('False', 'True')]:
            key = 'coords/%s/%s/%s/%s' % (seqid, a, b, tr)
            res, exc, so = call(lambda: rt.coords2fasta(fa_path, seqid, a, b, tr))
            d = digest(None, exc, so)
            d['stdout'] = so
            out[key] = d
    out['_inputs'] = {'genome': LOCUS_GENOME, 'gff': LOCUS_GFF}
    return out


ORFS_GENOME = ('>c1 first contig\nATGAAATAGCCCATGGGTAAATGccctgaNNNNatgRYKMtaaGGGTTTAAACCC\n'
               'ATGATGATGTAGTAGTGA\n>c2\nnnnnATGCCCGGGTTTAAATGA\n>z9\nACGTACGTACGTAAATAG\n'
               '>a0\nTTATTATTACATCATCAT\n>mm\nMMMMATGCCC\n')


def _match_genome():
    """Three contigs (one header with a description), soft-masked runs, N runs
    and IUPAC bytes; chrA is long enough for target coordinates to cross 999
    -> 1000 (vulgar2gff compares coordinate strings)."""
    rnd = random.Random(265)
    out = []
    for name, n in (('chrA', 1500), ('chrB desc text', 800), ('chrC', 300)):
        s = [rnd.choice('ACGT') for _ in range(n)]
        for _ in range(n // 120):
            a = rnd.randrange(n)
            for k in range(a, min(n, a + rnd.randrange(5, 60))):
                s[k] = s[k].lower()
        a = rnd.randrange(n - 20)
        for k in range(a, a + 7):
            s[k] = 'N'
        s[rnd.randrange(n)] = rnd.choice('RYKM')
        seq = ''.join(s)
        out.append('>' + name + '\n' + '\n'.join(seq[i:i + 70] for i in range(0, n, 70)) + '\n')
    return ''.join(out)


BLAST_CSV = '\n'.join([
    'q1,chrA,98.0,100,2,0,1,100,101,200,1e-40,180',
    'q2,chrA,97.5,80,2,0,1,80,400,321,1e-30,150',       # subject runs backwards: '-'
    'q1,chrC,90.0,50,5,0,1,50,10,59,1e-10,60',          # repeated query: q1-1
    'q1,chrA,90.0,50,5,0,1,50,1200,1151,1e-10,61',      # q1-2, '-'
    'q3,chrA,99.0,30,0,0,1,30,995,1024,1e-12,55',
    'q4,chrA,99.0,1,0,0,1,1,700,700,1,2',               # start == end: '-'
    'q5,chrB desc text,95.0,60,3,0,1,60,30,89,1e-20,100',
    'q6,chrC,95.0,60,3,0,1,60,270,330,1e-20,100',       # runs past the contig end
    'short,row,only',                                   # <= 8 fields: skipped
    'q7,chrA,91.0,40,4,0,1,40,1,40,1e-8,70',
]) + '\n'

BLAST_TRUNC = 'q8,chrB,95.0,60,3,0,1,60,100,159,1e-20,100\nq9,chrA,95.0,20,3,0,1,20,5,24,1,9\n'

EXONERATE = """Command line: [exonerate --model protein2genome p.fa g.fa]
Hostname: [box]

C4 Alignment:
------------
         Query: prot1 first protein
        Target: chrA
         Model: protein2genome:local
   Raw score: 240
vulgar: prot1 0 60 . chrA 100 330 + 240 M 30 90 5 0 2 I 0 40 3 0 2 M 20 60 F 0 1 M 10 30 G 0 3
C4 Alignment:
------------
         Query: prot2
        Target: chrA:[revcomp]
vulgar: prot2 0 40 . chrA 1050 900 - 150 M 20 60 5 0 2 I 0 20 3 0 2 S 1 2 M 19 57 N 0 3 G 2 0
C4 Alignment:
------------
         Query: prot2
        Target: chrA:[revcomp]
vulgar: prot2 5 30 . chrA 1300 1220 - 90 M 25 75 3 0 2
C4 Alignment:
------------
         Query: prot3 crossing
        Target: chrA 
vulgar: prot3 0 12 . chrA 980 1016 + 60 M 5 15 I 0 6 M 5 15
C4 Alignment:
------------
         Query: prot4
        Target: chrB desc text [revcomp]
vulgar: prot4 0 20 . chrB 300 240 - 50 M 20 60
-- completed exonerate analysis
"""


def make_matches(ref):
    """genome_tools blast_csv2fasta (:265-271), exonerate2fasta (:274-280) and
    get_seq_from_fasta (:483-485) of the reference, stdout captured; plus
    the library readers (read_blast_csv with find_truncated_locname, the
    Genome constructor's blast_csv / exonerate_output formats) and the
    Python-2 record order (the match dict after zero copies)."""
    sys.path.insert(0, PY3)
    import genome_tools as rt
    import tempfile
    fa_text = _match_genome()
    out = {'_inputs': {'genome': fa_text, 'blast_csv': BLAST_CSV, 'blast_trunc': BLAST_TRUNC,
                       'exonerate': EXONERATE}}
    with tempfile.TemporaryDirectory() as td:
        paths = {}
        for k, text in (('fa', fa_text), ('csv', BLAST_CSV), ('trunc', BLAST_TRUNC),
                        ('ex', EXONERATE), ('csv_bad', 'q1,chrA,1,1,1,1,1,1,x,20,1,1\n'),
                        ('csv_missing', 'q1,chrZ,1,1,1,1,1,1,10,20,1,1\n'),
                        ('csv_empty', 'no,rows\n'),
                        # a query named like a generated ID: KeyError in the reference
                        ('csv_clash', BLAST_CSV + 'q1-1,chrA,88.0,20,2,0,1,20,50,69,1e-3,30\n')):
            paths[k] = os.path.join(td, k)
            with open(paths[k], 'w') as fh:
                fh.write(text)
        for tag, fn, args in (
                ('blast', rt.blast_csv2fasta, (paths['fa'], paths['csv'])),
                ('blast_trunc_tool', rt.blast_csv2fasta, (paths['fa'], paths['trunc'])),
                ('blast_bad_int', rt.blast_csv2fasta, (paths['fa'], paths['csv_bad'])),
                ('blast_missing_seqid', rt.blast_csv2fasta, (paths['fa'], paths['csv_missing'])),
                ('blast_no_rows', rt.blast_csv2fasta, (paths['fa'], paths['csv_empty'])),
                ('blast_clash', rt.blast_csv2fasta, (paths['fa'], paths['csv_clash'])),
                ('exonerate', rt.exonerate2fasta, (paths['fa'], paths['ex'])),
                ('seq/chrA', rt.get_seq_from_fasta, (paths['fa'], 'chrA')),
                ('seq/chrB desc text', rt.get_seq_from_fasta, (paths['fa'], 'chrB desc text')),
                ('seq/chrB truncated', rt.get_seq_from_fasta, (paths['fa'], 'chrB', 'True')),
                ('seq/missing', rt.get_seq_from_fasta, (paths['fa'], 'chrQ'))):
            res, exc, so = call(lambda: fn(*args))
            out['tool/' + tag] = {'exc': exc, 'stdout': so}

        def lib(build):
            def run():
                g = build()
                d = g.annotations.match
                keys = list(d)
                res = {}
                for order, ks in (('insertion', keys), ('py2', mo.py2_dict_order(keys))):
                    res[order] = '\n'.join(d[k].get_fasta() for k in ks)
                prot = []
                for k in keys:  # per record: a record shorter than a codon raises
                    r, e, _ = call(lambda: d[k].get_fasta(seq_type='protein'))
                    prot.append({'exc': e} if e else r)
                res['protein'] = prot
                res['ids'] = sorted(g.annotations.match_part)
                return res
            return run

        def g_trunc():
            g = ref.Genome(paths['fa'])
            g.read_blast_csv(paths['trunc'], find_truncated_locname=True)
            return g

        for tag, build in (
                ('blast_ctor', lambda: ref.Genome(paths['fa'], paths['csv'],
                                                  annotation_format='blast_csv')),
                ('exonerate_ctor', lambda: ref.Genome(paths['fa'], paths['ex'],
                                                      annotation_format='exonerate_output')),
                ('blast_truncated_locname', g_trunc)):
            res, exc, so = call(lib(build))
            out['lib/' + tag] = {'exc': exc, 'stdout': so, 'result': res}
    return out


def _blast_case(rnd):
    """Random BLAST -outfmt 10 rows over _match_genome's contigs: repeated
    queries (renamed q-1, q-2 ..), subjects running backwards or of one base,
    coordinates at and past the contig ends, a truncated subject name, short
    rows, CRLF lines; rarely a missing subject or a bad integer (the
    reference raises)."""
    subjects = ['chrA', 'chrA', 'chrB desc text', 'chrC']
    lens = {'chrA': 1500, 'chrB desc text': 800, 'chrC': 300}
    rows = []
    for _ in range(rnd.randrange(0, 9)):
        r = rnd.random()
        if r < 0.08:
            rows.append('short,row,only')
            continue
        q = 'q%d' % rnd.randrange(4)
        s = rnd.choice(subjects)
        a = rnd.randrange(1, lens[s] + 40)
        b = a + rnd.choice([0, rnd.randrange(1, 120), -rnd.randrange(1, 120)])
        b = max(b, 1)
        if r > 0.97:
            s = 'chrZ'
        st, en = str(a), str(b)
        if 0.95 < r <= 0.97:
            en = 'x' + en
        rows.append('%s,%s,95.0,60,3,0,1,60,%s,%s,1e-20,100' % (q, s, st, en))
    eol = '\r\n' if rnd.random() < 0.2 else '\n'
    return eol.join(rows) + (eol if rows and rnd.random() < 0.8 else '')


def make_blast_fuzz(ref, n=100):
    """genome_tools.blast_csv2fasta (:265-271) of the reference on random
    BLAST tables over _match_genome(): stdout and exception
    (tests/test_matches.py)."""
    sys.path.insert(0, PY3)
    import genome_tools as rt
    import tempfile
    rnd = random.Random(20261021)
    fa_text = _match_genome()
    cases = []
    with tempfile.TemporaryDirectory() as td:
        fa = os.path.join(td, 'g.fa')
        with open(fa, 'w') as fh:
            fh.write(fa_text)
        for i in range(n):
            csv = _blast_case(rnd)
            path = os.path.join(td, 'b%d.csv' % i)
            with open(path, 'w', newline='') as fh:
                fh.write(csv)
            _, exc, so = call(lambda: rt.blast_csv2fasta(fa, path))
            cases.append({'csv': csv, 'exc': exc, 'stdout': so})
    return {'genome': fa_text, 'cases': cases}


def _fuzz_case(rnd):
    """A small random genome + GFF3 or GTF that walks many of read_gff's and
    get_fasta's branches: renamed duplicate IDs, reversed / zero / past-end
    coordinates, '.', '-' and mixed strands, duplicate coordinates, UTR and
    exon children, comment and short lines, shared parents."""
    alpha = 'ACGTACGTACGTacgtNRY'
    contigs = []
    for i in range(rnd.randrange(1, 4)):
        n = rnd.randrange(30, 260)
        contigs.append(('s%d' % i if rnd.random() < 0.8 else 's%d desc' % i,
                        ''.join(rnd.choice(alpha) for _ in range(n))))
    fasta = ''.join('>%s\n%s\n' % (nm, sq) for nm, sq in contigs)
    seqids = [nm for nm, _ in contigs]
    lens = {nm: len(sq) for nm, sq in contigs}

    def coords(sid):
        a = rnd.randrange(0, lens[sid] + 3)
        b = a + rnd.randrange(0, 60)
        if rnd.random() < 0.15:
            a, b = b, a
        return a, b

    lines = []
    gtf = rnd.random() < 0.3
    if gtf:
        for g in range(rnd.randrange(1, 6)):
            sid = rnd.choice(seqids)
            st = rnd.choice('++--.')
            for t in range(rnd.randrange(1, 3)):
                for _ in range(rnd.randrange(1, 5)):
                    a, b = coords(sid)
                    lines.append('%s\tsrc\tCDS\t%d\t%d\t.\t%s\t0\ttranscript_id "g%d.t%d"; '
                                 'gene_id "g%d";\n' % (sid, a, b, st, g, t, g))
    else:
        cds_ids = ['c%d' % k for k in range(4)]
        for g in range(rnd.randrange(1, 6)):
            sid = rnd.choice(seqids)
            st = rnd.choice('++--.')
            lines.append('%s\tsrc\tgene\t1\t%d\t.\t%s\t.\tID=g%d\n' % (sid, lens[sid], st, g))
            for t in range(rnd.randrange(1, 3)):
                tid = 'g%d.t%d' % (g, t)
                lines.append('%s\tsrc\tmRNA\t1\t%d\t.\t%s\t.\tID=%s;Parent=g%d\n'
                             % (sid, lens[sid], st, tid, g))
                kids = []
                for _ in range(rnd.randrange(1, 5)):
                    a, b = coords(sid)
                    if kids and rnd.random() < 0.1:
                        a, b = kids[-1]
                    kids.append((a, b))
                    cst = st if rnd.random() < 0.85 else rnd.choice('+-')
                    cid = rnd.choice(cds_ids) if rnd.random() < 0.5 else 'cds%d' % len(lines)
                    lines.append('%s\tsrc\tCDS\t%d\t%d\t.\t%s\t%d\tID=%s;Parent=%s\n'
                                 % (sid, a, b, cst, rnd.randrange(3), cid, tid))
                if rnd.random() < 0.15:
                    lines.append('%s\tsrc\texon\t1\t9\t.\t%s\t.\tID=e%d;Parent=%s\n'
                                 % (sid, st, len(lines), tid))
                if rnd.random() < 0.08:
                    lines.append('%s\tsrc\tfive_prime_UTR\t1\t4\t.\t%s\t.\tID=u%d;Parent=%s\n'
                                 % (sid, st, len(lines), tid))
        if rnd.random() < 0.3:
            lines.insert(rnd.randrange(len(lines) + 1), '# a comment\tline\n')
        if rnd.random() < 0.2:
            lines.insert(rnd.randrange(len(lines) + 1), 'short\tline\n')
    return fasta, ''.join(lines)


FUZZ_CALLS = [('nucleotide', False, 'insertion'), ('protein', False, 'insertion'),
              ('nucleotide', True, 'insertion'), ('nucleotide', False, 'py2'),
              ('protein', False, 'py2')]


def make_fuzz(ref, n=60, seed=20261016):
    """Random small annotation sets through the reference's gff2fasta path
    (Genome + read_gff + get_fasta, tests/test_fuzz.py).  fuzz3.json: 200 more
    from seed 20261017."""
    rnd = random.Random(seed)
    out = []
    for i in range(n):
        fasta, gff = _fuzz_case(rnd)
        rec = {'fasta': fasta, 'gff': gff, 'calls': {}}
        for seq_type, longest, order in FUZZ_CALLS:
            res, exc, so = ref_gff2fasta(ref, fasta, gff, seq_type, longest=longest, order=order)
            d = {'exc': exc, 'stdout': so}
            if res is not None:
                d['sha256'] = sha(res)
                if len(res) < 600:
                    d['text'] = res
            rec['calls']['%s/%d/%s' % (seq_type, int(longest), order)] = d
        out.append(rec)
    return out


def _fuzz_case2(rnd):
    """As _fuzz_case, with exon children beside the CDS (random coordinates,
    strands and IDs) so that from_exons=True has exon structures to read."""
    fasta, gff = _fuzz_case(rnd)
    seqs = {}
    for block in fasta.split('>')[1:]:
        name, sq = block.split('\n', 1)
        seqs[name] = len(sq.replace('\n', ''))
    lines = []
    for line in gff.splitlines(True):
        lines.append(line)
        f = line.split('\t')
        if len(f) == 9 and f[2] == 'CDS' and rnd.random() < 0.7:
            n = seqs.get(f[0], 100)
            for _ in range(rnd.randrange(1, 3)):
                a = rnd.randrange(0, n + 3)
                b = a + rnd.randrange(0, 80)
                if rnd.random() < 0.1:
                    a, b = b, a
                st = f[6] if rnd.random() < 0.9 else rnd.choice('+-')
                if 'Parent=' in f[8]:
                    par = f[8].split('Parent=')[1].split(';')[0].strip()
                    attr = 'ID=%s;Parent=%s\n' % (rnd.choice(['ex%d' % len(lines), 'e1', 'e2']), par)
                else:
                    attr = f[8]
                lines.append('\t'.join(f[:2] + ['exon', str(a), str(b), '.', st, '.', attr]))
    return fasta, ''.join(lines)


FUZZ2_CALLS = [('nucleotide', False, True, False, 'insertion'), ('protein', False, True, False, 'insertion'),
               ('protein', True, False, False, 'insertion'), ('nucleotide', False, False, True, 'insertion'),
               ('protein', False, False, True, 'insertion'), ('nucleotide', False, False, True, 'py2'),
               ('nucleotide', True, False, True, 'insertion')]


def make_fuzz2(ref, n=40, seed=20261017):
    """The gff2fasta options fuzz.json leaves out -- genomic=True, longest
    protein, from_exons=True (exon features read as CDS) -- on random cases
    with exon children (tests/test_fuzz.py).  fuzz4.json: 120 more from seed
    20261020."""
    rnd = random.Random(seed)
    out = []
    for i in range(n):
        fasta, gff = _fuzz_case2(rnd)
        rec = {'fasta': fasta, 'gff': gff, 'calls': {}}
        for seq_type, longest, genomic, from_exons, order in FUZZ2_CALLS:
            res, exc, so = ref_gff2fasta(ref, fasta, gff, seq_type, longest=longest, genomic=genomic,
                                         order=order, from_exons=from_exons)
            d = {'exc': exc, 'stdout': so}
            if res is not None:
                d['sha256'] = sha(res)
            rec['calls']['%s/%d/%d/%d/%s' % (seq_type, int(longest), int(genomic), int(from_exons),
                                             order)] = d
        out.append(rec)
    return out


def _cds_case(rnd):
    """Random CDS FASTA text for cds2pep: headers with spaces, records of 0 to
    90 bases (upper / lower case, N, IUPAC, '*'), sequence before the first
    header, CRLF lines, no final newline, and (rarely) a blank line, which the
    reference's line[0] turns into an IndexError.  ASCII only, no lone CR:
    the reference is run as its Python 3 copy, whose text-mode open() would
    split a lone CR where Python 2 does not."""
    alpha = 'ACGTACGTACGTacgtNRYn*'
    eol = '\r\n' if rnd.random() < 0.25 else '\n'
    lines = []
    if rnd.random() < 0.15:
        lines.append(''.join(rnd.choice(alpha) for _ in range(rnd.randrange(1, 20))))
    for r in range(rnd.randrange(1, 6)):
        lines.append('>rec%d%s' % (r, ' some description' if rnd.random() < 0.4 else ''))
        n = rnd.choice([0, 1, 2, 3, 4, 5, rnd.randrange(6, 91)])
        seq = ''.join(rnd.choice(alpha) for _ in range(n))
        w = rnd.randrange(5, 40)
        for k in range(0, len(seq), w):
            lines.append(seq[k:k + w])
    if rnd.random() < 0.06:
        lines.insert(rnd.randrange(1, len(lines) + 1), '')
    text = eol.join(lines)
    if rnd.random() < 0.8:
        text += eol
    return text


def make_cds2pep(ref_tools, n=40, seed=20261018):
    """genome_tools.cds2pep (:664-675) on random FASTA files: its stdout and
    exception (tests/test_cds2pep.py).  cds2pep2.json: 160 more from seed
    20261019."""
    import tempfile
    rnd = random.Random(seed)
    out = []
    with tempfile.TemporaryDirectory() as d:
        for i in range(n):
            text = _cds_case(rnd)
            path = os.path.join(d, 'c%d.fa' % i)
            with open(path, 'wb') as fh:
                fh.write(text.encode('ascii'))
            res, exc, so = call(lambda: ref_tools.cds2pep(path))
            out.append({'fasta': text, 'exc': exc, 'stdout': so})
    return out


def main():
    ref = reference_module()
    with open(os.path.join(HERE, 'translate_lib.json'), 'w') as fh:
        json.dump(make_translate_lib(ref), fh, indent=0, sort_keys=True)
    if '--only-translate-lib' in sys.argv:
        return
    if '--only-synth' in sys.argv:
        with open(os.path.join(HERE, 'synth_small.json'), 'w') as fh:
            json.dump(make_synth(ref), fh, indent=1, sort_keys=True)
        return
    if '--only-coords-fuzz' in sys.argv:
        with open(os.path.join(HERE, 'coords_fuzz.json'), 'w') as fh:
            json.dump(make_coords_fuzz(ref), fh, indent=0, sort_keys=True)
        return
    if '--only-blast-fuzz' in sys.argv:
        with open(os.path.join(HERE, 'blast_fuzz.json'), 'w') as fh:
            json.dump(make_blast_fuzz(ref), fh, indent=0, sort_keys=True)
        return
    if '--only-cds2pep2' in sys.argv:
        sys.path.insert(0, PY3)
        import genome_tools as ref_tools
        with open(os.path.join(HERE, 'cds2pep2.json'), 'w') as fh:
            json.dump(make_cds2pep(ref_tools, n=160, seed=20261019), fh, indent=0, sort_keys=True)
        return
    if '--only-fuzz3' in sys.argv:
        with open(os.path.join(HERE, 'fuzz3.json'), 'w') as fh:
            json.dump(make_fuzz(ref, n=200, seed=20261017), fh, indent=0, sort_keys=True)
        with open(os.path.join(HERE, 'fuzz4.json'), 'w') as fh:
            json.dump(make_fuzz2(ref, n=120, seed=20261020), fh, indent=0, sort_keys=True)
        return
    if '--only-flank-edges' in sys.argv:
        with open(os.path.join(HERE, 'flank_edges.json'), 'w') as fh:
            json.dump(make_flank_edges(ref), fh, indent=1, sort_keys=True)
        with open(os.path.join(HERE, 'flank_fuzz.json'), 'w') as fh:
            json.dump(make_flank_fuzz(ref), fh, indent=0, sort_keys=True)
        return
    with open(os.path.join(HERE, 'fuzz.json'), 'w') as fh:
        json.dump(make_fuzz(ref), fh, indent=0, sort_keys=True)
    with open(os.path.join(HERE, 'fuzz2.json'), 'w') as fh:
        json.dump(make_fuzz2(ref), fh, indent=0, sort_keys=True)
    with open(os.path.join(HERE, 'fuzz3.json'), 'w') as fh:
        json.dump(make_fuzz(ref, n=200, seed=20261017), fh, indent=0, sort_keys=True)
    with open(os.path.join(HERE, 'fuzz4.json'), 'w') as fh:
        json.dump(make_fuzz2(ref, n=120, seed=20261020), fh, indent=0, sort_keys=True)
    import genome_tools as ref_tools  # the reference's, from the same Python 3 copy
    with open(os.path.join(HERE, 'cds2pep.json'), 'w') as fh:
        json.dump(make_cds2pep(ref_tools), fh, indent=0, sort_keys=True)
    with open(os.path.join(HERE, 'cds2pep2.json'), 'w') as fh:
        json.dump(make_cds2pep(ref_tools, n=160, seed=20261019), fh, indent=0, sort_keys=True)
    with open(os.path.join(HERE, 'matches.json'), 'w') as fh:
        json.dump(make_matches(ref), fh, indent=1, sort_keys=True)
    with open(os.path.join(HERE, 'blast_fuzz.json'), 'w') as fh:
        json.dump(make_blast_fuzz(ref), fh, indent=0, sort_keys=True)
    with open(os.path.join(HERE, 'loci.json'), 'w') as fh:
        json.dump(make_locus(ref), fh, indent=1, sort_keys=True)
    with open(os.path.join(HERE, 'flank_edges.json'), 'w') as fh:
        json.dump(make_flank_edges(ref), fh, indent=1, sort_keys=True)
    with open(os.path.join(HERE, 'flank_fuzz.json'), 'w') as fh:
        json.dump(make_flank_fuzz(ref), fh, indent=0, sort_keys=True)
    with open(os.path.join(HERE, 'coords_fuzz.json'), 'w') as fh:
        json.dump(make_coords_fuzz(ref), fh, indent=0, sort_keys=True)
    with open(os.path.join(HERE, 'kat.json'), 'w') as fh:
        json.dump(make_kat(ref), fh, indent=0, sort_keys=True)
    with open(os.path.join(HERE, 'edge_cases.json'), 'w') as fh:
        json.dump(make_edges(ref), fh, indent=0, sort_keys=True)
    with open(os.path.join(HERE, 'fixtures.json'), 'w') as fh:
        json.dump(make_fixture_hashes(ref), fh, indent=1, sort_keys=True)
    with open(os.path.join(HERE, 'synth_small.json'), 'w') as fh:
        json.dump(make_synth(ref), fh, indent=1, sort_keys=True)
    print('golden vectors written to', HERE)


if __name__ == '__main__':
    main()
