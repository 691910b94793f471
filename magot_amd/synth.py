"""Seeded synthetic genomes + annotations of the shapes in SURVEY.md section 8(d).

A ``Workload`` holds a genome (one uint8 array, contigs as slices of it) and a
transcript set (exon intervals, 1-based inclusive as in GFF).  It can be
rendered as FASTA + GFF3/GTF text (to drive the full Python API) or turned
straight into the device plan tables the Python walker would produce (for
the benchmark, where parsing is not part of the measured path).

Genome values: i.i.d. uniform ACGT, soft-mask lowercase runs (geometric,
mean 300, ~40 % of bases), N runs (U[100, 10000], ~1 %), IUPAC RYKMSW
point exceptions.  Configs:
  C2  100 Mb, 16 equal contigs, 50k single-exon '+' CDS, len U[150,1850]
  C3  1 Gb, 64 lognormal contigs (sigma 1, min 1 Mb), 500k transcripts,
      1+Poisson(7) exons of U[50,250], introns U[60,5000], strand 50/50
  C5  3 Gb, 200 lognormal contigs, 2M transcripts, exon model of C3
Seeds: 20261015 + config index.  Draw order (round 5 on): contig lengths,
transcripts, then the genome bytes, so the record tables can be made without
the genome (``make(..., genome=False)``); rounds 1-4 drew the genome before the
transcripts, so their C2/C3/C5 record sets differ from these.
"""

import numpy as np

from ._lib import EXON_DTYPE, TX_DTYPE, RC_BIT

SEED_BASE = 20261015
_ASCII = np.frombuffer(b'ACGT', dtype=np.uint8)
_IUPAC = np.frombuffer(b'RYKMSW', dtype=np.uint8)


class Workload(object):
    def __init__(self, name, genome, contig_len, tx_contig, tx_strand, ex_count, ex_start, ex_len,
                 outputs):
        self.name = name
        self.genome = genome                    # uint8[G]
        self.contig_len = contig_len            # int64[C]
        self.contig_off = np.zeros(len(contig_len) + 1, dtype=np.int64)
        np.cumsum(contig_len, out=self.contig_off[1:])
        self.contig_names = ['ctg%d' % i for i in range(len(contig_len))]
        self.tx_contig = tx_contig              # int64[T]
        self.tx_strand = tx_strand              # int8[T]: +1 / -1
        self.ex_count = ex_count                # int64[T]
        self.ex_start = ex_start                # int64[E] 0-based, ascending within tx
        self.ex_len = ex_len                    # int64[E]
        self.outputs = outputs                  # 'nuc' | 'nuc+pep'

    # -- sizes ---------------------------------------------------------------
    @property
    def n_tx(self):
        return len(self.tx_contig)

    @property
    def n_exons(self):
        return len(self.ex_start)

    @property
    def cds_bases(self):
        return int(self.ex_len.sum())

    def contig_bytes(self, i):
        return self.genome[self.contig_off[i]:self.contig_off[i + 1]]

    def contigs(self):
        return [(self.contig_names[i], self.contig_bytes(i).tobytes())
                for i in range(len(self.contig_len))]

    def contig_views(self):
        """(name, uint8 view) per contig: the genome without a copy."""
        return [(self.contig_names[i], self.contig_bytes(i)) for i in range(len(self.contig_len))]

    # -- device plan tables (what the Python walker produces) -----------------
    def plan_tables(self, tx_subset=None):
        """(exons EXON_DTYPE, txs TX_DTYPE) in output order: '+' records
        ascending, '-' records descending with every interval reverse-
        complemented (genome.py:698-703, 607-608)."""
        first = np.zeros(self.n_tx + 1, dtype=np.int64)
        np.cumsum(self.ex_count, out=first[1:])
        tx_ids = np.arange(self.n_tx) if tx_subset is None else np.asarray(tx_subset)
        counts = self.ex_count[tx_ids]
        E = int(counts.sum())
        # index of each output exon in the ascending exon arrays
        tx_of = np.repeat(tx_ids, counts)
        k = np.arange(E) - np.repeat(np.cumsum(counts) - counts, counts)
        minus = self.tx_strand[tx_of] < 0
        src = first[tx_of] + np.where(minus, np.repeat(counts, counts) - 1 - k, k)
        ex = np.empty(E, dtype=EXON_DTYPE)
        # Python slice clamping at the contig end (genome.py:606)
        clen = self.contig_len[self.tx_contig[tx_of]]
        s0 = np.minimum(self.ex_start[src], clen)
        s1 = np.minimum(self.ex_start[src] + self.ex_len[src], clen)
        start = s0.astype(np.uint64)
        ex['start_rc'] = np.where(minus, start | RC_BIT, start)
        ex['contig'] = self.tx_contig[tx_of].astype(np.uint32)
        ex['len'] = np.maximum(s1 - s0, 0).astype(np.uint32)
        tx = np.zeros(len(tx_ids), dtype=TX_DTYPE)
        tx['exon_begin'] = np.cumsum(counts) - counts
        tx['n_exons'] = counts
        return ex, tx

    # -- text renderings -------------------------------------------------------
    def fasta_text(self, width=60):
        out = []
        for i in range(len(self.contig_len)):
            s = self.contig_bytes(i).tobytes().decode('latin-1')
            out.append('>' + self.contig_names[i] + '\n')
            for p in range(0, len(s), width):
                out.append(s[p:p + width] + '\n')
        return ''.join(out)

    def gff3_text(self, ids='synth'):
        """NCBI-like gene -> mRNA -> CDS; the CDS ID repeats within a transcript
        so read_gff's renaming path runs (genome.py:355-364).  ids='synth':
        gene<t> / rna<t> / cds<t>, whose renamed CDS IDs (cds<t>2, cds<t>-3 ..)
        collide with other transcripts' (cds52 is transcript 52's CDS and
        transcript 5's second), so read_gff's renaming cascades; ids='ncbi':
        gene-G<t> / rna-XM_<t>.1 / cds-XP_<t>.1 as NCBI's files name them,
        whose renamed IDs never meet another ID."""
        if ids == 'ncbi':
            return self._gff3_ncbi()
        lines = ['##gff-version 3\n']
        first = np.concatenate([[0], np.cumsum(self.ex_count)])
        for t in range(self.n_tx):
            c = self.contig_names[self.tx_contig[t]]
            st = '+' if self.tx_strand[t] > 0 else '-'
            a, b = first[t], first[t + 1]
            lo = int(self.ex_start[a]) + 1
            hi = int(self.ex_start[b - 1] + self.ex_len[b - 1])
            lines.append('%s\tsynth\tgene\t%d\t%d\t.\t%s\t.\tID=gene%d;Name=G%d\n'
                         % (c, lo, hi, st, t, t))
            lines.append('%s\tsynth\tmRNA\t%d\t%d\t.\t%s\t.\tID=rna%d;Parent=gene%d\n'
                         % (c, lo, hi, st, t, t))
            for e in range(a, b):
                s0 = int(self.ex_start[e]) + 1
                s1 = int(self.ex_start[e] + self.ex_len[e])
                lines.append('%s\tsynth\texon\t%d\t%d\t.\t%s\t.\tID=exon%d_%d;Parent=rna%d\n'
                             % (c, s0, s1, st, t, e - a, t))
                lines.append('%s\tsynth\tCDS\t%d\t%d\t.\t%s\t0\tID=cds%d;Parent=rna%d\n'
                             % (c, s0, s1, st, t, t))
        return ''.join(lines)

    def _gff3_ncbi(self):
        lines = ['##gff-version 3\n']
        first = np.concatenate([[0], np.cumsum(self.ex_count)])
        for t in range(self.n_tx):
            c = self.contig_names[self.tx_contig[t]]
            st = '+' if self.tx_strand[t] > 0 else '-'
            a, b = first[t], first[t + 1]
            lo = int(self.ex_start[a]) + 1
            hi = int(self.ex_start[b - 1] + self.ex_len[b - 1])
            lines.append('%s\tsynth\tgene\t%d\t%d\t.\t%s\t.\tID=gene-G%07d;Name=G%d\n'
                         % (c, lo, hi, st, t, t))
            lines.append('%s\tsynth\tmRNA\t%d\t%d\t.\t%s\t.\tID=rna-XM_%09d.1;Parent=gene-G%07d\n'
                         % (c, lo, hi, st, t, t))
            for e in range(a, b):
                s0 = int(self.ex_start[e]) + 1
                s1 = int(self.ex_start[e] + self.ex_len[e])
                lines.append('%s\tsynth\texon\t%d\t%d\t.\t%s\t.\tID=exon-XM_%09d.1-%d;'
                             'Parent=rna-XM_%09d.1\n' % (c, s0, s1, st, t, e - a + 1, t))
                lines.append('%s\tsynth\tCDS\t%d\t%d\t.\t%s\t0\tID=cds-XP_%09d.1;'
                             'Parent=rna-XM_%09d.1\n' % (c, s0, s1, st, t, t))
        return ''.join(lines)

    def gtf_text(self):
        lines = []
        first = np.concatenate([[0], np.cumsum(self.ex_count)])
        for t in range(self.n_tx):
            c = self.contig_names[self.tx_contig[t]]
            st = '+' if self.tx_strand[t] > 0 else '-'
            for e in range(first[t], first[t + 1]):
                s0 = int(self.ex_start[e]) + 1
                s1 = int(self.ex_start[e] + self.ex_len[e])
                lines.append('%s\tsynth\tCDS\t%d\t%d\t0.5\t%s\t0\ttranscript_id "g%d.t1"; '
                             'gene_id "g%d";\n' % (c, s0, s1, st, t, t))
        return ''.join(lines)


# ---------------------------------------------------------------------------
# generators
# ---------------------------------------------------------------------------

def _genome(rng, G, lower_frac=0.4, lower_mean=300.0, n_frac=0.01, iupac_rate=1e-6):
    g = _ASCII[rng.integers(0, 4, size=G, dtype=np.uint8)]
    # soft-mask runs: alternate gaps and runs with geometric lengths
    if lower_frac > 0:
        gap_mean = lower_mean * (1.0 - lower_frac) / lower_frac
        k = int(G / (lower_mean + gap_mean) * 1.2) + 16
        gaps = rng.geometric(1.0 / gap_mean, size=k)
        runs = rng.geometric(1.0 / lower_mean, size=k)
        starts = np.cumsum(gaps + runs) - runs
        ends = starts + runs
        keep = starts < G
        starts, ends = starts[keep], np.minimum(ends[keep], G)
        diff = np.zeros(G + 1, dtype=np.int8)
        np.add.at(diff, starts, 1)
        np.add.at(diff, ends, -1)
        mask = np.cumsum(diff[:G], dtype=np.int8).view(np.uint8)
        g |= (mask << 5)
    if n_frac > 0:
        n_runs = max(1, int(G * n_frac / 5050))
        pos = rng.integers(0, max(1, G - 100), size=n_runs)
        ln = rng.integers(100, 10001, size=n_runs)
        for p, l in zip(pos.tolist(), ln.tolist()):
            g[p:p + l] = ord('N')
    if iupac_rate > 0:
        n = max(1, int(G * iupac_rate))
        pos = rng.integers(0, G, size=n)
        g[pos] = _IUPAC[rng.integers(0, 6, size=n)]
    return g


def _lognormal_contigs(rng, G, n, min_len):
    w = rng.lognormal(0.0, 1.0, size=n)
    L = np.maximum(np.floor(w / w.sum() * G).astype(np.int64), min_len)
    # renormalise the excess onto the largest contigs
    excess = int(L.sum() - G)
    order = np.argsort(-L)
    i = 0
    while excess != 0:
        j = order[i % n]
        d = min(excess, int(L[j] - min_len)) if excess > 0 else excess
        L[j] -= d
        excess -= d
        i += 1
    return L


def _transcripts(rng, contig_len, n_tx, mean_extra_exons=7, ex_lo=50, ex_hi=250, in_lo=60,
                 in_hi=5000, minus_frac=0.5):
    p = contig_len / contig_len.sum()
    tx_contig = rng.choice(len(contig_len), size=n_tx, p=p)
    tx_contig.sort(kind='stable')                 # contig-ordered, as a GFF would be
    ex_count = 1 + rng.poisson(mean_extra_exons, size=n_tx)
    E = int(ex_count.sum())
    ex_len = rng.integers(ex_lo, ex_hi + 1, size=E)
    intr = rng.integers(in_lo, in_hi + 1, size=E)
    first = np.cumsum(ex_count) - ex_count
    last = first + ex_count - 1
    step = ex_len + intr
    step[last] = ex_len[last]                     # no intron after the last exon
    cs = np.cumsum(step)
    base = np.repeat(cs[first] - step[first], ex_count)
    rel = cs - step - base                        # offset of each exon in its transcript
    span = np.add.reduceat(step, first)
    room = np.maximum(contig_len[tx_contig] - span, 1)
    tx_start = (rng.random(n_tx) * room).astype(np.int64)
    ex_start = np.repeat(tx_start, ex_count) + rel
    strand = np.where(rng.random(n_tx) < minus_frac, -1, 1).astype(np.int8)
    return tx_contig.astype(np.int64), strand, ex_count.astype(np.int64), \
        ex_start.astype(np.int64), ex_len.astype(np.int64)


def _sort_by_position(w):
    """Order transcripts by (contig, start) as a coordinate-sorted GFF lists them."""
    first = np.concatenate([[0], np.cumsum(w.ex_count)])
    key = w.tx_contig * (1 << 40) + w.ex_start[first[:-1]]
    order = np.argsort(key, kind='stable')
    idx = np.concatenate([np.arange(first[t], first[t + 1]) for t in order]) if len(order) \
        else np.zeros(0, np.int64)
    w.tx_contig = w.tx_contig[order]
    w.tx_strand = w.tx_strand[order]
    w.ex_count = w.ex_count[order]
    w.ex_start = w.ex_start[idx]
    w.ex_len = w.ex_len[idx]
    return w


def make(config, seed=None, genome_bases=None, n_tx=None, iupac_rate=None, order='random',
         genome=True):
    """Build a named workload.  ``genome_bases`` / ``n_tx`` rescale it (tests).
    ``order``: 'random' (transcripts in placement order within each contig) or
    'sorted' (by start coordinate, as a coordinate-sorted GFF).
    ``genome=False``: the contig lengths and the transcript set only
    (``Workload.genome`` is None) -- the same tables a full ``make`` returns,
    since the generator draws the contigs, then the transcripts, then the
    genome bytes from one stream.  A rank of a multi-GPU job that receives the
    genome over the collective needs only these."""
    w = _make(config, seed, genome_bases, n_tx, iupac_rate, genome)
    if order == 'sorted':
        w = _sort_by_position(w)
    elif order != 'random':
        raise ValueError(order)
    return w


def _make(config, seed, genome_bases, n_tx, iupac_rate, with_genome=True):
    # draw order: contig lengths, transcripts, genome bytes (the tables never
    # depend on the genome draws, so genome=False skips them)
    idx = {'C2': 2, 'C3': 3, 'C5': 5, 'small': 9}[config]
    rng = np.random.default_rng(SEED_BASE + idx if seed is None else seed)
    if config == 'C2':
        G = genome_bases or 100_000_000
        T = n_tx or 50_000
        n_ctg = 16
        L = np.full(n_ctg, G // n_ctg, dtype=np.int64)
        L[-1] += G - L.sum()
        p = L / L.sum()
        tx_contig = np.sort(rng.choice(n_ctg, size=T, p=p))
        ex_len = rng.integers(150, 1851, size=T)
        room = L[tx_contig] - ex_len
        ex_start = (rng.random(T) * room).astype(np.int64)
        genome = _genome(rng, G, iupac_rate=1e-6 if iupac_rate is None else iupac_rate) \
            if with_genome else None
        return Workload('C2', genome, L, tx_contig.astype(np.int64), np.ones(T, np.int8),
                        np.ones(T, np.int64), ex_start, ex_len.astype(np.int64), 'nuc')
    if config in ('C3', 'C5', 'small'):
        G = genome_bases or {'C3': 1_000_000_000, 'C5': 3_000_000_000, 'small': 1_000_000}[config]
        T = n_tx or {'C3': 500_000, 'C5': 2_000_000, 'small': 500}[config]
        n_ctg = {'C3': 64, 'C5': 200, 'small': 8}[config]
        min_len = min(1_000_000, G // (2 * n_ctg))
        L = _lognormal_contigs(rng, G, n_ctg, min_len)
        tx = _transcripts(rng, L, T)
        rate = iupac_rate if iupac_rate is not None else (1e-6 if config != 'small' else 1e-3)
        genome = _genome(rng, G, iupac_rate=rate) if with_genome else None
        return Workload(config, genome, L, *tx, outputs='nuc+pep')
    raise ValueError(config)
