"""Genomes above one device plane (~4 Gbases: extract_kernel's 32-bit window
offsets).  engine.device_genome packs such a genome as several planes
(PartitionedGenome) and engine.extract_records runs one plan per plane;
records whose intervals lie in two planes are gathered as pieces and joined.

CPU: the contig -> plane assignment.  GPU (marked): a lowered plane size
(engine.PART_BASES patched) forces several planes on small genomes, and the
drop-in API / CLI output must not change; the slow test packs a real
4.4-Gbase genome and checks records past the 4 Gi boundary.
"""
import contextlib
import io

import numpy as np
import pytest

from oracle import magot_oracle as mo


def test_plan_parts():
    from magot_amd import engine
    assert engine.plan_parts([5, 5, 5, 5], limit=10).tolist() == [0, 0, 1, 1]
    assert engine.plan_parts([3, 8, 2, 9, 1], limit=10).tolist() == [0, 1, 1, 2, 2]
    assert engine.plan_parts([10, 10], limit=10).tolist() == [0, 1]
    assert engine.plan_parts([], limit=10).tolist() == []
    with pytest.raises(engine.MagotError):
        engine.plan_parts([4, 11], limit=10)


def test_native_loader_declines_oversized_genome():
    """magot_genome_load / _load_fasta answer MAGOT_ERR_UNSUPPORTED (not a
    crash) above one plane; checked by the constant the C side uses."""
    from magot_amd import engine
    assert engine.PART_BASES + 64 + 256 < 0xFFFFFFF0


CROSS_GENOME = ('>c1\nATGAAACCCGGGTTTaaacccgggNNNRYTTTAAACCCGGGATG\n'
                '>c2 two\nGGGAAATTTCCCgggaaatttcccATGCATGCATGCATGC\n'
                '>c3\nTTTTAAAACCCCGGGGttttaaaaccccggggACGTACGT\n')
# one gene per contig, plus genes whose CDS lie on two contigs (planes)
CROSS_GFF = ''.join([
    'c1\tt\tgene\t1\t40\t.\t+\t.\tID=g1\n', 'c1\tt\tmRNA\t1\t40\t.\t+\t.\tID=m1;Parent=g1\n',
    'c1\tt\tCDS\t1\t12\t.\t+\t0\tID=x1;Parent=m1\n', 'c1\tt\tCDS\t20\t33\t.\t+\t0\tID=x2;Parent=m1\n',
    'c1\tt\tgene\t1\t40\t.\t-\t.\tID=g2\n', 'c1\tt\tmRNA\t1\t40\t.\t-\t.\tID=m2;Parent=g2\n',
    'c1\tt\tCDS\t5\t16\t.\t-\t0\tID=x3;Parent=m2\n',
    'c2 two\tt\tCDS\t3\t20\t.\t-\t0\tID=x4;Parent=m2\n',
    'c3\tt\tgene\t1\t40\t.\t+\t.\tID=g3\n', 'c3\tt\tmRNA\t1\t40\t.\t+\t.\tID=m3;Parent=g3\n',
    'c3\tt\tCDS\t2\t19\t.\t+\t0\tID=x5;Parent=m3\n',
    'c2 two\tt\tCDS\t25\t38\t.\t+\t0\tID=x6;Parent=m3\n',
    'c1\tt\tCDS\t30\t41\t.\t+\t0\tID=x7;Parent=m3\n',
    'c2 two\tt\tgene\t1\t40\t.\t+\t.\tID=g4\n', 'c2 two\tt\tmRNA\t1\t40\t.\t+\t.\tID=m4;Parent=g4\n',
    'c2 two\tt\tCDS\t1\t36\t.\t+\t0\tID=x8;Parent=m4\n',
])


def _api(fasta, gff, seq_type, order='insertion'):
    from magot_amd import genome as G
    g = G.Genome(fasta)
    g.read_gff(gff)
    return g.annotations.get_fasta('gene', seq_type=seq_type, order=order)


@pytest.mark.gpu
@pytest.mark.parametrize('limit', [45, 90, 10 ** 9])
@pytest.mark.parametrize('seq_type', ['nucleotide', 'protein'])
def test_cross_plane_records_vs_oracle(monkeypatch, limit, seq_type):
    """Planes of one, two or all three contigs; records with CDS on two
    planes (both strands) are joined from pieces and translated after."""
    from magot_amd import engine
    monkeypatch.setattr(engine, 'PART_BASES', limit)
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        want = mo.gff2fasta(CROSS_GENOME, CROSS_GFF, seq_type=seq_type)[:-1]
    got = _api(CROSS_GENOME, CROSS_GFF, seq_type)
    assert got == want


@pytest.mark.gpu
@pytest.mark.parametrize('seq_type', ['nucleotide', 'protein'])
def test_partitioned_synthetic_vs_unpartitioned(monkeypatch, seq_type):
    from magot_amd import engine, synth
    w = synth.make('small', seed=31, genome_bases=2_000_000, n_tx=700, iupac_rate=1e-3)
    fa, gff = w.fasta_text(), w.gff3_text()
    whole = _api(fa, gff, seq_type, order='py2')
    monkeypatch.setattr(engine, 'PART_BASES', int(w.contig_len.max()) + 1)
    from magot_amd import genome as G
    g = G.Genome(fa)
    assert isinstance(g.genome_sequence.device(), engine.PartitionedGenome)
    assert len(g.genome_sequence.device().parts) > 1
    g.read_gff(gff)
    assert g.annotations.get_fasta('gene', seq_type=seq_type, order='py2') == whole


@pytest.mark.gpu
def test_partitioned_cli_and_loci(monkeypatch, tmp_path):
    """gff2fasta declines its native path on several planes (object path),
    coords2fasta gathers through extract_records: same bytes."""
    from magot_amd import engine, genome_tools, synth
    w = synth.make('small', seed=32, genome_bases=1_000_000, n_tx=300, iupac_rate=1e-3)
    fa, gf = tmp_path / 'g.fa', tmp_path / 'g.gff'
    fa.write_text(w.fasta_text())
    gf.write_text(w.gff3_text())

    def run(fn, *a):
        b = io.BytesIO()
        out = io.TextIOWrapper(b, encoding='latin-1', write_through=True)
        with contextlib.redirect_stdout(out):
            fn(*a)
        out.flush()
        return b.getvalue()

    base = run(genome_tools.gff2fasta, str(fa), str(gf))
    loc = run(genome_tools.coords2fasta, str(fa), w.contig_names[-1], '5', '900')
    monkeypatch.setattr(engine, 'PART_BASES', int(w.contig_len.max()) + 1)
    assert run(genome_tools.gff2fasta, str(fa), str(gf)) == base
    assert run(genome_tools.coords2fasta, str(fa), w.contig_names[-1], '5', '900') == loc


@pytest.mark.gpu
@pytest.mark.slow
def test_genome_above_4_gbases():
    """A 4.4-Gbase genome (four contigs) packs as two planes; records on the
    last contig, beyond 4 Gi bases into the genome, come out right."""
    from magot_amd import engine
    rng = np.random.default_rng(44)
    n = 1_100_000_000
    acgt = np.frombuffer(b'ACGTacgt', dtype=np.uint8)
    contigs = []
    for i in range(4):
        seq = acgt[rng.integers(0, 8, size=n, dtype=np.uint8)]
        contigs.append(('big%d' % i, seq.tobytes()))
        del seq
    dev = engine.device_genome(contigs)
    assert isinstance(dev, engine.PartitionedGenome) and len(dev.parts) == 2
    spans = [(3, 5, 300, False), (3, n - 400, 400, True), (2, 123456789, 999, True),
             (0, 7, 60, False), (3, 1_000_000_000, 4096, False)]
    ex = np.zeros(len(spans), dtype=engine.EXON_DTYPE)
    for i, (c, st, ln, rc) in enumerate(spans):
        ex[i] = ((st | (1 << 63)) if rc else st, c, ln)
    tx = np.zeros(len(spans), dtype=engine.TX_DTYPE)
    tx['exon_begin'] = np.arange(len(spans))
    tx['n_exons'] = 1
    nuc, noff, pep, poff = engine.extract_records(dev, ex, tx)
    for i, (c, st, ln, rc) in enumerate(spans):
        s = contigs[c][1][st:st + ln].decode('latin-1')
        want = mo.reverse_complement(s) if rc else s
        assert nuc[int(noff[i]):int(noff[i + 1])].tobytes().decode('latin-1') == want
        p = pep[int(poff[i]):int(poff[i + 1])].tobytes().decode('latin-1')
        if p[:1] == 'X':
            p = p[1:]
        assert p == (mo.translate(want) or '')
    dev.close()
