"""CPU-baseline calibration (build container only; never run on the GPU box).

bench.py's cpu_baseline times the pure-Python restatement of the reference
loop (oracle/magot_oracle.py, kind "port") because the reference itself
cannot travel to the GPU box.  This script times the REFERENCE (the
mechanical lib2to3 copy made by tests/golden/make_golden.py in /tmp) and the
port on the same seeded synthetic annotation, single-threaded, so a port
rate can be read in reference-equivalent terms.  Both sides time only the
extraction (get_fasta nucleotide + protein over every mRNA), not parsing.

Writes profiles/cpu_calibration.json.
"""
import contextlib
import io
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests', 'golden'))

from magot_amd import synth  # noqa: E402
from oracle import magot_oracle as mo  # noqa: E402


def _time_loop(fn, min_s=2.0):
    """Seconds per call of fn(), repeated until min_s has passed."""
    n, t0 = 0, time.perf_counter()
    while True:
        fn()
        n += 1
        el = time.perf_counter() - t0
        if el >= min_s:
            return el / n, n


def calibrate(ref, name, fa, gff):
    """One row: the reference's and the port's AnnotationSet.get_fasta('gene')
    (genome.py:578-582, the gff2fasta loop: every gene's records gathered,
    nucleotide then protein) on the same FASTA + annotation text, parsed
    beforehand (parsing is not timed)."""
    g = ref.Genome(fa)
    with contextlib.redirect_stdout(io.StringIO()):
        g.read_gff(gff)
    aset = mo.load(fa, gff)
    with contextlib.redirect_stdout(io.StringIO()):
        text = aset.get_fasta('gene', seq_type='nucleotide')
    lines = text.split('\n')
    bases = sum(len(x) for x in lines if not x.startswith('>'))
    records = sum(1 for x in lines if x.startswith('>'))

    def run_ref():
        with contextlib.redirect_stdout(io.StringIO()):
            g.annotations.get_fasta('gene', seq_type='nucleotide')
            g.annotations.get_fasta('gene', seq_type='protein')

    def run_port():
        with contextlib.redirect_stdout(io.StringIO()):
            aset.get_fasta('gene', seq_type='nucleotide')
            aset.get_fasta('gene', seq_type='protein')

    t_ref, n_ref = _time_loop(run_ref)
    t_port, n_port = _time_loop(run_port)
    row = {'workload': name, 'cds_bases': bases, 'records': records,
           'reference_s': t_ref, 'port_s': t_port, 'repeats': [n_ref, n_port],
           'reference_bases_per_s': bases / t_ref, 'port_bases_per_s': bases / t_port,
           'port_over_reference': t_ref / t_port}
    print(json.dumps(row), flush=True)
    return row


def main():
    import goldlib
    import make_golden
    ref = make_golden.reference_module()
    rows = []
    # C1: the reference's own O.biroi subset (BASELINE configs[0])
    with open(goldlib.path('O.biroi_refseqGenomeSubset.fasta')) as fh:
        fa = fh.read()
    with open(goldlib.path('O.biroi_NCBIrefseq_gff3Subset.gff')) as fh:
        gff = fh.read()
    rows.append(calibrate(ref, 'C1: O.biroi refseq subset (FASTA + GFF3)', fa, gff))
    # the reference's Chromosome14 test data, rebuilt from its CDS fixture
    # (tests/golden/goldlib.rebuild_c14), with its standard GTF
    with open(goldlib.path('StandardGTF.gtf')) as fh:
        gtf = fh.read()
    rows.append(calibrate(ref, 'C14: Chromosome14 (rebuilt) + StandardGTF.gtf',
                          goldlib.rebuild_c14(), gtf))
    for name, gb, ntx in (('synthetic 2 Mb / 1k tx', 2_000_000, 1000),
                          ('synthetic 10 Mb / 5k tx', 10_000_000, 5000)):
        w = synth.make('small', genome_bases=gb, n_tx=ntx)
        rows.append(calibrate(ref, name, w.fasta_text(), w.gff3_text()))
    ratios = [r['port_over_reference'] for r in rows]
    out = {'note': 'single-threaded, build container CPU; extraction only (AnnotationSet.get_fasta'
                   '(gene) nucleotide + protein, each loop repeated for >= 2 s); reference = '
                   'lib2to3 copy of genome.py (scripts/calibrate_cpu.py)',
           'rows': rows,
           'port_over_reference_mean': sum(ratios) / len(ratios),
           'port_over_reference_min': min(ratios),
           'port_over_reference_max': max(ratios)}
    with open(os.path.join(ROOT, 'profiles', 'cpu_calibration.json'), 'w') as fh:
        json.dump(out, fh, indent=1)
    print('port/reference speed ratio: %.1f (%.1f - %.1f)'
          % (out['port_over_reference_mean'], min(ratios), max(ratios)))


if __name__ == '__main__':
    main()
