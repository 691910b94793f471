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


def main():
    import make_golden
    ref = make_golden.reference_module()
    rows = []
    for name, gb, ntx in (('synthetic 2 Mb / 1k tx', 2_000_000, 1000),
                          ('synthetic 10 Mb / 5k tx', 10_000_000, 5000)):
        w = synth.make('small', genome_bases=gb, n_tx=ntx)
        fa, gff = w.fasta_text(), w.gff3_text()
        bases = int(w.cds_bases)
        # reference: Genome + read_gff, then get_fasta per mRNA
        g = ref.Genome(fa)
        with contextlib.redirect_stdout(io.StringIO()):
            g.read_gff(gff)
        mrnas = list(g.annotations.mRNA.values())
        t0 = time.perf_counter()
        with contextlib.redirect_stdout(io.StringIO()):
            for m in mrnas:
                m.get_fasta('nucleotide')
            for m in mrnas:
                m.get_fasta('protein')
        t_ref = time.perf_counter() - t0
        # port: same objects through the oracle restatement
        aset = mo.load(fa, gff)
        recs = list(aset.mRNA.values())
        t0 = time.perf_counter()
        with contextlib.redirect_stdout(io.StringIO()):
            for r in recs:
                mo.get_fasta(r, aset, 'nucleotide')
            for r in recs:
                mo.get_fasta(r, aset, 'protein')
        t_port = time.perf_counter() - t0
        rows.append({'workload': name, 'cds_bases': bases, 'transcripts': len(mrnas),
                     'reference_s': t_ref, 'port_s': t_port,
                     'reference_bases_per_s': bases / t_ref, 'port_bases_per_s': bases / t_port,
                     'port_over_reference': t_ref / t_port})
        print(json.dumps(rows[-1]), flush=True)
    out = {'note': 'single-threaded, build container CPU; extraction only (get_fasta nucleotide '
                   '+ protein over all mRNA); reference = lib2to3 copy of genome.py',
           'rows': rows,
           'port_over_reference_mean': sum(r['port_over_reference'] for r in rows) / len(rows)}
    with open(os.path.join(ROOT, 'profiles', 'cpu_calibration.json'), 'w') as fh:
        json.dump(out, fh, indent=1)
    print('port/reference speed ratio: %.1f' % out['port_over_reference_mean'])


if __name__ == '__main__':
    main()
