"""Times gff2fasta's longest=True (nucleotide and protein) and genomic=True variants,
cds2pep over the nucleotide output, and extract_upstream_downstream (1 kb up /
down of every gene), on the native path against the line loops,
over the files of an e2e_cli.py run (C3 by default), each in this process
after one warm call of the default variant (device start-up excluded).
Correctness of these variants is pinned by tests/test_gffplan.py (oracle) and
tests/test_fuzz.py (reference outputs); here only time and size are reported.

    python scripts/e2e_variants.py [--dir /tmp/magot_e2e]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from magot_amd import genome_tools  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--dir', default='/tmp/magot_e2e')
    a = ap.parse_args()
    fa, gf = os.path.join(a.dir, 'genome.fa'), os.path.join(a.dir, 'ann.gff3')
    genome_tools._gff2fasta_native(fa, gf, 'nucleotide', 'py2')[0]  # warm: device start-up
    rec = {}
    for name, st, kw in (('default_nucleotide', 'nucleotide', {}),
                         ('longest_nucleotide', 'nucleotide', {'longest': True}),
                         ('longest_protein', 'protein', {'longest': True}),
                         ('genomic', 'nucleotide', {'genomic': True})):
        t = time.perf_counter()
        text = genome_tools._gff2fasta_native(fa, gf, st, 'py2', **kw)[0]
        rec[name] = {'s': time.perf_counter() - t, 'native': text is not None,
                     'bytes': None if text is None else int(len(text)) + 1}
        if name == 'default_nucleotide':  # the CDS FASTA cds2pep reads below
            with open(os.path.join(a.dir, 'cds.fa'), 'wb') as fh:
                fh.write(bytes(text))
                fh.write(b'\n')
    # cds2pep (genome_tools.py:664-675) on that CDS FASTA (500k records)
    import io
    from contextlib import redirect_stdout
    outs = {}
    for native in ('True', 'False'):
        b = io.BytesIO()
        w = io.TextIOWrapper(b, encoding='latin-1', write_through=True)
        t = time.perf_counter()
        with redirect_stdout(w):
            genome_tools.cds2pep(os.path.join(a.dir, 'cds.fa'), native=native)
        w.flush()
        rec['cds2pep_' + ('native' if native == 'True' else 'line_loop')] = {
            's': time.perf_counter() - t, 'bytes': len(b.getvalue())}
        outs[native] = b.getvalue()
    rec['cds2pep_outputs_equal'] = outs['True'] == outs['False']
    # extract_upstream_downstream (genome_tools.py:457-480): 1 kb windows
    # before / after every gene, native (C++ scan + one extraction launch +
    # device text) against the line loop (Python scan + the same launch)
    for stream in ('up', 'down'):
        outs = {}
        for native in ('True', 'False'):
            b = io.BytesIO()
            w = io.TextIOWrapper(b, encoding='latin-1', write_through=True)
            t = time.perf_counter()
            with redirect_stdout(w):
                genome_tools.extract_upstream_downstream(fa, gf, '1000', stream, native=native)
            w.flush()
            rec['flank_%s_%s' % (stream, 'native' if native == 'True' else 'line_loop')] = {
                's': time.perf_counter() - t, 'bytes': len(b.getvalue())}
            outs[native] = b.getvalue()
        rec['flank_%s_outputs_equal' % stream] = outs['True'] == outs['False']
    print(json.dumps(rec), flush=True)


if __name__ == '__main__':
    main()
