"""Build the host parsers/packer with AddressSanitizer + UndefinedBehaviorSanitizer
and run them over the reference's fixtures, the generated parity cases and
seeded mutations of both (sanitizers on host code).

    python tests/sanitize/run.py [--mutations N] [--log PATH]

hipcc compiles pack.cpp, gffplan.cpp and fasta.cpp host-only
(--offload-host-only, each -fsanitize after -Xarch_host) together with the
driver host_check.cpp into tests/sanitize/build/host_check (git-ignored).
No GPU is used.  Exit status: the driver's (0 = clean).
"""

import argparse
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
CSRC = os.path.join(ROOT, 'magot_amd', 'csrc')
GOLD = os.path.join(ROOT, 'tests', 'golden')
BUILD = os.path.join(HERE, 'build')
EXE = os.path.join(BUILD, 'host_check')
SOURCES = [os.path.join(CSRC, f) for f in ('pack.cpp', 'gffplan.cpp', 'fasta.cpp')] + \
    [os.path.join(HERE, 'host_check.cpp')]
FLAGS = ['-std=c++17', '-O1', '-g', '-fno-omit-frame-pointer', '--offload-arch=gfx950',
         '-x', 'hip', '--offload-host-only', '-I' + os.path.join(ROOT, 'include'),
         '-Xarch_host', '-fsanitize=address', '-Xarch_host', '-fsanitize=undefined',
         '-Xarch_host', '-fno-sanitize-recover=undefined']


def build():
    os.makedirs(BUILD, exist_ok=True)
    deps = SOURCES + [os.path.join(CSRC, 'common.h'), os.path.join(ROOT, 'include', 'magot.h')]
    if os.path.exists(EXE) and all(os.path.getmtime(EXE) > os.path.getmtime(d) for d in deps):
        return EXE
    objs = []
    for src in SOURCES:
        obj = os.path.join(BUILD, os.path.basename(src) + '.o')
        subprocess.check_call(['/opt/rocm/bin/hipcc'] + FLAGS + ['-c', src, '-o', obj])
        objs.append(obj)
    subprocess.check_call(['/opt/rocm/bin/hipcc', '-fsanitize=address,undefined', '-fno-gpu-sanitize', '-o', EXE] +
                          objs + ['-lpthread'])
    return EXE


def write_inputs(d):
    """The input list: reference fixture files, then every generated case."""
    lines = []
    fa = os.path.join(GOLD, 'O.biroi_refseqGenomeSubset.fasta')
    lines.append('fasta %s' % fa)
    lines.append('gff %s %s' % (os.path.join(GOLD, 'O.biroi_NCBIrefseq_gff3Subset.gff'), fa))
    for ann in ('StandardGTF.gtf', 'transcriptlessGTF.gtf', 'minimalGFF3.gff'):
        lines.append('gff %s %s' % (os.path.join(GOLD, ann), fa))
    lines.append('cds %s' % os.path.join(GOLD, 'CDSannotations.cds'))
    for name in ('fuzz.json', 'fuzz2.json'):
        with open(os.path.join(GOLD, name)) as fh:
            cases = json.load(fh)
        for i, c in enumerate(cases):
            f = os.path.join(d, '%s_%d.fasta' % (name[:-5], i))
            g = os.path.join(d, '%s_%d.gff' % (name[:-5], i))
            with open(f, 'w', encoding='latin-1') as fh:
                fh.write(c['fasta'])
            with open(g, 'w', encoding='latin-1') as fh:
                fh.write(c['gff'])
            lines.append('fasta %s' % f)
            lines.append('gff %s %s' % (g, f))
    # a larger synthetic genome + GFF3/GTF twin (multi-threaded chunked parse)
    sys.path.insert(0, ROOT)
    from magot_amd import synth
    w = synth.make('small', seed=17, genome_bases=3_000_000, n_tx=3000, iupac_rate=1e-3)
    f = os.path.join(d, 'synth.fasta')
    with open(f, 'w', encoding='latin-1') as fh:
        fh.write(w.fasta_text())
    lines.append('fasta %s' % f)
    for ext, text in (('gff', w.gff3_text()), ('gtf', w.gtf_text())):
        g = os.path.join(d, 'synth.' + ext)
        with open(g, 'w', encoding='latin-1') as fh:
            fh.write(text)
        lines.append('gff %s %s' % (g, f))
    with open(os.path.join(GOLD, 'cds2pep.json')) as fh:
        for i, c in enumerate(json.load(fh)):
            f = os.path.join(d, 'cds_%d.fa' % i)
            with open(f, 'w', encoding='latin-1') as fh2:
                fh2.write(c['fasta'])
            lines.append('cds %s' % f)
    path = os.path.join(d, 'inputs.txt')
    with open(path, 'w') as fh:
        fh.write('\n'.join(lines) + '\n')
    return path


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument('--mutations', type=int, default=20)
    ap.add_argument('--log', default=None)
    a = ap.parse_args(argv)
    exe = build()
    os.makedirs(os.path.join(BUILD, 'inputs'), exist_ok=True)
    lst = write_inputs(os.path.join(BUILD, 'inputs'))
    env = dict(os.environ, ASAN_OPTIONS='detect_leaks=1:abort_on_error=0:halt_on_error=1',
               UBSAN_OPTIONS='print_stacktrace=1:halt_on_error=1')
    r = subprocess.run([exe, lst, str(a.mutations)], env=env, capture_output=True, text=True)
    text = ('$ %s %s %d\n%s%s[exit %d]\n' % (os.path.relpath(exe, ROOT), 'inputs.txt',
                                              a.mutations, r.stdout, r.stderr, r.returncode))
    if a.log:
        with open(a.log, 'w') as fh:
            fh.write(text)
    sys.stdout.write(text)
    return r.returncode


if __name__ == '__main__':
    sys.exit(main())
