"""End-to-end gff2fasta on a BASELINE-shaped synthetic (default C3): writes the
FASTA + GFF3 text files, then times each phase of the native CLI path
(genome_tools._gff2fasta_native) -- FASTA parse, native GFF plan, genome pack
+ H2D, plan upload, kernel, device text assembly, one D2H -- and checks the output
against the C oracle's record bytes.  Writes one JSON line.

    python scripts/e2e_cli.py [--config C3] [--seq-type protein] [--dir /tmp/magot_e2e]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from magot_amd import engine, genome, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='C3')
    ap.add_argument('--seq-type', default='protein')
    ap.add_argument('--dir', default='/tmp/magot_e2e')
    ap.add_argument('--order', default='py2')
    ap.add_argument('--ids', default='synth', choices=['synth', 'ncbi'],
                    help="the GFF3's IDs: 'synth' (renamed CDS IDs collide, read_gff's "
                         "renaming cascades) or 'ncbi' (NCBI-style, all distinct)")
    ap.add_argument('--whole', action='store_true',
                    help='time the CLI call (genome_tools._gff2fasta_native) on the files of '
                         'an earlier run, in this fresh process, and compare with its out.fa')
    ap.add_argument('--layout', default='record', choices=['record', 'genome'],
                    help='extraction plan layout for the phase run')
    a = ap.parse_args()
    os.makedirs(a.dir, exist_ok=True)
    fa, gf = os.path.join(a.dir, 'genome.fa'), os.path.join(a.dir, 'ann.gff3')
    if a.whole:
        from magot_amd import genome_tools
        clock = genome_tools._Clock()
        clock.on = True
        t = time.perf_counter()
        text = genome_tools._gff2fasta_native(fa, gf, a.seq_type, a.order, clock=clock)[0]
        total = time.perf_counter() - t
        # the call's device buffers and planner tables are freed on a
        # background thread after it returns (genome_tools._Release)
        if clock.release_thread is not None:
            clock.release_thread.join()
        released = time.perf_counter() - t
        with open(os.path.join(a.dir, 'out.fa'), 'rb') as fh:
            same = fh.read() == bytes(text) + b'\n'
        print(json.dumps({'config': a.config, 'seq_type': a.seq_type, 'order': a.order,
                          'cli_call_s': total, 'equals_phase_run_output': same,
                          'released_s': released,
                          'phases_s': clock.laps, 'stamps_s': clock.stamps}), flush=True)
        return
    t = time.perf_counter()
    w = synth.make(a.config)
    with open(fa, 'w') as fh:
        fh.write(w.fasta_text())
    with open(gf, 'w') as fh:
        fh.write(w.gff3_text(ids=a.ids))
    t_gen = time.perf_counter() - t
    ph = {}
    t0 = time.perf_counter()
    from magot_amd import _lib
    _lib.default_context()  # device start-up (HIP runtime, context, stream)
    ph['device_context'] = time.perf_counter() - t0
    t = time.perf_counter()
    dev = engine.FastaGenome.load(genome.read_buffer(fa))
    ph['fasta_read_pack_h2d_native'] = time.perf_counter() - t
    t = time.perf_counter()
    names = dev.names
    protein = a.seq_type == 'protein'
    plan = engine.GffPlan.build(genome.read_buffer(gf), names, [int(x) for x in dev.lengths],
                                protein=protein, order=a.order)
    ph['gff_read_and_plan_native'] = time.perf_counter() - t
    assert plan is not None
    t = time.perf_counter()
    # as the CLI builds it (record order: one launch does not repay the
    # genome-order layout's extra planning; --layout genome to compare)
    ex = engine.ExtractionPlan(dev, plan.exons, plan.txs,
                               (engine.OUT_PEP if protein else engine.OUT_NUC)
                               | (engine.OUT_GENOME_ORDER if a.layout == 'genome' else 0))
    ph['plan_h2d'] = time.perf_counter() - t
    t = time.perf_counter()
    ex.execute()
    ex.sync()
    ph['kernel'] = time.perf_counter() - t
    t = time.perf_counter()
    ft = engine.FastaText(plan, ex)
    ph['text_skeleton_h2d'] = time.perf_counter() - t
    t = time.perf_counter()
    ft.execute()
    ex.sync()
    ph['text_assembly_device'] = time.perf_counter() - t
    t = time.perf_counter()
    text = ft.fetch()
    ph['text_d2h'] = time.perf_counter() - t
    t = time.perf_counter()
    with open(os.path.join(a.dir, 'out.fa'), 'wb') as fh:
        fh.write(text)
        fh.write(b'\n')
    ph['write'] = time.perf_counter() - t
    total = time.perf_counter() - t0
    kernel_ms = ex.time(10)
    text_ms = ft.time(10)
    # host render of the fetched payloads (the previous CLI path) must agree
    nuc, noff, pep, poff = ex.fetch()
    t = time.perf_counter()
    host_text = plan.render(nuc, noff, pep, poff)
    host_render_s = time.perf_counter() - t
    text_match = host_text == text.tobytes()
    # payload check against the C oracle on the same tables
    from oracle import cds_oracle
    ex_t, tx_t = plan.exons, plan.txs
    st = ex_t['start_rc'].astype(np.uint64)
    rc = (st >> np.uint64(63)).astype(bool)
    start = (st & np.uint64((1 << 63) - 1)).astype(np.int64)
    rec_off = np.zeros(len(tx_t) + 1, dtype=np.int64)
    np.cumsum(tx_t['n_exons'].astype(np.int64), out=rec_off[1:])
    ref, roff, rst = cds_oracle.extract(w.genome, w.contig_off, rec_off, ex_t['contig'],
                                        start + 1, start + ex_t['len'].astype(np.int64),
                                        np.where(rc, ord('-'), ord('+')).astype(np.uint8),
                                        protein)
    if not protein:
        ok = bool(np.array_equal(nuc, ref) and np.array_equal(noff.astype(np.int64), roff))
    else:
        starts = poff[:-1].astype(np.int64)
        lens = (poff[1:] - poff[:-1]).astype(np.int64)
        first = np.zeros(len(starts), dtype=bool)
        first[lens > 0] = pep[starts[lens > 0]] == ord('X')
        keep = np.ones(len(pep), dtype=bool)
        keep[starts[first]] = False
        ok = bool(np.array_equal(pep[keep], ref))
    rec = {'config': a.config, 'seq_type': a.seq_type, 'order': a.order, 'ids': a.ids,
           'records': int(len(plan.txs)), 'intervals': int(len(plan.exons)),
           'cds_bases': int(w.cds_bases), 'output_bytes': len(text) + 1,
           'gff_lines': None, 'phases_s': ph, 'end_to_end_s': total,
           'kernel_ms_hip_events': kernel_ms, 'text_assembly_ms_hip_events': text_ms,
           'host_render_s_reference_point': host_render_s, 'generate_files_s': t_gen,
           'payload_check': ok, 'device_text_equals_host_render': text_match}
    print(json.dumps(rec), flush=True)


if __name__ == '__main__':
    main()
