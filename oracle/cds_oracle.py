"""ctypes wrapper of the C oracle (cds_oracle.c) -- TEST INFRASTRUCTURE ONLY.

``build()`` compiles it with gcc into oracle/build/libcds_oracle.so (git-
ignored, travels to the GPU box with the snapshot).  ``extract_workload``
runs the reference's per-record loop over a synth.Workload on the CPU.
"""

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, 'cds_oracle.c')
LIB = os.path.join(HERE, 'build', 'libcds_oracle.so')

ST_OK, ST_NONE_PIECE, ST_TRANSLATE_NONE = 0, 1, 2

_lib = None


def build(force=False):
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(SRC):
        subprocess.check_call(['gcc', '-O2', '-std=c99', '-shared', '-fPIC', '-o', LIB, SRC])
    return LIB


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        vp = ctypes.c_void_p
        L.oracle_extract.restype = ctypes.c_int64
        L.oracle_extract.argtypes = [vp, vp, ctypes.c_int64, ctypes.c_int64, vp, vp, vp, vp, vp,
                                     ctypes.c_int, vp, vp, vp]
        L.oracle_orf6_compare.restype = ctypes.c_int64
        L.oracle_orf6_compare.argtypes = [vp, vp, ctypes.c_int64, ctypes.c_int64, vp, vp, vp,
                                          ctypes.POINTER(ctypes.c_int64), vp, ctypes.c_int64]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def extract(genome, contig_off, rec_off, child_contig, child_c0, child_c1, child_strand,
            protein):
    """Run the oracle.  All arrays numpy; child_strand uint8 (raw bytes).
    Returns (out uint8[], out_off int64[n_rec+1], status int32[n_rec])."""
    genome = np.ascontiguousarray(genome, dtype=np.uint8)
    contig_off = np.ascontiguousarray(contig_off, dtype=np.int64)
    rec_off = np.ascontiguousarray(rec_off, dtype=np.int64)
    ck = np.ascontiguousarray(child_contig, dtype=np.int32)
    c0 = np.ascontiguousarray(child_c0, dtype=np.int64)
    c1 = np.ascontiguousarray(child_c1, dtype=np.int64)
    sk = np.ascontiguousarray(child_strand, dtype=np.uint8)
    n_rec = len(rec_off) - 1
    cap = int(np.maximum(c1 - c0 + 1, 0).sum()) + 64
    out = np.empty(cap, dtype=np.uint8)
    ooff = np.empty(n_rec + 1, dtype=np.int64)
    status = np.empty(max(n_rec, 1), dtype=np.int32)
    n = lib().oracle_extract(_p(genome), _p(contig_off), len(contig_off) - 1, n_rec, _p(rec_off),
                             _p(ck), _p(c0), _p(c1), _p(sk), int(bool(protein)), _p(out),
                             _p(ooff), _p(status))
    return out[:n], ooff, status[:n_rec]


def extract_workload(w, protein, tx_subset=None):
    """The reference loop over a synth.Workload (children in GFF order:
    ascending exons, all with the transcript's strand)."""
    first = np.zeros(w.n_tx + 1, dtype=np.int64)
    np.cumsum(w.ex_count, out=first[1:])
    tx_ids = np.arange(w.n_tx) if tx_subset is None else np.asarray(tx_subset)
    counts = w.ex_count[tx_ids]
    rec_off = np.zeros(len(tx_ids) + 1, dtype=np.int64)
    np.cumsum(counts, out=rec_off[1:])
    idx = np.concatenate([np.arange(first[t], first[t + 1]) for t in tx_ids]) if len(tx_ids) \
        else np.zeros(0, np.int64)
    tx_of = np.repeat(tx_ids, counts)
    c0 = w.ex_start[idx] + 1
    c1 = w.ex_start[idx] + w.ex_len[idx]
    strand = np.where(w.tx_strand[tx_of] < 0, ord('-'), ord('+')).astype(np.uint8)
    return extract(w.genome, w.contig_off, rec_off, w.tx_contig[tx_of], c0, c1, strand, protein)


def orf6_compare(seq, seq_off, dev_out, stream_off, stream_len, threads=1, bad_list=None):
    """Six-frame device output (magot_orf6_* layout) against the reference's
    translate(frame, strand) for every record and frame (genome.py:795-851),
    records split over ``threads`` threads (ctypes releases the GIL).
    Returns (mismatching streams, first mismatching stream or -1); with a list
    as ``bad_list``, the mismatching stream ids (up to 1000 per thread) are
    appended to it."""
    from concurrent.futures import ThreadPoolExecutor
    seq = np.ascontiguousarray(seq, dtype=np.uint8)
    so = np.ascontiguousarray(seq_off, dtype=np.int64)
    dev_out = np.ascontiguousarray(dev_out, dtype=np.uint8)
    soff = np.ascontiguousarray(stream_off, dtype=np.uint64)
    slen = np.ascontiguousarray(stream_len, dtype=np.uint64)
    n = len(so) - 1
    L = lib()
    bounds = np.linspace(0, n, max(1, threads) + 1).astype(np.int64)

    def run(i):
        fb = ctypes.c_int64()
        bl = np.full(1000, -1, dtype=np.int64)
        k = L.oracle_orf6_compare(_p(seq), _p(so), int(bounds[i]), int(bounds[i + 1]),
                                  _p(dev_out), _p(soff), _p(slen), ctypes.byref(fb), _p(bl),
                                  len(bl))
        if bad_list is not None:
            bad_list.extend(int(x) for x in bl[bl >= 0])
        return k, fb.value

    with ThreadPoolExecutor(max(1, threads)) as ex:
        res = list(ex.map(run, range(len(bounds) - 1)))
    bad = sum(k for k, _ in res)
    firsts = [f for _, f in res if f >= 0]
    return bad, (min(firsts) if firsts else -1)
