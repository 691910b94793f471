"""ctypes binding of libmagot.so (C ABI: include/magot.h).

The library is loaded from the package directory (built in-tree by
``magot_amd.build``).  There is no fallback: if the library is missing, or no
HIP device is visible when a device call is made, a ``MagotError`` is raised.
"""

import ctypes
import os
import threading

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# MAGOT_LIB: an alternative build of the same library (A/B kernel experiments)
LIB_PATH = os.environ.get('MAGOT_LIB') or os.path.join(HERE, 'libmagot.so')

OUT_NUC = 1
OUT_PEP = 2
OUT_GENOME_ORDER = 4  # layout flag: records in genome order in the device buffers

EXON_DTYPE = np.dtype([('start_rc', '<u8'), ('contig', '<u4'), ('len', '<u4')])
TX_DTYPE = np.dtype([('exon_begin', '<u8'), ('n_exons', '<u4'), ('flags', '<u4')])
RC_BIT = np.uint64(1 << 63)

# Every symbol include/magot.h declares (checked by tests/test_abi.py).
EXPORTS = (
    'magot_abi_version', 'magot_last_error', 'magot_device_count',
    'magot_ctx_create', 'magot_ctx_destroy', 'magot_ctx_sync', 'magot_ctx_info',
    'magot_genome_load', 'magot_genome_stats', 'magot_genome_destroy',
    'magot_plan_create', 'magot_plan_destroy', 'magot_plan_execute', 'magot_plan_fetch',
    'magot_run', 'magot_plan_time', 'magot_plan_time_b2b', 'magot_plan_device_outputs',
    'magot_plan_layout',
    'magot_plan_algorithmic_bytes',
    'magot_revcomp_batch', 'magot_translate_sizes', 'magot_translate_batch',
    'magot_codon_symbols', 'magot_revcomp', 'magot_translate',
    'magot_gff_plan', 'magot_gff_read', 'magot_gff_lower', 'magot_flank_plan',
    'magot_gffplan_tables', 'magot_gffplan_table_views', 'magot_gffplan_render',
    'magot_gffplan_destroy',
    'magot_gffplan_selections', 'magot_cds_scan', 'magot_cds_render',
    'magot_genome_export', 'magot_genome_copy_arena', 'magot_genome_attach',
    'magot_plan_copy_outputs',
    'magot_orf6_sizes', 'magot_orf6_batch', 'magot_plan_orf6', 'magot_orf6_execute',
    'magot_orf6_fetch', 'magot_orf6_time', 'magot_orf6_time_b2b', 'magot_orf6_destroy',
    'magot_genome_load_fasta', 'magot_genome_contigs', 'magot_fasta_read',
    'magot_fasta_text_create', 'magot_fasta_text_execute', 'magot_fasta_text_fetch',
    'magot_fasta_text_time', 'magot_fasta_text_destroy',
    'magot_genome_load_ex', 'magot_genome_wire_ranges', 'magot_genome_attach_wire',
    'magot_copy_segments', 'magot_ctx_mark', 'magot_ctx_elapsed', 'magot_orf6_copy_outputs',
    'magot_genome_wire_export', 'magot_genome_wire_import',
)

ERR_ARG = -1
ERR_HIP = -2
ERR_RANGE = -3
ERR_STATE = -4
ERR_UNSUPPORTED = -5
GFF_PROTEIN = 1
GFF_ORDER_PY2 = 2
GFF_LONGEST = 4
GFF_GENOMIC = 8
GFF_FROM_EXONS = 16
PACK_HOST = 1


class MagotError(RuntimeError):
    """A libmagot call failed (status + magot_last_error text)."""


_u8p = ctypes.POINTER(ctypes.c_uint8)
_u64p = ctypes.POINTER(ctypes.c_uint64)
_i64p = ctypes.POINTER(ctypes.c_int64)
_i32p = ctypes.POINTER(ctypes.c_int32)
_vp = ctypes.c_void_p

_lib = None
_lib_lock = threading.RLock()


def _declare(lib):
    sig = {
        'magot_abi_version': (ctypes.c_int, []),
        'magot_last_error': (ctypes.c_char_p, []),
        'magot_device_count': (ctypes.c_int, []),
        'magot_ctx_create': (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(_vp)]),
        'magot_ctx_destroy': (None, [_vp]),
        'magot_ctx_sync': (ctypes.c_int, [_vp]),
        'magot_ctx_info': (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_int),
                                          ctypes.POINTER(ctypes.c_int)]),
        'magot_genome_load': (ctypes.c_int, [_vp, ctypes.POINTER(_u8p), _u64p, ctypes.c_uint32,
                                             ctypes.POINTER(_vp)]),
        'magot_genome_stats': (ctypes.c_int, [_vp, _u64p, _u64p, _u64p]),
        'magot_genome_destroy': (None, [_vp]),
        'magot_plan_create': (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_uint64, _vp, ctypes.c_uint64,
                                             ctypes.c_uint32, ctypes.POINTER(_vp), _u64p, _u64p]),
        'magot_plan_destroy': (None, [_vp]),
        'magot_plan_execute': (ctypes.c_int, [_vp, _vp]),
        'magot_plan_fetch': (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp]),
        'magot_run': (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp]),
        'magot_plan_time': (ctypes.c_int, [_vp, _vp, ctypes.c_int,
                                           ctypes.POINTER(ctypes.c_double)]),
        'magot_plan_time_b2b': (ctypes.c_int, [_vp, _vp, ctypes.c_int,
                                               ctypes.POINTER(ctypes.c_double)]),
        'magot_plan_layout': (ctypes.c_int, [_vp, _vp, _vp]),
        'magot_plan_device_outputs': (ctypes.c_int, [_vp, ctypes.POINTER(_vp),
                                                     ctypes.POINTER(_vp)]),
        'magot_plan_algorithmic_bytes': (ctypes.c_uint64, [_vp]),
        'magot_revcomp_batch': (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_uint64, _vp]),
        'magot_translate_sizes': (ctypes.c_int, [_vp, ctypes.c_uint64, _vp, _vp, _vp]),
        'magot_translate_batch': (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_uint64, _vp, _vp, _vp,
                                                 _vp, _vp]),
        'magot_codon_symbols': (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, _vp, ctypes.c_uint32,
                                               _vp, _vp]),
        'magot_revcomp': (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, _vp]),
        'magot_translate': (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_int, _vp, _i64p]),
        'magot_gff_plan': (ctypes.c_int, [_vp, ctypes.c_uint64,
                                          ctypes.POINTER(ctypes.c_char_p), _u64p, ctypes.c_uint32,
                                          ctypes.c_char_p, ctypes.c_uint32, ctypes.POINTER(_vp),
                                          _u64p, _u64p]),
        'magot_gff_read': (ctypes.c_int, [_vp, ctypes.c_uint64, ctypes.c_uint32,
                                          ctypes.POINTER(_vp)]),
        'magot_gff_lower': (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_char_p), _u64p,
                                           ctypes.c_uint32, ctypes.c_char_p, ctypes.c_uint32,
                                           _u64p, _u64p]),
        'magot_flank_plan': (ctypes.c_int, [_vp, ctypes.c_uint64,
                                            ctypes.POINTER(ctypes.c_char_p), _u64p,
                                            ctypes.c_uint32, ctypes.c_char_p, ctypes.c_char_p,
                                            ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(_vp),
                                            _u64p, _u64p]),
        'magot_gffplan_tables': (ctypes.c_int, [_vp, _vp, _vp]),
        'magot_gffplan_table_views': (ctypes.c_int, [_vp, ctypes.POINTER(_vp),
                                                     ctypes.POINTER(_vp)]),
        'magot_gffplan_render': (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, ctypes.c_uint64,
                                                _u64p]),
        'magot_gffplan_destroy': (None, [_vp]),
        'magot_gffplan_selections': (ctypes.c_int, [_vp, _u64p]),
        'magot_cds_scan': (ctypes.c_int, [_vp, ctypes.c_uint64, _u64p, _u64p, _vp, _vp, _vp, _vp,
                                          ctypes.c_uint64]),
        'magot_cds_render': (ctypes.c_int, [_vp, ctypes.c_uint64, _vp, _vp, _vp, _vp, _vp, _vp,
                                            _vp, ctypes.c_uint64, _u64p]),
        'magot_genome_export': (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, _u64p, _u64p]),
        'magot_genome_copy_arena': (ctypes.c_int, [_vp, _vp]),
        'magot_genome_attach': (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, _vp,
                                               ctypes.POINTER(_vp)]),
        'magot_plan_copy_outputs': (ctypes.c_int, [_vp, _vp, _vp, _vp]),
        'magot_orf6_sizes': (ctypes.c_int, [_vp, ctypes.c_uint64, _vp, _vp, _vp]),
        'magot_orf6_batch': (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_uint64, _vp, _vp, _vp]),
        'magot_plan_orf6': (ctypes.c_int, [_vp, _vp, _vp, ctypes.POINTER(_vp), _u64p]),
        'magot_orf6_execute': (ctypes.c_int, [_vp, _vp]),
        'magot_orf6_fetch': (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp]),
        'magot_orf6_time': (ctypes.c_int, [_vp, _vp, ctypes.c_int,
                                           ctypes.POINTER(ctypes.c_double)]),
        'magot_orf6_time_b2b': (ctypes.c_int, [_vp, _vp, ctypes.c_int,
                                               ctypes.POINTER(ctypes.c_double)]),
        'magot_orf6_destroy': (None, [_vp]),
        'magot_fasta_text_create': (ctypes.c_int, [_vp, _vp, _vp, ctypes.POINTER(_vp), _u64p]),
        'magot_fasta_text_execute': (ctypes.c_int, [_vp, _vp]),
        'magot_fasta_text_fetch': (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_uint64, _u64p]),
        'magot_fasta_text_time': (ctypes.c_int, [_vp, _vp, ctypes.c_int,
                                                 ctypes.POINTER(ctypes.c_double)]),
        'magot_fasta_text_destroy': (None, [_vp]),
        'magot_genome_load_fasta': (ctypes.c_int, [_vp, _vp, ctypes.c_uint64,
                                                   ctypes.c_int, ctypes.POINTER(_vp)]),
        'magot_genome_contigs': (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_uint32), _vp, _vp,
                                                ctypes.c_uint64, _u64p]),
        'magot_genome_load_ex': (ctypes.c_int, [_vp, ctypes.POINTER(_u8p), _u64p, ctypes.c_uint32,
                                                ctypes.c_uint32, ctypes.POINTER(_vp)]),
        'magot_genome_wire_ranges': (ctypes.c_int, [_vp, _u64p, _u64p,
                                                    ctypes.POINTER(ctypes.c_uint32)]),
        'magot_genome_attach_wire': (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, _vp,
                                                    ctypes.POINTER(_vp)]),
        'magot_genome_wire_export': (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, _u64p]),
        'magot_genome_wire_import': (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, _vp,
                                                    ctypes.c_uint64, ctypes.POINTER(_vp)]),
        'magot_copy_segments': (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, _vp, _vp, _vp,
                                               ctypes.c_uint64]),
        'magot_ctx_mark': (ctypes.c_int, [_vp, ctypes.c_int]),
        'magot_orf6_copy_outputs': (ctypes.c_int, [_vp, _vp, _vp]),
        'magot_ctx_elapsed': (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_double)]),
        'magot_fasta_read': (ctypes.c_int, [_vp, ctypes.c_uint64, ctypes.c_int,
                                            ctypes.POINTER(ctypes.c_uint32), _vp, _vp,
                                            ctypes.c_uint64, _u64p, _vp, ctypes.c_uint64]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


def lib():
    """The loaded library (raises MagotError when it is not built)."""
    global _lib
    if _lib is None:
        with _lib_lock:
            if _lib is None:
                if not os.path.exists(LIB_PATH):
                    raise MagotError('libmagot.so not built at %s (run python -m magot_amd.build)'
                                     % LIB_PATH)
                _lib = _declare(ctypes.CDLL(LIB_PATH))
    return _lib


def check(rc, what):
    if rc != 0:
        msg = lib().magot_last_error().decode('utf-8', 'replace')
        raise MagotError('%s failed (status %d): %s' % (what, rc, msg))


def ptr(arr):
    """Address of a contiguous numpy array (or None for empty/None)."""
    if arr is None:
        return None
    return arr.ctypes.data_as(_vp)


class Context(object):
    """One device + one HIP stream (magot_ctx)."""

    def __init__(self, device=0):
        L = lib()
        n = L.magot_device_count()
        if n <= 0:
            raise MagotError('no HIP device visible: the MI355X extraction path needs a GPU')
        h = _vp()
        check(L.magot_ctx_create(int(device), ctypes.byref(h)), 'magot_ctx_create')
        self.handle = h
        self.device = int(device)

    def sync(self):
        check(lib().magot_ctx_sync(self.handle), 'magot_ctx_sync')

    def mark(self, which):
        """Record timing event `which` (0 = start, 1 = end) on the context
        stream (magot_ctx_mark)."""
        check(lib().magot_ctx_mark(self.handle, int(which)), 'magot_ctx_mark')

    def elapsed_ms(self):
        """GPU time between marks 0 and 1 (waits for mark 1)."""
        ms = ctypes.c_double()
        check(lib().magot_ctx_elapsed(self.handle, ctypes.byref(ms)), 'magot_ctx_elapsed')
        return ms.value

    def info(self):
        """{'n_cu', 'extract_blocks_per_cu'} of the device (magot_ctx_info)."""
        n_cu, blocks = ctypes.c_int(), ctypes.c_int()
        check(lib().magot_ctx_info(self.handle, ctypes.byref(n_cu), ctypes.byref(blocks)),
              'magot_ctx_info')
        return {'n_cu': n_cu.value, 'extract_blocks_per_cu': blocks.value}

    def close(self):
        if self.handle:
            lib().magot_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_default_ctx = None


def default_context():
    """Process-wide context on LOCAL_RANK's device (one process per GPU)."""
    global _default_ctx
    if _default_ctx is None:
        with _lib_lock:
            if _default_ctx is None:
                dev = int(os.environ.get('MAGOT_DEVICE', os.environ.get('LOCAL_RANK', '0')))
                _default_ctx = Context(dev)
    return _default_ctx
