/*
 * magot.h -- C ABI of libmagot.so, the MI355X (gfx950) extraction engine behind
 * the magot_amd Python package.
 *
 * The reference (Huangtianyu-caas/MAGOT, Python 2.7) has no FFI: its hot path is
 * the pure-Python call chain
 *     AnnotationSet.get_fasta          genome.py:578-582
 *       ParentAnnotation.get_fasta     genome.py:677-731
 *         BaseAnnotation.get_seq       genome.py:603-614
 *           Sequence.reverse_compliment genome.py:784-793
 *         Sequence.translate           genome.py:795-822
 * over a GenomeSequence dict (genome.py:854-877).  This header is the boundary
 * that chain is cut at: the Python layer (magot_amd/genome.py) walks the
 * annotation graph exactly as the reference does and hands the resulting
 * interval lists to this library; every byte of sequence output is produced
 * by HIP kernels.  Plain pointers and sizes only -- no torch types.
 *
 * Ownership: callers own every host buffer; the library owns device memory
 * behind the opaque handles, released by the matching *_destroy.
 * Errors: every int-returning call returns MAGOT_OK (0) or a negative status;
 * magot_last_error() gives a thread-local message.
 * Threading: a magot_ctx is bound to one device and one HIP stream and is not
 * thread-safe; use one context per host thread.  One process per GPU.
 */
#ifndef MAGOT_H
#define MAGOT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MAGOT_ABI_VERSION 1

enum magot_status {
  MAGOT_OK = 0,
  MAGOT_ERR_ARG = -1,      /* bad argument / inconsistent tables           */
  MAGOT_ERR_HIP = -2,      /* HIP runtime failure (no device, OOM, fault)   */
  MAGOT_ERR_RANGE = -3,    /* interval outside its contig                   */
  MAGOT_ERR_STATE = -4,    /* call out of order (e.g. fetch before execute) */
  MAGOT_ERR_UNSUPPORTED = -5 /* input takes a reference diagnostic path: use the
                                Python object path (magot_gff_plan)              */
};

/* Output selection for a plan (magot_plan_create.outputs). */
#define MAGOT_OUT_NUC 1u   /* spliced CDS nucleotides  (seq_type="nucleotide") */
#define MAGOT_OUT_PEP 2u   /* frame-0 translation      (seq_type="protein")    */
/* Layout flag: lay the records out in the device buffers in genome order (by
 * the coordinate of each record's first non-empty interval) instead of record
 * order.  Neighbouring loci then run in neighbouring tiles and share genome
 * lines.  magot_plan_fetch, magot_plan_copy_outputs and magot_fasta_text_*
 * still deliver record order (a device segment copy puts the records back);
 * magot_plan_layout gives each record's place in the device buffers.  Such a
 * plan has no six-frame plan (magot_plan_orf6 refuses it). */
#define MAGOT_OUT_GENOME_ORDER 4u

/*
 * One interval of one record, already in OUTPUT order.
 *   start_rc : bits 0..62 = 0-based start inside the contig (the Python slice
 *              contig[c0-1:c1] already normalised by slice.indices, so
 *              genome.py:606/608 semantics incl. clamping are resolved);
 *              bit 63 = reverse-complement this interval (strand '-',
 *              genome.py:607-608).
 *   contig   : index into the contig list given to magot_genome_load.
 *   len      : number of bases (0 allowed: empty Python slice).
 * Replaces: BaseAnnotation.get_seq (genome.py:603-614) per child, ordered as
 * ParentAnnotation.get_fasta orders them (genome.py:689-703).
 */
typedef struct magot_exon {
  uint64_t start_rc;
  uint32_t contig;
  uint32_t len;
} magot_exon;

/*
 * One output record = the contiguous exon range [exon_begin, exon_begin+n_exons).
 * Records must tile the exon table in order (exon_begin[t+1] ==
 * exon_begin[t] + n_exons[t]).  flags is reserved (0).
 * Replaces: the "".join of genome.py:702-705 for one ParentAnnotation.
 */
typedef struct magot_tx {
  uint64_t exon_begin;
  uint32_t n_exons;
  uint32_t flags;
} magot_tx;

typedef struct magot_ctx magot_ctx;
typedef struct magot_genome magot_genome;
typedef struct magot_plan magot_plan;

/* ABI version compiled into the library (== MAGOT_ABI_VERSION). */
int magot_abi_version(void);

/* Thread-local text of the last failure on this thread ("" if none). */
const char* magot_last_error(void);

/* Number of visible HIP devices (0 when none / runtime unavailable). */
int magot_device_count(void);

/* Bind a context to HIP device `device` with a private non-blocking stream. */
int magot_ctx_create(int device, magot_ctx** out);
void magot_ctx_destroy(magot_ctx* ctx);

/*
 * Pack a genome into HBM: a nibble plane (2-bit ACGT code, soft-mask bit,
 * exception bit per base) plus its reverse-complement mirror, and a run list
 * of every byte that is not ACGTacgt (N, IUPAC, '-', spaces ...) with a
 * 4096-base directory.  seqs[i] points at lens[i] raw bytes of contig i,
 * exactly the bytes genome.py:875 keeps (every byte except CR/LF).  One
 * device plane holds up to ~4 Gbases; above that MAGOT_ERR_UNSUPPORTED, and
 * the caller packs the contigs as several planes, one magot_genome each
 * (magot_amd.engine.PartitionedGenome: one plan per plane).
 * Replaces: GenomeSequence (genome.py:854-877) as the data the path reads.
 */
int magot_genome_load(magot_ctx* ctx, const uint8_t* const* seqs, const uint64_t* lens,
                      uint32_t n_contigs, magot_genome** out);
/*
 * The same with flags.  By default (and in magot_genome_load /
 * magot_genome_load_fasta) the packing runs on the device: the raw bytes are
 * streamed into HBM once through pinned buffers and kernels build the nibble
 * plane, its mirror and the exception runs (the run list's directory is built
 * on the host from the runs).  MAGOT_PACK_HOST packs on the host (pack.cpp,
 * the sanitizer-tested twin) and uploads the plane; both give the same arena
 * bytes (tests/test_gpu_replication.py).
 */
#define MAGOT_PACK_HOST 1u
int magot_genome_load_ex(magot_ctx* ctx, const uint8_t* const* seqs, const uint64_t* lens,
                         uint32_t n_contigs, uint32_t flags, magot_genome** out);
/*
 * Read FASTA text (GenomeSequence, genome.py:854-877, incl. truncate_names)
 * natively and pack it like magot_genome_load (MAGOT_ERR_UNSUPPORTED above
 * one device plane, as there).  MAGOT_ERR_UNSUPPORTED also for
 * headers whose whitespace split differs between the reference's Python 2
 * byte strings and Python 3 (bytes >= 0x80, 0x1c-0x1f) or that are empty
 * under truncate_names: the caller then uses the Python reader.
 * magot_genome_contigs: contig count, lengths and NUL-separated names (names
 * only for genomes read by magot_genome_load_fasta; NULL buffers = sizes).
 */
int magot_genome_load_fasta(magot_ctx* ctx, const char* text, uint64_t len, int truncate_names,
                            magot_genome** out);
int magot_genome_contigs(const magot_genome* g, uint32_t* n, uint64_t* lens, char* names,
                         uint64_t names_cap, uint64_t* names_len);
/* Host-only: the same FASTA reader into caller buffers (first call with NULL
 * buffers for the count, lengths and name bytes; lens needs n entries). */
int magot_fasta_read(const char* text, uint64_t len, int truncate_names, uint32_t* n,
                     uint64_t* lens, char* names, uint64_t names_cap, uint64_t* names_len,
                     uint8_t* seqs, uint64_t seqs_cap);

/*
 * cds2pep (genome_tools.py:664-675) without a per-line loop.  magot_cds_scan
 * splits `text` into lines ('\n'; a CR before it is dropped): lines starting
 * with '>' are headers (hdr_off / hdr_len[n_seg-1]), all others are appended
 * to the current sequence; segment k (seq[seg_off[k]:seg_off[k+1]], n_seg+1
 * offsets) is the sequence before header k, the last one follows the last
 * header.  Call with NULL buffers for n_seg / seq_bytes first.
 * MAGOT_ERR_UNSUPPORTED: an empty line (the reference's IndexError) or a CR
 * inside a line; the caller's line loop reproduces both.  magot_cds_render
 * writes the tool's stdout from the frame-0 translations of the segments
 * (magot_translate_batch layout: poff, codons < 0 for None): a translation
 * for every non-empty segment before a header and for the last one ("None"
 * when translate() returns None, one leading 'X' trimmed), each header after
 * its segment.  out == NULL: *out_len only.
 */
int magot_cds_scan(const char* text, uint64_t len, uint64_t* n_seg, uint64_t* seq_bytes,
                   uint64_t* seg_off, uint64_t* hdr_off, uint64_t* hdr_len, uint8_t* seq,
                   uint64_t seq_cap);
int magot_cds_render(const char* text, uint64_t n_seg, const uint64_t* seg_off,
                     const uint64_t* hdr_off, const uint64_t* hdr_len, const uint8_t* pep,
                     const uint64_t* poff, const int64_t* codons, uint8_t* out, uint64_t cap,
                     uint64_t* out_len);

/* Sizes of a loaded genome: total bases, exception runs, device bytes held. */
int magot_genome_stats(const magot_genome* g, uint64_t* total_bases, uint64_t* n_exc_runs,
                       uint64_t* device_bytes);
void magot_genome_destroy(magot_genome* g);

/*
 * Genome replication across ranks (one packed genome broadcast
 * over RCCL/xGMI instead of every rank packing its own).  The packed genome
 * is one device arena plus a host meta blob:
 *   magot_genome_export    meta blob (meta == NULL: size only) and arena size;
 *   magot_genome_copy_arena D2D copy of the arena into caller device memory
 *                          (e.g. the tensor a collective broadcasts);
 *   magot_genome_attach    a genome over caller device memory holding a
 *                          broadcast arena (not freed by magot_genome_destroy).
 */
int magot_genome_export(const magot_genome* g, uint8_t* meta, uint64_t cap, uint64_t* meta_len,
                        uint64_t* arena_bytes);
int magot_genome_copy_arena(const magot_genome* g, void* dst_dev);
int magot_genome_attach(magot_ctx* ctx, const uint8_t* meta, uint64_t meta_len, void* arena_dev,
                        magot_genome** out);
/*
 * What a replica must receive: magot_genome_wire_ranges gives the *n (= 2)
 * byte ranges [off[k], off[k]+len[k]) of the arena to transfer -- the forward
 * nibble plane (span/2 bytes), then the exception runs and their directory.
 * The reverse-strand mirror between them (as many bytes again) is a pure
 * function of the forward plane (genome.py:784-793), so
 * magot_genome_attach_wire attaches like magot_genome_attach and then rebuilds
 * the mirror on the receiving device: half the bytes cross xGMI.  The caller
 * memory must be arena_bytes long and hold the wire ranges at their offsets.
 */
int magot_genome_wire_ranges(const magot_genome* g, uint64_t* off, uint64_t* len, uint32_t* n);
int magot_genome_attach_wire(magot_ctx* ctx, const uint8_t* meta, uint64_t meta_len,
                             void* arena_dev, magot_genome** out);
/*
 * The compact replica image (what a multi-GPU job broadcasts; the north
 * star's 2-bit-packed genome): the forward strand's 2-bit codes (span/4
 * bytes), the soft-masked bases as sorted {start, end} u32 runs plus a
 * directory of one u32 per 4096 bases, and the arena's exception runs +
 * directory verbatim -- every GenomeSequence byte (genome.py:854-877), about
 * 0.27 B per base against the arena's 1 B.
 *   magot_genome_wire_export  writes the image of g into caller device memory
 *       of cap bytes (wire_dev == NULL: *wire_bytes only).  Synchronous.
 *   magot_genome_wire_import  a genome in its own new arena (freed by
 *       magot_genome_destroy) rebuilt on ctx's device from an image in device
 *       memory and the genome's meta blob (magot_genome_export): the nibble
 *       plane is unpacked and the mirror derived there; the arena equals the
 *       packed original byte for byte.  The image may be freed on return.
 *       An image that does not match the meta is refused (MAGOT_ERR_ARG).
 * No reference counterpart (the reference is single-process).
 */
int magot_genome_wire_export(const magot_genome* g, void* wire_dev, uint64_t cap,
                             uint64_t* wire_bytes);
int magot_genome_wire_import(magot_ctx* ctx, const uint8_t* meta, uint64_t meta_len,
                             const void* wire_dev, uint64_t wire_bytes, magot_genome** out);

/*
 * Reassembly of a sharded job's outputs on one device (outputs
 * gathered back, final order restored from the global record index): for
 * i < n, dst[dst_off[i], dst_off[i+1]) = src[src_off[i], src_off[i] +
 * dst_off[i+1] - dst_off[i]).  src (src_bytes long) and dst (dst_off[n] long)
 * are device memory (e.g. the buffer an RCCL gather filled, rank-major),
 * both 16-byte aligned (else MAGOT_ERR_ARG),
 * dst_off has n+1 non-decreasing entries, the offset tables are host arrays;
 * a segment reaching past src_bytes is refused (MAGOT_ERR_RANGE) before any
 * launch, and so is a segment of 4 GiB or more (MAGOT_ERR_ARG: the grouped
 * copy counts 16-byte chunks in 32 bits; split such a segment).  Synchronous.
 * No reference counterpart (the reference is single-process).
 */
int magot_copy_segments(magot_ctx* ctx, const void* src_dev, uint64_t src_bytes, void* dst_dev,
                        const uint64_t* src_off, const uint64_t* dst_off, uint64_t n);

/*
 * Build a device-resident plan: interval table -> output offsets, ~3 KiB
 * wave tiles, per-tile exon and record ranges, all uploaded to HBM.
 * nuc_bytes / pep_bytes receive the total output sizes (pep_bytes counts the
 * untrimmed frame-0 translation, floor(len/3) per record; the single leading
 * 'X' trim of genome.py:819-821 is applied by the caller on fetch).
 */
int magot_plan_create(magot_ctx* ctx, const magot_genome* g, const magot_exon* exons,
                      uint64_t n_exons, const magot_tx* txs, uint64_t n_tx, uint32_t outputs,
                      magot_plan** out, uint64_t* nuc_bytes, uint64_t* pep_bytes);
void magot_plan_destroy(magot_plan* p);

/* Enqueue the fused gather + reverse-complement + translate kernel on the
 * context stream (asynchronous; outputs stay in HBM). */
int magot_plan_execute(magot_ctx* ctx, magot_plan* p);

/* Block until the context stream is idle. */
int magot_ctx_sync(magot_ctx* ctx);

/* Timing marks on the context stream: magot_ctx_mark(ctx, 0) and (ctx, 1)
 * record events before and after a region of enqueued work (e.g. bench.py's
 * K timed steps); magot_ctx_elapsed waits for mark 1 and gives the GPU time
 * between them in ms.  No reference counterpart (measurement). */
int magot_ctx_mark(magot_ctx* ctx, int which);
int magot_ctx_elapsed(magot_ctx* ctx, double* ms);

/* Device facts of a context: compute units, and the extraction kernel's
 * resident workgroups per CU as launched (its occupancy cap included).  Any
 * pointer may be NULL.  No reference counterpart (diagnostics for bench.py). */
int magot_ctx_info(const magot_ctx* ctx, int* n_cu, int* extract_blocks_per_cu);

/* Copy outputs to caller buffers (synchronous).  Any pointer may be NULL to
 * skip it.  nuc_off / pep_off receive n_tx+1 prefix offsets.  A plan built
 * with MAGOT_OUT_GENOME_ORDER is put back into record order on the device on
 * the way down, through a transient device scratch of at most 256 MiB (or
 * the longest record, if longer) plus 16 bytes, batch by batch of records. */
int magot_plan_fetch(magot_ctx* ctx, magot_plan* p, uint8_t* nuc_out, uint64_t* nuc_off,
                     uint8_t* pep_out, uint64_t* pep_off);

/* execute + sync + fetch. */
int magot_run(magot_ctx* ctx, magot_plan* p, uint8_t* nuc_out, uint64_t* nuc_off,
              uint8_t* pep_out, uint64_t* pep_off);

/*
 * Kernel timing: execute `iters` times back to back on the context stream with
 * HIP events around each launch; *avg_ms receives the mean launch duration.
 */
int magot_plan_time(magot_ctx* ctx, magot_plan* p, int iters, double* avg_ms);
/* The same with ONE event pair around `iters` back-to-back launches: the
 * per-launch time of a step loop, the figure bench.py's roofline uses (it
 * agrees with rocprofv3's kernel-trace average; an isolated launch also pays
 * the launch latency, which dominates small plans such as C2). */
int magot_plan_time_b2b(magot_ctx* ctx, magot_plan* p, int iters, double* avg_ms);

/* D2D copy of a plan's outputs (nuc_bytes / pep_bytes) into caller device
 * memory, e.g. the buffers an output gather sends, in record order (a
 * genome-ordered plan's records are put back by a segment copy: its
 * destinations must then be 16-byte aligned, else MAGOT_ERR_ARG). */
int magot_plan_copy_outputs(magot_ctx* ctx, magot_plan* p, void* nuc_dst_dev, void* pep_dst_dev);

/* Device-resident output pointers of a plan (for on-device consumers/tests).
 * The buffers hold the records in the plan's layout order: record t starts at
 * magot_plan_layout's nuc_start[t] / pep_start[t] and is as long as its
 * prefix offsets (magot_plan_fetch) say. */
int magot_plan_device_outputs(magot_plan* p, void** nuc_dev, void** pep_dev);

/* Each record's start in the plan's device buffers (n_tx entries each; either
 * pointer may be NULL): the prefix offsets for a record-order plan, the
 * genome-order places for a MAGOT_OUT_GENOME_ORDER one.  No reference
 * counterpart (device layout). */
int magot_plan_layout(const magot_plan* p, uint64_t* nuc_start, uint64_t* pep_start);

/* Algorithmic byte count per execute of a plan (the roofline numerator):
 * ceil(B/4) + B*[nuc] + P*[pep] + 16*E + 32*T. */
uint64_t magot_plan_algorithmic_bytes(const magot_plan* p);

/*
 * Raw-sequence batch ops over n byte strings (seq_off has n+1 entries).
 * Replaces: Sequence.reverse_compliment (genome.py:784-793).
 * out must hold seq_off[n] bytes; record i lands at out[seq_off[i]...].
 */
int magot_revcomp_batch(magot_ctx* ctx, const uint8_t* seqs, const uint64_t* seq_off, uint64_t n,
                        uint8_t* out);

/*
 * Replaces: Sequence.translate (genome.py:795-822) for frame >= 0, strand
 * '+'/'-'.  codons_out[i] = number of emitted residues (before trimX), or -1
 * when the reference returns None (len <= 2 + frame).  pep_off (n+1) must be
 * filled by magot_translate_sizes first; out holds pep_off[n] bytes.
 * lut64 maps codon c0 + 4*c1 + 16*c2 (A=0,C=1,G=2,T=3) to a residue byte;
 * NULL = the standard code of genome.py:795-802.  The junk first codon of
 * frames 1/2 (genome.py:811-818) is emitted as 'X'.
 */
int magot_translate_sizes(const uint64_t* seq_off, uint64_t n, const int32_t* frames,
                          uint64_t* pep_off, int64_t* codons_out);
int magot_translate_batch(magot_ctx* ctx, const uint8_t* seqs, const uint64_t* seq_off, uint64_t n,
                          const int32_t* frames, const uint8_t* strands, const uint8_t* lut64,
                          const uint64_t* pep_off, uint8_t* out);

/*
 * Single-sequence forms of the two (the SURVEY 8(b) sketch), same semantics.
 * magot_revcomp: out holds len bytes.  magot_translate: standard code, frame
 * >= 0 (MAGOT_ERR_UNSUPPORTED below: the Python layer lays negative frames out
 * itself), strand '+' or '-', trimX 0/1; out must hold (len + 2) / 3 bytes
 * (frames 1 and 2 emit a junk first codon: frame 1 of a length with len % 3
 * == 2 gives (len + 1) / 3 residues before the trim); exactly *out_len bytes
 * are written; *out_len = residues, or -1 where the reference returns None.
 */
int magot_revcomp(magot_ctx* ctx, const uint8_t* seq, uint64_t len, uint8_t* out);
int magot_translate(magot_ctx* ctx, const uint8_t* seq, uint64_t len, int frame, int strand,
                    int trimX, uint8_t* out, int64_t* out_len);

/*
 * Sequence.translate with an arbitrary codon `library` (genome.py:795-818:
 * any dict -- keys that are not ACGT triplets, e.g. 'NNN', multi-character
 * values -- and any integer frame, negative included).  The caller lays out
 * the characters the reference's loop visits and drops the first (junk)
 * codon; this computes one symbol per full codon of seq[0, 3*n_codons):
 * out[k] = lut[c0 + K*c1 + K*K*c2], c = class256[byte] (upper-case folding
 * and the library's key characters folded into K = n_classes classes,
 * K^3 <= 32768).  The caller maps symbols to the library's values.
 */
int magot_codon_symbols(magot_ctx* ctx, const uint8_t* seq, uint64_t n_codons,
                        const uint8_t* class256, uint32_t n_classes, const uint8_t* lut,
                        uint8_t* out);

/*
 * Six-frame translation for Sequence.get_orfs (genome.py:824-851): for each
 * record, translate(frame=f, strand) for f = 0,1,2 and strand '-','+' in the
 * reference's loop order.  Stream j = 6*record + 2*f + (strand == '+') holds
 * the REAL codons only: frames 1/2 start with a junk 1-/2-base codon that
 * trimX always drops (genome.py:809-821), so it is not emitted; frame 0 is
 * untrimmed (the caller drops one leading 'X').  Streams start on 16-byte
 * boundaries, a record's three '-' streams before its three '+' streams
 * (strand-major: the kernel writes each strand's chunks in one pass):
 * stream_off (6n+1) are the padded offsets (stream_off[6n] the total),
 * stream_len (6n) the real residue counts, and the padding bytes are 0;
 * none_mask[j] = 1 where the reference returns None (len <= 2 + f).  Because
 * of the strand-major placement stream_off[j+1] is NOT where stream j's
 * padding ends: stream j occupies [stream_off[j], stream_off[j] +
 * pad16(stream_len[j])), pad16(x) = (x + 15) & ~15, and a record's six streams
 * are one contiguous block [stream_off[6r], stream_off[6r+6]).  Callers that
 * need the extents must pass stream_len; none_mask may be NULL.
 */
int magot_orf6_sizes(const uint64_t* seq_off, uint64_t n, uint64_t* stream_off,
                     uint64_t* stream_len, uint8_t* none_mask);
/* magot_orf6_batch: stream_off must be exactly magot_orf6_sizes' table for
 * seq_off (the kernel places every stream from its record's block start and
 * length); any other table is refused with MAGOT_ERR_ARG before a launch. */
int magot_orf6_batch(magot_ctx* ctx, const uint8_t* seqs, const uint64_t* seq_off, uint64_t n,
                     const uint8_t* lut64, const uint64_t* stream_off, uint8_t* out);
/* The same over an extraction plan's records, in HBM (BASELINE configs[4],
 * C5): one kernel gathers each record from the packed genome through the
 * plan's intervals and writes its six translations (the plan's nucleotide
 * output is not needed).  The kernel walks the records in genome order and
 * lays their six-stream blocks out in that order (its stores then stream
 * through the output): stream j is at the stream_off[j] magot_orf6_fetch
 * returns (16-byte aligned, stream_len[j] residues, zero padding), a record's
 * six streams form one contiguous block in the same strand-major order as
 * magot_orf6_sizes, and stream_off[6n] is the total.  MAGOT_ORF6_ORDER=record
 * keeps record order (then stream_off equals magot_orf6_sizes'). */
typedef struct magot_orf6 magot_orf6;
int magot_plan_orf6(magot_ctx* ctx, magot_plan* p, const uint8_t* lut64, magot_orf6** out,
                    uint64_t* total_res);
int magot_orf6_execute(magot_ctx* ctx, magot_orf6* o);
int magot_orf6_fetch(magot_ctx* ctx, magot_orf6* o, uint8_t* out, uint64_t* stream_off,
                     uint64_t* stream_len);
/* D2D copy of the padded residue bytes (total_res) into caller device memory
 * (e.g. the buffer an output gather sends). */
int magot_orf6_copy_outputs(magot_ctx* ctx, magot_orf6* o, void* dst_dev);
int magot_orf6_time(magot_ctx* ctx, magot_orf6* o, int iters, double* avg_ms);
int magot_orf6_time_b2b(magot_ctx* ctx, magot_orf6* o, int iters, double* avg_ms);
void magot_orf6_destroy(magot_orf6* o);

/*
 * Native batch planner for gff2fasta (genome_tools.py:324-330).
 * Parses GFF3/GTF text with read_gff's rules and default arguments
 * (genome.py:242-415: '#'/8-tab acceptance, version sniffing, ID synthesis
 * and de-duplication, v2 parent hierarchy, Base/Parent typing), keeps the
 * AnnotationSet model (global ID lookup: last matching type in sorted order,
 * genome.py:536-544) and lowers AnnotationSet.get_fasta(feature)
 * (genome.py:578-582, 677-731) to interval and record tables for
 * magot_plan_create plus a FASTA text skeleton.
 * seqids / contig_lens: the GenomeSequence (genome.py:854-877) in the order
 * its contigs were given to magot_genome_load.  flags: MAGOT_GFF_PROTEIN for
 * seq_type="protein", MAGOT_GFF_ORDER_PY2 for CPython 2.7 dict order,
 * MAGOT_GFF_GENOMIC for genomic=True (genome.py:680-682: one '+' interval per
 * feature over its get_coords() span, never translated, so the plan is a
 * nucleotide plan whatever MAGOT_GFF_PROTEIN says), MAGOT_GFF_LONGEST for
 * longest=True (genome.py:720-724: the child record with the longest
 * sequence, the later one on a tie).  For protein the lengths depend on the
 * leading-'X' trim, i.e. on the genome: every candidate is planned and
 * magot_gffplan_render picks (magot_gffplan_selections > 0; such a plan has
 * no device text assembly).  MAGOT_GFF_FROM_EXONS: gff2fasta's
 * from_exons="True" reading (genome_tools.py:326-327: "\texon\t" replaced by
 * "\tCDS\t" in each line, then every type that is a substring of "CDS"
 * ignored).
 * Returns MAGOT_ERR_UNSUPPORTED when the input would take one of the
 * reference's diagnostic paths (prints, None, exceptions): the caller then
 * uses the object path, which reproduces them.
 */
#define MAGOT_GFF_PROTEIN 1u
#define MAGOT_GFF_ORDER_PY2 2u
#define MAGOT_GFF_LONGEST 4u
#define MAGOT_GFF_GENOMIC 8u
#define MAGOT_GFF_FROM_EXONS 16u
typedef struct magot_gffplan magot_gffplan;
int magot_gff_plan(const char* gff, uint64_t gff_len, const char* const* seqids,
                   const uint64_t* contig_lens, uint32_t n_contigs, const char* feature,
                   uint32_t flags, magot_gffplan** out, uint64_t* n_exons, uint64_t* n_tx);
/*
 * magot_gff_plan in two steps, so the GFF can be read before the genome's
 * contig names are known (gff2fasta reads the GFF while another thread
 * loads the FASTA): magot_gff_read is read_gff (genome.py:242-415; flags:
 * MAGOT_GFF_FROM_EXONS is the only one it looks at), magot_gff_lower the
 * get_fasta lowering against the contigs (the other flags, as above; once
 * per plan, else MAGOT_ERR_STATE).  `gff` must stay valid until
 * magot_gff_lower returns.  Either returns MAGOT_ERR_UNSUPPORTED for a
 * diagnostic path; the plan handle from magot_gff_read is then still the
 * caller's to destroy.
 */
int magot_gff_read(const char* gff, uint64_t gff_len, uint32_t flags, magot_gffplan** out);
int magot_gff_lower(magot_gffplan* p, const char* const* seqids, const uint64_t* contig_lens,
                    uint32_t n_contigs, const char* feature, uint32_t flags, uint64_t* n_exons,
                    uint64_t* n_tx);
/*
 * extract_upstream_downstream (genome_tools.py:457-480) as a plan of the same
 * shape: one single-interval record per printed window (the `sequence_length`
 * bases before a '+' feature for stream "up", after it reverse-complemented
 * for "down"; mirrored on '-'), names from the last `namefrom=` attribute or
 * "seq<k>", a matching line whose strand is neither '+' nor '-' repeating the
 * previous window, windows shorter than sequence_length dropped, records
 * joined by "\n".  Render it with magot_gffplan_render or magot_fasta_text_*
 * like a gff2fasta plan (nucleotide).  sequence_length is the reference's
 * string argument.  MAGOT_ERR_UNSUPPORTED when the reference would raise
 * (unknown seqid, a bad integer, `namefrom` without '=', no window yet).
 */
int magot_flank_plan(const char* gff, uint64_t gff_len, const char* const* seqids,
                     const uint64_t* contig_lens, uint32_t n_contigs, const char* feature_type,
                     const char* namefrom, const char* sequence_length, const char* stream,
                     magot_gffplan** out, uint64_t* n_exons, uint64_t* n_tx);
/* Copy the planned tables (n_exons / n_tx entries from magot_gff_plan). */
int magot_gffplan_tables(const magot_gffplan* p, magot_exon* exons, magot_tx* txs);
/* The planned tables in place (n_exons / n_tx rows, valid until the plan is
 * destroyed; NULL when empty): magot_plan_create reads them without a copy. */
int magot_gffplan_table_views(const magot_gffplan* p, const magot_exon** exons,
                              const magot_tx** txs);
/* The FASTA text: skeleton + record payloads from magot_plan_fetch (nuc for
 * nucleotide plans, untrimmed pep for protein; the leading-'X' trim of
 * genome.py:819-821 is applied here).  out == NULL: *out_len = size only. */
int magot_gffplan_render(const magot_gffplan* p, const uint8_t* nuc, const uint64_t* noff,
                         const uint8_t* pep, const uint64_t* poff, uint8_t* out, uint64_t cap,
                         uint64_t* out_len);
/* Number of longest=True protein choices the render makes (0: none). */
int magot_gffplan_selections(const magot_gffplan* p, uint64_t* n_groups);
void magot_gffplan_destroy(magot_gffplan* p);

/*
 * The same FASTA text assembled on device: the skeleton of
 * `gp` is uploaded once, and each execute fills it with the payloads of
 * extraction plan `p` (built from gp's tables, with MAGOT_OUT_PEP for a
 * protein skeleton, MAGOT_OUT_NUC otherwise) in one device buffer: per-unit
 * lengths (trimX applied), a scan, and a copy kernel.  fetch synchronises and
 * copies the *out_len bytes (out == NULL: length only).  max_bytes bounds
 * *out_len.  p must outlive the handle.  Replaces the text building of
 * AnnotationSet.get_fasta / ParentAnnotation.get_fasta
 * (genome.py:578-582, 677-731) for the gff2fasta CLI (genome_tools.py:330).
 */
typedef struct magot_fasta_text magot_fasta_text;
int magot_fasta_text_create(magot_ctx* ctx, const magot_gffplan* gp, const magot_plan* p,
                            magot_fasta_text** out, uint64_t* max_bytes);
int magot_fasta_text_execute(magot_ctx* ctx, magot_fasta_text* t);
int magot_fasta_text_fetch(magot_ctx* ctx, magot_fasta_text* t, uint8_t* out, uint64_t cap,
                           uint64_t* out_len);
int magot_fasta_text_time(magot_ctx* ctx, magot_fasta_text* t, int iters, double* avg_ms);
void magot_fasta_text_destroy(magot_fasta_text* t);

#ifdef __cplusplus
}
#endif
#endif /* MAGOT_H */
