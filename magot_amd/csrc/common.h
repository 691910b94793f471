// Internal definitions shared by the libmagot translation units.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "../../include/magot.h"

namespace magot {

// ---------------------------------------------------------------------------
// Genome layout in HBM
// ---------------------------------------------------------------------------
// All contigs live in one global base coordinate space.  Coordinate 0 is
// preceded by kOrigin pad bases so that a 16-base window ending at any real
// base never starts below 0 (the reverse-strand gather reads [hi-15, hi]).
constexpr uint64_t kOrigin = 64;
// Exception-run directory granularity: one u32 per 4096 bases.
constexpr int kDirShift = 12;
constexpr uint32_t kDirClean = 0x80000000u;  // no run touches this block
constexpr uint64_t kRcBit = 1ull << 63;

// A maximal run of one byte that is not in ACGTacgt (N, n, IUPAC, '-', ' ' ...).
struct ExcRun {
  uint64_t start;  // global coordinate of the first base
  uint32_t len;
  uint32_t byte;   // the raw byte
};
static_assert(sizeof(ExcRun) == 16, "ExcRun must be 16 bytes");

struct HostPacked {
  // Forward nibble plane over [0, span) bases (span: multiple of 32 with >= 64
  // bases of zero padding past the last contig).  Base g is nibble g & 7 of
  // word g >> 3: bits 0-1 code (A C G T = 0..3), bit 2 soft-masked
  // (lower-case), bit 3 exception (byte kept in `runs`, code bits 0).  The
  // device mirrors it into the reverse-strand plane (mirror_planes).
  // Every word is written by the packer (no zero-fill pass).
  std::unique_ptr<uint32_t[]> nib;
  uint64_t nib_words = 0;
  uint64_t span = 0;
  std::vector<ExcRun> runs;       // sorted by start, sentinel appended
  std::vector<uint32_t> dir;      // per 4096-block first run with end > block start
  std::vector<uint64_t> contig_base;
  std::vector<uint64_t> contig_len;
  uint64_t extent = 0;            // first coordinate past the last contig
};

// A contig's bytes: contiguous (width == 0: ptr[0, len)), or still in FASTA
// line layout -- every line `width` sequence bytes then a `term`-byte line
// terminator, the last line holding the remainder -- so the packer reads
// the file text directly.
struct ContigSource {
  const uint8_t* ptr;
  uint64_t len;    // bases
  uint64_t width;  // 0: contiguous
  uint32_t term;   // 1 ("\n") or 2 ("\r\n")
};

// FASTA text -> contigs with GenomeSequence semantics (fasta.cpp).  Records
// whose lines are not uniform are stripped into `storage`.  Returns
// MAGOT_ERR_UNSUPPORTED for headers only the Python reader handles exactly.
struct FastaContigs {
  std::vector<std::string> names;
  std::vector<ContigSource> src;
  std::vector<std::string> storage;
};
int scan_fasta(const char* text, uint64_t n, bool truncate, FastaContigs* out);
// The contig's bases, contiguous, into dst[0, src.len).
void copy_contig(const ContigSource& src, uint8_t* dst);

// Packs contig bytes (multi-threaded host code, pack.cpp).
void pack_genome(const ContigSource* src, uint32_t n, HostPacked* out);
// The coordinate layout alone (contig bases, extent, span, nib_words).
void pack_layout(const ContigSource* src, uint32_t n, HostPacked* out);
// out->dir from out->runs (sorted, sentinel appended) and out->extent.
void exc_runs_directory(HostPacked* out);
// bases [pos, pos + n) of a contig, contiguous, into dst (fasta.cpp).
void copy_bases(const ContigSource& src, uint64_t pos, uint64_t n, uint8_t* dst);

// Device packing (devpack.hip): raw = the contigs' bytes concatenated in
// coordinate order (raw index i = global base kOrigin + i), n bytes, padded
// with readable bytes to a multiple of 32.
size_t devpack_scan_bytes(uint64_t n_groups);
// count[g] = exception runs starting in raw bytes [32g, 32g+32); slot = their
// exclusive prefix sum (n_groups = ceil(n / 32) entries each).
hipError_t launch_run_count(const uint8_t* raw, uint64_t n, uint32_t* count, uint64_t* slot,
                            void* scan_tmp, size_t scan_bytes, hipStream_t s);
// every run's first coordinate, end coordinate (exclusive) and byte, in order
void launch_run_write(const uint8_t* raw, uint64_t n, const uint64_t* slot, uint64_t* run_start,
                      uint64_t* run_end, uint8_t* run_byte, hipStream_t s);
// the forward nibble plane, nib_words words (pad bases 0)
void launch_nib_pack(const uint8_t* raw, uint64_t n, uint32_t* nib, uint64_t nib_words,
                     hipStream_t s);
// dst[dst_off[i], dst_off[i+1]) = src[src_off[i], ...) for i < n (devpack.hip)
void launch_segments_copy(const uint8_t* src, const uint64_t* src_off, const uint64_t* dst_off,
                          uint64_t n, uint8_t* dst, hipStream_t s);

// Compact replica image of a packed genome (wire.hip; magot_genome_wire_*).
constexpr uint64_t kWireMagic = 0x3257544f47414d00ull;  // "\0MAGOTW2"
struct WireHeader {
  uint64_t magic;
  uint64_t span;       // of the genome it was cut from
  uint64_t n_mask;     // soft-mask runs (the sentinel pair follows them)
  uint64_t n_mdir;     // mask directory entries
  uint64_t o_code2, o_mask, o_mdir, o_exc;  // byte offsets in the image
  uint64_t exc_bytes;  // the arena's exception runs + directory region
  uint64_t total;      // image bytes
  uint64_t meta_hash;  // FNV-1a of the genome's meta blob (magot_genome_export)
};
size_t wire_scan_bytes(uint64_t groups);
// count[g] = soft-mask runs starting in bases [32g, 32g+32) of the forward
// plane; slot = their exclusive prefix sum (span / 32 entries each)
hipError_t launch_wire_count(const uint32_t* nib, uint64_t span, uint32_t* count, uint64_t* slot,
                             void* scan_tmp, size_t scan_bytes, hipStream_t s);
// every mask run's {start, end} at its slot (u32 pairs)
void launch_wire_runs(const uint32_t* nib, uint64_t span, const uint64_t* slot, uint32_t* runs,
                      hipStream_t s);
void launch_wire_mdir(const uint32_t* runs, uint64_t n, uint64_t n_blocks, uint32_t* mdir,
                      hipStream_t s);
// the forward nibble plane (span / 8 words) from an image's pieces
void launch_wire_unpack(const uint32_t* code2, const uint32_t* mask, uint64_t n_mask,
                        const uint32_t* mdir, uint64_t n_mdir, const ExcRun* exc, uint64_t n_exc,
                        const uint32_t* edir, uint64_t n_edir, uint64_t span, uint32_t* nib,
                        hipStream_t s);

// ---------------------------------------------------------------------------
// Extraction tiling
// ---------------------------------------------------------------------------
constexpr int kThreads = 256;                 // one workgroup = 4 independent waves
constexpr int kWaves = kThreads / 64;
constexpr int kChunk = 16;                    // bytes per lane-store
// Chunk slots per lane per tile: 6 (6096-byte tiles) for large plans; 3
// (3024-byte tiles) for translating plans too small to fill the chip several
// times over (one GPU's share of an 8-GPU C4 job: -3.5 % per launch; 4-GPU
// share -2.7 %; but the 2-GPU share +8 %, C2 (nucleotides only) +5.5 %;
// EXPERIMENTS.md §3).  Full C3: 6 slots -2.5 to -3.1 % against 5 (a tile's
// fixed chain of dependent loads paid 17 % less often; 77 VGPRs, 26.4 KB LDS
// per block, still 6 blocks per CU), 7 slots (with 3 residue chunks per lane)
// no better than 5 (89 VGPRs: 5 blocks per CU), 4 slots +3.6 %
// (profiles/r05/large_tile/).
constexpr int kLaneChunksLarge = 6, kLaneChunksSmall = 3;
// Output bytes of a tile cut for `lane_chunks` slots per lane (3 slots of halo):
// 6096 for the large tile (<= 2032 residues, <= 127 residue chunks: within
// kPepSlots), 3024 for the small one.  Size any per-tile storage with the
// template's LC.
constexpr int tile_bytes(int lane_chunks) { return (64 * lane_chunks - 3) * 16; }
// plans whose large-tile count is below this use the small tile
constexpr uint64_t kSmallTilePlan = 40000;
// extraction tiles end on this output boundary where they can (bytes)
constexpr uint64_t kTileAlign = 128;
constexpr int kPepPerLane = 2;                // residue chunk slots per lane
constexpr int kHalo = 3 * kChunk;             // look-ahead decoded past the tile: codons of
                                              // the residues rounded up to a 16-byte store
constexpr int kExonCap = 128;  // intervals staged in LDS per tile (7 blocks of 4 waves fit a CU's LDS)
static_assert((kExonCap & (kExonCap - 1)) == 0, "kExonCap must be a power of two (row index masks)");
constexpr int kTxCap = 64;                    // records staged in LDS per tile
constexpr int kPepSlots = 64 * kPepPerLane;  // residue chunks per tile
constexpr uint64_t kExcBit = 1ull << 62;      // interval touches an exception run
constexpr uint64_t kSlowLitBit = 1ull << 61;  // ... whose byte has no literal class (below)
constexpr uint64_t kExFlagBits = kRcBit | kExcBit | kSlowLitBit;

// Exception bases carry a literal class in their nibble's low three bits
// (nibble = 8 | class): the bytes the kernels can write without the run
// list.  Forward strand: N n - R Y K M; any other byte is class 7 and its
// intervals take the run-list path.  The reverse-strand mirror holds the
// class of the reverse-complement literal (genome.py:787,792: N, n, - kept,
// everything else becomes n), which is always 0, 1 or 2.
__host__ __device__ constexpr uint32_t lit_class(uint32_t b) {
  return b == 'N' ? 0u : b == 'n' ? 1u : b == '-' ? 2u : b == 'R' ? 3u : b == 'Y' ? 4u
       : b == 'K' ? 5u : b == 'M' ? 6u : 7u;
}
constexpr uint32_t kLitLo = 0x522D6E4Eu;  // classes 0..3: N n - R (little-endian bytes)
constexpr uint32_t kLitHi = 0x4E4D4B59u;  // classes 4..7: Y K M (7: never written from here)

// One 16-byte output store with the non-temporal hint (global_store_dwordx4
// ... nt): the outputs are written once and never re-read by the kernel, so
// they stream through L2 instead of displacing genome lines.  A/B on one box
// (200 back-to-back C3 steps): 0.2905 -> 0.2779 ms per step (the plain-store
// variant: scripts/experiments/plain_store.patch).
__device__ __forceinline__ void store16(uint8_t* dst, uint4 v) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  u32x4 x = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(x, reinterpret_cast<u32x4*>(dst));
}

// Debug switches carried in ExtractArgs.outputs (env MAGOT_DEBUG_PATHS):
// force the general per-segment / per-residue paths.
constexpr uint32_t kDebugSlowNuc = 1u << 8;
constexpr uint32_t kDebugSlowPep = 1u << 9;

// One extraction tile (a wave's work): nucleotide output bytes [T0, T1),
// residues [Q0, Q1), staged intervals [e1, e2) and records [j1, j2).  Tiles
// are stored in launch order, which is not output order: tiles that may take
// the run-list path go first (magot_plan_create), so their extra dependent
// loads overlap the rest of the launch instead of extending its tail.
struct TileRec {
  uint64_t T0, T1, Q0, Q1;
  uint32_t e1, e2, j1, j2;
};
static_assert(sizeof(TileRec) == 48, "TileRec is 48 bytes");

// Device plan.  Zero-length intervals and records without a codon are
// compacted away on the host (they add no output); tiles are 16-byte aligned
// ranges of the nucleotide output of at most tile_bytes(lane_chunks) bytes, cut shorter where
// they would touch more than kExonCap intervals or kTxCap records.
struct ExtractArgs {
  // Nibble plane in unified coordinates: [0, span) forward strand, [span,
  // 2*span) reverse strand, where u = 2*span-1-g holds the complement of g.
  const uint32_t* nib;
  uint64_t span;
  const ExcRun* runs;
  const uint32_t* dir;
  const uint64_t* ex_g;       // per interval: global genome start | kRcBit
  const uint64_t* ex_out;     // n+1 output prefix offsets
  const uint64_t* tx_nuc;     // per codon-bearing record: output start (n+1, sentinel B)
  const uint64_t* tx_pep;     // per codon-bearing record: residue start (n+1, sentinel P)
  const TileRec* tiles;       // n_tiles, in launch order
  uint8_t* nuc;
  uint8_t* pep;
  uint64_t total_nuc;
  uint64_t total_pep;
  uint32_t n_tiles;
  uint32_t outputs;
  uint32_t lut[16];           // 64 residue bytes indexed c0 + 4*c1 + 16*c2
  uint32_t lane_chunks;       // tile size the plan was cut for (kLaneChunksLarge / Small)
};

// Wave-wide inclusive prefix sum with DPP row shifts and row broadcasts
// (gfx9 wave64: row_shr:1/2/4/8 inside rows of 16, then row_bcast:15/31).
// The row_bcast controls exist only on gfx9 (CDNA) wave64 targets.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__GFX9__)
#error "wave_scan uses DPP row_bcast:15/31, which exists only on gfx9 wave64 (gfx950) targets"
#endif
__device__ __forceinline__ uint32_t wave_scan(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, true);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, true);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, true);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);
  return v;
}

// Dynamic LDS (never touched by the kernel) that caps a kernel at `want`
// resident blocks per CU; 0 when it already fits or want <= 0.
inline size_t occupancy_lds_pad(const void* fn, int threads, int want) {
  if (want <= 0) return 0;
  int dev = 0, lds_cu = 0, n = 0;
  hipFuncAttributes at{};
  if (hipGetDevice(&dev) != hipSuccess || hipFuncGetAttributes(&at, fn) != hipSuccess ||
      hipDeviceGetAttribute(&lds_cu, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev) !=
          hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, threads, 0) != hipSuccess || n <= want)
    return 0;
  const size_t need = (size_t)lds_cu / (size_t)(want + 1) + 1;  // > 1/(want+1) of the CU's LDS
  return need > at.sharedSizeBytes ? need - at.sharedSizeBytes : 0;
}

void launch_extract(const ExtractArgs& a, hipStream_t s);
int extract_blocks_per_cu();
// Fill the reverse-strand half of the nibble plane.
void launch_mirror_planes(uint32_t* nib, uint64_t span, hipStream_t s);

// ---------------------------------------------------------------------------
// Raw sequence batch ops (seqops.hip)
// ---------------------------------------------------------------------------
void launch_revcomp(const uint8_t* in, const uint64_t* off, uint64_t n, uint64_t total,
                    uint8_t* out, hipStream_t s);
// Six translations per record for Sequence.get_orfs (orf6_kernel): stream
// j = 6*record + 2*frame + (strand == '+'); boff = n_rec+1 offsets of each
// record's block of six 16-byte padded streams (strand-major inside the block,
// magot_orf6_sizes; the kernel derives each stream's place from the record's
// length); noff = n_rec+1 offsets of the records in the concatenation.
// The records are either bytes (nuc, readable up to the next 16-byte
// boundary) or gathered from the genome plane through interval rows
// {unified anchor, start} (n_rows + a sentinel row {0, total}): base P of
// the concatenation is unified coordinate anchor + P of its interval.
// Tiles (orf6_plan_tiles): t0 = n_tiles+1 starts, r0 = record holding each
// start, e0 = interval holding each staged window's first base.
constexpr uint32_t kOrf6RowCap = 123;  // intervals per staged window
constexpr uint64_t kOrf6ExcRow = 1ull << 63;  // row start flag: the interval touches an exception run
struct Orf6Args {
  const uint8_t* nuc;
  const uint32_t* nib;
  uint64_t nib_words;      // both planes
  const uint32_t* code2;   // 2-bit codes of the same unified bases, 16 per word
  uint64_t code2_words;    // = nib_words / 2
  const uint32_t* exc1;    // exception bits of the same unified bases, 32 per word
  uint64_t exc1_words;     // = nib_words / 4
  const uint64_t* rows;
  uint64_t n_rows;
  const uint64_t* noff;
  uint64_t n_rec;
  uint64_t total;
  const uint64_t* boff;
  const uint64_t* tile_t0;
  const uint32_t* tile_r0;
  const uint32_t* tile_e0;
  const uint32_t* tile_m;  // rows of the tile's window (interval starts before its end), <= kOrf6RowCap
  uint64_t n_tiles;
  const uint8_t* tables;  // 256 bytes from orf6_tables
  uint8_t* out;
};
struct Orf6Tiles {
  std::vector<uint64_t> t0;
  std::vector<uint32_t> r0, e0, m;
};
void orf6_tables(const uint8_t lut64[64], uint8_t out[256]);
void orf6_plan_tiles(const uint64_t* noff, uint64_t n_rec, const uint64_t* row_start,
                     uint64_t n_rows, Orf6Tiles* out);
void launch_orf6(const Orf6Args& a, bool genome, hipStream_t s);
// The 2-bit code plane of a nibble plane (nib_words words, 8 bases each):
// word w holds the codes of unified bases 16w .. 16w+15 (base k at bits 2k).
void launch_code2(const uint32_t* nib, uint64_t nib_words, uint32_t* code2, hipStream_t s);
// The exception-bit plane: word w holds bit 3 of the nibbles of unified bases
// 32w .. 32w+31 (base k at bit k).
void launch_exc1(const uint32_t* nib, uint64_t nib_words, uint32_t* exc1, hipStream_t s);
void launch_translate(const uint8_t* in, const uint64_t* off, uint64_t n, const int32_t* frames,
                      const uint8_t* strands, const uint64_t* pep_off, uint64_t total_pep,
                      const uint32_t* lut16, uint8_t* out, hipStream_t s);
// Codon symbols over an extended alphabet (magot_codon_symbols): K classes,
// K^3 <= kMaxSymbolLut.
constexpr uint32_t kMaxSymbolLut = 32768;
void launch_codon_symbols(const uint8_t* in, uint64_t n_codons, const uint8_t* cls, uint32_t K,
                          const uint8_t* lut, uint8_t* out, hipStream_t s);

// ---------------------------------------------------------------------------
// FASTA text assembly (render.hip, gffplan.cpp)
// ---------------------------------------------------------------------------
// A run of skeleton text followed by at most one record payload.
constexpr uint32_t kNoRecord = 0xFFFFFFFFu;
struct TextUnit {
  uint64_t text_off;
  uint32_t text_len;
  uint32_t rec;  // record index, or kNoRecord
};
// Record indices in ascending key order, ties in index order (pack.cpp;
// magot_plan_create's genome-order layout).  key.size() < 2^32.
void radix_order(const std::vector<uint64_t>& key, std::vector<uint32_t>* out);
// The planner's skeleton as units (consecutive text pieces merged).
// Returns false when a record index does not fit a TextUnit.
bool gffplan_units(const magot_gffplan* p, const std::string** text, std::vector<TextUnit>* units,
                   bool* protein, uint64_t* n_rec);
size_t text_scan_bytes(uint64_t n);
void launch_text_assembly(const TextUnit* units, uint64_t n, const uint64_t* rspan,
                          const uint8_t* pay, int protein, const uint8_t* text, uint64_t* len,
                          uint64_t* psrc, uint64_t* end, void* scan_tmp, size_t scan_bytes,
                          uint8_t* out, hipStream_t s);

// Standard genetic code (genome.py:795-802) as a 64-byte table indexed
// c0 + 4*c1 + 16*c2 with A=0, C=1, G=2, T=3.
void standard_lut(uint8_t out[64]);

// ---------------------------------------------------------------------------
// Errors
// ---------------------------------------------------------------------------
void set_error(const std::string& msg);

}  // namespace magot

#define MAGOT_HIP_TRY(expr)                                                      \
  do {                                                                           \
    hipError_t e_ = (expr);                                                      \
    if (e_ != hipSuccess) {                                                      \
      ::magot::set_error(std::string(#expr) + ": " + hipGetErrorString(e_));     \
      return MAGOT_ERR_HIP;                                                      \
    }                                                                            \
  } while (0)
