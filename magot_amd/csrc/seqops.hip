// Batch kernels over raw byte strings (not the packed genome):
//   revcomp_kernel   -- Sequence.reverse_compliment  genome.py:784-793
//   translate_kernel -- Sequence.translate           genome.py:795-822
// Both are output-stationary: a lane owns 16 aligned output bytes, finds its
// record by binary search over the offset table and reads its inputs from L2.
#include <algorithm>
#include <type_traits>

#include "common.h"

namespace magot {
namespace {

constexpr int kOpsThreads = 256;

__device__ __forceinline__ uint32_t rc_byte(uint32_t b) {
  switch (b) {
    case 'a': return 't';
    case 't': return 'a';
    case 'g': return 'c';
    case 'c': return 'g';
    case 'A': return 'T';
    case 'T': return 'A';
    case 'G': return 'C';
    case 'C': return 'G';
    case 'n': return 'n';
    case 'N': return 'N';
    case '-': return '-';
    default: return 'n';
  }
}

// 2-bit code of an ACGT/acgt byte, or 4 for anything else (upper() then
// library lookup, genome.py:812-817: only the 64 ACGT triplets are keys).
// Branch-free: bits 1-2 of 'A' 'C' 'G' 'T' are 0 1 3 2 (Gray-decoded to
// 0 1 2 3); validity is a 20-bit mask over (b | 0x20) - 'a'.
__device__ __forceinline__ uint32_t code_of(uint32_t b) {
  const uint32_t x = (b >> 1) & 3u;
  const uint32_t v = (b | 0x20u) - 'a';  // a=0 c=2 g=6 t=19
  const bool ok = v < 20u && ((0x80045u >> v) & 1u);
  return ok ? (x ^ (x >> 1)) : 4u;
}

__device__ __forceinline__ uint64_t find_record(const uint64_t* off, uint64_t n, uint64_t p) {
  // last r with off[r] <= p
  uint64_t lo = 0, hi = n;
  while (lo < hi) {
    uint64_t mid = (lo + hi) >> 1;
    if (off[mid] <= p) lo = mid + 1;
    else hi = mid;
  }
  return lo - 1;
}

__global__ __launch_bounds__(kOpsThreads) void revcomp_kernel(const uint8_t* __restrict__ in,
                                                             const uint64_t* __restrict__ off,
                                                             uint64_t n, uint64_t total,
                                                             uint8_t* __restrict__ out) {
  const uint64_t c = ((uint64_t)blockIdx.x * kOpsThreads + threadIdx.x) * 16;
  if (c >= total) return;
  uint64_t r = find_record(off, n, c);
  uint64_t rb = off[r], re = off[r + 1];
  uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const uint64_t p = c + k;
    if (p < total) {
      while (p >= re) {
        ++r;
        rb = re;
        re = off[r + 1];
      }
      const uint32_t b = in[rb + (re - 1 - p)];
      w[k >> 2] |= rc_byte(b) << (8 * (k & 3));
    }
  }
  if (c + 16 <= total) {
    *reinterpret_cast<uint4*>(out + c) = make_uint4(w[0], w[1], w[2], w[3]);
  } else {
    for (int k = 0; c + k < total; ++k) out[c + k] = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
  }
}

struct TranslateLut {
  uint32_t w[16];
};

// Residue j of record r (frame f, strand s, length L):
//   first emitted triplet covers positions [f, pe], pe = f + ((2 - 2f) mod 3)
//   (genome.py:811-813); later triplets are [pe+1+3(j-1), pe+3+3(j-1)].
__global__ __launch_bounds__(kOpsThreads) void translate_kernel(
    const uint8_t* __restrict__ in, const uint64_t* __restrict__ off, uint64_t n,
    const int32_t* __restrict__ frames, const uint8_t* __restrict__ strands,
    const uint64_t* __restrict__ pep_off, uint64_t total, TranslateLut lut,
    uint8_t* __restrict__ out) {
  const uint64_t c = ((uint64_t)blockIdx.x * kOpsThreads + threadIdx.x) * 16;
  if (c >= total) return;
  uint64_t r = find_record(pep_off, n, c);
  uint64_t qb = pep_off[r], qe = pep_off[r + 1];
  uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const uint64_t q = c + k;
    if (q < total) {
      while (q >= qe) {
        ++r;
        qb = qe;
        qe = pep_off[r + 1];
      }
      const uint64_t sb = off[r];
      const uint64_t L = off[r + 1] - sb;
      const int64_t f = frames[r];
      const bool minus = strands[r] == '-';
      const int64_t head = ((2 - 2 * f) % 3 + 3) % 3;  // pe - f
      const uint64_t j = q - qb;
      uint32_t aa = 'X';
      if (!(j == 0 && head < 2)) {
        const uint64_t start = (j == 0) ? (uint64_t)f : (uint64_t)(f + head + 1) + 3 * (j - 1);
        uint32_t cd[3];
#pragma unroll
        for (int e = 0; e < 3; ++e) {
          const uint64_t p = start + e;
          const uint32_t b = minus ? in[sb + (L - 1 - p)] : in[sb + p];
          uint32_t v = code_of(b);
          if (minus && v < 4) v = 3 - v;
          cd[e] = v;
        }
        if (cd[0] < 4 && cd[1] < 4 && cd[2] < 4) {
          const uint32_t x = cd[0] + 4 * cd[1] + 16 * cd[2];
          aa = (lut.w[x >> 2] >> (8 * (x & 3))) & 0xFFu;
        }
      }
      w[k >> 2] |= aa << (8 * (k & 3));
    }
  }
  if (c + 16 <= total) {
    *reinterpret_cast<uint4*>(out + c) = make_uint4(w[0], w[1], w[2], w[3]);
  } else {
    for (int k = 0; c + k < total; ++k) out[c + k] = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
  }
}

// ---------------------------------------------------------------------------
// orf6_kernel -- the six translations Sequence.get_orfs splits into ORFs
// (genome.py:824-851): for frame f in 0,1,2 and strand '-','+' (in that
// order), translate(frame=f, strand) with the frame quirk of
// genome.py:809-818: frame 0 codons start at 0,3,..; frame 1 emits a junk
// 1-base codon then codons at 2,5,..; frame 2 a junk 2-base codon then codons
// at 4,7,...  Only real codons are produced (the junk 'X' is exactly what
// trimX removes for frames 1/2); frame 0 keeps its first residue and the
// caller applies trimX.  Stream j = 6*record + 2*f + (strand == '+').
//
// Output layout: a record's six streams are one block at boff[record], its
// three '-' streams then its three '+' streams, each on a 16-byte boundary
// (the places and real lengths follow from the record length); the bytes of
// a stream's last 16-byte chunk past its end are zero.
//
// Input-stationary: one wave owns a tile of kOrfTile bases of the
// concatenated records and every output chunk whose first codon starts in
// it (all six streams of every record the tile touches).  The tile plus a
// 48/50-base halo is staged once (over the genome: computed in registers
// from the 2-bit code and 1-bit exception planes), as one byte per position:
//   cidx[p] = c[p] | c[p+1] << 2 | c[p+2] << 4 | (any of the three not
//             ACGTacgt) << 6
// so a '+' residue is tbl[cidx[p]] and a '-' residue (codon read backwards,
// complemented) is tbl[128 + cidx[p]] with the second table pre-permuted:
// two LDS reads per residue, each input byte converted once for all six
// streams.  Each staged record byte feeds ~2 output bytes, so the kernel
// streams the nucleotides once and writes the residues once.
// ---------------------------------------------------------------------------
constexpr uint64_t kOrfTile = 3968;  // max bases per wave tile: + halo and alignment = 256 x 16 B
constexpr int kOrfVecs = 256;        // staged 16-byte vectors per wave
constexpr int kOrfBatch = 10;        // records per segment batch: one (record, stream) per lane
constexpr int kOrfSegs = 6 * kOrfBatch;
constexpr int kOrfRankWords = 128;   // chunk bitmap: a batch owns < 4096 chunks
// A batch's chunks start inside the tile: per stream of a record at most
// ov/48 + 1, ov = the record's overlap with the tile (sum over the batch <=
// kOrfTile), six streams per record; far below the 16-bit scan field.
static_assert(6 * (kOrfTile / 48 + 1 + kOrfBatch) < 32 * kOrfRankWords, "chunk bitmap too small");

// real codons of frame f in a record of L bases (0 when translate() is None)
__device__ __host__ __forceinline__ uint64_t orf_count(uint64_t L, uint32_t f) {
  return (L > 2 + f && L >= 2 * f + 3) ? (L - 2 * f) / 3 : 0;
}

// A run of output chunks of one stream, rebased so that the wave-wide chunk
// number q addresses it directly: chunk q writes out0 + 16q from staged
// position p0 + 48q ('+', residues ascending) or p0 - 48q ('-', first
// residue at the highest codon), |rem0| - 16q residues left.
struct OrfSeg {
  uint64_t out0;
  int32_t p0;
  int32_t rem0;  // < 0: '-' strand
};

__device__ __forceinline__ uint64_t div48(uint64_t v) {
  return v < (1ull << 32) ? (uint64_t)((uint32_t)v / 48u) : v / 48;
}

__device__ __forceinline__ uint32_t funnel4(uint32_t hi, uint32_t lo, uint32_t sh) {
  return __builtin_amdgcn_alignbit(hi, lo, sh);
}

// Sixteen nibbles (code | lower << 2 | exception << 3, base k of x0:x1 at
// nibble k) -> sixteen packed 2-bit codes (base k at bits 2k).
__device__ __forceinline__ uint32_t nib_codes(uint32_t x0, uint32_t x1) {
  const uint32_t y0 = (x0 & 0x03030303u) | ((x0 >> 2) & 0x0C0C0C0Cu);
  const uint32_t y1 = (x1 & 0x03030303u) | ((x1 >> 2) & 0x0C0C0C0Cu);
  const uint32_t z0 = (y0 & 0x0F0F0F0Fu) | ((y0 >> 4) & 0xF0F0F0F0u);
  const uint32_t z1 = (y1 & 0x0F0F0F0Fu) | ((y1 >> 4) & 0xF0F0F0F0u);
  return __builtin_amdgcn_perm(z1, z0, 0x06040200u);
}

// The exception bits (nibble bit 3) of sixteen nibbles as a 16-bit mask.
__device__ __forceinline__ uint32_t nib_exc16(uint32_t x0, uint32_t x1) {
  uint32_t e0 = (x0 >> 3) & 0x11111111u, e1 = (x1 >> 3) & 0x11111111u;
  e0 = (e0 | (e0 >> 3)) & 0x03030303u;
  e1 = (e1 | (e1 >> 3)) & 0x03030303u;
  e0 = (e0 | (e0 >> 6)) & 0x000F000Fu;
  e1 = (e1 | (e1 >> 6)) & 0x000F000Fu;
  e0 = (e0 | (e0 >> 12)) & 0xFFu;
  e1 = (e1 | (e1 >> 12)) & 0xFFu;
  return e0 | (e1 << 8);
}

// Staged tile, per wave: the 2-bit codes of its positions (16 per word) and
// their invalid bits (not ACGTacgt; 16 per half-word), each behind a guard
// of 64 positions ('-' chunks read from up to 45 positions before their
// first codon; what they read there is masked off by the stream end).
constexpr int kCodeGuard = 4;   // words of codes before position 0
constexpr int kInvGuard = 4;    // half-words of invalid bits before position 0

// 16-residue chunks, one per lane.  kMode 0: every lane '+', 1: every lane
// '-' (wave-uniform: table offsets fold into the LDS immediates), 2: mixed.
// A chunk's 48 positions of 2-bit codes come from four staged words, aligned
// by one funnel shift per word; codon k's index is then bits [6k, 6k+6) of
// that 96-bit window (a bit-field extract) and its residue one LDS byte read.
// Consecutive chunks of a segment start 48 positions (3 words) apart, so the
// word reads of a half-wave over one segment hit 32 different banks, and each
// 128-entry residue table is one word per bank.  A tile holding a non-ACGT
// base (tile_inv) patches codons with an invalid base to 'X' from the staged
// invalid bits.  (Two chunks per lane per pass, q and q + 64 with both chains
// of dependent LDS reads issued first, measured the same: 1.4737 / 1.4763 vs
// 1.4761 / 1.4787 ms per C5 step.)
struct OrfChunk {
  uint32_t Y[3];     // codes of positions P .. P+47
  int32_t P;         // window position of codon 0 (ascending)
  int32_t rem;       // residues left in the stream from this chunk
  uint64_t dst;      // output byte offset
  bool minus;
};

template <int kMode>
__device__ __forceinline__ OrfChunk orf_fetch(const uint32_t* codes, const OrfSeg* seg,
                                              const uint32_t* bm, const uint32_t* pre,
                                              uint32_t q) {
  // opaque per call: keeps the compiler from hoisting lane-invariant address
  // terms of all three variants out of the chunk loop (and spilling)
  __asm__ volatile("" : "+v"(q));
  const uint32_t wq = q >> 5;
  const uint32_t rank = pre[wq] + __popc(bm[wq] & (0xFFFFFFFFu >> (31 - (q & 31))));
  const OrfSeg g = seg[rank - 1];
  OrfChunk h;
  h.minus = kMode == 1 ? true : kMode == 0 ? false : g.rem0 < 0;
  h.rem = (h.minus ? -g.rem0 : g.rem0) - 16 * (int32_t)q;
  int32_t m48 = (int32_t)__umul24(q, 48u);  // full-rate 24-bit multiply (kept
  __asm__("" : "+v"(m48));                   // from folding into a -48 v_mul_lo)
  const int32_t p = h.minus ? g.p0 - m48 : g.p0 + m48;
  // ascending codon positions: '+' p, p+3, ..; '-' p-45, .., p (reversed later)
  h.P = h.minus ? p - 45 : p;
  h.dst = g.out0 + 16 * (uint64_t)q;
  const uint32_t* const cw = codes + (h.P >> 4);
  const uint32_t sh = 2u * (uint32_t)(h.P & 15);
  const uint32_t X0 = cw[0], X1 = cw[1], X2 = cw[2], X3 = cw[3];
  h.Y[0] = __builtin_amdgcn_alignbit(X1, X0, sh);
  h.Y[1] = __builtin_amdgcn_alignbit(X2, X1, sh);
  h.Y[2] = __builtin_amdgcn_alignbit(X3, X2, sh);
  return h;
}

// Residue bytes of a fetched chunk, ascending codons; an all-'-' iteration
// packs each quad in reverse byte order (the reversal is then a renaming).
template <int kMode>
__device__ __forceinline__ void orf_residues(const OrfChunk& h, const uint8_t* tbl, uint32_t o[4]) {
  const uint8_t* const tb = kMode == 2 ? tbl + (h.minus ? 128 : 0) : tbl + (kMode == 1 ? 128 : 0);
  uint32_t c[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int ob = 6 * k;
    c[k] = ((ob & 31) <= 26 ? (h.Y[ob >> 5] >> (ob & 31))
                            : __builtin_amdgcn_alignbit(h.Y[(ob >> 5) + 1], h.Y[ob >> 5], ob & 31)) &
           63u;
  }
#pragma unroll
  for (int s4 = 0; s4 < 4; ++s4) {
    constexpr int k0 = kMode == 1 ? 3 : 0, k1 = kMode == 1 ? 2 : 1;
    const uint32_t lo = (uint32_t)tb[c[4 * s4 + k0]] | ((uint32_t)tb[c[4 * s4 + k1]] << 8);
    const uint32_t hi = (uint32_t)tb[c[4 * s4 + 3 - k1]] | ((uint32_t)tb[c[4 * s4 + 3 - k0]] << 8);
    o[s4] = __builtin_amdgcn_perm(hi, lo, 0x05040100u);
  }
}

// Codons with a non-ACGT base (any of invalid bits 3k .. 3k+2) become 'X'.
template <int kMode>
__device__ __forceinline__ void orf_patch(const OrfChunk& h, const uint32_t* inv32, uint32_t o[4]) {
  const uint32_t* const iw = inv32 + (h.P >> 5);
  const uint32_t s1 = (uint32_t)(h.P & 31);
  const uint32_t I0 = iw[0], I1 = iw[1], I2 = iw[2];
  const uint32_t Z0 = __builtin_amdgcn_alignbit(I1, I0, s1);
  const uint32_t Z1 = __builtin_amdgcn_alignbit(I2, I1, s1);
  const uint32_t A = Z0 | __builtin_amdgcn_alignbit(Z1, Z0, 1) | __builtin_amdgcn_alignbit(Z1, Z0, 2);
  const uint32_t B = Z1 | (Z1 >> 1) | (Z1 >> 2);
  const uint32_t bad0 = A & 0x49249249u;  // codons 0..10 (bits 3k)
  const uint32_t bad1 = B & 0x00002492u;  // codons 11..15 (bits 3k - 32)
  const uint32_t f[4] = {bad0 & 0xFFFu, (bad0 >> 12) & 0xFFFu,
                         ((bad0 >> 24) | (bad1 << 8)) & 0xFFFu, (bad1 >> 4) & 0xFFFu};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    // bits 0,3,6,9 -> bytes 0..3 of word j; byte-reversed where the quads
    // were packed reversed
    uint32_t m = ((f[j] * 0x8421u) & 0x01010101u) * 0xFFu;
    if constexpr (kMode == 1) m = __builtin_amdgcn_perm(0u, m, 0x00010203u);
    o[j] = (o[j] & ~m) | (0x58585858u & m);
  }
}

template <int kMode>
__device__ __forceinline__ void orf_store(const Orf6Args& a, const OrfChunk& h, uint32_t o[4]) {
  if constexpr (kMode == 1) {  // bytes already reversed: reverse the words
    uint32_t t = o[0];
    o[0] = o[3];
    o[3] = t;
    t = o[1];
    o[1] = o[2];
    o[2] = t;
  } else if (kMode == 2) {
    const uint32_t r0 = __builtin_amdgcn_perm(0u, o[3], 0x00010203u);
    const uint32_t r1 = __builtin_amdgcn_perm(0u, o[2], 0x00010203u);
    const uint32_t r2 = __builtin_amdgcn_perm(0u, o[1], 0x00010203u);
    const uint32_t r3 = __builtin_amdgcn_perm(0u, o[0], 0x00010203u);
    o[0] = h.minus ? r0 : o[0];
    o[1] = h.minus ? r1 : o[1];
    o[2] = h.minus ? r2 : o[2];
    o[3] = h.minus ? r3 : o[3];
  }
  // stream end: the padding bytes are zero
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t drop = (uint32_t)min(max(4 * j + 4 - h.rem, 0), 4);  // bytes of word j
    o[j] &= (uint32_t)(0xFFFFFFFFull >> (8 * drop));
  }
  *reinterpret_cast<uint4*>(a.out + h.dst) = make_uint4(o[0], o[1], o[2], o[3]);
}

template <int kMode>
__device__ __forceinline__ void orf_chunks(const Orf6Args& a, const uint32_t* codes,
                                           const uint32_t* inv32, bool tile_inv,
                                           const uint8_t* tbl, const OrfSeg* seg,
                                           const uint32_t* bm, const uint32_t* pre, uint32_t q,
                                           uint32_t n_chunks) {
  if (q >= n_chunks) return;
  const OrfChunk h = orf_fetch<kMode>(codes, seg, bm, pre, q);
  uint32_t o[4];
  orf_residues<kMode>(h, tbl, o);
  if (tile_inv) orf_patch<kMode>(h, inv32, o);
  orf_store<kMode>(a, h, o);
}

// kGenome = false: the records are bytes in a.nuc (Sequence.get_orfs batch).
// kGenome = true:  the records are gathered from the genome's nibble plane
//                  through the plan's intervals (a.rows), never written out
//                  as nucleotides (C5: extraction fused with translation).
template <bool kGenome>
__global__ __launch_bounds__(kOpsThreads, 6) void orf6_kernel(Orf6Args a) {
  // residue of cidx: [0,128) '+', [128,256) '-'.  Every wave writes the
  // whole (identical) table and then reads only what it wrote itself, so no
  // workgroup barrier (and no wait for the table load) precedes staging, and
  // the table's fixed address folds into the LDS immediates.
  __shared__ uint32_t s_tblw[64];
  __shared__ uint8_t s_code[256];  // byte -> 2-bit code, or 0x40 when not ACGTacgt
  // staged codes (the histogram counters and the vector -> interval map
  // first) and invalid bits, behind their guards (orf_chunks)
  __shared__ __attribute__((aligned(16))) uint32_t
      s_codes[kOpsThreads / 64][kCodeGuard + kOrfVecs + 8];
  __shared__ __attribute__((aligned(16))) uint16_t
      s_inv[kOpsThreads / 64][kInvGuard + kOrfVecs + 8];
  // per wave: the staging window's interval rows, then (same bytes) the
  // segment table and the chunk bitmap with its prefix counts
  constexpr int kScratch = 2 * (kOrf6RowCap + 1);
  static_assert(kScratch * 8 >= kOrfSegs * 16 + 2 * kOrfRankWords * 4, "scratch too small");
  __shared__ uint64_t s_scratch[kOpsThreads / 64][kScratch];
  // wave-uniform (scalar) tile index: the tile's bounds and offsets are
  // scalar loads and their 64-bit arithmetic runs on the SALU
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (!kGenome) {
    const uint32_t c = code_of(threadIdx.x);
    s_code[threadIdx.x] = (uint8_t)(c < 4 ? c : 0x40u);
    __syncthreads();
  }
  // Tile order = block order, dealt round-robin to the 8 XCDs by the hardware.
  // Since the record blocks are laid out in walk order (magot_plan_orf6), all
  // XCDs then advance together through one stretch of the output.  Before that
  // layout, one contiguous run of tiles per XCD merged the partial lines two
  // tiles share in one L2 (WRITE_SIZE 5.26 -> 5.06 GB, C5 1.72 -> 1.65 ms); with
  // it, round-robin is 1 % faster than contiguous runs (1.406 / 1.408 / 1.406 vs
  // 1.420 / 1.422 / 1.422 ms) and than runs of 16 or 256 blocks (1.416-1.418 ms,
  // profiles/r04n/).
  const uint32_t vb = blockIdx.x;
  const uint64_t tile = (uint64_t)vb * (kOpsThreads / 64) + wave;
  if (tile >= a.n_tiles) return;  // wave-uniform
  s_tblw[lane] = reinterpret_cast<const uint32_t*>(a.tables)[lane];
  const uint8_t* const s_tbl = reinterpret_cast<const uint8_t*>(s_tblw);
  const uint64_t T0 = a.tile_t0[tile], T1 = a.tile_t0[tile + 1];
  const uint64_t W0 = (T0 >= 48 ? T0 - 48 : 0) & ~15ull;
  const uint64_t WE = min(T1 + 50, a.total);
  const uint32_t nvec = (uint32_t)((WE - W0 + 15) / 16);
  constexpr int kPer = kOrfVecs / 64;
  // lanes [0, 30): the '-' streams of the batch's 10 records, [30, 60): the
  // '+' streams, so the chunks of each strand are contiguous in q and most
  // chunk iterations are strand-uniform
  const uint32_t my_k = (uint32_t)(lane < kOrfSegs / 2 ? lane : lane - kOrfSegs / 2);
  const uint32_t my_rec = my_k / 3u, my_f = my_k % 3u;
  const bool my_plus = lane >= kOrfSegs / 2;
  // the first record batch's offsets, in flight with the staging loads
  // (unconditional clamped loads: a branch here would wait for them before
  // the staging loads are issued)
  uint64_t rb = a.tile_r0[tile];
  const uint64_t rr0 = min(rb + my_rec, a.n_rec - 1);
  const uint64_t nb_first = a.noff[rr0], ne_first = a.noff[rr0 + 1];
  uint64_t nb = 0, L = 0;
  bool rec = false;
  uint32_t* const codes = s_codes[wave] + kCodeGuard;
  uint16_t* const inv16 = s_inv[wave] + kInvGuard;
  bool any_inv = false;  // this lane staged a non-ACGT base
  if (!kGenome) {
    // raw bytes: all loads in flight at once, then 2-bit codes and invalid
    // bits per 16-byte vector
    uint4 v[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const uint32_t t = min((uint32_t)(lane + 64 * k), nvec - 1);
      v[k] = *reinterpret_cast<const uint4*>(a.nuc + W0 + 16 * (uint64_t)t);
    }
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const uint32_t w[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
      uint32_t cd = 0, bad = 0;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const uint32_t e = s_code[(w[j >> 2] >> (8 * (j & 3))) & 0xFFu];
        cd |= (e & 3u) << (2 * j);
        bad |= (e >> 6) << j;
      }
      codes[lane + 64 * k] = cd;
      inv16[lane + 64 * k] = (uint16_t)bad;
      any_inv |= bad != 0;
    }
  } else {
    // the window's intervals (<= kOrf6RowCap, host-planned), rebased once to
    // the window so that the per-vector math is 32-bit: {byte offset of the
    // plane word holding window position 0 (mod 2^32: only positions inside
    // the interval are read), 4 * nibble shift, window-relative start}
    uint4* const row = reinterpret_cast<uint4*>(s_scratch[wave]);
    uint32_t* const cnt = codes;  // 256 counters, then the vector -> interval map
    const uint64_t e0 = a.tile_e0[tile];
    const uint32_t mrow = a.tile_m[tile];
    const int32_t wlen = (int32_t)(WE - W0);
    int32_t rel[2];
    bool in[2];
    ulonglong2 rw[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      // rows e0 .. e0 + m (the window's intervals, then the first one past
      // its end); the other lanes load row m again, so a wave fetches the
      // lines of its ~30 rows instead of 128 rows (sentinel row n_rows)
      const uint64_t j = min(e0 + min((uint32_t)(lane + 64 * h), mrow), a.n_rows);
      rw[h] = *reinterpret_cast<const ulonglong2*>(a.rows + 2 * j);
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint32_t jj = lane + 64 * h;
      const uint64_t A = rw[h].x + W0;  // unified base of window position 0
      const uint64_t st = rw[h].y & ~kOrf6ExcRow;
      const int64_t rs = (int64_t)(st - W0);
      rel[h] = (int32_t)max(min(rs, (int64_t)(1 << 30)), -(int64_t)(1 << 30));
      in[h] = jj <= kOrf6RowCap && st < WE;
      // {code-plane byte offset of the word holding window position 0,
      //  A & 31 | exception flag << 5, window-relative start,
      //  exception-plane byte offset of the word holding window position 0}
      if (jj <= kOrf6RowCap)
        row[jj] = make_uint4((uint32_t)(A >> 4) << 2,
                             (uint32_t)(A & 31u) | ((rw[h].y & kOrf6ExcRow) ? 32u : 0u),
                             (uint32_t)rel[h], (uint32_t)(A >> 5) << 2);
    }
#pragma unroll
    for (int i = 0; i < kPer; ++i) cnt[kPer * lane + i] = 0u;  // vectors kPer lane .. + kPer-1
    const uint32_t m = (uint32_t)(__popcll(__ballot(in[0])) + __popcll(__ballot(in[1])));
    __builtin_amdgcn_wave_barrier();
    // first interval of every vector: count interval starts per vector
    // (a start in (16v - 16, 16v] counts at vector v), then prefix sums
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (in[h]) {
        const int32_t v = rel[h] <= 0 ? 0 : (rel[h] + 15) >> 4;
        if (v < kOrfVecs) atomicAdd(&cnt[v], 1u);
      }
    }
    __builtin_amdgcn_wave_barrier();
    {
      uint32_t c[kPer];  // running counts of vectors kPer lane .. + kPer-1
#pragma unroll
      for (int i = 0; i < kPer; ++i) c[i] = cnt[kPer * lane + i] + (i ? c[i - 1] : 0u);
      const uint32_t x = wave_scan(c[kPer - 1]);
      const uint32_t base = x - c[kPer - 1] - 1;
#pragma unroll
      for (int i = 0; i < kPer; ++i) cnt[kPer * lane + i] = base + c[i];
    }
    __builtin_amdgcn_wave_barrier();
    // Codon indices straight from the 2-bit code plane: translation ignores
    // case, so a vector needs only the codes of its 16 positions and of the
    // next two, plus, where an interval touches an exception run (flagged by
    // the host), the exception bits of those positions (1 bit per base).
    // Fast path: the 18 positions span at most two intervals, and every
    // window of all four vectors is in flight at once (one memory round
    // trip).  A window that is not needed (no second interval, interval not
    // flagged) is read from past the plane's end, which the buffer range
    // check answers with zeros and no memory request.
    const __amdgpu_buffer_rsrc_t plane2 = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint32_t*>(a.code2), (short)0,
        (int)(uint32_t)min(a.code2_words * 4, (uint64_t)0xFFFFFFFFu), 0x00020000);
    const __amdgpu_buffer_rsrc_t plane1 = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint32_t*>(a.exc1), (short)0,
        (int)(uint32_t)min(a.exc1_words * 4, (uint64_t)0xFFFFFFFFu), 0x00020000);
    uint32_t iv[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) iv[k] = min(cnt[lane + 64 * k], m - 1);
    uint32_t wa[kPer][2], wb[kPer][2], xa[kPer][2], xb[kPer][2];
    // Windows without a flagged interval (most) skip the exception plane:
    // no loads, no address math, no merge (wave-uniform).
    // (the 64-bit ballot is tested before readfirstlane, which takes 32 bits:
    // testing after it dropped rows 32-63 and 96-127, and a window whose only
    // flagged interval sat there decoded its exceptions as 'A')
    const bool wexc = __builtin_amdgcn_readfirstlane(
                          __ballot((in[0] && (rw[0].y & kOrf6ExcRow)) ||
                                   (in[1] && (rw[1].y & kOrf6ExcRow))) != 0);
    auto issue = [&](auto exc_tag) {
      constexpr bool kExc = decltype(exc_tag)::value;
#pragma unroll
      for (int k = 0; k < kPer; ++k) {
        const uint32_t t = lane + 64 * k;
        const int32_t t16 = 16 * (int32_t)t;
        const uint4 r0 = row[iv[k]], r1 = row[iv[k] + 1];
        const bool cross = (int32_t)r1.z < min(t16 + 16, wlen);
        const auto va = __builtin_amdgcn_raw_buffer_load_b64(plane2, r0.x + 4u * t, 0, 0);
        const auto vb =
            __builtin_amdgcn_raw_buffer_load_b64(plane2, cross ? r1.x + 4u * t : 0xFFFFFFF0u, 0, 0);
#pragma unroll
        for (int d = 0; d < 2; ++d) {
          wa[k][d] = va[d];
          wb[k][d] = vb[d];
        }
        if constexpr (kExc) {
          const uint32_t ea = r0.w + 4u * (((r0.y & 31u) + 16u * t) >> 5);
          const uint32_t eb = r1.w + 4u * (((r1.y & 31u) + 16u * t) >> 5);
          const auto ua =
              __builtin_amdgcn_raw_buffer_load_b64(plane1, (r0.y & 32u) ? ea : 0xFFFFFFF0u, 0, 0);
          const auto ub = __builtin_amdgcn_raw_buffer_load_b64(
              plane1, (cross && (r1.y & 32u)) ? eb : 0xFFFFFFF0u, 0, 0);
          xa[k][0] = ua[0];
          xa[k][1] = ua[1];
          xb[k][0] = ub[0];
          xb[k][1] = ub[1];
        } else {
          xa[k][0] = xa[k][1] = xb[k][0] = xb[k][1] = 0u;
        }
      }
    };
    if (wexc) issue(std::true_type{});
    else issue(std::false_type{});
    __builtin_amdgcn_sched_barrier(0);  // every window load is issued before the first is consumed
    uint32_t exact = 0;  // bit k: vector k takes the exact path below
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const uint32_t t = lane + 64 * k;
      const int32_t t16 = 16 * (int32_t)t;
      const int32_t et = min(t16 + 16, wlen);
      const uint4 r0 = row[iv[k]], r1 = row[iv[k] + 1];  // re-read: fewer live registers
      const bool cross = (int32_t)r1.z < et;
      // positions [j0, 16) come from the second interval (none: j0 = 32)
      const uint32_t j0 = cross ? (uint32_t)((int32_t)r1.z - t16) : 32u;
      const uint32_t mb = j0 >= 16 ? 0u : ~0u << (2 * j0);
      const uint32_t sa = 2u * (r0.y & 15u), sb = 2u * (r1.y & 15u);
      const uint32_t x0 = funnel4(wa[k][1], wa[k][0], sa);
      const uint32_t b0 = funnel4(wb[k][1], wb[k][0], sb);
      const uint32_t y0 = (b0 & mb) | (x0 & ~mb);  // codes of positions 0..15
      if (cross && (int32_t)row[iv[k] + 2].z < et) exact |= 1u << k;
      // exception bits of positions 0..15: bit j set = base j not ACGTacgt
      uint32_t ex = 0;
      if (wexc) {
        const uint32_t ma = j0 >= 32 ? 0u : ~0u << j0;
        const uint32_t va = funnel4(xa[k][1], xa[k][0], ((r0.y & 31u) + 16u * t) & 31u);
        const uint32_t vb = funnel4(xb[k][1], xb[k][0], ((r1.y & 31u) + 16u * t) & 31u);
        ex = (vb & ma) | (va & ~ma);
      }
      codes[t] = y0;
      inv16[t] = (uint16_t)ex;
      any_inv |= (ex & 0xFFFFu) != 0;
    }
    if (__builtin_amdgcn_readfirstlane(__ballot(exact != 0) != 0)) {
      // Exact path (rare): vectors over three or more intervals rebuild their
      // 16 positions from the nibble plane, interval by interval.
      const __amdgpu_buffer_rsrc_t plane = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<uint32_t*>(a.nib), (short)0,
          (int)(uint32_t)min(a.nib_words * 4, (uint64_t)0xFFFFFFFFu), 0x00020000);
#pragma unroll 1
      for (int k = 0; k < kPer; ++k) {
        if (!((exact >> k) & 1u)) continue;
        const uint32_t t = lane + 64 * k;
        const int32_t t16 = 16 * (int32_t)t;
        const int32_t et = min(t16 + 16, wlen);
        uint32_t x[2] = {0u, 0u};  // nibbles of positions 0..15
        uint32_t i = iv[k];
        int32_t pos = t16;
        while (pos < et) {
          const uint4 r = row[i];
          const int32_t nxt = min((int32_t)row[i + 1].z, et);
          // nibble-plane byte offset of the word holding window position 0
          const uint32_t nboff = 2u * r.x + 4u * ((r.y >> 3) & 1u);
          const uint32_t sh = 4u * (r.y & 7u);
          const auto w = __builtin_amdgcn_raw_buffer_load_b96(plane, nboff + 8u * t, 0, 0);
          const uint32_t c[2] = {funnel4(w[1], w[0], sh), funnel4(w[2], w[1], sh)};
          const int32_t j = pos - t16, n = nxt - pos;
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const int32_t lo = max(j - 8 * q, 0), hi = min(j + n - 8 * q, 8);
            if (lo < hi) {
              const uint32_t mh = hi >= 8 ? ~0u : (1u << (4 * hi)) - 1u;
              const uint32_t ml = (1u << (4 * lo)) - 1u;
              const uint32_t msk = mh & ~ml;
              x[q] = (c[q] & msk) | (x[q] & ~msk);
            }
          }
          pos = nxt;
          ++i;
        }
        codes[t] = nib_codes(x[0], x[1]);
        const uint32_t bad = nib_exc16(x[0], x[1]);
        inv16[t] = (uint16_t)bad;
        any_inv |= bad != 0;
      }
    }
  }
  // guards and tail: defined words around the staged positions
  if (lane < kCodeGuard) s_codes[wave][lane] = 0u;
  if (lane < kInvGuard) s_inv[wave][lane] = 0u;
  if (lane < 8) {
    codes[kOrfVecs + lane] = 0u;
    inv16[kOrfVecs + lane] = 0u;
  }
  const bool tile_inv = __builtin_amdgcn_readfirstlane(__ballot(any_inv) != 0);
  const uint32_t* const inv32 = reinterpret_cast<const uint32_t*>(s_inv[wave] + kInvGuard);

  OrfSeg* const seg = reinterpret_cast<OrfSeg*>(s_scratch[wave]);
  uint32_t* const bm = reinterpret_cast<uint32_t*>(s_scratch[wave] + 2 * kOrfSegs);
  uint32_t* const pre = bm + kOrfRankWords;
  bool first_batch = !kGenome;
  for (;; rb += kOrfBatch) {
    // ---- the batch's segments: one (record, stream) per lane
    const uint64_t r = rb + my_rec;
    rec = lane < kOrfSegs && r < a.n_rec;
    if (!first_batch) {
      nb = rec ? a.noff[r] : 0;
      L = rec ? a.noff[r + 1] - nb : 0;
    } else {  // raw bytes: the offsets loaded with the staging loads
      nb = rec ? nb_first : 0;
      L = rec ? ne_first - nb_first : 0;
    }
    const uint64_t nres = rec && nb < T1 ? orf_count(L, my_f) : 0;
    uint64_t lo = 0, hi = 0;
    if (nres) {
      if (my_plus) {  // '+': chunk c's first codon starts at x0 + 48c
        const uint64_t x0 = nb + 2 * my_f;
        lo = T0 > x0 ? div48(T0 - x0 + 47) : 0;
        hi = T1 > x0 ? div48(T1 - x0 + 47) : 0;
      } else {  // '-': chunk c's first codon (read backwards) lies at x0 - 48c
        const uint64_t x0 = nb + L - 3 - 2 * my_f;
        lo = x0 >= T1 ? div48(x0 - T1) + 1 : 0;
        hi = x0 >= T0 ? div48(x0 - T0) + 1 : 0;
      }
      hi = min(hi, (nres + 15) / 16);
      lo = min(lo, hi);
    }
    const uint32_t cnt = (uint32_t)(hi - lo);
    // wave-inclusive scans of chunk starts (low half: a batch owns < 1024
    // chunks, see kOrfRankWords) and compacted segment slots (high half), one
    // DPP scan for both
    const uint32_t sc = wave_scan(cnt | (cnt != 0 ? 1u << 16 : 0u));
    const uint32_t incl = sc & 0xFFFFu, incl_s = sc >> 16;
    const uint32_t n_chunks = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    // '-' chunks come first
    const uint32_t n_minus = (uint32_t)__builtin_amdgcn_readlane((int)incl, kOrfSegs / 2 - 1);
    // does the next batch still start inside the tile?
    const bool more = __builtin_amdgcn_readlane((int)(rec && nb + L < T1), kOrfSegs - 1) != 0 &&
                      rb + kOrfBatch < a.n_rec;
    bm[lane] = 0u;
    bm[lane + 64] = 0u;
    __builtin_amdgcn_wave_barrier();
    if (cnt) {
      const uint32_t start = incl - cnt;
      const int64_t p = my_plus ? (int64_t)(nb + 2 * my_f + 48 * lo)
                                : (int64_t)(nb + L - 3 - 2 * my_f - 48 * lo);
      OrfSeg g;
      // the stream's place in the record's block (magot_orf6_sizes): strand-
      // major, each of the three frames padded to 16 bytes
      const uint64_t p0 = (orf_count(L, 0) + 15) & ~15ull, p1 = (orf_count(L, 1) + 15) & ~15ull;
      const uint64_t p2 = (orf_count(L, 2) + 15) & ~15ull;
      const uint64_t within = (my_plus ? p0 + p1 + p2 : 0) + (my_f >= 1 ? p0 : 0) +
                              (my_f >= 2 ? p1 : 0);
      g.out0 = a.boff[r] + within + 16 * lo - 16 * (uint64_t)start;
      g.p0 = (int32_t)(p - (int64_t)W0 + (my_plus ? -48 : 48) * (int64_t)start);
      const int32_t rem = (int32_t)(nres - 16 * lo) + 16 * (int32_t)start;
      g.rem0 = my_plus ? rem : -rem;
      seg[incl_s - 1] = g;
      atomicOr(&bm[start >> 5], 1u << (start & 31));
    }
    __builtin_amdgcn_wave_barrier();
    {  // pre[w] = segment starts in words before w
      const uint32_t x0 = __popc(bm[2 * lane]), x1 = __popc(bm[2 * lane + 1]);
      const uint32_t x = wave_scan(x0 + x1);
      pre[2 * lane] = x - x0 - x1;
      pre[2 * lane + 1] = x - x1;
    }
    __builtin_amdgcn_wave_barrier();
    // ---- the batch's chunks, 64 at a time
    for (uint32_t q0 = 0; q0 < n_chunks; q0 += 64) {
      const uint32_t q = q0 + lane;
      if (q0 + 64 <= n_minus)
        orf_chunks<1>(a, codes, inv32, tile_inv, s_tbl, seg, bm, pre, q, n_chunks);
      else if (q0 >= n_minus)
        orf_chunks<0>(a, codes, inv32, tile_inv, s_tbl, seg, bm, pre, q, n_chunks);
      else
        orf_chunks<2>(a, codes, inv32, tile_inv, s_tbl, seg, bm, pre, q, n_chunks);
    }
    if (!more) break;
    first_batch = false;
    __builtin_amdgcn_wave_barrier();  // segment tables are rewritten
  }
}

// 2-bit code plane: word w = codes of unified bases 16w .. 16w+15 (nibble
// words 2w, 2w+1), base k at bits 2k.  Exception bases (code bits 0 in the
// nibble plane) become 'A'; the orf6 rows flag their intervals.
__global__ __launch_bounds__(256) void code2_kernel(const uint32_t* __restrict__ nib,
                                                    uint64_t n_words, uint32_t* __restrict__ code2) {
  const uint64_t w = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (w >= n_words) return;
  const uint2 x = reinterpret_cast<const uint2*>(nib)[w];
  // per byte: code(2k) | code(2k+1) << 2 in the low nibble, then four codes
  // in bytes 0 and 2
  const uint32_t y0 = (x.x & 0x03030303u) | ((x.x >> 2) & 0x0C0C0C0Cu);
  const uint32_t y1 = (x.y & 0x03030303u) | ((x.y >> 2) & 0x0C0C0C0Cu);
  const uint32_t z0 = (y0 & 0x0F0F0F0Fu) | ((y0 >> 4) & 0xF0F0F0F0u);
  const uint32_t z1 = (y1 & 0x0F0F0F0Fu) | ((y1 >> 4) & 0xF0F0F0F0u);
  code2[w] = __builtin_amdgcn_perm(z1, z0, 0x06040200u);
}

// Exception-bit plane: word w = bit 3 of the nibbles of unified bases 32w ..
// 32w+31 (nibble words 4w .. 4w+3), base k at bit k.
__global__ __launch_bounds__(256) void exc1_kernel(const uint32_t* __restrict__ nib,
                                                   uint64_t n_words, uint32_t* __restrict__ exc1) {
  const uint64_t w = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (w >= n_words) return;
  const uint4 x = reinterpret_cast<const uint4*>(nib)[w];
  const uint32_t v[4] = {x.x, x.y, x.z, x.w};
  uint32_t out = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint32_t y = (v[q] >> 3) & 0x11111111u;  // bits 0, 4, .., 28
    y = (y | (y >> 3)) & 0x03030303u;        // two per byte
    y = (y | (y >> 6)) & 0x000F000Fu;        // four per half
    y = (y | (y >> 12)) & 0xFFu;             // eight
    out |= y << (8 * q);
  }
  exc1[w] = out;
}

}  // namespace

void launch_exc1(const uint32_t* nib, uint64_t nib_words, uint32_t* exc1, hipStream_t s) {
  const uint64_t n = nib_words / 4;
  if (n == 0) return;
  hipLaunchKernelGGL(exc1_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, nib, n, exc1);
}

void launch_code2(const uint32_t* nib, uint64_t nib_words, uint32_t* code2, hipStream_t s) {
  const uint64_t n = nib_words / 2;
  if (n == 0) return;
  hipLaunchKernelGGL(code2_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, nib, n,
                     code2);
}

void orf6_tables(const uint8_t lut64[64], uint8_t out[256]) {
  // '+': cidx = c0 | c1 << 2 | c2 << 4 indexes the library directly;
  // '-': the codon is read backwards and complemented: c2' c1' c0'.
  for (uint32_t x = 0; x < 128; ++x) {
    const uint32_t c0 = x & 3u, c1 = (x >> 2) & 3u, c2 = (x >> 4) & 3u;
    const bool bad = (x >> 6) & 1u;
    out[x] = bad ? (uint8_t)'X' : lut64[x & 63u];
    out[128 + x] = bad ? (uint8_t)'X' : lut64[((3u - c2) | ((3u - c1) << 2) | ((3u - c0) << 4))];
  }
}

void orf6_plan_tiles(const uint64_t* noff, uint64_t n_rec, const uint64_t* row_start,
                     uint64_t n_rows, Orf6Tiles* out) {
  const uint64_t total = n_rec ? noff[n_rec] : 0;
  out->t0.clear();
  out->r0.clear();
  out->e0.clear();
  out->m.clear();
  uint64_t r = 0, e = 0, f = 0;
  for (uint64_t T = 0; T < total;) {
    const uint64_t W0 = (T >= 48 ? T - 48 : 0) & ~15ull;
    while (r + 1 < n_rec && noff[r + 1] <= T) ++r;  // the record holding base T
    uint64_t T1 = std::min(T + kOrfTile, total);
    if (row_start) {
      while (e + 1 < n_rows && row_start[e + 1] <= W0) ++e;  // the interval holding W0
      // at most kOrf6RowCap intervals may start before the staged window ends
      if (e + kOrf6RowCap < n_rows) {
        const uint64_t cap = row_start[e + kOrf6RowCap];
        if (T1 + 50 > cap) T1 = std::max(T + 1, cap - 50);
      }
      out->e0.push_back((uint32_t)e);
      // the window's rows: intervals starting before its end (the kernel
      // loads rows e .. e + m, the last one the sentinel)
      const uint64_t WE = std::min(T1 + 50, total);
      f = std::max(f, e);
      while (f < n_rows && row_start[f] < WE) ++f;
      out->m.push_back((uint32_t)std::min<uint64_t>(f - e, kOrf6RowCap));
    }
    out->t0.push_back(T);
    out->r0.push_back((uint32_t)r);
    T = T1;
  }
  out->t0.push_back(total);
}

constexpr int kOrf6BlocksPerCu = 7;

void launch_orf6(const Orf6Args& a, bool genome, hipStream_t s) {
  if (a.n_tiles == 0) return;
  const uint64_t blocks = (a.n_tiles + kOpsThreads / 64 - 1) / (kOpsThreads / 64);
  if (genome) {
    // Blocks per CU.  With codes staged (14.6 KB LDS, 52 VGPRs) 8 blocks fit;
    // 7 measured best: 1.4825 / 1.4839 / 1.4799 ms per C5 step against 1.508 /
    // 1.5071 / 1.5091 uncapped and 1.4868 / 1.488 / 1.4898 at 6 (one box,
    // alternating runs; the sweep override: scripts/experiments/occupancy_knobs.patch).
    static const size_t pad = occupancy_lds_pad(reinterpret_cast<const void*>(orf6_kernel<true>),
                                                kOpsThreads, kOrf6BlocksPerCu);
    hipLaunchKernelGGL(orf6_kernel<true>, dim3((uint32_t)blocks), dim3(kOpsThreads), pad, s, a);
  } else
    hipLaunchKernelGGL(orf6_kernel<false>, dim3((uint32_t)blocks), dim3(kOpsThreads), 0, s, a);
}

void launch_revcomp(const uint8_t* in, const uint64_t* off, uint64_t n, uint64_t total,
                    uint8_t* out, hipStream_t s) {
  if (total == 0) return;
  const uint64_t chunks = (total + 15) / 16;
  const uint64_t blocks = (chunks + kOpsThreads - 1) / kOpsThreads;
  hipLaunchKernelGGL(revcomp_kernel, dim3((uint32_t)blocks), dim3(kOpsThreads), 0, s, in, off, n,
                     total, out);
}

// Codon symbols over an extended alphabet (Sequence.translate with an
// arbitrary `library`, genome.py:795-818): byte -> class through a 256-entry
// table (upper-case folding and every character of the library's 3-char keys
// included), codon index c0 + K*c1 + K*K*c2, symbol = lut[index].  One lane
// per codon; the table and the LUT are staged in LDS by each block.
__global__ __launch_bounds__(256) void codon_symbols_kernel(const uint8_t* __restrict__ in,
                                                            uint64_t n_codons,
                                                            const uint8_t* __restrict__ cls,
                                                            uint32_t K,
                                                            const uint8_t* __restrict__ lut,
                                                            uint8_t* __restrict__ out) {
  __shared__ uint8_t s_cls[256];
  __shared__ uint8_t s_lut[kMaxSymbolLut];
  s_cls[threadIdx.x] = cls[threadIdx.x];
  const uint32_t nl = K * K * K;
  for (uint32_t i = threadIdx.x; i < nl; i += 256) s_lut[i] = lut[i];
  __syncthreads();
  const uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (k >= n_codons) return;
  const uint8_t* p = in + 3 * k;
  const uint32_t x = s_cls[p[0]] + K * (s_cls[p[1]] + K * s_cls[p[2]]);
  out[k] = s_lut[x];
}

void launch_translate(const uint8_t* in, const uint64_t* off, uint64_t n, const int32_t* frames,
                      const uint8_t* strands, const uint64_t* pep_off, uint64_t total_pep,
                      const uint32_t* lut16, uint8_t* out, hipStream_t s) {
  if (total_pep == 0) return;
  TranslateLut lut;
  for (int i = 0; i < 16; ++i) lut.w[i] = lut16[i];
  const uint64_t chunks = (total_pep + 15) / 16;
  const uint64_t blocks = (chunks + kOpsThreads - 1) / kOpsThreads;
  hipLaunchKernelGGL(translate_kernel, dim3((uint32_t)blocks), dim3(kOpsThreads), 0, s, in, off, n,
                     frames, strands, pep_off, total_pep, lut, out);
}

void launch_codon_symbols(const uint8_t* in, uint64_t n_codons, const uint8_t* cls, uint32_t K,
                          const uint8_t* lut, uint8_t* out, hipStream_t s) {
  if (n_codons == 0) return;
  const uint64_t blocks = (n_codons + 255) / 256;
  hipLaunchKernelGGL(codon_symbols_kernel, dim3((uint32_t)blocks), dim3(256), 0, s, in, n_codons,
                     cls, K, lut, out);
}

}  // namespace magot
