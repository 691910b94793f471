// Fused gather + reverse-complement + translate kernel for gfx950 (MI355X).
//
// Semantics restated from the reference's per-record loop:
//   BaseAnnotation.get_seq      genome.py:603-614  (slice, '-' => revcomp)
//   Sequence.reverse_compliment genome.py:784-793  (a<->t g<->c, n N - kept, else 'n')
//   ParentAnnotation.get_fasta  genome.py:686-707  (children joined in output order)
//   Sequence.translate          genome.py:795-822  (frame 0, upper-cased codons,
//                                                    unknown => 'X')
// The Python layer has already resolved child order, duplicate-coordinate
// collapse and slice clamping into an interval table (plan); this kernel only
// moves bytes.
//
// Work decomposition (output-stationary, HBM-bound):
//   * The host cuts the concatenated nucleotide output into 16-byte aligned
//     tiles of <= tile_bytes(LC) bytes, LC = the chunk slots per lane the plan
//     was cut for (6: 6096 bytes = 381 chunks of 16 for large plans; 3: 3024
//     bytes for translating plans under kSmallTilePlan tiles; shorter where a
//     tile would touch more than kExonCap intervals or kTxCap records).  A
//     tile belongs to ONE wavefront: 64 lanes x LC chunk slots (the tile's
//     chunks + a 3-chunk halo for codons that run past the tile end) and 1-2
//     residue chunks per lane, so there is no workgroup barrier (every wave
//     writes its own copy of the codon table).
//   * Staging: the tile's intervals go to wave-private LDS as {64-bit unified
//     anchor, tile-relative end, flags}; chunk -> interval and residue chunk
//     -> record maps come from an LDS histogram + one packed DPP wave scan.
//   * The genome is a nibble plane (code | soft-mask << 2, or 8 | literal
//     class for an exception byte) followed by its reverse-complement mirror,
//     so a '-' interval reads its strand forward exactly like a '+' interval.
//     A chunk is at most two interval segments on the fast path: one
//     buffer_load_dwordx3 window per segment, two funnel shifts, a nibble-mask
//     merge, v_perm nibble spread + v_perm ASCII table (a second table for the
//     literal classes N n - R Y K M when the wave holds exception nibbles),
//     one 16-byte store.  Intervals over a byte without a literal class
//     (flagged per interval by the host) and chunks over 3+ intervals take
//     build_chunk_slow, which patches literals from the run list.
//   * 2-bit codes and validity bits of the tile stay in LDS; a residue chunk
//     funnel-shifts 48 bases of codes out of LDS per record segment (<= 2 on
//     the fast path), looks the 16 codons up in a 64-byte LDS table and
//     stores 16 bytes.
#include "common.h"

namespace magot {
namespace {

constexpr int kGuard = 4;  // LDS words before codes[0] (codons of residue chunk 0 may start < 0)

template <int LC>
struct WaveLds {
  static constexpr int kS = 64 * LC;      // chunk slots
  uint4 ex[kExonCap];                     // {plane byte offset, anchor lo, end (tile-rel), flags}
  uint32_t vb[kExonCap];                  // reverse-forward rows: forward-plane byte offset
  int64_t tn[kTxCap + 1];                 // record codon-0 output position, tile-relative
  int64_t tp[kTxCap + 1];                 // record first residue, relative to the tile's Q0
  uint32_t codes_g[kGuard + kS + 8];      // 2-bit codes per chunk (histogram scratch first)
  uint32_t valid_g[kGuard + (kS > 2 * kPepSlots ? kS : 2 * kPepSlots) / 2 + 8];  // 16 validity
                                          // bits per chunk (residue-chunk histogram first)
  uint8_t cmap[kS];                       // chunk slot -> interval
  uint8_t pmap[kPepSlots];                // residue chunk -> record
};

constexpr uint32_t kFlagRc = 1u;
constexpr uint32_t kFlagExc = 2u;      // touches an exception run
constexpr uint32_t kFlagSlowLit = 4u;  // ... one without a literal class (run-list path)
// '-' interval without exceptions: the fast path reads it from the forward
// plane, descending (vb, shift in bits 13..15), and reverse-complements the
// chunk in registers; its mirror anchor stays for the slow path and for
// chunks whose other segment is not reverse-forward
constexpr uint32_t kFlagRevFwd = 32u;

__device__ __forceinline__ uint32_t funnel(uint32_t hi, uint32_t lo, uint32_t sh) {
  return __builtin_amdgcn_alignbit(hi, lo, sh);  // (hi:lo >> sh)[31:0], sh in 0..31
}

__device__ __forceinline__ uint32_t bfi(uint32_t mask, uint32_t a, uint32_t b) {
  return (a & mask) | (b & ~mask);  // v_bfi_b32 / v_bitop3
}

__device__ __forceinline__ uint32_t spread_bits(uint32_t m4) {
  // four bits -> four bytes 0/1
  const uint32_t x = m4 | (m4 << 7);
  return (x | (x << 14)) & 0x01010101u;
}

__device__ __forceinline__ uint32_t rc_literal(uint32_t b) {
  // genome.py:787,792 for a byte that is not ACGTacgt
  return (b == 'n' || b == 'N' || b == '-') ? b : (uint32_t)'n';
}

// Sixteen output bytes as nibbles (chunk byte k = nibble k of x0:x1), the
// exception bytes among them and their literal values.
struct Chunk {
  uint32_t x0, x1;  // nibbles: code | lower << 2 | exception << 3
  uint32_t exc;     // 16 x "literal byte" bit
  uint32_t lit[4];  // literal bytes, little-endian by chunk byte
};

__device__ __forceinline__ void put_literal(Chunk& o, int ka, int kb, uint32_t byte) {
  const uint32_t n = (uint32_t)(kb - ka + 1);
  const uint32_t bits = ((n >= 32u) ? 0xFFFFFFFFu : ((1u << n) - 1u)) << ka;
  o.exc |= bits;
  const uint32_t rep = byte | (byte << 8) | (byte << 16) | (byte << 24);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t b01 = spread_bits((bits >> (4 * q)) & 0xFu);
    const uint32_t bm = (b01 << 8) - b01;
    o.lit[q] = (o.lit[q] & ~bm) | (rep & bm);
  }
}

// Eight nibbles -> two words of selector bytes (one nibble per byte).
__device__ __forceinline__ void spread_nibbles(uint32_t x, uint32_t& s0, uint32_t& s1) {
  const uint32_t lo = x & 0x0F0F0F0Fu;          // nibbles 0 2 4 6
  const uint32_t hi = (x >> 4) & 0x0F0F0F0Fu;   // nibbles 1 3 5 7
  s0 = __builtin_amdgcn_perm(hi, lo, 0x05010400u);
  s1 = __builtin_amdgcn_perm(hi, lo, 0x07030602u);
}

// 16 bytes of ASCII: selector bit 2 (soft mask) picks the 'acgt' half of the
// table; exception bytes (selector >= 8) are patched from the literal words.
__device__ __forceinline__ uint4 chunk_ascii(uint32_t x0, uint32_t x1, uint32_t exc,
                                             const uint32_t lit[4]) {
  uint32_t s[4];
  spread_nibbles(x0, s[0], s[1]);
  spread_nibbles(x1, s[2], s[3]);
  uint32_t w[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) w[q] = __builtin_amdgcn_perm(0x74676361u, 0x54474341u, s[q]);
  if (exc) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t b01 = spread_bits((exc >> (4 * q)) & 0xFu);
      const uint32_t em = (b01 << 8) - b01;
      w[q] = (w[q] & ~em) | (lit[q] & em);
    }
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// As chunk_ascii, for chunks that may hold exception nibbles (8 | literal
// class): a second 8-entry table gives N n - R Y K M, selected per byte by
// the exception bit.
__device__ __forceinline__ uint4 chunk_ascii_lit(uint32_t x0, uint32_t x1, uint32_t exc,
                                                 const uint32_t lit[4]) {
  uint32_t s[4];
  spread_nibbles(x0, s[0], s[1]);
  spread_nibbles(x1, s[2], s[3]);
  uint32_t w[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t base = __builtin_amdgcn_perm(0x74676361u, 0x54474341u, s[q] & 0x07070707u);
    const uint32_t lits = __builtin_amdgcn_perm(kLitHi, kLitLo, s[q] & 0x07070707u);
    const uint32_t m = ((s[q] >> 3) & 0x01010101u) * 0xFFu;
    w[q] = bfi(m, lits, base);
  }
  if (exc) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t b01 = spread_bits((exc >> (4 * q)) & 0xFu);
      const uint32_t em = (b01 << 8) - b01;
      w[q] = (w[q] & ~em) | (lit[q] & em);
    }
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// The exception bits (nibble bit 3) of 16 nibbles as a 16-bit mask.
__device__ __forceinline__ uint32_t exc_bits(uint32_t x0, uint32_t x1) {
  uint32_t e0 = (x0 >> 3) & 0x11111111u, e1 = (x1 >> 3) & 0x11111111u;
  e0 = (e0 | (e0 >> 3)) & 0x03030303u;
  e1 = (e1 | (e1 >> 3)) & 0x03030303u;
  e0 = (e0 | (e0 >> 6)) & 0x000F000Fu;
  e1 = (e1 | (e1 >> 6)) & 0x000F000Fu;
  e0 = (e0 | (e0 >> 12)) & 0xFFu;
  e1 = (e1 | (e1 >> 12)) & 0xFFu;
  return e0 | (e1 << 8);
}

// 16 nibbles -> 16 packed 2-bit codes (base k at bits 2k) for translation.
__device__ __forceinline__ uint32_t pack_codes(uint32_t x0, uint32_t x1) {
  // per byte: code(2k) | code(2k+1) << 2 in the low nibble (high nibble junk)
  const uint32_t y0 = bfi(0x03030303u, x0, x0 >> 2), y1 = bfi(0x03030303u, x1, x1 >> 2);
  // bytes 0 and 2: four codes each
  const uint32_t z0 = bfi(0x0F0F0F0Fu, y0, y0 >> 4), z1 = bfi(0x0F0F0F0Fu, y1, y1 >> 4);
  return __builtin_amdgcn_perm(z1, z0, 0x06040200u);
}

// Output store: plain for the 128-byte lines a tile shares with its
// neighbours (L2 merges the two tiles' halves of such a line), non-temporal
// elsewhere.  A/B on one box, 200 back-to-back C3 steps: 0.2827 -> 0.2813 ms,
// WRITE_SIZE 0.826 -> 0.823 GB per launch.
__device__ __forceinline__ void store16_edge(uint8_t* dst, uint4 v, bool edge) {
  if (edge)
    *reinterpret_cast<uint4*>(dst) = v;
  else
    store16(dst, v);
}

struct Planes {
  const uint32_t* __restrict__ nib;
  const uint32_t* __restrict__ dir;
  const ExcRun* __restrict__ runs;
  uint64_t span;
};

// Nibbles of the 16 unified bases starting at u.
__device__ __forceinline__ void window(const uint32_t* nib, uint64_t u, uint32_t& x0,
                                       uint32_t& x1) {
  const uint32_t* w = nib + (u >> 3);
  const uint32_t sh = 4u * (uint32_t)(u & 7);
  const uint32_t w0 = w[0], w1 = w[1], w2 = w[2];
  x0 = funnel(w1, w0, sh);
  x1 = funnel(w2, w1, sh);
}

// Patch literal bytes of forward genome interval [glo, ghi] (chunk bytes from j0).
__device__ __forceinline__ void patch_runs(const Planes& a, uint64_t glo, uint64_t ghi, bool rc,
                                           int j0, Chunk& o) {
  const uint32_t d0 = a.dir[glo >> kDirShift];
  const uint32_t d1 = a.dir[ghi >> kDirShift];
  if ((d0 & kDirClean) && (d1 & kDirClean)) return;
  for (uint32_t d = d0 & ~kDirClean;; ++d) {
    const ExcRun r = a.runs[d];
    if (r.start > ghi) break;
    const uint64_t rend = r.start + r.len;
    if (rend > glo) {
      const uint64_t ovl = max(glo, r.start);
      const uint64_t ovh = min(ghi, rend - 1);
      if (!rc) put_literal(o, j0 + (int)(ovl - glo), j0 + (int)(ovh - glo), r.byte);
      else put_literal(o, j0 + (int)(ghi - ovh), j0 + (int)(ghi - ovl), rc_literal(r.byte));
    }
  }
}

// Unified coordinate U of tile byte 0 for interval row {gw, o0, o1}: chunk
// byte p of the tile reads unified base U + p (forward strand g = gs + (p -
// s), reverse strand 2*span-1 - (gs + len-1 - (p - s)), s = o0 - T0).  U may
// wrap below 0 for an interval that starts far into the tile; U + p does not,
// and it is below 2^33 (genome < 4 Gbases), so 33 bits of U are enough.
__device__ __forceinline__ uint64_t row_anchor(uint64_t gw, uint64_t o0, uint64_t o1, uint64_t T0,
                                               uint64_t span) {
  const uint64_t gs = gw & ~kExFlagBits;
  const uint64_t s = o0 - T0;
  return (gw & kRcBit) ? 2 * span - gs - (o1 - o0) - s : gs - s;
}
constexpr uint64_t kUMask = (1ull << 33) - 1;

// General chunk assembly: any number of interval segments, exception runs.
__device__ __noinline__ Chunk build_chunk_slow(Planes a, int p, int lim, int i,
                                               const uint4* ex) {
  Chunk o;
  o.x0 = 0;
  o.x1 = 0;
  o.exc = 0;
  o.lit[0] = o.lit[1] = o.lit[2] = o.lit[3] = 0;
  const int end = min(p + kChunk, lim);
  int pos = p;
  while (pos < end) {
    uint4 X = ex[i];
    while ((int)X.z <= pos) X = ex[++i];
    const int j0 = pos - p;
    const int n = min((int)X.z, end) - pos;
    const bool rc = (X.w & kFlagRc) != 0;
    const uint64_t U = (uint64_t)X.y | ((uint64_t)((X.w >> 12) & 1u) << 32);  // U mod 2^33
    uint32_t x0, x1;
    window(a.nib, (U + (uint64_t)p) & kUMask, x0, x1);  // chunk byte k <- unified base U + p + k
    const uint64_t m = (n >= 16 ? ~0ull : ((1ull << (4 * n)) - 1ull)) << (4 * j0);
    o.x0 = bfi((uint32_t)m, x0, o.x0);
    o.x1 = bfi((uint32_t)(m >> 32), x1, o.x1);
    if (X.w & kFlagExc) {
      // forward coordinates of chunk bytes j0 .. j0+n-1
      const uint64_t u0 = (U + (uint64_t)pos) & kUMask;
      const uint64_t glo = rc ? 2 * a.span - 1 - (u0 + (uint64_t)(n - 1)) : u0;
      patch_runs(a, glo, glo + (uint64_t)(n - 1), rc, j0, o);
    }
    pos += n;
  }
  return o;
}

struct TileDesc {
  uint64_t T0, T1, Q0, Q1;
  uint32_t eb, m, tb, nt;
};

// Uniform loads through the constant address space: scalar (s_load) even in
// the persistent loop after vector stores.
template <class T>
__device__ __forceinline__ T sload(const T* p, uint32_t i) {
  typedef const __attribute__((address_space(4))) T CT;
  return ((CT*)p)[i];
}

__device__ __forceinline__ TileDesc load_desc(const ExtractArgs& a, uint32_t t) {
  typedef const __attribute__((address_space(4))) TileRec CT;
  CT* r = (CT*)a.tiles + t;  // one round of scalar loads (48 bytes)
  TileDesc d;
  d.T0 = r->T0;
  d.T1 = r->T1;
  d.Q0 = r->Q0;
  d.Q1 = r->Q1;
  d.eb = r->e1;
  d.m = r->e2 - r->e1;
  d.tb = r->j1;
  d.nt = r->j2 - r->j1;
  return d;
}

// Per-lane rows of one tile: intervals lane and lane+64, record lane.
struct TileRows {
  uint64_t o0[2], o1[2], g[2];
  uint64_t tn, tp, tq;
};

__device__ __forceinline__ TileRows load_rows(const ExtractArgs& a, const TileDesc& d, int lane) {
  TileRows r;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const uint32_t j = min((uint32_t)(lane + 64 * h), d.m);  // clamped: rows stay in bounds
    r.o0[h] = a.ex_out[d.eb + j];
    r.o1[h] = a.ex_out[d.eb + j + 1];
    r.g[h] = a.ex_g[d.eb + j];
  }
  const uint32_t j = min((uint32_t)lane, d.nt);
  r.tn = a.tx_nuc[d.tb + j];
  r.tp = a.tx_pep[d.tb + j];
  r.tq = a.tx_pep[d.tb + j + 1];
  return r;
}

// Derived per-tile quantities (all wave-uniform).
struct TileGeom {
  int span, lim, n_out, n_all, qshift, n_res, n_pc;
  uint64_t qbase;
};

__device__ __forceinline__ TileGeom geom(const ExtractArgs& a, const TileDesc& d) {
  TileGeom g;
  g.span = (int)(d.T1 - d.T0);
  g.lim = (int)min((uint64_t)(g.span + kHalo), a.total_nuc - d.T0);
  g.n_out = (g.span + kChunk - 1) / kChunk;
  g.n_all = (g.lim + kChunk - 1) / kChunk;
  g.qbase = d.Q0 & ~15ull;
  g.qshift = (int)(d.Q0 - g.qbase);
  g.n_res = (int)(d.Q1 - d.Q0);
  g.n_pc = (g.n_res + g.qshift + 15) >> 4;
  return g;
}

// Stage one tile into the wave's LDS: interval rows {anchor, end, flags},
// record rows, and the chunk->interval / residue chunk->record maps
// (histogram of first chunks + wave prefix scan).
template <int LC>
__device__ __forceinline__ void stage(WaveLds<LC>& L, uint32_t* codes, uint32_t* valid32,
                                      const TileDesc& d, const TileGeom& g, const TileRows& rows,
                                      uint64_t span, int lane) {
  const int m = (int)d.m, nt = (int)d.nt;
#pragma unroll
  for (int h = 0; h < LC; ++h) codes[lane + 64 * h] = 0;
#pragma unroll
  for (int h = 0; h < kPepPerLane; ++h) valid32[lane + 64 * h] = 0;
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int j = lane + 64 * h;
    if (j < m) {
      const uint64_t o0 = rows.o0[h], o1 = rows.o1[h], gw = rows.g[h];
      const int64_t s = (int64_t)(o0 - d.T0);
      const int64_t e = (int64_t)(o1 - d.T0);
      const uint64_t U = row_anchor(gw, o0, o1, d.T0, span);
      const uint32_t end32 = (uint32_t)min(e, (int64_t)(tile_bytes(LC) + 4 * kHalo));
      // reverse-forward: chunk c's 16 bytes are the forward bases V - 16c ..
      // V - 16c + 15, reversed and complemented (V = gs + len - 16 + s)
      const bool revfwd = (gw & kRcBit) && !(gw & kExcBit);
      const int64_t V = (int64_t)(gw & ~kExFlagBits) + (int64_t)(o1 - d.T0) - 16;
      const uint32_t fl = ((gw & kRcBit) ? kFlagRc : 0u) | ((gw & kExcBit) ? kFlagExc : 0u) |
                          ((gw & kSlowLitBit) ? kFlagSlowLit : 0u) | ((uint32_t)(U & 7) << 8) |
                          ((uint32_t)(U >> 32) & 1u) << 12 |
                          (revfwd ? kFlagRevFwd | ((uint32_t)(V & 7) << 13) : 0u);
      L.vb[j] = (uint32_t)(V >> 3) << 2;
      // byte offset of the plane word holding tile byte 0's base (mod 2^32:
      // U may wrap below 0, the chunks the row serves do not); chunk c reads
      // its window at bN + 8c, funnel shift 4 * (U & 7).  The slow path takes
      // U mod 2^33 from {y, flag bit 12}.
      const uint32_t bN = (uint32_t)((int64_t)U >> 3) << 2;
      L.ex[j] = make_uint4(bN, (uint32_t)U, end32, fl);
      if (j >= 1) {
        const int cj = ((int)s + kChunk - 1) / kChunk;
        if (cj < g.n_all) atomicAdd(&codes[cj], 1u);
      }
    }
  }
  if (lane < nt) {
    const int64_t tp = (int64_t)(rows.tp - d.Q0);
    L.tn[lane] = (int64_t)(rows.tn - d.T0);
    L.tp[lane] = tp;
    if (lane == nt - 1) L.tp[nt] = (int64_t)(rows.tq - d.Q0);
    if (lane >= 1) {
      const int pj = ((int)tp + g.qshift + 15) >> 4;
      if (pj < g.n_pc) atomicAdd(&valid32[pj], 1u);
    }
  }
  __builtin_amdgcn_wave_barrier();
  // lane l scans chunk slots LC*l .. and residue chunks
  // kPepPerLane*l .. (inclusive running counts)
  uint32_t hc[LC], pc[kPepPerLane];
#pragma unroll
  for (int i = 0; i < LC; ++i) hc[i] = codes[LC * lane + i] + (i ? hc[i - 1] : 0u);
#pragma unroll
  for (int i = 0; i < kPepPerLane; ++i) pc[i] = valid32[kPepPerLane * lane + i] + (i ? pc[i - 1] : 0u);
  const uint32_t ct = hc[LC - 1], pt = pc[kPepPerLane - 1];
  // both scans in one: interval counts (<= kExonCap) low, record counts high
  const uint32_t sc = wave_scan(ct | (pt << 16));
  const uint32_t cx = (sc & 0xFFFFu) - ct;
  const uint32_t px = (sc >> 16) - pt;
#pragma unroll
  for (int i = 0; i < LC; ++i) L.cmap[LC * lane + i] = (uint8_t)(cx + hc[i]);
#pragma unroll
  for (int i = 0; i < kPepPerLane; ++i) L.pmap[kPepPerLane * lane + i] = (uint8_t)(px + pc[i]);
  __builtin_amdgcn_wave_barrier();
}

// Three plane words holding unified bases u .. u+15 at byte offset (u >> 3) * 4.
// The plane stays below 4 GiB (genome < 4 Gbases, checked at genome load), so
// the offset is 32-bit (one alignbit + and) and the load is a raw buffer
// load off a scalar descriptor.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t plane_rsrc(const uint32_t* plane) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(plane), (short)0,
                                           (int)0xFFFFFFFFu, 0x00020000);
}

__device__ __forceinline__ uint3 load_window(__amdgpu_buffer_rsrc_t plane, uint32_t off) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b96(plane, off, 0, 0);  // default cache policy
  return make_uint3(v[0], v[1], v[2]);
}

// Fast-path chunk assembly from prefetched windows: both segments read their
// strand's half of the plane forward, so this is two funnel shifts per
// segment and a masked merge at nibble n1.
// Nibble masks of segment A by n1 (bytes from A, 1..16) for x0 and x1.
__device__ __forceinline__ uint2 seg_masks(uint32_t n1) {
  const uint32_t mlo = n1 >= 8 ? 0xFFFFFFFFu : ((1u << (4 * n1)) - 1u);
  const uint32_t mhi = n1 >= 16 ? 0xFFFFFFFFu : (n1 <= 8 ? 0u : ((1u << (4 * (n1 - 8))) - 1u));
  return make_uint2(mlo, mhi);
}

// Eight nibbles reversed, codes complemented (A<->T, C<->G: code ^ 3; the
// soft-mask bit kept).  For nibbles without the exception bit only.
__device__ __forceinline__ uint32_t revcomp8(uint32_t w) {
  const uint32_t b = __builtin_amdgcn_perm(0u, w, 0x00010203u);  // bytes reversed
  return bfi(0x0F0F0F0Fu, b >> 4, b << 4) ^ 0x33333333u;           // nibbles in each byte
}

__device__ __forceinline__ void fast_chunk(uint3 A, uint3 B, uint32_t mt, const uint2* masks,
                                           uint32_t& x0, uint32_t& x1) {
  const uint32_t sa = (mt >> 6) & 28u, sb = (mt >> 14) & 28u;  // 4 * (u & 7)
  const uint32_t a0 = funnel(A.y, A.x, sa), a1 = funnel(A.z, A.y, sa);
  const uint32_t b0 = funnel(B.y, B.x, sb), b1 = funnel(B.z, B.y, sb);
  // n1 = bytes from segment A (16 when the chunk is one segment): masks from
  // the wave's LDS table (seg_masks)
  const uint2 m = masks[(mt >> 24) & 63u];
  x0 = bfi(m.x, a0, b0);
  x1 = bfi(m.y, a1, b1);
}

template <int LC>
__global__ __launch_bounds__(kThreads) void extract_kernel(ExtractArgs a) {
  __shared__ WaveLds<LC> s_wave[kWaves];
  __shared__ __attribute__((aligned(16))) uint8_t s_lut[64];
  __shared__ uint2 s_mask[34];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  WaveLds<LC>& L = s_wave[wave];
  uint32_t* const codes = L.codes_g + kGuard;
  uint32_t* const valid32 = L.valid_g + kGuard;
  uint16_t* const valid16 = reinterpret_cast<uint16_t*>(valid32);
  const bool want_nuc = (a.outputs & MAGOT_OUT_NUC) != 0;
  const bool want_pep = (a.outputs & MAGOT_OUT_PEP) != 0;

  // XCD-aware tile order in short runs: the hardware deals blocks round-robin
  // to the 8 XCDs; here each XCD takes kXcdRun consecutive blocks in turn, so
  // most tile boundaries (an interval read by both tiles, a 128-byte output
  // line written by both) fall inside one XCD's L2.  A/B, 200 steps: runs of
  // 2 / 4 / 16 / 64 / 256 blocks -0.5 / -0.5 / -0.7 / +0.8 / +5 % per step
  // against round-robin; one contiguous run per XCD +7 %.  Complete groups of
  // 8 runs only, the tail keeps the identity order (a bijection).
  constexpr uint32_t kXcdRun = 16;
  const uint32_t xb = blockIdx.x, grp = xb / (8 * kXcdRun);
  const uint32_t vb = (grp + 1) * 8 * kXcdRun <= gridDim.x
                          ? grp * 8 * kXcdRun + (xb % 8) * kXcdRun + (xb / 8) % kXcdRun : xb;
  const uint32_t t = vb * kWaves + wave;
  if (t >= a.n_tiles) return;
  // Every wave writes the whole (identical) codon table from scalar kernel
  // arguments and then reads only what it wrote itself: no workgroup
  // barrier and no memory round trip before the tile's own loads.
  {
    // lane i takes word i of the table from the scalar argument (v_writelane)
    int v = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) asm("v_writelane_b32 %0, %1, %2" : "+v"(v) : "s"(a.lut[i]), "i"(i));
    if (lane < 16) reinterpret_cast<uint32_t*>(s_lut)[lane] = (uint32_t)v;
    // identical in every wave: [n] low n nibbles, [17 + n] high n nibbles
    if (lane < 34) {
      const uint2 lo = seg_masks(lane <= 16 ? (uint32_t)lane : (uint32_t)(33 - lane));
      s_mask[lane] = lane <= 16 ? lo : make_uint2(~lo.x, ~lo.y);
    }
  }
  if (lane < kGuard) {
    L.codes_g[lane] = 0;
    L.valid_g[lane] = 0;
  }
  const TileDesc d = load_desc(a, t);
  const TileGeom g = geom(a, d);
  stage(L, codes, valid32, d, g, load_rows(a, d, lane), a.span, lane);
  const uint64_t T0 = d.T0;

  // Chunks at tile bytes p < edge_lo or p >= edge_hi lie in the 128-byte lines
  // the tile shares with its neighbours (plain stores there, store16_edge);
  // a tile boundary on a line boundary shares none (the planner cuts there).
  const int edge_lo = (int)((((T0 + 127) >> 7) << 7) - T0);
  const int edge_hi = (int)(((d.T1 >> 7) << 7) - T0);

  // ---- nucleotide chunks: issue every window load first -------------------
  const __amdgpu_buffer_rsrc_t nib_rs = plane_rsrc(a.nib);
  uint3 wA[LC], wB[LC];
  uint32_t meta[LC];  // bit0 active, 2 reversed, 4 slow, 8..10 / 16..18 nibble
                               // shift of the A / B window, 24..29 mask index
#pragma unroll
  for (int k = 0; k < LC; ++k) {
    const int c = min(lane + 64 * k, g.n_all - 1);  // clamped: inactive lanes redo a chunk
    const int p = c * kChunk;
    const int i = L.cmap[c];
    const uint4 X = L.ex[i];
    const uint4 Y = L.ex[min(i + 1, (int)d.m - 1)];
    const int cend = min(p + kChunk, g.lim);
    const int n1 = min((int)X.z, cend) - p;  // bytes of segment A (1..16)
    const bool two = n1 < cend - p;
    const uint32_t fb = two ? Y.w : X.w;
    const bool slow = ((X.w | fb) & kFlagSlowLit) != 0 || (two && (int)Y.z < cend) ||
                      (a.outputs & kDebugSlowNuc);
    // both segments reverse-forward (or one that is): forward-plane windows,
    // descending; the merged chunk is reverse-complemented below.  A chunk
    // whose other segment is not reverse-forward reads the mirror instead.
    const bool rev = (X.w & fb & kFlagRevFwd) != 0;
    const uint32_t c8 = 8u * (uint32_t)c;
    // every candidate offset computed unconditionally (selects, no branches
    // around LDS reads)
    uint32_t fa = X.x + c8, ra = L.vb[i] - c8;
    const uint32_t ib = (uint32_t)min(i + 1, (int)d.m - 1) & (kExonCap - 1);  // < kExonCap (a power of two)
    uint32_t fb2 = Y.x + c8, rb = L.vb[ib] - c8;
    __asm__("" : "+v"(fa), "+v"(ra), "+v"(fb2), "+v"(rb));
    const uint32_t offa = rev ? ra : fa;
    const uint32_t offb = two ? (rev ? rb : fb2) : offa;
    const uint32_t sha = (rev ? X.w >> 5 : X.w) & 0x700u, shb = (rev ? fb >> 5 : fb) & 0x700u;
    // mask index: segment A's bytes are the low n1 nibbles, or (reversed) the
    // high n1 nibbles (s_mask[17 + n1])
    const uint32_t mi = (uint32_t)(two ? n1 : 16) + (rev ? 17u : 0u);
    meta[k] = ((lane + 64 * k) < g.n_all ? 1u : 0u) | (rev ? 4u : 0u) | (slow ? 16u : 0u) |
              sha | (shb << 8) | (mi << 24);
    wA[k] = load_window(nib_rs, offa);
    wB[k] = load_window(nib_rs, offb);
  }
  uint32_t x0k[LC], x1k[LC];
#pragma unroll
  for (int k = 0; k < LC; ++k) {
    fast_chunk(wA[k], wB[k], meta[k], s_mask, x0k[k], x1k[k]);
    const uint32_t r0 = revcomp8(x1k[k]), r1 = revcomp8(x0k[k]);
    const bool rv = (meta[k] & 4u) != 0;
    x0k[k] = rv ? r0 : x0k[k];
    x1k[k] = rv ? r1 : x1k[k];
  }
  uint32_t slow_any = 0, exc_any = 0;
#pragma unroll
  for (int k = 0; k < LC; ++k) {
    slow_any |= meta[k] & 16u;
    exc_any |= (meta[k] & 1u) ? (x0k[k] | x1k[k]) & 0x88888888u : 0u;
  }
  const bool any_slow = __builtin_amdgcn_readfirstlane(__ballot(slow_any != 0) != 0);
  // exception nibbles on the fast path (N runs, IUPAC with a literal class):
  // the wave decodes them from the nibble, without the run list
  const bool any_exc = __builtin_amdgcn_readfirstlane(__ballot(exc_any != 0) != 0);
#pragma unroll
  for (int k = 0; k < LC; ++k) {
    const int c = lane + 64 * k;
    const int p = c * kChunk;
    const uint32_t mt = meta[k];
    uint32_t ex = 0;
    uint32_t lit[4] = {0u, 0u, 0u, 0u};
    if (any_slow && (mt & 17u) == 17u) {
      const Planes pl{a.nib, a.dir, a.runs, a.span};
      const Chunk o = build_chunk_slow(pl, p, g.lim, L.cmap[c], L.ex);
      x0k[k] = o.x0;
      x1k[k] = o.x1;
      ex = o.exc;
      lit[0] = o.lit[0];
      lit[1] = o.lit[1];
      lit[2] = o.lit[2];
      lit[3] = o.lit[3];
    }
    if (mt & 1u) {
      if (want_nuc && c < g.n_out)
        store16_edge(a.nuc + T0 + (uint64_t)p,
                     any_exc ? chunk_ascii_lit(x0k[k], x1k[k], ex, lit) : chunk_ascii(x0k[k], x1k[k], ex, lit),
                     p < edge_lo || p >= edge_hi);
      if (want_pep) {
        codes[c] = pack_codes(x0k[k], x1k[k]);
        valid16[c] = (uint16_t)~(any_exc ? (ex | exc_bits(x0k[k], x1k[k])) : ex);
      }
    }
  }
  if (!want_pep || g.n_res <= 0) return;
  if (lane < 5) {
    codes[g.n_all + lane] = 0;  // defined words past the decoded bytes
    valid16[g.n_all + lane] = 0;
  }
  __builtin_amdgcn_wave_barrier();

  // ---- translation: kPepPerLane residue chunks per lane --------------------
#pragma unroll 1
  for (int c = lane; c < g.n_pc; c += 64) {
  const int q_first = c * 16 - g.qshift;  // residue of slot 0 (rel Q0)
  const int kk0 = c == 0 ? g.qshift : 0;
  const int kk1 = min(16, g.n_res - q_first);
  const int j = L.pmap[c];
  const int64_t tpj = L.tp[j], tpn = L.tp[j + 1];
  // segment 1: record j from slot 0; segment 2: record j+1 from slot s
  const int r1 = (int)(L.tn[j] + 3 * ((int64_t)q_first - tpj));
  const int s = (int)min(tpn - (int64_t)q_first, (int64_t)16);
  const bool two = s < kk1;
  int r2 = 0;
  bool slow = (a.outputs & kDebugSlowPep) != 0;
  if (two) {
    r2 = (int)L.tn[j + 1] - 3 * s;  // >= r1: record j+1 follows record j
    slow = slow || (L.tp[j + 2] - (int64_t)q_first) < (int64_t)kk1;
  }
  uint32_t w[4] = {0u, 0u, 0u, 0u};
  if (!slow) {
    // 16 codon indices (6 bits each) and "all three bases plain" bits (bit 3k)
    // of record j from r1 and of record j+1 from r2, merged at residue s, so
    // the table lookups run once per lane whatever the segment count.
    uint32_t Y[2][3], OK[2][2];
#pragma unroll
    for (int seg = 0; seg < 2; ++seg) {
      const int r0 = (seg == 1 && two) ? r2 : r1;
      const int cw = r0 >> 4;
      const uint32_t sh = (uint32_t)(2 * (r0 & 15));
      const uint32_t X0 = codes[cw], X1 = codes[cw + 1], X2 = codes[cw + 2], X3 = codes[cw + 3];
      Y[seg][0] = funnel(X1, X0, sh);
      Y[seg][1] = funnel(X2, X1, sh);
      Y[seg][2] = funnel(X3, X2, sh);
      const int vw = r0 >> 5;
      const uint32_t vsh = (uint32_t)(r0 & 31);
      const uint32_t V0 = valid32[vw], V1 = valid32[vw + 1], V2 = valid32[vw + 2];
      const uint32_t Z0 = funnel(V1, V0, vsh), Z1 = funnel(V2, V1, vsh);
      OK[seg][0] = Z0 & funnel(Z1, Z0, 1) & funnel(Z1, Z0, 2);
      OK[seg][1] = Z1 & (Z1 >> 1) & (Z1 >> 2);
    }
    const int sc = min(s, 16);  // residues taken from record j
    uint32_t Ym[3], ok0, ok1;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int nb = min(max(6 * sc - 32 * q, 0), 32);
      Ym[q] = bfi(nb >= 32 ? 0xFFFFFFFFu : ((1u << nb) - 1u), Y[0][q], Y[1][q]);
    }
    {
      const int n0 = min(3 * sc, 32), n1 = max(3 * sc - 32, 0);
      ok0 = bfi(n0 >= 32 ? 0xFFFFFFFFu : ((1u << n0) - 1u), OK[0][0], OK[1][0]);
      ok1 = bfi((1u << n1) - 1u, OK[0][1], OK[1][1]);
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int ob = 6 * k;
      const uint32_t idx = ((ob & 31) <= 26 ? (Ym[ob >> 5] >> (ob & 31))
                                            : funnel(Ym[(ob >> 5) + 1], Ym[ob >> 5], ob & 31)) &
                           63u;
      w[k >> 2] |= (uint32_t)s_lut[idx] << (8 * (k & 3));
    }
    // residues whose codon holds a non-ACGT base become 'X'.  Bit 3k of
    // (bad1:bad0) flags residue k; spread each word's 4 flags to byte masks.
    const uint32_t bad0 = ~ok0 & 0x49249249u;  // residues 0..10
    const uint32_t bad1 = ~ok1 & 0x00002492u;  // residues 11..15 (bits 3k-32)
    if (__builtin_amdgcn_ballot_w64((bad0 | bad1) != 0)) {
      const uint32_t f[4] = {bad0 & 0xFFFu, (bad0 >> 12) & 0xFFFu,
                             ((bad0 >> 24) | (bad1 << 8)) & 0xFFFu, (bad1 >> 4) & 0xFFFu};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        // bits 0,3,6,9 -> 0,8,16,24 (partial products never collide)
        const uint32_t m = ((f[q] * 0x8421u) & 0x01010101u) * 0xFFu;
        w[q] = (w[q] & ~m) | (0x58585858u & m);
      }
    }
  } else {
    int jj = j;
    for (int kk = kk0; kk < kk1; ++kk) {
      const int q = q_first + kk;
      while ((int64_t)q >= L.tp[jj + 1]) ++jj;
      const int r = (int)(L.tn[jj] + 3 * ((int64_t)q - L.tp[jj]));
      const int cw = r >> 4;
      const uint32_t x = funnel(codes[cw + 1], codes[cw], (uint32_t)(2 * (r & 15))) & 63u;
      const uint32_t vv = funnel(valid32[(r >> 5) + 1], valid32[r >> 5], (uint32_t)(r & 31));
      const uint32_t aa = ((vv & 7u) == 7u) ? s_lut[x] : (uint32_t)'X';
      w[kk >> 2] |= aa << (8 * (kk & 3));
    }
  }
  uint8_t* const pdst = a.pep + g.qbase + 16 * (uint64_t)c;
  if (kk0 == 0 && kk1 == 16) {
    const uint64_t pq = (uint64_t)(pdst - a.pep);
    store16_edge(pdst, make_uint4(w[0], w[1], w[2], w[3]),
                 (pq >> 7) == (d.Q0 >> 7) || (pq >> 7) == ((d.Q1 - 1) >> 7));
  } else {
#pragma unroll
    for (int kk = 0; kk < 16; ++kk)
      if (kk >= kk0 && kk < kk1) pdst[kk] = (uint8_t)(w[kk >> 2] >> (8 * (kk & 3)));
  }
  }
}

__global__ __launch_bounds__(256) void mirror_planes_kernel(uint32_t* __restrict__ nib,
                                                            uint64_t nw) {
  // reverse-strand word w: forward word nw-1-w with its nibbles reversed and
  // the codes complemented (soft-mask and exception bits kept)
  const uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= nw) return;
  const uint32_t b = __builtin_bswap32(nib[nw - 1 - w]);
  const uint32_t x = ((b >> 4) & 0x0F0F0F0Fu) | ((b << 4) & 0xF0F0F0F0u);
  // exception nibbles (8 | class): class of the reverse-complement literal,
  // N n - kept (0 1 2), every other class becomes n (1)
  const uint32_t e = (x >> 3) & 0x11111111u;
  const uint32_t emask = e * 0xFu;
  const uint32_t cls = x & 0x77777777u;
  const uint32_t big = ((cls + 0x55555555u) >> 3) & 0x11111111u;  // class >= 3
  const uint32_t rc = (cls & ~(big * 7u)) | big;
  nib[nw + w] = ((x ^ 0x33333333u) & ~emask) | ((0x88888888u | rc) & emask);
}

}  // namespace

void launch_mirror_planes(uint32_t* nib, uint64_t span, hipStream_t s) {
  const uint64_t nw = span / 8;
  if (nw == 0) return;
  hipLaunchKernelGGL(mirror_planes_kernel, dim3((uint32_t)((nw + 255) / 256)), dim3(256), 0, s,
                     nib, nw);
}

// Blocks of extract_kernel per CU.  Its registers and LDS allow 7 (70 VGPRs,
// 22.4 KB per block); 6 runs faster: fewer tiles in flight contend less in the
// memory system it is bound by.  A/B on one box, 3 alternating runs of the
// default bench: 0.2729 / 0.2730 / 0.2728 ms per step at 6 blocks against
// 0.2761 / 0.2761 / 0.2763 at 7 (5 blocks: 0.2749 / 0.2754 / 0.2762).  The cap
// is dynamic LDS that the kernel never touches (an override for occupancy
// sweeps: scripts/experiments/occupancy_knobs.patch).
constexpr int kExtractBlocksPerCu = 6;

template <int LC>
size_t extract_lds_pad() {
  static const size_t pad = occupancy_lds_pad(reinterpret_cast<const void*>(extract_kernel<LC>),
                                              kThreads, kExtractBlocksPerCu);
  return pad;
}

void launch_extract(const ExtractArgs& a, hipStream_t s) {
  if (a.n_tiles == 0) return;
  const uint32_t grid = (a.n_tiles + kWaves - 1) / kWaves;  // one tile per wave
  if (a.lane_chunks == kLaneChunksSmall)
    hipLaunchKernelGGL(extract_kernel<kLaneChunksSmall>, dim3(grid), dim3(kThreads),
                       extract_lds_pad<kLaneChunksSmall>(), s, a);
  else
    hipLaunchKernelGGL(extract_kernel<kLaneChunksLarge>, dim3(grid), dim3(kThreads),
                       extract_lds_pad<kLaneChunksLarge>(), s, a);
}

int extract_blocks_per_cu() {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, extract_kernel<kLaneChunksLarge>, kThreads,
                                                   extract_lds_pad<kLaneChunksLarge>()) !=
      hipSuccess)
    return 0;
  return n;
}

}  // namespace magot
