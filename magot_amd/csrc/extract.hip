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
//   * The concatenated nucleotide output of all records is cut by the host
//     planner into tiles of <= 12 KiB (16-byte aligned; shorter only where a
//     tile would hold more than kExonCap intervals or kTxCap records), one
//     256-thread workgroup per tile.  Every lane owns 16-byte aligned output
//     chunks, so every nucleotide store is one 16-byte global_store whatever
//     the record or interval boundaries.
//   * Prologue: the tile's intervals and records are staged in LDS, each as a
//     32-bit tile-relative boundary plus a 64-bit genome "anchor" (genome
//     coordinate of tile byte 0 along that interval, +p forward / -p reverse),
//     and every chunk / residue chunk is told its interval / record by a
//     scatter over boundaries -- no per-lane search.
//   * A chunk inside one interval reads one 16-base window of the 2-bit code
//     plane and of the soft-mask plane (two dword loads each; all three of a
//     lane's chunks are issued before any is consumed), reverses it
//     in-register for '-' intervals (bit-reverse, pair swap, complement),
//     becomes ASCII with one v_perm per 4 bytes, and is patched from the
//     exception run list only where the 4096-base directory flags a run.
//     Chunks that cross an interval boundary take a per-segment loop.
//   * The tile's codes and validity bits stay in LDS; a residue chunk (16
//     residues of one record) funnel-shifts 48 bases of codes out of LDS,
//     looks the 16 codons up in an LDS table and stores 16 bytes.  Ragged
//     residue chunks (record boundary inside, tile edges) take a per-residue
//     path.  Residue chunks of a tile are contiguous in the output.
#include "common.h"

namespace magot {
namespace {

constexpr int kPepChunks = kTile / 3 / 16 + 2;
constexpr int kLdsChunks = kTileChunks + 4;

__device__ __forceinline__ uint32_t rev_pairs(uint32_t x) {
  // reverse the order of the sixteen 2-bit fields of x
  x = __builtin_bitreverse32(x);
  return ((x >> 1) & 0x55555555u) | ((x & 0x55555555u) << 1);
}

__device__ __forceinline__ uint32_t spread_codes(uint32_t c8) {
  // four 2-bit codes -> four bytes 0..3
  return (c8 | (c8 << 6) | (c8 << 12) | (c8 << 18)) & 0x03030303u;
}

__device__ __forceinline__ uint32_t spread_bits(uint32_t m4) {
  // four bits -> four bytes 0/1
  return (m4 | (m4 << 7) | (m4 << 14) | (m4 << 21)) & 0x01010101u;
}

__device__ __forceinline__ uint32_t rc_literal(uint32_t b) {
  // genome.py:787,792 for a byte that is not ACGTacgt
  return (b == 'n' || b == 'N' || b == '-') ? b : (uint32_t)'n';
}

__device__ __forceinline__ uint32_t funnel(uint32_t hi, uint32_t lo, uint32_t sh) {
  return __builtin_amdgcn_alignbit(hi, lo, sh);  // (hi:lo >> sh)[31:0], sh in 0..31
}

struct Chunk {
  uint32_t codes;   // 16 x 2-bit, byte k at bits 2k (already complemented for rc)
  uint32_t low;     // 16 x soft-mask bit
  uint32_t exc;     // 16 x "literal byte" bit
  uint32_t lit[4];  // literal bytes, little-endian by chunk byte
};

__device__ __forceinline__ void put_literal(Chunk& o, int ka, int kb, uint32_t byte) {
  const uint32_t n = (uint32_t)(kb - ka + 1);
  const uint32_t bits = ((n >= 32u) ? 0xFFFFFFFFu : ((1u << n) - 1u)) << ka;
  o.exc |= bits;
  const uint32_t rep = byte * 0x01010101u;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t bm = spread_bits((bits >> (4 * q)) & 0xFu) * 0xFFu;
    o.lit[q] = (o.lit[q] & ~bm) | (rep & bm);
  }
}

__device__ __forceinline__ uint4 chunk_ascii(const Chunk& o) {
  uint32_t w[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t sel = spread_codes((o.codes >> (8 * q)) & 0xFFu);
    // bytes 'A','C','G','T' in both perm sources: selector 0..3 picks one.
    uint32_t asc = __builtin_amdgcn_perm(0x54474341u, 0x54474341u, sel);
    asc |= spread_bits((o.low >> (4 * q)) & 0xFu) << 5;
    const uint32_t em = spread_bits((o.exc >> (4 * q)) & 0xFu) * 0xFFu;
    w[q] = (asc & ~em) | (o.lit[q] & em);
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// Patch literal bytes (exception runs) of genome interval [glo, ghi] that maps
// to chunk bytes starting at j0 (forward) or ending at j0 (reverse).
__device__ __noinline__ Chunk patch_runs(const ExcRun* __restrict__ runs, uint32_t d, uint64_t glo,
                                         uint64_t ghi, bool rc, int j0, Chunk o) {
  for (;;) {
    const ExcRun r = runs[d];
    if (r.start > ghi) break;
    const uint64_t rend = r.start + r.len;
    if (rend > glo) {
      const uint64_t ovl = max(glo, r.start);
      const uint64_t ovh = min(ghi, rend - 1);
      if (!rc) put_literal(o, j0 + (int)(ovl - glo), j0 + (int)(ovh - glo), r.byte);
      else put_literal(o, j0 + (int)(ghi - ovh), j0 + (int)(ghi - ovl), rc_literal(r.byte));
    }
    ++d;
  }
  return o;
}

// Codes / soft-mask bits of the 16 genome bases starting at wbase.
struct Planes {
  const uint32_t* __restrict__ codes;
  const uint32_t* __restrict__ lower;
  const uint32_t* __restrict__ dir;
  const ExcRun* __restrict__ runs;
};

__device__ __forceinline__ void window(const Planes& a, uint64_t wbase, uint32_t& t,
                                       uint32_t& lt) {
  const uint64_t ci = wbase >> 4;
  const uint32_t c0 = a.codes[ci], c1 = a.codes[ci + 1];
  const uint64_t li = wbase >> 5;
  const uint32_t l0 = a.lower[li], l1 = a.lower[li + 1];
  t = funnel(c1, c0, (uint32_t)(2 * (wbase & 15)));
  lt = funnel(l1, l0, (uint32_t)(wbase & 31)) & 0xFFFFu;
}

// General chunk assembly: any number of interval segments.
__device__ __noinline__ Chunk build_chunk_slow(Planes a, int p, int lim, int i,
                                               const int32_t* s_es, const uint64_t* s_anchor,
                                               const uint8_t* s_rc) {
  Chunk o;
  o.codes = 0;
  o.low = 0;
  o.exc = 0;
  o.lit[0] = o.lit[1] = o.lit[2] = o.lit[3] = 0;
  const int end = min(p + kChunk, lim);
  int pos = p;
  while (pos < end) {
    while (s_es[i + 1] <= pos) ++i;
    const int j0 = pos - p;
    const int n = min(s_es[i + 1], end) - pos;
    const uint64_t A = s_anchor[i];
    const bool rc = s_rc[i] != 0;
    uint64_t glo, ghi, wbase;
    if (!rc) {
      glo = A + (uint64_t)pos;
      ghi = glo + (uint64_t)(n - 1);
      wbase = glo;
    } else {
      ghi = A - (uint64_t)pos;
      glo = ghi - (uint64_t)(n - 1);
      wbase = ghi - 15;
    }
    uint32_t t, lt;
    window(a, wbase, t, lt);
    if (rc) {
      t = ~rev_pairs(t);
      lt = __builtin_bitreverse32(lt) >> 16;
    }
    const uint32_t m2 = (n >= 16 ? 0xFFFFFFFFu : ((1u << (2 * n)) - 1u)) << (2 * j0);
    o.codes |= (t << (2 * j0)) & m2;
    o.low |= (lt << j0) & (((1u << n) - 1u) << j0);
    const uint32_t d0 = a.dir[glo >> kDirShift];
    const uint32_t d1 = a.dir[ghi >> kDirShift];
    if (!((d0 & kDirClean) && (d1 & kDirClean)))
      o = patch_runs(a.runs, d0 & ~kDirClean, glo, ghi, rc, j0, o);
    pos += n;
  }
  return o;
}

__global__ __launch_bounds__(kThreads) void extract_kernel(ExtractArgs a) {
  __shared__ uint64_t s_anchor[kExonCap];
  __shared__ int32_t s_es[kExonCap + 1];
  __shared__ uint8_t s_rc[kExonCap];
  __shared__ uint16_t s_cmap[kLdsChunks];
  __shared__ uint32_t s_codes[kLdsChunks];
  __shared__ uint32_t s_valid32[kLdsChunks / 2 + 2];
  __shared__ int64_t s_tn[kTxCap + 1];
  __shared__ int64_t s_tp[kTxCap + 1];
  __shared__ uint16_t s_pmap[kPepChunks + 2];
  __shared__ uint32_t s_lut[64];

  uint16_t* s_valid = reinterpret_cast<uint16_t*>(s_valid32);
  const Planes pl{a.codes, a.lower, a.dir, a.runs};
  const int tid = threadIdx.x;
  const uint32_t tile = blockIdx.x;
  const uint64_t T0 = a.tile_start[tile];
  const uint64_t T1 = a.tile_start[tile + 1];
  const uint32_t eb = a.tile_ex[2 * tile];
  const int m = (int)(a.tile_ex[2 * tile + 1] - eb);
  const uint32_t tb = a.tile_tx[2 * tile];
  const int nt = (int)(a.tile_tx[2 * tile + 1] - tb);
  const uint64_t Q0 = a.tile_q[tile];
  const uint64_t Q1 = a.tile_q[tile + 1];

  const int span = (int)(T1 - T0);                                       // bytes stored
  const int lim = (int)min((uint64_t)(span + kHalo), a.total_nuc - T0);  // bytes decoded
  const int n_out = (span + kChunk - 1) / kChunk;
  const int n_all = (lim + kChunk - 1) / kChunk;
  const uint64_t qbase = Q0 & ~15ull;
  const int qshift = (int)(Q0 - qbase);
  const int n_res = (int)(Q1 - Q0);
  const int n_pc = (n_res + qshift + 15) >> 4;

  // ---- prologue: stage intervals / records, scatter chunk owners -----------
  if (tid < 64) s_lut[tid] = (a.lut[tid >> 2] >> (8 * (tid & 3))) & 0xFFu;
  for (int j = tid; j < m; j += kThreads) {
    const uint64_t o0 = a.ex_out[eb + j];
    const uint64_t o1 = a.ex_out[eb + j + 1];
    const uint64_t gw = a.ex_g[eb + j];
    const bool rc = (gw & kRcBit) != 0;
    const uint64_t g = gw & ~kRcBit;
    const int64_t s = (int64_t)(o0 - T0);
    const int64_t e = (int64_t)(o1 - T0);
    s_anchor[j] = rc ? g + (o1 - o0) - 1 + (uint64_t)s : g - (uint64_t)s;
    s_rc[j] = rc ? 1 : 0;
    const int s32 = s < 0 ? 0 : (int)s;
    const int e32 = e > (int64_t)(kTile + 2 * kHalo) ? kTile + 2 * kHalo : (int)e;
    s_es[j] = s32;
    if (j == m - 1) s_es[m] = e32;
    const int c_hi = min((e32 + kChunk - 1) / kChunk, n_all);
    for (int c = (s32 + kChunk - 1) / kChunk; c < c_hi; ++c) s_cmap[c] = (uint16_t)j;
  }
  for (int j = tid; j < nt; j += kThreads) {
    const int64_t tn = (int64_t)(a.tx_nuc[tb + j] - T0);
    const int64_t tp = (int64_t)(a.tx_pep[tb + j] - Q0);
    const int64_t tq = (int64_t)(a.tx_pep[tb + j + 1] - Q0);
    s_tn[j] = tn;
    s_tp[j] = tp;
    if (j == nt - 1) s_tp[nt] = tq;
    // residue chunk c starts at relative residue max(16c - qshift, 0)
    const int64_t lo = tp <= 0 ? 0 : (tp + qshift + 15) / 16;
    const int64_t hi = min((tq + qshift + 15) / 16, (int64_t)n_pc);
    for (int64_t c = lo; c < hi; ++c) s_pmap[c] = (uint16_t)j;
  }
  __syncthreads();

  // ---- nucleotide phase: up to 3 chunks per lane + 1 halo chunk -----------
  const bool want_nuc = (a.outputs & MAGOT_OUT_NUC) != 0;
  uint32_t t[kChunksPerThread], lt[kChunksPerThread], d0[kChunksPerThread],
      d1[kChunksPerThread];
  bool single[kChunksPerThread];
  int ex_i[kChunksPerThread];
#pragma unroll
  for (int k = 0; k < kChunksPerThread; ++k) {
    const int c = tid + k * kThreads;
    const int p = c * kChunk;
    single[k] = false;
    ex_i[k] = 0;
    if (c < n_all) {
      const int i = s_cmap[c];
      ex_i[k] = i;
      single[k] = s_es[i + 1] >= min(p + kChunk, lim);
    }
    if (single[k]) {
      const int i = ex_i[k];
      const uint64_t A = s_anchor[i];
      const bool rc = s_rc[i] != 0;
      const int n = min(p + kChunk, lim) - p;
      const uint64_t glo = rc ? A - (uint64_t)(p + n - 1) : A + (uint64_t)p;
      const uint64_t ghi = glo + (uint64_t)(n - 1);
      window(pl, rc ? A - (uint64_t)p - 15 : glo, t[k], lt[k]);
      d0[k] = a.dir[glo >> kDirShift];
      d1[k] = a.dir[ghi >> kDirShift];
    }
  }
#pragma unroll
  for (int k = 0; k < kChunksPerThread + 1; ++k) {
    const int c = tid + k * kThreads;
    if (k == kChunksPerThread && tid != 0) break;
    if (c >= n_all) continue;
    const int p = c * kChunk;
    Chunk o;
    if (k < kChunksPerThread && single[k]) {
      const int i = ex_i[k];
      const bool rc = s_rc[i] != 0;
      const int n = min(p + kChunk, lim) - p;
      uint32_t tt = t[k], ll = lt[k];
      if (rc) {
        tt = ~rev_pairs(tt);
        ll = __builtin_bitreverse32(ll) >> 16;
      }
      const uint32_t m1 = n >= 16 ? 0xFFFFu : ((1u << n) - 1u);
      o.codes = n >= 16 ? tt : (tt & ((1u << (2 * n)) - 1u));
      o.low = ll & m1;
      o.exc = 0;
      o.lit[0] = o.lit[1] = o.lit[2] = o.lit[3] = 0;
      if (!((d0[k] & kDirClean) && (d1[k] & kDirClean))) {
        const uint64_t A = s_anchor[i];
        const uint64_t glo = rc ? A - (uint64_t)(p + n - 1) : A + (uint64_t)p;
        o = patch_runs(a.runs, d0[k] & ~kDirClean, glo, glo + (uint64_t)(n - 1), rc, 0, o);
      }
    } else {
      o = build_chunk_slow(pl, p, lim, s_cmap[c], s_es, s_anchor, s_rc);
    }
    if (want_nuc && c < n_out) *reinterpret_cast<uint4*>(a.nuc + T0 + p) = chunk_ascii(o);
    s_codes[c] = o.codes;
    s_valid[c] = (uint16_t)(~o.exc);
  }
  if (!(a.outputs & MAGOT_OUT_PEP) || n_res <= 0) return;
  if (tid < 4) {
    // zero the tail so window reads past the decoded bytes see defined words
    s_codes[n_all + tid] = 0;
    s_valid[n_all + tid] = 0;
  }
  __syncthreads();

  // ---- translation phase ---------------------------------------------------
  for (int c = tid; c < n_pc; c += kThreads) {
    const int kk0 = c == 0 ? qshift : 0;                   // first residue slot used
    const int q_first = c * 16 - qshift;                   // residue of slot 0 (rel Q0)
    const int kk1 = min(16, n_res - q_first);              // slots [kk0, kk1)
    int j = s_pmap[c];
    uint32_t w[4] = {0u, 0u, 0u, 0u};
    if (kk0 == 0 && kk1 == 16 && (int64_t)(q_first + 16) <= s_tp[j + 1]) {
      // 16 residues of one record: codons at r0, r0+3, ..., r0+45
      const int r0 = (int)(s_tn[j] + 3 * ((int64_t)q_first - s_tp[j]));
      const int cw = r0 >> 4;
      const uint32_t sh = (uint32_t)(2 * (r0 & 15));
      const uint32_t X0 = s_codes[cw], X1 = s_codes[cw + 1], X2 = s_codes[cw + 2],
                     X3 = s_codes[cw + 3], X4 = s_codes[cw + 4];
      const uint32_t Y[4] = {funnel(X1, X0, sh), funnel(X2, X1, sh), funnel(X3, X2, sh),
                             funnel(X4, X3, sh)};
      const int vw = r0 >> 5;
      const uint32_t vsh = (uint32_t)(r0 & 31);
      const uint32_t V0 = s_valid32[vw], V1 = s_valid32[vw + 1], V2 = s_valid32[vw + 2];
      const uint32_t Z0 = funnel(V1, V0, vsh), Z1 = funnel(V2, V1, vsh);
      // bit 3k of OK = all three bases of codon k are plain ACGT
      const uint32_t ok0 = Z0 & funnel(Z1, Z0, 1) & funnel(Z1, Z0, 2);
      const uint32_t ok1 = Z1 & (Z1 >> 1) & (Z1 >> 2);
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int ob = 6 * k;
        const uint32_t idx = ((ob & 31) <= 26 ? (Y[ob >> 5] >> (ob & 31))
                                              : funnel(Y[(ob >> 5) + 1], Y[ob >> 5], ob & 31)) &
                             63u;
        const int vb = 3 * k;
        const uint32_t okb = vb < 32 ? (ok0 >> vb) : (ok1 >> (vb - 32));
        const uint32_t aa = (okb & 1u) ? s_lut[idx] : (uint32_t)'X';
        w[k >> 2] |= aa << (8 * (k & 3));
      }
      *reinterpret_cast<uint4*>(a.pep + qbase + 16 * (uint64_t)c) = make_uint4(w[0], w[1], w[2], w[3]);
    } else {
      for (int kk = kk0; kk < kk1; ++kk) {
        const int q = q_first + kk;
        while ((int64_t)q >= s_tp[j + 1]) ++j;
        const int r = (int)(s_tn[j] + 3 * ((int64_t)q - s_tp[j]));
        const int cw = r >> 4;
        const uint32_t x = funnel(s_codes[cw + 1], s_codes[cw], (uint32_t)(2 * (r & 15))) & 63u;
        const uint32_t v = funnel(s_valid32[(r >> 5) + 1], s_valid32[r >> 5], (uint32_t)(r & 31));
        const uint32_t aa = ((v & 7u) == 7u) ? s_lut[x] : (uint32_t)'X';
        a.pep[qbase + 16 * (uint64_t)c + kk] = (uint8_t)aa;
      }
    }
  }
}

}  // namespace

void launch_extract(const ExtractArgs& a, hipStream_t s) {
  if (a.n_tiles == 0) return;
  hipLaunchKernelGGL(extract_kernel, dim3(a.n_tiles), dim3(kThreads), 0, s, a);
}

}  // namespace magot
