// Batch kernels over raw byte strings (not the packed genome):
//   revcomp_kernel   -- Sequence.reverse_compliment  genome.py:784-793
//   translate_kernel -- Sequence.translate           genome.py:795-822
// Both are output-stationary: a lane owns 16 aligned output bytes, finds its
// record by binary search over the offset table and reads its inputs from L2.
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
// Output layout: every stream starts on a 16-byte boundary (soff holds the
// padded offsets, the real lengths follow from the record length); the
// residues of a 16-byte chunk past the stream's end repeat its last residue.
//
// Input-stationary: one wave owns a tile of kOrfTile bases of the
// concatenated records and every output chunk whose first codon starts in
// it (all six streams of every record the tile touches).  The tile plus a
// 48/50-base halo is staged once, as one byte per position:
//   cidx[p] = c[p] | c[p+1] << 2 | c[p+2] << 4 | (any of the three not
//             ACGTacgt) << 6
// so a '+' residue is tbl[cidx[p]] and a '-' residue (codon read backwards,
// complemented) is tbl[128 + cidx[p]] with the second table pre-permuted:
// two LDS reads per residue, each input byte converted once for all six
// streams.  Each staged record byte feeds ~2 output bytes, so the kernel
// streams the nucleotides once and writes the residues once.
// ---------------------------------------------------------------------------
constexpr int64_t kOrfTile = 3968;  // bases per wave tile: + halo and alignment = 256 x 16 B
constexpr int kOrfVecs = 256;       // staged 16-byte vectors per wave
constexpr int kOrfBatch = 32;       // records per segment batch
constexpr int kOrfSegs = 6 * kOrfBatch;

// real codons of frame f in a record of L bases (0 when translate() is None)
__device__ __host__ __forceinline__ uint64_t orf_count(uint64_t L, uint32_t f) {
  return (L > 2 + f && L >= 2 * f + 3) ? (L - 2 * f) / 3 : 0;
}

// tile_r0[t] = the record holding base t * kOrfTile of the concatenation.
__global__ __launch_bounds__(kOpsThreads) void orf6_index_kernel(const uint64_t* __restrict__ noff,
                                                                uint64_t n_rec,
                                                                uint32_t* __restrict__ tile_r0) {
  const uint64_t r = (uint64_t)blockIdx.x * kOpsThreads + threadIdx.x;
  if (r >= n_rec) return;
  const uint64_t a = noff[r], b = noff[r + 1];
  for (uint64_t t = (a + kOrfTile - 1) / kOrfTile; (uint64_t)t * kOrfTile < b; ++t)
    tile_r0[t] = (uint32_t)r;
}

struct OrfSeg {
  uint64_t out0;  // output byte of the segment's first chunk
  int32_t p0;     // staged position of its first residue's codon
  int32_t rem0;   // residues from there to the stream's end; < 0: '-' strand
};

__global__ __launch_bounds__(kOpsThreads) void orf6_kernel(
    const uint8_t* __restrict__ nuc, const uint64_t* __restrict__ noff, uint64_t n_rec,
    uint64_t total, const uint64_t* __restrict__ soff, const uint32_t* __restrict__ tile_r0,
    const uint8_t* __restrict__ tables, uint64_t n_tiles, uint8_t* __restrict__ out) {
  __shared__ uint32_t s_tbl[64];  // bytes: [0,128) '+', [128,256) '-'
  __shared__ uint4 s_stage[kOpsThreads / 64][kOrfVecs];
  __shared__ OrfSeg s_seg[kOpsThreads / 64][kOrfSegs];
  __shared__ uint32_t s_start[kOpsThreads / 64][kOrfSegs + 1];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (threadIdx.x < 64) s_tbl[threadIdx.x] = reinterpret_cast<const uint32_t*>(tables)[threadIdx.x];
  __syncthreads();
  const uint64_t tile = (uint64_t)blockIdx.x * (kOpsThreads / 64) + wave;
  if (tile >= n_tiles) return;  // wave-uniform
  const uint64_t T0 = tile * kOrfTile, T1 = min(T0 + kOrfTile, total);
  const uint64_t W0 = (T0 >= 48 ? T0 - 48 : 0) & ~15ull;
  const uint64_t WE = min(T1 + 50, total);
  const uint32_t nvec = (uint32_t)((WE - W0 + 15) / 16);
  // staging loads first (one memory latency), converted after the record reads
  constexpr int kPer = kOrfVecs / 64;
  uint4 v[kPer];
  uint32_t nx[kPer];
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const uint32_t t = min((uint32_t)(lane + 64 * k), nvec - 1);
    v[k] = *reinterpret_cast<const uint4*>(nuc + W0 + 16 * (uint64_t)t);
    nx[k] = *reinterpret_cast<const uint32_t*>(nuc + W0 + 16 * (uint64_t)min(t + 1, nvec - 1));
  }
  const uint8_t* const stage = reinterpret_cast<const uint8_t*>(s_stage[wave]);
  const uint8_t* const tbl = reinterpret_cast<const uint8_t*>(s_tbl);
  OrfSeg* const seg = s_seg[wave];
  uint32_t* const start = s_start[wave];
  bool staged = false;
  for (uint64_t rb = tile_r0[tile];; rb += kOrfBatch) {
    // ---- this batch's segments: lane < kOrfBatch owns record rb + lane
    const uint64_t r = rb + (uint64_t)lane;
    uint64_t nb = 0, L = 0;
    const bool rec = lane < kOrfBatch && r < n_rec;
    if (rec) {
      nb = noff[r];
      L = noff[r + 1] - nb;
    }
    const bool mine = rec && nb < T1;
    uint32_t cnt[6];
    uint32_t lane_total = 0;
#pragma unroll
    for (int s = 0; s < 6; ++s) {
      const uint32_t f = (uint32_t)s >> 1;
      const bool plus = s & 1;
      const int64_t nres = mine ? (int64_t)orf_count(L, f) : 0;
      const int64_t nch = (nres + 15) / 16;
      int64_t lo = 0, hi = 0, p = 0;
      if (plus) {  // chunk c's first codon starts at x0 + 48c
        const int64_t x0 = (int64_t)(nb + 2 * f);
        lo = (int64_t)T0 > x0 ? ((int64_t)T0 - x0 + 47) / 48 : 0;
        hi = (int64_t)T1 > x0 ? ((int64_t)T1 - x0 + 47) / 48 : 0;
        p = x0 + 48 * lo;
      } else {  // chunk c's first codon (read backwards) lies at x0 - 48c
        const int64_t x0 = (int64_t)(nb + L) - 3 - 2 * (int64_t)f;
        lo = x0 >= (int64_t)T1 ? (x0 - (int64_t)T1) / 48 + 1 : 0;
        hi = x0 >= (int64_t)T0 ? (x0 - (int64_t)T0) / 48 + 1 : 0;
        p = x0 - 48 * lo;
      }
      hi = min(hi, nch);
      lo = min(lo, hi);
      cnt[s] = (uint32_t)(hi - lo);
      if (cnt[s]) {
        const uint64_t j = 6 * r + (uint64_t)s;
        OrfSeg g;
        g.out0 = soff[j] + 16 * (uint64_t)lo;
        g.p0 = (int32_t)((int64_t)p - (int64_t)W0);
        const int32_t rem = (int32_t)(nres - 16 * lo);
        g.rem0 = plus ? rem : -rem;
        seg[6 * lane + s] = g;
      }
      lane_total += cnt[s];
    }
    // wave-inclusive scan of the lane totals
    uint32_t incl = lane_total;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(incl, d, 64);
      if (lane >= d) incl += y;
    }
    const uint32_t n_chunks = __shfl(incl, 63, 64);
    if (lane < kOrfBatch) {
      uint32_t acc = incl - lane_total;
#pragma unroll
      for (int s = 0; s < 6; ++s) {
        start[6 * lane + s] = acc;
        acc += cnt[s];
      }
    }
    if (lane == 0) start[kOrfSegs] = n_chunks;
    // does the next batch still start inside the tile?
    const bool more = __shfl((int)(rec && nb + L < T1), kOrfBatch - 1, 64) &&
                      rb + kOrfBatch < n_rec;
    if (!staged) {
#pragma unroll
      for (int k = 0; k < kPer; ++k) {
        const uint32_t t = lane + 64 * k;
        const uint32_t w[5] = {v[k].x, v[k].y, v[k].z, v[k].w, nx[k]};
        uint32_t c[18];
#pragma unroll
        for (int i = 0; i < 18; ++i) c[i] = code_of((w[i >> 2] >> (8 * (i & 3))) & 0xFFu);
        uint32_t o[4] = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const uint32_t x = (c[i] & 3u) | ((c[i + 1] & 3u) << 2) | ((c[i + 2] & 3u) << 4) |
                             (((c[i] | c[i + 1] | c[i + 2]) & 4u) << 4);
          o[i >> 2] |= x << (8 * (i & 3));
        }
        if (t < nvec) s_stage[wave][t] = make_uint4(o[0], o[1], o[2], o[3]);
      }
      staged = true;
    }
    __builtin_amdgcn_wave_barrier();
    // ---- the batch's chunks, 64 at a time
    for (uint32_t q = lane; q < n_chunks; q += 64) {
      uint32_t a = 0, b = kOrfSegs;  // last segment with start <= q (and chunks)
      while (b - a > 1) {
        const uint32_t m = (a + b) >> 1;
        if (start[m] <= q) a = m;
        else b = m;
      }
      const OrfSeg g = seg[a];
      const uint32_t k = q - start[a];
      const bool minus = g.rem0 < 0;
      const int32_t rem = (minus ? -g.rem0 : g.rem0) - 16 * (int32_t)k;
      const int32_t nr = min(16, rem);
      const int32_t step = minus ? -3 : 3;
      const int32_t p = g.p0 + 16 * step * (int32_t)k;
      const uint32_t toff = minus ? 128u : 0u;
      uint32_t o[4] = {0u, 0u, 0u, 0u};
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int32_t pi = min(max(p + step * min(i, nr - 1), 0), 16 * kOrfVecs - 1);
        const uint32_t aa = tbl[toff + stage[pi]];
        o[i >> 2] |= aa << (8 * (i & 3));
      }
      *reinterpret_cast<uint4*>(out + g.out0 + 16 * (uint64_t)k) = make_uint4(o[0], o[1], o[2], o[3]);
    }
    if (!more) break;
    __builtin_amdgcn_wave_barrier();  // segment tables are rewritten
  }
}

}  // namespace

uint64_t orf6_index_words(uint64_t total_nuc) {
  return (total_nuc + kOrfTile - 1) / kOrfTile + 1;
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

void launch_orf6_index(const uint64_t* noff, uint64_t n_rec, uint32_t* tile_r0, hipStream_t s) {
  if (n_rec == 0) return;
  hipLaunchKernelGGL(orf6_index_kernel, dim3((uint32_t)((n_rec + kOpsThreads - 1) / kOpsThreads)),
                     dim3(kOpsThreads), 0, s, noff, n_rec, tile_r0);
}

void launch_orf6(const uint8_t* nuc, const uint64_t* noff, uint64_t n_rec, uint64_t total_nuc,
                 const uint64_t* soff, const uint32_t* tile_r0, const uint8_t* tables_dev,
                 uint8_t* out, hipStream_t s) {
  if (total_nuc == 0 || n_rec == 0) return;
  const uint64_t n_tiles = (total_nuc + kOrfTile - 1) / kOrfTile;
  const uint64_t blocks = (n_tiles + kOpsThreads / 64 - 1) / (kOpsThreads / 64);
  hipLaunchKernelGGL(orf6_kernel, dim3((uint32_t)blocks), dim3(kOpsThreads), 0, s, nuc, noff,
                     n_rec, total_nuc, soff, tile_r0, tables_dev, n_tiles, out);
}

void launch_revcomp(const uint8_t* in, const uint64_t* off, uint64_t n, uint64_t total,
                    uint8_t* out, hipStream_t s) {
  if (total == 0) return;
  const uint64_t chunks = (total + 15) / 16;
  const uint64_t blocks = (chunks + kOpsThreads - 1) / kOpsThreads;
  hipLaunchKernelGGL(revcomp_kernel, dim3((uint32_t)blocks), dim3(kOpsThreads), 0, s, in, off, n,
                     total, out);
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

}  // namespace magot
