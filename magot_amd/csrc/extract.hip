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
//   * The concatenated nucleotide output of all records is cut into 12 KiB
//     tiles, one 256-thread workgroup per tile.  Every lane owns 16-byte
//     aligned output chunks, so every nucleotide store is one 16-byte
//     global_store regardless of record or exon boundaries.
//   * A chunk is assembled from <=16-base windows of the 2-bit code plane and
//     the soft-mask plane (two dword loads each), reversed in-register for
//     reverse-strand intervals (bit-reverse + pair swap + complement), turned
//     into ASCII with one v_perm per 4 bytes, and patched from the exception
//     run list only when the 4096-base directory says a run is present.
//   * The tile's 2-bit codes and validity bits stay in LDS; the translation
//     phase reads codons from LDS (a codon may run 2 bytes into the halo
//     chunk) and writes the tile's contiguous residue range with 16-byte
//     stores (byte stores only on the two ragged edges of the range).
#include "common.h"

namespace magot {
namespace {

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

struct Chunk {
  uint32_t codes;   // 16 x 2-bit, byte k at bits 2k (already complemented for rc)
  uint32_t low;     // 16 x soft-mask bit
  uint32_t exc;     // 16 x "literal byte" bit
  uint32_t lit[4];  // literal bytes, little-endian by chunk byte
};

__device__ __forceinline__ void put_literal(Chunk& o, int ka, int kb, uint32_t byte) {
  uint32_t n = (uint32_t)(kb - ka + 1);
  uint32_t bits = ((n >= 32u) ? 0xFFFFFFFFu : ((1u << n) - 1u)) << ka;
  o.exc |= bits;
  uint32_t rep = byte * 0x01010101u;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint32_t bm = spread_bits((bits >> (4 * q)) & 0xFu) * 0xFFu;
    o.lit[q] = (o.lit[q] & ~bm) | (rep & bm);
  }
}

__device__ __forceinline__ uint4 chunk_ascii(const Chunk& o) {
  uint32_t w[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint32_t sel = spread_codes((o.codes >> (8 * q)) & 0xFFu);
    // bytes 'A','C','G','T' in both perm sources: selector 0..3 picks one.
    uint32_t asc = __builtin_amdgcn_perm(0x54474341u, 0x54474341u, sel);
    asc |= spread_bits((o.low >> (4 * q)) & 0xFu) << 5;
    uint32_t em = spread_bits((o.exc >> (4 * q)) & 0xFu) * 0xFFu;
    w[q] = (asc & ~em) | (o.lit[q] & em);
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

struct LdsU64 {
  const uint64_t* p;
  __device__ __forceinline__ uint64_t operator()(int i) const { return p[i]; }
};

// Assemble the 16 output bytes starting at output coordinate P.
// S(i) = output start of cached exon i (S(m) = end of the last one),
// G(i) = its genome start | kRcBit.
template <class SA, class GA>
__device__ __forceinline__ void build_chunk(const ExtractArgs& a, uint64_t P, SA S, GA G, int m,
                                            Chunk& o) {
  o.codes = 0;
  o.low = 0;
  o.exc = 0;
  o.lit[0] = o.lit[1] = o.lit[2] = o.lit[3] = 0;
  int lo = 0, hi = m;
  while (lo < hi) {
    int mid = (lo + hi) >> 1;
    if (S(mid) <= P) lo = mid + 1;
    else hi = mid;
  }
  int i = lo - 1;
  const uint64_t limit = min(P + (uint64_t)kChunk, a.total_nuc);
  uint64_t pos = P;
  int j0 = 0;
  while (pos < limit) {
    uint64_t ee = S(i + 1);
    while (ee <= pos) {
      ++i;
      ee = S(i + 1);
    }
    const uint64_t es = S(i);
    const uint64_t gw = G(i);
    const bool rc = (gw & kRcBit) != 0;
    const uint64_t g = gw & ~kRcBit;
    const int n = (int)(min(ee, limit) - pos);
    const uint64_t off = pos - es;
    uint64_t glo, ghi, wbase;
    if (!rc) {
      glo = g + off;
      ghi = glo + (uint64_t)(n - 1);
      wbase = glo;
    } else {
      ghi = g + (ee - es - 1 - off);
      glo = ghi - (uint64_t)(n - 1);
      wbase = ghi - 15;  // >= 0 thanks to the kOrigin pad
    }
    const uint64_t ci = wbase >> 4;
    const uint64_t cv = (uint64_t)a.codes[ci] | ((uint64_t)a.codes[ci + 1] << 32);
    uint32_t t = (uint32_t)(cv >> (2 * (wbase & 15)));
    const uint64_t li = wbase >> 5;
    const uint64_t lv = (uint64_t)a.lower[li] | ((uint64_t)a.lower[li + 1] << 32);
    uint32_t lt = (uint32_t)(lv >> (wbase & 31)) & 0xFFFFu;
    if (rc) {
      t = ~rev_pairs(t);                         // reverse + complement (A<->T, C<->G)
      lt = __builtin_bitreverse32(lt) >> 16;     // reverse the mask too
    }
    const uint32_t m2 = (n >= 16 ? 0xFFFFFFFFu : ((1u << (2 * n)) - 1u)) << (2 * j0);
    o.codes |= (t << (2 * j0)) & m2;
    o.low |= (lt << j0) & (((1u << n) - 1u) << j0);

    // Exception runs: skip unless the directory flags a run in these blocks.
    const uint32_t d0 = a.dir[glo >> kDirShift];
    const uint32_t d1 = a.dir[ghi >> kDirShift];
    if (!((d0 & kDirClean) && (d1 & kDirClean))) {
      uint32_t d = d0 & ~kDirClean;
      for (;;) {
        const ExcRun r = a.runs[d];
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
    }
    j0 += n;
    pos += (uint64_t)n;
  }
}

__global__ __launch_bounds__(kThreads) void extract_kernel(ExtractArgs a) {
  __shared__ uint64_t s_start[kExonCap + 1];
  __shared__ uint64_t s_g[kExonCap];
  __shared__ uint32_t s_codes[kTileChunks + 2];
  __shared__ uint16_t s_valid[kTileChunks + 2];
  __shared__ uint32_t s_lut[64];

  const uint32_t tile = blockIdx.x;
  const uint64_t T0 = (uint64_t)tile * kTile;
  const uint32_t eb = a.tile_ex[2 * tile];
  const int m = (int)(a.tile_ex[2 * tile + 1] - eb);
  const bool cached = m <= kExonCap;
  const int tid = threadIdx.x;

  if (tid < 64) s_lut[tid] = (a.lut[tid >> 2] >> (8 * (tid & 3))) & 0xFFu;
  if (cached) {
    for (int k = tid; k <= m; k += kThreads) s_start[k] = a.ex_out[eb + k];
    for (int k = tid; k < m; k += kThreads) s_g[k] = a.ex_g[eb + k];
  }
  __syncthreads();

  // ---- nucleotide phase: 768 chunks + 1 halo chunk (LDS only) -------------
  const bool want_nuc = (a.outputs & MAGOT_OUT_NUC) != 0;
  for (int ch = tid; ch <= kTileChunks; ch += kThreads) {
    const uint64_t P = T0 + (uint64_t)ch * kChunk;
    Chunk o;
    if (P < a.total_nuc) {
      if (cached) {
        build_chunk(a, P, LdsU64{s_start}, LdsU64{s_g}, m, o);
      } else {
        build_chunk(a, P, LdsU64{a.ex_out + eb}, LdsU64{a.ex_g + eb}, m, o);
      }
      if (want_nuc && ch < kTileChunks) *reinterpret_cast<uint4*>(a.nuc + P) = chunk_ascii(o);
    } else {
      o.codes = 0;
      o.exc = 0xFFFFu;
    }
    s_codes[ch] = o.codes;
    s_valid[ch] = (uint16_t)(~o.exc);
  }
  if (tid == 0) {
    s_codes[kTileChunks + 1] = 0;
    s_valid[kTileChunks + 1] = 0;
  }
  if (!(a.outputs & MAGOT_OUT_PEP)) return;
  __syncthreads();

  // ---- translation phase: residues whose codon starts inside the tile ----
  const uint64_t Q0 = a.tile_q[tile];
  const uint64_t Q1 = a.tile_q[tile + 1];
  if (Q0 >= Q1) return;
  const uint32_t tA = a.tile_t[tile];
  const uint32_t tB = a.tile_t[tile + 1];
  const uint64_t c0 = Q0 & ~15ull;
  const int nch = (int)((Q1 - c0 + 15) >> 4);
  for (int k = tid; k < nch; k += kThreads) {
    const uint64_t c = c0 + (uint64_t)k * 16;
    const uint64_t qf = max(c, Q0);
    uint32_t lo = tA, hi = tB + 1;
    while (lo < hi) {
      uint32_t mid = (lo + hi) >> 1;
      if (a.tx_pep[mid] <= qf) lo = mid + 1;
      else hi = mid;
    }
    uint32_t t = lo - 1;
    uint64_t pb = a.tx_pep[t], pe = a.tx_pep[t + 1], nb = a.tx_nuc[t];
    uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
      const uint64_t q = c + kk;
      if (q >= qf && q < Q1) {
        while (q >= pe) {
          ++t;
          pb = pe;
          pe = a.tx_pep[t + 1];
          nb = a.tx_nuc[t];
        }
        const uint32_t r = (uint32_t)(nb + 3 * (q - pb) - T0);
        const uint32_t wi = r >> 4;
        const uint64_t v = (uint64_t)s_codes[wi] | ((uint64_t)s_codes[wi + 1] << 32);
        const uint32_t x = (uint32_t)(v >> (2 * (r & 15))) & 63u;
        const uint32_t vv = ((uint32_t)s_valid[wi] | ((uint32_t)s_valid[wi + 1] << 16)) >> (r & 15);
        const uint32_t aa = ((vv & 7u) == 7u) ? s_lut[x] : (uint32_t)'X';
        w[kk >> 2] |= aa << (8 * (kk & 3));
      }
    }
    if (c >= Q0 && c + 16 <= Q1) {
      *reinterpret_cast<uint4*>(a.pep + c) = make_uint4(w[0], w[1], w[2], w[3]);
    } else {
#pragma unroll
      for (int kk = 0; kk < 16; ++kk) {
        const uint64_t q = c + kk;
        if (q >= Q0 && q < Q1) a.pep[q] = (uint8_t)(w[kk >> 2] >> (8 * (kk & 3)));
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
