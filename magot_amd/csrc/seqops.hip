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
// padded offsets, the real lengths follow from the record length), so a lane
// owns one 16-residue chunk of exactly one stream and always stores 16 bytes.
// A wave's 64 chunks read neighbouring bytes (forward or backward), so the
// wave stages that byte range into LDS with 16-byte loads and each codon
// reads three LDS bytes, mapped byte -> code -> residue through LDS tables.
// ---------------------------------------------------------------------------
constexpr int kOrfStage = 4096;  // bytes of input staged per wave (3 per residue + slack)
constexpr uint64_t kOrfWaveResidues = 64 * 16;

// real codons of frame f in a record of L bases (0 when translate() is None)
__device__ __host__ __forceinline__ uint64_t orf_count(uint64_t L, uint32_t f) {
  return (L > 2 + f && L >= 2 * f + 3) ? (L - 2 * f) / 3 : 0;
}

// wave_j0[w] = the stream holding padded residue w * kOrfWaveResidues.
__global__ __launch_bounds__(kOpsThreads) void orf6_index_kernel(const uint64_t* __restrict__ soff,
                                                                uint64_t n_streams,
                                                                uint32_t* __restrict__ wave_j0) {
  const uint64_t j = (uint64_t)blockIdx.x * kOpsThreads + threadIdx.x;
  if (j >= n_streams) return;
  const uint64_t a = soff[j], b = soff[j + 1];
  for (uint64_t w = (a + kOrfWaveResidues - 1) / kOrfWaveResidues; w * kOrfWaveResidues < b; ++w)
    wave_j0[w] = (uint32_t)j;
}

// 16 residues from codons at x0, x0 +- 3, ... of src (LDS stage or global);
// residues past nres repeat the last one (stream padding).
template <class P>
__device__ __forceinline__ uint4 orf_codons(P src, int64_t x0, bool minus, int nres,
                                            const uint8_t* code, const uint8_t* lut) {
  const int d = minus ? -1 : 1;
  const uint32_t flip = minus ? 63u : 0u;
  uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int64_t x = x0 + (int64_t)(3 * d) * min(i, nres - 1);
    const uint32_t t0 = code[src[x]], t1 = code[src[x + d]], t2 = code[src[x + 2 * d]];
    const uint32_t idx = ((t0 & 3u) | ((t1 & 3u) << 2) | ((t2 & 3u) << 4)) ^ flip;
    const uint32_t aa = ((t0 | t1 | t2) & 4u) ? (uint32_t)'X' : (uint32_t)lut[idx];
    w[i >> 2] |= aa << (8 * (i & 3));
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

__global__ __launch_bounds__(kOpsThreads) void orf6_kernel(
    const uint8_t* __restrict__ nuc, const uint64_t* __restrict__ noff,
    const uint64_t* __restrict__ soff, uint64_t n_streams, uint64_t total,
    const uint32_t* __restrict__ wave_j0, const uint8_t* __restrict__ lut64,
    uint8_t* __restrict__ out) {
  __shared__ uint8_t s_lut[64];
  __shared__ uint8_t s_code[256];  // byte -> 2-bit code | 4 when not ACGTacgt
  __shared__ uint4 s_stage[kOpsThreads / 64][kOrfStage / 16 + 2];
  __shared__ uint64_t s_soff[kOpsThreads / 64][65];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (threadIdx.x < 64) s_lut[threadIdx.x] = lut64[threadIdx.x];
  s_code[threadIdx.x] = (uint8_t)code_of(threadIdx.x);
  __syncthreads();
  const uint64_t wq0 = ((uint64_t)blockIdx.x * kOpsThreads + (uint64_t)wave * 64) * 16;
  if (wq0 >= total) return;  // wave-uniform
  // the wave's streams: j0 (orf6_index_kernel) and the next 64 offsets in LDS
  const uint64_t j0 = wave_j0[wq0 / kOrfWaveResidues];
  uint64_t* const win = s_soff[wave];
  win[lane] = soff[min(j0 + lane, n_streams)];
  if (lane == 0) win[64] = soff[min(j0 + 64, n_streams)];
  __builtin_amdgcn_wave_barrier();
  const uint64_t q0 = wq0 + 16 * (uint64_t)lane;
  const bool active = q0 < total;
  // this lane's stream: last j with soff[j] <= q0 (inside the window nearly always)
  uint64_t j;
  if (win[64] > q0 || j0 + 64 >= n_streams) {
    uint32_t lo = 0, hi = (uint32_t)min((uint64_t)64, n_streams - j0);
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (win[mid] <= q0) lo = mid;
      else hi = mid;
    }
    j = j0 + lo;
  } else {
    uint64_t lo = j0 + 64, hi = n_streams;
    while (hi - lo > 1) {
      const uint64_t mid = (lo + hi) >> 1;
      if (soff[mid] <= q0) lo = mid;
      else hi = mid;
    }
    j = lo;
  }
  const uint32_t r = (uint32_t)(j / 6), cfg = (uint32_t)(j - 6 * (uint64_t)r), f = cfg >> 1;
  const bool minus = (cfg & 1) == 0;
  const uint64_t b = noff[r], L = noff[r + 1] - b;
  const uint64_t k0 = q0 - (j - j0 < 64 ? win[j - j0] : soff[j]);
  const int nres = active ? (int)min((uint64_t)16, orf_count(L, f) - k0) : 1;
  const uint64_t s0 = 2 * f + 3 * k0;
  const uint64_t pos0 = minus ? b + L - 1 - s0 : b + s0;
  const uint64_t span = 3 * (uint64_t)(nres - 1) + 2;
  uint64_t lo = active ? (minus ? pos0 - span : pos0) : ~0ull;
  uint64_t hi = active ? (minus ? pos0 : pos0 + span) : 0;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    lo = min(lo, (uint64_t)__shfl_xor((unsigned long long)lo, d, 64));
    hi = max(hi, (uint64_t)__shfl_xor((unsigned long long)hi, d, 64));
  }
  const uint64_t base = lo & ~15ull;
  const bool staged = hi - base < (uint64_t)kOrfStage;  // wave-uniform
  if (staged) {
    // all loads in flight before the first LDS write (one memory latency)
    const uint32_t n16 = (uint32_t)((hi - base) / 16 + 1);
    constexpr int kPer = kOrfStage / 16 / 64;
    uint4 v[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {  // clamped, unconditional: the values stay in VGPRs
      const uint32_t t = min((uint32_t)(lane + 64 * k), n16 - 1);
      v[k] = *reinterpret_cast<const uint4*>(nuc + base + 16 * (uint64_t)t);
    }
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const uint32_t t = lane + 64 * k;
      if (t < n16) s_stage[wave][t] = v[k];
    }
    __builtin_amdgcn_wave_barrier();
  }
  if (!active) return;
  const uint4 res = staged ? orf_codons(reinterpret_cast<const uint8_t*>(s_stage[wave]),
                                        (int64_t)(pos0 - base), minus, nres, s_code, s_lut)
                           : orf_codons(nuc, (int64_t)pos0, minus, nres, s_code, s_lut);
  *reinterpret_cast<uint4*>(out + q0) = res;
}

}  // namespace

uint64_t orf6_index_words(uint64_t total) {
  return (total + kOrfWaveResidues - 1) / kOrfWaveResidues + 1;
}

void launch_orf6_index(const uint64_t* soff, uint64_t n_rec, uint32_t* wave_j0, hipStream_t s) {
  const uint64_t n = 6 * n_rec;
  if (n == 0) return;
  hipLaunchKernelGGL(orf6_index_kernel, dim3((uint32_t)((n + kOpsThreads - 1) / kOpsThreads)),
                     dim3(kOpsThreads), 0, s, soff, n, wave_j0);
}

void launch_orf6(const uint8_t* nuc, const uint64_t* noff, uint64_t n_rec, const uint64_t* soff,
                 uint64_t total, const uint32_t* wave_j0, const uint8_t* lut64_dev, uint8_t* out,
                 hipStream_t s) {
  if (total == 0) return;
  const uint64_t chunks = (total + 15) / 16;
  const uint64_t blocks = (chunks + kOpsThreads - 1) / kOpsThreads;
  hipLaunchKernelGGL(orf6_kernel, dim3((uint32_t)blocks), dim3(kOpsThreads), 0, s, nuc, noff, soff,
                     6 * n_rec, total, wave_j0, lut64_dev, out);
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
