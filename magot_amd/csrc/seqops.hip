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
__device__ __forceinline__ uint32_t code_of(uint32_t b) {
  switch (b | 0x20u) {
    case 'a': return 0;
    case 'c': return 1;
    case 'g': return 2;
    case 't': return 3;
    default: return 4;
  }
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

}  // namespace

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
