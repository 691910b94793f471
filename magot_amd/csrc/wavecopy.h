// One wave copies one byte span: dst[d0, d1) = src[s0, s0 + d1 - d0), any
// alignment.  The 16-byte aligned chunks of the destination are stored whole,
// their source read as two aligned 16-byte blocks and funnel-shifted by the
// span's (wave-uniform) misalignment; the partial chunks at the two ends are
// written byte by byte, so spans that share a chunk can be copied by
// different waves.  Every aligned source block read holds a byte of the span
// (it stays inside the source allocation).  Used by segments_copy_kernel
// (devpack.hip) and the FASTA text assembly (render.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace magot {

__device__ __forceinline__ uint4 funnel16(uint4 a, uint4 b, uint32_t sh) {
  // bytes [sh, sh+16) of the 32-byte concatenation a:b (sh wave-uniform)
  const uint32_t r = 8 * (sh & 3);
  uint32_t w0, w1, w2, w3, w4;
  switch (sh >> 2) {
    case 0: w0 = a.x; w1 = a.y; w2 = a.z; w3 = a.w; w4 = b.x; break;
    case 1: w0 = a.y; w1 = a.z; w2 = a.w; w3 = b.x; w4 = b.y; break;
    case 2: w0 = a.z; w1 = a.w; w2 = b.x; w3 = b.y; w4 = b.z; break;
    default: w0 = a.w; w1 = b.x; w2 = b.y; w3 = b.z; w4 = b.w; break;
  }
  if (!r) return make_uint4(w0, w1, w2, w3);
  return make_uint4(__builtin_amdgcn_alignbit(w1, w0, r), __builtin_amdgcn_alignbit(w2, w1, r),
                    __builtin_amdgcn_alignbit(w3, w2, r), __builtin_amdgcn_alignbit(w4, w3, r));
}

constexpr int kCopyUnroll = 4;

__device__ __forceinline__ void wave_copy_span(const uint8_t* __restrict__ src, uint64_t s0,
                                               uint8_t* __restrict__ dst, uint64_t d0, uint64_t d1,
                                               uint32_t lane) {
  if (d1 <= d0) return;
  const uint64_t a = (d0 + 15) & ~15ull, b = d1 & ~15ull;
  // partial chunks: [d0, min(a, d1)) and, when a <= b, [b, d1)
  const uint64_t head_end = a < d1 ? a : d1;
  if (lane < 16) {
    const uint64_t p = d0 + lane;
    if (p < head_end) dst[p] = src[s0 + (p - d0)];
  } else if (lane < 32 && a <= b) {
    const uint64_t p = b + (lane - 16);
    if (p < d1) dst[p] = src[s0 + (p - d0)];
  }
  if (a >= b) return;
  // full chunks [a, b): the source of chunk A is s0 + (A - d0)
  const uint64_t sa = s0 + (a - d0);
  const uint32_t sh = (uint32_t)(sa & 15);
  const uint8_t* sbase = src + (sa & ~15ull);
  const uint64_t nchunks = (b - a) >> 4;
  for (uint64_t c0 = 0; c0 < nchunks; c0 += 64 * kCopyUnroll) {
    uint4 lo[kCopyUnroll], hi[kCopyUnroll];
#pragma unroll
    for (int k = 0; k < kCopyUnroll; ++k) {
      const uint64_t c = c0 + lane + 64 * k;
      if (c < nchunks) {
        lo[k] = *reinterpret_cast<const uint4*>(sbase + 16 * c);
        hi[k] = sh ? *reinterpret_cast<const uint4*>(sbase + 16 * c + 16) : lo[k];
      }
    }
#pragma unroll
    for (int k = 0; k < kCopyUnroll; ++k) {
      const uint64_t c = c0 + lane + 64 * k;
      if (c < nchunks) *reinterpret_cast<uint4*>(dst + a + 16 * c) = funnel16(lo[k], hi[k], sh);
    }
  }
}

}  // namespace magot
