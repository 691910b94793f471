// Grouped span copies on device: one wave writes a group of consecutive
// pieces of one output range (text and payload parts), dealing its lanes
// across the whole 16-byte chunks and the remaining bytes.  Used by
// segments_copy_kernel (devpack.hip) and the FASTA text assembly (render.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "common.h"

namespace magot {

// ---------------------------------------------------------------------------
// Grouped span copy: one wave writes kSpanGroup consecutive pieces of one
// output range, piece k = a text part [o[k], te[k]) from text + toff[k] then
// a payload part [te[k], o[k+1]) from pay + src[k].  Whole 16-byte chunks
// inside a payload are stored as vectors (a funnel-shifted pair of aligned
// 16-byte loads), everything else byte by byte; lanes are dealt across the
// group's whole chunks and then across its remaining bytes (wave scans of
// the per-piece counts), so every lane's loads are independent.  A chunk
// shared with another piece or group is never stored whole, so every output
// byte is written exactly once.  Used by text_copy_kernel (render.hip) and
// segments_copy_kernel (devpack.hip, no text parts).
// ---------------------------------------------------------------------------
constexpr int kSpanGroup = 16;   // pieces per wave
constexpr int kSpanUnroll = 4;   // whole chunks per lane with their loads in flight together
constexpr int kSpanBytes = 8;    // byte-stored bytes per lane loaded together

struct SpanGroup {
  uint64_t o[kSpanGroup + 1];  // piece starts in the output, and the group's end
  uint64_t te[kSpanGroup];     // end of each piece's text part (its payload's start)
  uint64_t toff[kSpanGroup];   // text part in `text`
  uint64_t src[kSpanGroup];    // payload start in `pay`
  uint64_t fa[kSpanGroup];     // first whole payload chunk (16-byte aligned)
  uint64_t g[kSpanGroup];      // start of the payload's partial tail chunk
  uint32_t hl[kSpanGroup];     // head bytes: text part + payload bytes before fa
  uint32_t fc[kSpanGroup];     // whole chunks of pieces 0..k (inclusive count)
  uint32_t bc[kSpanGroup];     // byte-stored bytes of pieces 0..k (inclusive count)
};

// bytes [sh, sh+16) of the 32-byte concatenation a:b, sh per lane (selects,
// no branches: the chunks of one wave have different misalignments)
__device__ __forceinline__ uint4 funnel16_lane(uint4 a, uint4 b, uint32_t sh) {
  const uint32_t q = sh >> 2, r = 8 * (sh & 3);
  const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  uint32_t v[5];
#pragma unroll
  for (int i = 0; i < 5; ++i)
    v[i] = q == 0 ? w[i] : q == 1 ? w[i + 1] : q == 2 ? w[i + 2] : w[i + 3];
  return make_uint4(__builtin_amdgcn_alignbit(v[1], v[0], r), __builtin_amdgcn_alignbit(v[2], v[1], r),
                    __builtin_amdgcn_alignbit(v[3], v[2], r), __builtin_amdgcn_alignbit(v[4], v[3], r));
}

// number of entries of the non-decreasing c[0..m) that are <= q (m <= kSpanGroup)
__device__ __forceinline__ uint32_t count_le(const uint32_t* c, uint32_t m, uint32_t q) {
  uint32_t pos = 0;
#pragma unroll
  for (uint32_t s = kSpanGroup / 2; s; s >>= 1)
    if (pos + s <= m && c[pos + s - 1] <= q) pos += s;
  return pos;
}

// The group's copy, once L.o[0..m], L.te, L.toff, L.src are staged (m >= 1
// pieces, every lane of the wave active; `text` must be a valid pointer even
// when no piece has a text part)
__device__ __forceinline__ void span_group_copy(SpanGroup& L, uint32_t m,
                                                const uint8_t* __restrict__ text,
                                                const uint8_t* __restrict__ pay,
                                                uint8_t* __restrict__ out, uint32_t lane) {
  // Each unit's bytes: whole 16-byte payload chunks [fa, g), stored as
  // vectors; the rest -- text piece and payload head [o, fa), payload tail
  // [g, e) -- byte by byte.  A chunk shared with another unit or group is
  // never whole, so every output byte is written exactly once.
  uint32_t nf = 0, nb = 0;
  if (lane < m) {
    const uint64_t o = L.o[lane], te = L.te[lane], e = L.o[lane + 1];
    const uint64_t a16 = (te + 15) & ~15ull;
    uint64_t fa = e, g = e;
    if (a16 + 16 <= e) {
      fa = a16;
      g = e & ~15ull;
      nf = (uint32_t)((g - fa) >> 4);
    }
    L.fa[lane] = fa;
    L.g[lane] = g;
    L.hl[lane] = (uint32_t)(fa - o);
    nb = (uint32_t)(fa - o + e - g);
  }
  const uint32_t fc = wave_scan(nf), bc = wave_scan(nb);
  if (lane < m) {
    L.fc[lane] = fc;
    L.bc[lane] = bc;
  }
  const uint32_t n_fast = (uint32_t)__builtin_amdgcn_readlane((int)fc, (int)m - 1);
  const uint32_t n_bytes = (uint32_t)__builtin_amdgcn_readlane((int)bc, (int)m - 1);
  __builtin_amdgcn_wave_barrier();
  // whole chunks, kSpanUnroll per lane with their loads in flight together
  for (uint32_t q0 = 0; q0 < n_fast; q0 += 64 * kSpanUnroll) {
    uint4 lo[kSpanUnroll], hi[kSpanUnroll];
    uint64_t dst[kSpanUnroll];
    uint32_t sh[kSpanUnroll];
#pragma unroll
    for (int j = 0; j < kSpanUnroll; ++j) {
      const uint32_t q = q0 + lane + 64 * j;
      if (q < n_fast) {
        const uint32_t k = count_le(L.fc, m, q);
        const uint64_t C = L.fa[k] + 16ull * (q - (k ? L.fc[k - 1] : 0u));
        const uint64_t sa = L.src[k] + (C - L.te[k]);
        dst[j] = C;
        sh[j] = (uint32_t)(sa & 15);
        const uint8_t* sb = pay + (sa & ~15ull);
        lo[j] = *reinterpret_cast<const uint4*>(sb);
        hi[j] = sh[j] ? *reinterpret_cast<const uint4*>(sb + 16) : lo[j];
      }
    }
#pragma unroll
    for (int j = 0; j < kSpanUnroll; ++j)
      if (q0 + lane + 64 * j < n_fast)
        *reinterpret_cast<uint4*>(out + dst[j]) = funnel16_lane(lo[j], hi[j], sh[j]);
  }
  // the byte-stored bytes, kSpanBytes per lane loaded together
  for (uint32_t i0 = 0; i0 < n_bytes; i0 += 64 * kSpanBytes) {
    const uint8_t* sp[kSpanBytes];
    uint64_t x[kSpanBytes];
#pragma unroll
    for (int j = 0; j < kSpanBytes; ++j) {
      const uint32_t i = i0 + lane + 64 * j;
      sp[j] = nullptr;
      if (i < n_bytes) {
        const uint32_t k = count_le(L.bc, m, i);
        const uint32_t r = i - (k ? L.bc[k - 1] : 0u);
        x[j] = r < L.hl[k] ? L.o[k] + r : L.g[k] + (r - L.hl[k]);
        sp[j] = x[j] < L.te[k] ? text + L.toff[k] + (x[j] - L.o[k])
                               : pay + L.src[k] + (x[j] - L.te[k]);
      }
    }
    uint8_t v[kSpanBytes];
#pragma unroll
    for (int j = 0; j < kSpanBytes; ++j) v[j] = sp[j] ? *sp[j] : 0;
#pragma unroll
    for (int j = 0; j < kSpanBytes; ++j)
      if (sp[j]) out[x[j]] = v[j];
  }
}

}  // namespace magot
