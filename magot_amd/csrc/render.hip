// FASTA text assembly on device: the gff2fasta output
// ("\n".join of '>'+ID+'\n'+payload records and blank gene lines,
// genome.py:578-582 / 677-731) written into one device buffer from the
// planner's skeleton and the extraction kernel's payloads, so the host does
// one D2H of the final bytes instead of building the text itself.
//
// The skeleton is a list of units: a run of text (headers, joiners) followed
// by at most one record payload.  Three steps on the context stream:
//   text_len_kernel  per unit: text bytes + payload bytes (a protein payload
//                    drops one leading 'X', trimX genome.py:819-821), and
//                    where its payload starts in the plan's buffer
//   inclusive scan   unit ends (rocPRIM)
//   text_copy_kernel one wave per group of kTextGroup consecutive units (one
//                    contiguous range of the output): the whole 16-byte
//                    chunks inside payloads as funnel-shifted pairs of
//                    16-byte loads and one store each; the text pieces and
//                    the payloads' partial head / tail chunks byte by byte.
//                    Lanes are dealt across the group's chunks and bytes
//                    (wave scans of the per-unit counts), so their loads are
//                    independent; no chunk is stored whole by two waves.
// A wave per unit (round 4) left the copy latency-bound: ~1M waves, each a
// chain of dependent loads for a few hundred bytes.
#include <hip/hip_runtime.h>

#include <rocprim/device/device_scan.hpp>

#include "common.h"

namespace magot {
namespace {

constexpr int kWave = 64;
constexpr int kTextGroup = 16;   // units per wave
constexpr int kTextUnroll = 4;   // whole chunks per lane with their loads in flight together
constexpr int kTextBytes = 8;    // byte-stored bytes per lane loaded together

// rspan: each record's {start, end} in the payload buffer (the plan's layout)
__device__ inline void unit_payload(const TextUnit& u, const uint64_t* rspan, const uint8_t* pay,
                                    int protein, uint64_t* a, uint64_t* len) {
  if (u.rec == kNoRecord) {
    *a = 0;
    *len = 0;
    return;
  }
  uint64_t s = rspan[2 * (uint64_t)u.rec];
  const uint64_t e = rspan[2 * (uint64_t)u.rec + 1];
  if (protein && e > s && pay[s] == 'X') ++s;
  *a = s;
  *len = e - s;
}

__global__ void text_len_kernel(const TextUnit* __restrict__ units, uint64_t n,
                                const uint64_t* __restrict__ rspan, const uint8_t* __restrict__ pay,
                                int protein, uint64_t* __restrict__ len,
                                uint64_t* __restrict__ psrc) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const TextUnit u = units[i];
  uint64_t a, pl;
  unit_payload(u, rspan, pay, protein, &a, &pl);
  len[i] = u.text_len + pl;
  psrc[i] = a;
}

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

struct GroupLds {
  uint64_t o[kTextGroup + 1];  // unit starts in the output, and the group's end
  uint64_t te[kTextGroup];     // end of each unit's text piece (its payload's start)
  uint64_t toff[kTextGroup];   // text piece in the skeleton text
  uint64_t src[kTextGroup];    // payload start in the plan's buffer
  uint64_t fa[kTextGroup];     // first whole payload chunk (16-byte aligned)
  uint64_t g[kTextGroup];      // start of the payload's partial tail chunk
  uint32_t hl[kTextGroup];     // head bytes: text piece + payload bytes before fa
  uint32_t fc[kTextGroup];     // whole chunks of units 0..k (inclusive count)
  uint32_t bc[kTextGroup];     // byte-stored bytes of units 0..k (inclusive count)
};

// number of entries of the non-decreasing c[0..m) that are <= q (m <= 16)
__device__ __forceinline__ uint32_t count_le(const uint32_t* c, uint32_t m, uint32_t q) {
  uint32_t pos = 0;
#pragma unroll
  for (uint32_t s = kTextGroup / 2; s; s >>= 1)
    if (pos + s <= m && c[pos + s - 1] <= q) pos += s;
  return pos;
}

__global__ __launch_bounds__(256) void text_copy_kernel(
    const TextUnit* __restrict__ units, uint64_t n, const uint64_t* __restrict__ psrc,
    const uint8_t* __restrict__ pay, const uint8_t* __restrict__ text,
    const uint64_t* __restrict__ end, uint8_t* __restrict__ out) {
  __shared__ GroupLds lds[256 / kWave];
  const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const uint32_t lane = threadIdx.x % kWave;
  const uint64_t u0 = ((uint64_t)blockIdx.x * (256 / kWave) + wv) * kTextGroup;
  if (u0 >= n) return;
  const uint32_t m = (uint32_t)(n - u0 < kTextGroup ? n - u0 : kTextGroup);
  GroupLds& L = lds[wv];
  if (lane < m) {
    const uint64_t u = u0 + lane;
    const TextUnit t = units[u];
    const uint64_t o = u ? end[u - 1] : 0;
    L.o[lane] = o;
    L.te[lane] = o + t.text_len;
    L.toff[lane] = t.text_off;
    L.src[lane] = psrc[u];
    if (lane == m - 1) L.o[m] = end[u];
  }
  __builtin_amdgcn_wave_barrier();
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
  // whole chunks, kTextUnroll per lane with their loads in flight together
  for (uint32_t q0 = 0; q0 < n_fast; q0 += kWave * kTextUnroll) {
    uint4 lo[kTextUnroll], hi[kTextUnroll];
    uint64_t dst[kTextUnroll];
    uint32_t sh[kTextUnroll];
#pragma unroll
    for (int j = 0; j < kTextUnroll; ++j) {
      const uint32_t q = q0 + lane + kWave * j;
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
    for (int j = 0; j < kTextUnroll; ++j)
      if (q0 + lane + kWave * j < n_fast)
        *reinterpret_cast<uint4*>(out + dst[j]) = funnel16_lane(lo[j], hi[j], sh[j]);
  }
  // the byte-stored bytes, kTextBytes per lane loaded together
  for (uint32_t i0 = 0; i0 < n_bytes; i0 += kWave * kTextBytes) {
    const uint8_t* sp[kTextBytes];
    uint64_t x[kTextBytes];
#pragma unroll
    for (int j = 0; j < kTextBytes; ++j) {
      const uint32_t i = i0 + lane + kWave * j;
      sp[j] = nullptr;
      if (i < n_bytes) {
        const uint32_t k = count_le(L.bc, m, i);
        const uint32_t r = i - (k ? L.bc[k - 1] : 0u);
        x[j] = r < L.hl[k] ? L.o[k] + r : L.g[k] + (r - L.hl[k]);
        sp[j] = x[j] < L.te[k] ? text + L.toff[k] + (x[j] - L.o[k])
                               : pay + L.src[k] + (x[j] - L.te[k]);
      }
    }
    uint8_t v[kTextBytes];
#pragma unroll
    for (int j = 0; j < kTextBytes; ++j) v[j] = sp[j] ? *sp[j] : 0;
#pragma unroll
    for (int j = 0; j < kTextBytes; ++j)
      if (sp[j]) out[x[j]] = v[j];
  }
}

}  // namespace

size_t text_scan_bytes(uint64_t n) {
  size_t bytes = 0;
  (void)rocprim::inclusive_scan(nullptr, bytes, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                (size_t)n, rocprim::plus<uint64_t>(), hipStream_t(0));
  return bytes;
}

void launch_text_assembly(const TextUnit* units, uint64_t n, const uint64_t* rspan,
                          const uint8_t* pay, int protein, const uint8_t* text, uint64_t* len,
                          uint64_t* psrc, uint64_t* end, void* scan_tmp, size_t scan_bytes,
                          uint8_t* out, hipStream_t s) {
  if (!n) return;
  text_len_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(units, n, rspan, pay, protein, len,
                                                               psrc);
  (void)rocprim::inclusive_scan(scan_tmp, scan_bytes, len, end, (size_t)n,
                                rocprim::plus<uint64_t>(), s);
  const uint64_t groups = (n + kTextGroup - 1) / kTextGroup;
  const uint64_t waves_per_block = 256 / kWave;
  text_copy_kernel<<<(unsigned)((groups + waves_per_block - 1) / waves_per_block), 256, 0, s>>>(
      units, n, psrc, pay, text, end, out);
}

}  // namespace magot
