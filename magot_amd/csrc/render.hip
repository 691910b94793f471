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
//   text_copy_kernel one wave per group of kSpanGroup consecutive units (one
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
#include "wavecopy.h"

namespace magot {
namespace {

constexpr int kWave = 64;

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

__global__ __launch_bounds__(256) void text_copy_kernel(
    const TextUnit* __restrict__ units, uint64_t n, const uint64_t* __restrict__ psrc,
    const uint8_t* __restrict__ pay, const uint8_t* __restrict__ text,
    const uint64_t* __restrict__ end, uint8_t* __restrict__ out) {
  __shared__ SpanGroup lds[256 / kWave];
  const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const uint32_t lane = threadIdx.x % kWave;
  const uint64_t u0 = ((uint64_t)blockIdx.x * (256 / kWave) + wv) * kSpanGroup;
  if (u0 >= n) return;
  const uint32_t m = (uint32_t)(n - u0 < kSpanGroup ? n - u0 : kSpanGroup);
  SpanGroup& L = lds[wv];
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
  span_group_copy(L, m, text, pay, out, lane);
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
  const uint64_t groups = (n + kSpanGroup - 1) / kSpanGroup;
  const uint64_t waves_per_block = 256 / kWave;
  text_copy_kernel<<<(unsigned)((groups + waves_per_block - 1) / waves_per_block), 256, 0, s>>>(
      units, n, psrc, pay, text, end, out);
}

}  // namespace magot
