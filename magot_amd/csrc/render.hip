// FASTA text assembly on device: the gff2fasta output
// ("\n".join of '>'+ID+'\n'+payload records and blank gene lines,
// genome.py:578-582 / 677-731) written into one device buffer from the
// planner's skeleton and the extraction kernel's payloads, so the host does
// one D2H of the final bytes instead of building the text itself.
//
// The skeleton is a list of units: a run of text (headers, joiners) followed
// by at most one record payload.  Three steps on the context stream:
//   text_len_kernel  per unit: text bytes + payload bytes (a protein payload
//                    drops one leading 'X', trimX genome.py:819-821)
//   inclusive scan   unit ends (rocPRIM)
//   text_copy_kernel one wave per unit: the unit's bytes, 8 loads in flight
//                    per lane before the stores
// Byte-granular copies are coalesced by the wave (64 consecutive bytes per
// instruction); the payload reads and text writes are the HBM traffic.
#include <hip/hip_runtime.h>

#include <rocprim/device/device_scan.hpp>

#include "common.h"

namespace magot {
namespace {

constexpr int kWave = 64;
constexpr int kUnroll = 8;

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
                                int protein, uint64_t* __restrict__ len) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const TextUnit u = units[i];
  uint64_t a, pl;
  unit_payload(u, rspan, pay, protein, &a, &pl);
  len[i] = u.text_len + pl;
}

__global__ __launch_bounds__(256) void text_copy_kernel(
    const TextUnit* __restrict__ units, uint64_t n, const uint64_t* __restrict__ rspan,
    const uint8_t* __restrict__ pay, int protein, const uint8_t* __restrict__ text,
    const uint64_t* __restrict__ end, uint8_t* __restrict__ out) {
  // wave index: readfirstlane takes 32 bits, so the (wave-uniform) block part
  // stays 64-bit outside it (units may exceed 2^32 / 4 blocks)
  const uint64_t w = (uint64_t)blockIdx.x * (blockDim.x / kWave) +
                     (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  if (w >= n) return;
  const int lane = threadIdx.x % kWave;
  const TextUnit u = units[w];
  uint64_t a, pl;
  unit_payload(u, rspan, pay, protein, &a, &pl);
  const uint64_t tl = u.text_len;
  const uint64_t total = tl + pl;
  const uint8_t* t = text + u.text_off;
  const uint8_t* p = pay + a - tl;  // p[idx] for idx >= tl
  uint8_t* o = out + (w ? end[w - 1] : 0);
  for (uint64_t base = 0; base < total; base += kWave * kUnroll) {
    uint8_t v[kUnroll];
#pragma unroll
    for (int k = 0; k < kUnroll; ++k) {
      const uint64_t idx = base + lane + kWave * k;
      v[k] = idx < tl ? t[idx] : (idx < total ? p[idx] : 0);
    }
#pragma unroll
    for (int k = 0; k < kUnroll; ++k) {
      const uint64_t idx = base + lane + kWave * k;
      if (idx < total) o[idx] = v[k];
    }
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
                          uint64_t* end, void* scan_tmp, size_t scan_bytes, uint8_t* out,
                          hipStream_t s) {
  if (!n) return;
  text_len_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(units, n, rspan, pay, protein, len);
  (void)rocprim::inclusive_scan(scan_tmp, scan_bytes, len, end, (size_t)n,
                                rocprim::plus<uint64_t>(), s);
  const uint64_t waves_per_block = 256 / kWave;
  text_copy_kernel<<<(unsigned)((n + waves_per_block - 1) / waves_per_block), 256, 0, s>>>(
      units, n, rspan, pay, protein, text, end, out);
}

}  // namespace magot
