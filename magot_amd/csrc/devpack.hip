// Genome packing on the device, and the reassembly copy of a sharded job's
// gathered outputs.
//
// Packing (magot_genome_load, SURVEY 8(a) a2: GenomeSequence,
// genome.py:854-877 -- every byte except CR/LF, case kept).  The raw contig
// bytes are streamed into HBM once, concatenated in global coordinate order
// (raw index i = global coordinate kOrigin + i, common.h), and three passes
// over them build what pack.cpp builds on the host:
//   run_count_kernel  per 32 raw bytes: how many exception runs start there
//                     (a run = maximal stretch of one byte outside ACGTacgt)
//   (rocPRIM exclusive scan of the counts)
//   run_write_kernel  the start, end and byte of every run, at scanned slots
//   nib_pack_kernel   the forward nibble plane: 4 words (32 bases) per lane,
//                     one 32-byte load, the byte -> nibble map from LDS
// The host turns the (few) run ends into the ExcRun list and its directory
// (pack.cpp: exc_runs_directory) and the mirror kernel fills the reverse
// strand.  HBM-bound byte work: ~1 B read + 0.5 B written per base.
//
// Reassembly (magot_copy_segments): after an RCCL gather of every
// rank's outputs into one buffer, dst is the job's output in global record
// order, a concatenation of n segments each copied from anywhere in src.
// One wave per group of 16 segments (wavecopy.h span_group_copy): whole
// 16-byte destination chunks from funnel-shifted pairs of aligned 16-byte
// source blocks, the partial chunks at the segments' ends byte by byte.
#include <rocprim/device/device_scan.hpp>

#include "common.h"
#include "wavecopy.h"

namespace magot {
namespace {

constexpr int kPackThreads = 256;

// nibble of a raw byte (pack.cpp ByteClass): ACGT -> code, acgt -> code | 4,
// anything else -> 8 | literal class
__device__ __forceinline__ uint32_t nibble_of(uint32_t b) {
  const uint32_t lo = b | 0x20u;
  const uint32_t code = lo == 'a' ? 0u : lo == 'c' ? 1u : lo == 'g' ? 2u : lo == 't' ? 3u : 4u;
  if (code < 4u) return code | ((b & 0x20u) >> 3);
  return 8u | lit_class(b);
}

__device__ __forceinline__ void fill_nibble_table(uint8_t* tbl) {
  for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) tbl[i] = (uint8_t)nibble_of(i);
  __syncthreads();
}

// 32 raw bytes [32t, 32t+32) of a buffer of n bytes, zero past the end (the
// staging buffer is padded to a multiple of 32, so the vector load stays in it).
__device__ __forceinline__ void load32(const uint8_t* raw, uint64_t n, uint64_t t, uint32_t w[8]) {
  const uint4* p = reinterpret_cast<const uint4*>(raw + 32 * t);
  const uint4 a = p[0], b = p[1];
  w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
  w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
  const uint64_t have = n > 32 * t ? n - 32 * t : 0;
  if (have < 32) {
#pragma unroll
    for (int k = 0; k < 32; ++k)
      if ((uint64_t)k >= have) w[k >> 2] &= ~(0xFFu << (8 * (k & 3)));
  }
}

__device__ __forceinline__ uint32_t byte_at(const uint32_t w[8], int k) {
  return (w[k >> 2] >> (8 * (k & 3))) & 0xFFu;
}

// Bit k set: raw byte 32t+k starts (ends) an exception run.  *open_in: a run
// that started before byte 32t is still open at it.
__device__ __forceinline__ void run_masks(const uint8_t* tbl, const uint8_t* raw, uint64_t n,
                                          uint64_t t, uint32_t* starts, uint32_t* ends,
                                          uint32_t* open_in) {
  uint32_t w[8];
  load32(raw, n, t, w);
  const uint64_t i0 = 32 * t;
  const uint32_t prev = i0 > 0 && i0 - 1 < n ? raw[i0 - 1] : 0x100u;     // no byte: differs
  const uint32_t next = i0 + 32 < n ? raw[i0 + 32] : 0x100u;
  uint32_t s = 0, e = 0;
#pragma unroll
  for (int k = 0; k < 32; ++k) {
    if (i0 + k >= n) break;
    const uint32_t b = byte_at(w, k);
    if (!(tbl[b] & 8u)) continue;
    const uint32_t bp = k ? byte_at(w, k - 1) : prev;
    const uint32_t bn = k < 31 ? (i0 + k + 1 < n ? byte_at(w, k + 1) : 0x100u) : next;
    if (bp != b) s |= 1u << k;
    if (bn != b) e |= 1u << k;
  }
  *starts = s;
  *ends = e;
  *open_in = (prev < 0x100u && (tbl[prev] & 8u) && prev == byte_at(w, 0)) ? 1u : 0u;
}

__global__ __launch_bounds__(kPackThreads) void run_count_kernel(const uint8_t* __restrict__ raw,
                                                                 uint64_t n, uint64_t n_groups,
                                                                 uint32_t* __restrict__ count) {
  __shared__ uint8_t tbl[256];
  fill_nibble_table(tbl);
  const uint64_t t = (uint64_t)blockIdx.x * kPackThreads + threadIdx.x;
  if (t >= n_groups) return;
  uint32_t s, e, open_in;
  run_masks(tbl, raw, n, t, &s, &e, &open_in);
  count[t] = __popc(s);
}

__global__ __launch_bounds__(kPackThreads) void run_write_kernel(
    const uint8_t* __restrict__ raw, uint64_t n, uint64_t n_groups,
    const uint64_t* __restrict__ slot, uint64_t* __restrict__ run_start,
    uint64_t* __restrict__ run_end, uint8_t* __restrict__ run_byte) {
  __shared__ uint8_t tbl[256];
  fill_nibble_table(tbl);
  const uint64_t t = (uint64_t)blockIdx.x * kPackThreads + threadIdx.x;
  if (t >= n_groups) return;
  uint32_t s, e, open_in;
  run_masks(tbl, raw, n, t, &s, &e, &open_in);
  if (!(s | e)) return;
  // starts and ends pair up in order (runs never overlap): the k-th start and
  // the k-th end are one run, so the ends of this group are numbered from the
  // starts before it minus the run still open when it begins
  const uint64_t first = slot[t];
  uint64_t ks = first, ke = first - open_in;
  const uint64_t i0 = 32 * t;
  while (s) {
    const int k = __builtin_ctz(s);
    s &= s - 1;
    run_start[ks] = kOrigin + i0 + k;
    run_byte[ks] = raw[i0 + k];
    ++ks;
  }
  while (e) {
    const int k = __builtin_ctz(e);
    e &= e - 1;
    run_end[ke++] = kOrigin + i0 + k + 1;
  }
}

// Forward nibble plane word group t: global bases [32t, 32t+32) = raw bytes
// [32t - kOrigin, 32t + 32 - kOrigin); bases outside the raw range are 0.
__global__ __launch_bounds__(kPackThreads) void nib_pack_kernel(const uint8_t* __restrict__ raw,
                                                                uint64_t n, uint64_t n_groups,
                                                                uint32_t* __restrict__ nib) {
  __shared__ uint8_t tbl[256];
  fill_nibble_table(tbl);
  const uint64_t t = (uint64_t)blockIdx.x * kPackThreads + threadIdx.x;
  if (t >= n_groups) return;
  static_assert(kOrigin % 32 == 0, "raw groups align with plane word groups");
  uint32_t out[4] = {0u, 0u, 0u, 0u};
  if (32 * t >= kOrigin && 32 * t - kOrigin < n) {
    uint32_t w[8];
    load32(raw, n, t - kOrigin / 32, w);
    const uint64_t have = n - (32 * t - kOrigin);
#pragma unroll
    for (int k = 0; k < 32; ++k) {
      const uint32_t v = (uint64_t)k < have ? tbl[byte_at(w, k)] : 0u;
      out[k >> 3] |= v << (4 * (k & 7));
    }
  }
  reinterpret_cast<uint4*>(nib)[t] = make_uint4(out[0], out[1], out[2], out[3]);
}

// ---------------------------------------------------------------------------
// Segment copy
// ---------------------------------------------------------------------------

// one wave per group of kSpanGroup consecutive segments (their destinations
// are one contiguous range: dst_off is a prefix table)
__global__ __launch_bounds__(256) void segments_copy_kernel(const uint8_t* __restrict__ src,
                                                            const uint64_t* __restrict__ src_off,
                                                            const uint64_t* __restrict__ dst_off,
                                                            uint64_t n, uint8_t* __restrict__ dst) {
  __shared__ SpanGroup lds[4];
  const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x / 64);
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t s0 = ((uint64_t)blockIdx.x * 4 + wv) * kSpanGroup;
  if (s0 >= n) return;
  const uint32_t m = (uint32_t)(n - s0 < kSpanGroup ? n - s0 : kSpanGroup);
  SpanGroup& L = lds[wv];
  if (lane < m) {
    const uint64_t o = dst_off[s0 + lane];
    L.o[lane] = o;
    L.te[lane] = o;  // no text parts
    L.toff[lane] = 0;
    L.src[lane] = src_off[s0 + lane];
    if (lane == m - 1) L.o[m] = dst_off[s0 + m];
  }
  __builtin_amdgcn_wave_barrier();
  span_group_copy(L, m, src, src, dst, lane);  // no text parts: `text` is never read
}

}  // namespace

// --- device packing --------------------------------------------------------

size_t devpack_scan_bytes(uint64_t n_groups) {
  size_t bytes = 0;
  (void)rocprim::exclusive_scan(nullptr, bytes, (const uint32_t*)nullptr, (uint64_t*)nullptr,
                                uint64_t(0), (size_t)n_groups, rocprim::plus<uint64_t>(),
                                hipStream_t(0));
  return bytes;
}

hipError_t launch_run_count(const uint8_t* raw, uint64_t n, uint32_t* count, uint64_t* slot,
                            void* scan_tmp, size_t scan_bytes, hipStream_t s) {
  const uint64_t groups = (n + 31) / 32;
  if (!groups) return hipSuccess;
  hipLaunchKernelGGL(run_count_kernel, dim3((uint32_t)((groups + kPackThreads - 1) / kPackThreads)),
                     dim3(kPackThreads), 0, s, raw, n, groups, count);
  if (hipError_t e = hipGetLastError()) return e;
  return rocprim::exclusive_scan(scan_tmp, scan_bytes, count, slot, uint64_t(0), (size_t)groups,
                                 rocprim::plus<uint64_t>(), s);
}

void launch_run_write(const uint8_t* raw, uint64_t n, const uint64_t* slot, uint64_t* run_start,
                      uint64_t* run_end, uint8_t* run_byte, hipStream_t s) {
  const uint64_t groups = (n + 31) / 32;
  if (!groups) return;
  hipLaunchKernelGGL(run_write_kernel, dim3((uint32_t)((groups + kPackThreads - 1) / kPackThreads)),
                     dim3(kPackThreads), 0, s, raw, n, groups, slot, run_start, run_end, run_byte);
}

void launch_nib_pack(const uint8_t* raw, uint64_t n, uint32_t* nib, uint64_t nib_words,
                     hipStream_t s) {
  const uint64_t groups = nib_words / 4;  // nib_words: span / 8, span a multiple of 32
  if (!groups) return;
  hipLaunchKernelGGL(nib_pack_kernel, dim3((uint32_t)((groups + kPackThreads - 1) / kPackThreads)),
                     dim3(kPackThreads), 0, s, raw, n, groups, nib);
}

// --- segment copy ----------------------------------------------------------

void launch_segments_copy(const uint8_t* src, const uint64_t* src_off, const uint64_t* dst_off,
                          uint64_t n, uint8_t* dst, hipStream_t s) {
  if (!n) return;
  const uint64_t groups = (n + kSpanGroup - 1) / kSpanGroup;
  hipLaunchKernelGGL(segments_copy_kernel, dim3((uint32_t)((groups + 3) / 4)), dim3(256), 0, s, src,
                     src_off, dst_off, n, dst);
}

}  // namespace magot
