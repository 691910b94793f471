// The compact replica image of a packed genome: what crosses xGMI when a
// multi-GPU job broadcasts its genome (the north star's "2-bit
// packed genome ... RCCL-broadcast").  GenomeSequence (genome.py:854-877)
// keeps every byte of the FASTA; the image keeps them all in about 0.27 B
// per base instead of the arena's 1 B:
//
//   header  WireHeader (below)
//   code2   the forward strand's 2-bit codes, 16 bases per u32 (the
//           code2_kernel layout, seqops.hip): 0.25 B per base
//   mask    the soft-masked (lower-case acgt) bases as maximal runs
//           {start, end} (u32 pairs, sorted, then a sentinel {~0, ~0})
//   mdir    one u32 per 4096 bases: the first mask run ending past the
//           block start
//   exc     the arena's exception runs + their directory, verbatim (every
//           byte outside ACGTacgt, with its literal)
//
// Sender (magot_genome_wire_export): code2_kernel over the forward plane,
// wire_count_kernel + a rocPRIM scan + wire_runs_kernel for the mask runs
// (the same start/end pairing as devpack's exception runs), wire_mdir_kernel.
// Receiver (magot_genome_wire_import): wire_unpack_kernel rebuilds the
// forward nibble plane -- 32 bases per lane: 8 bytes of codes spread to
// nibbles, the mask runs and exception runs overlapping the lane's bases
// found through the two directories -- then the mirror kernel derives the
// reverse strand, as after a local pack.  All HBM-bound byte work.
#include <rocprim/device/device_scan.hpp>

#include "common.h"

namespace magot {
namespace {

constexpr int kWireThreads = 256;

// bit k = base 32t+k of the 4 nibble words is soft-masked: nibble bit 2 set
// and bit 3 (exception) clear
__device__ __forceinline__ uint32_t mask_bits(uint4 x) {
  const uint32_t v[4] = {x.x, x.y, x.z, x.w};
  uint32_t out = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint32_t y = ((v[q] >> 2) & ~(v[q] >> 3)) & 0x11111111u;  // bits 0, 4, .., 28
    y = (y | (y >> 3)) & 0x03030303u;
    y = (y | (y >> 6)) & 0x000F000Fu;
    y = (y | (y >> 12)) & 0xFFu;
    out |= y << (8 * q);
  }
  return out;
}

__device__ __forceinline__ uint32_t nib_masked(uint32_t word, int k) {
  return ((word >> (4 * k)) & 0xCu) == 0x4u ? 1u : 0u;
}

// starts / ends of mask runs among bases [32t, 32t+32); *open_in: a run is
// open across the group's left edge
__device__ __forceinline__ void mask_edges(const uint32_t* __restrict__ nib, uint64_t groups,
                                           uint64_t t, uint32_t* starts, uint32_t* ends,
                                           uint32_t* open_in) {
  const uint32_t m = mask_bits(reinterpret_cast<const uint4*>(nib)[t]);
  const uint32_t prev = t ? nib_masked(nib[4 * t - 1], 7) : 0u;
  const uint32_t next = t + 1 < groups ? nib_masked(nib[4 * t + 4], 0) : 0u;
  *starts = m & ~((m << 1) | prev);
  *ends = m & ~((m >> 1) | (next << 31));
  *open_in = prev & m & 1u;
}

__global__ __launch_bounds__(kWireThreads) void wire_count_kernel(const uint32_t* __restrict__ nib,
                                                                  uint64_t groups,
                                                                  uint32_t* __restrict__ count) {
  const uint64_t t = (uint64_t)blockIdx.x * kWireThreads + threadIdx.x;
  if (t >= groups) return;
  uint32_t s, e, o;
  mask_edges(nib, groups, t, &s, &e, &o);
  count[t] = __popc(s);
}

__global__ __launch_bounds__(kWireThreads) void wire_runs_kernel(const uint32_t* __restrict__ nib,
                                                                 uint64_t groups,
                                                                 const uint64_t* __restrict__ slot,
                                                                 uint32_t* __restrict__ runs) {
  const uint64_t t = (uint64_t)blockIdx.x * kWireThreads + threadIdx.x;
  if (t >= groups) return;
  uint32_t s, e, o;
  mask_edges(nib, groups, t, &s, &e, &o);
  if (!(s | e)) return;
  // the k-th start and the k-th end are one run (runs never overlap)
  uint64_t ks = slot[t], ke = slot[t] - o;
  const uint32_t b0 = (uint32_t)(32 * t);
  while (s) {
    runs[2 * ks++] = b0 + (uint32_t)__builtin_ctz(s);
    s &= s - 1;
  }
  while (e) {
    runs[2 * ke++ + 1] = b0 + (uint32_t)__builtin_ctz(e) + 1u;
    e &= e - 1;
  }
}

// mdir[b] = first run r (of n, sentinel at n) with end > 4096 b
__global__ __launch_bounds__(kWireThreads) void wire_mdir_kernel(const uint32_t* __restrict__ runs,
                                                                 uint64_t n, uint64_t n_blocks,
                                                                 uint32_t* __restrict__ mdir) {
  const uint64_t b = (uint64_t)blockIdx.x * kWireThreads + threadIdx.x;
  if (b >= n_blocks) return;
  const uint64_t bs = b << kDirShift;
  uint64_t lo = 0, hi = n;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if ((uint64_t)runs[2 * mid + 1] > bs) hi = mid; else lo = mid + 1;
  }
  mdir[b] = (uint32_t)lo;
}

// 8 two-bit codes (bits 2k) -> 8 nibbles (bits 4k)
__device__ __forceinline__ uint32_t spread2(uint32_t x) {
  x &= 0xFFFFu;
  x = (x | (x << 8)) & 0x00FF00FFu;
  x = (x | (x << 4)) & 0x0F0F0F0Fu;
  return (x | (x << 2)) & 0x33333333u;
}

// 8 bits -> bit k at bit 4k
__device__ __forceinline__ uint32_t spread1(uint32_t x) {
  x &= 0xFFu;
  x = (x | (x << 12)) & 0x000F000Fu;
  x = (x | (x << 6)) & 0x03030303u;
  return (x | (x << 3)) & 0x11111111u;
}

// bits [a, b) of a 32-bit mask, 0 <= a < b <= 32
__device__ __forceinline__ uint32_t bit_range(uint32_t a, uint32_t b) {
  const uint32_t hi = b >= 32 ? 0xFFFFFFFFu : ((1u << b) - 1u);
  return hi & ~((1u << a) - 1u);
}

struct UnpackArgs {
  const uint2* code2;       // 2 words (32 bases) per group
  const uint32_t* mask;     // {start, end} pairs, sentinel at n_mask
  const uint32_t* mdir;
  uint64_t n_mdir;
  uint64_t n_mask;
  const ExcRun* exc;        // sentinel at n_exc
  const uint32_t* edir;
  uint64_t n_edir;
  uint64_t n_exc;
  uint64_t groups;          // span / 32
  uint4* nib;               // forward plane, 4 words per group
};

__global__ __launch_bounds__(kWireThreads) void wire_unpack_kernel(UnpackArgs a) {
  const uint64_t t = (uint64_t)blockIdx.x * kWireThreads + threadIdx.x;
  if (t >= a.groups) return;
  const uint64_t lo = 32 * t, hi = lo + 32;
  const uint64_t blk = lo >> kDirShift;
  const uint2 c = a.code2[t];
  uint32_t w[4] = {spread2(c.x), spread2(c.x >> 16), spread2(c.y), spread2(c.y >> 16)};

  // soft-mask: the first run ending past lo lies in [mdir[blk], mdir[blk+1]]
  // (directory entries clamped to the run count: a corrupt image whose header
  // matches the genome reads no run past the list's sentinel)
  {
    uint64_t r0 = min((uint64_t)a.mdir[blk], a.n_mask);
    uint64_t r1 = blk + 1 < a.n_mdir ? min((uint64_t)a.mdir[blk + 1], a.n_mask) : a.n_mask;
    while (r0 < r1) {
      const uint64_t mid = (r0 + r1) >> 1;
      if ((uint64_t)a.mask[2 * mid + 1] > lo) r1 = mid; else r0 = mid + 1;
    }
    uint32_t m = 0;
    for (uint64_t r = r0; r < a.n_mask; ++r) {
      const uint64_t s = a.mask[2 * r], e = a.mask[2 * r + 1];
      if (s >= hi) break;
      m |= bit_range((uint32_t)((s > lo ? s : lo) - lo), (uint32_t)((e < hi ? e : hi) - lo));
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) w[j] |= spread1(m >> (8 * j)) << 2;
  }
  // exceptions: the literal class of every byte outside ACGTacgt (nibble 8 | class)
  const uint32_t d = a.edir[blk];
  if (!(d & kDirClean)) {
    uint64_t r0 = min((uint64_t)(d & ~kDirClean), a.n_exc);
    uint64_t r1 = blk + 1 < a.n_edir ? min((uint64_t)(a.edir[blk + 1] & ~kDirClean), a.n_exc)
                                     : a.n_exc;
    while (r0 < r1) {
      const uint64_t mid = (r0 + r1) >> 1;
      if (a.exc[mid].start + a.exc[mid].len > lo) r1 = mid; else r0 = mid + 1;
    }
    for (uint64_t r = r0; r < a.n_exc; ++r) {
      const ExcRun x = a.exc[r];
      if (x.start >= hi) break;
      const uint64_t e = x.start + x.len;
      const uint32_t m = bit_range((uint32_t)((x.start > lo ? x.start : lo) - lo),
                                   (uint32_t)((e < hi ? e : hi) - lo));
      const uint32_t v = (8u | lit_class(x.byte)) * 0x11111111u;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t nm = spread1(m >> (8 * j)) * 0xFu;
        w[j] = (w[j] & ~nm) | (v & nm);
      }
    }
  }
  a.nib[t] = make_uint4(w[0], w[1], w[2], w[3]);
}

}  // namespace

size_t wire_scan_bytes(uint64_t groups) {
  size_t bytes = 0;
  (void)rocprim::exclusive_scan(nullptr, bytes, (const uint32_t*)nullptr, (uint64_t*)nullptr,
                                uint64_t(0), (size_t)groups, rocprim::plus<uint64_t>(),
                                hipStream_t(0));
  return bytes;
}

hipError_t launch_wire_count(const uint32_t* nib, uint64_t span, uint32_t* count, uint64_t* slot,
                             void* scan_tmp, size_t scan_bytes, hipStream_t s) {
  const uint64_t groups = span / 32;
  if (!groups) return hipSuccess;
  hipLaunchKernelGGL(wire_count_kernel, dim3((uint32_t)((groups + kWireThreads - 1) / kWireThreads)),
                     dim3(kWireThreads), 0, s, nib, groups, count);
  if (hipError_t e = hipGetLastError()) return e;
  return rocprim::exclusive_scan(scan_tmp, scan_bytes, count, slot, uint64_t(0), (size_t)groups,
                                 rocprim::plus<uint64_t>(), s);
}

void launch_wire_runs(const uint32_t* nib, uint64_t span, const uint64_t* slot, uint32_t* runs,
                      hipStream_t s) {
  const uint64_t groups = span / 32;
  if (!groups) return;
  hipLaunchKernelGGL(wire_runs_kernel, dim3((uint32_t)((groups + kWireThreads - 1) / kWireThreads)),
                     dim3(kWireThreads), 0, s, nib, groups, slot, runs);
}

void launch_wire_mdir(const uint32_t* runs, uint64_t n, uint64_t n_blocks, uint32_t* mdir,
                      hipStream_t s) {
  if (!n_blocks) return;
  hipLaunchKernelGGL(wire_mdir_kernel, dim3((uint32_t)((n_blocks + kWireThreads - 1) / kWireThreads)),
                     dim3(kWireThreads), 0, s, runs, n, n_blocks, mdir);
}

void launch_wire_unpack(const uint32_t* code2, const uint32_t* mask, uint64_t n_mask,
                        const uint32_t* mdir, uint64_t n_mdir, const ExcRun* exc, uint64_t n_exc,
                        const uint32_t* edir, uint64_t n_edir, uint64_t span, uint32_t* nib,
                        hipStream_t s) {
  UnpackArgs a;
  a.code2 = reinterpret_cast<const uint2*>(code2);
  a.mask = mask;
  a.mdir = mdir;
  a.n_mdir = n_mdir;
  a.n_mask = n_mask;
  a.exc = exc;
  a.edir = edir;
  a.n_edir = n_edir;
  a.n_exc = n_exc;
  a.groups = span / 32;
  a.nib = reinterpret_cast<uint4*>(nib);
  if (!a.groups) return;
  hipLaunchKernelGGL(wire_unpack_kernel, dim3((uint32_t)((a.groups + kWireThreads - 1) / kWireThreads)),
                     dim3(kWireThreads), 0, s, a);
}

}  // namespace magot
