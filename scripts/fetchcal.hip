// FETCH_SIZE calibration for extract_kernel's genome reads (VERDICT r4 item 3;
// MI355X_MICROARCH.md "HBM": FETCH_SIZE is exact x1/2 only for 16-B-per-lane
// streaming reads, other widths must be calibrated on a known byte count).
//
// extract_kernel reads the nibble plane with buffer_load_dwordx3 (12-byte
// windows at 4-byte aligned offsets) off a scalar buffer descriptor, one
// window per 16-base chunk segment.  Each kernel below issues exactly that
// load over a fresh 1 GiB region (far past the 256 MiB Infinity Cache, with a
// 1 GiB write flush between kernels), in a pattern whose unique bytes and
// 128-byte lines are known:
//   cal_stream12   windows at 12 i: every byte once (streaming, no overlap)
//   cal_overlap8   windows at 8 i: consecutive chunks' windows overlap by 4 B
//                  (the kernel's +strand chunk walk); every byte once
//   cal_line_any   one window in every 3rd 128-B line, anywhere in the line
//   cal_line_lo    ... inside the line's first 64 bytes
//   cal_line_hi    ... inside its second 64 bytes
//   cal_line_cross ... straddling the two 64-byte halves (offset 58)
//   cal_line_pair  two windows in every 3rd line, one in each half
//   cal_b64_stream / cal_b64_line  the same with orf6_kernel's 8-byte
//                  buffer_load_dwordx2 windows (code plane staging)
// Run it under `rocprofv3 --pmc FETCH_SIZE` (and separately under
// --kernel-trace --stats); scripts/fetchcal_summary.py divides each kernel's
// FETCH_SIZE by its known bytes and lines.
//   hipcc -O3 --offload-arch=gfx950 scripts/fetchcal.hip -o scripts/fetchcal.bin
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      printf("%s: %s\n", #x, hipGetErrorString(e));                              \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

constexpr uint64_t kRegion = 1ull << 30;
constexpr uint64_t kLines = kRegion / 128;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const uint8_t* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(p), (short)0, (int)0xFFFFFFFFu,
                                           0x00020000);
}

__device__ __forceinline__ uint32_t win(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b96(r, off, 0, 0);
  return v[0] ^ v[1] ^ v[2];
}

__device__ __forceinline__ uint32_t win8(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
  return v[0] ^ v[1];
}

// mode: 0 stream12, 1 overlap8, 2 line_any, 3 line_lo, 4 line_hi, 5 line_cross, 6 line_pair,
//       7 b64 stream, 8 b64 one per 3rd line
template <int kMode>
__global__ __launch_bounds__(256) void cal(const uint8_t* base, uint64_t n, uint32_t* sink) {
  const __amdgpu_buffer_rsrc_t r = rsrc(base);
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  uint32_t acc;
  if (kMode == 0) {
    acc = win(r, (uint32_t)(12 * i));
  } else if (kMode == 1) {
    acc = win(r, (uint32_t)(8 * i));
  } else if (kMode == 7) {
    acc = win8(r, (uint32_t)(8 * i));
  } else if (kMode == 8) {
    const uint32_t h = (uint32_t)((i * 2654435761ull) >> 7);
    acc = win8(r, (uint32_t)(3 * i) * 128 + 8 * (h % 16));
  } else {
    const uint32_t line = (uint32_t)(3 * i);
    const uint32_t h = (uint32_t)((i * 2654435761ull) >> 7);
    uint32_t o;
    if (kMode == 2) o = 4 * (h % 30);             // 0 .. 116
    else if (kMode == 3) o = 4 * (h % 14);        // 0 .. 52
    else if (kMode == 4) o = 64 + 4 * (h % 14);   // 64 .. 116
    else if (kMode == 5) o = 56 + 4 * (h & 1);    // 56 / 60: crosses byte 64
    else o = 4 * (h % 14);
    acc = win(r, line * 128 + o);
    if (kMode == 6) acc ^= win(r, line * 128 + 64 + 4 * ((h >> 4) % 14));
  }
  if (acc == 0x9E3779B9u) *sink = acc;
}

__global__ __launch_bounds__(256) void flush(uint4* p, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) p[i] = make_uint4((uint32_t)i, 1, 2, 3);
}

template <int kMode>
void run(const char* name, const uint8_t* region, uint64_t n, uint64_t bytes, uint64_t lines,
         uint4* fl, uint32_t* sink) {
  const uint64_t nf = kRegion / 16;
  hipLaunchKernelGGL(flush, dim3((uint32_t)((nf + 255) / 256)), dim3(256), 0, 0, fl, nf);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, 0));
  hipLaunchKernelGGL(cal<kMode>, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, 0, region, n, sink);
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  printf("{\"kernel\": \"%s\", \"mode\": %d, \"windows\": %llu, \"unique_bytes\": %llu, "
         "\"lines_touched\": %llu, \"ms\": %.4f}\n",
         name, kMode, (unsigned long long)n, (unsigned long long)bytes, (unsigned long long)lines,
         ms);
}

int main() {
  uint8_t* buf = nullptr;
  uint32_t* sink = nullptr;
  uint4* fl = nullptr;
  CK(hipMalloc(&buf, 9 * kRegion));
  CK(hipMalloc(&fl, kRegion));
  CK(hipMalloc(&sink, 4));
  CK(hipMemset(buf, 0x5A, 9 * kRegion));
  CK(hipDeviceSynchronize());
  const uint64_t nl = kLines / 3;  // every 3rd line
  run<0>("cal_stream12", buf + 0 * kRegion, kRegion / 12, kRegion / 12 * 12, kLines, fl, sink);
  run<1>("cal_overlap8", buf + 1 * kRegion, kRegion / 8 - 1, kRegion, kLines, fl, sink);
  run<2>("cal_line_any", buf + 2 * kRegion, nl, nl * 12, nl, fl, sink);
  run<3>("cal_line_lo", buf + 3 * kRegion, nl, nl * 12, nl, fl, sink);
  run<4>("cal_line_hi", buf + 4 * kRegion, nl, nl * 12, nl, fl, sink);
  run<5>("cal_line_cross", buf + 5 * kRegion, nl, nl * 12, nl, fl, sink);
  run<6>("cal_line_pair", buf + 6 * kRegion, nl, nl * 24, nl, fl, sink);
  run<7>("cal_b64_stream", buf + 7 * kRegion, kRegion / 8, kRegion, kLines, fl, sink);
  run<8>("cal_b64_line", buf + 8 * kRegion, nl, nl * 8, nl, fl, sink);
  CK(hipDeviceSynchronize());
  return 0;
}
