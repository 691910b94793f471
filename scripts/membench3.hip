// Write-path calibration on gfx950: plain vs non-temporal 16-byte stores,
// alone and mixed with a scattered 128-B-line read stream in the same kernel.
//   hipcc -O3 --offload-arch=gfx950 scripts/membench3.hip -o scripts/membench3.bin
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void st16(uint4* p, uint4 v, bool nt) {
  v4u x = {v.x, v.y, v.z, v.w};
  if (nt) __builtin_nontemporal_store(x, reinterpret_cast<v4u*>(p));
  else *reinterpret_cast<v4u*>(p) = x;
}

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      printf("%s: %s\n", #x, hipGetErrorString(e));                              \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

template <bool NT>
__global__ void store16(uint4* __restrict__ out, size_t n16) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) {
    const uint4 v = make_uint4((uint32_t)i, 1u, 2u, 3u);
    st16(out + i, v, NT);
  }
}

// one wave = one 3 KB output tile (3 x 1 KB stores) + 12 scattered line reads
template <bool NT>
__global__ void tile_mix(const uint8_t* __restrict__ tab, uint64_t nlines, uint4* __restrict__ out,
                         size_t ntiles, uint32_t* sink) {
  const size_t w = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (w >= ntiles) return;
  uint32_t acc = 0;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const uint64_t line = ((w * 64 + lane) * 2 + k) * 0x9E3779B97F4A7C15ull % nlines;
    const uint3 v = *reinterpret_cast<const uint3*>(tab + line * 128 + 16);
    acc ^= v.x ^ v.y ^ v.z;
  }
  uint4* o = out + w * 256;  // 4 KB per tile (3 KB nuc + 1 KB pep)
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint4 v = make_uint4(acc, lane, k, (uint32_t)w);
    st16(o + k * 64 + lane, v, NT);
  }
  if (acc == 0x12345678u) *sink = acc;
}

int main() {
  const size_t out_bytes = 800ull << 20, tab_bytes = 1ull << 30;
  uint4* out;
  uint8_t* tab;
  uint32_t* sink;
  CK(hipMalloc(&out, out_bytes));
  CK(hipMalloc(&tab, tab_bytes));
  CK(hipMalloc(&sink, 4));
  CK(hipMemset(tab, 1, tab_bytes));
  CK(hipMemset(out, 0, out_bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  const size_t n16 = out_bytes / 16;
  float ms;
  auto timeit = [&](auto launch, const char* name, double bytes) {
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipEventRecord(e0));
      for (int i = 0; i < 10; ++i) launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
    }
    printf("%-34s %.3f ms  %.0f GB/s\n", name, ms / 10, bytes / (ms / 10) / 1e6);
  };
  for (int bpc : {8, 32}) {
    const int grid = ncu * bpc;
    char nm[64];
    snprintf(nm, sizeof nm, "store16 plain grid=%d", grid);
    timeit([&] { hipLaunchKernelGGL(store16<false>, grid, 256, 0, 0, out, n16); }, nm, out_bytes);
    snprintf(nm, sizeof nm, "store16 nontemporal grid=%d", grid);
    timeit([&] { hipLaunchKernelGGL(store16<true>, grid, 256, 0, 0, out, n16); }, nm, out_bytes);
  }
  const size_t ntiles = out_bytes / 4096;
  const int blocks = (int)((ntiles * 64 + 255) / 256);
  // reads: ntiles * 128 lines * 128 B
  const double rbytes = (double)ntiles * 128 * 128;
  timeit([&] { hipLaunchKernelGGL(tile_mix<false>, blocks, 256, 0, 0, tab, tab_bytes / 128, out, ntiles, sink); },
         "tile_mix plain (bytes = W+R lines)", out_bytes + rbytes);
  timeit([&] { hipLaunchKernelGGL(tile_mix<true>, blocks, 256, 0, 0, tab, tab_bytes / 128, out, ntiles, sink); },
         "tile_mix nontemporal", out_bytes + rbytes);
  return 0;
}
