// Write bandwidth of gfx950 by store pattern and size: what rate could
// extract_kernel's 0.80 GB of C3 stores (one wave per 5072 + 1696-byte tile,
// non-temporal 16-byte lane stores, 6 blocks per CU) reach?
//   hipcc -O3 --offload-arch=gfx950 scripts/membench4.hip -o scripts/membench4.bin
//   scripts/membench4.bin > gpurun_out/membench4.txt
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      printf("%s: %s\n", #x, hipGetErrorString(e));                              \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

__device__ __forceinline__ void st16(uint8_t* p, v4u v, bool nt) {
  if (nt) __builtin_nontemporal_store(v, reinterpret_cast<v4u*>(p));
  else *reinterpret_cast<v4u*>(p) = v;
}

// grid-stride 16-byte stores (a fill)
template <bool NT>
__global__ void fill_gs(uint8_t* __restrict__ out, size_t n16) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride)
    st16(out + 16 * i, v4u{(uint32_t)i, 1u, 2u, 3u}, NT);
}

// one wave per tile of `tb` bytes (64 lanes x 16 B per instruction), then a
// second region of `pb` bytes per tile elsewhere (the peptides)
template <bool NT>
__global__ void tiles(uint8_t* __restrict__ nuc, uint8_t* __restrict__ pep, size_t ntiles,
                      uint32_t tb, uint32_t pb) {
  const size_t w = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint32_t lane = threadIdx.x & 63;
  if (w >= ntiles) return;
  uint8_t* o = nuc + w * tb;
  for (uint32_t k = 16 * lane; k < tb; k += 1024) st16(o + k, v4u{k, lane, 7u, (uint32_t)w}, NT);
  uint8_t* q = pep + w * pb;
  for (uint32_t k = 16 * lane; k < pb; k += 1024) st16(q + k, v4u{k, lane, 9u, (uint32_t)w}, NT);
}

int main() {
  const size_t max_bytes = 4ull << 30;
  uint8_t *a, *b;
  CK(hipMalloc(&a, max_bytes));
  CK(hipMalloc(&b, max_bytes / 2));
  CK(hipMemset(a, 0, max_bytes));
  CK(hipMemset(b, 0, max_bytes / 2));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  auto timeit = [&](auto launch, const char* name, double bytes) {
    float ms = 0;
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipEventRecord(e0));
      for (int i = 0; i < 20; ++i) launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
    }
    printf("%-46s %8.4f ms  %6.0f GB/s\n", name, ms / 20, bytes / (ms / 20) / 1e6);
  };
  char nm[96];
  for (size_t mb : {200, 800, 3200}) {
    const size_t bytes = mb << 20, n16 = bytes / 16;
    for (int bpc : {4, 8, 16}) {
      const int grid = ncu * bpc;
      snprintf(nm, sizeof nm, "fill %zu MiB plain grid=%d x256", mb, grid);
      timeit([&] { hipLaunchKernelGGL(fill_gs<false>, grid, 256, 0, 0, a, n16); }, nm, bytes);
      snprintf(nm, sizeof nm, "fill %zu MiB nt    grid=%d x256", mb, grid);
      timeit([&] { hipLaunchKernelGGL(fill_gs<true>, grid, 256, 0, 0, a, n16); }, nm, bytes);
    }
    snprintf(nm, sizeof nm, "hipMemsetAsync %zu MiB", mb);
    timeit([&] { CK(hipMemsetAsync(a, 1, bytes, 0)); }, nm, bytes);
  }
  // C3's tile shape: 118,000 tiles x (5072 + 1696) bytes = 0.80 GB
  const size_t nt = 118000;
  for (uint32_t tb : {5072u, 4992u, 8192u}) {
    const uint32_t pb = tb == 8192u ? 2048u : 1696u;
    const int blocks = (int)((nt * 64 + 255) / 256);
    snprintf(nm, sizeof nm, "tiles %u+%u B plain", tb, pb);
    timeit([&] { hipLaunchKernelGGL(tiles<false>, blocks, 256, 0, 0, a, b, nt, tb, pb); }, nm,
           (double)nt * (tb + pb));
    snprintf(nm, sizeof nm, "tiles %u+%u B nt", tb, pb);
    timeit([&] { hipLaunchKernelGGL(tiles<true>, blocks, 256, 0, 0, a, b, nt, tb, pb); }, nm,
           (double)nt * (tb + pb));
  }
  return 0;
}
