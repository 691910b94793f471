// Write bandwidth of gfx950 by store cache policy: hipMemsetAsync fills at
// 6.5-6.8 TB/s while a plain or non-temporal 16-byte-store fill reaches
// 4.3-4.9 TB/s (membench4).  Which global_store_dwordx4 policy bits
// (nt / sc0 / sc1) and which wave-level address pattern close the gap?
//   hipcc -O3 --offload-arch=gfx950 scripts/membench5.hip -o /tmp/membench5.bin
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

template <int P>
__device__ __forceinline__ void st16(uint8_t* p, v4u v) {
  if constexpr (P == 0) asm volatile("global_store_dwordx4 %0, %1, off" ::"v"(p), "v"(v) : "memory");
  if constexpr (P == 1) asm volatile("global_store_dwordx4 %0, %1, off nt" ::"v"(p), "v"(v) : "memory");
  if constexpr (P == 2) asm volatile("global_store_dwordx4 %0, %1, off sc0" ::"v"(p), "v"(v) : "memory");
  if constexpr (P == 3) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
  if constexpr (P == 4) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
  if constexpr (P == 5) asm volatile("global_store_dwordx4 %0, %1, off nt sc0" ::"v"(p), "v"(v) : "memory");
  if constexpr (P == 6) asm volatile("global_store_dwordx4 %0, %1, off nt sc1" ::"v"(p), "v"(v) : "memory");
  if constexpr (P == 7) asm volatile("global_store_dwordx4 %0, %1, off nt sc0 sc1" ::"v"(p), "v"(v) : "memory");
}
const char* kPol[8] = {"plain", "nt", "sc0", "sc1", "sc0 sc1", "nt sc0", "nt sc1", "nt sc0 sc1"};

// grid-stride fill, 16 B per lane per step
template <int P>
__global__ void fill_gs(uint8_t* __restrict__ out, size_t n16) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride)
    st16<P>(out + 16 * i, v4u{(uint32_t)i, 1u, 2u, 3u});
}

// one wave per tile: C3's extract_kernel shape (5072 nucleotide + 1696 residue bytes)
template <int P>
__global__ void tiles(uint8_t* __restrict__ nuc, uint8_t* __restrict__ pep, size_t ntiles,
                      uint32_t tb, uint32_t pb) {
  const size_t w = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint32_t lane = threadIdx.x & 63;
  if (w >= ntiles) return;
  uint8_t* o = nuc + w * tb;
  for (uint32_t k = 16 * lane; k < tb; k += 1024) st16<P>(o + k, v4u{k, lane, 7u, (uint32_t)w});
  uint8_t* q = pep + w * pb;
  for (uint32_t k = 16 * lane; k < pb; k += 1024) st16<P>(q + k, v4u{k, lane, 9u, (uint32_t)w});
}

int main() {
  const size_t bytes = 3200ull << 20;
  uint8_t *a, *b;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes / 2));
  CK(hipMemset(a, 0, bytes));
  CK(hipMemset(b, 0, bytes / 2));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  auto timeit = [&](auto launch, const char* name, double nbytes) {
    float ms = 0;
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipEventRecord(e0));
      for (int i = 0; i < 20; ++i) launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
    }
    printf("%-46s %8.4f ms  %6.0f GB/s\n", name, ms / 20, nbytes / (ms / 20) / 1e6);
  };
  char nm[96];
  const size_t n16 = bytes / 16;
  if (getenv("MB5_PROBE")) {
    // the box's write path in four numbers: sequential fills vs C3's tiled
    // stream (DESIGN.md 4, C5's two states)
    timeit([&] { CK(hipMemsetAsync(a, 1, bytes, 0)); }, "probe memset 3200 MiB", bytes);
    timeit([&] { hipLaunchKernelGGL(fill_gs<1>, (int)(n16 / 256), 256, 0, 0, a, n16); },
           "probe fill nt one store per lane", bytes);
    const size_t ntl = 118000;
    const int bl = (int)((ntl * 64 + 255) / 256);
    const double tb = (double)ntl * (5072 + 1696);
    timeit([&] { hipLaunchKernelGGL(tiles<1>, bl, 256, 0, 0, a, b, ntl, 5072u, 1696u); },
           "probe C3 tiles 0.80 GB nt", tb);
    timeit([&] { hipLaunchKernelGGL(tiles<0>, bl, 256, 0, 0, a, b, ntl, 5072u, 1696u); },
           "probe C3 tiles 0.80 GB plain", tb);
    return 0;
  }
  timeit([&] { CK(hipMemsetAsync(a, 1, bytes, 0)); }, "hipMemsetAsync 3200 MiB", bytes);
  // grid size sweep of the plain fill (grid-stride), and one store per lane
  for (int bpc : {1, 2, 4, 16, 32, 64, 128}) {
    const int g = ncu * bpc;
    snprintf(nm, sizeof nm, "fill 3200 MiB plain grid=%d x256", g);
    timeit([&] { hipLaunchKernelGGL(fill_gs<0>, g, 256, 0, 0, a, n16); }, nm, bytes);
  }
  snprintf(nm, sizeof nm, "fill 3200 MiB plain one store per lane");
  timeit([&] { hipLaunchKernelGGL(fill_gs<0>, (int)(n16 / 256), 256, 0, 0, a, n16); }, nm, bytes);
  snprintf(nm, sizeof nm, "fill 3200 MiB nt one store per lane");
  timeit([&] { hipLaunchKernelGGL(fill_gs<1>, (int)(n16 / 256), 256, 0, 0, a, n16); }, nm, bytes);
  const int grid = ncu * 8;
#define FILL(P)                                                                              \
  snprintf(nm, sizeof nm, "fill 3200 MiB %s", kPol[P]);                                    \
  timeit([&] { hipLaunchKernelGGL(fill_gs<P>, grid, 256, 0, 0, a, n16); }, nm, bytes);
  FILL(0) FILL(1) FILL(2) FILL(3) FILL(4) FILL(5) FILL(6) FILL(7)
  const size_t nt = 118000;
  const int blocks = (int)((nt * 64 + 255) / 256);
  const double tbytes = (double)nt * (5072 + 1696);
#define TILES(P)                                                                             \
  snprintf(nm, sizeof nm, "C3 tiles 0.80 GB %s", kPol[P]);                                   \
  timeit([&] { hipLaunchKernelGGL(tiles<P>, blocks, 256, 0, 0, a, b, nt, 5072u, 1696u); }, nm, \
         tbytes);
  TILES(0) TILES(1) TILES(2) TILES(3) TILES(4) TILES(5) TILES(6) TILES(7)
  timeit([&] { CK(hipMemsetAsync(a, 1, (size_t)tbytes, 0)); }, "hipMemsetAsync 0.80 GB", tbytes);
  if (getenv("MB5_SIZES")) {
    // the same tile shape at other output sizes: rewriting the same outputs
    // every launch, does a share small enough for the 256 MB Infinity Cache
    // write faster per byte?
    for (size_t tiles_n : {14750ul, 29500ul, 59000ul, 118000ul, 236000ul}) {
      const int bl = (int)((tiles_n * 64 + 255) / 256);
      const double tb = (double)tiles_n * (5072 + 1696);
      snprintf(nm, sizeof nm, "tiles %.2f GB nt", tb / 1e9);
      timeit([&] { hipLaunchKernelGGL(tiles<1>, bl, 256, 0, 0, a, b, tiles_n, 5072u, 1696u); }, nm, tb);
      snprintf(nm, sizeof nm, "tiles %.2f GB plain", tb / 1e9);
      timeit([&] { hipLaunchKernelGGL(tiles<0>, bl, 256, 0, 0, a, b, tiles_n, 5072u, 1696u); }, nm, tb);
    }
  }
  return 0;
}
