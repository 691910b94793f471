// Does the HBM write rate of a tiled store stream depend on the address window
// the resident waves write into?  One wave per tile of T bytes (16-byte lane
// stores, optionally idling between stores: the compute of a real kernel),
// blocks dispatched in order so the resident waves hold consecutive tiles,
// residency capped by untouched dynamic LDS.  Window = resident waves x T.
// Output 0.8 / 4.9 GB per launch.
//   hipcc -O3 --offload-arch=gfx950 scripts/membench6.hip -o /tmp/membench6.bin
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

template <bool NT>
__device__ __forceinline__ void st16(uint8_t* p, v4u v) {
  if constexpr (NT) __builtin_nontemporal_store(v, reinterpret_cast<v4u*>(p));
  else *reinterpret_cast<v4u*>(p) = v;
}

// one wave per block and tile, blocks dispatched in order: the resident waves
// hold consecutive tiles; dynamic LDS the kernel never touches caps how many
// waves a CU holds
template <bool NT, int SLEEP>
__global__ __launch_bounds__(64) void tiles_lds(uint8_t* __restrict__ out, unsigned tb) {
  const unsigned lane = threadIdx.x, t = blockIdx.x;
  uint8_t* o = out + (size_t)t * tb;
  for (unsigned k = 16 * lane; k < tb; k += 1024) {
    st16<NT>(o + k, v4u{k, lane, 7u, t});
    if constexpr (SLEEP > 0) __builtin_amdgcn_s_sleep(SLEEP);
  }
}

int main() {
  const size_t bytes = 5000ull << 20;
  uint8_t* a;
  CK(hipMalloc(&a, bytes));
  CK(hipMemset(a, 0, bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](auto launch, const char* name, double nbytes) {
    float ms = 0;
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipEventRecord(e0));
      for (int i = 0; i < 10; ++i) launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
    }
    printf("%-52s %8.4f ms  %6.0f GB/s\n", name, ms / 10, nbytes / (ms / 10) / 1e6);
    fflush(stdout);
  };
  char nm[128];
  timeit([&] { CK(hipMemsetAsync(a, 1, 800u << 20, 0)); }, "hipMemsetAsync 0.84 GB", 800u << 20);
  CK(hipFuncSetAttribute((const void*)tiles_lds<false, 0>,
                         hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  CK(hipFuncSetAttribute((const void*)tiles_lds<true, 0>,
                         hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  CK(hipFuncSetAttribute((const void*)tiles_lds<true, 8>,
                         hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  for (size_t total : {800ull << 20, 4700ull << 20}) {
    for (unsigned tb : {2048u, 8192u, 32768u}) {
      const unsigned nt = (unsigned)(total / tb);
      for (int per_cu : {2, 4, 8, 16, 32}) {
        // LDS per one-wave block so that at most per_cu fit a CU's 160 KB
        const unsigned lds = per_cu >= 32 ? 0 : ((160u * 1024u) / per_cu & ~511u) - 512u * (per_cu > 2);
        const int waves = 256 * per_cu;
#define RUN(NT, S, tag)                                                                       \
  snprintf(nm, sizeof nm, "%.2f GB T=%5u waves/CU=%2d win=%6.1f MB %s", total / 1e9, tb,    \
           per_cu, waves * (double)tb / 1e6, tag);                                            \
  timeit([&] { hipLaunchKernelGGL((tiles_lds<NT, S>), nt, 64, lds, 0, a, tb); }, nm,         \
         (double)nt * tb);
        RUN(false, 0, "plain")
        RUN(true, 0, "nt")
        if (total < (1ull << 30)) { RUN(true, 8, "nt sleep8") }
      }
    }
  }
  return 0;
}
