// Speed-of-light replays of the two measured kernels' memory traffic, with
// no decode work: what the memory system gives a launch of the same shape
// (waves, bytes written per wave and how, line fills per wave), so a kernel's
// time can be read against what its own bytes allow and not only against the
// 8 TB/s spec peak.
//   hipcc -O3 --offload-arch=gfx950 scripts/solbench.hip -o /tmp/solbench
//
// c3: one wave per extraction tile (C3: 118,356 tiles of 5072 nucleotide
//     bytes + their residues, 16-B-aligned and contiguous, non-temporal
//     16-B stores as extract_kernel; L scattered 12-B window loads over the
//     two 1-GB nibble planes, each one 128-B line fill; 6 blocks of 4 waves
//     per CU as the launch cap).
// c5: one wave per orf6 tile (605,096 tiles): R residue bytes per wave in
//     runs of one record's six streams (~2.1 KB) at scattered 16-B-aligned
//     places (the genome-order walk writes records in an order unrelated to
//     their output offsets), plain 16-B stores, one store per lane per
//     pass as orf6_kernel's chunk loop; L line fills per wave from a 1.5-GB
//     code plane, walked in genome order (neighbouring tiles read
//     neighbouring lines).  Variants: runs written sequentially (the
//     record-order walk), inside a moving 25-MB window (one contig's records,
//     genome-order walk), scattered over the whole output.
// c5 chain: the same stores after 1, 3 or 5 dependent load round trips per
//     wave (staging's shape), with loads and stores in the same or in
//     separate waves, and with extra load instructions per round.
// c5 now: the chain over round 4's layout and block order.
// c3now: the C3 launch with its records laid out in genome order (round 5):
//     35 line fills per tile (0.53 GB per launch, PMC), tile w's lines
//     following tile w-1's, the same stores.
//   usage: solbench c3 | solbench c3now | solbench c5 [chain | now]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      printf("%s: %s\n", #x, hipGetErrorString(e));                              \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  return x ^ (x >> 33);
}

__device__ __forceinline__ void st16(uint8_t* p, uint4 v, bool nt) {
  v4u x = {v.x, v.y, v.z, v.w};
  if (nt) __builtin_nontemporal_store(x, reinterpret_cast<v4u*>(p));
  else *reinterpret_cast<v4u*>(p) = x;
}

struct C3Args {
  const uint8_t* plane;
  uint64_t plane_lines;
  uint8_t* nuc;
  uint8_t* pep;
  uint32_t ntiles, lines, nuc_bytes, pep_bytes;
  uint32_t* sink;
  uint32_t win_tiles;     // reads: inside a moving window (one contig) of this many tiles (0: anywhere)
  uint64_t win_lines;     // lines per window
  uint32_t seq;           // reads walk the planes in tile order (genome-order layout)
};

__global__ __launch_bounds__(256) void c3_replay(C3Args a) {
  const uint64_t w = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (w >= a.ntiles) return;
  uint32_t acc = 0;
  // scattered window loads, all in flight at once
  uint3 v[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const uint32_t l = lane + 64 * k;
    const uint64_t line = a.seq ? (w * a.lines + l) % a.plane_lines
                          : a.win_tiles ? ((w / a.win_tiles) * a.win_lines + mix(w * 256 + l) % a.win_lines) % a.plane_lines
                                      : mix(w * 256 + l) % a.plane_lines;
    v[k] = l < a.lines ? *reinterpret_cast<const uint3*>(a.plane + line * 128 + 16 * (l & 7))
                       : make_uint3(0, 0, 0);
  }
#pragma unroll
  for (int k = 0; k < 2; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z;
  // nucleotide chunks, 5 slots per lane, then the residue chunks
  uint8_t* const n0 = a.nuc + w * a.nuc_bytes;
#pragma unroll
  for (int s = 0; s < 5; ++s) {
    const uint32_t c = 64 * s + lane;
    if (16 * c < a.nuc_bytes) st16(n0 + 16 * c, make_uint4(acc, c, s, (uint32_t)w), true);
  }
  uint8_t* const p0 = a.pep + w * a.pep_bytes;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const uint32_t c = 64 * s + lane;
    if (16 * c < a.pep_bytes) st16(p0 + 16 * c, make_uint4(acc, c, s, (uint32_t)w), true);
  }
  if (acc == 0x12345678u) *a.sink = acc;
}

// store-only variants of C3's output stream: each wave writes `per_wave`
// consecutive tiles (nuc then pep per tile), nt or plain 16-B stores, in
// the launch's XCD runs of `xrun` blocks (0: hardware round-robin)
template <bool kNt>
__global__ __launch_bounds__(256) void c3_stores(uint8_t* nuc, uint8_t* pep, uint32_t ntiles,
                                                 uint32_t nuc_bytes, uint32_t pep_bytes,
                                                 uint32_t per_wave, uint32_t xrun) {
  uint32_t vb = blockIdx.x;
  if (xrun) {
    // runs of xrun consecutive blocks per XCD (extract_kernel's kXcdRun order)
    const uint32_t nb = gridDim.x, xcd = vb & 7, k = vb >> 3;
    const uint32_t run = k / xrun, in = k % xrun;
    const uint32_t v = (run * 8 + xcd) * xrun + in;
    vb = v < nb ? v : vb;
  }
  const uint64_t w = (uint64_t)vb * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  for (uint32_t j = 0; j < per_wave; ++j) {
    const uint64_t t = w * per_wave + j;
    if (t >= ntiles) return;
    uint8_t* const n0 = nuc + t * nuc_bytes;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const uint32_t c = 64 * s + lane;
      if (16 * c < nuc_bytes) st16(n0 + 16 * c, make_uint4(c, s, (uint32_t)t, 1), kNt);
    }
    uint8_t* const p0 = pep + t * pep_bytes;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const uint32_t c = 64 * s + lane;
      if (16 * c < pep_bytes) st16(p0 + 16 * c, make_uint4(c, s, (uint32_t)t, 2), kNt);
    }
  }
}

// flat store streams over one buffer (what a fill kernel does): grid-stride
// 16-byte stores, consecutive lanes on consecutive chunks (kLanes64 false), or
// each lane writing 64 consecutive bytes as four stores (true)
template <bool kLanes64, bool kNt>
__global__ __launch_bounds__(256) void flat_stores(uint8_t* p, uint64_t chunks) {
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t nthr = (uint64_t)gridDim.x * blockDim.x;
  if (!kLanes64) {
    for (uint64_t c = tid; c < chunks; c += nthr)
      st16(p + 16 * c, kNt ? make_uint4((uint32_t)c, 1, 2, 3)
                           : make_uint4(0x07070707u, 0x07070707u, 0x07070707u, 0x07070707u),
           kNt);
  } else {
    for (uint64_t c = 4 * tid; c < chunks; c += 4 * nthr)
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (c + k < chunks) st16(p + 16 * (c + k), make_uint4((uint32_t)c, k, 2, 3), kNt);
  }
}

struct C5Args {
  const uint8_t* plane;
  uint64_t plane_lines;
  uint8_t* out;
  uint64_t out_runs;  // run slots of run_bytes in the output
  uint32_t ntiles, lines, run_bytes, runs;
  uint32_t* sink;
  uint32_t win_tiles;  // scattered runs: within the output window of this many tiles (0: anywhere)
};

// kSeq: runs laid out in walk order (tile w's runs follow tile w-1's), as
// the record-order walk writes; else scattered (genome-order walk)
template <bool kSeq, bool kNt>
__global__ __launch_bounds__(256) void c5_replay(C5Args a) {
  const uint32_t xnb = gridDim.x, xb = blockIdx.x;
  const uint32_t xq = xnb >> 3, xr = xnb & 7, xcd = xb & 7, xk = xb >> 3;
  const uint32_t vb = xcd < xr ? xcd * (xq + 1) + xk : xr * (xq + 1) + (xcd - xr) * xq + xk;
  const uint64_t w = (uint64_t)vb * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (w >= a.ntiles) return;
  // genome-order reads: tile w's lines follow tile w-1's
  uint32_t acc = 0;
  {
    const uint32_t l = lane;
    const uint64_t line = (w * a.lines + l) % a.plane_lines;
    const uint2 x = l < a.lines ? *reinterpret_cast<const uint2*>(a.plane + line * 128 + 8 * (l & 15))
                                : make_uint2(0, 0);
    acc = x.x ^ x.y;
  }
  // residue runs: the wave's records, one run of run_bytes each, at
  // scattered places; 16-B chunks q = 64 i + lane over the concatenated runs
  const uint32_t per = a.run_bytes / 16, total = per * a.runs;
  for (uint32_t q = lane; q < total; q += 64) {
    const uint32_t r = q / per, c = q - r * per;
    const uint64_t wr = (uint64_t)a.win_tiles * a.runs;
    const uint64_t slot = kSeq ? (w * a.runs + r) % a.out_runs
                          : a.win_tiles ? ((w / a.win_tiles) * wr + mix(w * 64 + r) % wr) % a.out_runs
                                        : mix(w * 64 + r) % a.out_runs;
    st16(a.out + slot * a.run_bytes + 16 * c, make_uint4(acc, q, r, (uint32_t)w), kNt);
  }
  if (acc == 0x12345678u) *a.sink = acc;
}

// C5 with the staging chain: `chain` dependent load round trips per wave
// (each round's addresses depend on every lane's previous load, as staging's
// rows -> windows -> batch offsets do), `lines` fills in all, then the
// stores.  kSplit: even waves only load (their odd partner's fills too), odd
// waves only store (their partner's runs too): loads never queue behind the
// same wave's stores (a producer / consumer split of the staging and chunk
// phases, without the hand-off).
// kNow: orf6_kernel as of round 4 -- blocks in the hardware's round-robin
// XCD order and the records' blocks laid out in walk order (tile w's runs
// follow tile w-1's)
// kRr: the hardware's round-robin block order (else one contiguous run of
// tiles per XCD)
template <bool kSplit, bool kNow = false, bool kRr = kNow>
__global__ __launch_bounds__(256) void c5_chain(C5Args a, uint32_t chain, uint32_t extra) {
  const uint32_t xnb = gridDim.x, xb = blockIdx.x;
  const uint32_t xq = xnb >> 3, xr = xnb & 7, xcd = xb & 7, xk = xb >> 3;
  const uint32_t vb = kRr ? xb : xcd < xr ? xcd * (xq + 1) + xk : xr * (xq + 1) + (xcd - xr) * xq + xk;
  const uint64_t w = (uint64_t)vb * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (w >= a.ntiles) return;
  const bool do_load = !kSplit || (w & 1) == 0, do_store = !kSplit || (w & 1) == 1;
  const uint32_t lines = kSplit ? 2 * a.lines : a.lines;
  uint32_t acc = 0, dep = 0;
  if (do_load) {
    for (uint32_t k = 0; k < chain; ++k) {
      const uint32_t l0 = k * lines / chain, l1 = (k + 1) * lines / chain;
      for (uint32_t l = l0 + lane; l < l1; l += 64) {
        const uint64_t line = (w * a.lines + l + dep) % a.plane_lines;
        const uint2 x = *reinterpret_cast<const uint2*>(a.plane + line * 128 + 8 * (l & 15));
        acc ^= x.x + x.y;
      }
      // `extra` more load instructions per round over the same lines (L2
      // hits: staging's row, table, window and offset loads)
      for (uint32_t x = 0; x < extra; ++x) {
        const uint64_t line = (w * a.lines + ((lane + x) % a.lines) + dep) % a.plane_lines;
        const uint2 y = *reinterpret_cast<const uint2*>(a.plane + line * 128 + 8 * ((lane + x) & 15));
        acc ^= y.x + y.y;
      }
      dep = (uint32_t)__ballot(acc == 0x12345u);  // 0, known only once every lane's load is back
    }
  }
  if (do_store) {
    const uint32_t per = a.run_bytes / 16, runs = kSplit ? 2 * a.runs : a.runs, total = per * runs;
    const uint64_t wr = (uint64_t)a.win_tiles * a.runs;
    for (uint32_t q = lane; q < total; q += 64) {
      const uint32_t r = q / per, c = q - r * per;
      const uint64_t slot = kNow ? (w * runs + r) % a.out_runs
                                 : ((w / a.win_tiles) * wr + mix(w * 64 + r) % wr) % a.out_runs;
      st16(a.out + slot * a.run_bytes + 16 * c, make_uint4(acc, q, r, (uint32_t)w), false);
    }
  }
  if (acc == 0x12345678u) *a.sink = acc;
}

// occupancy cap as the product launches use it: dynamic LDS nobody touches
static size_t lds_pad(const void* fn, int want) {
  int per = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, fn, 256, 0));
  if (want <= 0 || want >= per) return 0;
  return 160 * 1024 / want - 1024;
}

int main(int argc, char** argv) {
  const char* mode = argc > 1 ? argv[1] : "c3";
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  uint32_t* sink;
  CK(hipMalloc(&sink, 4));
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  auto timeit = [&](auto launch, const char* name, double wbytes, double rbytes) {
    float ms = 0;
    for (int i = 0; i < 50; ++i) launch();  // settle
    CK(hipDeviceSynchronize());
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipEventRecord(e0));
      for (int i = 0; i < 100; ++i) launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
      ms /= 100;
      printf("%-44s %.4f ms  writes %.3f GB  line fills %.3f GB  %.0f GB/s\n", name, ms,
             wbytes / 1e9, rbytes / 1e9, (wbytes + rbytes) / (ms * 1e6));
    }
  };
  if (!strcmp(mode, "c3now")) {
    // profiles/r05/final: 118,356 tiles, reads 0.536 GB (35 lines per tile)
    const uint32_t ntiles = 118356, nuc = 5072, pep = 1696;
    const uint64_t plane = 2ull << 30;
    uint8_t *pl, *o1, *o2;
    CK(hipMalloc(&pl, plane));
    CK(hipMalloc(&o1, (uint64_t)ntiles * nuc));
    CK(hipMalloc(&o2, (uint64_t)ntiles * pep));
    CK(hipMemset(pl, 1, plane));
    const size_t pad = lds_pad(reinterpret_cast<const void*>(c3_replay), 6);
    const int grid = (int)((ntiles + 3) / 4);
    for (uint32_t seq : {1u, 0u}) {
      for (uint32_t lines : {35u, 0u}) {
        C3Args a{pl, plane / 128, o1, o2, ntiles, lines, nuc, pep, sink, 0u, 0u, seq};
        char nm[96];
        snprintf(nm, sizeof nm, "c3now: %u fills per tile, %s", lines,
                 seq ? "in tile order" : "scattered");
        timeit([&] { hipLaunchKernelGGL(c3_replay, grid, 256, pad, 0, a); }, nm,
               (double)ntiles * (nuc + pep), (double)ntiles * lines * 128);
      }
    }
    for (uint32_t per : {1u, 2u, 4u, 8u})
      for (uint32_t xrun : {0u, 16u})
        for (int nt = 1; nt >= 0; --nt) {
          const int g = (int)((ntiles + 4 * per - 1) / (4 * per));
          char nm[96];
          snprintf(nm, sizeof nm, "stores: %u tiles/wave, xrun %u, %s", per, xrun,
                   nt ? "nt" : "plain");
          if (nt)
            timeit([&] { hipLaunchKernelGGL(c3_stores<true>, g, 256, pad, 0, o1, o2, ntiles,
                                            nuc, pep, per, xrun); },
                   nm, (double)ntiles * (nuc + pep), 0.0);
          else
            timeit([&] { hipLaunchKernelGGL(c3_stores<false>, g, 256, pad, 0, o1, o2, ntiles,
                                            nuc, pep, per, xrun); },
                   nm, (double)ntiles * (nuc + pep), 0.0);
        }
    for (uint32_t tb : {3024u, 4096u, 4608u, 5056u, 5072u, 5120u, 5632u, 6144u, 7168u}) {
      // the nucleotide stream alone at other tile sizes (XCD runs of 16 blocks, nt)
      const uint32_t nt_tiles = (uint32_t)((uint64_t)ntiles * nuc / tb);
      const int g = (int)((nt_tiles + 3) / 4);
      char nm[96];
      snprintf(nm, sizeof nm, "stores: nucleotide stream only, %u-byte tiles", tb);
      timeit([&] { hipLaunchKernelGGL(c3_stores<true>, g, 256, pad, 0, o1, o2, nt_tiles, tb, 0u,
                                      1u, 16u); },
             nm, (double)nt_tiles * tb, 0.0);
    }
    for (int nt = 1; nt >= 0; --nt) {
      // the nucleotide stream alone (no residue stream interleaved)
      const int g = (int)((ntiles + 3) / 4);
      if (nt)
        timeit([&] { hipLaunchKernelGGL(c3_stores<true>, g, 256, pad, 0, o1, o2, ntiles, nuc, 0u,
                                        1u, 16u); },
               "stores: nucleotide stream only, nt", (double)ntiles * nuc, 0.0);
      else
        timeit([&] { hipLaunchKernelGGL(c3_stores<false>, g, 256, pad, 0, o1, o2, ntiles, nuc, 0u,
                                        1u, 16u); },
               "stores: nucleotide stream only, plain", (double)ntiles * nuc, 0.0);
    }
    timeit([&] { (void)hipMemsetAsync(o1, 7, (uint64_t)ntiles * nuc); },
           "hipMemset of the nucleotide bytes", (double)ntiles * nuc, 0.0);
    {
      const uint64_t ch = (uint64_t)ntiles * nuc / 16;
      for (int blocks : {256 * 6, 256 * 8, 256 * 32, 1000, 1280, 1792, 2560, 3000, 3072, 4096, 5000, 12000}) {
        char nm[96];
        snprintf(nm, sizeof nm, "flat: lane-contiguous, %d blocks, nt", blocks);
        timeit([&] { hipLaunchKernelGGL((flat_stores<false, true>), blocks, 256, 0, 0, o1, ch); },
               nm, (double)ntiles * nuc, 0.0);
        snprintf(nm, sizeof nm, "flat: lane-contiguous, %d blocks, plain, constant bytes", blocks);
        timeit([&] { hipLaunchKernelGGL((flat_stores<false, false>), blocks, 256, 0, 0, o1, ch); },
               nm, (double)ntiles * nuc, 0.0);
        snprintf(nm, sizeof nm, "flat: 64 B per lane, %d blocks, plain", blocks);
        timeit([&] { hipLaunchKernelGGL((flat_stores<true, false>), blocks, 256, 0, 0, o1, ch); },
               nm, (double)ntiles * nuc, 0.0);
      }
    }
    {
      // one flat grid-stride fill of the same bytes (what a library memset does)
      CK(hipMemsetAsync(o1, 7, (uint64_t)ntiles * nuc));
      timeit([&] {
        (void)hipMemsetAsync(o1, 7, (uint64_t)ntiles * nuc);
        (void)hipMemsetAsync(o2, 7, (uint64_t)ntiles * pep);
      }, "hipMemset of the same bytes", (double)ntiles * (nuc + pep), 0.0);
    }
    C3Args c{pl, plane / 128, o1, o2, ntiles, 35u, 0u, 0u, sink, 0u, 0u, 1u};
    timeit([&] { hipLaunchKernelGGL(c3_replay, grid, 256, pad, 0, c); },
           "c3now: 35 fills in tile order, no stores", 0.0, (double)ntiles * 35 * 128);
  } else if (!strcmp(mode, "c3")) {
    // C3 (profiles/r03_close2): 118,356 tiles; 600.3 MB nucleotides and
    // 199.9 MB residues; PMC line fills 0.86 GB per launch (~57 per tile)
    const uint32_t ntiles = 118356, nuc = 5072, pep = 1696;
    const uint64_t plane = 2ull << 30;
    uint8_t *pl, *o1, *o2;
    CK(hipMalloc(&pl, plane));
    CK(hipMalloc(&o1, (uint64_t)ntiles * nuc));
    CK(hipMalloc(&o2, (uint64_t)ntiles * pep));
    CK(hipMemset(pl, 1, plane));
    const size_t pad = lds_pad(reinterpret_cast<const void*>(c3_replay), 6);
    const int grid = (int)((ntiles + 3) / 4);
    for (uint32_t lines : {0u, 57u, 96u}) {
      C3Args a{pl, plane / 128, o1, o2, ntiles, lines, nuc, pep, sink, 0u, 0u, 0u};
      char nm[96];
      snprintf(nm, sizeof nm, "c3 replay: %u line fills per tile", lines);
      timeit([&] { hipLaunchKernelGGL(c3_replay, grid, 256, pad, 0, a); }, nm,
             (double)ntiles * (nuc + pep), (double)ntiles * lines * 128);
    }
    C3Args a{pl, plane / 128, o1, o2, ntiles, 57u, nuc, 0u, sink, 0u, 0u, 0u};
    timeit([&] { hipLaunchKernelGGL(c3_replay, grid, 256, pad, 0, a); },
           "c3 replay: nucleotide stores only + 57 fills", (double)ntiles * nuc,
           (double)ntiles * 57 * 128);
    C3Args c{pl, plane / 128, o1, o2, ntiles, 57u, 0u, 0u, sink, 0u, 0u, 0u};
    timeit([&] { hipLaunchKernelGGL(c3_replay, grid, 256, pad, 0, c); },
           "c3 replay: 57 fills, no stores", 0.0, (double)ntiles * 57 * 128);
    // C3's records are contig-major (random within a contig): the tiles of
    // one contig (64 contigs: ~1850 tiles) read inside its stretch of the two
    // planes (~2 x 7.8 MB)
    const uint64_t wl = (2ull * 7800000) / 128;
    C3Args d{pl, plane / 128, o1, o2, ntiles, 57u, nuc, pep, sink, 1850u, wl, 0u};
    timeit([&] { hipLaunchKernelGGL(c3_replay, grid, 256, pad, 0, d); },
           "c3 replay: 57 fills within a contig's planes", (double)ntiles * (nuc + pep),
           (double)ntiles * 57 * 128);
    C3Args e{pl, plane / 128, o1, o2, ntiles, 57u, 0u, 0u, sink, 1850u, wl, 0u};
    timeit([&] { hipLaunchKernelGGL(c3_replay, grid, 256, pad, 0, e); },
           "c3 replay: 57 fills within a contig, no stores", 0.0, (double)ntiles * 57 * 128);
  } else {
    // C5 (profiles/r03_close2): 605,096 tiles; 5.07 GB written per launch
    // (PMC), reads 1.64 GB; a tile touches ~4 records (six streams each)
    const uint32_t ntiles = 605096, run = 2096, runs = 4;
    const uint64_t plane = 1536ull << 20, out = 5ull << 30;
    uint8_t *pl, *o;
    CK(hipMalloc(&pl, plane));
    CK(hipMalloc(&o, out));
    CK(hipMemset(pl, 1, plane));
    const size_t pad = lds_pad(reinterpret_cast<const void*>(c5_replay<false, false>), 7);
    const int grid = (int)((ntiles + 3) / 4);
    const double wb = (double)ntiles * run * runs, rb = (double)ntiles * 21 * 128;
    for (uint32_t lines : {0u, 21u}) {
      C5Args a{pl, plane / 128, o, out / run, ntiles, lines, run, runs, sink, 0u};
      char nm[96];
      snprintf(nm, sizeof nm, "c5 replay: %u line fills per tile", lines);
      timeit([&] { hipLaunchKernelGGL((c5_replay<false, false>), grid, 256, pad, 0, a); }, nm,
             wb, (double)ntiles * lines * 128);
    }
    C5Args a{pl, plane / 128, o, out / run, ntiles, 21u, run, runs, sink, 0u};
    timeit([&] { hipLaunchKernelGGL((c5_replay<false, true>), grid, 256, pad, 0, a); },
           "c5 replay: 21 fills, scattered runs, nt", wb, rb);
    timeit([&] { hipLaunchKernelGGL((c5_replay<true, false>), grid, 256, pad, 0, a); },
           "c5 replay: 21 fills, sequential runs", wb, rb);
    timeit([&] { hipLaunchKernelGGL((c5_replay<true, true>), grid, 256, pad, 0, a); },
           "c5 replay: 21 fills, sequential runs, nt", wb, rb);
    // the same scattered replay over two more, separately allocated outputs
    // (is a slow C5 process a property of its allocation?)
    for (int extra = 0; extra < 2; ++extra) {
      uint8_t* o2;
      CK(hipMalloc(&o2, out));
      C5Args c{pl, plane / 128, o2, out / run, ntiles, 21u, run, runs, sink, 0u};
      char nm[96];
      snprintf(nm, sizeof nm, "c5 replay: 21 fills, scattered, buffer %d", extra + 2);
      timeit([&] { hipLaunchKernelGGL((c5_replay<false, false>), grid, 256, pad, 0, c); }, nm, wb, rb);
    }
    timeit([&] { hipLaunchKernelGGL((c5_replay<false, false>), grid, 256, pad, 0, a); },
           "c5 replay: 21 fills, scattered, buffer 1 again", wb, rb);
    if (argc > 2 && !strcmp(argv[2], "now")) {
      // round 4's orf6: walk-order layout, round-robin blocks, 2.00 GB of
      // fills per launch (profiles/r04_close/traffic_C5: ~26 lines per tile)
      const uint32_t l4 = 26;
      C5Args b{pl, plane / 128, o, out / run, ntiles, l4, run, runs, sink, 3000u};
      const double rb4 = (double)ntiles * l4 * 128;
      const size_t padc = lds_pad(reinterpret_cast<const void*>(c5_chain<false, true>), 7);
      for (uint32_t chain : {1u, 3u, 5u}) {
        char nm[96];
        snprintf(nm, sizeof nm, "c5 now: %u dependent load rounds", chain);
        timeit([&] { hipLaunchKernelGGL((c5_chain<false, true>), grid, 256, padc, 0, b, chain, 0u); },
               nm, wb, rb4);
      }
      C5Args z{pl, plane / 128, o, out / run, ntiles, 0u, run, runs, sink, 3000u};
      timeit([&] { hipLaunchKernelGGL((c5_chain<false, true>), grid, 256, padc, 0, z, 1u, 0u); },
             "c5 now: stores only", wb, 0.0);
      timeit([&] { hipLaunchKernelGGL((c5_chain<true, true>), grid, 256, padc, 0, b, 5u, 0u); },
             "c5 now: 5 rounds, load/store waves split", wb, rb4);
      // the same walk-order layout with one contiguous run of tiles per XCD
      // (round 3's order: 1.64 GB of fills, ~21 lines per tile)
      C5Args c{pl, plane / 128, o, out / run, ntiles, 21u, run, runs, sink, 3000u};
      timeit([&] { hipLaunchKernelGGL((c5_chain<false, true, false>), grid, 256, padc, 0, c, 5u, 0u); },
             "c5 now, XCD runs, 21 fills: 5 rounds", wb, (double)ntiles * 21 * 128);
      timeit([&] { hipLaunchKernelGGL((c5_chain<false, true, true>), grid, 256, padc, 0, c, 5u, 0u); },
             "c5 now, round-robin, 21 fills: 5 rounds", wb, (double)ntiles * 21 * 128);
      timeit([&] { hipLaunchKernelGGL((c5_chain<false, true, false>), grid, 256, padc, 0, z, 1u, 0u); },
             "c5 now, XCD runs: stores only", wb, 0.0);
      return 0;
    }
    if (argc > 2 && !strcmp(argv[2], "chain")) {
      C5Args b{pl, plane / 128, o, out / run, ntiles, 21u, run, runs, sink, 3000u};
      const size_t padc = lds_pad(reinterpret_cast<const void*>(c5_chain<false>), 7);
      for (uint32_t chain : {1u, 3u, 5u}) {
        char nm[96];
        snprintf(nm, sizeof nm, "c5 chain: %u dependent load rounds", chain);
        timeit([&] { hipLaunchKernelGGL((c5_chain<false>), grid, 256, padc, 0, b, chain, 0u); }, nm, wb, rb);
        snprintf(nm, sizeof nm, "c5 chain: %u rounds, load/store waves split", chain);
        timeit([&] { hipLaunchKernelGGL((c5_chain<true>), grid, 256, padc, 0, b, chain, 0u); }, nm, wb, rb);
      }
      for (uint32_t extra : {3u, 6u}) {
        char nm[96];
        snprintf(nm, sizeof nm, "c5 chain: 5 rounds + %u L2-hit load insts each", extra);
        timeit([&] { hipLaunchKernelGGL((c5_chain<false>), grid, 256, padc, 0, b, 5u, extra); }, nm, wb, rb);
      }
      C5Args z{pl, plane / 128, o, out / run, ntiles, 0u, run, runs, sink, 3000u};
      timeit([&] { hipLaunchKernelGGL((c5_chain<false>), grid, 256, padc, 0, z, 1u, 0u); },
             "c5 chain: stores only (moving window)", wb, 0.0);
      return 0;
    }
    // runs scattered inside a window of 3000 tiles' output (~25 MB) that
    // advances with the walk: one contig's records, output in record order,
    // walked in genome order
    C5Args b{pl, plane / 128, o, out / run, ntiles, 21u, run, runs, sink, 3000u};
    timeit([&] { hipLaunchKernelGGL((c5_replay<false, false>), grid, 256, pad, 0, b); },
           "c5 replay: 21 fills, runs in a moving 25-MB window", wb, rb);
  }
  return 0;
}
