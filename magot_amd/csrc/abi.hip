// C ABI of libmagot.so (declarations and contracts: include/magot.h).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <thread>

#include "common.h"

namespace magot {

namespace {
thread_local std::string g_last_error;
}

void set_error(const std::string& msg) { g_last_error = msg; }

void standard_lut(uint8_t out[64]) {
  // genome.py:795-802, walked in TCAG order (first, second, third base).
  static const char kAA[] = "FFLLSSSSYY**CC*WLLLLPPPPHHQQRRRRIIIMTTTTNNKKSSRRVVVVAAAADDEEGGGG";
  static const int kTcagToCode[4] = {3, 1, 0, 2};  // T C A G -> A=0 C=1 G=2 T=3
  int n = 0;
  for (int a = 0; a < 4; ++a)
    for (int b = 0; b < 4; ++b)
      for (int c = 0; c < 4; ++c) {
        int x = kTcagToCode[a] + 4 * kTcagToCode[b] + 16 * kTcagToCode[c];
        out[x] = (uint8_t)kAA[n++];
      }
}

}  // namespace magot

using namespace magot;

struct magot_ctx {
  int device = 0;
  int n_cu = 0;
  int blocks_per_cu = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  hipEvent_t mark0 = nullptr, mark1 = nullptr;  // magot_ctx_mark
  // pinned staging ring for genome uploads (allocated on first use); loads on
  // one context from several host threads take turns on it
  uint8_t* pin[2] = {nullptr, nullptr};
  hipEvent_t pin_ev[2] = {nullptr, nullptr};
  std::mutex pin_mu;
};

struct magot_genome {
  magot_ctx* ctx = nullptr;
  void* arena = nullptr;
  uint64_t arena_bytes = 0;
  bool owns_arena = true;  // false: caller memory (magot_genome_attach)
  uint32_t* nib = nullptr;  // forward then reverse-strand nibble plane (ExtractArgs::span)
  uint64_t span = 0;
  ExcRun* runs = nullptr;
  uint32_t* dir = nullptr;
  std::vector<uint64_t> contig_base, contig_len;
  std::vector<std::string> names;  // contig names (magot_genome_load_fasta)
  std::vector<ExcRun> host_runs;   // host copies for per-interval exception flags
  std::vector<uint32_t> host_dir;
  uint64_t extent = 0, total_bases = 0, n_runs = 0;
};

struct magot_plan {
  magot_ctx* ctx = nullptr;
  const magot_genome* g = nullptr;
  void* arena = nullptr;       // tables (intervals, records, tiles, layout)
  uint64_t arena_bytes = 0;
  void* out_arena = nullptr;   // output buffers (nucleotides, residues)
  uint64_t out_bytes = 0;
  ExtractArgs args{};
  std::vector<uint64_t> nuc_off, pep_off;  // host copies, n_tx+1 (record order)
  // MAGOT_OUT_GENOME_ORDER: records laid out in genome order; each record's
  // place in the output buffers (record order; device copies for reassembly)
  bool genome_order = false;
  std::vector<uint64_t> lay_nuc, lay_pep;
  const uint64_t* d_lay_nuc = nullptr;  // T
  const uint64_t* d_lay_pep = nullptr;  // T
  const uint64_t* d_nuc_off = nullptr;  // T+1
  const uint64_t* d_pep_off = nullptr;  // T+1
  uint64_t n_exons = 0, n_tx = 0;
  uint64_t n_ex_c = 0;  // compacted (non-empty) intervals in args.ex_g / ex_out
  bool executed = false;
};

namespace {

// Sub-allocate 256-byte aligned slices of one device allocation.
struct Carve {
  uint64_t used = 0;
  template <class T>
  uint64_t take(uint64_t count) {
    uint64_t at = used;
    used += (count * sizeof(T) + 255) & ~255ull;
    return at;
  }
};

int bind(magot_ctx* ctx) {
  if (!ctx) {
    set_error("null context");
    return MAGOT_ERR_ARG;
  }
  MAGOT_HIP_TRY(hipSetDevice(ctx->device));
  return MAGOT_OK;
}

}  // namespace

// Host meta blob of a packed genome (magot_genome_export / _attach).
namespace {

struct MetaWriter {
  std::vector<uint8_t> buf;
  template <class T>
  void put(const T& v) {
    const uint8_t* p = reinterpret_cast<const uint8_t*>(&v);
    buf.insert(buf.end(), p, p + sizeof(T));
  }
  template <class T>
  void put_vec(const std::vector<T>& v) {
    put<uint64_t>(v.size());
    const uint8_t* p = reinterpret_cast<const uint8_t*>(v.data());
    buf.insert(buf.end(), p, p + v.size() * sizeof(T));
  }
};

struct MetaReader {
  const uint8_t* p;
  const uint8_t* end;
  template <class T>
  bool get(T* v) {
    if ((uint64_t)(end - p) < sizeof(T)) return false;
    memcpy(v, p, sizeof(T));
    p += sizeof(T);
    return true;
  }
  template <class T>
  bool get_vec(std::vector<T>* v) {
    uint64_t n;
    if (!get(&n) || n > (uint64_t)(end - p) / sizeof(T)) return false;
    v->resize(n);
    memcpy(v->data(), p, n * sizeof(T));
    p += n * sizeof(T);
    return true;
  }
};

constexpr uint64_t kMetaMagic = 0x4d41474f54474e31ull;  // "MAGOTGN1"

std::vector<uint8_t> genome_meta(const magot_genome* g) {
  MetaWriter w;
  w.put(kMetaMagic);
  w.put(g->arena_bytes);
  w.put<uint64_t>((const char*)g->nib - (const char*)g->arena);
  w.put<uint64_t>((const char*)g->runs - (const char*)g->arena);
  w.put<uint64_t>((const char*)g->dir - (const char*)g->arena);
  w.put(g->span);
  w.put(g->extent);
  w.put(g->total_bases);
  w.put(g->n_runs);
  w.put_vec(g->contig_base);
  w.put_vec(g->contig_len);
  w.put_vec(g->host_runs);
  w.put_vec(g->host_dir);
  return w.buf;
}

// Parse a meta blob into g's host fields; the piece offsets into *o.
bool parse_genome_meta(const uint8_t* meta, uint64_t meta_len, magot_genome* g, uint64_t o[3]) {
  MetaReader r{meta, meta + meta_len};
  uint64_t magic = 0;
  bool ok = r.get(&magic) && magic == kMetaMagic && r.get(&g->arena_bytes) && r.get(&o[0]) &&
            r.get(&o[1]) && r.get(&o[2]) && r.get(&g->span) && r.get(&g->extent) &&
            r.get(&g->total_bases) && r.get(&g->n_runs) && r.get_vec(&g->contig_base) &&
            r.get_vec(&g->contig_len) && r.get_vec(&g->host_runs) && r.get_vec(&g->host_dir);
  return ok && o[0] < g->arena_bytes && o[1] < g->arena_bytes && o[2] < g->arena_bytes &&
         g->host_runs.size() == g->n_runs + 1 && g->span % 32 == 0 &&
         o[0] + (2 * (g->span / 8) + 4) * 4 <= o[1] && o[1] <= o[2];
}

// Pack the contigs and place the planes in HBM (magot_genome_load*): on the
// device by default, on the host (pack.cpp) with MAGOT_PACK_HOST.
int load_packed(magot_ctx* ctx, const ContigSource* src, uint32_t n_contigs, uint32_t flags,
                magot_genome** out);

}  // namespace

extern "C" {

int magot_abi_version(void) { return MAGOT_ABI_VERSION; }

const char* magot_last_error(void) { return g_last_error.c_str(); }

int magot_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int magot_ctx_create(int device, magot_ctx** out) {
  if (!out) {
    set_error("magot_ctx_create: null out");
    return MAGOT_ERR_ARG;
  }
  *out = nullptr;
  int n = 0;
  MAGOT_HIP_TRY(hipGetDeviceCount(&n));
  if (device < 0 || device >= n) {
    set_error("magot_ctx_create: device " + std::to_string(device) + " out of range (" +
              std::to_string(n) + " visible)");
    return MAGOT_ERR_ARG;
  }
  std::unique_ptr<magot_ctx> c(new magot_ctx());
  c->device = device;
  MAGOT_HIP_TRY(hipSetDevice(device));
  MAGOT_HIP_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  MAGOT_HIP_TRY(hipEventCreate(&c->ev0));
  MAGOT_HIP_TRY(hipEventCreate(&c->ev1));
  MAGOT_HIP_TRY(hipEventCreate(&c->mark0));
  MAGOT_HIP_TRY(hipEventCreate(&c->mark1));
  MAGOT_HIP_TRY(hipDeviceGetAttribute(&c->n_cu, hipDeviceAttributeMultiprocessorCount, device));
  c->blocks_per_cu = extract_blocks_per_cu();
  *out = c.release();
  return MAGOT_OK;
}

void magot_ctx_destroy(magot_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  if (ctx->ev0) (void)hipEventDestroy(ctx->ev0);
  if (ctx->ev1) (void)hipEventDestroy(ctx->ev1);
  if (ctx->mark0) (void)hipEventDestroy(ctx->mark0);
  if (ctx->mark1) (void)hipEventDestroy(ctx->mark1);
  for (int k = 0; k < 2; ++k) {
    if (ctx->pin_ev[k]) (void)hipEventDestroy(ctx->pin_ev[k]);
    if (ctx->pin[k]) (void)hipHostFree(ctx->pin[k]);
  }
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
}

int magot_ctx_info(const magot_ctx* ctx, int* n_cu, int* extract_blocks_per_cu) {
  if (!ctx) {
    set_error("magot_ctx_info: null context");
    return MAGOT_ERR_ARG;
  }
  if (n_cu) *n_cu = ctx->n_cu;
  if (extract_blocks_per_cu) *extract_blocks_per_cu = ctx->blocks_per_cu;
  return MAGOT_OK;
}

int magot_ctx_sync(magot_ctx* ctx) {
  if (int rc = bind(ctx)) return rc;
  MAGOT_HIP_TRY(hipStreamSynchronize(ctx->stream));
  return MAGOT_OK;
}

int magot_ctx_mark(magot_ctx* ctx, int which) {
  if (int rc = bind(ctx)) return rc;
  if (which != 0 && which != 1) {
    set_error("magot_ctx_mark: which must be 0 or 1");
    return MAGOT_ERR_ARG;
  }
  MAGOT_HIP_TRY(hipEventRecord(which ? ctx->mark1 : ctx->mark0, ctx->stream));
  return MAGOT_OK;
}

int magot_ctx_elapsed(magot_ctx* ctx, double* ms) {
  if (int rc = bind(ctx)) return rc;
  if (!ms) {
    set_error("magot_ctx_elapsed: null argument");
    return MAGOT_ERR_ARG;
  }
  MAGOT_HIP_TRY(hipEventSynchronize(ctx->mark1));
  float f = 0.f;
  MAGOT_HIP_TRY(hipEventElapsedTime(&f, ctx->mark0, ctx->mark1));
  *ms = f;
  return MAGOT_OK;
}

int magot_genome_load_ex(magot_ctx* ctx, const uint8_t* const* seqs, const uint64_t* lens,
                         uint32_t n_contigs, uint32_t flags, magot_genome** out) {
  if (int rc = bind(ctx)) return rc;
  if (!out || (n_contigs && (!seqs || !lens))) {
    set_error("magot_genome_load: null argument");
    return MAGOT_ERR_ARG;
  }
  if (flags & ~MAGOT_PACK_HOST) {
    set_error("magot_genome_load_ex: unknown flags");
    return MAGOT_ERR_ARG;
  }
  *out = nullptr;
  for (uint32_t i = 0; i < n_contigs; ++i)
    if (lens[i] && !seqs[i]) {
      set_error("magot_genome_load: null contig pointer");
      return MAGOT_ERR_ARG;
    }
  std::vector<ContigSource> src(n_contigs);
  for (uint32_t i = 0; i < n_contigs; ++i) src[i] = ContigSource{seqs[i], lens[i], 0, 0};
  return load_packed(ctx, src.data(), n_contigs, flags, out);
}

int magot_genome_load(magot_ctx* ctx, const uint8_t* const* seqs, const uint64_t* lens,
                      uint32_t n_contigs, magot_genome** out) {
  return magot_genome_load_ex(ctx, seqs, lens, n_contigs, 0u, out);
}

}  // extern "C"

namespace {

struct Lap {
  const char* tag;
  const bool on;
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  explicit Lap(const char* env = "MAGOT_GENOME_TIMING", const char* tag_ = "genome")
      : tag(tag_), on(std::getenv(env) != nullptr) {}
  void operator()(const char* what) {
    if (!on) return;
    const auto t1 = std::chrono::steady_clock::now();
    fprintf(stderr, "[%s] %-10s %.4f s\n", tag, what,
            std::chrono::duration<double>(t1 - t0).count());
    t0 = t1;
  }
};

// Host threads for staging copies: the GPU's share of the host (OMP_NUM_THREADS
// on the pool's boxes), at most 16.
unsigned host_threads() {
  unsigned hw = std::max(1u, std::thread::hardware_concurrency());
  if (const char* e = std::getenv("OMP_NUM_THREADS")) {
    const int v = atoi(e);
    if (v > 0) hw = (unsigned)v;
  }
  return std::min(hw, 16u);
}

// fn(lo, hi, part) over `parts` contiguous ranges of [0, n), part 0 on the
// calling thread; fn must not throw.
template <class F>
void parallel_ranges(uint64_t n, unsigned parts, F fn) {
  if (parts <= 1 || n < 2) {
    fn(0, n, 0u);
    return;
  }
  std::vector<std::thread> pool;
  pool.reserve(parts - 1);
  for (unsigned k = 1; k < parts; ++k)
    pool.emplace_back([&fn, n, parts, k]() { fn(n * k / parts, n * (k + 1) / parts, k); });
  fn(0, n / parts, 0u);
  for (std::thread& th : pool) th.join();
}

// A host array left uninitialised (POD rows the planner writes itself, in
// parallel: no sequential zero fill, and its pages fault in on the writing threads).
template <class T>
struct HostBuf {
  std::unique_ptr<T[]> p;
  uint64_t n = 0;
  explicit HostBuf(uint64_t count = 0) : p(count ? new T[count] : nullptr), n(count) {}
  T& operator[](uint64_t i) { return p[i]; }
  const T& operator[](uint64_t i) const { return p[i]; }
  T* data() { return p.get(); }
  const T* data() const { return p.get(); }
};

// Host rows bound for one device allocation (dev_off into it).
struct HostPiece {
  uint64_t dev_off;
  const void* src;
  uint64_t bytes;
};

constexpr uint64_t kPinRing = 64ull << 20;  // each of the context's two pinned staging buffers

int ensure_pin_ring(magot_ctx* ctx) {  // callers hold ctx->pin_mu
  for (int k = 0; k < 2; ++k)
    if (!ctx->pin[k]) {
      MAGOT_HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&ctx->pin[k]), kPinRing,
                                  hipHostMallocDefault));
      MAGOT_HIP_TRY(hipEventCreateWithFlags(&ctx->pin_ev[k], hipEventDisableTiming));
    }
  return MAGOT_OK;
}

// Upload host rows through the context's two pinned staging buffers: host
// threads copy one 64 MiB piece in while the DMA engine drains the other (a
// pageable hipMemcpy stages through the runtime's own small buffers at a
// fraction of the link rate).  Synchronous: the rows are on the device when
// it returns.
int upload_pieces(magot_ctx* ctx, char* dev, const std::vector<HostPiece>& pieces) {
  std::lock_guard<std::mutex> lock(ctx->pin_mu);
  if (int rc = ensure_pin_ring(ctx)) return rc;
  const unsigned nt = host_threads();
  uint64_t k = 0;
  for (const HostPiece& pc : pieces)
    for (uint64_t q0 = 0; q0 < pc.bytes; q0 += kPinRing, ++k) {
      const int b = (int)(k & 1);
      const uint64_t q1 = std::min(pc.bytes, q0 + kPinRing);
      MAGOT_HIP_TRY(hipEventSynchronize(ctx->pin_ev[b]));
      const char* src = static_cast<const char*>(pc.src) + q0;
      uint8_t* ring = ctx->pin[b];
      parallel_ranges(q1 - q0, q1 - q0 >= (4ull << 20) ? nt : 1u,
                      [&](uint64_t lo, uint64_t hi, unsigned) { memcpy(ring + lo, src + lo, hi - lo); });
      MAGOT_HIP_TRY(hipMemcpyAsync(dev + pc.dev_off + q0, ring, q1 - q0, hipMemcpyHostToDevice,
                                   ctx->stream));
      MAGOT_HIP_TRY(hipEventRecord(ctx->pin_ev[b], ctx->stream));
    }
  MAGOT_HIP_TRY(hipStreamSynchronize(ctx->stream));
  return MAGOT_OK;
}

// Stream the contigs' bytes (FASTA line layout removed) into dev[0, total),
// total = extent - kOrigin, through two pinned 64 MiB host buffers: host
// threads fill one while the DMA engine uploads the other.
int upload_raw(magot_ctx* ctx, const ContigSource* src, const HostPacked& lay, uint8_t* dev) {
  const uint64_t total = lay.extent - kOrigin;
  if (!total) return MAGOT_OK;
  constexpr uint64_t kRing = kPinRing;
  std::lock_guard<std::mutex> lock(ctx->pin_mu);
  if (int rc = ensure_pin_ring(ctx)) return rc;
  const unsigned nt = host_threads();
  const auto& base = lay.contig_base;
  auto fill = [&](uint8_t* dst, uint64_t x0, uint64_t x1) {  // raw [x0, x1) -> dst
    size_t c = std::upper_bound(base.begin(), base.end(), x0 + kOrigin) - base.begin();
    c = c ? c - 1 : 0;
    for (; c < base.size() && x0 < x1; ++c) {
      const uint64_t cb = base[c] - kOrigin, ce = cb + lay.contig_len[c];
      if (ce <= x0) continue;
      const uint64_t hi = std::min(ce, x1);
      copy_bases(src[c], x0 - cb, hi - x0, dst);
      dst += hi - x0;
      x0 = hi;
    }
  };
  for (uint64_t q0 = 0, k = 0; q0 < total; q0 += kRing, ++k) {
    const int b = (int)(k & 1);
    const uint64_t q1 = std::min(total, q0 + kRing);
    // the buffer's previous DMA (of this load, or of an earlier one whose
    // last copies may still be in flight) has drained
    MAGOT_HIP_TRY(hipEventSynchronize(ctx->pin_ev[b]));
    const uint64_t step = ((q1 - q0) + nt - 1) / nt;
    std::vector<std::thread> pool;
    for (unsigned i = 1; i < nt && q0 + i * step < q1; ++i) {
      const uint64_t x0 = q0 + i * step, x1 = std::min(q1, x0 + step);
      pool.emplace_back([&, x0, x1] { fill(ctx->pin[b] + (x0 - q0), x0, x1); });
    }
    fill(ctx->pin[b], q0, std::min(q1, q0 + step));
    for (auto& t : pool) t.join();
    MAGOT_HIP_TRY(hipMemcpyAsync(dev + q0, ctx->pin[b], q1 - q0, hipMemcpyHostToDevice,
                                 ctx->stream));
    MAGOT_HIP_TRY(hipEventRecord(ctx->pin_ev[b], ctx->stream));
  }
  return MAGOT_OK;
}

// RAII device scratch
struct DevBuf {
  void* p = nullptr;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
};

// A genome-ordered plan's output (nucleotides, or residues) put back into
// record order at dst (16-byte aligned device memory): one segment copy per
// record from its layout place to its record-order offset, on the context stream.
int plan_reassemble(magot_ctx* ctx, const magot_plan* p, bool residues, void* dst) {
  if (!p->n_tx) return MAGOT_OK;
  launch_segments_copy(residues ? p->args.pep : p->args.nuc,
                       residues ? p->d_lay_pep : p->d_lay_nuc,
                       residues ? p->d_pep_off : p->d_nuc_off, p->n_tx,
                       static_cast<uint8_t*>(dst), ctx->stream);
  MAGOT_HIP_TRY(hipGetLastError());
  return MAGOT_OK;
}

// A genome-ordered plan's output copied down in record order through a
// bounded device scratch: consecutive records in batches of at most
// kFetchBatchBytes (or one longer record) are put back into record order on
// the device (one segment-copy launch per batch), then copied to the host.
// The scratch is 16-byte aligned and the batch's first record keeps its
// offset mod 16, so the copy kernel's aligned stores stay aligned.
constexpr uint64_t kFetchBatchBytes = 256ull << 20;

uint64_t fetch_batch_bytes() {  // MAGOT_FETCH_BATCH_BYTES: test hook (small batches)
  const char* e = std::getenv("MAGOT_FETCH_BATCH_BYTES");
  const uint64_t v = e ? strtoull(e, nullptr, 10) : 0;
  return v ? v : kFetchBatchBytes;
}

int plan_fetch_reordered(magot_ctx* ctx, const magot_plan* p, bool residues, uint8_t* host) {
  const std::vector<uint64_t>& off = residues ? p->pep_off : p->nuc_off;
  const uint64_t T = p->n_tx;
  if (!T || off[T] == 0) return MAGOT_OK;
  uint64_t longest = 0;
  for (uint64_t t = 0; t < T; ++t) longest = std::max(longest, off[t + 1] - off[t]);
  const uint64_t cap = std::max(std::min(off[T], fetch_batch_bytes()), longest);
  DevBuf scratch;
  MAGOT_HIP_TRY(hipMalloc(&scratch.p, cap + 16));
  uint8_t* S = static_cast<uint8_t*>(scratch.p);
  const uint8_t* src = residues ? p->args.pep : p->args.nuc;
  const uint64_t* lay = residues ? p->d_lay_pep : p->d_lay_nuc;
  const uint64_t* doff = residues ? p->d_pep_off : p->d_nuc_off;
  for (uint64_t r0 = 0; r0 < T;) {
    uint64_t r1 = r0 + 1;
    while (r1 < T && off[r1 + 1] - off[r0] <= cap) ++r1;
    const uint64_t base = off[r0], bytes = off[r1] - base;
    if (bytes) {
      // record-order offset x lands at S + (x - (base & ~15))
      launch_segments_copy(src, lay + r0, doff + r0, r1 - r0, S - (base & ~15ull), ctx->stream);
      MAGOT_HIP_TRY(hipGetLastError());
      MAGOT_HIP_TRY(hipMemcpyAsync(host + base, S + (base & 15), bytes, hipMemcpyDeviceToHost,
                                   ctx->stream));
    }
    r0 = r1;
  }
  MAGOT_HIP_TRY(hipStreamSynchronize(ctx->stream));
  return MAGOT_OK;
}

// Device packing: raw bytes streamed to HBM once, runs counted and written by
// kernels (devpack.hip), the nibble plane packed and mirrored on the device;
// only the run list (and its directory, built from it) passes through the host.
int load_device_packed(magot_ctx* ctx, const ContigSource* src, uint32_t n_contigs,
                       magot_genome** out) {
  Lap lap;
  HostPacked hp;
  pack_layout(src, n_contigs, &hp);
  const uint64_t n = hp.extent - kOrigin;
  const uint64_t groups = (n + 31) / 32;
  const size_t scan_bytes = devpack_scan_bytes(groups);
  Carve sc;
  const uint64_t o_raw = sc.take<uint8_t>(32 * groups + 64);
  const uint64_t o_cnt = sc.take<uint32_t>(groups + 1);
  const uint64_t o_slot = sc.take<uint64_t>(groups + 1);
  const uint64_t o_tmp = sc.take<uint8_t>(scan_bytes + 1);
  DevBuf scratch;
  MAGOT_HIP_TRY(hipMalloc(&scratch.p, sc.used));
  char* sbase = static_cast<char*>(scratch.p);
  uint8_t* raw = reinterpret_cast<uint8_t*>(sbase + o_raw);
  uint32_t* cnt = reinterpret_cast<uint32_t*>(sbase + o_cnt);
  uint64_t* slot = reinterpret_cast<uint64_t*>(sbase + o_slot);
  // the padding past n is read by the 32-byte loads (and masked)
  MAGOT_HIP_TRY(hipMemsetAsync(raw + n, 0, 32 * groups + 64 - n, ctx->stream));
  if (int rc = upload_raw(ctx, src, hp, raw)) return rc;
  lap("upload");
  MAGOT_HIP_TRY(launch_run_count(raw, n, cnt, slot, sbase + o_tmp, scan_bytes, ctx->stream));
  uint64_t n_runs = 0;
  if (groups) {
    uint64_t last_slot = 0;
    uint32_t last_cnt = 0;
    MAGOT_HIP_TRY(hipMemcpyAsync(&last_slot, slot + groups - 1, 8, hipMemcpyDeviceToHost, ctx->stream));
    MAGOT_HIP_TRY(hipMemcpyAsync(&last_cnt, cnt + groups - 1, 4, hipMemcpyDeviceToHost, ctx->stream));
    MAGOT_HIP_TRY(hipStreamSynchronize(ctx->stream));
    n_runs = last_slot + last_cnt;
  }
  if (n_runs + 1 >= (uint64_t)kDirClean) {
    set_error("magot_genome_load: too many exception runs");
    return MAGOT_ERR_ARG;
  }
  DevBuf runs_tmp;
  std::vector<uint64_t> rs(n_runs), re(n_runs);
  std::vector<uint8_t> rb(n_runs);
  if (n_runs) {
    MAGOT_HIP_TRY(hipMalloc(&runs_tmp.p, n_runs * 17 + 16));
    uint64_t* d_rs = static_cast<uint64_t*>(runs_tmp.p);
    uint64_t* d_re = d_rs + n_runs;
    uint8_t* d_rb = reinterpret_cast<uint8_t*>(d_re + n_runs);
    launch_run_write(raw, n, slot, d_rs, d_re, d_rb, ctx->stream);
    MAGOT_HIP_TRY(hipGetLastError());
    MAGOT_HIP_TRY(hipMemcpyAsync(rs.data(), d_rs, n_runs * 8, hipMemcpyDeviceToHost, ctx->stream));
    MAGOT_HIP_TRY(hipMemcpyAsync(re.data(), d_re, n_runs * 8, hipMemcpyDeviceToHost, ctx->stream));
    MAGOT_HIP_TRY(hipMemcpyAsync(rb.data(), d_rb, n_runs, hipMemcpyDeviceToHost, ctx->stream));
    MAGOT_HIP_TRY(hipStreamSynchronize(ctx->stream));
  }
  // ExcRun list: runs longer than the 31-bit length field are split (as the
  // host packer does), then the sentinel and the directory
  hp.runs.clear();
  hp.runs.reserve(n_runs + 1);
  for (uint64_t k = 0; k < n_runs; ++k) {
    for (uint64_t a = rs[k]; a < re[k];) {
      const uint64_t len = std::min<uint64_t>(re[k] - a, 0x7fffffffull);
      hp.runs.push_back(ExcRun{a, (uint32_t)len, rb[k]});
      a += len;
    }
  }
  hp.runs.push_back(ExcRun{~0ull, 0, 0});
  if (hp.runs.size() >= (size_t)kDirClean) {
    set_error("magot_genome_load: too many exception runs");
    return MAGOT_ERR_ARG;
  }
  exc_runs_directory(&hp);
  lap("runs");
  std::unique_ptr<magot_genome> g(new magot_genome());
  g->ctx = ctx;
  Carve cv;
  const uint64_t o_nib = cv.take<uint32_t>(2 * hp.nib_words + 4);
  const uint64_t o_runs = cv.take<ExcRun>(hp.runs.size());
  const uint64_t o_dir = cv.take<uint32_t>(hp.dir.size());
  MAGOT_HIP_TRY(hipMalloc(&g->arena, cv.used));
  g->arena_bytes = cv.used;
  char* base = static_cast<char*>(g->arena);
  g->nib = reinterpret_cast<uint32_t*>(base + o_nib);
  g->runs = reinterpret_cast<ExcRun*>(base + o_runs);
  g->dir = reinterpret_cast<uint32_t*>(base + o_dir);
  launch_nib_pack(raw, n, g->nib, hp.nib_words, ctx->stream);
  MAGOT_HIP_TRY(hipGetLastError());
  MAGOT_HIP_TRY(hipMemsetAsync(g->nib + 2 * hp.nib_words, 0, 16, ctx->stream));
  launch_mirror_planes(g->nib, hp.span, ctx->stream);
  MAGOT_HIP_TRY(hipGetLastError());
  MAGOT_HIP_TRY(hipMemcpyAsync(g->runs, hp.runs.data(), hp.runs.size() * sizeof(ExcRun),
                               hipMemcpyHostToDevice, ctx->stream));
  MAGOT_HIP_TRY(hipMemcpyAsync(g->dir, hp.dir.data(), hp.dir.size() * 4, hipMemcpyHostToDevice,
                               ctx->stream));
  MAGOT_HIP_TRY(hipStreamSynchronize(ctx->stream));
  g->span = hp.span;
  g->contig_base = std::move(hp.contig_base);
  g->contig_len = std::move(hp.contig_len);
  g->n_runs = hp.runs.size() - 1;
  g->host_runs = std::move(hp.runs);
  g->host_dir = std::move(hp.dir);
  g->extent = hp.extent;
  g->total_bases = hp.extent - kOrigin;
  lap("pack");
  *out = g.release();
  return MAGOT_OK;
}

int load_packed(magot_ctx* ctx, const ContigSource* src, uint32_t n_contigs, uint32_t flags,
                magot_genome** out) {
  {
    uint64_t total = 0;
    for (uint32_t i = 0; i < n_contigs; ++i) total += src[i].len;
    // the packed span (kOrigin + bases + padding, pack_genome) must stay below
    // 4 Gi nibble bytes: 32-bit window offsets in extract_kernel
    if (total + kOrigin + 256 > 0xFFFFFFF0ull) {
      set_error("magot_genome_load: genomes above 4 Gbases take several device planes "
                "(engine.PartitionedGenome)");
      return MAGOT_ERR_UNSUPPORTED;
    }
  }
  if (!(flags & MAGOT_PACK_HOST)) return load_device_packed(ctx, src, n_contigs, out);
  Lap lap;
  HostPacked hp;
  pack_genome(src, n_contigs, &hp);
  lap("pack");
  if (hp.runs.size() >= (size_t)kDirClean) {
    set_error("magot_genome_load: too many exception runs");
    return MAGOT_ERR_ARG;
  }
  if (2 * hp.nib_words * 4 + 16 > 0xFFFFFFFFull) {  // 32-bit buffer offsets (extract.hip)
    set_error("magot_genome_load: genomes above 4 Gbases take several device planes");
    return MAGOT_ERR_UNSUPPORTED;
  }
  std::unique_ptr<magot_genome> g(new magot_genome());
  g->ctx = ctx;
  Carve cv;
  // forward + reverse-strand planes, 4 words of slack for window over-reads
  uint64_t o_nib = cv.take<uint32_t>(2 * hp.nib_words + 4);
  uint64_t o_runs = cv.take<ExcRun>(hp.runs.size());
  uint64_t o_dir = cv.take<uint32_t>(hp.dir.size());
  MAGOT_HIP_TRY(hipMalloc(&g->arena, cv.used));
  g->arena_bytes = cv.used;
  char* base = static_cast<char*>(g->arena);
  g->nib = reinterpret_cast<uint32_t*>(base + o_nib);
  g->runs = reinterpret_cast<ExcRun*>(base + o_runs);
  g->dir = reinterpret_cast<uint32_t*>(base + o_dir);
  MAGOT_HIP_TRY(hipMemcpy(g->nib, hp.nib.get(), hp.nib_words * 4, hipMemcpyHostToDevice));
  MAGOT_HIP_TRY(hipMemset(g->nib + 2 * hp.nib_words, 0, 16));
  launch_mirror_planes(g->nib, hp.span, ctx->stream);
  MAGOT_HIP_TRY(hipGetLastError());
  MAGOT_HIP_TRY(hipStreamSynchronize(ctx->stream));
  g->span = hp.span;
  MAGOT_HIP_TRY(hipMemcpy(g->runs, hp.runs.data(), hp.runs.size() * sizeof(ExcRun),
                          hipMemcpyHostToDevice));
  MAGOT_HIP_TRY(hipMemcpy(g->dir, hp.dir.data(), hp.dir.size() * 4, hipMemcpyHostToDevice));
  g->contig_base = std::move(hp.contig_base);
  g->contig_len = std::move(hp.contig_len);
  g->n_runs = hp.runs.size() - 1;
  g->host_runs = std::move(hp.runs);
  g->host_dir = std::move(hp.dir);
  g->extent = hp.extent;
  g->total_bases = hp.extent - kOrigin;
  lap("upload");
  *out = g.release();
  return MAGOT_OK;
}

}  // namespace

extern "C" {

int magot_genome_load_fasta(magot_ctx* ctx, const char* text, uint64_t len, int truncate_names,
                            magot_genome** out) {
  if (int rc = bind(ctx)) return rc;
  if (!out || (len && !text)) {
    set_error("magot_genome_load_fasta: null argument");
    return MAGOT_ERR_ARG;
  }
  *out = nullptr;
  FastaContigs fc;
  const auto t0 = std::chrono::steady_clock::now();
  if (int rc = scan_fasta(text, len, truncate_names != 0, &fc)) {
    set_error("magot_genome_load_fasta: header needs the Python reader");
    return rc;
  }
  if (std::getenv("MAGOT_GENOME_TIMING"))
    fprintf(stderr, "[genome] scan     %.3f s\n",
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
  magot_genome* g = nullptr;
  if (int rc = load_packed(ctx, fc.src.data(), (uint32_t)fc.src.size(), 0u, &g)) return rc;
  g->names = std::move(fc.names);
  *out = g;
  return MAGOT_OK;
}

int magot_genome_contigs(const magot_genome* g, uint32_t* n, uint64_t* lens, char* names,
                         uint64_t names_cap, uint64_t* names_len) {
  if (!g || !n) {
    set_error("magot_genome_contigs: null argument");
    return MAGOT_ERR_ARG;
  }
  *n = (uint32_t)g->contig_len.size();
  if (lens) std::memcpy(lens, g->contig_len.data(), g->contig_len.size() * 8);
  uint64_t need = 0;
  for (const auto& s : g->names) need += s.size() + 1;
  if (names_len) *names_len = need;
  if (names) {
    if (names_cap < need) {
      set_error("magot_genome_contigs: names buffer too small");
      return MAGOT_ERR_ARG;
    }
    for (const auto& s : g->names) {
      std::memcpy(names, s.data(), s.size());
      names += s.size();
      *names++ = '\0';
    }
  }
  return MAGOT_OK;
}

int magot_genome_stats(const magot_genome* g, uint64_t* total_bases, uint64_t* n_exc_runs,
                       uint64_t* device_bytes) {
  if (!g) {
    set_error("magot_genome_stats: null genome");
    return MAGOT_ERR_ARG;
  }
  if (total_bases) *total_bases = g->total_bases;
  if (n_exc_runs) *n_exc_runs = g->n_runs;
  if (device_bytes) *device_bytes = g->arena_bytes;
  return MAGOT_OK;
}

void magot_genome_destroy(magot_genome* g) {
  if (!g) return;
  if (g->ctx) (void)hipSetDevice(g->ctx->device);
  if (g->arena && g->owns_arena) (void)hipFree(g->arena);
  delete g;
}

// --- replication (one packed genome broadcast to every rank) ---------------

int magot_genome_export(const magot_genome* g, uint8_t* meta, uint64_t cap, uint64_t* meta_len,
                        uint64_t* arena_bytes) {
  if (!g || !meta_len) {
    set_error("magot_genome_export: null argument");
    return MAGOT_ERR_ARG;
  }
  const std::vector<uint8_t> m = genome_meta(g);
  *meta_len = m.size();
  if (arena_bytes) *arena_bytes = g->arena_bytes;
  if (!meta) return MAGOT_OK;
  if (cap < m.size()) {
    set_error("magot_genome_export: meta buffer too small");
    return MAGOT_ERR_ARG;
  }
  memcpy(meta, m.data(), m.size());
  return MAGOT_OK;
}

int magot_genome_copy_arena(const magot_genome* g, void* dst_dev) {
  if (!g || !dst_dev) {
    set_error("magot_genome_copy_arena: null argument");
    return MAGOT_ERR_ARG;
  }
  if (int rc = bind(g->ctx)) return rc;
  MAGOT_HIP_TRY(hipMemcpyAsync(dst_dev, g->arena, g->arena_bytes, hipMemcpyDeviceToDevice,
                               g->ctx->stream));
  MAGOT_HIP_TRY(hipStreamSynchronize(g->ctx->stream));
  return MAGOT_OK;
}

int magot_genome_attach(magot_ctx* ctx, const uint8_t* meta, uint64_t meta_len, void* arena_dev,
                        magot_genome** out) {
  if (int rc = bind(ctx)) return rc;
  if (!meta || !arena_dev || !out) {
    set_error("magot_genome_attach: null argument");
    return MAGOT_ERR_ARG;
  }
  *out = nullptr;
  std::unique_ptr<magot_genome> g(new magot_genome());
  uint64_t o[3];
  if (!parse_genome_meta(meta, meta_len, g.get(), o)) {
    set_error("magot_genome_attach: malformed genome meta");
    return MAGOT_ERR_ARG;
  }
  g->ctx = ctx;
  g->arena = arena_dev;
  g->owns_arena = false;
  char* base = static_cast<char*>(arena_dev);
  g->nib = reinterpret_cast<uint32_t*>(base + o[0]);
  g->runs = reinterpret_cast<ExcRun*>(base + o[1]);
  g->dir = reinterpret_cast<uint32_t*>(base + o[2]);
  *out = g.release();
  return MAGOT_OK;
}

int magot_genome_wire_ranges(const magot_genome* g, uint64_t* off, uint64_t* len, uint32_t* n) {
  if (!g || !off || !len || !n) {
    set_error("magot_genome_wire_ranges: null argument");
    return MAGOT_ERR_ARG;
  }
  // [forward nibble plane] and [exception runs .. directory end]: the mirror
  // plane between them (and its 16 bytes of slack) is derived on attach
  const char* a = static_cast<const char*>(g->arena);
  off[0] = (uint64_t)((const char*)g->nib - a);
  len[0] = g->span / 2;  // span bases, 8 per 4-byte word
  off[1] = (uint64_t)((const char*)g->runs - a);
  len[1] = g->arena_bytes - off[1];
  *n = 2;
  return MAGOT_OK;
}

int magot_genome_attach_wire(magot_ctx* ctx, const uint8_t* meta, uint64_t meta_len,
                             void* arena_dev, magot_genome** out) {
  if (int rc = magot_genome_attach(ctx, meta, meta_len, arena_dev, out)) return rc;
  magot_genome* g = *out;
  const uint64_t nw = g->span / 8;
  if ((uint64_t)((char*)g->runs - (char*)g->arena) < (2 * nw + 4) * 4) {
    magot_genome_destroy(g);
    *out = nullptr;
    set_error("magot_genome_attach_wire: malformed genome meta");
    return MAGOT_ERR_ARG;
  }
  hipError_t e = hipMemsetAsync(g->nib + 2 * nw, 0, 16, ctx->stream);
  if (e == hipSuccess) {
    launch_mirror_planes(g->nib, g->span, ctx->stream);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  if (e != hipSuccess) {
    magot_genome_destroy(g);
    *out = nullptr;
    set_error(std::string("magot_genome_attach_wire: ") + hipGetErrorString(e));
    return MAGOT_ERR_HIP;
  }
  return MAGOT_OK;
}

// --- the compact replica image (wire.hip) ---------------------------------

namespace {

uint64_t fnv1a(const uint8_t* p, uint64_t n) {
  uint64_t h = 0xcbf29ce484222325ull;
  for (uint64_t i = 0; i < n; ++i) h = (h ^ p[i]) * 0x100000001b3ull;
  return h;
}

// The image layout of a genome (span bases, arena_bytes with the exception
// runs at runs_off, meta blob hash) with n_mask soft-mask runs.
WireHeader wire_layout(uint64_t span, uint64_t arena_bytes, uint64_t runs_off, uint64_t n_mask,
                       uint64_t meta_hash) {
  WireHeader h{};
  h.magic = kWireMagic;
  h.meta_hash = meta_hash;
  h.span = span;
  h.n_mask = n_mask;
  h.n_mdir = (span >> kDirShift) + 2;
  Carve cv;
  cv.take<WireHeader>(1);
  h.o_code2 = cv.take<uint32_t>(span / 16);
  h.o_mask = cv.take<uint32_t>(2 * (n_mask + 1));
  h.o_mdir = cv.take<uint32_t>(h.n_mdir);
  h.exc_bytes = arena_bytes - runs_off;
  h.o_exc = cv.take<uint8_t>(h.exc_bytes);
  h.total = cv.used;
  return h;
}

}  // namespace

int magot_genome_wire_export(const magot_genome* g, void* wire_dev, uint64_t cap,
                             uint64_t* wire_bytes) {
  if (!g || !wire_bytes) {
    set_error("magot_genome_wire_export: null argument");
    return MAGOT_ERR_ARG;
  }
  if (int rc = bind(g->ctx)) return rc;
  hipStream_t st = g->ctx->stream;
  const uint64_t groups = g->span / 32;
  const size_t scan_bytes = wire_scan_bytes(groups);
  Carve sc;
  const uint64_t o_cnt = sc.take<uint32_t>(groups + 1);
  const uint64_t o_slot = sc.take<uint64_t>(groups + 1);
  const uint64_t o_tmp = sc.take<uint8_t>(scan_bytes + 1);
  DevBuf scratch;
  MAGOT_HIP_TRY(hipMalloc(&scratch.p, sc.used));
  char* sb = static_cast<char*>(scratch.p);
  uint32_t* cnt = reinterpret_cast<uint32_t*>(sb + o_cnt);
  uint64_t* slot = reinterpret_cast<uint64_t*>(sb + o_slot);
  MAGOT_HIP_TRY(launch_wire_count(g->nib, g->span, cnt, slot, sb + o_tmp, scan_bytes, st));
  uint64_t n_mask = 0;
  if (groups) {
    uint64_t last_slot = 0;
    uint32_t last_cnt = 0;
    MAGOT_HIP_TRY(hipMemcpyAsync(&last_slot, slot + groups - 1, 8, hipMemcpyDeviceToHost, st));
    MAGOT_HIP_TRY(hipMemcpyAsync(&last_cnt, cnt + groups - 1, 4, hipMemcpyDeviceToHost, st));
    MAGOT_HIP_TRY(hipStreamSynchronize(st));
    n_mask = last_slot + last_cnt;
  }
  const std::vector<uint8_t> meta = genome_meta(g);
  const WireHeader h = wire_layout(g->span, g->arena_bytes,
                                   (uint64_t)((const char*)g->runs - (const char*)g->arena), n_mask,
                                   fnv1a(meta.data(), meta.size()));
  *wire_bytes = h.total;
  if (!wire_dev) return MAGOT_OK;
  if (cap < h.total) {
    set_error("magot_genome_wire_export: image buffer too small");
    return MAGOT_ERR_ARG;
  }
  char* wb = static_cast<char*>(wire_dev);
  uint32_t* runs = reinterpret_cast<uint32_t*>(wb + h.o_mask);
  launch_code2(g->nib, g->span / 8, reinterpret_cast<uint32_t*>(wb + h.o_code2), st);
  MAGOT_HIP_TRY(hipGetLastError());
  launch_wire_runs(g->nib, g->span, slot, runs, st);
  MAGOT_HIP_TRY(hipGetLastError());
  MAGOT_HIP_TRY(hipMemsetAsync(runs + 2 * n_mask, 0xFF, 8, st));  // sentinel {~0, ~0}
  launch_wire_mdir(runs, n_mask, h.n_mdir, reinterpret_cast<uint32_t*>(wb + h.o_mdir), st);
  MAGOT_HIP_TRY(hipGetLastError());
  MAGOT_HIP_TRY(hipMemcpyAsync(wb + h.o_exc, g->runs, h.exc_bytes, hipMemcpyDeviceToDevice, st));
  MAGOT_HIP_TRY(hipMemcpyAsync(wb, &h, sizeof(h), hipMemcpyHostToDevice, st));
  MAGOT_HIP_TRY(hipStreamSynchronize(st));
  return MAGOT_OK;
}

int magot_genome_wire_import(magot_ctx* ctx, const uint8_t* meta, uint64_t meta_len,
                             const void* wire_dev, uint64_t wire_bytes, magot_genome** out) {
  if (int rc = bind(ctx)) return rc;
  if (!meta || !wire_dev || !out) {
    set_error("magot_genome_wire_import: null argument");
    return MAGOT_ERR_ARG;
  }
  *out = nullptr;
  std::unique_ptr<magot_genome> g(new magot_genome());
  uint64_t o[3];
  if (!parse_genome_meta(meta, meta_len, g.get(), o)) {
    set_error("magot_genome_wire_import: malformed genome meta");
    return MAGOT_ERR_ARG;
  }
  if (wire_bytes < sizeof(WireHeader)) {
    set_error("magot_genome_wire_import: image too small");
    return MAGOT_ERR_ARG;
  }
  WireHeader h{};
  MAGOT_HIP_TRY(hipMemcpyAsync(&h, wire_dev, sizeof(h), hipMemcpyDeviceToHost, ctx->stream));
  MAGOT_HIP_TRY(hipStreamSynchronize(ctx->stream));
  g->ctx = ctx;
  // the image must have been cut from the genome the meta describes
  const WireHeader want = wire_layout(g->span, g->arena_bytes, o[1], h.n_mask,
                                      fnv1a(meta, meta_len));
  if (h.magic != kWireMagic || h.total > wire_bytes || h.n_mask >= (1ull << 32) ||
      std::memcmp(&h, &want, sizeof(h)) != 0) {
    set_error("magot_genome_wire_import: image does not match the genome meta");
    return MAGOT_ERR_ARG;
  }
  DevBuf arena;  // owned by the genome once everything below succeeded
  MAGOT_HIP_TRY(hipMalloc(&arena.p, g->arena_bytes));
  g->arena = arena.p;
  g->owns_arena = true;
  char* base = static_cast<char*>(g->arena);
  g->nib = reinterpret_cast<uint32_t*>(base + o[0]);
  g->runs = reinterpret_cast<ExcRun*>(base + o[1]);
  g->dir = reinterpret_cast<uint32_t*>(base + o[2]);
  const char* wb = static_cast<const char*>(wire_dev);
  const ExcRun* w_exc = reinterpret_cast<const ExcRun*>(wb + h.o_exc);
  const uint32_t* w_edir = reinterpret_cast<const uint32_t*>(wb + h.o_exc + (o[2] - o[1]));
  const uint64_t nw = g->span / 8;
  hipStream_t st = ctx->stream;
  launch_wire_unpack(reinterpret_cast<const uint32_t*>(wb + h.o_code2),
                     reinterpret_cast<const uint32_t*>(wb + h.o_mask), h.n_mask,
                     reinterpret_cast<const uint32_t*>(wb + h.o_mdir), h.n_mdir, w_exc, g->n_runs,
                     w_edir, g->host_dir.size(), g->span, g->nib, st);
  MAGOT_HIP_TRY(hipGetLastError());
  MAGOT_HIP_TRY(hipMemsetAsync(g->nib + 2 * nw, 0, 16, st));
  launch_mirror_planes(g->nib, g->span, st);
  MAGOT_HIP_TRY(hipGetLastError());
  MAGOT_HIP_TRY(hipMemcpyAsync(g->runs, w_exc, h.exc_bytes, hipMemcpyDeviceToDevice, st));
  MAGOT_HIP_TRY(hipStreamSynchronize(st));
  arena.p = nullptr;
  *out = g.release();
  return MAGOT_OK;
}

int magot_copy_segments(magot_ctx* ctx, const void* src_dev, uint64_t src_bytes, void* dst_dev,
                        const uint64_t* src_off, const uint64_t* dst_off, uint64_t n) {
  if (int rc = bind(ctx)) return rc;
  if (!src_off || !dst_off) {
    set_error("magot_copy_segments: null argument");
    return MAGOT_ERR_ARG;
  }
  if (!n || dst_off[n] == dst_off[0]) return MAGOT_OK;
  if (!src_dev || !dst_dev) {
    set_error("magot_copy_segments: null buffer");
    return MAGOT_ERR_ARG;
  }
  // the kernel reads whole 16-byte blocks of src (each holds a byte of its
  // segment, so an aligned block never leaves the allocation's pages) and
  // stores 16-byte chunks at 16-aligned dst offsets
  if ((reinterpret_cast<uintptr_t>(src_dev) | reinterpret_cast<uintptr_t>(dst_dev)) & 15u) {
    set_error("magot_copy_segments: src and dst must be 16-byte aligned");
    return MAGOT_ERR_ARG;
  }
  for (uint64_t i = 0; i < n; ++i) {
    if (dst_off[i + 1] < dst_off[i]) {
      set_error("magot_copy_segments: dst_off must be non-decreasing");
      return MAGOT_ERR_ARG;
    }
    const uint64_t len = dst_off[i + 1] - dst_off[i];
    if (len && (src_off[i] > src_bytes || len > src_bytes - src_off[i])) {
      set_error("magot_copy_segments: segment " + std::to_string(i) + " reads past src_bytes");
      return MAGOT_ERR_RANGE;
    }
    // the grouped copy counts a group's 16-byte chunks in 32 bits (wavecopy.h):
    // below 4 GiB per segment, a group of kSpanGroup stays below 2^32 chunks
    if (len >> 32) {
      set_error("magot_copy_segments: segment " + std::to_string(i) +
                " is 4 GiB or longer (split it)");
      return MAGOT_ERR_ARG;
    }
  }
  DevBuf tables;
  MAGOT_HIP_TRY(hipMalloc(&tables.p, (2 * n + 1) * 8));
  uint64_t* d_src = static_cast<uint64_t*>(tables.p);
  uint64_t* d_dst = d_src + n;
  MAGOT_HIP_TRY(hipMemcpyAsync(d_src, src_off, n * 8, hipMemcpyHostToDevice, ctx->stream));
  MAGOT_HIP_TRY(hipMemcpyAsync(d_dst, dst_off, (n + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
  launch_segments_copy(static_cast<const uint8_t*>(src_dev), d_src, d_dst, n,
                       static_cast<uint8_t*>(dst_dev), ctx->stream);
  MAGOT_HIP_TRY(hipGetLastError());
  MAGOT_HIP_TRY(hipStreamSynchronize(ctx->stream));
  return MAGOT_OK;
}

int magot_plan_create(magot_ctx* ctx, const magot_genome* g, const magot_exon* exons,
                      uint64_t n_exons, const magot_tx* txs, uint64_t n_tx, uint32_t outputs,
                      magot_plan** out, uint64_t* nuc_bytes, uint64_t* pep_bytes) {
  if (int rc = bind(ctx)) return rc;
  if (!g || !out || (n_exons && !exons) || (n_tx && !txs)) {
    set_error("magot_plan_create: null argument");
    return MAGOT_ERR_ARG;
  }
  if (outputs & ~(MAGOT_OUT_NUC | MAGOT_OUT_PEP | MAGOT_OUT_GENOME_ORDER)) {
    set_error("magot_plan_create: unknown output flags");
    return MAGOT_ERR_ARG;
  }
  const bool by_genome = (outputs & MAGOT_OUT_GENOME_ORDER) != 0;
  outputs &= ~MAGOT_OUT_GENOME_ORDER;
  if (n_tx >= 0xFFFFFFFFull || n_exons >= 0xFFFFFFFFull) {
    set_error("magot_plan_create: table too large for one plan (split it)");
    return MAGOT_ERR_ARG;
  }
  *out = nullptr;
  Lap lap("MAGOT_PLAN_TIMING", "plan");
  const uint64_t E = n_exons, T = n_tx;
  // --- validate and build per-record offsets --------------------------------
  uint64_t expect = 0;
  for (uint64_t t = 0; t < T; ++t) {
    if (txs[t].exon_begin != expect) {
      set_error("magot_plan_create: record " + std::to_string(t) +
                " does not start where the previous one ended");
      return MAGOT_ERR_ARG;
    }
    expect += txs[t].n_exons;
    if (expect > E) {
      set_error("magot_plan_create: records reference more exons than given");
      return MAGOT_ERR_ARG;
    }
  }
  if (expect != E) {
    set_error("magot_plan_create: exons not covered by records");
    return MAGOT_ERR_ARG;
  }
  const uint64_t n_contigs = g->contig_base.size();
  // Host threads over record ranges for the per-interval passes (a large
  // plan: C3's 4M intervals); small plans stay on the calling thread.
  const unsigned nth = T >= (1u << 15) ? host_threads() : 1u;
  // Pass 1, record order: every interval validated, flagged and compacted
  // (zero-length intervals add no output) into words w_g / lengths w_len;
  // record t's compacted intervals are [rec_ex[t], rec_ex[t+1]).  Two
  // parallel sweeps: counts (and the first bad interval of each range), then,
  // after a prefix over the counts, the words.
  std::vector<uint64_t> rec_ex(T + 1), rec_len(T);
  std::vector<uint64_t> first_bad(nth, ~0ull);
  parallel_ranges(T, nth, [&](uint64_t t0, uint64_t t1, unsigned part) {
    for (uint64_t t = t0; t < t1; ++t) {
      uint64_t len = 0, nz = 0;
      const uint64_t e0 = txs[t].exon_begin, e1 = e0 + txs[t].n_exons;
      for (uint64_t e = e0; e < e1; ++e) {
        const magot_exon& x = exons[e];
        const uint64_t st = x.start_rc & ~kRcBit;
        if (x.contig >= n_contigs || st > g->contig_len[x.contig] ||
            st + x.len > g->contig_len[x.contig]) {
          first_bad[part] = e;
          return;
        }
        len += x.len;
        nz += x.len != 0;
      }
      rec_len[t] = len;
      rec_ex[t] = nz;
    }
  });
  for (uint64_t e : first_bad)  // ranges ascend: the first bad range holds the first bad interval
    if (e != ~0ull) {
      set_error("magot_plan_create: exon " + std::to_string(e) + " outside its contig");
      return MAGOT_ERR_RANGE;
    }
  uint64_t Ec = 0, B = 0, P = 0;
  for (uint64_t t = 0; t < T; ++t) {
    const uint64_t c = rec_ex[t];
    rec_ex[t] = Ec;
    Ec += c;
    B += rec_len[t];
    P += rec_len[t] / 3;
  }
  rec_ex[T] = Ec;
  // The output buffers' size is known now: allocate them on another thread
  // while this one plans (hipMalloc of C3's 0.8 GB takes ~10 ms).
  const uint64_t out_nuc = (outputs & MAGOT_OUT_NUC) ? B + 64 : 64;
  const uint64_t out_pep = (outputs & MAGOT_OUT_PEP) ? P + 64 : 64;
  const uint64_t out_bytes = ((out_nuc + 255) & ~255ull) + out_pep;
  void* out_arena = nullptr;
  hipError_t out_err = hipSuccess;
  std::thread out_alloc([&]() {
    out_err = hipSetDevice(ctx->device);
    if (out_err == hipSuccess) out_err = hipMalloc(&out_arena, out_bytes);
  });
  struct JoinFree {  // the allocation is joined, and freed unless the plan took it
    std::thread& th;
    void*& mem;
    ~JoinFree() {
      if (th.joinable()) th.join();
      if (mem) (void)hipFree(mem);
    }
  } out_guard{out_alloc, out_arena};
  HostBuf<uint64_t> w_g(Ec + 1);
  HostBuf<uint32_t> w_len(Ec);
  parallel_ranges(T, nth, [&](uint64_t t0, uint64_t t1, unsigned) {
    for (uint64_t t = t0; t < t1; ++t) {
      uint64_t k = rec_ex[t];
      const uint64_t e0 = txs[t].exon_begin, e1 = e0 + txs[t].n_exons;
      for (uint64_t e = e0; e < e1; ++e) {
        const magot_exon& x = exons[e];
        if (x.len == 0) continue;
        const uint64_t gs = g->contig_base[x.contig] + (x.start_rc & ~kRcBit);
        // does [gs, gs+len) touch an exception run?  (dir: first run ending past the block)
        uint64_t d = g->host_dir[gs >> kDirShift] & ~kDirClean;
        while (g->host_runs[d].start + g->host_runs[d].len <= gs) ++d;
        uint64_t exc = g->host_runs[d].start < gs + x.len ? kExcBit : 0;
        if (exc && !(x.start_rc & kRcBit)) {
          // forward strand: a byte without a literal class needs the run list
          for (uint64_t r = d; g->host_runs[r].start < gs + x.len; ++r)
            if (lit_class(g->host_runs[r].byte) == 7u) {
              exc |= kSlowLitBit;
              break;
            }
        }
        w_g[k] = gs | (x.start_rc & kRcBit) | exc;
        w_len[k] = x.len;
        ++k;
      }
    }
  });
  lap("pass1");
  // Layout order of the records: record order, or (MAGOT_OUT_GENOME_ORDER) by
  // the genome position of each record's first non-empty interval (records
  // without output last), so that records sharing genome lines run in
  // neighbouring tiles (C3: fills 0.89 -> 0.54 GB per launch); the places come
  // back through magot_plan_layout, and fetch / copy_outputs restore record order.
  std::vector<uint32_t> order;
  if (by_genome) {
    std::vector<uint64_t> key(T);
    for (uint64_t t = 0; t < T; ++t)
      key[t] = rec_ex[t] < rec_ex[t + 1] ? w_g[rec_ex[t]] & ~kExFlagBits : g->span;
    radix_order(key, &order);
  }
  lap("order");
  // Pass 2, layout order: each record's place (lay_*, indexed by record) from
  // one sweep in layout order, then the interval table with its output
  // offsets, record ranges in parallel (each record's rows are one block)
  std::vector<uint64_t> lay_nuc(T), lay_pep(T);
  HostBuf<uint64_t> lay_ex(T);
  {
    uint64_t acc = 0, q = 0, ek = 0;
    for (uint64_t k = 0; k < T; ++k) {
      const uint64_t t = by_genome ? order[k] : k;
      lay_nuc[t] = acc;
      lay_pep[t] = q;
      lay_ex[t] = ek;
      acc += rec_len[t];
      q += rec_len[t] / 3;
      ek += rec_ex[t + 1] - rec_ex[t];
    }
  }
  // interval rows in layout order (the record-order rows themselves when the
  // layout is record order), one padding row past each table (the kernel
  // prefetches clamped rows j <= n)
  HostBuf<uint64_t> ex_perm(by_genome ? Ec + 1 : 0), ex_out(Ec + 2);
  uint64_t* const ex_g = by_genome ? ex_perm.data() : w_g.data();
  parallel_ranges(T, nth, [&](uint64_t t0, uint64_t t1, unsigned) {
    for (uint64_t t = t0; t < t1; ++t) {
      uint64_t k = lay_ex[t], o = lay_nuc[t];
      for (uint64_t i = rec_ex[t]; i < rec_ex[t + 1]; ++i, ++k) {
        if (by_genome) ex_g[k] = w_g[i];
        ex_out[k] = o;
        o += w_len[i];
      }
    }
  });
  ex_g[Ec] = 0;
  ex_out[Ec] = B;
  ex_out[Ec + 1] = B;
  // Compacted record table in layout order: records with at least one codon.
  std::vector<uint64_t> tn, tp;
  tn.reserve(T + 3);
  tp.reserve(T + 3);
  for (uint64_t k = 0; k < T; ++k) {
    const uint64_t t = by_genome ? order[k] : k;
    if (rec_len[t] >= 3) {
      tn.push_back(lay_nuc[t]);
      tp.push_back(lay_pep[t]);
    }
  }
  // record-order prefix offsets (what fetch returns)
  std::vector<uint64_t> nuc_off(T + 1), pep_off(T + 1);
  nuc_off[0] = pep_off[0] = 0;
  for (uint64_t t = 0; t < T; ++t) {
    nuc_off[t + 1] = nuc_off[t] + rec_len[t];
    pep_off[t + 1] = pep_off[t] + rec_len[t] / 3;
  }
  const uint64_t Tc = tn.size();
  tn.push_back(B);
  tp.push_back(P);
  lap("pass2");
  if (Ec >= 0xFFFFFFFFull || Tc >= 0xFFFFFFFFull) {
    set_error("magot_plan_create: table too large for one plan (split it)");
    return MAGOT_ERR_ARG;
  }

  // --- tiles ----------------------------------------------------------------
  // A tile owns nucleotide bytes [T0, T1) and residues [R0, R1).  Residue
  // ownership is rounded up to 16-residue (16-byte) store chunks, so nearly
  // every peptide store is a full aligned chunk; the residues a tile owns past
  // its last codon start are decoded from its kHalo bytes of look-ahead.
  // Every query below is monotone over the cut (tile ends, decode ends and
  // residue bounds only grow), so the searches are cursors that move forward:
  // O(records + tiles) per cut instead of a binary search per query.
  struct Cursor {  // upper_bound over a non-decreasing table, for non-decreasing queries
    const uint64_t* v;
    uint64_t n, j;
    uint64_t operator()(uint64_t x) {
      while (j < n && v[j] <= x) ++j;
      return j;
    }
  };
  auto pcount = [&](Cursor& c, uint64_t T) -> uint64_t {  // residues whose codon starts before T
    const uint64_t j = c(T);
    if (j == 0) return 0;
    const uint64_t into = T - tn[j - 1];
    return tp[j - 1] + std::min((into + 2) / 3, tp[j] - tp[j - 1]);
  };
  auto rec_of = [&](Cursor& c, uint64_t q) -> uint64_t {  // compacted record holding residue q < P
    return c(q) - 1;
  };
  std::vector<uint64_t> tile_start, tile_q;
  std::vector<uint32_t> tile_ex, tile_tx;
  // cut the output into tiles of at most `tile` bytes (see tile_bytes)
  auto cut = [&](uint64_t tile) -> int {
    tile_start.clear();
    tile_q.clear();
    tile_ex.clear();
    tile_tx.clear();
    Cursor c_end{tn.data(), Tc, 0}, c_dec{tn.data(), Tc, 0};    // pcount(T1), pcount(dec_end - 2)
    Cursor c_r0{tp.data(), Tc, 0}, c_r1{tp.data(), Tc, 0};      // rec_of(R0), rec_of(R1 - 1)
    uint64_t e1 = 0, e2 = 0;
    uint64_t T0 = 0, R0 = 0;
    while (T0 < B) {
      while (e1 < Ec && ex_out[e1 + 1] <= T0) ++e1;           // interval containing T0
      const uint64_t j1 = R0 < P ? rec_of(c_r0, R0) : Tc;      // record holding residue R0
      uint64_t T1 = std::min<uint64_t>(T0 + tile, B);
      if (e1 + kExonCap < Ec) T1 = std::min<uint64_t>(T1, ex_out[e1 + kExonCap] - kHalo);
      if (j1 + kTxCap - kChunk < Tc) T1 = std::min<uint64_t>(T1, tn[j1 + kTxCap - kChunk]);
      // cut on a 128-byte line boundary where the tile keeps one (no
      // nucleotide line is then written by two tiles), else on a chunk
      if (T1 < B) T1 = (T1 & ~(uint64_t)(kTileAlign - 1)) > T0 ? T1 & ~(uint64_t)(kTileAlign - 1)
                                                             : T1 & ~(uint64_t)(kChunk - 1);
      if (T1 < T0 + kChunk) T1 = std::min<uint64_t>(T0 + kChunk, B);
      const uint64_t dec_end = std::min<uint64_t>(T1 + kHalo, B);
      // residues owned: every codon starting before T1, rounded up to a chunk,
      // but only codons that end inside the decoded range and at most kPepSlots chunks
      uint64_t R1 = P;
      if (T1 < B) {
        R1 = std::min<uint64_t>((pcount(c_end, T1) + kChunk - 1) & ~(uint64_t)(kChunk - 1), P);
        R1 = std::min<uint64_t>(R1, pcount(c_dec, dec_end - 2));
        R1 = std::min<uint64_t>(R1, (R0 & ~(uint64_t)(kChunk - 1)) + kPepSlots * kChunk);
      }
      if (R1 < R0) R1 = R0;
      if (e2 < e1) e2 = e1;
      while (e2 < Ec && ex_out[e2] < dec_end) ++e2;           // intervals touching the decode range
      const uint64_t jl = R1 > R0 ? rec_of(c_r1, R1 - 1) : 0;  // record holding the last residue
      const uint64_t j2 = R1 > R0 ? jl + 1 : j1;               // records holding residues [R0, R1)
      if (e2 - e1 > (uint64_t)kExonCap || (R1 > R0 && j2 - j1 > (uint64_t)kTxCap) ||
          (R1 > R0 && tn[jl] + 3 * (R1 - 1 - tp[jl]) + 3 > dec_end)) {
        set_error("magot_plan_create: internal tiling error");
        return MAGOT_ERR_STATE;
      }
      tile_start.push_back(T0);
      tile_q.push_back(R0);
      tile_ex.push_back((uint32_t)e1);
      tile_ex.push_back((uint32_t)e2);
      tile_tx.push_back((uint32_t)(R1 > R0 ? j1 : 0));
      tile_tx.push_back((uint32_t)(R1 > R0 ? j2 : 0));
      T0 = T1;
      R0 = R1;
    }
    if (R0 != P) {
      set_error("magot_plan_create: internal tiling error (residues)");
      return MAGOT_ERR_STATE;
    }
    return MAGOT_OK;
  };
  // the large tile, or the small one for translating plans too small to fill
  // the chip several times over (MAGOT_EXTRACT_LANE_CHUNKS=3|6 forces one, for
  // A/Bs); nucleotide-only plans keep the large tile (C2: 0.0164 vs 0.0172 ms)
  uint32_t lane_chunks = kLaneChunksLarge;
  if (int rc = cut(tile_bytes(kLaneChunksLarge))) return rc;
  const char* lc_env = std::getenv("MAGOT_EXTRACT_LANE_CHUNKS");
  const int lc_force = lc_env ? std::atoi(lc_env) : 0;
  if (lc_force == kLaneChunksSmall ||
      (lc_force != kLaneChunksLarge && (outputs & MAGOT_OUT_PEP) &&
       tile_start.size() < kSmallTilePlan)) {
    lane_chunks = kLaneChunksSmall;
    if (int rc = cut(tile_bytes(kLaneChunksSmall))) return rc;
  }
  tile_start.push_back(B);
  tile_q.push_back(P);
  lap("tiles");
  const uint64_t n_tiles64 = tile_start.size() - 1;
  if (n_tiles64 >= 0x7FFFFFFFull) {
    set_error("magot_plan_create: output too large for one launch");
    return MAGOT_ERR_ARG;
  }
  const uint32_t n_tiles = (uint32_t)n_tiles64;
  // Launch order: tiles that may take the run-list path first -- a staged
  // interval over a byte without a literal class (kSlowLitBit), or one short
  // enough that a chunk can span three intervals.  Their chains of dependent
  // run-list loads then overlap the rest of the launch; at the end of the grid
  // they set its tail (C2: 0.0174 ms with the 23 such tiles where they fall,
  // 0.0151 ms with none).  Every other tile keeps output order.
  std::vector<uint8_t> slow_tile(n_tiles);
  parallel_ranges(n_tiles, n_tiles >= (1u << 14) ? nth : 1u, [&](uint64_t t0, uint64_t t1, unsigned) {
    for (uint64_t t = t0; t < t1; ++t) {
      bool slow = false;
      for (uint32_t e = tile_ex[2 * t]; e < tile_ex[2 * t + 1] && !slow; ++e)
        slow = (ex_g[e] & kSlowLitBit) || ex_out[e + 1] - ex_out[e] < (uint64_t)kChunk;
      slow_tile[t] = slow;
    }
  });
  std::vector<TileRec> tiles(n_tiles);
  std::vector<TileRec> tail;
  uint32_t n_first = 0;
  for (uint32_t t = 0; t < n_tiles; ++t) {
    const TileRec r{tile_start[t], tile_start[t + 1], tile_q[t], tile_q[t + 1],
                    tile_ex[2 * t], tile_ex[2 * t + 1], tile_tx[2 * t], tile_tx[2 * t + 1]};
    if (slow_tile[t]) tiles[n_first++] = r;
    else tail.push_back(r);
  }
  std::copy(tail.begin(), tail.end(), tiles.begin() + n_first);
  lap("launch_ord");

  // --- device arena -----------------------------------------------------------
  std::unique_ptr<magot_plan> p(new magot_plan());
  p->ctx = ctx;
  p->g = g;
  Carve cv;
  // one padding row past each table: the kernel prefetches clamped rows j <= n
  tn.push_back(B);
  tp.push_back(P);
  const uint64_t o_exg = cv.take<uint64_t>(Ec + 1);
  const uint64_t o_exo = cv.take<uint64_t>(Ec + 2);
  const uint64_t o_txn = cv.take<uint64_t>(Tc + 2);
  const uint64_t o_txp = cv.take<uint64_t>(Tc + 2);
  const uint64_t o_tiles = cv.take<TileRec>(n_tiles + 1);
  // genome order: {layout place, record-order offsets} per output, for the
  // reassembly copies (magot_plan_fetch / copy_outputs)
  const uint64_t lay_rows = by_genome ? T : 0;
  const uint64_t o_lay_nuc = cv.take<uint64_t>(lay_rows);
  const uint64_t o_rec_nuc = cv.take<uint64_t>(by_genome ? T + 1 : 0);
  const uint64_t o_lay_pep = cv.take<uint64_t>(lay_rows);
  const uint64_t o_rec_pep = cv.take<uint64_t>(by_genome ? T + 1 : 0);
  MAGOT_HIP_TRY(hipMalloc(&p->arena, cv.used));
  p->arena_bytes = cv.used;
  out_alloc.join();
  MAGOT_HIP_TRY(out_err);
  p->out_arena = out_arena;
  p->out_bytes = out_bytes;
  out_arena = nullptr;  // the plan owns it now
  lap("malloc");
  char* base = static_cast<char*>(p->arena);
  std::vector<HostPiece> pieces = {{o_exg, ex_g, (Ec + 1) * 8},
                                   {o_exo, ex_out.data(), (Ec + 2) * 8},
                                   {o_txn, tn.data(), (Tc + 2) * 8},
                                   {o_txp, tp.data(), (Tc + 2) * 8},
                                   {o_tiles, tiles.data(), tiles.size() * sizeof(TileRec)}};
  if (by_genome) {
    pieces.push_back({o_lay_nuc, lay_nuc.data(), T * 8});
    pieces.push_back({o_rec_nuc, nuc_off.data(), (T + 1) * 8});
    pieces.push_back({o_lay_pep, lay_pep.data(), T * 8});
    pieces.push_back({o_rec_pep, pep_off.data(), (T + 1) * 8});
  }
  if (int rc = upload_pieces(ctx, base, pieces)) return rc;
  if (by_genome) {
    p->genome_order = true;
    p->d_lay_nuc = reinterpret_cast<const uint64_t*>(base + o_lay_nuc);
    p->d_nuc_off = reinterpret_cast<const uint64_t*>(base + o_rec_nuc);
    p->d_lay_pep = reinterpret_cast<const uint64_t*>(base + o_lay_pep);
    p->d_pep_off = reinterpret_cast<const uint64_t*>(base + o_rec_pep);
  }
  lap("upload");

  ExtractArgs& a = p->args;
  a.nib = g->nib;
  a.span = g->span;
  a.runs = g->runs;
  a.dir = g->dir;
  a.ex_g = reinterpret_cast<const uint64_t*>(base + o_exg);
  a.ex_out = reinterpret_cast<const uint64_t*>(base + o_exo);
  a.tx_nuc = reinterpret_cast<const uint64_t*>(base + o_txn);
  a.tx_pep = reinterpret_cast<const uint64_t*>(base + o_txp);
  a.tiles = reinterpret_cast<const TileRec*>(base + o_tiles);
  a.nuc = static_cast<uint8_t*>(p->out_arena);
  a.pep = static_cast<uint8_t*>(p->out_arena) + ((out_nuc + 255) & ~255ull);
  a.total_nuc = B;
  a.total_pep = P;
  a.n_tiles = n_tiles;
  a.outputs = outputs;
  a.lane_chunks = lane_chunks;
  if (const char* dbg = std::getenv("MAGOT_DEBUG_PATHS")) {
    const int v = std::atoi(dbg);
    if (v & 1) a.outputs |= kDebugSlowNuc;
    if (v & 2) a.outputs |= kDebugSlowPep;
  }
  uint8_t lut[64];
  standard_lut(lut);
  std::memcpy(a.lut, lut, 64);

  p->nuc_off = std::move(nuc_off);
  p->pep_off = std::move(pep_off);
  p->lay_nuc = std::move(lay_nuc);
  p->lay_pep = std::move(lay_pep);
  p->n_exons = E;
  p->n_ex_c = Ec;
  p->n_tx = T;
  if (nuc_bytes) *nuc_bytes = B;
  if (pep_bytes) *pep_bytes = P;
  *out = p.release();
  return MAGOT_OK;
}

void magot_plan_destroy(magot_plan* p) {
  if (!p) return;
  if (p->ctx) (void)hipSetDevice(p->ctx->device);
  if (p->arena) (void)hipFree(p->arena);
  if (p->out_arena) (void)hipFree(p->out_arena);
  delete p;
}

int magot_plan_execute(magot_ctx* ctx, magot_plan* p) {
  if (int rc = bind(ctx)) return rc;
  if (!p) {
    set_error("magot_plan_execute: null plan");
    return MAGOT_ERR_ARG;
  }
  launch_extract(p->args, ctx->stream);
  MAGOT_HIP_TRY(hipGetLastError());
  p->executed = true;
  return MAGOT_OK;
}

int magot_plan_fetch(magot_ctx* ctx, magot_plan* p, uint8_t* nuc_out, uint64_t* nuc_off,
                     uint8_t* pep_out, uint64_t* pep_off) {
  if (int rc = bind(ctx)) return rc;
  if (!p) {
    set_error("magot_plan_fetch: null plan");
    return MAGOT_ERR_ARG;
  }
  if (!p->executed) {
    set_error("magot_plan_fetch: plan not executed");
    return MAGOT_ERR_STATE;
  }
  MAGOT_HIP_TRY(hipStreamSynchronize(ctx->stream));
  if ((nuc_out && p->args.total_nuc && !(p->args.outputs & MAGOT_OUT_NUC)) ||
      (pep_out && p->args.total_pep && !(p->args.outputs & MAGOT_OUT_PEP))) {
    set_error(std::string("magot_plan_fetch: plan built without ") +
              (nuc_out && !(p->args.outputs & MAGOT_OUT_NUC) ? "MAGOT_OUT_NUC" : "MAGOT_OUT_PEP"));
    return MAGOT_ERR_STATE;
  }
  const bool want_nuc = nuc_out && p->args.total_nuc, want_pep = pep_out && p->args.total_pep;
  if (want_nuc) {
    if (p->genome_order) {
      if (int rc = plan_fetch_reordered(ctx, p, false, nuc_out)) return rc;
    } else {
      MAGOT_HIP_TRY(hipMemcpyAsync(nuc_out, p->args.nuc, p->args.total_nuc,
                                   hipMemcpyDeviceToHost, ctx->stream));
      MAGOT_HIP_TRY(hipStreamSynchronize(ctx->stream));
    }
  }
  if (want_pep) {
    if (p->genome_order) {
      if (int rc = plan_fetch_reordered(ctx, p, true, pep_out)) return rc;
    } else {
      MAGOT_HIP_TRY(hipMemcpyAsync(pep_out, p->args.pep, p->args.total_pep,
                                   hipMemcpyDeviceToHost, ctx->stream));
      MAGOT_HIP_TRY(hipStreamSynchronize(ctx->stream));
    }
  }
  if (nuc_off) std::memcpy(nuc_off, p->nuc_off.data(), p->nuc_off.size() * 8);
  if (pep_off) std::memcpy(pep_off, p->pep_off.data(), p->pep_off.size() * 8);
  return MAGOT_OK;
}

int magot_run(magot_ctx* ctx, magot_plan* p, uint8_t* nuc_out, uint64_t* nuc_off, uint8_t* pep_out,
              uint64_t* pep_off) {
  if (int rc = magot_plan_execute(ctx, p)) return rc;
  return magot_plan_fetch(ctx, p, nuc_out, nuc_off, pep_out, pep_off);
}

int magot_plan_time(magot_ctx* ctx, magot_plan* p, int iters, double* avg_ms) {
  if (int rc = bind(ctx)) return rc;
  if (!p || iters <= 0 || !avg_ms) {
    set_error("magot_plan_time: bad argument");
    return MAGOT_ERR_ARG;
  }
  double total = 0.0;
  for (int i = 0; i < iters; ++i) {
    MAGOT_HIP_TRY(hipEventRecord(ctx->ev0, ctx->stream));
    launch_extract(p->args, ctx->stream);
    MAGOT_HIP_TRY(hipGetLastError());
    MAGOT_HIP_TRY(hipEventRecord(ctx->ev1, ctx->stream));
    MAGOT_HIP_TRY(hipEventSynchronize(ctx->ev1));
    float ms = 0.f;
    MAGOT_HIP_TRY(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
    total += ms;
  }
  p->executed = true;
  *avg_ms = total / iters;
  return MAGOT_OK;
}

int magot_plan_time_b2b(magot_ctx* ctx, magot_plan* p, int iters, double* avg_ms) {
  if (int rc = bind(ctx)) return rc;
  if (!p || iters <= 0 || !avg_ms) {
    set_error("magot_plan_time_b2b: bad argument");
    return MAGOT_ERR_ARG;
  }
  // one event pair around `iters` back-to-back launches: the per-launch time
  // of a step loop (no host round trip between launches)
  MAGOT_HIP_TRY(hipEventRecord(ctx->ev0, ctx->stream));
  for (int i = 0; i < iters; ++i) launch_extract(p->args, ctx->stream);
  MAGOT_HIP_TRY(hipGetLastError());
  MAGOT_HIP_TRY(hipEventRecord(ctx->ev1, ctx->stream));
  MAGOT_HIP_TRY(hipEventSynchronize(ctx->ev1));
  float ms = 0.f;
  MAGOT_HIP_TRY(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
  p->executed = true;
  *avg_ms = (double)ms / iters;
  return MAGOT_OK;
}

int magot_plan_copy_outputs(magot_ctx* ctx, magot_plan* p, void* nuc_dst_dev, void* pep_dst_dev) {
  if (int rc = bind(ctx)) return rc;
  if (!p) {
    set_error("magot_plan_copy_outputs: null plan");
    return MAGOT_ERR_ARG;
  }
  if (p->genome_order && ((nuc_dst_dev && (reinterpret_cast<uintptr_t>(nuc_dst_dev) & 15)) ||
                          (pep_dst_dev && (reinterpret_cast<uintptr_t>(pep_dst_dev) & 15)))) {
    set_error("magot_plan_copy_outputs: a genome-ordered plan needs 16-byte aligned destinations");
    return MAGOT_ERR_ARG;
  }
  if (nuc_dst_dev && p->args.total_nuc && (p->args.outputs & MAGOT_OUT_NUC)) {
    if (p->genome_order) {
      if (int rc = plan_reassemble(ctx, p, false, nuc_dst_dev)) return rc;
    } else {
      MAGOT_HIP_TRY(hipMemcpyAsync(nuc_dst_dev, p->args.nuc, p->args.total_nuc,
                                   hipMemcpyDeviceToDevice, ctx->stream));
    }
  }
  if (pep_dst_dev && p->args.total_pep && (p->args.outputs & MAGOT_OUT_PEP)) {
    if (p->genome_order) {
      if (int rc = plan_reassemble(ctx, p, true, pep_dst_dev)) return rc;
    } else {
      MAGOT_HIP_TRY(hipMemcpyAsync(pep_dst_dev, p->args.pep, p->args.total_pep,
                                   hipMemcpyDeviceToDevice, ctx->stream));
    }
  }
  MAGOT_HIP_TRY(hipStreamSynchronize(ctx->stream));
  return MAGOT_OK;
}

int magot_plan_layout(const magot_plan* p, uint64_t* nuc_start, uint64_t* pep_start) {
  if (!p) {
    set_error("magot_plan_layout: null plan");
    return MAGOT_ERR_ARG;
  }
  const uint64_t T = p->n_tx;
  if (nuc_start) {
    if (p->genome_order) std::memcpy(nuc_start, p->lay_nuc.data(), T * 8);
    else std::memcpy(nuc_start, p->nuc_off.data(), T * 8);
  }
  if (pep_start) {
    if (p->genome_order) std::memcpy(pep_start, p->lay_pep.data(), T * 8);
    else std::memcpy(pep_start, p->pep_off.data(), T * 8);
  }
  return MAGOT_OK;
}

int magot_plan_device_outputs(magot_plan* p, void** nuc_dev, void** pep_dev) {
  if (!p) {
    set_error("magot_plan_device_outputs: null plan");
    return MAGOT_ERR_ARG;
  }
  if (nuc_dev) *nuc_dev = p->args.nuc;
  if (pep_dev) *pep_dev = p->args.pep;
  return MAGOT_OK;
}

uint64_t magot_plan_algorithmic_bytes(const magot_plan* p) {
  if (!p) return 0;
  const uint64_t B = p->args.total_nuc, P = p->args.total_pep;
  uint64_t bytes = (B + 3) / 4 + 16 * p->n_exons + 32 * p->n_tx;
  if (p->args.outputs & MAGOT_OUT_NUC) bytes += B;
  if (p->args.outputs & MAGOT_OUT_PEP) bytes += P;
  return bytes;
}

int magot_revcomp_batch(magot_ctx* ctx, const uint8_t* seqs, const uint64_t* seq_off, uint64_t n,
                        uint8_t* out) {
  if (int rc = bind(ctx)) return rc;
  if (!seq_off) {
    set_error("magot_revcomp_batch: null argument");
    return MAGOT_ERR_ARG;
  }
  const uint64_t total = n ? seq_off[n] : 0;
  if (total == 0) return MAGOT_OK;  // empty strings only: nothing to read or write
  if (!seqs || !out) {
    set_error("magot_revcomp_batch: null argument");
    return MAGOT_ERR_ARG;
  }
  for (uint64_t i = 0; i < n; ++i)
    if (seq_off[i + 1] < seq_off[i]) {
      set_error("magot_revcomp_batch: offsets not monotone");
      return MAGOT_ERR_ARG;
    }
  void* d = nullptr;
  const uint64_t off_bytes = (n + 1) * 8, pad = 64;
  MAGOT_HIP_TRY(hipMalloc(&d, 2 * (total + pad) + off_bytes));
  uint8_t* d_in = static_cast<uint8_t*>(d);
  uint8_t* d_out = d_in + total + pad;
  uint64_t* d_off = reinterpret_cast<uint64_t*>(d_out + total + pad);
  int rc = MAGOT_OK;
  hipError_t e = hipMemcpyAsync(d_in, seqs, total, hipMemcpyHostToDevice, ctx->stream);
  if (e == hipSuccess)
    e = hipMemcpyAsync(d_off, seq_off, off_bytes, hipMemcpyHostToDevice, ctx->stream);
  if (e == hipSuccess) {
    launch_revcomp(d_in, d_off, n, total, d_out, ctx->stream);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpyAsync(out, d_out, total, hipMemcpyDeviceToHost, ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  if (e != hipSuccess) {
    set_error(std::string("magot_revcomp_batch: ") + hipGetErrorString(e));
    rc = MAGOT_ERR_HIP;
  }
  (void)hipFree(d);
  return rc;
}

int magot_translate_sizes(const uint64_t* seq_off, uint64_t n, const int32_t* frames,
                          uint64_t* pep_off, int64_t* codons_out) {
  if (!seq_off || !pep_off || (n && !frames)) {
    set_error("magot_translate_sizes: null argument");
    return MAGOT_ERR_ARG;
  }
  uint64_t acc = 0;
  for (uint64_t i = 0; i < n; ++i) {
    const int64_t f = frames[i];
    if (f < 0) {
      set_error("magot_translate_sizes: negative frame");
      return MAGOT_ERR_ARG;
    }
    const int64_t L = (int64_t)(seq_off[i + 1] - seq_off[i]);
    int64_t c = -1;
    if (L > 2 + f) {
      const int64_t pe = f + ((2 - 2 * f) % 3 + 3) % 3;
      c = 1 + (L - 1 - pe) / 3;
    }
    pep_off[i] = acc;
    if (codons_out) codons_out[i] = c;
    if (c > 0) acc += (uint64_t)c;
  }
  pep_off[n] = acc;
  return MAGOT_OK;
}

int magot_translate_batch(magot_ctx* ctx, const uint8_t* seqs, const uint64_t* seq_off, uint64_t n,
                          const int32_t* frames, const uint8_t* strands, const uint8_t* lut64,
                          const uint64_t* pep_off, uint8_t* out) {
  if (int rc = bind(ctx)) return rc;
  if (!seq_off || !pep_off || (n && (!frames || !strands))) {
    set_error("magot_translate_batch: null argument");
    return MAGOT_ERR_ARG;
  }
  for (uint64_t i = 0; i < n; ++i)
    if (strands[i] != '+' && strands[i] != '-') {
      set_error("magot_translate_batch: strand must be '+' or '-'");
      return MAGOT_ERR_ARG;
    }
  const uint64_t total = n ? seq_off[n] : 0, total_pep = n ? pep_off[n] : 0;
  if (total_pep == 0) return MAGOT_OK;
  if (!seqs || !out) {
    set_error("magot_translate_batch: null buffer");
    return MAGOT_ERR_ARG;
  }
  uint8_t lut[64];
  if (lut64) std::memcpy(lut, lut64, 64);
  else standard_lut(lut);
  uint32_t lut16[16];
  std::memcpy(lut16, lut, 64);
  const uint64_t pad = 64, ob = (n + 1) * 8;
  const uint64_t bytes = (total + pad) + (total_pep + pad) + 2 * ob + n * 4 + n + pad;
  void* d = nullptr;
  MAGOT_HIP_TRY(hipMalloc(&d, bytes));
  uint8_t* d_in = static_cast<uint8_t*>(d);
  uint8_t* d_out = d_in + total + pad;
  uint64_t* d_off = reinterpret_cast<uint64_t*>((reinterpret_cast<uintptr_t>(d_out + total_pep + pad) + 7) & ~7ull);
  uint64_t* d_poff = d_off + (n + 1);
  int32_t* d_fr = reinterpret_cast<int32_t*>(d_poff + (n + 1));
  uint8_t* d_st = reinterpret_cast<uint8_t*>(d_fr + n);
  hipError_t e = hipSuccess;
  if (total) e = hipMemcpyAsync(d_in, seqs, total, hipMemcpyHostToDevice, ctx->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(d_off, seq_off, ob, hipMemcpyHostToDevice, ctx->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(d_poff, pep_off, ob, hipMemcpyHostToDevice, ctx->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(d_fr, frames, n * 4, hipMemcpyHostToDevice, ctx->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(d_st, strands, n, hipMemcpyHostToDevice, ctx->stream);
  if (e == hipSuccess) {
    launch_translate(d_in, d_off, n, d_fr, d_st, d_poff, total_pep, lut16, d_out, ctx->stream);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpyAsync(out, d_out, total_pep, hipMemcpyDeviceToHost, ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  int rc = MAGOT_OK;
  if (e != hipSuccess) {
    set_error(std::string("magot_translate_batch: ") + hipGetErrorString(e));
    rc = MAGOT_ERR_HIP;
  }
  (void)hipFree(d);
  return rc;
}

int magot_codon_symbols(magot_ctx* ctx, const uint8_t* seq, uint64_t n_codons,
                        const uint8_t* class256, uint32_t n_classes, const uint8_t* lut,
                        uint8_t* out) {
  if (int rc = bind(ctx)) return rc;
  const uint64_t nl = (uint64_t)n_classes * n_classes * n_classes;
  if (!class256 || !lut || n_classes == 0 || nl > kMaxSymbolLut || (n_codons && (!seq || !out))) {
    set_error("magot_codon_symbols: bad argument");
    return MAGOT_ERR_ARG;
  }
  for (int b = 0; b < 256; ++b)
    if (class256[b] >= n_classes) {
      set_error("magot_codon_symbols: class out of range");
      return MAGOT_ERR_ARG;
    }
  if (n_codons == 0) return MAGOT_OK;
  const uint64_t in_bytes = 3 * n_codons;
  void* d = nullptr;
  MAGOT_HIP_TRY(hipMalloc(&d, in_bytes + n_codons + 256 + nl + 64));
  uint8_t* d_in = static_cast<uint8_t*>(d);
  uint8_t* d_out = d_in + in_bytes;
  uint8_t* d_cls = d_out + n_codons;
  uint8_t* d_lut = d_cls + 256;
  hipError_t e = hipMemcpyAsync(d_in, seq, in_bytes, hipMemcpyHostToDevice, ctx->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(d_cls, class256, 256, hipMemcpyHostToDevice, ctx->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(d_lut, lut, nl, hipMemcpyHostToDevice, ctx->stream);
  if (e == hipSuccess) {
    launch_codon_symbols(d_in, n_codons, d_cls, n_classes, d_lut, d_out, ctx->stream);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpyAsync(out, d_out, n_codons, hipMemcpyDeviceToHost, ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  (void)hipFree(d);
  if (e != hipSuccess) {
    set_error(std::string("magot_codon_symbols: ") + hipGetErrorString(e));
    return MAGOT_ERR_HIP;
  }
  return MAGOT_OK;
}

// --- single sequences (SURVEY 8(b) sketch) ---------------------------------

int magot_revcomp(magot_ctx* ctx, const uint8_t* seq, uint64_t len, uint8_t* out) {
  const uint64_t off[2] = {0, len};
  return magot_revcomp_batch(ctx, seq, off, 1, out);
}

int magot_translate(magot_ctx* ctx, const uint8_t* seq, uint64_t len, int frame, int strand,
                    int trimX, uint8_t* out, int64_t* out_len) {
  if (!out_len || (len && !seq)) {
    set_error("magot_translate: null argument");
    return MAGOT_ERR_ARG;
  }
  if (strand != '+' && strand != '-') {
    set_error("magot_translate: strand must be '+' or '-'");
    return MAGOT_ERR_ARG;
  }
  if (frame < 0) {
    set_error("magot_translate: negative frame (the Python layer lays those out itself)");
    return MAGOT_ERR_UNSUPPORTED;
  }
  const uint64_t off[2] = {0, len};
  const int32_t fr = frame;
  uint64_t poff[2];
  int64_t codons = 0;
  if (int rc = magot_translate_sizes(off, 1, &fr, poff, &codons)) return rc;
  if (codons < 0) {  // translate() returns None (len <= 2 + frame)
    *out_len = -1;
    return MAGOT_OK;
  }
  if (codons && !out) {
    set_error("magot_translate: null output");
    return MAGOT_ERR_ARG;
  }
  const uint8_t st = (uint8_t)strand;
  // translated into a private buffer, so exactly *out_len bytes reach `out`
  std::vector<uint8_t> tmp((size_t)codons + 1);
  if (int rc = magot_translate_batch(ctx, seq, off, 1, &fr, &st, nullptr, poff, tmp.data()))
    return rc;
  int64_t n = codons;
  const uint8_t* res = tmp.data();
  if (trimX && n > 0 && res[0] == 'X') {  // genome.py:819-821
    ++res;
    --n;
  }
  if (n) std::memcpy(out, res, (size_t)n);
  *out_len = n;
  return MAGOT_OK;
}

// --- six-frame translation (Sequence.get_orfs, genome.py:824-851) ----------

int magot_orf6_sizes(const uint64_t* seq_off, uint64_t n, uint64_t* stream_off,
                     uint64_t* stream_len, uint8_t* none_mask) {
  if (!seq_off || !stream_off) {
    set_error("magot_orf6_sizes: null argument");
    return MAGOT_ERR_ARG;
  }
  // A record's streams are placed strand-major: its three '-' streams, then
  // its three '+' streams.  orf6_kernel writes every '-' chunk of a record
  // batch before its '+' chunks (strand-uniform chunk passes), so each pass
  // then stores one contiguous run per record instead of three runs with
  // gaps the other pass fills later (whose shared 128-B lines leave L2 half
  // written).
  uint64_t acc = 0;
  for (uint64_t r = 0; r < n; ++r) {
    const uint64_t L = seq_off[r + 1] - seq_off[r];
    for (int st = 0; st < 2; ++st) {
      for (uint32_t f = 0; f < 3; ++f) {
        // real codons start at 2f, 2f+3, ... (frames 1/2 emit a junk codon first)
        const bool none = L <= 2 + f;
        const uint64_t c = (!none && L >= 2 * f + 3) ? (L - 2 * f) / 3 : 0;
        const uint64_t j = 6 * r + 2 * f + st;
        stream_off[j] = acc;  // streams start on 16-byte boundaries
        if (stream_len) stream_len[j] = c;
        if (none_mask) none_mask[j] = none ? 1 : 0;
        acc += (c + 15) & ~15ull;
      }
    }
  }
  stream_off[6 * n] = acc;
  return MAGOT_OK;
}

int magot_orf6_batch(magot_ctx* ctx, const uint8_t* seqs, const uint64_t* seq_off, uint64_t n,
                     const uint8_t* lut64, const uint64_t* stream_off, uint8_t* out) {
  if (int rc = bind(ctx)) return rc;
  if (!seq_off || !stream_off) {
    set_error("magot_orf6_batch: null argument");
    return MAGOT_ERR_ARG;
  }
  for (uint64_t r = 0; r < n; ++r)
    if (seq_off[r + 1] < seq_off[r]) {
      set_error("magot_orf6_batch: seq_off must be non-decreasing");
      return MAGOT_ERR_ARG;
    }
  {
    // the kernel places each stream from its record's block start and length
    // (magot_orf6_sizes' layout); a different table would send its stores
    // past the caller's buffer, so it is refused
    std::vector<uint64_t> want(6 * n + 1);
    magot_orf6_sizes(seq_off, n, want.data(), nullptr, nullptr);
    if (std::memcmp(want.data(), stream_off, want.size() * 8) != 0) {
      set_error("magot_orf6_batch: stream_off is not magot_orf6_sizes' table for seq_off");
      return MAGOT_ERR_ARG;
    }
  }
  const uint64_t total = n ? seq_off[n] : 0, total_res = n ? stream_off[6 * n] : 0;
  if (total_res == 0) return MAGOT_OK;
  if (!seqs || !out) {
    set_error("magot_orf6_batch: null buffer");
    return MAGOT_ERR_ARG;
  }
  uint8_t lut[64], tables[256];
  if (lut64) std::memcpy(lut, lut64, 64);
  else standard_lut(lut);
  orf6_tables(lut, tables);
  Orf6Tiles tiles;
  orf6_plan_tiles(seq_off, n, nullptr, 0, &tiles);
  const uint64_t n_tiles = tiles.r0.size();
  Carve cv;
  const uint64_t o_in = cv.take<uint8_t>(total + 64);
  const uint64_t o_out = cv.take<uint8_t>(total_res + 64);
  const uint64_t o_off = cv.take<uint64_t>(n + 1);
  const uint64_t o_boff = cv.take<uint64_t>(n + 1);
  const uint64_t o_t0 = cv.take<uint64_t>(n_tiles + 1);
  const uint64_t o_r0 = cv.take<uint32_t>(n_tiles);
  const uint64_t o_lut = cv.take<uint8_t>(256);
  void* d = nullptr;
  MAGOT_HIP_TRY(hipMalloc(&d, cv.used));
  char* base = static_cast<char*>(d);
  hipError_t e = hipMemcpyAsync(base + o_in, seqs, total, hipMemcpyHostToDevice, ctx->stream);
  if (e == hipSuccess)
    e = hipMemcpyAsync(base + o_lut, tables, 256, hipMemcpyHostToDevice, ctx->stream);
  if (e == hipSuccess)
    e = hipMemcpyAsync(base + o_off, seq_off, (n + 1) * 8, hipMemcpyHostToDevice, ctx->stream);
  // the kernel takes each record's block start (its streams' places follow
  // from the record length, magot_orf6_sizes' layout)
  std::vector<uint64_t> boff(n + 1);
  for (uint64_t r = 0; r <= n; ++r) boff[r] = stream_off[6 * r];
  if (e == hipSuccess)
    e = hipMemcpyAsync(base + o_boff, boff.data(), (n + 1) * 8, hipMemcpyHostToDevice, ctx->stream);
  if (e == hipSuccess)
    e = hipMemcpyAsync(base + o_t0, tiles.t0.data(), (n_tiles + 1) * 8, hipMemcpyHostToDevice,
                       ctx->stream);
  if (e == hipSuccess && n_tiles)
    e = hipMemcpyAsync(base + o_r0, tiles.r0.data(), n_tiles * 4, hipMemcpyHostToDevice,
                       ctx->stream);
  if (e == hipSuccess) {
    Orf6Args a{};
    a.nuc = reinterpret_cast<const uint8_t*>(base + o_in);
    a.noff = reinterpret_cast<const uint64_t*>(base + o_off);
    a.n_rec = n;
    a.total = total;
    a.boff = reinterpret_cast<const uint64_t*>(base + o_boff);
    a.tile_t0 = reinterpret_cast<const uint64_t*>(base + o_t0);
    a.tile_r0 = reinterpret_cast<const uint32_t*>(base + o_r0);
    a.n_tiles = n_tiles;
    a.tables = reinterpret_cast<const uint8_t*>(base + o_lut);
    a.out = reinterpret_cast<uint8_t*>(base + o_out);
    launch_orf6(a, false, ctx->stream);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpyAsync(out, base + o_out, total_res, hipMemcpyDeviceToHost, ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  int rc = MAGOT_OK;
  if (e != hipSuccess) {
    set_error(std::string("magot_orf6_batch: ") + hipGetErrorString(e));
    rc = MAGOT_ERR_HIP;
  }
  (void)hipFree(d);
  return rc;
}

// Six frames over an extraction plan: the records are gathered from the
// genome plane through the plan's intervals inside the kernel (fused; the
// plan's nucleotide output is not read).
struct magot_orf6 {
  magot_ctx* ctx = nullptr;
  magot_plan* plan = nullptr;
  void* arena = nullptr;
  Orf6Args args{};
  uint8_t* out = nullptr;
  uint64_t n_rec = 0, total = 0;
  std::vector<uint64_t> host_soff;
  void launch(hipStream_t s) const { launch_orf6(args, true, s); }
};

int magot_plan_orf6(magot_ctx* ctx, magot_plan* p, const uint8_t* lut64, magot_orf6** out,
                    uint64_t* total_res) {
  if (int rc = bind(ctx)) return rc;
  if (!p || !out) {
    set_error("magot_plan_orf6: null argument");
    return MAGOT_ERR_ARG;
  }
  *out = nullptr;
  if (p->genome_order) {
    // the six-frame plan walks the plan's intervals against record-order
    // offsets (and lays its own walk out in genome order anyway)
    set_error("magot_plan_orf6: plan built with MAGOT_OUT_GENOME_ORDER (build it without)");
    return MAGOT_ERR_ARG;
  }
  std::unique_ptr<magot_orf6> o(new magot_orf6());
  o->ctx = ctx;
  o->plan = p;
  o->n_rec = p->n_tx;
  o->host_soff.resize(6 * o->n_rec + 1);
  if (int rc = magot_orf6_sizes(p->nuc_off.data(), o->n_rec, o->host_soff.data(), nullptr, nullptr))
    return rc;
  o->total = o->host_soff.back();
  const uint64_t total_nuc = p->nuc_off.back();
  // interval rows {unified anchor, start} from the plan's compacted table
  // (a '-' interval reads the mirror plane forward; staging every interval
  // from the forward planes instead, '-' read backwards and reverse-
  // complemented in registers, measured 5 % slower: DESIGN.md 4, round 4)
  const uint64_t ne = p->n_ex_c;
  std::vector<uint64_t> ex_g(ne), ex_out(ne + 1), rows(2 * (ne + 1));
  if (ne) {
    MAGOT_HIP_TRY(hipMemcpy(ex_g.data(), p->args.ex_g, ne * 8, hipMemcpyDeviceToHost));
    MAGOT_HIP_TRY(hipMemcpy(ex_out.data(), p->args.ex_out, (ne + 1) * 8, hipMemcpyDeviceToHost));
  }
  const uint64_t span = p->args.span;
  std::vector<uint64_t> starts(ne + 1);
  for (uint64_t i = 0; i < ne; ++i) {
    const uint64_t gw = ex_g[i], o0 = ex_out[i], len = ex_out[i + 1] - o0;
    const uint64_t gs = gw & ~kExFlagBits;
    rows[2 * i] = (gw & kRcBit) ? 2 * span - gs - len - o0 : gs - o0;
    rows[2 * i + 1] = o0 | ((gw & kExcBit) ? kOrf6ExcRow : 0ull);  // the exact path's flag
    starts[i] = o0;
  }
  rows[2 * ne] = 0;
  rows[2 * ne + 1] = total_nuc;
  starts[ne] = total_nuc;
  // Processing order.  The kernel walks a concatenation of the records; every
  // stream is found through its offset, so the walk may follow the genome
  // instead: records sorted by the plane position of their first interval
  // put neighbouring loci into concurrently running tiles (one XCD sweeps one
  // contiguous range), whose plane reads then share L2 lines.  The records'
  // six-stream blocks are laid out in the same walk order, so each XCD's
  // stores advance through one contiguous stretch of the output (record
  // order would scatter them in ~2 KB runs); magot_orf6_fetch returns every
  // stream's offset.  MAGOT_ORF6_ORDER=record keeps record order (walk and
  // layout).
  std::vector<uint64_t> noff_k, soff_k;
  uint64_t ne_k = ne;
  {
    const char* env = getenv("MAGOT_ORF6_ORDER");
    const bool genome_order = !(env && std::strcmp(env, "record") == 0);
    const uint64_t n = o->n_rec;
    const uint64_t* noff = p->nuc_off.data();
    if (genome_order && ne && n > 1) {
      std::vector<uint64_t> ie(n + 1), key(n), perm(n);
      uint64_t i = 0;
      for (uint64_t r = 0; r < n; ++r) {  // record r's intervals: [ie[r], ie[r+1])
        while (i < ne && starts[i] < noff[r]) ++i;
        ie[r] = i;
      }
      ie[n] = ne;
      for (uint64_t r = 0; r < n; ++r)
        key[r] = noff[r + 1] > noff[r] && ie[r] < ie[r + 1] ? rows[2 * ie[r]] + starts[ie[r]]
                                                             : ~0ull;
      for (uint64_t r = 0; r < n; ++r) perm[r] = r;
      std::stable_sort(perm.begin(), perm.end(),
                       [&](uint64_t x, uint64_t y) { return key[x] < key[y]; });
      noff_k.resize(n + 1);
      soff_k.resize(6 * n + 1);
      std::vector<uint64_t> rows_k(2 * (ne + 1)), starts_k(ne + 1);
      uint64_t j = 0;
      noff_k[0] = 0;
      for (uint64_t k = 0; k < n; ++k) {
        const uint64_t r = perm[k];
        noff_k[k + 1] = noff_k[k] + (noff[r + 1] - noff[r]);
        for (uint64_t e = ie[r]; e < ie[r + 1]; ++e) {
          const uint64_t st = starts[e];
          if (starts[e + 1] == st || st >= noff[r + 1]) continue;  // empty
          // the remap assumes no compacted interval crosses a record end
          // (compaction only drops empty intervals, magot_plan_create)
          if (starts[e + 1] > noff[r + 1]) {
            set_error("magot_plan_orf6: an interval crosses the end of its record");
            return MAGOT_ERR_STATE;
          }
          const uint64_t st_k = noff_k[k] + (st - noff[r]);
          rows_k[2 * j] = rows[2 * e] + st - st_k;  // the same unified anchor
          rows_k[2 * j + 1] = st_k | (rows[2 * e + 1] & kOrf6ExcRow);
          starts_k[j] = st_k;
          ++j;
        }
      }
      // the blocks in walk order; the fetch table maps record r's streams there
      if (int rc = magot_orf6_sizes(noff_k.data(), n, soff_k.data(), nullptr, nullptr)) return rc;
      for (uint64_t k = 0; k < n; ++k)
        for (int s = 0; s < 6; ++s) o->host_soff[6 * perm[k] + s] = soff_k[6 * k + s];
      o->host_soff[6 * n] = soff_k[6 * n];
      rows_k[2 * j] = 0;
      rows_k[2 * j + 1] = total_nuc;
      starts_k[j] = total_nuc;
      rows_k.resize(2 * (j + 1));
      starts_k.resize(j + 1);
      rows.swap(rows_k);
      starts.swap(starts_k);
      ne_k = j;
    } else {
      noff_k.assign(noff, noff + n + 1);
      soff_k = o->host_soff;
    }
  }
  Orf6Tiles tiles;
  orf6_plan_tiles(noff_k.data(), o->n_rec, starts.data(), ne_k, &tiles);
  const uint64_t n_tiles = tiles.r0.size();
  uint8_t lut[64], tables[256];
  if (lut64) std::memcpy(lut, lut64, 64);
  else standard_lut(lut);
  orf6_tables(lut, tables);
  Carve cv;
  const uint64_t o_off = cv.take<uint64_t>(o->n_rec + 1);
  const uint64_t o_boff = cv.take<uint64_t>(o->n_rec + 1);
  const uint64_t o_out = cv.take<uint8_t>(o->total + 64);
  const uint64_t o_rows = cv.take<uint64_t>(2 * (ne_k + 1));
  const uint64_t o_t0 = cv.take<uint64_t>(n_tiles + 1);
  const uint64_t o_r0 = cv.take<uint32_t>(n_tiles);
  const uint64_t o_e0 = cv.take<uint32_t>(n_tiles);
  const uint64_t o_m = cv.take<uint32_t>(n_tiles);
  const uint64_t o_lut = cv.take<uint8_t>(256);
  const uint64_t nib_words = p->args.span / 4;  // forward + reverse planes, 8 bases per word
  const uint64_t code2_words = nib_words / 2;
  const uint64_t o_code2 = cv.take<uint32_t>(code2_words + 4);
  const uint64_t exc1_words = nib_words / 4;
  const uint64_t o_exc1 = cv.take<uint32_t>(exc1_words + 4);
  MAGOT_HIP_TRY(hipMalloc(&o->arena, cv.used));
  char* base = static_cast<char*>(o->arena);
  auto up = [&](uint64_t off, const void* src, uint64_t bytes) {
    return bytes ? hipMemcpy(base + off, src, bytes, hipMemcpyHostToDevice) : hipSuccess;
  };
  uint32_t* code2 = reinterpret_cast<uint32_t*>(base + o_code2);
  uint32_t* exc1 = reinterpret_cast<uint32_t*>(base + o_exc1);
  launch_code2(p->args.nib, nib_words, code2, ctx->stream);
  launch_exc1(p->args.nib, nib_words, exc1, ctx->stream);
  MAGOT_HIP_TRY(hipGetLastError());
  MAGOT_HIP_TRY(hipStreamSynchronize(ctx->stream));
  MAGOT_HIP_TRY(up(o_off, noff_k.data(), (o->n_rec + 1) * 8));
  std::vector<uint64_t> boff_k(o->n_rec + 1);  // block starts in walk order
  for (uint64_t k = 0; k <= o->n_rec; ++k) boff_k[k] = soff_k[6 * k];
  MAGOT_HIP_TRY(up(o_boff, boff_k.data(), (o->n_rec + 1) * 8));
  MAGOT_HIP_TRY(up(o_rows, rows.data(), rows.size() * 8));
  MAGOT_HIP_TRY(up(o_t0, tiles.t0.data(), (n_tiles + 1) * 8));
  MAGOT_HIP_TRY(up(o_r0, tiles.r0.data(), n_tiles * 4));
  MAGOT_HIP_TRY(up(o_e0, tiles.e0.data(), n_tiles * 4));
  MAGOT_HIP_TRY(up(o_m, tiles.m.data(), n_tiles * 4));
  MAGOT_HIP_TRY(up(o_lut, tables, 256));
  o->out = reinterpret_cast<uint8_t*>(base + o_out);
  Orf6Args& a = o->args;
  a.nib = p->args.nib;
  a.nib_words = nib_words;
  a.code2 = code2;
  a.code2_words = code2_words;
  a.exc1 = exc1;
  a.exc1_words = exc1_words;
  a.rows = reinterpret_cast<const uint64_t*>(base + o_rows);
  a.n_rows = ne_k;
  a.noff = reinterpret_cast<const uint64_t*>(base + o_off);
  a.n_rec = o->n_rec;
  a.total = total_nuc;
  a.boff = reinterpret_cast<const uint64_t*>(base + o_boff);
  a.tile_t0 = reinterpret_cast<const uint64_t*>(base + o_t0);
  a.tile_r0 = reinterpret_cast<const uint32_t*>(base + o_r0);
  a.tile_e0 = reinterpret_cast<const uint32_t*>(base + o_e0);
  a.tile_m = reinterpret_cast<const uint32_t*>(base + o_m);
  a.n_tiles = n_tiles;
  a.tables = reinterpret_cast<const uint8_t*>(base + o_lut);
  a.out = o->out;
  if (total_res) *total_res = o->total;
  *out = o.release();
  return MAGOT_OK;
}

int magot_orf6_execute(magot_ctx* ctx, magot_orf6* o) {
  if (int rc = bind(ctx)) return rc;
  if (!o) {
    set_error("magot_orf6_execute: null handle");
    return MAGOT_ERR_ARG;
  }
  o->launch(ctx->stream);
  MAGOT_HIP_TRY(hipGetLastError());
  return MAGOT_OK;
}

int magot_orf6_fetch(magot_ctx* ctx, magot_orf6* o, uint8_t* out, uint64_t* stream_off,
                     uint64_t* stream_len) {
  if (int rc = bind(ctx)) return rc;
  if (!o) {
    set_error("magot_orf6_fetch: null handle");
    return MAGOT_ERR_ARG;
  }
  MAGOT_HIP_TRY(hipStreamSynchronize(ctx->stream));
  if (out && o->total) MAGOT_HIP_TRY(hipMemcpy(out, o->out, o->total, hipMemcpyDeviceToHost));
  if (stream_off)
    std::memcpy(stream_off, o->host_soff.data(), o->host_soff.size() * sizeof(uint64_t));
  if (stream_len) {
    std::vector<uint64_t> tmp(6 * o->n_rec + 1);
    return magot_orf6_sizes(o->plan->nuc_off.data(), o->n_rec, tmp.data(), stream_len, nullptr);
  }
  return MAGOT_OK;
}

int magot_orf6_copy_outputs(magot_ctx* ctx, magot_orf6* o, void* dst_dev) {
  if (int rc = bind(ctx)) return rc;
  if (!o || !dst_dev) {
    set_error("magot_orf6_copy_outputs: null argument");
    return MAGOT_ERR_ARG;
  }
  if (o->total)
    MAGOT_HIP_TRY(hipMemcpyAsync(dst_dev, o->out, o->total, hipMemcpyDeviceToDevice, ctx->stream));
  MAGOT_HIP_TRY(hipStreamSynchronize(ctx->stream));
  return MAGOT_OK;
}

int magot_orf6_time(magot_ctx* ctx, magot_orf6* o, int iters, double* avg_ms) {
  if (int rc = bind(ctx)) return rc;
  if (!o || !avg_ms || iters <= 0) {
    set_error("magot_orf6_time: bad argument");
    return MAGOT_ERR_ARG;
  }
  double total = 0;
  for (int i = 0; i < iters; ++i) {
    MAGOT_HIP_TRY(hipEventRecord(ctx->ev0, ctx->stream));
    o->launch(ctx->stream);
    MAGOT_HIP_TRY(hipEventRecord(ctx->ev1, ctx->stream));
    MAGOT_HIP_TRY(hipEventSynchronize(ctx->ev1));
    float ms = 0;
    MAGOT_HIP_TRY(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
    total += ms;
  }
  *avg_ms = total / iters;
  return MAGOT_OK;
}

int magot_orf6_time_b2b(magot_ctx* ctx, magot_orf6* o, int iters, double* avg_ms) {
  if (int rc = bind(ctx)) return rc;
  if (!o || !avg_ms || iters <= 0) {
    set_error("magot_orf6_time_b2b: bad argument");
    return MAGOT_ERR_ARG;
  }
  MAGOT_HIP_TRY(hipEventRecord(ctx->ev0, ctx->stream));
  for (int i = 0; i < iters; ++i) o->launch(ctx->stream);
  MAGOT_HIP_TRY(hipGetLastError());
  MAGOT_HIP_TRY(hipEventRecord(ctx->ev1, ctx->stream));
  MAGOT_HIP_TRY(hipEventSynchronize(ctx->ev1));
  float ms = 0;
  MAGOT_HIP_TRY(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
  *avg_ms = (double)ms / iters;
  return MAGOT_OK;
}

void magot_orf6_destroy(magot_orf6* o) {
  if (!o) return;
  if (o->ctx) (void)hipSetDevice(o->ctx->device);
  if (o->arena) (void)hipFree(o->arena);
  delete o;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// FASTA text assembly on device (render.hip)
// ---------------------------------------------------------------------------

struct magot_fasta_text {
  magot_ctx* ctx = nullptr;
  const magot_plan* plan = nullptr;
  void* arena = nullptr;
  const TextUnit* units = nullptr;
  const uint64_t* roff = nullptr;
  const uint8_t* text = nullptr;
  uint64_t* len = nullptr;
  uint64_t* psrc = nullptr;  // each unit's payload start in the plan's buffer
  uint64_t* end = nullptr;
  void* scan_tmp = nullptr;
  size_t scan_bytes = 0;
  uint8_t* out = nullptr;
  uint64_t n_units = 0, cap = 0;
  int protein = 0;
  void launch(hipStream_t s) const {
    launch_text_assembly(units, n_units, roff, protein ? plan->args.pep : plan->args.nuc,
                         protein, text, len, psrc, end, scan_tmp, scan_bytes, out, s);
  }
};

extern "C" {

int magot_fasta_text_create(magot_ctx* ctx, const magot_gffplan* gp, const magot_plan* p,
                            magot_fasta_text** out, uint64_t* max_bytes) {
  if (int rc = bind(ctx)) return rc;
  if (!gp || !p || !out) {
    set_error("magot_fasta_text_create: null argument");
    return MAGOT_ERR_ARG;
  }
  *out = nullptr;
  const std::string* text = nullptr;
  std::vector<TextUnit> units;
  bool protein = false;
  uint64_t n_rec = 0;
  if (!gffplan_units(gp, &text, &units, &protein, &n_rec)) {
    set_error("magot_fasta_text_create: too many records, or longest=True protein choices "
              "(magot_gffplan_selections; render those on the host)");
    return MAGOT_ERR_ARG;
  }
  if (n_rec != p->n_tx || !(p->args.outputs & (protein ? MAGOT_OUT_PEP : MAGOT_OUT_NUC))) {
    set_error("magot_fasta_text_create: the plan was not built from this skeleton's tables");
    return MAGOT_ERR_ARG;
  }
  std::unique_ptr<magot_fasta_text> o(new magot_fasta_text());
  o->ctx = ctx;
  o->plan = p;
  o->protein = protein;
  o->n_units = units.size();
  // each record's {start, end} in the plan's device buffer (its layout order)
  const std::vector<uint64_t>& roff = protein ? p->pep_off : p->nuc_off;
  const std::vector<uint64_t>& lay = p->genome_order ? (protein ? p->lay_pep : p->lay_nuc) : roff;
  std::vector<uint64_t> span(2 * n_rec);
  for (uint64_t r = 0; r < n_rec; ++r) {
    span[2 * r] = lay[r];
    span[2 * r + 1] = lay[r] + (roff[r + 1] - roff[r]);
  }
  o->cap = text->size() + (roff.empty() ? 0 : roff.back());
  o->scan_bytes = text_scan_bytes(o->n_units);
  Carve cv;
  const uint64_t o_units = cv.take<TextUnit>(o->n_units);
  const uint64_t o_roff = cv.take<uint64_t>(span.size());
  const uint64_t o_text = cv.take<uint8_t>(text->size());
  const uint64_t o_len = cv.take<uint64_t>(o->n_units);
  const uint64_t o_psrc = cv.take<uint64_t>(o->n_units);
  const uint64_t o_end = cv.take<uint64_t>(o->n_units);
  const uint64_t o_tmp = cv.take<uint8_t>(o->scan_bytes);
  const uint64_t o_out = cv.take<uint8_t>(o->cap);
  MAGOT_HIP_TRY(hipMalloc(&o->arena, cv.used));
  char* base = static_cast<char*>(o->arena);
  o->units = reinterpret_cast<const TextUnit*>(base + o_units);
  o->roff = reinterpret_cast<const uint64_t*>(base + o_roff);
  o->text = reinterpret_cast<const uint8_t*>(base + o_text);
  o->len = reinterpret_cast<uint64_t*>(base + o_len);
  o->psrc = reinterpret_cast<uint64_t*>(base + o_psrc);
  o->end = reinterpret_cast<uint64_t*>(base + o_end);
  o->scan_tmp = base + o_tmp;
  o->out = reinterpret_cast<uint8_t*>(base + o_out);
  if (!units.empty())
    MAGOT_HIP_TRY(hipMemcpy(base + o_units, units.data(), units.size() * sizeof(TextUnit),
                            hipMemcpyHostToDevice));
  if (!span.empty())
    MAGOT_HIP_TRY(hipMemcpy(base + o_roff, span.data(), span.size() * 8, hipMemcpyHostToDevice));
  if (!text->empty())
    MAGOT_HIP_TRY(hipMemcpy(base + o_text, text->data(), text->size(), hipMemcpyHostToDevice));
  if (max_bytes) *max_bytes = o->cap;
  *out = o.release();
  return MAGOT_OK;
}

int magot_fasta_text_execute(magot_ctx* ctx, magot_fasta_text* o) {
  if (int rc = bind(ctx)) return rc;
  if (!o) {
    set_error("magot_fasta_text_execute: null handle");
    return MAGOT_ERR_ARG;
  }
  if (!o->plan->executed) {
    set_error("magot_fasta_text_execute: execute the extraction plan first");
    return MAGOT_ERR_ARG;
  }
  o->launch(ctx->stream);
  MAGOT_HIP_TRY(hipGetLastError());
  return MAGOT_OK;
}

int magot_fasta_text_fetch(magot_ctx* ctx, magot_fasta_text* o, uint8_t* out, uint64_t cap,
                           uint64_t* out_len) {
  if (int rc = bind(ctx)) return rc;
  if (!o || !out_len) {
    set_error("magot_fasta_text_fetch: null argument");
    return MAGOT_ERR_ARG;
  }
  MAGOT_HIP_TRY(hipStreamSynchronize(ctx->stream));
  uint64_t n = 0;
  if (o->n_units)
    MAGOT_HIP_TRY(hipMemcpy(&n, o->end + o->n_units - 1, 8, hipMemcpyDeviceToHost));
  *out_len = n;
  if (!out) return MAGOT_OK;
  if (cap < n) {
    set_error("magot_fasta_text_fetch: output buffer too small");
    return MAGOT_ERR_ARG;
  }
  if (n) MAGOT_HIP_TRY(hipMemcpy(out, o->out, n, hipMemcpyDeviceToHost));
  return MAGOT_OK;
}

int magot_fasta_text_time(magot_ctx* ctx, magot_fasta_text* o, int iters, double* avg_ms) {
  if (int rc = bind(ctx)) return rc;
  if (!o || !avg_ms || iters <= 0) {
    set_error("magot_fasta_text_time: bad argument");
    return MAGOT_ERR_ARG;
  }
  double total = 0;
  for (int i = 0; i < iters; ++i) {
    MAGOT_HIP_TRY(hipEventRecord(ctx->ev0, ctx->stream));
    o->launch(ctx->stream);
    MAGOT_HIP_TRY(hipEventRecord(ctx->ev1, ctx->stream));
    MAGOT_HIP_TRY(hipEventSynchronize(ctx->ev1));
    float ms = 0;
    MAGOT_HIP_TRY(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
    total += ms;
  }
  *avg_ms = total / iters;
  return MAGOT_OK;
}

void magot_fasta_text_destroy(magot_fasta_text* o) {
  if (!o) return;
  if (o->ctx) (void)hipSetDevice(o->ctx->device);
  if (o->arena) (void)hipFree(o->arena);
  delete o;
}

}  // extern "C"
