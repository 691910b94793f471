// Host-side genome packer: raw contig bytes -> nibble plane (2-bit code,
// soft-mask bit, exception bit per base), exception runs and their block
// directory (layout: common.h).
//
// The bytes packed are exactly what GenomeSequence keeps (genome.py:870-877):
// every byte of every sequence line except CR/LF, case preserved.  ACGTacgt
// become codes; every other byte value is kept verbatim in a run list, so the
// device path can reproduce any input byte exactly.
#include <algorithm>
#include <atomic>
#include <thread>

#include "common.h"

namespace magot {
namespace {

struct ByteClass {
  uint8_t nib[256];    // nibble for ACGTacgt, 8 | lit_class (exception) otherwise
  uint8_t plain[256];  // 1 for ACGTacgt
  ByteClass() {
    for (int i = 0; i < 256; ++i) {
      nib[i] = (uint8_t)(8u | lit_class((uint32_t)i));
      plain[i] = 0;
    }
    const char up[4] = {'A', 'C', 'G', 'T'};
    for (int c = 0; c < 4; ++c) {
      nib[(uint8_t)up[c]] = (uint8_t)c;
      plain[(uint8_t)up[c]] = 1;
      nib[(uint8_t)(up[c] | 0x20)] = (uint8_t)(c | 4);
      plain[(uint8_t)(up[c] | 0x20)] = 1;
    }
  }
};

const ByteClass& byte_class() {
  static const ByteClass k;
  return k;
}

// Pack global coordinates [p0, p1) (p0, p1 multiples of 32, so no plane word
// is shared with another piece): every word of the piece is written once,
// bases accumulated in a register.
void pack_piece(const ContigSource* src, const HostPacked& layout, uint64_t p0, uint64_t p1,
                uint32_t* nib, std::vector<ExcRun>* runs) {
  const ByteClass& bc = byte_class();
  const auto& base = layout.contig_base;
  const auto& len = layout.contig_len;
  const size_t n = base.size();
  // first contig whose end > p0
  size_t c = std::upper_bound(base.begin(), base.end(), p0) - base.begin();
  c = c == 0 ? 0 : c - 1;
  ExcRun cur{0, 0, 0};
  bool open = false;
  uint64_t aw = p0 >> 3;  // word being accumulated
  uint32_t acc = 0;
  for (; c < n; ++c) {
    const uint64_t cb = base[c], ce = base[c] + len[c];
    if (cb >= p1) break;
    uint64_t lo = std::max(cb, p0);
    const uint64_t hi = std::min(ce, p1);
    if (lo >= hi) continue;
    const ContigSource& S = src[c];
    uint64_t pos = lo - cb;
    while (lo < hi) {
      const uint8_t* s;
      uint64_t seg;
      if (!S.width) {
        s = S.ptr + pos;
        seg = hi - lo;
      } else {  // FASTA line layout: the rest of the current line
        const uint64_t line = pos / S.width, off = pos - line * S.width;
        s = S.ptr + line * (S.width + S.term) + off;
        seg = std::min(S.width - off, hi - lo);
      }
      pos += seg;
      const uint8_t* e = s + seg;
      for (;;) {
        // whole words of plain bases: 8 lookups, one store
        while ((lo & 7) == 0 && e - s >= 8) {
          uint32_t w = 0;
          for (int k = 0; k < 8; ++k) w |= (uint32_t)bc.nib[s[k]] << (4 * k);
          if (w & 0x88888888u) break;  // an exception byte: per-base path
          if (open) {
            runs->push_back(cur);
            open = false;
          }
          if ((lo >> 3) != aw) nib[aw] = acc;
          aw = lo >> 3;
          acc = w;
          s += 8;
          lo += 8;
        }
        if (s == e) break;
        const uint8_t b = *s;
        if ((lo >> 3) != aw) {
          nib[aw] = acc;
          acc = 0;
          aw = lo >> 3;
        }
        acc |= (uint32_t)bc.nib[b] << (4 * (lo & 7));
        if (bc.plain[b]) {
          if (open) {
            runs->push_back(cur);
            open = false;
          }
        } else {
          if (open && cur.byte == b && cur.start + cur.len == lo && cur.len < 0x7fffffffu) {
            ++cur.len;
          } else {
            if (open) runs->push_back(cur);
            cur = ExcRun{lo, 1, b};
            open = true;
          }
        }
        ++s;
        ++lo;
      }
    }
  }
  if (open) runs->push_back(cur);
  // the last accumulated word, then the zero words up to p1 (padding)
  nib[aw] = acc;
  for (uint64_t w = aw + 1; w < (p1 >> 3); ++w) nib[w] = 0;
}

}  // namespace

void pack_layout(const ContigSource* src, uint32_t n, HostPacked* out) {
  out->contig_base.resize(n);
  out->contig_len.resize(n);
  uint64_t cur = kOrigin;
  for (uint32_t i = 0; i < n; ++i) {
    out->contig_base[i] = cur;
    out->contig_len[i] = src[i].len;
    cur += src[i].len;
  }
  out->extent = cur;
  const uint64_t padded = cur + 64;
  out->span = (padded + 64 + 31) & ~31ull;
  out->nib_words = out->span / 8;
}

void exc_runs_directory(HostPacked* out) {
  // Directory: first run whose end lies past the block start.
  const uint64_t padded = out->extent + 64;
  const uint64_t nblocks = ((padded + 4095) >> kDirShift) + 2;
  out->dir.assign(nblocks, 0);
  size_t r = 0, nr = out->runs.size() - 1;
  for (uint64_t b = 0; b < nblocks; ++b) {
    uint64_t bs = b << kDirShift, be = bs + (1ull << kDirShift);
    while (r < nr && out->runs[r].start + out->runs[r].len <= bs) ++r;
    uint32_t v = (uint32_t)r;
    if (out->runs[r].start >= be) v |= kDirClean;
    out->dir[b] = v;
  }
}

void pack_genome(const ContigSource* src, uint32_t n, HostPacked* out) {
  pack_layout(src, n, out);
  out->nib.reset(new uint32_t[out->nib_words]);  // written in full by the pieces, except
  // the words of the kOrigin pad bases, which no piece reaches (the first
  // contig starts at kOrigin): zero them here (the device packer's arena
  // matched everywhere but these seven words, tests/test_gpu_replication.py)
  for (uint64_t w = 0; w < std::min<uint64_t>(kOrigin / 8, out->nib_words); ++w) out->nib[w] = 0;

  // Split [0, span) into 32-aligned pieces for the worker threads.
  unsigned hw = std::max(1u, std::min(32u, std::thread::hardware_concurrency()));
  const uint64_t min_piece = 1ull << 22;
  const uint64_t span = out->span;
  uint64_t npieces = std::max<uint64_t>(1, std::min<uint64_t>(hw * 4, span / min_piece + 1));
  uint64_t step = ((span + npieces - 1) / npieces + 31) & ~31ull;
  std::vector<std::vector<ExcRun>> piece_runs(npieces);
  std::vector<std::thread> pool;
  std::atomic<uint64_t> next{0};
  auto worker = [&]() {
    for (;;) {
      uint64_t k = next.fetch_add(1);
      if (k >= npieces) return;
      uint64_t p0 = k * step, p1 = std::min(span, p0 + step);
      if (p0 < p1) pack_piece(src, *out, p0, p1, out->nib.get(), &piece_runs[k]);
    }
  };
  unsigned nthreads = (unsigned)std::min<uint64_t>(hw, npieces);
  for (unsigned t = 1; t < nthreads; ++t) pool.emplace_back(worker);
  worker();
  for (auto& t : pool) t.join();

  // Concatenate, merging runs split at piece boundaries.
  out->runs.clear();
  for (auto& pr : piece_runs) {
    for (const ExcRun& r : pr) {
      if (!out->runs.empty()) {
        ExcRun& last = out->runs.back();
        if (last.byte == r.byte && last.start + last.len == r.start &&
            (uint64_t)last.len + r.len < 0x7fffffffull) {
          last.len += r.len;
          continue;
        }
      }
      out->runs.push_back(r);
    }
  }
  out->runs.push_back(ExcRun{~0ull, 0, 0});  // sentinel
  exc_runs_directory(out);
}

// --- planner helper (host) ---------------------------------------------------

// Record indices in ascending key order, ties in index order: an LSD radix
// sort in 11-bit digits, as many passes as the largest key needs.
void radix_order(const std::vector<uint64_t>& key, std::vector<uint32_t>* out) {
  const uint64_t n = key.size();
  uint64_t top = 0;
  for (uint64_t k : key) top = std::max(top, k);
  std::vector<uint32_t> a(n), b(n);
  for (uint64_t i = 0; i < n; ++i) a[i] = (uint32_t)i;
  for (int shift = 0; shift < 64 && (top >> shift); shift += 11) {
    std::vector<uint64_t> cnt(2049, 0);
    for (uint64_t i = 0; i < n; ++i) ++cnt[((key[a[i]] >> shift) & 2047) + 1];
    for (int d = 0; d < 2048; ++d) cnt[d + 1] += cnt[d];
    for (uint64_t i = 0; i < n; ++i) b[cnt[(key[a[i]] >> shift) & 2047]++] = a[i];
    a.swap(b);
  }
  out->swap(a);
}

}  // namespace magot
