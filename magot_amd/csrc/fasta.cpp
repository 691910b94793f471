// Native FASTA reader for the batch path: GenomeSequence.__init__
// (genome.py:854-877) straight from the file bytes to the packer, without
// building Python strings or, for the usual fixed-width files, any copy of
// the sequence at all.
//
// Semantics kept: a record starts at every line whose first byte is '>'; its
// name is the rest of the line without '\r' (truncate_names: the first
// whitespace-separated word); its sequence is every following byte except
// '\r' and '\n', up to the next '>' line; empty sequences are not stored;
// a repeated name keeps its first position and takes the last non-empty
// sequence (dict assignment); text before the first '>' is the record "".
// Headers that Python 3's str.split() would split differently from the
// reference's Python 2 byte-string split (bytes >= 0x80, 0x1c-0x1f), and
// empty names under truncate_names (IndexError), return
// MAGOT_ERR_UNSUPPORTED so the caller uses the Python reader.
//
// Layout detection: a record whose CR/LF bytes sit exactly at the ends of
// equal-width lines (width from its first line) is handed to the packer as
// a line layout (ContigSource::width); the proof is a count -- the record's
// non-CR/LF bytes equal what the layout predicts and every predicted
// terminator byte is CR or LF, so no other byte is.  Other records are
// stripped into a buffer.  Both passes run on all host threads.
#include <algorithm>
#include <atomic>
#include <cstring>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "common.h"

namespace magot {
namespace {

inline bool is_crlf(uint8_t c) { return c == '\n' || c == '\r'; }

unsigned host_threads() {
  return std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
}

template <class F>
void parallel_for(size_t n, F&& f) {
  std::atomic<size_t> next{0};
  auto work = [&]() {
    for (size_t i; (i = next.fetch_add(1)) < n;) f(i);
  };
  std::vector<std::thread> pool;
  const unsigned t = (unsigned)std::min<size_t>(host_threads(), n);
  for (unsigned k = 1; k < t; ++k) pool.emplace_back(work);
  work();
  for (auto& th : pool) th.join();
}

struct Rec {
  std::string name;
  uint64_t b, e;             // body byte range [b, e) in the text
  uint64_t width = 0;        // candidate line layout (0: none)
  uint32_t term = 0;
  uint64_t full_lines = 0;   // lines of width + term bytes
  uint64_t expect = 0;       // sequence bytes the layout predicts
  std::atomic<uint64_t> seq{0};       // counted sequence (non-CR/LF) bytes
  std::atomic<bool> layout_ok{true};  // every predicted terminator byte is CR/LF
  Rec(std::string n, uint64_t b_, uint64_t e_) : name(std::move(n)), b(b_), e(e_) {}
};

int header_name(const char* text, uint64_t h, uint64_t eol, bool truncate, std::string* name) {
  std::string head;
  head.reserve(eol - h);
  for (uint64_t i = h + 1; i < eol; ++i)
    if (text[i] != '\r') head.push_back(text[i]);
  if (truncate) {
    for (unsigned char c : head)
      if (c >= 0x80 || (c >= 0x1c && c <= 0x1f)) return MAGOT_ERR_UNSUPPORTED;
    auto ws = [](char c) {
      return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\v' || c == '\f';
    };
    size_t i = 0;
    while (i < head.size() && ws(head[i])) ++i;
    size_t j = i;
    while (j < head.size() && !ws(head[j])) ++j;
    if (i == j) return MAGOT_ERR_UNSUPPORTED;  // IndexError
    head = head.substr(i, j - i);
  }
  *name = std::move(head);
  return MAGOT_OK;
}

// The line layout a record would have, from its first line and its length.
void candidate_layout(const char* text, Rec& r) {
  const uint64_t lb = r.e - r.b;
  const char* nl = static_cast<const char*>(memchr(text + r.b, '\n', lb));
  if (!nl) return;  // one unterminated line: contiguous if it holds no '\r'
  const uint64_t raw = (uint64_t)(nl - text) - r.b;
  const uint32_t t = raw && text[r.b + raw - 1] == '\r' ? 2 : 1;
  const uint64_t w = raw + 1 - t;
  if (!w) return;
  const uint64_t full = lb / (w + t), rem = lb % (w + t);
  uint64_t last = rem;  // sequence bytes of a short last line
  if (rem && is_crlf((uint8_t)text[r.e - 1])) {
    if (rem <= t) return;  // a blank last line
    last = rem - t;
    for (uint32_t j = 0; j < t; ++j)
      if (!is_crlf((uint8_t)text[r.e - t + j])) return;
  }
  r.width = w;
  r.term = t;
  r.full_lines = full;
  r.expect = full * w + last;
}

}  // namespace

int scan_fasta(const char* text, uint64_t n, bool truncate, FastaContigs* out) {
  // records: a '>' at a line start opens one
  std::vector<std::unique_ptr<Rec>> recs;
  std::string name;
  bool have = false;
  uint64_t body = 0, p = 0;
  for (;;) {
    uint64_t h = n;
    for (uint64_t q = p; q < n;) {
      const char* f = static_cast<const char*>(memchr(text + q, '>', n - q));
      if (!f) break;
      const uint64_t at = (uint64_t)(f - text);
      if (at == 0 || text[at - 1] == '\n') {
        h = at;
        break;
      }
      q = at + 1;
    }
    if (have || h > body) recs.emplace_back(new Rec(name, body, h));
    if (h == n) break;
    const char* nl = static_cast<const char*>(memchr(text + h, '\n', n - h));
    const uint64_t eol = nl ? (uint64_t)(nl - text) : n;
    if (int rc = header_name(text, h, eol, truncate, &name)) return rc;
    have = true;
    body = p = std::min(eol + 1, n);
  }
  for (auto& r : recs) candidate_layout(text, *r);

  // count sequence bytes and check predicted terminators, in chunks
  constexpr uint64_t kChunk = 8ull << 20;
  struct Task {
    Rec* r;
    uint64_t x, y;
  };
  std::vector<Task> tasks;
  for (auto& r : recs)
    for (uint64_t x = r->b; x < r->e; x += kChunk)
      tasks.push_back({r.get(), x, std::min(r->e, x + kChunk)});
  parallel_for(tasks.size(), [&](size_t i) {
    const Task& T = tasks[i];
    Rec& r = *T.r;
    const uint8_t* s = reinterpret_cast<const uint8_t*>(text);
    uint64_t crlf = 0;
    for (uint64_t k = T.x; k < T.y; ++k) crlf += is_crlf(s[k]);
    r.seq += (T.y - T.x) - crlf;
    if (!r.width) return;
    const uint64_t stride = r.width + r.term;
    // terminators of full lines that start in [x, y)
    uint64_t line = T.x > r.b ? (T.x - r.b + stride - 1) / stride : 0;
    bool ok = true;
    for (uint64_t at = r.b + line * stride; at < T.y && line < r.full_lines;
         ++line, at += stride)
      for (uint32_t j = 0; j < r.term; ++j) ok &= is_crlf(s[at + r.width + j]);
    if (!ok) r.layout_ok = false;
  });

  // dict semantics: first position, last non-empty value
  std::unordered_map<std::string, size_t> at;
  std::vector<Rec*> chosen;
  for (auto& r : recs) {
    if (!r->seq.load()) continue;
    auto it = at.find(r->name);
    if (it == at.end()) {
      at.emplace(r->name, chosen.size());
      out->names.push_back(r->name);
      chosen.push_back(r.get());
    } else {
      chosen[it->second] = r.get();
    }
  }
  const uint8_t* s = reinterpret_cast<const uint8_t*>(text);
  out->src.resize(chosen.size());
  std::vector<size_t> strip;
  for (size_t i = 0; i < chosen.size(); ++i) {
    Rec& r = *chosen[i];
    const uint64_t len = r.seq.load();
    if (len == r.e - r.b) {
      out->src[i] = ContigSource{s + r.b, len, 0, 0};
    } else if (r.width && r.layout_ok.load() && len == r.expect) {
      out->src[i] = ContigSource{s + r.b, len, r.width, r.term};
    } else {
      out->src[i] = ContigSource{nullptr, len, 0, 0};
      strip.push_back(i);
    }
  }
  out->storage.assign(strip.size(), std::string());
  parallel_for(strip.size(), [&](size_t k) {
    const size_t i = strip[k];
    const Rec& r = *chosen[i];
    std::string& dst = out->storage[k];
    dst.resize(out->src[i].len);
    size_t o = 0;
    for (uint64_t j = r.b; j < r.e; ++j)
      if (!is_crlf(s[j])) dst[o++] = (char)s[j];
  });
  for (size_t k = 0; k < strip.size(); ++k)
    out->src[strip[k]].ptr = reinterpret_cast<const uint8_t*>(out->storage[k].data());
  return MAGOT_OK;
}

void copy_bases(const ContigSource& src, uint64_t pos, uint64_t n, uint8_t* dst) {
  if (!n) return;
  if (!src.width) {
    memcpy(dst, src.ptr + pos, n);
    return;
  }
  uint64_t line = pos / src.width, off = pos - line * src.width;
  const uint8_t* p = src.ptr + line * (src.width + src.term) + off;
  while (n) {
    const uint64_t k = std::min(n, src.width - off);
    memcpy(dst, p, k);
    dst += k;
    n -= k;
    p += k + src.term;
    off = 0;
  }
}

void copy_contig(const ContigSource& src, uint8_t* dst) {
  if (!src.width) {
    if (src.len) memcpy(dst, src.ptr, src.len);
    return;
  }
  const uint8_t* p = src.ptr;
  for (uint64_t left = src.len; left;) {
    const uint64_t k = std::min(left, src.width);
    memcpy(dst, p, k);
    dst += k;
    p += src.width + src.term;
    left -= k;
  }
}

}  // namespace magot

extern "C" int magot_fasta_read(const char* text, uint64_t len, int truncate_names, uint32_t* n,
                                uint64_t* lens, char* names, uint64_t names_cap,
                                uint64_t* names_len, uint8_t* seqs, uint64_t seqs_cap) {
  if (!n || (len && !text)) {
    magot::set_error("magot_fasta_read: null argument");
    return MAGOT_ERR_ARG;
  }
  magot::FastaContigs fc;
  if (int rc = magot::scan_fasta(text, len, truncate_names != 0, &fc)) {
    magot::set_error("magot_fasta_read: header needs the Python reader");
    return rc;
  }
  const size_t k = fc.names.size();
  *n = (uint32_t)k;
  uint64_t need_names = 0, need_seqs = 0;
  std::vector<uint64_t> at(k);
  for (size_t i = 0; i < k; ++i) {
    need_names += fc.names[i].size() + 1;
    at[i] = need_seqs;
    need_seqs += fc.src[i].len;
    if (lens) lens[i] = fc.src[i].len;
  }
  if (names_len) *names_len = need_names;
  if ((names && names_cap < need_names) || (seqs && seqs_cap < need_seqs)) {
    magot::set_error("magot_fasta_read: buffer too small");
    return MAGOT_ERR_ARG;
  }
  if (names)
    for (size_t i = 0; i < k; ++i) {
      memcpy(names, fc.names[i].data(), fc.names[i].size());
      names += fc.names[i].size();
      *names++ = '\0';
    }
  if (seqs) magot::parallel_for(k, [&](size_t i) { magot::copy_contig(fc.src[i], seqs + at[i]); });
  return MAGOT_OK;
}

// ---------------------------------------------------------------------------
// cds2pep (genome_tools.py:664-675): the file's lines with '\n' and '\r'
// removed; a line starting with '>' is echoed and ends the sequence gathered
// so far (translated if non-empty), every other line is appended to it, and
// the last sequence is translated whatever its length.
// ---------------------------------------------------------------------------

extern "C" int magot_cds_scan(const char* text, uint64_t len, uint64_t* n_seg,
                              uint64_t* seq_bytes, uint64_t* seg_off, uint64_t* hdr_off,
                              uint64_t* hdr_len, uint8_t* seq, uint64_t seq_cap) {
  if (!n_seg || !seq_bytes || (len && !text)) {
    magot::set_error("magot_cds_scan: null argument");
    return MAGOT_ERR_ARG;
  }
  uint64_t k = 0, m = 0;  // headers seen, sequence bytes
  if (seg_off) seg_off[0] = 0;
  for (uint64_t pos = 0; pos < len;) {
    const char* nl = static_cast<const char*>(memchr(text + pos, '\n', len - pos));
    const uint64_t end = nl ? (uint64_t)(nl - text) : len;
    uint64_t e = end;
    if (e > pos && text[e - 1] == '\r') --e;  // CRLF
    if (e == pos) {  // empty after the strip: line[0] raises IndexError
      magot::set_error("magot_cds_scan: empty line (the line loop reproduces the IndexError)");
      return MAGOT_ERR_UNSUPPORTED;
    }
    if (memchr(text + pos, '\r', e - pos)) {  // a CR inside the line: the line loop strips it
      magot::set_error("magot_cds_scan: carriage return inside a line");
      return MAGOT_ERR_UNSUPPORTED;
    }
    if (text[pos] == '>') {
      if (hdr_off) {
        hdr_off[k] = pos;
        hdr_len[k] = e - pos;
      }
      ++k;
      if (seg_off) seg_off[k] = m;
    } else {
      if (seq) {
        if (m + (e - pos) > seq_cap) {
          magot::set_error("magot_cds_scan: buffer too small");
          return MAGOT_ERR_ARG;
        }
        memcpy(seq + m, text + pos, e - pos);
      }
      m += e - pos;
    }
    pos = nl ? end + 1 : len;
  }
  *n_seg = k + 1;
  *seq_bytes = m;
  if (seg_off) seg_off[k + 1] = m;
  return MAGOT_OK;
}

extern "C" int magot_cds_render(const char* text, uint64_t n_seg, const uint64_t* seg_off,
                                const uint64_t* hdr_off, const uint64_t* hdr_len,
                                const uint8_t* pep, const uint64_t* poff, const int64_t* codons,
                                uint8_t* out, uint64_t cap, uint64_t* out_len) {
  if (!out_len || !n_seg || !seg_off || !poff || !codons || (n_seg > 1 && (!text || !hdr_off || !hdr_len))) {
    magot::set_error("magot_cds_render: null argument");
    return MAGOT_ERR_ARG;
  }
  uint64_t n = 0;
  auto put = [&](const void* s, uint64_t l) {
    if (out && n + l <= cap) memcpy(out + n, s, l);
    n += l;
  };
  for (uint64_t k = 0; k < n_seg; ++k) {
    if (k == n_seg - 1 || seg_off[k + 1] > seg_off[k]) {
      if (codons[k] < 0) {
        put("None", 4);  // translate() returned None (genome.py:810)
      } else {
        uint64_t a = poff[k];
        const uint64_t b = poff[k + 1];
        if (b > a && pep[a] == 'X') ++a;  // trimX (genome.py:819-821)
        put(pep + a, b - a);
      }
      put("\n", 1);
    }
    if (k + 1 < n_seg) {
      put(text + hdr_off[k], hdr_len[k]);
      put("\n", 1);
    }
  }
  *out_len = n;
  if (out && n > cap) {
    magot::set_error("magot_cds_render: buffer too small");
    return MAGOT_ERR_ARG;
  }
  return MAGOT_OK;
}
