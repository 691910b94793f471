// Native FASTA reader for the batch path: GenomeSequence.__init__
// (genome.py:854-877) straight from the file bytes into contig buffers that
// magot_genome_load packs, without building Python strings.
//
// Semantics kept: a record starts at every line whose first byte is '>'; its
// name is the rest of the line without '\r' (truncate_names: the first
// whitespace-separated word); its sequence is every following line with '\r'
// and '\n' removed, up to the next '>' line; empty sequences are not stored;
// a repeated name keeps its first position and takes the last non-empty
// sequence (dict assignment); text before the first '>' is the record "".
// Headers that Python 3's str.split() would split differently from the
// reference's Python 2 byte-string split (bytes >= 0x80, 0x1c-0x1f), and
// empty names under truncate_names (IndexError), return
// MAGOT_ERR_UNSUPPORTED so the caller uses the Python reader.
#include <algorithm>
#include <atomic>
#include <cstring>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "common.h"

namespace magot {

int parse_fasta(const char* text, uint64_t n, bool truncate, std::vector<std::string>* names,
                std::vector<std::string>* seqs) {
  struct Rec {
    std::string name;
    uint64_t b, e;  // body byte range [b, e) in text (lines, with newlines)
  };
  std::vector<Rec> recs;
  uint64_t pos = 0;
  std::string name;
  bool have = false;
  uint64_t body = 0;
  auto close_rec = [&](uint64_t end) {
    if (have || end > body) recs.push_back(Rec{name, body, end});
  };
  while (pos < n) {
    if (text[pos] == '>') {
      close_rec(pos);
      const char* nl = static_cast<const char*>(memchr(text + pos, '\n', n - pos));
      const uint64_t eol = nl ? (uint64_t)(nl - text) : n;
      std::string head;
      head.reserve(eol - pos);
      for (uint64_t i = pos + 1; i < eol; ++i)
        if (text[i] != '\r') head.push_back(text[i]);
      if (truncate) {
        for (unsigned char c : head)
          if (c >= 0x80 || (c >= 0x1c && c <= 0x1f)) return MAGOT_ERR_UNSUPPORTED;
        size_t i = 0;
        auto ws = [](char c) {
          return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\v' || c == '\f';
        };
        while (i < head.size() && ws(head[i])) ++i;
        size_t j = i;
        while (j < head.size() && !ws(head[j])) ++j;
        if (i == j) return MAGOT_ERR_UNSUPPORTED;  // IndexError
        head = head.substr(i, j - i);
      }
      name = head;
      have = true;
      pos = eol + 1;
      body = std::min(pos, n);
      continue;
    }
    // skip to the next line that starts with '>'
    const char* p = text + pos;
    const char* end = text + n;
    for (;;) {
      const char* nl = static_cast<const char*>(memchr(p, '\n', end - p));
      if (!nl) {
        pos = n;
        break;
      }
      p = nl + 1;
      if (p < end && *p == '>') {
        pos = (uint64_t)(p - text);
        break;
      }
      if (p >= end) {
        pos = n;
        break;
      }
    }
  }
  close_rec(n);
  // sequences: line bodies without '\r' / '\n' (records in parallel)
  std::vector<std::string> body_seq(recs.size());
  auto work = [&](size_t k) {
    const Rec& r = recs[k];
    std::string& s = body_seq[k];
    s.resize(r.e - r.b);
    size_t o = 0;
    for (uint64_t i = r.b; i < r.e; ++i) {
      const char c = text[i];
      if (c != '\n' && c != '\r') s[o++] = c;
    }
    s.resize(o);
  };
  {
    std::vector<std::thread> pool;
    const unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::vector<size_t> order(recs.size());
    for (size_t i = 0; i < order.size(); ++i) order[i] = i;
    std::sort(order.begin(), order.end(),
              [&](size_t a, size_t b) { return recs[a].e - recs[a].b > recs[b].e - recs[b].b; });
    std::atomic<size_t> next{0};
    for (unsigned t = 0; t < hw; ++t)
      pool.emplace_back([&]() {
        for (size_t i; (i = next.fetch_add(1)) < order.size();) work(order[i]);
      });
    for (auto& t : pool) t.join();
  }
  // dict semantics: first position, last non-empty value
  std::unordered_map<std::string, size_t> at;
  names->clear();
  seqs->clear();
  for (size_t k = 0; k < recs.size(); ++k) {
    if (body_seq[k].empty()) continue;
    auto it = at.find(recs[k].name);
    if (it == at.end()) {
      at.emplace(recs[k].name, names->size());
      names->push_back(recs[k].name);
      seqs->push_back(std::move(body_seq[k]));
    } else {
      (*seqs)[it->second] = std::move(body_seq[k]);
    }
  }
  return MAGOT_OK;
}

}  // namespace magot

extern "C" int magot_fasta_read(const char* text, uint64_t len, int truncate_names, uint32_t* n,
                                uint64_t* lens, char* names, uint64_t names_cap,
                                uint64_t* names_len, uint8_t* seqs, uint64_t seqs_cap) {
  if (!n || (len && !text)) {
    magot::set_error("magot_fasta_read: null argument");
    return MAGOT_ERR_ARG;
  }
  std::vector<std::string> nm, sq;
  if (int rc = magot::parse_fasta(text, len, truncate_names != 0, &nm, &sq)) {
    magot::set_error("magot_fasta_read: header needs the Python reader");
    return rc;
  }
  *n = (uint32_t)nm.size();
  uint64_t need_names = 0, need_seqs = 0;
  for (size_t i = 0; i < nm.size(); ++i) {
    need_names += nm[i].size() + 1;
    need_seqs += sq[i].size();
    if (lens) lens[i] = sq[i].size();
  }
  if (names_len) *names_len = need_names;
  if ((names && names_cap < need_names) || (seqs && seqs_cap < need_seqs)) {
    magot::set_error("magot_fasta_read: buffer too small");
    return MAGOT_ERR_ARG;
  }
  for (size_t i = 0; i < nm.size(); ++i) {
    if (names) {
      memcpy(names, nm[i].data(), nm[i].size());
      names += nm[i].size();
      *names++ = '\0';
    }
    if (seqs) {
      memcpy(seqs, sq[i].data(), sq[i].size());
      seqs += sq[i].size();
    }
  }
  return MAGOT_OK;
}
