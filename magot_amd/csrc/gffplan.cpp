// Native batch planner for the gff2fasta hot path (genome_tools.py:324-330).
//
// Parses GFF3/GTF text with the reference's read_gff rules (genome.py:242-415),
// keeps its annotation model (per-type tables, global ID lookup where the
// lexicographically last type wins, genome.py:536-544), orders the records of
// one feature table (insertion order, or CPython 2.7 dict order after the
// deepcopy of genome.py:415), and lowers AnnotationSet.get_fasta
// (genome.py:578-582, ParentAnnotation.get_fasta genome.py:677-731) to the
// interval / record tables the extraction kernel consumes plus a text
// skeleton (headers and joiners) that render() fills with the kernel output.
//
// Anything that would take one of the reference's diagnostic paths (stdout
// prints followed by None / TypeError / AttributeError ...)
// returns MAGOT_ERR_UNSUPPORTED so the caller can run the object path, which
// reproduces those diagnostics exactly.  This file never touches sequence
// bytes: the extraction itself is the HIP kernel's.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <memory>
#include <mutex>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

#include <sys/mman.h>

#include "common.h"

namespace magot {
namespace {

struct Feature {
  uint32_t type = 0;
  uint32_t seqid = 0;   // index into Model::seqids
  int64_t lo = 0, hi = 0;
  uint32_t strand = 0;  // index into Model::strands
  bool base = false;
  uint32_t kids = ~0u;  // its child list (Model::kid_head), ~0u: none yet
};

struct Table {
  std::string name;
  std::vector<uint32_t> keys;  // IDs in insertion order
};

struct Unsupported {};  // a diagnostic path of the reference: use the object path

// The first exception a worker thread caught, rethrown by the caller.
struct FirstError {
  std::mutex mu;
  std::exception_ptr err;
  void set() {
    std::lock_guard<std::mutex> g(mu);
    if (!err) err = std::current_exception();
  }
  void rethrow() {
    if (err) std::rethrow_exception(err);
  }
};

using sv = std::string_view;

// Interned strings with stable storage (views stay valid as the pool grows),
// found through a flat open-addressing table (linear probing, load <= 1/2).
inline uint64_t hash_sv(sv s) {
  uint64_t h = 0x9E3779B97F4A7C15ull ^ s.size();
  size_t i = 0;
  for (; i + 8 <= s.size(); i += 8) {
    uint64_t w;
    memcpy(&w, s.data() + i, 8);
    h = (h ^ w) * 0xFF51AFD7ED558CCDull;
    h ^= h >> 32;
  }
  uint64_t w = 0;
  memcpy(&w, s.data() + i, s.size() - i);
  h = (h ^ w) * 0xC4CEB9FE1A85EC53ull;
  return h ^ (h >> 29);
}

// Zero-filled words from calloc: a large table comes straight from the
// kernel's zero pages instead of being written once by a fill and again by use.
struct ZeroWords {
  uint64_t* p = nullptr;
  size_t n = 0;
  explicit ZeroWords(size_t count) : p(static_cast<uint64_t*>(calloc(count, 8))), n(count) {
    if (!p) throw std::bad_alloc();
  }
  ZeroWords(const ZeroWords&) = delete;
  ZeroWords& operator=(const ZeroWords&) = delete;
  ~ZeroWords() { free(p); }
  size_t size() const { return n; }
  uint64_t& operator[](size_t i) { return p[i]; }
  const uint64_t& operator[](size_t i) const { return p[i]; }
  void swap(ZeroWords& o) {
    std::swap(p, o.p);
    std::swap(n, o.n);
  }
};

struct Pool {
  std::vector<std::unique_ptr<char[]>> chunks;
  size_t left = 0;
  char* cur = nullptr;
  std::vector<sv> strs;
  // slot word: (hash bits for quick rejects) << 32 | (id + 1); 0 = empty
  ZeroWords slots{64};

  void reserve(size_t n) {
    strs.reserve(n);
    size_t cap = 64;
    while (cap < 2 * n) cap <<= 1;
    if (cap > slots.size()) rehash(cap);
  }
  sv store(sv s) {
    if (s.size() > left) {
      const size_t n = std::max<size_t>(s.size(), 1 << 20);
      chunks.emplace_back(new char[n]);
      cur = chunks.back().get();
      left = n;
    }
    if (!s.empty()) memcpy(cur, s.data(), s.size());
    sv out(cur, s.size());
    cur += s.size();
    left -= s.size();
    return out;
  }
  static uint64_t word(uint64_t h, uint32_t id) { return (h >> 32 << 32) | (id + 1ull); }
  void rehash(size_t cap) {
    ZeroWords ns(cap);
    const size_t mask = cap - 1;
    for (uint32_t id = 0; id < strs.size(); ++id) {
      const uint64_t h = hash_sv(strs[id]);
      size_t i = h & mask;
      while (ns[i]) i = (i + 1) & mask;
      ns[i] = word(h, id);
    }
    slots.swap(ns);
  }
  // slot of s (occupied when found, else the empty slot where it goes)
  size_t probe(sv s, uint64_t h) const {
    const size_t mask = slots.size() - 1;
    size_t i = h & mask;
    const uint64_t tg = h >> 32;
    for (;;) {
      const uint64_t v = slots[i];
      if (!v || ((v >> 32) == tg && strs[(uint32_t)v - 1] == s)) return i;
      i = (i + 1) & mask;
    }
  }
  int64_t find(sv s) const { return find(s, hash_sv(s)); }
  int64_t find(sv s, uint64_t h) const {
    const uint64_t v = slots[probe(s, h)];
    return v ? (int64_t)(uint32_t)v - 1 : -1;
  }
  void prefetch(uint64_t h) const { __builtin_prefetch(&slots[h & (slots.size() - 1)]); }
  uint32_t intern(sv s) { return intern(s, hash_sv(s)); }
  uint32_t intern(sv s, uint64_t h) {
    size_t i = probe(s, h);
    if (slots[i]) return (uint32_t)slots[i] - 1;
    const uint32_t id = (uint32_t)strs.size();
    strs.push_back(store(s));
    if (2 * strs.size() > slots.size()) {
      rehash(slots.size() * 2);
      return id;
    }
    slots[i] = word(h, id);
    return id;
  }
};

struct Model {
  Pool ids, seqids, strands;
  std::vector<uint64_t> id_types;  // bitmask of tables holding the ID (<= 64 tables)
  // feature stored under (table, ID): the ID's first table in `first_feat`,
  // further tables (rare: the same ID under two types) in `more_feat`
  std::vector<uint8_t> first_table;
  std::vector<uint32_t> first_feat;
  std::unordered_map<uint64_t, uint32_t> more_feat;
  std::vector<Table> tables;
  std::unordered_map<std::string, uint32_t> table_index;
  std::vector<uint32_t> rank;      // table -> rank in sorted-name order
  std::vector<Feature> feats;
  // Child IDs (ids) per parent feature, as chains through one pair of link
  // arrays in append order (no allocation per list: C3 has a million
  // parents); children() walks a chain.
  std::vector<uint32_t> kid_head, kid_tail;     // per list
  std::vector<uint32_t> link_child, link_next;  // per appended child

  Model() {
    // AnnotationSet.__init__ (genome.py:528-533) creates these dicts
    for (const char* t : {"gene", "transcript", "CDS", "UTR"}) table(t);
  }

  struct Kids {
    const Model* m;
    uint32_t head;  // first link, ~0u: no children
    struct It {
      const Model* m;
      uint32_t k;
      uint32_t operator*() const { return m->link_child[k]; }
      It& operator++() {
        k = m->link_next[k];
        return *this;
      }
      bool operator!=(const It& o) const { return k != o.k; }
    };
    It begin() const { return It{m, head}; }
    It end() const { return It{m, ~0u}; }
    bool empty() const { return head == ~0u; }
    uint32_t front() const { return m->link_child[head]; }
  };
  Kids children(const Feature& f) const {
    return Kids{this, f.kids == ~0u ? ~0u : kid_head[f.kids]};
  }
  bool has_child(const Feature& f, uint32_t child) const {
    for (uint32_t c : children(f))
      if (c == child) return true;
    return false;
  }
  void add_child(Feature& f, uint32_t child) {
    const uint32_t k = (uint32_t)link_child.size();
    link_child.push_back(child);
    link_next.push_back(~0u);
    if (f.kids == ~0u) {
      f.kids = (uint32_t)kid_head.size();
      kid_head.push_back(k);
      kid_tail.push_back(k);
      return;
    }
    link_next[kid_tail[f.kids]] = k;
    kid_tail[f.kids] = k;
  }

  uint32_t id(sv s) { return id(s, hash_sv(s)); }
  uint32_t id(sv s, uint64_t h) {
    const uint32_t k = ids.intern(s, h);
    while (id_types.size() < ids.strs.size()) {
      id_types.push_back(0);
      first_table.push_back(0);
      first_feat.push_back(0);
    }
    return k;
  }
  // feature of ID idk in table t (-1 when absent)
  int64_t slot(uint32_t t, uint32_t idk) const {
    if (!((id_types[idk] >> t) & 1)) return -1;
    if (first_table[idk] == t) return first_feat[idk];
    return more_feat.at(((uint64_t)idk << 6) | t);
  }
  uint32_t table(sv name_sv) {
    for (const Table& t : tables)  // few tables: a linear scan beats hashing
      if (sv(t.name) == name_sv) return (uint32_t)(&t - tables.data());
    return table_slow(name_sv);
  }
  uint32_t table_slow(sv name_sv) {
    const std::string name(name_sv);
    auto it = table_index.find(name);
    if (it != table_index.end()) return it->second;
    // attributes of the instance that are not dicts (genome.py:524-545, plus
    // the object path's copy counter) cannot become feature tables
    if (name == "genome" || name == "_magot_copies" || tables.size() >= 64) throw Unsupported();
    const uint32_t k = (uint32_t)tables.size();
    tables.push_back(Table{name, {}});
    table_index.emplace(name, k);
    std::vector<uint32_t> order(tables.size());
    for (uint32_t i = 0; i < order.size(); ++i) order[i] = i;
    std::sort(order.begin(), order.end(),
              [&](uint32_t a, uint32_t b) { return tables[a].name < tables[b].name; });
    rank.assign(tables.size(), 0);
    for (uint32_t r = 0; r < order.size(); ++r) rank[order[r]] = r;
    return k;
  }
  // AnnotationSet.__getitem__ (genome.py:536-544): -1 when no table holds it
  int64_t lookup(uint32_t idk) const {
    const uint64_t m = idk < id_types.size() ? id_types[idk] : 0;
    if (!m) return -1;
    if (!(m & (m - 1))) return first_feat[idk];
    int best = -1;
    for (uint32_t t = 0; t < tables.size(); ++t)
      if ((m >> t) & 1)
        if (best < 0 || rank[t] > rank[(uint32_t)best]) best = (int)t;
    return slot((uint32_t)best, idk);
  }
  int64_t lookup(sv s) const {
    const int64_t k = ids.find(s);
    return k < 0 ? -1 : lookup((uint32_t)k);
  }
  // table[ID] = feature (a dict assignment: an existing key keeps its position)
  void put(uint32_t t, uint32_t idk, uint32_t f) {
    const uint64_t m = id_types[idk];
    if ((m >> t) & 1) {  // existing key: new value, same position
      if (first_table[idk] == t) first_feat[idk] = f;
      else more_feat[((uint64_t)idk << 6) | t] = f;
      return;
    }
    tables[t].keys.push_back(idk);
    if (!m) {
      first_table[idk] = (uint8_t)t;
      first_feat[idk] = f;
    } else {
      more_feat[((uint64_t)idk << 6) | t] = f;
    }
    id_types[idk] = m | (1ull << t);
  }
};

// ---------------------------------------------------------------------------
// read_gff (genome.py:242-415) with the default arguments of gff2fasta
// ---------------------------------------------------------------------------

inline bool is_space(char c) {
  return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\v' || c == '\f';
}

void split_ws(sv s, std::vector<sv>& out) {  // str.split()
  out.clear();
  size_t i = 0, n = s.size();
  while (i < n) {
    while (i < n && is_space(s[i])) ++i;
    if (i >= n) break;
    size_t j = i;
    while (j < n && !is_space(s[j])) ++j;
    out.push_back(s.substr(i, j - i));
    i = j;
  }
}

// int() of a coordinate column: optional surrounding whitespace and sign,
// decimal digits.  Anything else (ValueError in the reference) -> object path.
int64_t parse_int(sv s) {
  size_t i = 0, n = s.size();
  while (i < n && is_space(s[i])) ++i;
  while (n > i && is_space(s[n - 1])) --n;
  bool neg = false;
  if (i < n && (s[i] == '+' || s[i] == '-')) neg = s[i++] == '-';
  if (i >= n || n - i > 18) throw Unsupported();
  int64_t v = 0;
  for (; i < n; ++i) {
    if (s[i] < '0' || s[i] > '9') throw Unsupported();
    v = v * 10 + (s[i] - '0');
  }
  return neg ? -v : v;
}

struct Tags {  // a dict: later assignments update the value in place
  std::vector<std::pair<sv, sv>> kv;
  const sv* get(sv k) const {
    for (const auto& p : kv)
      if (p.first == k) return &p.second;
    return nullptr;
  }
  void set(sv k, sv v) {
    for (auto& p : kv)
      if (p.first == k) {
        p.second = v;
        return;
      }
    kv.emplace_back(k, v);
  }
};

// Stable byte storage for lines / IDs the parser has to rewrite.
struct Arena {
  std::vector<std::unique_ptr<char[]>> blocks;
  char* cur = nullptr;
  size_t left = 0;
  char* alloc(size_t n) {
    if (n > left) {
      const size_t sz = std::max<size_t>(n, 1 << 16);
      blocks.emplace_back(new char[sz]);
      cur = blocks.back().get();
      left = sz;
    }
    char* p = cur;
    cur += n;
    left -= n;
    return p;
  }
  sv join(std::initializer_list<sv> parts) {
    size_t n = 0;
    for (sv p : parts) n += p.size();
    char* out = alloc(n);
    char* o = out;
    for (sv p : parts) {
      if (!p.empty()) memcpy(o, p.data(), p.size());
      o += p.size();
    }
    return sv(out, n);
  }
};

// Settings read_gff fixes on the first accepted line (genome.py:262-292).
struct GffFormat {
  int version = 0;  // 0 = auto (no accepted line yet)
  // gff2fasta(from_exons="True") (genome_tools.py:326-327): features_to_replace
  // [('exon', 'CDS')] and features_to_ignore="CDS", a str, so `in` is a
  // substring test
  bool from_exons = false;
  bool have_id_field = true, have_parent_field = true;  // IDfield='ID', parent_field='Parent'
  std::vector<std::string> hierarchy;
};

// One accepted, non-ignored line after the per-line work that does not touch
// the model: columns, coordinates, tags, the ID (before de-duplication) and
// the parent / hierarchy values, each with its hash.
struct GffLine {
  sv id, parent;
  uint64_t h_id, h_parent;
  // j-th repeat of the previous line's ID (0: differs): the ordered pass
  // likely renames it to ID2 (j = 1) or ID-(j+1); h_dup is that name's hash
  uint64_t h_dup;
  uint32_t dup_run;
  int64_t lo, hi;
  uint32_t seqid, ftype, strand;  // chunk-local codes (LocalIntern)
  uint8_t has_parent, hv_mask;
};

// The hierarchy values of a GTF line (gene_id / transcript_id), kept beside
// the lines only when the format has a hierarchy: GFF3's lines stay compact.
struct GffHier {
  sv hv[2];
  uint64_t h_hv[2];
};

// Chunk-local string codes (seqid, type, strand) so that the ordered pass
// maps a few codes per chunk to the model's instead of comparing text.
struct LocalIntern {
  std::vector<sv> strs;
  std::unordered_map<sv, uint32_t> map;
  uint32_t last = ~0u;
  uint32_t code(sv s) {
    if (last != ~0u && strs[last] == s) return last;
    auto it = map.find(s);
    if (it == map.end()) {
      it = map.emplace(s, (uint32_t)strs.size()).first;
      strs.push_back(s);
    }
    return last = it->second;
  }
};

// The line's columns (the 8 tabs exactly; '\r' stripped, '\n' ends a line).
// Returns false for lines read_gff skips.
inline bool split_line(const char* raw, uint64_t rl, Arena& arena, sv cols[9]) {
  if (rl == 0 || raw[0] == '#') return false;
  uint32_t tpos[9];
  int tabs = 0;
  bool cr = false;
  for (uint64_t i = 0; i < rl; ++i) {
    const char ch = raw[i];
    if (ch == '\t') {
      if (tabs < 9) tpos[tabs] = (uint32_t)i;
      ++tabs;
    }
    cr |= ch == '\r';
  }
  if (tabs != 8) return false;
  sv line(raw, rl);
  if (cr) {  // line.replace('\n', '').replace('\r', '')
    char* o = arena.alloc(rl);
    size_t m = 0;
    for (uint64_t i = 0; i < rl; ++i)
      if (raw[i] != '\n' && raw[i] != '\r') o[m++] = raw[i];
    line = sv(o, m);
    tabs = 0;
    for (size_t i = 0; i < line.size(); ++i)
      if (line[i] == '\t') tpos[tabs++] = (uint32_t)i;
  } else if (raw[rl - 1] == '\n') {
    line = sv(raw, rl - 1);
  }
  size_t b = 0;
  for (int c = 0; c < 8; ++c) {
    cols[c] = line.substr(b, tpos[c] - b);
    b = tpos[c] + 1;
  }
  cols[8] = line.substr(b);
  return true;
}

// Version / ID-field / hierarchy detection from the first accepted line.
void detect_format(GffFormat& F, sv tags_text) {
  if (tags_text.find('=') != sv::npos) {
    F.version = 3;
    return;
  }
  F.version = 2;
  std::string spaced = " " + std::string(tags_text);
  std::replace(spaced.begin(), spaced.end(), ';', ' ');
  if (F.have_id_field && F.hierarchy.empty() && spaced.find(" ID ") == std::string::npos) {
    F.have_id_field = false;
    F.have_parent_field = false;
    const bool g = tags_text.find("gene_id") != sv::npos;
    const bool t = tags_text.find("transcript_id") != sv::npos;
    if (g && t) F.hierarchy = {"transcript_id", "gene_id"};
    else if (g) F.hierarchy = {"gene_id"};
  }
}

// The de-duplicated name of the r-th line (r >= 2) holding an existing ID
// (genome.py:330-338): ID2, then ID-3, ID-4 ...
inline void dup_name(sv id, uint32_t j, std::string& out) {
  char buf[16];
  char* e = buf + sizeof buf;
  char* p = e;
  if (j == 1) {
    *--p = '2';
  } else {
    for (uint32_t v = j + 1; v; v /= 10) *--p = (char)('0' + v % 10);
    *--p = '-';
  }
  out.assign(id.data(), id.size());
  out.append(p, (size_t)(e - p));
}

struct LineParser {
  const GffFormat& F;
  Arena arena;
  Tags tags;
  std::vector<sv> words;
  LocalIntern seqids, ftypes, strands;
  sv prev_id;
  uint32_t prev_run = 0;
  std::string dup;
  std::vector<uint64_t> type_lines;  // accepted lines per local type code

  // false: the line is skipped; throws Unsupported on a diagnostic path
  bool parse(const char* raw, uint64_t rl, GffLine& L, GffHier& H) {
    if (F.from_exons && sv(raw, rl).find("\texon\t") != sv::npos) {
      // line.replace("\texon\t", "\tCDS\t") (genome.py:285-286): left to right,
      // non-overlapping; the tab count (checked before, :283) is unchanged
      // (into the arena: the parsed line's views must outlive this call)
      const sv line(raw, rl);
      char* o = arena.alloc(rl);
      size_t m = 0, b = 0;
      for (size_t e; (e = line.find("\texon\t", b)) != sv::npos; b = e + 6) {
        memcpy(o + m, line.data() + b, e - b);
        m += e - b;
        memcpy(o + m, "\tCDS\t", 5);
        m += 5;
      }
      memcpy(o + m, line.data() + b, rl - b);
      m += rl - b;
      raw = o;
      rl = m;
    }
    sv cols[9];
    if (!split_line(raw, rl, arena, cols)) return false;
    const sv tags_text = cols[8];
    const sv ftype = cols[2];
    // features_to_ignore: ['exon'] by default; "CDS" (substring test) for from_exons
    if (F.from_exons ? sv("CDS").find(ftype) != sv::npos : ftype == "exon") return false;
    int64_t lo = parse_int(cols[3]), hi = parse_int(cols[4]);
    if (lo > hi) std::swap(lo, hi);
    L.lo = lo;
    L.hi = hi;
    L.seqid = seqids.code(cols[0]);
    L.ftype = ftypes.code(ftype);
    if (L.ftype >= type_lines.size()) type_lines.resize(L.ftype + 1, 0);
    ++type_lines[L.ftype];
    L.strand = strands.code(cols[6]);
    tags.kv.clear();
    size_t b = 0;
    for (;;) {
      const size_t e = tags_text.find(';', b);
      const sv item = tags_text.substr(b, e == sv::npos ? sv::npos : e - b);
      if (!item.empty()) {
        if (F.version == 2) {
          split_ws(item, words);
          if (words.empty()) throw Unsupported();  // IndexError
          const size_t q = item.find('"');
          if (q != sv::npos) {
            const size_t q2 = item.find('"', q + 1);
            tags.set(words[0], item.substr(q + 1, q2 == sv::npos ? sv::npos : q2 - q - 1));
          } else if (words.size() > 1) {
            tags.set(words[0], words[1]);
          } else {
            throw Unsupported();  // print(item); return None
          }
        } else {
          const size_t q = item.find('=');
          if (q == sv::npos) throw Unsupported();  // IndexError
          const size_t q2 = item.find('=', q + 1);
          tags.set(item.substr(0, q), item.substr(q + 1, q2 == sv::npos ? sv::npos : q2 - q - 1));
        }
      }
      if (e == sv::npos) break;
      b = e + 1;
    }
    const sv* parent = nullptr;
    if (F.have_parent_field) {
      parent = tags.get("Parent");
    } else {
      for (const std::string& k : F.hierarchy)
        if ((parent = tags.get(k))) break;
    }
    const sv* id = F.have_id_field ? tags.get("ID") : nullptr;
    if (id) L.id = *id;
    else if (F.have_id_field && !parent) throw Unsupported();  // ID None
    else if (parent) L.id = arena.join({*parent, "-", ftype});
    else L.id = arena.join({cols[0], "-", ftype, cols[3]});
    L.h_id = hash_sv(L.id);
    L.dup_run = L.id == prev_id ? prev_run + 1 : 0;
    prev_id = L.id;
    prev_run = L.dup_run;
    if (L.dup_run) {
      dup_name(L.id, L.dup_run, dup);
      L.h_dup = hash_sv(dup);
    }
    L.has_parent = parent != nullptr;
    L.hv_mask = 0;
    if (parent) {
      L.parent = *parent;
      L.h_parent = hash_sv(L.parent);
      for (size_t level = 0; level < F.hierarchy.size(); ++level)
        if (const sv* pid = tags.get(F.hierarchy[level])) {
          H.hv[level] = *pid;
          H.h_hv[level] = hash_sv(*pid);
          L.hv_mask |= (uint8_t)(1u << level);
        }
    }
    return true;
  }
};

// Pages of freshly reserved buffers mapped ahead of their first writes,
// madvise(MADV_POPULATE_WRITE) over page-aligned pieces on several threads
// (the kernel zeroes the pages without a fault per page).  Best effort: a
// kernel without it leaves the pages to fault in on use.
struct Prefault {
  struct Range {
    uintptr_t a, b;
  };
  std::vector<Range> ranges;
  void add(const void* p, size_t bytes) {
    const uintptr_t pg = 4096;
    const uintptr_t a = (reinterpret_cast<uintptr_t>(p) + pg - 1) & ~(pg - 1);
    const uintptr_t b = (reinterpret_cast<uintptr_t>(p) + bytes) & ~(pg - 1);
    for (uintptr_t x = a; x < b; x += (8u << 20)) ranges.push_back({x, std::min(b, x + (8u << 20))});
  }
  void run(unsigned threads) {
    std::atomic<size_t> next{0};
    auto work = [&]() {
      for (size_t i; (i = next.fetch_add(1)) < ranges.size();)
        (void)madvise(reinterpret_cast<void*>(ranges[i].a), ranges[i].b - ranges[i].a,
                      kMadvPopulateWrite);
    };
    std::vector<std::thread> pool;
    for (unsigned t = 1; t < std::min<size_t>(threads, ranges.size()); ++t) pool.emplace_back(work);
    work();
    for (auto& t : pool) t.join();
  }
  size_t bytes() const {
    size_t n = 0;
    for (const Range& r : ranges) n += r.b - r.a;
    return n;
  }
  static constexpr int kMadvPopulateWrite = 23;  // MADV_POPULATE_WRITE (Linux 5.14)
};

// read_gff in two passes: the per-line work (columns, tags, IDs, hashes) in
// parallel over newline-aligned chunks of the text, then the model updates
// (de-duplication, tables, parents) in file order.  Any diagnostic path
// anywhere declines the whole input, so chunks may find them out of order.
void read_gff(Model& M, const char* text, uint64_t n, bool from_exons) {
  const auto t_start = std::chrono::steady_clock::now();
  GffFormat F;
  F.from_exons = from_exons;
  {  // the first accepted line fixes the format
    Arena arena;
    sv cols[9];
    for (uint64_t pos = 0; pos < n;) {
      const char* nl = static_cast<const char*>(memchr(text + pos, '\n', n - pos));
      const uint64_t end = nl ? (uint64_t)(nl - text) + 1 : n;
      const bool ok = split_line(text + pos, end - pos, arena, cols);
      pos = end;
      if (ok) {
        detect_format(F, cols[8]);
        break;
      }
    }
  }
  if (F.version == 0) return;
  // chunks split at line starts
  unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  if (const char* e = std::getenv("MAGOT_GFF_THREADS")) hw = std::max(1, atoi(e));
  uint64_t n_chunks = n < (1u << 20) ? 1 : std::min<uint64_t>(hw * 8ull, n >> 16);
  if (const char* e = std::getenv("MAGOT_GFF_CHUNKS"))  // test hook: force the split
    n_chunks = std::max<uint64_t>(1, std::min<uint64_t>(strtoull(e, nullptr, 10), n));
  std::vector<uint64_t> cut(n_chunks + 1, n);
  cut[0] = 0;
  for (uint64_t c = 1; c < n_chunks; ++c) {
    uint64_t p = std::max(cut[c - 1], n * c / n_chunks);
    const char* nl = p ? static_cast<const char*>(memchr(text + p - 1, '\n', n - p + 1)) : text;
    cut[c] = !nl ? n : (p ? (uint64_t)(nl - text) + 1 : 0);
  }
  std::vector<std::vector<GffLine>> lines(n_chunks);
  std::vector<std::vector<GffHier>> hiers(n_chunks);  // GTF only
  const bool hier = !F.hierarchy.empty();
  std::vector<std::unique_ptr<LineParser>> parsers(n_chunks);
  FirstError failed;
  std::atomic<bool> unsupported{false};
  std::atomic<uint64_t> next{0};
  auto work = [&]() {
    for (uint64_t c; (c = next.fetch_add(1)) < n_chunks && !unsupported.load();) {
      parsers[c].reset(new LineParser{F, {}, {}, {}});
      LineParser& P = *parsers[c];
      std::vector<GffLine>& out = lines[c];
      std::vector<GffHier>& hout = hiers[c];
      out.reserve((cut[c + 1] - cut[c]) / 96 + 16);
      if (hier) hout.reserve(out.capacity());
      try {
        GffLine L;
        GffHier H;
        for (uint64_t pos = cut[c]; pos < cut[c + 1];) {
          const char* nl =
              static_cast<const char*>(memchr(text + pos, '\n', cut[c + 1] - pos));
          const uint64_t end = nl ? (uint64_t)(nl - text) + 1 : cut[c + 1];
          if (P.parse(text + pos, end - pos, L, H)) {
            out.push_back(L);
            if (hier) hout.push_back(H);
          }
          pos = end;
        }
      } catch (const Unsupported&) {
        unsupported = true;
      } catch (...) {
        failed.set();
        unsupported = true;
      }
    }
  };
  {
    std::vector<std::thread> pool;
    for (unsigned t = 1; t < std::min<uint64_t>(hw, n_chunks); ++t) pool.emplace_back(work);
    work();
    for (auto& t : pool) t.join();
  }
  failed.rethrow();
  if (unsupported) throw Unsupported();
  if (std::getenv("MAGOT_GFF_TIMING"))
    fprintf(stderr, "[gffplan] parse pass %.3f s (%llu chunks)\n",
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count(),
            (unsigned long long)n_chunks);
  uint64_t total = 0;
  for (auto& v : lines) total += v.size();
  M.ids.reserve(total + 16);
  M.feats.reserve(total + 16);
  M.id_types.reserve(total + 16);
  M.first_table.reserve(total + 16);
  M.first_feat.reserve(total + 16);
  M.ids.strs.reserve(total + 16);
  M.link_child.reserve(total + 16);  // one child per line with a parent (GFF3)
  M.link_next.reserve(total + 16);
  // model updates in file order
  std::vector<uint32_t> renamed;  // per ID: 0, or the last suffix used
  renamed.reserve(total + 16);
  // the hierarchy's tables, then every line type's table in first-seen order
  // (chunk by chunk: what the pass below would create at each type's first
  // line), so the tables' key lists can be reserved for their lines
  std::vector<uint32_t> hier_table;
  for (const std::string& hk : F.hierarchy)
    hier_table.push_back(M.table(sv(hk).substr(0, hk.find('_'))));
  {
    std::vector<uint64_t> want(M.tables.size(), 0);
    for (uint64_t c = 0; c < n_chunks; ++c) {
      const LineParser& P = *parsers[c];
      for (size_t k = 0; k < P.ftypes.strs.size(); ++k) {
        const uint32_t t = M.table(P.ftypes.strs[k]);
        if (t >= want.size()) want.resize(t + 1, 0);
        want[t] += k < P.type_lines.size() ? P.type_lines[k] : 0;
      }
    }
    for (size_t t = 0; t < want.size(); ++t) M.tables[t].keys.reserve(want[t] + 16);
  }
  {
    // the ordered pass below writes these in growing order; their pages are
    // mapped here, on every host thread at once (C3: ~0.5 GB that the pass
    // would otherwise fault in one page at a time)
    Prefault pf;
    for (const Table& t : M.tables) pf.add(t.keys.data(), t.keys.capacity() * 4);
    pf.add(&M.ids.slots[0], M.ids.slots.size() * 8);
    pf.add(M.ids.strs.data(), M.ids.strs.capacity() * sizeof(sv));
    pf.add(M.feats.data(), M.feats.capacity() * sizeof(Feature));
    pf.add(M.id_types.data(), M.id_types.capacity() * 8);
    pf.add(M.first_table.data(), M.first_table.capacity());
    pf.add(M.first_feat.data(), M.first_feat.capacity() * 4);
    pf.add(renamed.data(), renamed.capacity() * 4);
    pf.add(M.link_child.data(), M.link_child.capacity() * 4);
    pf.add(M.link_next.data(), M.link_next.capacity() * 4);
    pf.run(hw);
    if (std::getenv("MAGOT_GFF_TIMING"))
      fprintf(stderr, "[gffplan] prefault  %.3f s (%zu MiB)\n",
              std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count(),
              pf.bytes() >> 20);
  }
  std::string nid;
  std::vector<uint32_t> sq_of, st_of, ty_of;  // chunk code -> model index
  std::vector<uint8_t> ty_base;
  constexpr size_t kAhead = 16;
  sv last_id, last_parent;
  int64_t last_k0 = -1, last_pk = -1;
  for (uint64_t c = 0; c < n_chunks; ++c) {
    const std::vector<GffLine>& V = lines[c];
    const std::vector<GffHier>& HV = hiers[c];
    const LineParser& P = *parsers[c];
    sq_of.assign(P.seqids.strs.size(), ~0u);
    st_of.assign(P.strands.strs.size(), ~0u);
    ty_of.assign(P.ftypes.strs.size(), ~0u);
    ty_base.assign(P.ftypes.strs.size(), 0);
    for (size_t li = 0; li < V.size(); ++li) {
      if (li + kAhead < V.size()) {
        const GffLine& A = V[li + kAhead];
        M.ids.prefetch(A.dup_run ? A.h_dup : A.h_id);
        if (A.has_parent) M.ids.prefetch(A.h_parent);
      }
      const GffLine& L = V[li];
      // de-duplicate against every table; the new name is not re-checked
      uint32_t idk;
      const size_t n_ids = M.ids.strs.size();
      {
        // runs of lines share an ID (CDS parts) or a parent: IDs are never
        // removed, so the last string's index stays valid
        int64_t k0;
        if (L.id == last_id) {
          k0 = last_k0;
        } else {
          k0 = M.ids.find(L.id, L.h_id);
        }
        if (k0 >= 0 && M.lookup((uint32_t)k0) >= 0) {
          if (renamed.size() <= (size_t)k0) renamed.resize(M.ids.strs.size() + 1, 0);
          uint32_t& r = renamed[(size_t)k0];
          r = r ? r + 1 : 2;
          dup_name(L.id, r - 1, nid);
          idk = L.dup_run == r - 1 ? M.id(nid, L.h_dup) : M.id(nid);
        } else {
          idk = M.id(L.id, L.h_id);
          k0 = idk;
        }
        last_id = L.id;
        last_k0 = k0;
      }
      // seqids / strands interned in first-seen order, as the Python strings are
      if (sq_of[L.seqid] == ~0u) sq_of[L.seqid] = M.seqids.intern(P.seqids.strs[L.seqid]);
      if (st_of[L.strand] == ~0u) st_of[L.strand] = M.strands.intern(P.strands.strs[L.strand]);
      const uint32_t sq = sq_of[L.seqid], st = st_of[L.strand];
      if (L.has_parent) {
        uint32_t child = idk;
        for (size_t level = 0; level < F.hierarchy.size(); ++level) {
          if (!((L.hv_mask >> level) & 1)) continue;
          const uint32_t t = hier_table[level];
          const uint32_t pk = M.id(HV[li].hv[level], HV[li].h_hv[level]);
          const int64_t have = M.slot(t, pk);
          if (have >= 0) {
            Feature& hf = M.feats[(size_t)have];
            if (!M.has_child(hf, child)) M.add_child(hf, child);
          } else {
            Feature f;
            f.type = t;
            f.seqid = sq;
            f.strand = st;
            f.base = false;
            M.add_child(f, child);
            M.feats.push_back(std::move(f));
            M.put(t, pk, (uint32_t)M.feats.size() - 1);
          }
          child = pk;
        }
        if (L.parent != last_parent) {
          last_pk = M.ids.find(L.parent, L.h_parent);
          last_parent = L.parent;
        }
        const int64_t pk = last_pk;
        const int64_t h = pk < 0 ? -1 : M.lookup((uint32_t)pk);
        if (h < 0) throw Unsupported();        // orphan: print, return None
        Feature& holder = M.feats[(size_t)h];
        if (holder.base) throw Unsupported();  // BaseAnnotation has no child_list
        // without a hierarchy, a name interned on this line is in no child list yet
        if ((idk >= n_ids && F.hierarchy.empty()) || !M.has_child(holder, idk))
          M.add_child(holder, idk);
      }
      if (ty_of[L.ftype] == ~0u) {  // the table is created at the type's first line
        const sv ft = P.ftypes.strs[L.ftype];
        ty_of[L.ftype] = M.table(ft);
        ty_base[L.ftype] = ft == "CDS" || ft == "match_part" || ft == "similarity" || ft == "region";
      }
      Feature f;
      f.type = ty_of[L.ftype];
      f.seqid = sq;
      f.lo = L.lo;
      f.hi = L.hi;
      f.strand = st;
      f.base = ty_base[L.ftype];
      const uint32_t ty = f.type;
      M.feats.push_back(std::move(f));
      M.put(ty, idk, (uint32_t)M.feats.size() - 1);
    }
  }
}

// ---------------------------------------------------------------------------
// CPython 2.7 dict order (magot_amd/py2order.py)
// ---------------------------------------------------------------------------

uint64_t py2_hash(sv s) {
  if (s.empty()) return 0;
  uint64_t h = (uint64_t)(uint8_t)s[0] << 7;
  for (unsigned char c : s) h = (h * 1000003ull) ^ c;
  h ^= (uint64_t)s.size();
  if (h == ~0ull) h = ~0ull - 1;
  return h;
}

std::vector<uint32_t> py2_dict_order(const std::vector<uint32_t>& keys,
                                     const std::vector<uint64_t>& hash) {
  std::vector<int64_t> slots(8, -1);
  uint64_t used = 0;
  auto place = [&](std::vector<int64_t>& tab, uint32_t k) -> bool {
    const uint64_t mask = tab.size() - 1, h = hash[k];
    uint64_t i = h & mask, perturb = h;
    for (;;) {
      int64_t& cur = tab[i & mask];
      if (cur < 0) {
        cur = k;
        return true;
      }
      if ((uint32_t)cur == k) return false;
      i = i * 5 + perturb + 1;
      perturb >>= 5;
    }
  };
  constexpr size_t kAhead = 8;  // the slot a key probes first, fetched a few keys ahead
  for (size_t q = 0; q < keys.size(); ++q) {
    if (q + kAhead < keys.size())
      __builtin_prefetch(&slots[hash[keys[q + kAhead]] & (slots.size() - 1)]);
    const uint32_t k = keys[q];
    if (!place(slots, k)) continue;
    ++used;
    if (used * 3 >= slots.size() * 2) {
      const uint64_t want = (used > 50000 ? 2 : 4) * used;
      uint64_t size = 8;
      while (size <= want) size <<= 1;
      std::vector<int64_t> fresh(size, -1);
      for (int64_t k2 : slots)
        if (k2 >= 0) place(fresh, (uint32_t)k2);
      slots.swap(fresh);
    }
  }
  std::vector<uint32_t> out;
  out.reserve(used);
  for (int64_t k : slots)
    if (k >= 0) out.push_back((uint32_t)k);
  return out;
}

}  // namespace
}  // namespace magot

// ---------------------------------------------------------------------------
// get_fasta lowering + C ABI
// ---------------------------------------------------------------------------

namespace magot {
// Lowered output: interval / record tables for magot_plan_create and the
// text skeleton (pieces are text slices or record payload slots).
struct Piece {
  uint64_t off, len;  // text piece, or ...
  int64_t rec;        // ... record payload index (>= 0)
};
struct Lowered {
  std::vector<magot_exon> exons;
  std::vector<magot_tx> txs;
  std::string text;
  std::vector<Piece> pieces;
  // longest=True over protein candidates (genome.py:720-724): the choice
  // depends on the peptides' trimmed lengths, so it is made at render time.
  // Per group: the first piece of each candidate, then the group's end piece.
  std::vector<std::vector<uint64_t>> groups;
};
}  // namespace magot

struct magot_gffplan : magot::Lowered {
  magot::Model model;
  bool protein = false;
  int stage = 0;  // 1: read (magot_gff_read), 2: lowered (magot_gff_lower)
};

namespace magot {
namespace {

void append_lowered(Lowered& all, const Lowered& part);

struct Lowering {
  Lowered& P;
  const Model& M;
  const bool protein;
  const std::vector<int64_t>& contig_idx;  // seqid -> contig (-1: missing)
  const uint64_t* contig_len;
  const std::vector<uint32_t>& id_of_feat;  // the ID a feature was stored under
  bool longest = false;  // get_fasta(longest=True), applied at the top level only
  std::vector<std::pair<std::pair<int64_t, int64_t>, magot_exon>> by_;  // base-branch scratch

  void text(sv s) {
    if (s.empty()) return;
    P.pieces.push_back({P.text.size(), s.size(), -1});
    P.text += s;
  }
  void header(sv id) {  // ">" + ID + "\n"
    P.pieces.push_back({P.text.size(), id.size() + 2, -1});
    P.text += '>';
    P.text += id;
    P.text += '\n';
  }

  // slice contig[a:b] (Python rules, step 1) -> (start, length)
  static void slice(int64_t a, int64_t b, int64_t len, uint64_t* start, uint64_t* length) {
    auto norm = [&](int64_t x) {
      if (x < 0) {
        x += len;
        if (x < 0) x = 0;
      } else if (x > len) {
        x = len;
      }
      return x;
    };
    const int64_t s = norm(a), e = norm(b);
    *start = (uint64_t)s;
    *length = (uint64_t)std::max<int64_t>(0, e - s);
  }

  // ParentAnnotation.get_fasta (genome.py:677-731), longest=False, genomic=False.
  // Returns the number of records emitted ("" <=> 0).
  uint64_t fasta(uint32_t fi, bool first_in_join) {
    const Feature& F = M.feats[fi];
    if (M.children(F).empty()) return 0;
    const int64_t first = M.lookup(M.children(F).front());
    if (first < 0) throw Unsupported();  // KeyError
    if (M.feats[(size_t)first].base) {
      // base branch: child_dict keyed by coords (last wins), order by the last
      // child's strand, each child reverse-complemented by its own strand
      auto& by = by_;  // reused: the base branch does not recurse
      by.clear();
      uint32_t strand = 0;
      for (uint32_t c : M.children(F)) {
        const int64_t o = M.lookup(c);
        if (o < 0) throw Unsupported();
        const Feature& C = M.feats[(size_t)o];
        if (!C.base) throw Unsupported();  // mixed children: print
        const sv sd = M.strands.strs[C.strand];
        if (sd != "+" && sd != "." && sd != "-") throw Unsupported();  // invalid strand: print
        const int64_t cix = contig_idx[C.seqid];
        if (cix < 0) throw Unsupported();  // missing seqid: print
        magot_exon x;
        uint64_t st, ln;
        slice(C.lo - 1, C.hi, (int64_t)contig_len[cix], &st, &ln);
        x.start_rc = st | (sd == "-" ? kRcBit : 0);
        x.contig = (uint32_t)cix;
        x.len = (uint32_t)ln;
        if (ln >= 0xFFFFFFFFull) throw Unsupported();
        const std::pair<int64_t, int64_t> key(C.lo, C.hi);
        bool found = false;
        for (auto& e : by)
          if (e.first == key) {
            e.second = x;
            found = true;
            break;
          }
        if (!found) by.emplace_back(key, x);
        strand = C.strand;
      }
      std::stable_sort(by.begin(), by.end(),
                       [](const auto& a, const auto& b) { return a.first < b.first; });
      if (M.strands.strs[strand] == "-") std::reverse(by.begin(), by.end());
      uint64_t total = 0;
      for (auto& e : by) total += e.second.len;
      if (protein && total <= 2) throw Unsupported();  // translate() -> None
      if (!first_in_join) text("\n");
      header(M.ids.strs[id_of_feat[fi]]);
      magot_tx t;
      t.exon_begin = P.exons.size();
      t.n_exons = (uint32_t)by.size();
      t.flags = 0;
      for (auto& e : by) P.exons.push_back(e.second);
      P.pieces.push_back({0, 0, (int64_t)P.txs.size()});
      P.txs.push_back(t);
      return 1;
    }
    if (longest) return fasta_longest(F);
    uint64_t n = 0;
    for (uint32_t c : M.children(F)) {
      const int64_t o = M.lookup(c);
      if (o < 0) throw Unsupported();
      if (M.feats[(size_t)o].base) throw Unsupported();  // mixed children: print
      n += fasta((uint32_t)o, first_in_join && n == 0);
    }
    return n;
  }

  // Parent branch with longest=True (genome.py:711-724): each child's
  // get_fasta (longest=False) is a candidate unless it is ""; the key of a
  // candidate string is len("".join(seq.split('\n')[1:])), a dict keyed by it
  // keeps the later candidate of a length, and the maximal key wins.  No
  // candidate: max() of an empty list, ValueError.
  uint64_t fasta_longest(const Feature& F) {
    if (protein) return fasta_longest_protein(F);
    Lowered best;
    uint64_t best_key = 0;
    bool have = false;
    for (uint32_t c : M.children(F)) {
      const int64_t o = M.lookup(c);
      if (o < 0) throw Unsupported();
      if (M.feats[(size_t)o].base) throw Unsupported();  // mixed children: print
      Lowered T;
      Lowering sub{T, M, protein, contig_idx, contig_len, id_of_feat};
      if (sub.fasta((uint32_t)o, true) == 0) continue;  // child_fasta == ""
      const uint64_t key = candidate_key(T);
      if (!have || key >= best_key) {
        best = std::move(T);
        best_key = key;
        have = true;
      }
    }
    if (!have) throw Unsupported();
    append_lowered(P, best);
    return 1;
  }

  // Protein: a peptide's length depends on the genome (the leading-'X' trim),
  // so every candidate is lowered and the render picks (magot_gffplan_render).
  uint64_t fasta_longest_protein(const Feature& F) {
    std::vector<Lowered> cands;
    for (uint32_t c : M.children(F)) {
      const int64_t o = M.lookup(c);
      if (o < 0) throw Unsupported();
      if (M.feats[(size_t)o].base) throw Unsupported();  // mixed children: print
      Lowered T;
      Lowering sub{T, M, protein, contig_idx, contig_len, id_of_feat};
      if (sub.fasta((uint32_t)o, true) == 0) continue;  // child_fasta == ""
      cands.push_back(std::move(T));
    }
    if (cands.empty()) throw Unsupported();  // max() of an empty list
    std::vector<uint64_t> group;
    for (const Lowered& T : cands) {
      group.push_back(P.pieces.size());
      append_lowered(P, T);
    }
    group.push_back(P.pieces.size());
    if (cands.size() > 1) P.groups.push_back(std::move(group));
    return 1;
  }

  // Characters of a lowered candidate string that are not '\n', after its
  // first line (nucleotide payloads: the records' interval lengths).
  static uint64_t candidate_key(const Lowered& T) {
    uint64_t n = 0, first_line = 0;
    bool in_first = true;
    for (const Piece& pc : T.pieces) {
      if (pc.rec >= 0) {
        const magot_tx& t = T.txs[(size_t)pc.rec];
        uint64_t len = 0;
        for (uint64_t e = t.exon_begin; e < t.exon_begin + t.n_exons; ++e) len += T.exons[e].len;
        n += len;
        if (in_first) first_line += len;
        continue;
      }
      for (uint64_t k = pc.off; k < pc.off + pc.len; ++k) {
        if (T.text[k] == '\n') {
          in_first = false;
          continue;
        }
        ++n;
        if (in_first) ++first_line;
      }
    }
    return n - first_line;
  }

  // get_coords() (genome.py:663-675): min and max over the children's coords,
  // recursively.  A parent without children returns None, and the caller's
  // [0] raises TypeError.
  void coords(const Feature& F, int64_t& lo, int64_t& hi) const {
    if (M.children(F).empty()) throw Unsupported();
    for (uint32_t c : M.children(F)) {
      const int64_t o = M.lookup(c);
      if (o < 0) throw Unsupported();  // KeyError
      const Feature& C = M.feats[(size_t)o];
      if (C.base) {
        lo = std::min(lo, C.lo);
        hi = std::max(hi, C.hi);
      } else {
        coords(C, lo, hi);
      }
    }
  }

  // genomic=True (genome.py:680-682): ">" + ID + "\n" + contig[lo-1:hi] + "\n",
  // forward strand, never translated.
  void genomic(uint32_t fi) {
    const Feature& F = M.feats[fi];
    int64_t lo = INT64_MAX, hi = INT64_MIN;
    coords(F, lo, hi);
    const int64_t cix = contig_idx[F.seqid];
    if (cix < 0) throw Unsupported();  // KeyError
    uint64_t st, ln;
    slice(lo - 1, hi, (int64_t)contig_len[cix], &st, &ln);
    if (ln >= 0xFFFFFFFFull) throw Unsupported();
    header(M.ids.strs[id_of_feat[fi]]);
    magot_tx t;
    t.exon_begin = P.exons.size();
    t.n_exons = 1;
    t.flags = 0;
    magot_exon x;
    x.start_rc = st;
    x.contig = (uint32_t)cix;
    x.len = (uint32_t)ln;
    P.exons.push_back(x);
    P.pieces.push_back({0, 0, (int64_t)P.txs.size()});
    P.txs.push_back(t);
    text("\n");
  }

};

// Appends `part` (lowered from a later run of keys) to `all`.
void append_lowered(Lowered& all, const Lowered& part) {
  const uint64_t x0 = all.exons.size(), t0 = all.txs.size(), c0 = all.text.size();
  for (std::vector<uint64_t> g : part.groups) {
    for (uint64_t& b : g) b += all.pieces.size();
    all.groups.push_back(std::move(g));
  }
  all.exons.insert(all.exons.end(), part.exons.begin(), part.exons.end());
  for (magot_tx t : part.txs) {
    t.exon_begin += x0;
    all.txs.push_back(t);
  }
  all.text += part.text;
  for (Piece pc : part.pieces) {
    if (pc.rec < 0) pc.off += c0;
    else pc.rec += (int64_t)t0;
    all.pieces.push_back(pc);
  }
}

// Appends parts[1..] to all (= part 0) in order: offsets from the sizes, one
// resize per table, then every part copied into its own slice on host
// threads (C3: 64 parts, 4M intervals, 1.5M text pieces).
void merge_parts(Lowered& all, std::vector<Lowered>& parts) {
  const size_t n = parts.size();
  if (n <= 1) return;
  std::vector<uint64_t> x(n + 1), t(n + 1), c(n + 1), p(n + 1);
  x[1] = all.exons.size();
  t[1] = all.txs.size();
  c[1] = all.text.size();
  p[1] = all.pieces.size();
  for (size_t q = 1; q < n; ++q) {
    x[q + 1] = x[q] + parts[q].exons.size();
    t[q + 1] = t[q] + parts[q].txs.size();
    c[q + 1] = c[q] + parts[q].text.size();
    p[q + 1] = p[q] + parts[q].pieces.size();
  }
  for (size_t q = 1; q < n; ++q)  // selection groups (longest=True over peptides): few
    for (std::vector<uint64_t> g : parts[q].groups) {
      for (uint64_t& b : g) b += p[q];
      all.groups.push_back(std::move(g));
    }
  all.exons.resize(x[n]);
  all.txs.resize(t[n]);
  all.text.resize(c[n]);
  all.pieces.resize(p[n]);
  std::atomic<size_t> next{1};
  auto work = [&]() {
    for (size_t q; (q = next.fetch_add(1)) < n;) {
      Lowered& part = parts[q];
      if (!part.exons.empty())
        memcpy(&all.exons[x[q]], part.exons.data(), part.exons.size() * sizeof(magot_exon));
      for (size_t i = 0; i < part.txs.size(); ++i) {
        magot_tx tx = part.txs[i];
        tx.exon_begin += x[q];
        all.txs[t[q] + i] = tx;
      }
      if (!part.text.empty()) memcpy(&all.text[c[q]], part.text.data(), part.text.size());
      for (size_t i = 0; i < part.pieces.size(); ++i) {
        Piece pc = part.pieces[i];
        if (pc.rec < 0) pc.off += c[q];
        else pc.rec += (int64_t)t[q];
        all.pieces[p[q] + i] = pc;
      }
      part = Lowered();
    }
  };
  const unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  std::vector<std::thread> pool;
  for (unsigned i = 1; i < std::min<size_t>(hw, n - 1); ++i) pool.emplace_back(work);
  work();
  for (auto& th : pool) th.join();
}

}  // namespace
}  // namespace magot

using magot::Unsupported;

extern "C" {

namespace {
// MAGOT_GFF_TIMING: per-phase wall times on stderr
struct GffLap {
  const bool on = std::getenv("MAGOT_GFF_TIMING") != nullptr;
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  void operator()(const char* what) {
    if (!on) return;
    const auto t1 = std::chrono::steady_clock::now();
    fprintf(stderr, "[gffplan] %-10s %.3f s\n", what,
            std::chrono::duration<double>(t1 - t0).count());
    t0 = t1;
  }
};
}  // namespace

int magot_gff_read(const char* gff, uint64_t gff_len, uint32_t flags, magot_gffplan** out) {
  if (!out || (gff_len && !gff)) {
    magot::set_error("magot_gff_read: null argument");
    return MAGOT_ERR_ARG;
  }
  *out = nullptr;
  std::unique_ptr<magot_gffplan> P(new magot_gffplan());
  GffLap lap;
  try {
    magot::read_gff(P->model, gff, gff_len, (flags & MAGOT_GFF_FROM_EXONS) != 0);
    lap("read_gff");
  } catch (const Unsupported&) {
    magot::set_error("magot_gff_read: input takes a diagnostic path; use the object path");
    return MAGOT_ERR_UNSUPPORTED;
  } catch (const std::exception& e) {
    magot::set_error(std::string("magot_gff_read: ") + e.what());
    return MAGOT_ERR_ARG;
  }
  P->stage = 1;
  *out = P.release();
  return MAGOT_OK;
}

int magot_gff_lower(magot_gffplan* P, const char* const* seqids, const uint64_t* contig_lens,
                    uint32_t n_contigs, const char* feature, uint32_t flags, uint64_t* n_exons,
                    uint64_t* n_tx) {
  if (!P || (n_contigs && (!seqids || !contig_lens)) || !feature) {
    magot::set_error("magot_gff_lower: null argument");
    return MAGOT_ERR_ARG;
  }
  if (P->stage != 1) {
    magot::set_error("magot_gff_lower: plan not read (magot_gff_read) or already lowered");
    return MAGOT_ERR_STATE;
  }
  P->stage = 2;
  const bool genomic = (flags & MAGOT_GFF_GENOMIC) != 0;
  P->protein = (flags & MAGOT_GFF_PROTEIN) != 0 && !genomic;  // genomic: never translated
  GffLap lap;
  try {
    magot::Model& M = P->model;
    std::unordered_map<std::string, uint32_t> contig_of;
    for (uint32_t i = 0; i < n_contigs; ++i) contig_of[seqids[i]] = i;  // last duplicate wins
    std::vector<int64_t> contig_idx(M.seqids.strs.size(), -1);
    for (size_t q = 0; q < contig_idx.size(); ++q) {
      auto ci = contig_of.find(std::string(M.seqids.strs[q]));
      if (ci != contig_of.end()) contig_idx[q] = ci->second;
    }
    std::vector<uint32_t> id_of_feat(M.feats.size(), 0);
    for (uint32_t ti2 = 0; ti2 < M.tables.size(); ++ti2)
      for (uint32_t k : M.tables[ti2].keys) id_of_feat[(size_t)M.slot(ti2, k)] = k;
    lap("feat_ids");
    auto ti = M.table_index.find(feature);
    if (ti == M.table_index.end()) throw Unsupported();  // AttributeError
    const magot::Table& T = M.tables[ti->second];
    std::vector<uint32_t> keys = T.keys;
    if (flags & MAGOT_GFF_ORDER_PY2) {
      // the dict simulation runs on positions in `keys` (hash per position:
      // no table sized for every ID of the model)
      std::vector<uint64_t> hash(keys.size());
      std::vector<uint32_t> pos(keys.size());
      for (size_t i = 0; i < keys.size(); ++i) {
        hash[i] = magot::py2_hash(M.ids.strs[keys[i]]);
        pos[i] = (uint32_t)i;
      }
      lap("py2_hash");
      pos = magot::py2_dict_order(pos, hash);  // the table as built ...
      pos = magot::py2_dict_order(pos, hash);  // ... and as deep-copied (genome.py:415)
      std::vector<uint32_t> ordered(pos.size());
      for (size_t i = 0; i < pos.size(); ++i) ordered[i] = keys[pos[i]];
      keys.swap(ordered);
    }
    lap("order");
    // "\n".join(obj.get_fasta() for obj in table.values()): every object adds
    // its records (a blank line when it has none).  The model is read-only
    // here, so runs of keys are lowered in parallel and appended in order.
    const uint32_t table = ti->second;
    const size_t n_keys = keys.size();
    size_t n_parts = n_keys < 4096 ? 1 : std::min<size_t>(64, n_keys / 2048);
    if (const char* e = std::getenv("MAGOT_GFF_CHUNKS"))  // test hook: force the split
      n_parts = std::max<size_t>(1, std::min<size_t>(strtoull(e, nullptr, 10), n_keys));
    std::vector<magot::Lowered> parts(n_parts);
    magot::FirstError failed;
    std::atomic<bool> unsupported{false};
    std::atomic<size_t> next{0};
    auto work = [&]() {
      for (size_t q; (q = next.fetch_add(1)) < n_parts && !unsupported.load();) {
        magot::Lowered& out = q ? parts[q] : *P;
        magot::Lowering L{out, M, P->protein, contig_idx, contig_lens, id_of_feat};
        L.longest = (flags & MAGOT_GFF_LONGEST) != 0;
        try {
          for (size_t i = n_keys * q / n_parts; i < n_keys * (q + 1) / n_parts; ++i) {
            const uint32_t fi = (uint32_t)M.slot(table, keys[i]);
            if (M.feats[fi].base) throw Unsupported();  // BaseAnnotation has no get_fasta
            if (i) L.text("\n");
            if (genomic) L.genomic(fi);
            else L.fasta(fi, true);
          }
        } catch (const Unsupported&) {
          unsupported = true;
        } catch (...) {
          failed.set();
          unsupported = true;
        }
      }
    };
    {
      const unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
      std::vector<std::thread> pool;
      for (unsigned t = 1; t < std::min<size_t>(hw, n_parts); ++t) pool.emplace_back(work);
      work();
      for (auto& t : pool) t.join();
    }
    failed.rethrow();
    if (unsupported) throw Unsupported();
    magot::merge_parts(*P, parts);
    lap("lower");
  } catch (const Unsupported&) {
    magot::set_error("magot_gff_lower: input takes a diagnostic path; use the object path");
    return MAGOT_ERR_UNSUPPORTED;
  } catch (const std::exception& e) {
    magot::set_error(std::string("magot_gff_lower: ") + e.what());
    return MAGOT_ERR_ARG;
  }
  if (n_exons) *n_exons = P->exons.size();
  if (n_tx) *n_tx = P->txs.size();
  return MAGOT_OK;
}

int magot_gff_plan(const char* gff, uint64_t gff_len, const char* const* seqids,
                   const uint64_t* contig_lens, uint32_t n_contigs, const char* feature,
                   uint32_t flags, magot_gffplan** out, uint64_t* n_exons, uint64_t* n_tx) {
  if (!out || (gff_len && !gff) || (n_contigs && (!seqids || !contig_lens)) || !feature) {
    magot::set_error("magot_gff_plan: null argument");
    return MAGOT_ERR_ARG;
  }
  *out = nullptr;
  magot_gffplan* P = nullptr;
  if (int rc = magot_gff_read(gff, gff_len, flags, &P)) return rc;
  if (int rc = magot_gff_lower(P, seqids, contig_lens, n_contigs, feature, flags, n_exons, n_tx)) {
    magot_gffplan_destroy(P);
    return rc;
  }
  *out = P;
  return MAGOT_OK;
}

// extract_upstream_downstream (genome_tools.py:457-480) lowered to the same
// plan shape as gff2fasta: one single-interval record per printed window and
// a skeleton ">" name "\n" [record] joined by "\n".  Lines are scanned in
// parallel chunks; the output count ('seq' + count names) and the quirk that a
// matching line with a strand other than '+' / '-' prints the previous
// window again are resolved in one ordered pass.  Every reference error path
// (KeyError, ValueError, IndexError, UnboundLocalError) declines.
int magot_flank_plan(const char* gff, uint64_t gff_len, const char* const* seqids,
                     const uint64_t* contig_lens, uint32_t n_contigs, const char* feature_type,
                     const char* namefrom, const char* sequence_length, const char* stream,
                     magot_gffplan** out, uint64_t* n_exons, uint64_t* n_tx) {
  using magot::sv;
  if (!out || (gff_len && !gff) || (n_contigs && (!seqids || !contig_lens)) || !feature_type ||
      !namefrom || !sequence_length || !stream) {
    magot::set_error("magot_flank_plan: null argument");
    return MAGOT_ERR_ARG;
  }
  *out = nullptr;
  std::unique_ptr<magot_gffplan> P(new magot_gffplan());
  // one matching line: a window of its own, or the previous one again
  struct Hit {
    uint64_t start;
    uint32_t contig, len;
    bool own, rc, has_name;
    sv name;  // into the GFF text; "\r" / "\n" still inside
  };
  try {
    const int64_t n = magot::parse_int(sv(sequence_length));  // int(sequence_length)
    const sv ftype(feature_type), key(namefrom), st(stream);
    const bool up = st == "up", down = st == "down";
    std::unordered_map<sv, uint32_t> contig_of;
    for (uint32_t i = 0; i < n_contigs; ++i) contig_of[sv(seqids[i])] = i;  // last duplicate wins
    unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    uint64_t n_chunks = gff_len < (1u << 20) ? 1 : std::min<uint64_t>(hw * 8ull, gff_len >> 16);
    if (const char* e = std::getenv("MAGOT_GFF_CHUNKS"))  // test hook: force the split
      n_chunks = std::max<uint64_t>(1, std::min<uint64_t>(strtoull(e, nullptr, 10), gff_len));
    std::vector<uint64_t> cut(n_chunks + 1, gff_len);
    cut[0] = 0;
    for (uint64_t c = 1; c < n_chunks; ++c) {
      const uint64_t p = std::max(cut[c - 1], gff_len * c / n_chunks);
      const char* nl =
          p ? static_cast<const char*>(memchr(gff + p - 1, '\n', gff_len - p + 1)) : gff;
      cut[c] = !nl ? gff_len : (p ? (uint64_t)(nl - gff) + 1 : 0);
    }
    std::vector<std::vector<Hit>> hits(n_chunks);
    magot::FirstError failed;
    std::atomic<bool> unsupported{false};
    std::atomic<uint64_t> next{0};
    auto work = [&]() {
      for (uint64_t c; (c = next.fetch_add(1)) < n_chunks && !unsupported.load();) {
        try {
          for (uint64_t pos = cut[c]; pos < cut[c + 1];) {
            // `for line in open(gff)`: lines end after '\n', which they keep
            const char* nl = static_cast<const char*>(memchr(gff + pos, '\n', cut[c + 1] - pos));
            const uint64_t end = nl ? (uint64_t)(nl - gff) + 1 : cut[c + 1];
            const sv line(gff + pos, end - pos);
            pos = end;
            if (line.empty() || line[0] == '#') continue;
            // fields = line.split('\t'), needed when line.count('\t') > 5
            uint32_t tab[8];
            int tabs = 0;
            size_t last = 0;
            for (size_t i = 0; i < line.size(); ++i)
              if (line[i] == '\t') {
                if (tabs < 8) tab[tabs] = (uint32_t)i;
                ++tabs;
                last = i;
              }
            if (tabs < 6) continue;
            auto field = [&](int k) {  // k <= 6; fields[6] may be the last one
              const size_t b = k ? tab[k - 1] + 1 : 0;
              const size_t e = k < tabs ? tab[k] : line.size();
              return line.substr(b, e - b);
            };
            if (field(2) != ftype) continue;
            int64_t lo = magot::parse_int(field(3)), hi = magot::parse_int(field(4));
            if (lo > hi) std::swap(lo, hi);
            Hit h{};
            // the last attribute whose text before its first '=' is namefrom;
            // its name is the text between the first and second '='
            const sv attrs = line.substr(last + 1);
            for (size_t b = 0;;) {
              const size_t e = attrs.find(';', b);
              const sv a = attrs.substr(b, e == sv::npos ? sv::npos : e - b);
              const size_t q = a.find('=');
              if (a.substr(0, q) == key) {
                if (q == sv::npos) throw Unsupported();  // IndexError
                const size_t q2 = a.find('=', q + 1);
                h.name = a.substr(q + 1, q2 == sv::npos ? sv::npos : q2 - q - 1);
                h.has_name = true;
              }
              if (e == sv::npos) break;
              b = e + 1;
            }
            const sv strand = field(6);
            const bool plus = strand == "+", minus = strand == "-";
            int64_t a = 0, b = 0;
            if ((up && plus) || (down && minus)) {  // stop - n .. stop, as printed
              a = lo - 1 - n;
              b = lo - 1;
              h.own = true;
            } else if ((down && plus) || (up && minus)) {  // start .. start + n, reverse complement
              a = hi;
              b = hi + n;
              h.own = h.rc = true;
            }
            if (h.own) {
              const auto ci = contig_of.find(field(0));
              if (ci == contig_of.end()) throw Unsupported();  // KeyError
              const int64_t L = (int64_t)contig_lens[ci->second];
              auto norm = [&](int64_t x) { return x < 0 ? std::max<int64_t>(x + L, 0) : std::min(x, L); };
              const int64_t s = norm(a), e = norm(b);
              const uint64_t ln = (uint64_t)std::max<int64_t>(0, e - s);
              if (ln >= 0xFFFFFFFFull) throw Unsupported();
              h.start = (uint64_t)s;
              h.len = (uint32_t)ln;
              h.contig = ci->second;
            }
            hits[c].push_back(h);
          }
        } catch (const Unsupported&) {
          unsupported = true;
        } catch (...) {
          failed.set();
          unsupported = true;
        }
      }
    };
    {
      std::vector<std::thread> pool;
      for (unsigned t = 1; t < std::min<uint64_t>(hw, n_chunks); ++t) pool.emplace_back(work);
      work();
      for (auto& t : pool) t.join();
    }
    failed.rethrow();
    if (unsupported) throw Unsupported();
    // ordered pass: names, the reused window, "\n".join(output_seqs)
    bool bound = false;
    Hit cur{};
    uint64_t count = 0;
    char num[24];
    for (const auto& V : hits)
      for (const Hit& h : V) {
        if (h.own) {
          cur = h;
          bound = true;
        } else if (!bound) {
          throw Unsupported();  // UnboundLocalError
        }
        if (n < 0 || (int64_t)cur.len != n) continue;
        const uint64_t t0 = P->text.size();
        if (count) P->text += '\n';
        P->text += '>';
        if (h.has_name) {
          for (char ch : h.name)
            if (ch != '\r' && ch != '\n') P->text += ch;
        } else {
          const int k = snprintf(num, sizeof num, "seq%llu", (unsigned long long)count);
          P->text.append(num, (size_t)k);
        }
        P->text += '\n';
        P->pieces.push_back({t0, P->text.size() - t0, -1});
        magot_tx t;
        t.exon_begin = P->exons.size();
        t.n_exons = 1;
        t.flags = 0;
        magot_exon x;
        x.start_rc = cur.start | (cur.rc ? magot::kRcBit : 0);
        x.contig = cur.contig;
        x.len = cur.len;
        P->exons.push_back(x);
        P->pieces.push_back({0, 0, (int64_t)P->txs.size()});
        P->txs.push_back(t);
        ++count;
      }
  } catch (const Unsupported&) {
    magot::set_error("magot_flank_plan: input takes a diagnostic path; use the object path");
    return MAGOT_ERR_UNSUPPORTED;
  } catch (const std::exception& e) {
    magot::set_error(std::string("magot_flank_plan: ") + e.what());
    return MAGOT_ERR_ARG;
  }
  if (n_exons) *n_exons = P->exons.size();
  if (n_tx) *n_tx = P->txs.size();
  *out = P.release();
  return MAGOT_OK;
}

int magot_gffplan_table_views(const magot_gffplan* p, const magot_exon** exons,
                              const magot_tx** txs) {
  if (!p || !exons || !txs) {
    magot::set_error("magot_gffplan_table_views: null argument");
    return MAGOT_ERR_ARG;
  }
  *exons = p->exons.empty() ? nullptr : p->exons.data();
  *txs = p->txs.empty() ? nullptr : p->txs.data();
  return MAGOT_OK;
}

int magot_gffplan_tables(const magot_gffplan* p, magot_exon* exons, magot_tx* txs) {
  if (!p) {
    magot::set_error("magot_gffplan_tables: null plan");
    return MAGOT_ERR_ARG;
  }
  if (exons && !p->exons.empty()) memcpy(exons, p->exons.data(), p->exons.size() * sizeof(magot_exon));
  if (txs && !p->txs.empty()) memcpy(txs, p->txs.data(), p->txs.size() * sizeof(magot_tx));
  return MAGOT_OK;
}

}  // extern "C"

namespace magot {

bool gffplan_units(const magot_gffplan* p, const std::string** text, std::vector<TextUnit>* units,
                   bool* protein, uint64_t* n_rec) {
  *text = &p->text;
  *protein = p->protein;
  *n_rec = p->txs.size();
  if (p->txs.size() >= kNoRecord || !p->groups.empty()) return false;
  units->clear();
  TextUnit cur{0, 0, kNoRecord};
  for (const Piece& pc : p->pieces) {
    if (pc.rec >= 0) {
      cur.rec = (uint32_t)pc.rec;
      units->push_back(cur);
      cur = TextUnit{0, 0, kNoRecord};
      continue;
    }
    // text pieces are laid out back to back in `text`, so runs merge
    if (cur.text_len && (cur.text_off + cur.text_len != pc.off ||
                         cur.text_len + pc.len > 0xFFFFFFFFull)) {
      units->push_back(cur);
      cur = TextUnit{0, 0, kNoRecord};
    }
    if (pc.len > 0xFFFFFFFFull) return false;
    if (!cur.text_len) cur.text_off = pc.off;
    cur.text_len += (uint32_t)pc.len;
  }
  if (cur.text_len) units->push_back(cur);
  return true;
}

}  // namespace magot

extern "C" {

// Record payload: nucleotide bytes, or the translation with one leading 'X'
// dropped (trimX, genome.py:819-821).
static inline void payload(const magot_gffplan* p, int64_t r, const uint8_t* nuc,
                           const uint64_t* noff, const uint8_t* pep, const uint64_t* poff,
                           const uint8_t** src, uint64_t* len) {
  if (!p->protein) {
    *src = nuc + noff[r];
    *len = noff[r + 1] - noff[r];
  } else {
    uint64_t a = poff[r];
    const uint64_t b = poff[r + 1];
    if (b > a && pep[a] == 'X') ++a;
    *src = pep + a;
    *len = b - a;
  }
}

int magot_gffplan_render(const magot_gffplan* p, const uint8_t* nuc, const uint64_t* noff,
                         const uint8_t* pep, const uint64_t* poff, uint8_t* out, uint64_t cap,
                         uint64_t* out_len) {
  if (!p || !out_len || (p->protein ? (!pep || !poff) : (!nuc || !noff))) {
    magot::set_error("magot_gffplan_render: null argument");
    return MAGOT_ERR_ARG;
  }
  // pieces [b, e): appended to `o` (when non-null), returns the byte count
  auto emit = [&](uint64_t b, uint64_t e, uint8_t* o) {
    uint64_t n = 0;
    for (uint64_t i = b; i < e; ++i) {
      const auto& pc = p->pieces[i];
      const uint8_t* s;
      uint64_t l;
      if (pc.rec < 0) {
        s = reinterpret_cast<const uint8_t*>(p->text.data()) + pc.off;
        l = pc.len;
      } else {
        payload(p, pc.rec, nuc, noff, pep, poff, &s, &l);
      }
      if (o) memcpy(o + n, s, l);
      n += l;
    }
    return n;
  };
  // longest=True candidate key: len("".join(seq.split('\n')[1:])) of the
  // candidate string (genome.py:722)
  auto key = [&](uint64_t b, uint64_t e) {
    uint64_t n = 0, first = 0;
    bool in_first = true;
    for (uint64_t i = b; i < e; ++i) {
      const auto& pc = p->pieces[i];
      if (pc.rec >= 0) {
        const uint8_t* s;
        uint64_t l;
        payload(p, pc.rec, nuc, noff, pep, poff, &s, &l);
        n += l;
        if (in_first) first += l;
        continue;
      }
      for (uint64_t k = pc.off; k < pc.off + pc.len; ++k) {
        if (p->text[k] == '\n') {
          in_first = false;
          continue;
        }
        ++n;
        if (in_first) ++first;
      }
    }
    return n - first;
  };
  // the render: pieces in order, each selection group replaced by its
  // longest candidate (the later one on a tie: a dict keyed by the length)
  auto render = [&](uint8_t* o) {
    uint64_t n = 0, i = 0;
    for (const auto& g : p->groups) {
      n += emit(i, g.front(), o ? o + n : nullptr);
      size_t best = 0;
      uint64_t best_key = 0;
      for (size_t c = 0; c + 1 < g.size(); ++c) {
        const uint64_t k = key(g[c], g[c + 1]);
        if (c == 0 || k >= best_key) {
          best = c;
          best_key = k;
        }
      }
      n += emit(g[best], g[best + 1], o ? o + n : nullptr);
      i = g.back();
    }
    return n + emit(i, p->pieces.size(), o ? o + n : nullptr);
  };
  const uint64_t total = render(nullptr);
  *out_len = total;
  if (!out) return MAGOT_OK;
  if (cap < total) {
    magot::set_error("magot_gffplan_render: output buffer too small");
    return MAGOT_ERR_ARG;
  }
  render(out);
  return MAGOT_OK;
}

int magot_gffplan_selections(const magot_gffplan* p, uint64_t* n_groups) {
  if (!p || !n_groups) {
    magot::set_error("magot_gffplan_selections: null argument");
    return MAGOT_ERR_ARG;
  }
  *n_groups = p->groups.size();
  return MAGOT_OK;
}

void magot_gffplan_destroy(magot_gffplan* p) { delete p; }

}  // extern "C"
