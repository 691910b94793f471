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
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <memory>
#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

#include "common.h"

namespace magot {
namespace {

struct Feature {
  uint32_t type = 0;
  uint32_t seqid = 0;   // index into Model::seqids
  int64_t lo = 0, hi = 0;
  uint32_t strand = 0;  // index into Model::strands
  bool base = false;
  std::vector<uint32_t> children;  // child IDs (Model::ids)
};

struct Table {
  std::string name;
  std::vector<uint32_t> keys;  // IDs in insertion order
};

struct Unsupported {};  // a diagnostic path of the reference: use the object path

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

struct Pool {
  std::vector<std::unique_ptr<char[]>> chunks;
  size_t left = 0;
  char* cur = nullptr;
  std::vector<sv> strs;
  std::vector<uint32_t> slots{std::vector<uint32_t>(64, 0)};  // id + 1, 0 = empty
  std::vector<uint32_t> tags{std::vector<uint32_t>(64, 0)};   // hash bits for quick rejects

  void reserve(size_t n) {
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
  void rehash(size_t cap) {
    std::vector<uint32_t> ns(cap, 0), nt(cap, 0);
    const size_t mask = cap - 1;
    for (uint32_t id = 0; id < strs.size(); ++id) {
      const uint64_t h = hash_sv(strs[id]);
      size_t i = h & mask;
      while (ns[i]) i = (i + 1) & mask;
      ns[i] = id + 1;
      nt[i] = (uint32_t)(h >> 32);
    }
    slots.swap(ns);
    tags.swap(nt);
  }
  // slot of s (occupied when found, else the empty slot where it goes)
  size_t probe(sv s, uint64_t h) const {
    const size_t mask = slots.size() - 1;
    size_t i = h & mask;
    const uint32_t tg = (uint32_t)(h >> 32);
    for (;;) {
      const uint32_t v = slots[i];
      if (!v || (tags[i] == tg && strs[v - 1] == s)) return i;
      i = (i + 1) & mask;
    }
  }
  int64_t find(sv s) const {
    const uint32_t v = slots[probe(s, hash_sv(s))];
    return v ? (int64_t)v - 1 : -1;
  }
  uint32_t intern(sv s) {
    const uint64_t h = hash_sv(s);
    size_t i = probe(s, h);
    if (slots[i]) return slots[i] - 1;
    const uint32_t id = (uint32_t)strs.size();
    strs.push_back(store(s));
    if (2 * strs.size() > slots.size()) {
      rehash(slots.size() * 2);
      return id;
    }
    slots[i] = id + 1;
    tags[i] = (uint32_t)(h >> 32);
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

  Model() {
    // AnnotationSet.__init__ (genome.py:528-533) creates these dicts
    for (const char* t : {"gene", "transcript", "CDS", "UTR"}) table(t);
  }

  uint32_t id(sv s) {
    const uint32_t k = ids.intern(s);
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

void read_gff(Model& M, const char* text, uint64_t n) {
  {
    // size the ID table from the line count (about one new ID per line)
    uint64_t lines = 0;
    for (const char* q = text; (q = static_cast<const char*>(memchr(q, '\n', text + n - q)));
         ++q)
      ++lines;
    M.ids.reserve(lines / 2 + 16);
    M.feats.reserve(lines / 2 + 16);
  }
  int version = 0;  // 0 = auto
  bool have_id_field = true, have_parent_field = true;  // IDfield='ID', parent_field='Parent'
  std::vector<std::string> hierarchy;
  std::unordered_map<uint32_t, int64_t> renamed;
  std::string scratch, idbuf;
  std::vector<sv> words;
  Tags tags;
  sv last_seqid, last_strand;
  uint32_t last_sq = 0, last_st = 0;
  bool first_line = true;
  uint64_t pos = 0;
  while (pos < n) {
    const char* nl = static_cast<const char*>(memchr(text + pos, '\n', n - pos));
    const uint64_t end = nl ? (uint64_t)(nl - text) + 1 : n;
    const char* raw = text + pos;
    const uint64_t rl = end - pos;
    pos = end;
    if (raw[0] == '#') continue;
    // the 8 tabs (exactly) of an accepted line
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
    if (tabs != 8) continue;
    // line.replace('\n', '').replace('\r', '')  ('\n' only ends a line)
    sv line(raw, rl);
    if (cr) {
      scratch.clear();
      for (uint64_t i = 0; i < rl; ++i)
        if (raw[i] != '\n' && raw[i] != '\r') scratch.push_back(raw[i]);
      line = sv(scratch);
      tabs = 0;
      for (size_t i = 0; i < line.size(); ++i)
        if (line[i] == '\t') tpos[tabs++] = (uint32_t)i;
    } else if (rl && raw[rl - 1] == '\n') {
      line = sv(raw, rl - 1);
    }
    sv cols[9];
    {
      size_t b = 0;
      for (int c = 0; c < 8; ++c) {
        cols[c] = line.substr(b, tpos[c] - b);
        b = tpos[c] + 1;
      }
      cols[8] = line.substr(b);
    }
    const sv tags_text = cols[8];
    if (version == 0) {
      if (tags_text.find('=') != sv::npos) {
        version = 3;
      } else {
        version = 2;
        std::string spaced = " " + std::string(tags_text);
        std::replace(spaced.begin(), spaced.end(), ';', ' ');
        if (have_id_field && hierarchy.empty() && spaced.find(" ID ") == std::string::npos) {
          have_id_field = false;
          have_parent_field = false;
          const bool g = tags_text.find("gene_id") != sv::npos;
          const bool t = tags_text.find("transcript_id") != sv::npos;
          if (g && t) hierarchy = {"transcript_id", "gene_id"};
          else if (g) hierarchy = {"gene_id"};
        }
      }
    }
    const sv seqid = cols[0];
    const sv ftype = cols[2];
    if (ftype == "exon") continue;  // features_to_ignore default
    int64_t lo = parse_int(cols[3]), hi = parse_int(cols[4]);
    if (lo > hi) std::swap(lo, hi);
    const sv strand = cols[6];
    tags.kv.clear();
    {
      size_t b = 0;
      for (;;) {
        const size_t e = tags_text.find(';', b);
        const sv item = tags_text.substr(b, e == sv::npos ? sv::npos : e - b);
        if (!item.empty()) {
          if (version == 2) {
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
    }
    const sv* parent = nullptr;
    if (have_parent_field) {
      parent = tags.get("Parent");
    } else {
      for (const std::string& k : hierarchy)
        if ((parent = tags.get(k))) break;
    }
    sv ID;
    if (have_id_field && tags.get("ID")) {
      ID = *tags.get("ID");
    } else if (have_id_field && !parent) {
      throw Unsupported();  // ID None
    } else if (parent) {
      idbuf.assign(parent->data(), parent->size());
      idbuf += '-';
      idbuf.append(ftype.data(), ftype.size());
      ID = idbuf;
    } else {
      idbuf.assign(seqid.data(), seqid.size());
      idbuf += '-';
      idbuf.append(ftype.data(), ftype.size());
      idbuf.append(cols[3].data(), cols[3].size());
      ID = idbuf;
    }
    // de-duplicate against every table; the new name is not re-checked
    uint32_t idk;
    {
      const int64_t k0 = M.ids.find(ID);
      if (k0 >= 0 && M.lookup((uint32_t)k0) >= 0) {
        auto it = renamed.find((uint32_t)k0);
        std::string nid(ID);
        if (it != renamed.end()) {
          it->second += 1;
          nid += "-" + std::to_string(it->second);
        } else {
          renamed.emplace((uint32_t)k0, 2);
          nid += "2";
        }
        idk = M.id(nid);
      } else {
        idk = M.id(ID);
      }
    }
    // consecutive lines nearly always share seqid and strand
    if (first_line || seqid != last_seqid) {
      last_sq = M.seqids.intern(seqid);
      last_seqid = M.seqids.strs[last_sq];
    }
    if (first_line || strand != last_strand) {
      last_st = M.strands.intern(strand);
      last_strand = M.strands.strs[last_st];
    }
    first_line = false;
    const uint32_t sq = last_sq, st = last_st;
    if (parent) {
      uint32_t child = idk;
      for (size_t level = 0; level < hierarchy.size(); ++level) {
        const sv* pid = tags.get(hierarchy[level]);
        if (!pid) continue;
        const std::string& hk = hierarchy[level];
        const uint32_t t = M.table(sv(hk).substr(0, hk.find('_')));
        const uint32_t pk = M.id(*pid);
        const int64_t have = M.slot(t, pk);
        if (have >= 0) {
          auto& ch = M.feats[(size_t)have].children;
          if (std::find(ch.begin(), ch.end(), child) == ch.end()) ch.push_back(child);
        } else {
          Feature f;
          f.type = t;
          f.seqid = sq;
          f.strand = st;
          f.base = false;
          f.children.push_back(child);
          M.feats.push_back(std::move(f));
          M.put(t, pk, (uint32_t)M.feats.size() - 1);
        }
        child = pk;
      }
      const int64_t h = M.lookup(*parent);
      if (h < 0) throw Unsupported();                    // orphan: print, return None
      Feature& holder = M.feats[(size_t)h];
      if (holder.base) throw Unsupported();              // BaseAnnotation has no child_list
      if (std::find(holder.children.begin(), holder.children.end(), idk) == holder.children.end())
        holder.children.push_back(idk);
    }
    Feature f;
    f.type = M.table(ftype);
    f.seqid = sq;
    f.lo = lo;
    f.hi = hi;
    f.strand = st;
    f.base = ftype == "CDS" || ftype == "match_part" || ftype == "similarity" || ftype == "region";
    M.feats.push_back(std::move(f));
    M.put(M.feats.back().type, idk, (uint32_t)M.feats.size() - 1);
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
  for (uint32_t k : keys) {
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

struct magot_gffplan {
  magot::Model model;
  // interval / record tables for magot_plan_create
  std::vector<magot_exon> exons;
  std::vector<magot_tx> txs;
  // skeleton: text pieces (offset/length into `text`) and record slots
  std::string text;
  struct Piece {
    uint64_t off, len;  // text piece, or ...
    int64_t rec;        // ... record payload index (>= 0)
  };
  std::vector<Piece> pieces;
  bool protein = false;
};

namespace magot {
namespace {

struct Lowering {
  magot_gffplan& P;
  const std::unordered_map<std::string, uint32_t>& contig_of;
  const uint64_t* contig_len;

  void text(const std::string& s) {
    if (s.empty()) return;
    P.pieces.push_back({P.text.size(), s.size(), -1});
    P.text += s;
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
    const Model& M = P.model;
    const Feature& F = M.feats[fi];
    if (F.children.empty()) return 0;
    const int64_t first = M.lookup(F.children[0]);
    if (first < 0) throw Unsupported();  // KeyError
    if (M.feats[(size_t)first].base) {
      // base branch: child_dict keyed by coords (last wins), order by the last
      // child's strand, each child reverse-complemented by its own strand
      std::vector<std::pair<std::pair<int64_t, int64_t>, magot_exon>> by;
      uint32_t strand = 0;
      for (uint32_t c : F.children) {
        const int64_t o = M.lookup(c);
        if (o < 0) throw Unsupported();
        const Feature& C = M.feats[(size_t)o];
        if (!C.base) throw Unsupported();  // mixed children: print
        const sv sd = M.strands.strs[C.strand];
        if (sd != "+" && sd != "." && sd != "-") throw Unsupported();  // invalid strand: print
        if (contig_idx.size() < M.seqids.strs.size()) contig_idx.resize(M.seqids.strs.size(), -2);
        int64_t& cix = contig_idx[C.seqid];
        if (cix == -2) {
          auto ci = contig_of.find(std::string(M.seqids.strs[C.seqid]));
          cix = ci == contig_of.end() ? -1 : (int64_t)ci->second;
        }
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
      if (P.protein && total <= 2) throw Unsupported();  // translate() -> None
      if (!first_in_join) text("\n");
      text(">" + std::string(M.ids.strs[idk_of(fi)]) + "\n");
      magot_tx t;
      t.exon_begin = P.exons.size();
      t.n_exons = (uint32_t)by.size();
      t.flags = 0;
      for (auto& e : by) P.exons.push_back(e.second);
      P.pieces.push_back({0, 0, (int64_t)P.txs.size()});
      P.txs.push_back(t);
      return 1;
    }
    uint64_t n = 0;
    for (uint32_t c : F.children) {
      const int64_t o = M.lookup(c);
      if (o < 0) throw Unsupported();
      if (M.feats[(size_t)o].base) throw Unsupported();  // mixed children: print
      n += fasta((uint32_t)o, first_in_join && n == 0);
    }
    return n;
  }

  // the ID a feature was stored under (ParentAnnotation.ID)
  std::vector<uint32_t> id_of_feat;
  std::vector<int64_t> contig_idx;  // seqid -> contig (-1 missing, -2 unknown yet)
  uint32_t idk_of(uint32_t fi) const { return id_of_feat[fi]; }
};

}  // namespace
}  // namespace magot

using magot::Unsupported;

extern "C" {

int magot_gff_plan(const char* gff, uint64_t gff_len, const char* const* seqids,
                   const uint64_t* contig_lens, uint32_t n_contigs, const char* feature,
                   uint32_t flags, magot_gffplan** out, uint64_t* n_exons, uint64_t* n_tx) {
  if (!out || (gff_len && !gff) || (n_contigs && (!seqids || !contig_lens)) || !feature) {
    magot::set_error("magot_gff_plan: null argument");
    return MAGOT_ERR_ARG;
  }
  *out = nullptr;
  std::unique_ptr<magot_gffplan> P(new magot_gffplan());
  P->protein = (flags & MAGOT_GFF_PROTEIN) != 0;
  const bool timing = std::getenv("MAGOT_GFF_TIMING") != nullptr;
  auto now = [] { return std::chrono::steady_clock::now(); };
  auto t0 = now();
  auto lap = [&](const char* what) {
    if (!timing) return;
    const auto t1 = now();
    fprintf(stderr, "[gffplan] %-10s %.3f s\n", what,
            std::chrono::duration<double>(t1 - t0).count());
    t0 = t1;
  };
  try {
    magot::read_gff(P->model, gff, gff_len);
    lap("read_gff");
    magot::Model& M = P->model;
    std::unordered_map<std::string, uint32_t> contig_of;
    for (uint32_t i = 0; i < n_contigs; ++i) contig_of[seqids[i]] = i;  // last duplicate wins
    magot::Lowering L{*P, contig_of, contig_lens, {}, {}};
    L.id_of_feat.assign(M.feats.size(), 0);
    for (uint32_t ti2 = 0; ti2 < M.tables.size(); ++ti2)
      for (uint32_t k : M.tables[ti2].keys) L.id_of_feat[(size_t)M.slot(ti2, k)] = k;
    auto ti = M.table_index.find(feature);
    if (ti == M.table_index.end()) throw Unsupported();  // AttributeError
    const magot::Table& T = M.tables[ti->second];
    std::vector<uint32_t> keys = T.keys;
    if (flags & MAGOT_GFF_ORDER_PY2) {
      std::vector<uint64_t> hash(M.ids.strs.size());
      for (uint32_t k : keys) hash[k] = magot::py2_hash(M.ids.strs[k]);
      keys = magot::py2_dict_order(keys, hash);  // the table as built ...
      keys = magot::py2_dict_order(keys, hash);  // ... and as deep-copied (genome.py:415)
    }
    lap("order");
    // "\n".join(obj.get_fasta() for obj in table.values()): every object adds
    // its records (a blank line when it has none)
    for (size_t i = 0; i < keys.size(); ++i) {
      const uint32_t fi = (uint32_t)M.slot(ti->second, keys[i]);
      if (M.feats[fi].base) throw Unsupported();  // BaseAnnotation has no get_fasta
      if (i) L.text("\n");
      L.fasta(fi, true);
    }
    lap("lower");
  } catch (const Unsupported&) {
    magot::set_error("magot_gff_plan: input takes a diagnostic path; use the object path");
    return MAGOT_ERR_UNSUPPORTED;
  } catch (const std::exception& e) {
    magot::set_error(std::string("magot_gff_plan: ") + e.what());
    return MAGOT_ERR_ARG;
  }
  if (n_exons) *n_exons = P->exons.size();
  if (n_tx) *n_tx = P->txs.size();
  *out = P.release();
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
  uint64_t total = 0;
  for (const auto& pc : p->pieces) {
    if (pc.rec < 0) {
      total += pc.len;
    } else {
      const uint8_t* s;
      uint64_t l;
      payload(p, pc.rec, nuc, noff, pep, poff, &s, &l);
      total += l;
    }
  }
  *out_len = total;
  if (!out) return MAGOT_OK;
  if (cap < total) {
    magot::set_error("magot_gffplan_render: output buffer too small");
    return MAGOT_ERR_ARG;
  }
  uint8_t* o = out;
  for (const auto& pc : p->pieces) {
    if (pc.rec < 0) {
      memcpy(o, p->text.data() + pc.off, pc.len);
      o += pc.len;
    } else {
      const uint8_t* s;
      uint64_t l;
      payload(p, pc.rec, nuc, noff, pep, poff, &s, &l);
      memcpy(o, s, l);
      o += l;
    }
  }
  return MAGOT_OK;
}

void magot_gffplan_destroy(magot_gffplan* p) { delete p; }

}  // extern "C"
