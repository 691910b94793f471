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
#include <cstring>
#include <exception>
#include <memory>
#include <string>
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
  std::vector<uint32_t> keys;                   // IDs in insertion order
  std::unordered_map<uint32_t, uint32_t> slot;  // ID -> feature index
};

struct Unsupported {};  // a diagnostic path of the reference: use the object path

struct Model {
  std::vector<std::string> ids;
  std::unordered_map<std::string, uint32_t> id_index;
  std::vector<uint64_t> id_types;  // bitmask of tables holding the ID (<= 64 tables)
  std::vector<Table> tables;
  std::unordered_map<std::string, uint32_t> table_index;
  std::vector<uint32_t> rank;      // table -> rank in sorted-name order
  std::vector<std::string> seqids, strands;
  std::unordered_map<std::string, uint32_t> seqid_index, strand_index;
  std::vector<Feature> feats;

  Model() {
    // AnnotationSet.__init__ (genome.py:528-533) creates these dicts
    for (const char* t : {"gene", "transcript", "CDS", "UTR"}) table(t);
  }

  uint32_t intern(std::unordered_map<std::string, uint32_t>& idx, std::vector<std::string>& pool,
                  const std::string& s) {
    auto it = idx.find(s);
    if (it != idx.end()) return it->second;
    const uint32_t k = (uint32_t)pool.size();
    pool.push_back(s);
    idx.emplace(s, k);
    return k;
  }
  uint32_t id(const std::string& s) {
    const uint32_t k = intern(id_index, ids, s);
    if (id_types.size() < ids.size()) id_types.resize(ids.size(), 0);
    return k;
  }
  uint32_t table(const std::string& name) {
    auto it = table_index.find(name);
    if (it != table_index.end()) return it->second;
    // attributes of the instance that are not dicts (genome.py:524-545, plus
    // the object path's copy counter) cannot become feature tables
    if (name == "genome" || name == "_magot_copies" || tables.size() >= 64) throw Unsupported();
    const uint32_t k = (uint32_t)tables.size();
    tables.push_back(Table{name, {}, {}});
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
    int best = -1;
    for (uint32_t t = 0; t < tables.size(); ++t)
      if ((m >> t) & 1)
        if (best < 0 || rank[t] > rank[(uint32_t)best]) best = (int)t;
    return tables[(uint32_t)best].slot.at(idk);
  }
  // table[ID] = feature (a dict assignment: an existing key keeps its position)
  void put(uint32_t t, uint32_t idk, uint32_t f) {
    Table& tb = tables[t];
    auto it = tb.slot.find(idk);
    if (it == tb.slot.end()) {
      tb.slot.emplace(idk, f);
      tb.keys.push_back(idk);
      id_types[idk] |= 1ull << t;
    } else {
      it->second = f;
    }
  }
};

// ---------------------------------------------------------------------------
// read_gff (genome.py:242-415) with the default arguments of gff2fasta
// ---------------------------------------------------------------------------

bool is_space(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\v' || c == '\f'; }

std::vector<std::string> split_ws(const std::string& s) {  // str.split()
  std::vector<std::string> out;
  size_t i = 0, n = s.size();
  while (i < n) {
    while (i < n && is_space(s[i])) ++i;
    if (i >= n) break;
    size_t j = i;
    while (j < n && !is_space(s[j])) ++j;
    out.push_back(s.substr(i, j - i));
    i = j;
  }
  return out;
}

std::vector<std::string> split_on(const std::string& s, char c) {  // str.split(c)
  std::vector<std::string> out;
  size_t i = 0;
  for (;;) {
    const size_t j = s.find(c, i);
    if (j == std::string::npos) {
      out.push_back(s.substr(i));
      return out;
    }
    out.push_back(s.substr(i, j - i));
    i = j + 1;
  }
}

// int() of a coordinate column: optional surrounding whitespace and sign,
// decimal digits.  Anything else (ValueError in the reference) -> object path.
int64_t parse_int(const std::string& s) {
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

struct Tags {
  std::vector<std::pair<std::string, std::string>> kv;
  const std::string* get(const std::string& k) const {
    for (auto it = kv.rbegin(); it != kv.rend(); ++it)
      if (it->first == k) return &it->second;
    return nullptr;
  }
  void set(const std::string& k, const std::string& v) {
    for (auto& p : kv)
      if (p.first == k) {
        p.second = v;
        return;
      }
    kv.emplace_back(k, v);
  }
};

void read_gff(Model& M, const char* text, uint64_t n) {
  int version = 0;  // 0 = auto
  bool have_id_field = true, have_parent_field = true;  // IDfield='ID', parent_field='Parent'
  std::vector<std::string> hierarchy;
  std::unordered_map<uint32_t, int64_t> renamed;
  uint64_t pos = 0;
  std::string line;
  while (pos < n) {
    const char* nl = static_cast<const char*>(memchr(text + pos, '\n', n - pos));
    const uint64_t end = nl ? (uint64_t)(nl - text) + 1 : n;
    const char* raw = text + pos;
    const uint64_t rl = end - pos;
    pos = end;
    if (raw[0] == '#') continue;
    uint64_t tabs = 0;
    for (uint64_t i = 0; i < rl; ++i) tabs += raw[i] == '\t';
    if (tabs != 8) continue;
    line.clear();
    for (uint64_t i = 0; i < rl; ++i)
      if (raw[i] != '\n' && raw[i] != '\r') line.push_back(raw[i]);
    const std::vector<std::string> cols = split_on(line, '\t');
    const std::string& tags_text = cols[8];
    if (version == 0) {
      if (tags_text.find('=') != std::string::npos) {
        version = 3;
      } else {
        version = 2;
        std::string spaced = " " + tags_text;
        std::replace(spaced.begin(), spaced.end(), ';', ' ');
        if (have_id_field && hierarchy.empty() && spaced.find(" ID ") == std::string::npos) {
          have_id_field = false;
          have_parent_field = false;
          const bool g = tags_text.find("gene_id") != std::string::npos;
          const bool t = tags_text.find("transcript_id") != std::string::npos;
          if (g && t) hierarchy = {"transcript_id", "gene_id"};
          else if (g) hierarchy = {"gene_id"};
        }
      }
    }
    const std::string& seqid = cols[0];
    const std::string& ftype = cols[2];
    if (ftype == "exon") continue;  // features_to_ignore default
    int64_t lo = parse_int(cols[3]), hi = parse_int(cols[4]);
    if (lo > hi) std::swap(lo, hi);
    const std::string& strand = cols[6];
    Tags tags;
    for (const std::string& item : split_on(tags_text, ';')) {
      if (item.empty()) continue;
      if (version == 2) {
        const std::vector<std::string> words = split_ws(item);
        if (words.empty()) throw Unsupported();  // IndexError
        const size_t q = item.find('"');
        if (q != std::string::npos) {
          const size_t q2 = item.find('"', q + 1);
          tags.set(words[0], item.substr(q + 1, q2 == std::string::npos ? std::string::npos
                                                                         : q2 - q - 1));
        } else if (words.size() > 1) {
          tags.set(words[0], words[1]);
        } else {
          throw Unsupported();  // print(item); return None
        }
      } else {
        const size_t e = item.find('=');
        if (e == std::string::npos) throw Unsupported();  // IndexError
        const size_t e2 = item.find('=', e + 1);
        tags.set(item.substr(0, e),
                 item.substr(e + 1, e2 == std::string::npos ? std::string::npos : e2 - e - 1));
      }
    }
    const std::string* parent = nullptr;
    if (have_parent_field) {
      parent = tags.get("Parent");
    } else {
      for (const std::string& k : hierarchy)
        if ((parent = tags.get(k))) break;
    }
    std::string ID;
    if (have_id_field) {
      if (const std::string* v = tags.get("ID")) ID = *v;
      else if (parent) ID = *parent + "-" + ftype;
      else throw Unsupported();  // ID None
    } else if (parent) {
      ID = *parent + "-" + ftype;
    } else {
      ID = seqid + "-" + ftype + cols[3];
    }
    // de-duplicate against every table; the new name is not re-checked
    {
      const uint32_t k = M.id(ID);
      if (M.lookup(k) >= 0) {
        auto it = renamed.find(k);
        if (it != renamed.end()) {
          it->second += 1;
          ID = ID + "-" + std::to_string(it->second);
        } else {
          renamed.emplace(k, 2);
          ID = ID + "2";
        }
      }
    }
    const uint32_t idk = M.id(ID);
    const uint32_t sq = M.intern(M.seqid_index, M.seqids, seqid);
    const uint32_t st = M.intern(M.strand_index, M.strands, strand);
    if (parent) {
      uint32_t child = idk;
      for (size_t level = 0; level < hierarchy.size(); ++level) {
        const std::string* pid = tags.get(hierarchy[level]);
        if (!pid) continue;
        const std::string ptype = hierarchy[level].substr(0, hierarchy[level].find('_'));
        const uint32_t t = M.table(ptype);
        const uint32_t pk = M.id(*pid);
        auto it = M.tables[t].slot.find(pk);
        if (it != M.tables[t].slot.end()) {
          auto& ch = M.feats[it->second].children;
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
      const int64_t h = M.lookup(M.id(*parent));
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

uint64_t py2_hash(const std::string& s) {
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
        const std::string& sd = M.strands[C.strand];
        if (sd != "+" && sd != "." && sd != "-") throw Unsupported();  // invalid strand: print
        auto ci = contig_of.find(M.seqids[C.seqid]);
        if (ci == contig_of.end()) throw Unsupported();  // missing seqid: print
        magot_exon x;
        uint64_t st, ln;
        slice(C.lo - 1, C.hi, (int64_t)contig_len[ci->second], &st, &ln);
        x.start_rc = st | (sd == "-" ? kRcBit : 0);
        x.contig = ci->second;
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
      if (M.strands[strand] == "-") std::reverse(by.begin(), by.end());
      uint64_t total = 0;
      for (auto& e : by) total += e.second.len;
      if (P.protein && total <= 2) throw Unsupported();  // translate() -> None
      if (!first_in_join) text("\n");
      text(">" + M.ids[idk_of(fi)] + "\n");
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
  try {
    magot::read_gff(P->model, gff, gff_len);
    magot::Model& M = P->model;
    std::unordered_map<std::string, uint32_t> contig_of;
    for (uint32_t i = 0; i < n_contigs; ++i) contig_of[seqids[i]] = i;  // last duplicate wins
    magot::Lowering L{*P, contig_of, contig_lens, {}};
    L.id_of_feat.assign(M.feats.size(), 0);
    for (const magot::Table& t : M.tables)
      for (uint32_t k : t.keys) L.id_of_feat[t.slot.at(k)] = k;
    auto ti = M.table_index.find(feature);
    if (ti == M.table_index.end()) throw Unsupported();  // AttributeError
    const magot::Table& T = M.tables[ti->second];
    std::vector<uint32_t> keys = T.keys;
    if (flags & MAGOT_GFF_ORDER_PY2) {
      std::vector<uint64_t> hash(M.ids.size());
      for (uint32_t k : keys) hash[k] = magot::py2_hash(M.ids[k]);
      keys = magot::py2_dict_order(keys, hash);  // the table as built ...
      keys = magot::py2_dict_order(keys, hash);  // ... and as deep-copied (genome.py:415)
    }
    // "\n".join(obj.get_fasta() for obj in table.values()): every object adds
    // its records (a blank line when it has none)
    for (size_t i = 0; i < keys.size(); ++i) {
      const uint32_t fi = T.slot.at(keys[i]);
      if (M.feats[fi].base) throw Unsupported();  // BaseAnnotation has no get_fasta
      if (i) L.text("\n");
      L.fasta(fi, true);
    }
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
