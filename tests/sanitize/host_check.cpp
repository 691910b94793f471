// Host-code sanitizer driver (AddressSanitizer + UndefinedBehaviorSanitizer).
//
// Builds against the HOST translation units of libmagot (pack.cpp,
// gffplan.cpp, fasta.cpp: the code that parses untrusted GFF / FASTA / CDS
// text, with threads and hand-rolled hashing) compiled with
// -fsanitize=address,undefined, and drives every host entry point (FASTA
// reader and packer, gff2fasta and flank planners, cds2pep) over the
// reference's fixture files, the generated parity cases and seeded mutations
// of them.  Built and run by tests/sanitize/run.py; no GPU involved.
//
//   host_check LIST      LIST lines:  fasta PATH | gff GFF FASTA | cds PATH
//
// Exit status 0 = every input processed (ASan/UBSan abort on the first
// finding with a report on stderr); the packer's output is also checked
// against a scalar restatement of the nibble layout (common.h HostPacked).
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "../../magot_amd/csrc/common.h"

namespace magot {
static std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }
}  // namespace magot

using namespace magot;

static int g_failures = 0;
#define CHECK(cond, ...)                                   \
  do {                                                     \
    if (!(cond)) {                                         \
      fprintf(stderr, "CHECK failed %s:%d: ", __FILE__, __LINE__); \
      fprintf(stderr, __VA_ARGS__);                        \
      fprintf(stderr, "\n");                               \
      ++g_failures;                                        \
    }                                                      \
  } while (0)

static std::string slurp(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

// deterministic mutations (xorshift): deletions, insertions of the parsers'
// delimiters, duplications and truncation
struct Rng {
  uint64_t s;
  explicit Rng(uint64_t seed) : s(seed * 0x9E3779B97F4A7C15ull + 1) {}
  uint64_t next() {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    return s;
  }
  uint64_t below(uint64_t n) { return n ? next() % n : 0; }
};

static std::string mutate(const std::string& in, Rng& r) {
  std::string s = in;
  static const char kDelims[] = "\t\n\r;=\" #>.-+0123456789ACGTNacgtn,\x01\xff";
  const int edits = 1 + (int)r.below(8);
  for (int k = 0; k < edits && !s.empty(); ++k) {
    const uint64_t p = r.below(s.size());
    switch (r.below(5)) {
      case 0: s.erase(p, 1 + r.below(16)); break;
      case 1: s.insert(s.begin() + p, kDelims[r.below(sizeof(kDelims) - 1)]); break;
      case 2: s[p] = kDelims[r.below(sizeof(kDelims) - 1)]; break;
      case 3: {
        const uint64_t q = r.below(s.size());
        const uint64_t n = std::min<uint64_t>(1 + r.below(64), s.size() - q);
        s.insert(p, s.substr(q, n));
        break;
      }
      default: s.resize(p); break;
    }
  }
  return s;
}

// --- FASTA: magot_fasta_read (both passes), scan_fasta + pack_genome ---------

struct Genome {
  std::vector<std::string> names;
  std::vector<uint64_t> lens;
  bool ok = false;
};

static uint32_t expect_nibble(uint8_t b) {
  switch (b) {
    case 'A': return 0; case 'C': return 1; case 'G': return 2; case 'T': return 3;
    case 'a': return 4; case 'c': return 5; case 'g': return 6; case 't': return 7;
    default: return 8u | lit_class(b);
  }
}

static void check_pack(const std::vector<ContigSource>& src) {
  HostPacked hp;
  pack_genome(src.data(), (uint32_t)src.size(), &hp);
  CHECK(hp.span % 32 == 0 && hp.nib_words * 8 == hp.span, "span %llu", (unsigned long long)hp.span);
  CHECK(!hp.runs.empty() && hp.runs.back().start == ~0ull, "run sentinel");
  uint64_t total = 0;
  for (size_t i = 0; i < src.size(); ++i) total += src[i].len;
  CHECK(hp.extent == kOrigin + total, "extent");
  // every base's nibble, and every exception byte in exactly one run
  std::vector<uint8_t> bytes;
  size_t run = 0;
  for (size_t i = 0; i < src.size(); ++i) {
    bytes.resize(src[i].len);
    copy_contig(src[i], bytes.data());
    const uint64_t base = hp.contig_base[i];
    for (uint64_t j = 0; j < src[i].len; ++j) {
      const uint64_t g = base + j;
      const uint32_t nib = (hp.nib[g >> 3] >> (4 * (g & 7))) & 15u;
      const uint32_t want = expect_nibble(bytes[j]);
      if (nib != want) {
        CHECK(false, "contig %zu base %llu byte %u: nibble %u want %u", i, (unsigned long long)j,
              bytes[j], nib, want);
        return;
      }
      if (want & 8u) {
        while (run < hp.runs.size() && hp.runs[run].start + hp.runs[run].len <= g) ++run;
        CHECK(run < hp.runs.size() && hp.runs[run].start <= g && hp.runs[run].byte == bytes[j],
              "exception byte at %llu not in its run", (unsigned long long)g);
      }
    }
  }
  for (uint64_t g = hp.extent; g < hp.span; ++g)
    CHECK(((hp.nib[g >> 3] >> (4 * (g & 7))) & 15u) == 0, "padding nibble at %llu",
          (unsigned long long)g);
  for (uint64_t g = 0; g < kOrigin && g < hp.span; ++g)  // the leading pad too
    CHECK(((hp.nib[g >> 3] >> (4 * (g & 7))) & 15u) == 0, "leading pad nibble at %llu",
          (unsigned long long)g);
  // directory: first run whose end lies past the block start
  for (size_t b = 0; b < hp.dir.size(); ++b) {
    const uint64_t bs = (uint64_t)b << kDirShift;
    const uint32_t d = hp.dir[b] & ~kDirClean;
    CHECK(d < hp.runs.size(), "dir index");
    if (d < hp.runs.size() - 1) CHECK(hp.runs[d].start + hp.runs[d].len > bs, "dir run ends before block");
    if (d > 0) CHECK(hp.runs[d - 1].start + hp.runs[d - 1].len <= bs, "dir skips a run");
  }
}

static Genome do_fasta(const std::string& text, bool pack) {
  Genome g;
  for (int trunc = 0; trunc < 2; ++trunc) {
    uint32_t n = 0;
    uint64_t nl = 0;
    int rc = magot_fasta_read(text.data(), text.size(), trunc, &n, nullptr, nullptr, 0, &nl,
                              nullptr, 0);
    if (rc) continue;
    std::vector<uint64_t> lens(n ? n : 1);
    std::vector<char> names(nl ? nl : 1);
    rc = magot_fasta_read(text.data(), text.size(), trunc, &n, lens.data(), names.data(), nl, &nl,
                          nullptr, 0);
    CHECK(rc == 0, "fasta pass 2: %s", g_err.c_str());
    uint64_t tot = 0;
    for (uint32_t i = 0; i < n; ++i) tot += lens[i];
    std::vector<uint8_t> seqs(tot ? tot : 1);
    rc = magot_fasta_read(text.data(), text.size(), trunc, &n, lens.data(), names.data(), nl, &nl,
                          seqs.data(), seqs.size());
    CHECK(rc == 0, "fasta pass 3: %s", g_err.c_str());
    if (rc) continue;
    // a buffer one byte short must be refused, not overrun
    if (tot > 0) {
      std::vector<uint8_t> shortbuf(tot - 1 ? tot - 1 : 1);
      rc = magot_fasta_read(text.data(), text.size(), trunc, &n, lens.data(), names.data(), nl,
                            &nl, shortbuf.data(), tot - 1);
      CHECK(rc != 0, "short sequence buffer accepted");
    }
    if (!trunc) {
      g.ok = true;
      g.lens.assign(lens.begin(), lens.begin() + n);
      const char* p = names.data();
      for (uint32_t i = 0; i < n; ++i) {
        g.names.emplace_back(p);
        p += g.names.back().size() + 1;
      }
    }
    if (pack) {
      FastaContigs fc;
      if (scan_fasta(text.data(), text.size(), trunc != 0, &fc) == 0) {
        check_pack(fc.src);
        // the same bytes contiguous
        std::vector<std::vector<uint8_t>> flat(fc.src.size());
        std::vector<ContigSource> src(fc.src.size());
        for (size_t i = 0; i < fc.src.size(); ++i) {
          flat[i].resize(fc.src[i].len);
          copy_contig(fc.src[i], flat[i].data());
          src[i] = ContigSource{flat[i].data(), fc.src[i].len, 0, 0};
        }
        check_pack(src);
      }
    }
  }
  return g;
}

// --- GFF: magot_gff_plan under every flag combination, tables, render --------

// tables, selections, render (sized, exact, one byte short) and the device
// text units of one plan; destroys it
static void check_plan(magot_gffplan* p, uint64_t ne, uint64_t nt) {
  std::vector<magot_exon> ex(ne ? ne : 1);
  std::vector<magot_tx> tx(nt ? nt : 1);
  CHECK(magot_gffplan_tables(p, ex.data(), tx.data()) == 0, "tables");
  uint64_t groups = 0;
  CHECK(magot_gffplan_selections(p, &groups) == 0, "selections");
  // payloads of the right sizes (nucleotide 'a'.., untrimmed peptide 'X'/'M')
  std::vector<uint64_t> noff(nt + 1, 0), poff(nt + 1, 0);
  for (uint64_t t = 0; t < nt; ++t) {
    uint64_t len = 0;
    CHECK(tx[t].exon_begin + tx[t].n_exons <= ne, "record %llu exons out of range",
          (unsigned long long)t);
    for (uint64_t e = tx[t].exon_begin; e < tx[t].exon_begin + tx[t].n_exons && e < ne; ++e)
      len += ex[e].len;
    noff[t + 1] = noff[t] + len;
    poff[t + 1] = poff[t] + len / 3;
  }
  std::vector<uint8_t> nuc(noff[nt] + 1, 'a'), pep(poff[nt] + 1, 'M');
  for (uint64_t t = 0; t < nt; ++t)
    if (poff[t + 1] > poff[t] && (t & 1)) pep[poff[t]] = 'X';
  uint64_t sz = 0;
  int r2 = magot_gffplan_render(p, nuc.data(), noff.data(), pep.data(), poff.data(), nullptr, 0,
                                &sz);
  CHECK(r2 == 0, "render size: %s", g_err.c_str());
  if (r2 == 0) {
    std::vector<uint8_t> out(sz + 1);
    r2 = magot_gffplan_render(p, nuc.data(), noff.data(), pep.data(), poff.data(), out.data(),
                              sz, &sz);
    CHECK(r2 == 0, "render: %s", g_err.c_str());
    if (sz > 0) {
      // one byte short: refused, not overrun
      std::vector<uint8_t> small(sz - 1 ? sz - 1 : 1);
      r2 = magot_gffplan_render(p, nuc.data(), noff.data(), pep.data(), poff.data(),
                                small.data(), sz - 1, &sz);
      CHECK(r2 != 0, "short render buffer accepted");
    }
  }
  const std::string* text = nullptr;
  std::vector<TextUnit> units;
  bool protein = false;
  uint64_t n_rec = 0;
  if (gffplan_units(p, &text, &units, &protein, &n_rec)) {
    for (const TextUnit& u : units) {
      CHECK(u.text_off + u.text_len <= text->size(), "unit text range");
      CHECK(u.rec == kNoRecord || u.rec < n_rec, "unit record");
    }
  }
  magot_gffplan_destroy(p);
}

static int do_gff(const std::string& gff, const Genome& g, bool full) {
  std::vector<const char*> ids;
  for (auto& s : g.names) ids.push_back(s.c_str());
  int planned = 0;
  const uint32_t max_flags = full ? 32 : 4;
  for (uint32_t flags = 0; flags < max_flags; ++flags) {
    for (const char* feature : {"gene", "mRNA"}) {
      if (!full && feature[0] == 'm') continue;
      magot_gffplan* p = nullptr;
      uint64_t ne = 0, nt = 0;
      const int rc = magot_gff_plan(gff.data(), gff.size(), ids.data(), g.lens.data(),
                                    (uint32_t)ids.size(), feature, flags, &p, &ne, &nt);
      if (rc) {
        CHECK(p == nullptr, "plan handle on failure");
        continue;
      }
      ++planned;
      check_plan(p, ne, nt);
    }
  }
  return planned;
}

// --- extract_upstream_downstream: magot_flank_plan ---------------------------

static int do_flank(const std::string& gff, const Genome& g, bool full) {
  std::vector<const char*> ids;
  for (auto& s : g.names) ids.push_back(s.c_str());
  int planned = 0;
  static const char* kLengths[] = {"0", "1", "7", "100", " 3 ", "-2", "+5", "x", "99999999999"};
  static const char* kNames[] = {"ID", "Name", "Parent", ""};
  for (const char* len : kLengths) {
    for (const char* stream : {"up", "down", "sideways"}) {
      for (const char* ftype : {"gene", "CDS", "mRNA"}) {
        for (const char* namefrom : kNames) {
          if (!full && (ftype[0] != 'g' || namefrom[0] != 'I')) continue;
          magot_gffplan* p = nullptr;
          uint64_t ne = 0, nt = 0;
          const int rc = magot_flank_plan(gff.data(), gff.size(), ids.data(), g.lens.data(),
                                          (uint32_t)ids.size(), ftype, namefrom, len, stream, &p,
                                          &ne, &nt);
          if (rc) {
            CHECK(p == nullptr, "flank plan handle on failure");
            continue;
          }
          ++planned;
          CHECK(ne == nt, "flank: one interval per record (%llu vs %llu)",
                (unsigned long long)ne, (unsigned long long)nt);
          check_plan(p, ne, nt);
        }
      }
    }
  }
  return planned;
}

// --- cds2pep: magot_cds_scan + magot_cds_render --------------------------------

static void do_cds(const std::string& text) {
  uint64_t nseg = 0, sb = 0;
  int rc = magot_cds_scan(text.data(), text.size(), &nseg, &sb, nullptr, nullptr, nullptr, nullptr,
                          0);
  if (rc) return;
  std::vector<uint64_t> seg(nseg + 1), ho(nseg ? nseg : 1), hl(nseg ? nseg : 1);
  std::vector<uint8_t> seq(sb + 1);
  rc = magot_cds_scan(text.data(), text.size(), &nseg, &sb, seg.data(), ho.data(), hl.data(),
                      seq.data(), sb);
  CHECK(rc == 0, "cds scan: %s", g_err.c_str());
  if (rc) return;
  if (sb > 0) {
    std::vector<uint8_t> small(sb);
    uint64_t n2 = nseg, s2 = sb;
    CHECK(magot_cds_scan(text.data(), text.size(), &n2, &s2, seg.data(), ho.data(), hl.data(),
                         small.data(), sb - 1) != 0, "short cds buffer accepted");
  }
  // translations of the segments: frame-0 residues or None (codons < 0)
  std::vector<uint64_t> poff(nseg + 2, 0);
  std::vector<int64_t> codons(nseg + 1);
  for (uint64_t k = 0; k <= nseg; ++k) {
    const uint64_t len = seg[k + 1 < seg.size() ? k + 1 : k] - seg[k];
    codons[k] = len <= 2 ? -1 : (int64_t)(len / 3);
    poff[k + 1] = poff[k] + (codons[k] < 0 ? 0 : (uint64_t)codons[k]);
  }
  std::vector<uint8_t> pep(poff[nseg + 1] + 1, 'K');
  uint64_t sz = 0;
  rc = magot_cds_render(text.data(), nseg, seg.data(), ho.data(), hl.data(), pep.data(),
                        poff.data(), codons.data(), nullptr, 0, &sz);
  CHECK(rc == 0, "cds render size: %s", g_err.c_str());
  if (rc) return;
  std::vector<uint8_t> out(sz + 1);
  rc = magot_cds_render(text.data(), nseg, seg.data(), ho.data(), hl.data(), pep.data(),
                        poff.data(), codons.data(), out.data(), sz, &sz);
  CHECK(rc == 0, "cds render: %s", g_err.c_str());
}

// --- synthetic genomes for the packer: every byte value, block edges ----------

static void synthetic_packs() {
  Rng r(7);
  const uint64_t sizes[] = {0, 1, 7, 8, 31, 32, 33, 63, 64, 65, 4095, 4096, 4097, 8191, 70000};
  for (int trial = 0; trial < 40; ++trial) {
    const int nc = 1 + (int)r.below(6);
    std::vector<std::vector<uint8_t>> data(nc);
    std::vector<ContigSource> src(nc);
    for (int c = 0; c < nc; ++c) {
      const uint64_t n = sizes[r.below(sizeof(sizes) / sizeof(sizes[0]))] + r.below(3);
      data[c].resize(n);
      const int mode = (int)r.below(4);
      for (uint64_t j = 0; j < n; ++j) {
        uint8_t b = "ACGTacgt"[r.below(8)];
        if (mode == 1 && r.below(50) == 0) b = (uint8_t)r.below(256);
        if (mode == 2 && (j / 37) % 3 == 0) b = 'N';
        if (mode == 3) b = (uint8_t)r.below(256);
        data[c][j] = b;
      }
      src[c] = ContigSource{n ? data[c].data() : nullptr, n, 0, 0};
    }
    check_pack(src);
  }
  // a long run across many directory blocks and piece boundaries
  std::vector<uint8_t> big(3u << 22, 'A');
  for (size_t j = 100000; j < 100000 + 3 * 4096 + 17; ++j) big[j] = 'n';
  for (size_t j = (1u << 22) - 5; j < (1u << 22) + 5; ++j) big[j] = 'R';
  ContigSource one{big.data(), big.size(), 0, 0};
  check_pack(std::vector<ContigSource>{one});
}

// magot_plan_create's genome-order layout: radix_order against std::stable_sort
// (empty, one record, equal keys, small / wide / sparse key ranges)
static void synthetic_orders() {
  Rng rng(7);
  const uint64_t sizes[] = {0, 1, 2, 17, 4096, 100003};
  const uint64_t ranges[] = {1, 3, 2048, 2049, 1ull << 22, 1ull << 40, ~0ull};
  for (uint64_t n : sizes)
    for (uint64_t range : ranges) {
      std::vector<uint64_t> key(n);
      for (uint64_t i = 0; i < n; ++i) key[i] = range == ~0ull ? rng.next() : rng.below(range);
      std::vector<uint32_t> got;
      radix_order(key, &got);
      std::vector<uint32_t> want(n);
      for (uint64_t i = 0; i < n; ++i) want[i] = (uint32_t)i;
      std::stable_sort(want.begin(), want.end(),
                       [&](uint32_t a, uint32_t b) { return key[a] < key[b]; });
      CHECK(got == want, "radix_order n=%llu range=%llu differs from stable_sort",
            (unsigned long long)n, (unsigned long long)range);
    }
}

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: host_check LIST [mutations]\n");
    return 2;
  }
  const int n_mut = argc > 2 ? atoi(argv[2]) : 20;
  std::ifstream list(argv[1]);
  std::string line;
  int n_fa = 0, n_gff = 0, n_cds = 0, planned = 0, flanks = 0, n_mutated = 0;
  Rng rng(20261017);
  while (std::getline(list, line)) {
    std::istringstream ls(line);
    std::string kind, a, b;
    ls >> kind >> a >> b;
    if (kind == "fasta") {
      const std::string t = slurp(a);
      do_fasta(t, true);
      for (int k = 0; k < n_mut; ++k) do_fasta(mutate(t, rng), k < 4);
      ++n_fa;
    } else if (kind == "gff") {
      const Genome g = do_fasta(slurp(b), false);
      if (!g.ok) continue;
      const std::string t = slurp(a);
      for (const char* chunks : {"1", "2", "7", "64"}) {
        setenv("MAGOT_GFF_CHUNKS", chunks, 1);
        planned += do_gff(t, g, chunks[0] == '1');
      }
      for (const char* chunks : {"1", "5"}) {
        setenv("MAGOT_GFF_CHUNKS", chunks, 1);
        flanks += do_flank(t, g, chunks[0] == '1');
      }
      setenv("MAGOT_GFF_CHUNKS", "3", 1);
      for (int k = 0; k < n_mut; ++k) {
        const std::string m = mutate(t, rng);
        do_gff(m, g, false);
        if (k < 8) do_flank(m, g, false);
        ++n_mutated;
      }
      unsetenv("MAGOT_GFF_CHUNKS");
      ++n_gff;
    } else if (kind == "cds") {
      const std::string t = slurp(a);
      do_cds(t);
      for (int k = 0; k < n_mut; ++k) do_cds(mutate(t, rng));
      ++n_cds;
    }
  }
  synthetic_packs();
  synthetic_orders();
  printf("host_check: %d fasta, %d gff (%d plans, %d flank plans, %d mutated gff), %d cds "
         "inputs; %d check failure(s)\n", n_fa, n_gff, planned, flanks, n_mutated, n_cds,
         g_failures);
  return g_failures ? 1 : 0;
}
