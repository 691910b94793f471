/*
 * CPU ORACLE (C restatement) of MAGOT's per-record extraction -- TEST
 * INFRASTRUCTURE ONLY.  Used by tests/ and bench.py to check the HIP path at
 * sizes where the pure-Python oracle (magot_oracle.py) is too slow.  Never
 * linked into libmagot.so.
 *
 * Restates, for one record whose children are all BaseAnnotations:
 *   ParentAnnotation.get_fasta  genome.py:686-710  child_dict keyed by coords
 *                               (last duplicate wins), keys sorted, reversed
 *                               when the LAST child's strand is '-', joined;
 *                               protein => translate()
 *   BaseAnnotation.get_seq      genome.py:603-614  contig[c0-1:c1] (Python
 *                               slice rules), '-' => reverse complement,
 *                               other strands / missing contig => None
 *   Sequence.reverse_compliment genome.py:784-793
 *   Sequence.translate          genome.py:795-822  frame 0, trimX
 * and, per record sequence (oracle_orf6_compare):
 *   Sequence.get_orfs           genome.py:824-851  translate(frame, strand)
 *                               for frame 0,1,2 x strand '-','+' (any frame,
 *                               either strand, trimX, None when len <= 2+frame)
 *
 * Build: gcc -O2 -shared -fPIC -o oracle/build/libcds_oracle.so oracle/cds_oracle.c
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

enum { ST_OK = 0, ST_NONE_PIECE = 1, ST_TRANSLATE_NONE = 2 };

static unsigned char rc_map[256];
static signed char code_map[256];
static const char *AA_TCAG = "FFLLSSSSYY**CC*WLLLLPPPPHHQQRRRRIIIMTTTTNNKKSSRRVVVVAAAADDEEGGGG";
static char aa_tab[64]; /* index 16*b0 + 4*b1 + b2 with T=0 C=1 A=2 G=3 */
static int ready = 0;

static void init_tables(void) {
  if (ready) return;
  for (int i = 0; i < 256; ++i) {
    rc_map[i] = 'n';
    code_map[i] = -1;
  }
  rc_map['a'] = 't'; rc_map['t'] = 'a'; rc_map['g'] = 'c'; rc_map['c'] = 'g';
  rc_map['A'] = 'T'; rc_map['T'] = 'A'; rc_map['G'] = 'C'; rc_map['C'] = 'G';
  rc_map['n'] = 'n'; rc_map['N'] = 'N'; rc_map['-'] = '-';
  /* upper-case triplets only: the reference upper()s every residue */
  code_map['T'] = 0; code_map['C'] = 1; code_map['A'] = 2; code_map['G'] = 3;
  code_map['t'] = 0; code_map['c'] = 1; code_map['a'] = 2; code_map['g'] = 3;
  for (int i = 0; i < 64; ++i) aa_tab[i] = AA_TCAG[i];
  ready = 1;
}

static void py_slice(int64_t n, int64_t a, int64_t b, int64_t *start, int64_t *len) {
  if (a < 0) { a += n; if (a < 0) a = 0; } else if (a > n) a = n;
  if (b < 0) { b += n; if (b < 0) b = 0; } else if (b > n) b = n;
  *start = a;
  *len = b > a ? b - a : 0;
}

typedef struct { int64_t c0, c1; int64_t idx; } key_t_;

static int cmp_key(const void *x, const void *y) {
  const key_t_ *a = (const key_t_ *)x, *b = (const key_t_ *)y;
  if (a->c0 != b->c0) return a->c0 < b->c0 ? -1 : 1;
  if (a->c1 != b->c1) return a->c1 < b->c1 ? -1 : 1;
  return a->idx < b->idx ? -1 : (a->idx > b->idx);
}

/*
 * genome: all contig bytes back to back, contig i = genome[coff[i]..coff[i+1])
 * record r owns children [roff[r], roff[r+1]); child k: contig ck[k] (-1 =
 * seqid not in the FASTA), sorted coords c0[k] <= c1[k] (genome.py:309-311),
 * strand sk[k] (raw byte).  protein = 0/1.
 * out receives each record's sequence back to back (caller sizes it as the
 * sum of child slice lengths), ooff[r..r+1] its extent, status[r] a code.
 * Returns total bytes written.
 */
int64_t oracle_extract(const unsigned char *genome, const int64_t *coff, int64_t n_contigs,
                       int64_t n_rec, const int64_t *roff, const int32_t *ck, const int64_t *c0,
                       const int64_t *c1, const unsigned char *sk, int protein,
                       unsigned char *out, int64_t *ooff, int32_t *status) {
  init_tables();
  int64_t w = 0;
  int64_t cap = 64;
  key_t_ *keys = (key_t_ *)malloc(sizeof(key_t_) * cap);
  unsigned char *tmp = NULL;
  int64_t tmp_cap = 0;
  for (int64_t r = 0; r < n_rec; ++r) {
    const int64_t kb = roff[r], ke = roff[r + 1], nk = ke - kb;
    ooff[r] = w;
    status[r] = ST_OK;
    if (nk > cap) {
      cap = nk * 2;
      keys = (key_t_ *)realloc(keys, sizeof(key_t_) * cap);
    }
    for (int64_t k = 0; k < nk; ++k) {
      keys[k].c0 = c0[kb + k];
      keys[k].c1 = c1[kb + k];
      keys[k].idx = kb + k;
    }
    qsort(keys, (size_t)nk, sizeof(key_t_), cmp_key);
    /* collapse duplicates: last child (largest idx) wins */
    int64_t m = 0;
    for (int64_t k = 0; k < nk; ++k) {
      if (m > 0 && keys[m - 1].c0 == keys[k].c0 && keys[m - 1].c1 == keys[k].c1) keys[m - 1] = keys[k];
      else keys[m++] = keys[k];
    }
    const int reverse = nk > 0 && sk[ke - 1] == '-';
    int64_t total = 0;
    for (int64_t q = 0; q < m; ++q) {
      const int64_t i = keys[reverse ? m - 1 - q : q].idx;
      const unsigned char s = sk[i];
      if (ck[i] < 0 || ck[i] >= n_contigs || !(s == '+' || s == '.' || s == '-')) {
        status[r] = ST_NONE_PIECE;
        continue;
      }
      const unsigned char *ctg = genome + coff[ck[i]];
      int64_t st, ln;
      py_slice(coff[ck[i] + 1] - coff[ck[i]], c0[i] - 1, c1[i], &st, &ln);
      if (total + ln > tmp_cap) {
        tmp_cap = (total + ln) * 2 + 64;
        tmp = (unsigned char *)realloc(tmp, (size_t)tmp_cap);
      }
      if (s == '-') {
        for (int64_t j = 0; j < ln; ++j) tmp[total + j] = rc_map[ctg[st + ln - 1 - j]];
      } else {
        memcpy(tmp + total, ctg + st, (size_t)ln);
      }
      total += ln;
    }
    if (status[r] != ST_OK) continue;
    if (!protein) {
      if (total) memcpy(out + w, tmp, (size_t)total);
      w += total;
      continue;
    }
    if (total <= 2) {
      status[r] = ST_TRANSLATE_NONE;
      continue;
    }
    const int64_t start_w = w;
    for (int64_t p = 0; p + 2 < total; p += 3) {
      const int a = code_map[tmp[p]], b = code_map[tmp[p + 1]], c = code_map[tmp[p + 2]];
      out[w++] = (a < 0 || b < 0 || c < 0) ? 'X' : (unsigned char)aa_tab[16 * a + 4 * b + c];
    }
    if (w > start_w && out[start_w] == 'X') {
      memmove(out + start_w, out + start_w + 1, (size_t)(w - start_w - 1));
      --w;
    }
  }
  ooff[n_rec] = w;
  free(keys);
  free(tmp);
  return w;
}

/*
 * Sequence.translate (genome.py:795-822), literally: strand '-' reverse-
 * complements first (:805-808); None (returns -1) unless len > 2 + frame
 * (:809); for p in range(frame, len) the upper()ed residue joins the triplet
 * and a codon is emitted when (p + frame) % 3 == 2 (:810-812), looked up in
 * the standard code, 'X' for anything else -- a junk 1- or 2-char triplet, or
 * one with a non-ACGT base (:813-816); trimX drops one leading 'X' (:819-821).
 * tmp holds len bytes (the reverse complement).  Returns residues written.
 */
static int64_t translate_ref(const unsigned char *seq, int64_t len, int frame, int minus,
                             unsigned char *tmp, unsigned char *out) {
  if (!(len > 2 + frame)) return -1;
  const unsigned char *s = seq;
  if (minus) {
    for (int64_t j = 0; j < len; ++j) tmp[j] = rc_map[seq[len - 1 - j]];
    s = tmp;
  }
  int64_t w = 0;
  int n = 0;
  int code[3];
  for (int64_t p = frame; p < len; ++p) {
    if (n < 3) code[n] = code_map[s[p]];
    ++n;
    if ((p + frame) % 3 == 2) {
      out[w++] = (n == 3 && code[0] >= 0 && code[1] >= 0 && code[2] >= 0)
                     ? (unsigned char)aa_tab[16 * code[0] + 4 * code[1] + code[2]] : 'X';
      n = 0;
    }
  }
  if (w > 0 && out[0] == 'X') {
    memmove(out, out + 1, (size_t)(w - 1));
    --w;
  }
  return w;
}

/*
 * Check six-frame device output against translate_ref for records
 * [r0, r1) of n: record r is seq[seq_off[r] .. seq_off[r+1]).  Device stream
 * j = 6r + 2f + (strand == '+') holds the residues at dev[stream_off[j] ..
 * + stream_len[j]) in the layout of include/magot.h (magot_orf6_*): frames 1/2
 * without their junk first codon, frame 0 untrimmed (one leading 'X' is
 * dropped here before comparing), length 0 where the reference returns None.
 * Returns the number of mismatching streams; *first_bad = the first one (or -1),
 * and the first bad_cap of them in bad_list (may be NULL).
 */
int64_t oracle_orf6_compare(const unsigned char *seq, const int64_t *seq_off, int64_t r0,
                            int64_t r1, const unsigned char *dev, const uint64_t *stream_off,
                            const uint64_t *stream_len, int64_t *first_bad, int64_t *bad_list,
                            int64_t bad_cap) {
  init_tables();
  int64_t bad = 0;
  *first_bad = -1;
  int64_t cap = 0;
  unsigned char *tmp = NULL, *ref = NULL;
  for (int64_t r = r0; r < r1; ++r) {
    const int64_t len = seq_off[r + 1] - seq_off[r];
    if (len + 16 > cap) {
      cap = 2 * len + 64;
      tmp = (unsigned char *)realloc(tmp, (size_t)cap);
      ref = (unsigned char *)realloc(ref, (size_t)cap);
    }
    for (int f = 0; f < 3; ++f) {
      for (int plus = 0; plus < 2; ++plus) {
        const int64_t j = 6 * r + 2 * f + plus;
        const int64_t n = translate_ref(seq + seq_off[r], len, f, !plus, tmp, ref);
        const unsigned char *g = dev + stream_off[j];
        int64_t gl = (int64_t)stream_len[j];
        if (f == 0 && gl > 0 && g[0] == 'X') { ++g; --gl; }
        const int ok = n < 0 ? stream_len[j] == 0
                             : (gl == n && (n == 0 || memcmp(g, ref, (size_t)n) == 0));
        if (!ok) {
          if (*first_bad < 0) *first_bad = j;
          if (bad_list && bad < bad_cap) bad_list[bad] = j;
          ++bad;
        }
      }
    }
  }
  free(tmp);
  free(ref);
  return bad;
}
