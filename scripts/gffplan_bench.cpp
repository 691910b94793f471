// Host-only timing of the native gff2fasta planner (magot_gff_plan) on a GFF
// file: the reference's read_gff + get_fasta lowering, no device.  Built by
// scripts/gffplan_ab.sh against two versions of gffplan.cpp for an A/B.
//
//   gffplan_bench GFF CONTIGS REPS      CONTIGS lines: "name length"
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "magot.h"

namespace magot {
void set_error(const std::string& msg) { fprintf(stderr, "error: %s\n", msg.c_str()); }
}  // namespace magot

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: gffplan_bench GFF CONTIGS [REPS]\n");
    return 2;
  }
  std::ifstream f(argv[1], std::ios::binary);
  std::stringstream ss;
  ss << f.rdbuf();
  const std::string gff = ss.str();
  std::ifstream c(argv[2]);
  std::vector<std::string> names;
  std::vector<uint64_t> lens;
  std::string n;
  uint64_t l;
  while (c >> n >> l) {
    names.push_back(n);
    lens.push_back(l);
  }
  std::vector<const char*> np;
  for (auto& s : names) np.push_back(s.c_str());
  const int reps = argc > 3 ? atoi(argv[3]) : 1;
  for (int r = 0; r < reps; ++r) {
    const auto t = std::chrono::steady_clock::now();
    magot_gffplan* p = nullptr;
    uint64_t ne = 0, nt = 0;
    const int rc = magot_gff_plan(gff.data(), gff.size(), np.data(), lens.data(),
                                  (uint32_t)np.size(), "gene",
                                  MAGOT_GFF_PROTEIN | MAGOT_GFF_ORDER_PY2, &p, &ne, &nt);
    const double s =
        std::chrono::duration<double>(std::chrono::steady_clock::now() - t).count();
    printf("rc %d exons %llu records %llu plan_s %.4f\n", rc, (unsigned long long)ne,
           (unsigned long long)nt, s);
    if (p) magot_gffplan_destroy(p);
  }
  return 0;
}
