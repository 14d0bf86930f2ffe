// oracle/ref_isneighbor.cpp -- TEST INFRASTRUCTURE ONLY (never linked into the product).
//
// Runs the reference's own CFindMatch::isNeighbor(lhs, rhs, hunit, threshold) and
// CFindMatch::isNeighborRadius (findMatch.cpp:125-185), compiled unmodified from
// $(REF)/source/pmvs/findMatch.cpp by oracle/Makefile, on patch pairs, so the restatement
// oracle/filter_oracle.h:is_neighbor_h (and through it the device's findNeighbors tests) is pinned
// to reference object code (tests/test_isneighbor_pinning.py).
//
// The two members read only their arguments (no member of CFindMatch), so they are called on storage
// of the class's size that is never constructed: constructing a CFindMatch would run the constructors
// of its organizer / optimizer members, whose TUs (optim.cpp, image.cpp, mylapack.cpp) need nlopt,
// CImg and Eigen and are not built here.  Those unused symbols stay unresolved (the Makefile links
// with --unresolved-symbols=ignore-all and lazy binding); no stand-in is written for any of them.
//
// stdin:  int32 n, then n records of 21 float32: lhs coord[4] normal[4] dscale, rhs coord[4]
//         normal[4] dscale, hunit, threshold, radius
// stdout: n records of 2 int32: isNeighbor(lhs, rhs, hunit, threshold),
//         isNeighborRadius(lhs, rhs, hunit, threshold, radius)
#include <cstdint>
#include <cstdio>
#include <vector>

#include "pmvs/findMatch.hpp"

int main() {
  int32_t n = 0;
  if (std::fread(&n, sizeof(n), 1, stdin) != 1 || n < 0) return 2;
  std::vector<float> in((size_t)n * 21);
  if (n && std::fread(in.data(), sizeof(float), in.size(), stdin) != in.size()) return 2;
  alignas(PMVS3::CFindMatch) static unsigned char raw[sizeof(PMVS3::CFindMatch)];
  const PMVS3::CFindMatch& fm = *reinterpret_cast<const PMVS3::CFindMatch*>(raw);
  std::vector<int32_t> out((size_t)n * 2);
  Patch::CPatch lhs, rhs;
  for (int32_t i = 0; i < n; ++i) {
    const float* r = &in[(size_t)i * 21];
    for (int k = 0; k < 4; ++k) {
      lhs._coord[k] = r[k];
      lhs._normal[k] = r[4 + k];
      rhs._coord[k] = r[9 + k];
      rhs._normal[k] = r[13 + k];
    }
    lhs._dscale = r[8];
    rhs._dscale = r[17];
    out[2 * i] = fm.isNeighbor(lhs, rhs, r[18], r[19]);
    out[2 * i + 1] = fm.isNeighborRadius(lhs, rhs, r[18], r[19], r[20]);
  }
  return std::fwrite(out.data(), sizeof(int32_t), out.size(), stdout) == out.size() ? 0 : 3;
}
