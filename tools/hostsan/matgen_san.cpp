#include "sdig.hpp"
#include "field_params.hpp"
#include <cstdio>
using namespace lcpc;
int main() {
  uint64_t p[2];
  for (int i = 0; i < 2; i++) p[i] = (uint64_t)Ft127::P[2 * i] | ((uint64_t)Ft127::P[2 * i + 1] << 32);
  int bad = 0;
  for (int code = 1; code <= 6; code++)
    for (size_t n : {64, 4096, 70001}) {
      std::vector<CsrHost> pre, post;
      if (!sdig_generate(2, 127, p, code, n, 3, pre, post)) { printf("code %d n %zu: no levels\n", code, n); continue; }
      for (auto *v : {&pre, &post})
        for (auto &m : *v) {
          if (m.ptr.size() != m.rows + 1 || m.ptr.back() != m.idx.size() || m.val.size() != 2 * m.idx.size()) bad++;
          for (size_t r = 0; r < m.rows; r++) if (m.ptr[r] > m.ptr[r + 1]) bad++;
          for (auto i : m.idx) if (i >= m.cols) bad++;
        }
      printf("code %d n %zu levels %zu cw %zu\n", code, n, pre.size(), sdig_codeword_length(pre, post));
    }
  printf("bad %d\n", bad);
  return bad != 0;
}
