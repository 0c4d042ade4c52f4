#include "transcript.hpp"
#include <cstdio>
#include <cstring>
#include <vector>
#include <random>
using namespace lcpc;
int main() {
  std::mt19937_64 rng(1);
  int bad = 0;
  for (size_t ml : {8, 16, 24, 32, 3, 17}) {
    for (size_t ln : {6, 2, 9}) {
      for (size_t pre = 0; pre < 200; pre += 7) {
        for (size_t n : {0, 1, 5, 37, 300}) {
          std::vector<uint8_t> lab(ln), pre_msg(pre), msgs(n * ml);
          for (auto &b : lab) b = rng();
          for (auto &b : pre_msg) b = rng();
          for (auto &b : msgs) b = rng();
          Transcript a((const uint8_t *)"x", 1), b((const uint8_t *)"x", 1);
          a.append_message((const uint8_t *)"p", 1, pre_msg.data(), pre);
          b.append_message((const uint8_t *)"p", 1, pre_msg.data(), pre);
          a.append_messages(lab.data(), ln, msgs.data(), ml, n);
          for (size_t i = 0; i < n; i++) b.append_message(lab.data(), ln, msgs.data() + i * ml, ml);
          uint8_t da[64], db[64];
          a.challenge_bytes((const uint8_t *)"c", 1, da, 64);
          b.challenge_bytes((const uint8_t *)"c", 1, db, 64);
          if (std::memcmp(da, db, 64)) bad++;
        }
      }
    }
  }
  printf("impl %s mismatches %d\n", keccak_impl(), bad);
  return bad != 0;
}
