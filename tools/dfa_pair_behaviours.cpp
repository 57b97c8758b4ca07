// dfa_pair_behaviours.cpp -- how many distinct byte-pair behaviours the pair DFA
// has (round 6): a table indexed by (state, pair class) needs a
// code per distinct column (the state after both bytes, the two event bits) over
// every state.  With the 15 byte classes of rhp_dfa.h there are 103, so a 4-byte
// step indexed by two pair codes (103 x 103) cannot fit a u8 code or the LDS.
//   g++ -std=c++17 -O1 -fconstexpr-ops-limit=1000000000 -Ilibreactorng_amd/csrc -Iinclude \
//       tools/dfa_pair_behaviours.cpp -o /tmp/dfa_pair_behaviours && /tmp/dfa_pair_behaviours
#include <stdio.h>
#include <map>
#include <vector>
#include "rhp_dfa.h"
using namespace rhp;
int main()
{
  std::map<std::vector<int>, std::vector<int>> pairs;
  for (uint32_t k0 = 0; k0 < kClasses; k0++)
    for (uint32_t k1 = 0; k1 < kClasses; k1++) {
      std::vector<int> col;
      for (uint32_t s = 0; s < S_COUNT; s++) {
        const uint32_t s1 = step(s, class_rep(k0)), s2 = step(s1, class_rep(k1));
        col.push_back((int) (s2 * 4 + (s1 >= S_NUM_PLAIN) + 2 * (s2 >= S_NUM_PLAIN)));
      }
      pairs[col].push_back((int) (k0 * 16 + k1));
    }
  std::map<std::vector<int>, int> bytes;
  for (uint32_t k = 0; k < kClasses; k++) {
    std::vector<int> col;
    for (uint32_t s = 0; s < S_COUNT; s++) col.push_back((int) step(s, class_rep(k)));
    bytes[col]++;
  }
  printf("states %d, byte classes %d (distinct byte behaviours %zu), distinct pair behaviours %zu of %d\n",
         (int) S_COUNT, (int) kClasses, bytes.size(), pairs.size(), (int) (kClasses * kClasses));
  return 0;
}
