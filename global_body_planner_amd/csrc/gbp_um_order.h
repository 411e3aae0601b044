// gbp_um_order.h — the iteration order of the reference's vertex map.
//
// GraphClass keeps a tree's vertices in a std::unordered_map<int, State>
// (graph_class.h:155) filled by addVertex with keys 0, 1, 2, ... and never
// erased from (graph_class.cpp:28-31, :141-145).  PlannerClass::neighborhoodDist
// walks it begin() to end() (planner_class.cpp:176-179), and RRT*'s
// choose-parent and rewire loops consume the neighbours in that order
// (rrt_star_connect.cpp:31-44, :51-64): a choose-parent tie goes to the first,
// and a rewire lowers the g of a whole subtree that a later neighbour's test
// then reads.  So the engine lists neighbours in the map's order, not by index.
//
// libstdc++ (this image's GCC 11.4) keeps one singly linked node list: a key
// whose bucket is empty is linked at the front, and a rehash relinks the nodes
// in list order, each at the front of the new list (it reverses the list).
// With int keys hashed to themselves and load factor <= 1, every key below the
// bucket count has a bucket of its own, so keys 0..n-1 iterate as
//     order(n) = [n-1, n-2, ..., r] ++ reverse(order(r)),
// r the last rehash point <= n-1 (the element counts at which
// _Prime_rehash_policy grows the table).  Equivalently the key at position p:
//     key(p, n) = p < n - r ? n-1-p : key(n-1-p, r)
// and the position of key k:
//     rank(k, n) = k >= r ? n-1-k : n-1-rank(k, r).
// tests/test_um_order.py checks both against a real std::unordered_map.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define GBP_UM_HD __host__ __device__
#else
#define GBP_UM_HD
#endif

namespace gbp {

// the element counts at which inserting one more key rehashes (libstdc++
// _Prime_rehash_policy with max_load_factor 1: the first insertion into the
// single-bucket empty map, then each bucket count from __prime_list)
constexpr int GBP_UM_NREHASH = 28;
GBP_UM_HD inline int64_t um_rehash_point(int i) {
  // a switch keeps the table in the instruction stream on the device (no
  // scratch copy of a local array, no device global to initialise)
  switch (i) {
    case 0: return 0;
    case 1: return 13;
    case 2: return 29;
    case 3: return 59;
    case 4: return 127;
    case 5: return 257;
    case 6: return 541;
    case 7: return 1109;
    case 8: return 2357;
    case 9: return 5087;
    case 10: return 10273;
    case 11: return 20753;
    case 12: return 42043;
    case 13: return 85229;
    case 14: return 172933;
    case 15: return 351061;
    case 16: return 712697;
    case 17: return 1447153;
    case 18: return 2938679;
    case 19: return 5967347;
    case 20: return 12117689;
    case 21: return 24607243;
    case 22: return 49969847;
    case 23: return 101473717;
    case 24: return 206062531;
    case 25: return 418451333;
    case 26: return 849749479;
    default: return 1725587117;
  }
}

// index of the last rehash point <= n - 1 (n >= 1)
GBP_UM_HD inline int um_epoch(int64_t n) {
  int m = 0;
  while (m + 1 < GBP_UM_NREHASH && um_rehash_point(m + 1) <= n - 1) m++;
  return m;
}

// the key at iteration position p (0 <= p < n) of a map holding keys 0..n-1;
// m = um_epoch(n)
GBP_UM_HD inline int64_t um_key_at(int64_t p, int64_t n, int m) {
  for (;;) {
    const int64_t r = um_rehash_point(m);
    if (p < n - r) return n - 1 - p;
    p = n - 1 - p;
    n = r;
    m--;  // um_epoch(r) == m - 1: the points strictly increase
  }
}

// the iteration position of key k (0 <= k < n)
GBP_UM_HD inline int64_t um_rank(int64_t k, int64_t n) {
  int64_t acc = 0, sign = 1;
  int m = um_epoch(n);
  for (;;) {
    const int64_t r = um_rehash_point(m);
    if (k >= r) return acc + sign * (n - 1 - k);
    acc += sign * (n - 1);
    sign = -sign;
    n = r;
    m--;
  }
}

}  // namespace gbp
