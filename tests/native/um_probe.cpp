// Test infrastructure: the iteration order of a real libstdc++
// std::unordered_map<int, State> filled the way GraphClass::addVertex fills
// its vertex map (graph_class.cpp:28-31: vertices[idx] = q for idx = 0, 1, ...;
// graph_class.h:155).  Built by tests/test_um_order.py with this image's g++;
// it checks the oracle's and the engine's restatement of that order.
#include <array>
#include <cstdint>
#include <unordered_map>

extern "C" void um_probe_order(int64_t n, int32_t *out) {
  std::unordered_map<int, std::array<double, 8>> vertices;
  for (int64_t k = 0; k < n; k++) vertices[(int)k] = std::array<double, 8>{};
  int64_t p = 0;
  for (auto it = vertices.begin(); it != vertices.end(); ++it) out[p++] = it->first;
}

// the element counts at which inserting one more key rehashes, from the
// container itself (bucket_count changes), up to n keys
extern "C" int64_t um_probe_rehash_points(int64_t n, int64_t *out, int64_t max_out) {
  std::unordered_map<int, std::array<double, 8>> m;
  std::size_t bc = m.bucket_count();
  int64_t c = 0;
  for (int64_t k = 0; k < n; k++) {
    m[(int)k];
    if (m.bucket_count() != bc) {
      if (c < max_out) out[c] = k;
      c++;
      bc = m.bucket_count();
    }
  }
  return c;
}
