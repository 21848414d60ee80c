// Resident-workgroup counts per (device, kernel, threads, dynamic LDS bytes),
// queried once and cached for the persistent-grid launches (k_rowgemm).
// Host-only and free of HIP types so that tests/test_occupancy_cache_cpu.py
// can compile it with g++ against a counting stand-in for the occupancy query.
//
// Round 5 cached the count per [prefetch][column tiles] alone; the occupancy
// also depends on the dynamic LDS size, which follows the GEMM's inner
// dimension, so the first shape run with a given tile count fixed the grid of
// every later shape.  The key here carries
// every input the query takes, plus the device.
#pragma once
#include <cstddef>
#include <cstdint>
#include <map>
#include <mutex>
#include <tuple>

namespace cg {

class ResidentCache {
 public:
  // query(kernel, threads, lds, &blocks_per_cu, &cus) -> true on success.
  // Returns blocks resident on the whole chip, or -1 when unknown (the query
  // failed; callers keep their static cap).
  template <typename Query>
  int get(int device, const void* kernel, int threads, size_t lds, Query&& query) {
    const Key key{device, kernel, threads, lds};
    {
      std::lock_guard<std::mutex> g(mu_);
      auto it = map_.find(key);
      if (it != map_.end()) return it->second;
    }
    int per_cu = 0, cus = 0;
    const bool ok = query(kernel, threads, lds, &per_cu, &cus) && per_cu > 0 && cus > 0;
    const int v = ok ? per_cu * cus : -1;
    std::lock_guard<std::mutex> g(mu_);
    map_.emplace(key, v);  // a racing thread's equal answer wins harmlessly
    return v;
  }
  size_t size() {
    std::lock_guard<std::mutex> g(mu_);
    return map_.size();
  }

 private:
  using Key = std::tuple<int, const void*, int, size_t>;
  std::mutex mu_;
  std::map<Key, int> map_;
};

// Persistent grid: at most `cap` blocks, at most `resident / planes` so that
// no block runs as a tail round, at least 1, and never more than the tiles.
inline unsigned persistent_grid(int64_t ntiles, int resident, int planes, unsigned cap = 1024) {
  unsigned gx = unsigned(ntiles < int64_t(cap) ? ntiles : int64_t(cap));
  if (resident > 0 && planes >= 1) {
    const unsigned per_plane = unsigned(resident) / unsigned(planes);
    if (per_plane >= 1 && gx > per_plane) gx = per_plane;
  }
  return gx < 1 ? 1u : gx;
}

}  // namespace cg
