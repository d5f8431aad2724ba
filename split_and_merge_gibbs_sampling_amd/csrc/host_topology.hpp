// host_topology.hpp -- where a context's host worker pool lives.
//
// The per-iteration host phases (update_phi's serial draws and their worker-pool phases) hand
// data between cores every iteration, so a context's pool is pinned to distinct physical cores
// of one L3 domain next to its GPU.  The choice is a pure function of the topology (tested on
// the CPU by tests/cpp/host_topology_test.cpp); engine.cpp reads the topology from sysfs and
// keeps one pool per chosen domain, so contexts on GPUs with different homes (an R session
// running replicas on two GPUs) get pools on different domains.
#pragma once

#include <algorithm>
#include <cstddef>
#include <functional>
#include <vector>

namespace hdpm {

// The home L3 domain of the slot-th of `share` GPUs whose local CPUs are `mine`: the usable
// CPUs of `mine` grouped by L3 domain (l3_key(cpu): the first CPU of its L3 sharing list), the
// GPUs spread over the domains in order, keeping off the first domain (CPU 0's: interrupts
// and daemons) while there are more domains than GPUs.  Empty when nothing is usable.
inline std::vector<int> choose_home_domain(const std::vector<int>& mine, int slot, int share,
                                           const std::function<int(int)>& l3_key,
                                           const std::function<bool(int)>& usable) {
  std::vector<std::vector<int>> doms;
  std::vector<int> keys;
  for (int c : mine) {
    if (!usable(c)) continue;
    const int key = l3_key(c);
    size_t q = 0;
    while (q < keys.size() && keys[q] != key) ++q;
    if (q == keys.size()) {
      keys.push_back(key);
      doms.emplace_back();
    }
    doms[q].push_back(c);
  }
  if (doms.empty() || share <= 0 || slot < 0 || slot >= share) return {};
  const size_t nd = doms.size();
  return doms[std::min(nd - 1, (size_t)(slot + 1) * nd / (size_t)(share + 1))];
}

}  // namespace hdpm
