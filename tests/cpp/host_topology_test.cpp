// CPU test of the host-pool home choice (csrc/host_topology.hpp choose_home_domain), on
// synthetic topologies: GPUs sharing a NUMA node's CPUs get distinct L3 domains, the first
// domain (CPU 0's) is avoided while there are more domains than GPUs, unusable CPUs are
// skipped, and an empty or invalid description gives no home (the creating thread's).
#include <cstdio>
#include <cstdlib>
#include <set>
#include <vector>

#include "../../split_and_merge_gibbs_sampling_amd/csrc/host_topology.hpp"

using hdpm::choose_home_domain;

static int fails = 0;
#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c);      \
      ++fails;                                                     \
    }                                                              \
  } while (0)

int main() {
  // a node of 64 CPUs in 8 L3 domains of 8 (EPYC-like CCDs); all usable
  std::vector<int> cpus(64);
  for (int c = 0; c < 64; ++c) cpus[c] = c;
  auto l3 = [](int c) { return c / 8 * 8; };
  auto all = [](int) { return true; };

  // one GPU alone: a domain in the middle, never CPU 0's
  {
    const std::vector<int> d = choose_home_domain(cpus, 0, 1, l3, all);
    CHECK(d.size() == 8);
    CHECK(d.front() == 32);
  }
  // two GPUs on the same CPUs: different domains, neither CPU 0's
  {
    const std::vector<int> a = choose_home_domain(cpus, 0, 2, l3, all);
    const std::vector<int> b = choose_home_domain(cpus, 1, 2, l3, all);
    CHECK(!a.empty() && !b.empty());
    CHECK(a != b);
    CHECK(a.front() != 0 && b.front() != 0);
  }
  // four GPUs: four distinct domains
  {
    std::set<int> homes;
    for (int g = 0; g < 4; ++g) homes.insert(choose_home_domain(cpus, g, 4, l3, all).front());
    CHECK(homes.size() == 4);
    CHECK(!homes.count(0));
  }
  // eight GPUs on eight domains: one each
  {
    std::set<int> homes;
    for (int g = 0; g < 8; ++g) homes.insert(choose_home_domain(cpus, g, 8, l3, all).front());
    CHECK(homes.size() == 8);
  }
  // only some CPUs usable (a container's cpuset): the home holds usable CPUs only
  {
    auto some = [](int c) { return c >= 16 && c < 40; };
    const std::vector<int> d = choose_home_domain(cpus, 0, 1, l3, some);
    CHECK(!d.empty());
    for (int c : d) CHECK(c >= 16 && c < 40);
  }
  // no usable CPU, no GPUs, a slot outside the share: no home
  {
    CHECK(choose_home_domain(cpus, 0, 1, l3, [](int) { return false; }).empty());
    CHECK(choose_home_domain(cpus, 0, 0, l3, all).empty());
    CHECK(choose_home_domain(cpus, 3, 2, l3, all).empty());
    CHECK(choose_home_domain({}, 0, 1, l3, all).empty());
  }
  // one domain only: every GPU shares it
  {
    auto one = [](int) { return 0; };
    CHECK(choose_home_domain(cpus, 0, 2, one, all).size() == 64);
    CHECK(choose_home_domain(cpus, 1, 2, one, all).size() == 64);
  }
  if (fails) return 1;
  std::printf("host topology ok\n");
  return 0;
}
