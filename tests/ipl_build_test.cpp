// Host-only check of the LDS IP-table builder (retina_amd/csrc/ipl_build.h): reads
// "n_sets" then per set "n ip slot..." from stdin, builds, probes every key and a sample
// of absent IPs with the host mirror of the kernel probe, prints one line per set:
//   built nb seed bytes load_pct found_ok absent_ok
#include <algorithm>
#include <cstdio>
#include <random>

#include "ipl_build.h"

using namespace gpuagg;

int main() {
  int sets = 0;
  if (scanf("%d", &sets) != 1) return 2;
  for (int s = 0; s < sets; ++s) {
    size_t n = 0;
    if (scanf("%zu", &n) != 1) return 2;
    std::vector<std::pair<uint32_t, uint32_t>> ents(n);
    for (auto &e : ents)
      if (scanf("%u %u", &e.first, &e.second) != 2) return 2;
    IplImage im;
    const bool ok = ipl_build(ents, &im);
    long found = 0, absent_ok = 0;
    if (ok) {
      for (const auto &e : ents) found += ipl_probe(im.bytes.data(), im.nb, im.seed, e.first) == e.second;
      std::mt19937 rng(s);
      std::vector<uint32_t> sorted;
      for (const auto &e : ents) sorted.push_back(e.first);
      std::sort(sorted.begin(), sorted.end());
      for (int i = 0; i < 100000; ++i) {
        const uint32_t ip = rng();
        if (std::binary_search(sorted.begin(), sorted.end(), ip)) continue;
        absent_ok += ipl_probe(im.bytes.data(), im.nb, im.seed, ip) == kIplNoSlot;
      }
    }
    // the radix image of the same set (when its prefixes allow one): same answers
    IprImage ir;
    const bool rok = ipr_build(ents, &ir);
    long rfound = 0, rabsent = 0;  // rabsent: absent IPs that did NOT miss
    if (rok) {
      for (const auto &e : ents) rfound += ipr_probe(ir, e.first) == e.second;
      std::mt19937 rng(s + 1000);
      std::vector<uint32_t> sorted;
      for (const auto &e : ents) sorted.push_back(e.first);
      std::sort(sorted.begin(), sorted.end());
      for (int i = 0; i < 100000; ++i) {
        // half random, half near the pod IPs (same /16 and /24 prefixes)
        uint32_t ip = rng();
        if (i & 1 && !sorted.empty()) ip = (sorted[rng() % sorted.size()] & 0x00FFFFFFu) | (rng() & 0xFF000000u);
        if (std::binary_search(sorted.begin(), sorted.end(), ip)) continue;
        rabsent += ipr_probe(ir, ip) != kIplNoSlot;  // wrong answers
      }
    }
    // the dense radix image (per-prefix third-octet runs): same answers
    IprdImage id;
    const bool dok = iprd_build(ents, &id);
    long dfound = 0, dabsent = 0;
    if (dok) {
      for (const auto &e : ents) dfound += iprd_probe(id, e.first) == e.second;
      std::mt19937 rng(s + 2000);
      std::vector<uint32_t> sorted;
      for (const auto &e : ents) sorted.push_back(e.first);
      std::sort(sorted.begin(), sorted.end());
      for (int i = 0; i < 100000; ++i) {
        uint32_t ip = rng();
        if (i & 1 && !sorted.empty()) ip = (sorted[rng() % sorted.size()] & 0x00FFFFFFu) | (rng() & 0xFF000000u);
        if (i % 3 == 0 && !sorted.empty()) ip = (sorted[rng() % sorted.size()] & 0xFF00FFFFu) | (rng() & 0x00FF0000u);
        if (std::binary_search(sorted.begin(), sorted.end(), ip)) continue;
        dabsent += iprd_probe(id, ip) != kIplNoSlot;  // wrong answers
      }
    }
    printf("%d %u %u %zu %.1f %ld %ld %d %u %u %zu %ld %ld %d %u %zu %ld %ld\n", ok ? 1 : 0, im.nb, im.seed,
           im.bytes.size(), ok ? 100.0 * n / (im.nb * kIplWays) : 0.0, found, absent_ok, rok ? 1 : 0, ir.npfx,
           ir.nblk, ir.bytes.size(), rfound, rabsent, dok ? 1 : 0, id.nblk, id.bytes.size(), dfound, dabsent);
  }
  return 0;
}
