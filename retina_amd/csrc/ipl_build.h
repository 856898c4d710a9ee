// Host builder of the LDS-resident IP table image used by the tier-1 dense kernel
// (gpuagg_internal.h, "LDS-resident IP table").  Header-only so that a host-only test
// (tests/ipl_build_test.cpp) exercises exactly the code the runtime runs.
#pragma once
#include <cstdint>
#include <cstring>
#include <utility>
#include <vector>

#include "gpuagg_internal.h"

namespace gpuagg {

struct IplImage {
  uint32_t nb = 0, seed = 0;
  std::vector<uint8_t> bytes;  // ipl_image_bytes(nb): keys u32[nb*2], then vals u16[nb*2]
};

// (ip, slot) entries with distinct IPs.  Returns false when the set cannot be imaged
// (a slot >= 0xFFFF, the key 0xFFFFFFFF, or no cuckoo placement within kIplMaxBytes);
// the caller then keeps the IP table in HBM.
inline bool ipl_build(const std::vector<std::pair<uint32_t, uint32_t>> &ents, IplImage *out,
                      uint32_t load_pct = 88) {
  for (const auto &e : ents)
    if (e.second >= kIplNoSlot || e.first == kIplEmptyKey) return false;
  uint32_t nb = (uint32_t)((ents.size() * 100 + load_pct * kIplWays - 1) / (load_pct * kIplWays));
  if (nb == 0) nb = 1;
  std::vector<uint32_t> keys;
  std::vector<uint16_t> vals;
  uint32_t seed = 0x6A09E667u;
  for (int attempt = 0; attempt < 96; ++attempt) {
    if (attempt && attempt % 8 == 0) nb = nb + nb / 16 + 1;
    if (nb >= kIplMaxBuckets || ipl_image_bytes(nb) > kIplMaxBytes) return false;
    seed = (uint32_t)fmix64((uint64_t)seed + 0xBB67AE8584CAA73BULL * (uint64_t)(attempt + 1));
    keys.assign((size_t)nb * kIplWays, kIplEmptyKey);
    vals.assign((size_t)nb * kIplWays + 1, (uint16_t)kIplNoSlot);  // + sentinel
    bool ok = true;
    uint64_t rng = seed | 1ULL;
    for (const auto &e : ents) {
      uint32_t k = e.first;
      uint16_t v = (uint16_t)e.second;
      uint32_t b1, b2;
      ipl_buckets(k, seed, nb, b1, b2);
      uint32_t b = b1;
      for (int kicks = 0;; ++kicks) {
        ipl_buckets(k, seed, nb, b1, b2);
        int slot = -1;
        for (uint32_t bb : {b1, b2}) {
          for (uint32_t w = 0; w < kIplWays && slot < 0; ++w)
            if (keys[(size_t)bb * kIplWays + w] == kIplEmptyKey) slot = (int)(bb * kIplWays + w);
          if (slot >= 0) break;
        }
        if (slot >= 0) {
          keys[slot] = k;
          vals[slot] = v;
          break;
        }
        if (kicks >= 2000) {
          ok = false;
          break;
        }
        // random walk: evict a random resident of the bucket not used last time
        b = (b == b1) ? b2 : b1;
        rng ^= rng << 13, rng ^= rng >> 7, rng ^= rng << 17;
        const size_t victim = (size_t)b * kIplWays + (uint32_t)(rng % kIplWays);
        std::swap(k, keys[victim]);
        std::swap(v, vals[victim]);
      }
      if (!ok) break;
    }
    if (!ok) continue;
    out->nb = nb;
    out->seed = seed;
    out->bytes.assign(ipl_image_bytes(nb), 0);
    memcpy(out->bytes.data(), keys.data(), keys.size() * 4);
    memcpy(out->bytes.data() + ipl_vals_offset(nb), vals.data(), vals.size() * 2);
    return true;
  }
  return false;
}

// Host mirror of the kernel's probe (dense_lds_kernel): slot or kIplNoSlot.
inline uint32_t ipl_probe(const uint8_t *img, uint32_t nb, uint32_t seed, uint32_t ip) {
  uint32_t b1, b2;
  ipl_buckets(ip, seed, nb, b1, b2);
  const uint32_t *keys = (const uint32_t *)img;
  const uint16_t *vals = (const uint16_t *)(img + ipl_vals_offset(nb));
  uint32_t j = nb * kIplWays;  // sentinel
  for (uint32_t c : {b1 * 2, b1 * 2 + 1, b2 * 2, b2 * 2 + 1})
    if (keys[c] == ip) j = c;
  return vals[j];
}

// ---- radix LDS image (gpuagg_internal.h, "Radix LDS image") --------------------------
struct IprImage {
  uint32_t npfx = 0, nblk = 0;
  uint32_t pfx[kIprMaxPfx] = {kIprNoPfx, kIprNoPfx, kIprNoPfx, kIprNoPfx};
  std::vector<uint8_t> bytes;  // ipr_image_bytes(npfx, nblk)
};

// Returns false when the set needs more than kIprMaxPfx /16 prefixes, a slot >= 0xFFFF,
// or more than max_bytes of image; the caller then uses the cuckoo image.
inline bool ipr_build(const std::vector<std::pair<uint32_t, uint32_t>> &ents, IprImage *out,
                      uint32_t max_bytes = kIplMaxBytes) {
  IprImage im;
  std::vector<uint32_t> rowblk;  // (prefix, third octet) -> block, 0 = none yet
  for (const auto &e : ents) {
    if (e.second >= kIplNoSlot) return false;
    const uint32_t p = e.first & 0xFFFFu;
    uint32_t j = 0;
    while (j < im.npfx && im.pfx[j] != p) ++j;
    if (j == im.npfx) {
      if (im.npfx == kIprMaxPfx) return false;
      im.pfx[im.npfx++] = p;
    }
  }
  rowblk.assign((size_t)kIprMaxPfx * 256, 0);
  std::vector<uint16_t> blk(256, (uint16_t)kIplNoSlot);  // block 0: no pod
  for (const auto &e : ents) {
    const uint32_t row = ipr_row(e.first, im.pfx[0], im.pfx[1], im.pfx[2], im.pfx[3], im.npfx);
    if (!rowblk[row]) {
      if (im.nblk + 1 >= 0xFFFFu) return false;
      rowblk[row] = ++im.nblk;
      blk.resize((size_t)(im.nblk + 1) * 256, (uint16_t)kIplNoSlot);
    }
    blk[(size_t)rowblk[row] * 256 + (e.first >> 24)] = (uint16_t)e.second;
  }
  if (ipr_image_bytes(im.npfx, im.nblk) > max_bytes) return false;
  im.bytes.assign(ipr_image_bytes(im.npfx, im.nblk), 0);
  uint16_t *bidx = (uint16_t *)im.bytes.data();
  for (uint32_t r = 0; r < im.npfx * 256; ++r) bidx[r] = (uint16_t)rowblk[r];
  memcpy(im.bytes.data() + ipr_blk_offset(im.npfx), blk.data(), blk.size() * 2);
  *out = std::move(im);
  return true;
}

// Host mirror of the kernel's radix probe: slot or kIplNoSlot.
inline uint32_t ipr_probe(const IprImage &im, uint32_t ip) {
  const uint16_t *bidx = (const uint16_t *)im.bytes.data();
  const uint16_t *blk = (const uint16_t *)(im.bytes.data() + ipr_blk_offset(im.npfx));
  const uint32_t row = ipr_row(ip, im.pfx[0], im.pfx[1], im.pfx[2], im.pfx[3], im.npfx);
  return blk[((uint32_t)bidx[row] << 8) | (ip >> 24)];
}

// ---- dense radix LDS image (gpuagg_internal.h, "Dense radix LDS image") ---------------
struct IprdImage {
  uint32_t npfx = 0, nblk = 0;
  uint32_t pfx[kIprMaxPfx] = {kIprNoPfx, kIprNoPfx, kIprNoPfx, kIprNoPfx};
  uint32_t dr[kIprMaxPfx] = {0, 0, 0, 0};
  std::vector<uint8_t> bytes;  // blk u16[(nblk + 1) * 256]
};

// Returns false when the set needs more than kIprMaxPfx /16 prefixes, a slot >= 0xFFFF, or
// more than max_bytes of image once each prefix's third-octet run [min, max] is filled
// (holes included); the caller then tries the radix image with its row table.
inline bool iprd_build(const std::vector<std::pair<uint32_t, uint32_t>> &ents, IprdImage *out,
                       uint32_t max_bytes = kIplMaxBytes) {
  IprdImage im;
  uint32_t lo[kIprMaxPfx] = {255, 255, 255, 255}, hi[kIprMaxPfx] = {0, 0, 0, 0};
  auto pfx_of = [&](uint32_t ip) {
    uint32_t j = 0;
    while (j < im.npfx && im.pfx[j] != (ip & 0xFFFFu)) ++j;
    return j;
  };
  for (const auto &e : ents) {
    if (e.second >= kIplNoSlot) return false;
    uint32_t j = pfx_of(e.first);
    if (j == im.npfx) {
      if (im.npfx == kIprMaxPfx) return false;
      im.pfx[im.npfx++] = e.first & 0xFFFFu;
    }
    const uint32_t o3 = (e.first >> 16) & 0xFFu;
    lo[j] = o3 < lo[j] ? o3 : lo[j];
    hi[j] = o3 > hi[j] ? o3 : hi[j];
  }
  uint32_t base = 1;
  for (uint32_t j = 0; j < im.npfx; ++j) {
    const uint32_t cnt = hi[j] - lo[j] + 1;
    im.dr[j] = lo[j] | (cnt << 8) | (base << 17);
    base += cnt;
  }
  im.nblk = base - 1;
  if ((size_t)(im.nblk + 1) * 512 > max_bytes) return false;
  std::vector<uint16_t> blk((size_t)(im.nblk + 1) * 256, (uint16_t)kIplNoSlot);
  for (const auto &e : ents) {
    const uint32_t b = iprd_block(e.first, im.pfx[0], im.pfx[1], im.pfx[2], im.pfx[3], im.dr[0], im.dr[1],
                                  im.dr[2], im.dr[3]);
    blk[((size_t)b << 8) | (e.first >> 24)] = (uint16_t)e.second;
  }
  im.bytes.assign(blk.size() * 2, 0);
  memcpy(im.bytes.data(), blk.data(), blk.size() * 2);
  *out = std::move(im);
  return true;
}

// Host mirror of the kernel's dense radix probe: slot or kIplNoSlot.
inline uint32_t iprd_probe(const IprdImage &im, uint32_t ip) {
  const uint16_t *blk = (const uint16_t *)im.bytes.data();
  const uint32_t b = iprd_block(ip, im.pfx[0], im.pfx[1], im.pfx[2], im.pfx[3], im.dr[0], im.dr[1], im.dr[2],
                                im.dr[3]);
  return blk[(b << 8) | (ip >> 24)];
}

}  // namespace gpuagg
