// Internal definitions shared by the HIP kernels and the host runtime.
//
// Key design (DESIGN.md sections 3-5):
//  * A metric "group" is one (family, context-options) pair. forward_count and
//    forward_bytes with the same options share a group: every group accumulates a
//    count and a byte sum per key, so Inc() and Add(PacketSize) both come out of it
//    (forward.go:217-224, drops.go:388-395).
//  * Local-context groups whose label values depend only on the endpoint slot
//    (options among namespace/podname/workload/service) are DENSE: counters indexed by
//    (slot, side, sub).  Everything else (remote context, ip/port options, DNS) is
//    SPARSE: a 192-bit key in an HBM open-addressed table.
//  * The device groups on a key at least as fine as the label tuple; the host turns
//    keys into label values and sums equal tuples, so the result is exact.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define GA_HD __host__ __device__ __forceinline__
#else
#define GA_HD inline
#endif

namespace gpuagg {

// ---- record meta word (include/gpuagg.h) -----------------------------------------
GA_HD uint32_t meta_proto(uint32_t m) { return m & 0xFFu; }
// The column holds the verdict the producer passed to utils.ToFlow, which turns 0 into
// FORWARDED (flow_utils.go:94-96).
GA_HD uint32_t meta_verdict(uint32_t m) {
  const uint32_t v = (m >> 8) & 0xFFu;
  return v ? v : 1u;
}
GA_HD uint32_t meta_tdir(uint32_t m) { return (m >> 16) & 3u; }
GA_HD uint32_t meta_reason(uint32_t m) { return (m >> 18) & 7u; }
GA_HD uint32_t meta_flags(uint32_t m) { return (m >> 21) & 0x3Fu; }
GA_HD uint32_t meta_dnstype(uint32_t m) { return (m >> 28) & 3u; }

constexpr uint32_t kVerdictForwarded = 1, kVerdictDropped = 2, kVerdictRetrans = 15,
                   kVerdictDns = 16;
// decoded raw row whose field does not fit the meta word: no metric consumes it
constexpr uint32_t kVerdictUnencodable = 255;
constexpr uint32_t kDnsQuery = 1, kDnsResponse = 2;

// ---- host decode of one raw perf record ---------------------------------------------
// The host restatement of packet_decode_kernel / drop_decode_kernel (gpuagg_decode.hip:
// field offsets and meta packing documented there), shared by the CPU backend and the
// host-decoding raw feed (gpuagg_feed.cpp).  `w` are the record's little-endian dwords.
struct RawRow {
  uint32_t src, dst, bytes, meta, ports, tcp_id;
  uint64_t time_ns;
  bool bad;  // a field that does not fit the meta word (verdict kVerdictUnencodable)
};
inline uint32_t raw_swap_ports(uint32_t w) {  // utils.HostToNetShort of both u16 halves
  return ((w & 0xFFu) << 8) | ((w >> 8) & 0xFFu) | ((w & 0xFF0000u) << 8) | ((w >> 8) & 0xFF0000u);
}
// struct packet of packetparser (72 B, conntrack.c:34-49; packetparser_linux.go:571-631)
inline RawRow decode_packet_words(const uint32_t *w, uint64_t time_offset) {
  const uint32_t obs = w[10] & 0xFFu, tdir = (w[10] >> 8) & 0xFFu, proto = (w[10] >> 16) & 0xFFu;
  const uint32_t tcp_flags = proto == 6u ? ((w[10] >> 24) & 0x3Fu) : 0u;
  RawRow r;
  r.bad = tdir > 3u;
  r.src = w[3];
  r.dst = w[4];
  r.bytes = w[2];
  r.meta = proto | ((r.bad ? kVerdictUnencodable : kVerdictForwarded) << 8) | ((tdir & 3u) << 16) |
           (tcp_flags << 21) | ((w[11] & 0xFFu) ? (1u << 27) : 0u) | ((obs <= 3u ? obs : 0u) << 30);
  r.ports = raw_swap_ports(w[5]);
  r.tcp_id = obs == 3u ? w[8] : obs == 2u ? w[9] : 0u;
  r.time_ns = ((uint64_t)w[0] | ((uint64_t)w[1] << 32)) + time_offset;
  return r;
}
// struct packet of dropreason (32 B, drop_reason.c:39-54; dropreason_linux.go:345-386)
inline RawRow decode_drop_words(const uint32_t *d, uint64_t time_offset) {
  const uint32_t drop_type = d[5] & 0xFFFFu, proto = (d[5] >> 16) & 0xFFu;
  RawRow r;
  r.bad = drop_type > 7u;
  r.src = d[0];
  r.dst = d[1];
  r.bytes = d[3];
  r.meta = proto | ((r.bad ? kVerdictUnencodable : kVerdictDropped) << 8) | (1u << 16) | ((drop_type & 7u) << 18) |
           (2u << 30);
  r.ports = raw_swap_ports(d[2]);
  r.tcp_id = 0u;
  r.time_ns = ((uint64_t)d[6] | ((uint64_t)d[7] << 32)) + time_offset;
  return r;
}

// kernel flag bits (pkg/plugin/packetparser/types_linux.go:22-31)
constexpr uint32_t kFin = 1, kSyn = 2, kRst = 4, kPsh = 8, kAck = 16, kUrg = 32;

// TCP flag label indices, in getFlagValues order (tcpflags.go:134-175).
enum FlagIdx : uint32_t { F_FIN = 0, F_SYNACK, F_SYN, F_ACK, F_RST, F_PSH, F_URG, F_COUNT };

// Bit set of FlagIdx that getFlagValues returns for a kernel flag byte.
GA_HD uint32_t flag_label_mask(uint32_t f) {
  uint32_t m = 0;
  if (f & kFin) m |= 1u << F_FIN;
  if ((f & kSyn) && (f & kAck)) {
    m |= 1u << F_SYNACK;
  } else {
    if (f & kSyn) m |= 1u << F_SYN;
    if (f & kAck) m |= 1u << F_ACK;
  }
  if (f & kRst) m |= 1u << F_RST;
  if (f & kPsh) m |= 1u << F_PSH;
  if (f & kUrg) m |= 1u << F_URG;
  return m;
}

// ---- metric plan -------------------------------------------------------------------
enum Family : uint8_t {
  FAM_FWD = 0, FAM_DROP, FAM_TCPFLAGS, FAM_RETRANS, FAM_DNS_REQ, FAM_DNS_RESP, FAM_COUNT
};
// Context option bits (types.go:300-327).
enum Opt : uint8_t {
  OPT_IP = 1, OPT_NS = 2, OPT_POD = 4, OPT_WL = 8, OPT_SVC = 16, OPT_PORT = 32
};
constexpr uint8_t OPT_EP = OPT_NS | OPT_POD | OPT_WL;  // options read from the endpoint

constexpr int kMaxGroups = 16;

struct GroupPlan {
  uint8_t family;
  uint8_t sparse;    // 0 dense, 1 sparse
  uint8_t src_opts;  // local: the single local ctx; remote: source ctx
  uint8_t dst_opts;  // remote: destination ctx
  uint32_t nsub;     // dense: sub-bins per (key, side): 1 or 8
  uint64_t dense_base;
  uint32_t key_mode;  // dense: 0 constant key, 1 slot key
  uint32_t nbins;     // dense: bins of this group (nkeys * 2 * nsub)
};

struct Plan {
  int32_t local;
  int32_t ngroups;
  uint32_t need_ports;
  uint32_t need_dns;
  uint32_t need_bytes;  // some group adds packet bytes (forward / drop)
  GroupPlan g[kMaxGroups];
};

// ---- hashing -----------------------------------------------------------------------
GA_HD uint64_t fmix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdULL;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ULL;
  k ^= k >> 33;
  return k;
}

// dist.shard_of (retina_amd/dist.py), the Go plugin's shardOf and the feeds: fmix64 of the
// direction-free 5-tuple -- lo <= hi the two (ip << 16 | port) ends, so a request and its
// reply meet on one device for the latency join -- mod n.
GA_HD uint32_t shard_5tuple(uint32_t src, uint32_t dst, uint32_t ports, uint32_t proto, uint32_t n) {
  const uint64_t a = ((uint64_t)src << 16) | (ports & 0xFFFFu), b = ((uint64_t)dst << 16) | (ports >> 16);
  const uint64_t lo = a < b ? a : b, hi = a < b ? b : a;
  const uint64_t h = fmix64(lo ^ fmix64(hi ^ ((uint64_t)(proto & 0xFFu) << 48) ^ 0x1F2E3D4C5B6A7988ULL));
  return (uint32_t)(h % n);
}

// IP table: open addressing, linear probing. Entry = ip | slot << 32 | apiserver << 53.
constexpr uint64_t kIpEmpty = ~0ULL;
constexpr uint32_t kSlotBits = 21;
// Radix IP table (when the pod IPs fall in few /16s, as cluster pod CIDRs do): a 64k
// u16 table maps the first two address octets (the low 16 bits of the LE u32) to a block
// of 64k u32 entries indexed by the last two octets; entry = slot | apiserver << 31, or
// kRadixEmpty.  Two loads per IP, the first to a table of a few hot lines.
constexpr uint32_t kRadixEmpty = 0xFFFFFFFFu, kRadixNoBlock = 0xFFFFu, kRadixMaxBlocks = 64;
constexpr uint32_t kRadixSmall = 8;  // prefixes resolved by compares (DevIpTable::rp)
constexpr uint32_t kMaxSlot = (1u << kSlotBits) - 2;  // slot ids 0..kMaxSlot
GA_HD uint32_t ip_hash(uint32_t ip) {  // murmur3 fmix32: 2 mul + 3 xorshift
  ip ^= ip >> 16;
  ip *= 0x85ebca6bu;
  ip ^= ip >> 13;
  ip *= 0xc2b2ae35u;
  ip ^= ip >> 16;
  return ip;
}
// Cuckoo IP table (2 choices, one 8-byte entry each): a lookup is exactly two
// independent loads, no probe loop.  seed = (seed1, seed2) chosen by the host builder.
// One multiply per choice (32-bit multiplies are quarter rate on CDNA).
GA_HD uint32_t ip_pre(uint32_t ip, uint32_t seed) {
  const uint32_t x = ip ^ seed;
  return x ^ (x >> 16);
}
GA_HD uint32_t ip_h1(uint32_t ip, uint32_t seed) {
  const uint32_t h = ip_pre(ip, seed) * 0x9E3779B1u;
  return h ^ (h >> 15);
}
GA_HD uint32_t ip_h2(uint32_t ip, uint32_t seed) {
  const uint32_t h = ip_pre(ip, seed) * 0x85EBCA77u;
  return h ^ (h >> 13);
}
// Dense bins kept in LDS per workgroup: u64 = count << 44 | bytes.  A workgroup
// aggregates <= 2^20 records between flushes and an update carries < 2^24 bytes in
// LDS (bigger packets add their bytes with a global atomic), so both fields are exact.
// LDS layout: bins [0, L), 64 per-lane dummy words [L, L+64) that absorb predicated-
// off updates, then kMaxSpillWindows u32 spill-window counters.
constexpr uint32_t kLdsBytes = 160 * 1024;
// 256 windows x 2^13 bins: dense spaces up to ~2M bins beyond the LDS prefix (C5's
// 100k-pod tcpflags + retransmit groups) still fold in LDS instead of global atomics
constexpr uint32_t kMaxSpillWindows = 256;
constexpr uint32_t kSpillRing = 128;  // staged spill appends per window (dense_local_kernel kStage)
constexpr uint32_t kHotKeyBytes = 48;    // LDS hot-key cache entry (aggregate_kernel)
constexpr uint32_t kHotKeys = 2048;      // entries when the plan has HBM-table keys
// wide_kernel (remote context) takes the LDS image of every pod IP when it fits next to a
// hot-key cache of >= kWideIplMinHot entries and a 2^kWideIplMinDoor-bit doorkeeper.  C4
// remote, 100M records: 2048 entries + image + 2^15-bit doorkeeper 1.14 ms, 1024 entries
// + image + 2^17 bits 1.34 ms, no image (2048 + 2^18 bits) 1.32 ms
// (profiles/round3/exp/v3_wide_ipl.jsonl)
constexpr uint32_t kWideIplMinHot = 2048;
constexpr uint32_t kWideIplMinDoor = 13;
constexpr uint32_t kLdsExtraWords = 64 + kMaxSpillWindows / 2;  // 64 dummies + u32 spill-window counters
constexpr uint32_t kLdsMaxBins = kLdsBytes / 8 - kLdsExtraWords;
constexpr uint32_t kLdsCountShift = 44;
constexpr uint32_t kLdsByteLimit = 1u << 24;
constexpr uint64_t kLdsCountOne = 1ULL << kLdsCountShift;
constexpr uint64_t kLdsBytesMask = kLdsCountOne - 1;
constexpr uint64_t kMaxRecordsPerBlock = (1ULL << 20) - 4;  // count field < 2^20, multiple of 4
// fold windows: 2^13 u64 bins (64 KiB of LDS, two fold workgroups per CU) so a spilled
// bin's window is a shift.  Spill entries are u32: the bin's offset in its window
// (13 bits) | bytes << 13; a packet of >= 2^19 bytes adds its bytes with a global
// atomic and spills 0.
constexpr uint32_t kFoldWindowShift = 13, kFoldWindowBins = 1u << kFoldWindowShift;
// Bit 31 of a spill entry marks a row-mask entry: offset = the first bin of an 8-bin
// tcpflags row, bits [win_shift, win_shift + 8) = the flags to count (+1 each); plain
// entries carry < 2^(31 - win_shift) bytes, so the bit is free.
constexpr uint32_t kSpillRowMask = 1u << 31;

// ---- LDS-resident IP table (tier-1 dense kernel) ------------------------------------
// Bucketized cuckoo: 2 candidate buckets of 2 keys (8 B, one ds_read_b64 each),
// keys u32 (0xFFFFFFFF = empty), values u16 slot ids in a parallel array.  Only built
// for pods that are not the apiserver pseudo pod: in local context such an endpoint is
// treated exactly like "no endpoint" (types.go:407-413).
constexpr uint32_t kIplWays = 2;  // 2 choices x 2-way buckets: one ds_read_b64 per choice
constexpr uint32_t kIplEmptyKey = 0xFFFFFFFFu;
constexpr uint32_t kIplNoSlot = 0xFFFFu;
constexpr uint32_t kIplMaxBytes = 112 * 1024;
constexpr uint32_t kIplMaxBuckets = 1u << 16;  // bucket math uses 24-bit multiplies
// 24-bit multiplies are full rate on CDNA (32-bit ones are quarter rate)
GA_HD uint32_t mul_u24(uint32_t a, uint32_t b) { return (a & 0xFFFFFFu) * (b & 0xFFFFFFu); }
GA_HD uint32_t mulhi_u24(uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  // one v_mul_hi_u32_u24; written as asm because the compiler otherwise folds a later
  // shift of the result into a full 48-bit product (mul_lo + mul_hi + alignbit)
  uint32_t r;
  asm("v_mul_hi_u32_u24 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
#else
  return (uint32_t)(((uint64_t)(a & 0xFFFFFFu) * (uint64_t)(b & 0xFFFFFFu)) >> 32);
#endif
}
// Both bucket choices of an IP (nb < 2^16).  The fold x ^ x>>12 (a bijection) brings
// the high byte, which varies most in little-endian pod IPs, into the 24 bits the
// multiplies see; the two choices use different multipliers.
GA_HD void ipl_buckets(uint32_t ip, uint32_t seed, uint32_t nb, uint32_t &b1, uint32_t &b2) {
  uint32_t x = ip ^ seed;
  x ^= x >> 12;
  b1 = mulhi_u24(mul_u24(x, 0x9E3779u) >> 8, nb << 8);  // = (h1>>8) * nb >> 24
  b2 = mulhi_u24(mul_u24(x, 0xC2B2AFu) >> 8, nb << 8);
}
// Image: keys u32[nb*2] (16-byte padded), then vals u16[nb*2 + 1]; the extra value at
// index nb*2 is the "not found" sentinel (kIplNoSlot), so a probe needs no branch.
GA_HD uint32_t ipl_image_bytes(uint32_t nb) {
  return ((nb * kIplWays * 4 + 15) & ~15u) + ((nb * kIplWays * 2 + 2 + 15) & ~15u);
}
GA_HD uint32_t ipl_vals_offset(uint32_t nb) { return (nb * kIplWays * 4 + 15) & ~15u; }
// Radix LDS image (tier-1, when every pod IP falls in at most kIprMaxPfx /16 prefixes, as
// cluster pod CIDRs do): a /16 prefix is matched by compares against kernel arguments,
// the third octet indexes that prefix's row of u16 block ids, and the block's 256 u16
// slots are indexed by the fourth octet -- two dependent u16 reads and ~8 VALU per IP
// instead of two 8-byte bucket reads, a slot read and ~20 VALU.  Node pod CIDRs are /24s,
// so the blocks are the populated /24s (C2's 10k pods + secondaries: 80 blocks, 42 KiB).
// Layout: bidx u16[(npfx + 1) * 256] (row npfx: no prefix matched, all 0), then
// blk u16[(nblk + 1) * 256] with block 0 the "no pod" block (all kIplNoSlot).
constexpr uint32_t kIprMaxPfx = 4;
constexpr uint32_t kIprNoPfx = 0xFFFFFFFFu;  // unused prefix value: never equals ip & 0xFFFF
GA_HD uint32_t ipr_blk_offset(uint32_t npfx) { return (npfx + 1) * 256 * 2; }
GA_HD uint32_t ipr_image_bytes(uint32_t npfx, uint32_t nblk) { return ipr_blk_offset(npfx) + (nblk + 1) * 256 * 2; }
// row of bidx for ip: prefix index (npfx when none matches) << 8 | third octet
GA_HD uint32_t ipr_row(uint32_t ip, uint32_t p0, uint32_t p1, uint32_t p2, uint32_t p3, uint32_t npfx) {
  const uint32_t p = ip & 0xFFFFu;
  uint32_t j = npfx;
  j = p == p3 ? 3u : j;
  j = p == p2 ? 2u : j;
  j = p == p1 ? 1u : j;
  j = p == p0 ? 0u : j;
  return (j << 8) | ((ip >> 16) & 0xFFu);
}

// Dense radix LDS image (the common case of the radix image: every prefix's populated /24s
// form one run of third octets, as node pod CIDRs carved in order from a cluster /16 do):
// no row table -- the block of an address is computed, so a lookup is ONE u16 read and a
// few VALU ops instead of two dependent reads.  Per prefix j a descriptor
// dr[j] = lo | cnt << 8 | base << 17 (third octets [lo, lo + cnt) map to blocks base ..);
// the image is blk u16[(nblk + 1) * 256] with block 0 the "no pod" block; holes inside a
// run get empty blocks of their own.
GA_HD uint32_t iprd_block(uint32_t ip, uint32_t p0, uint32_t p1, uint32_t p2, uint32_t p3, uint32_t d0,
                          uint32_t d1, uint32_t d2, uint32_t d3) {
  const uint32_t p = ip & 0xFFFFu;
  uint32_t d = 0u;
  d = p == p3 ? d3 : d;
  d = p == p2 ? d2 : d;
  d = p == p1 ? d1 : d;
  d = p == p0 ? d0 : d;
  const uint32_t rel = ((ip >> 16) & 0xFFu) - (d & 0xFFu);
  return rel < ((d >> 8) & 0x1FFu) ? (d >> 17) + rel : 0u;
}

// 32-bit LDS bins of the tier-1 kernel: bytes families pack count:12 | bytes:20 and
// correct the rare carry / wrap exactly with global atomics; count-only families
// (tcpflags, tcpretrans) use the whole word (<= 2^20 records per workgroup).
// tier-1 kernel signatures: per group 4 bits (family + 1 | in-LDS << 3), group 0 lowest
constexpr uint32_t sig_group(uint32_t fam, bool inl) { return (fam + 1) | (inl ? 8u : 0u); }
constexpr uint32_t kSigFwdLds = sig_group(0, true);                                  // FAM_FWD
constexpr uint32_t kSigFwdLdsDropLds = kSigFwdLds | sig_group(1, true) << 4;         // + FAM_DROP
constexpr uint32_t kSigFwdLdsDropSpill = kSigFwdLds | sig_group(1, false) << 4;
// C5: tcpflags + retransmissions spilled, DNS request / response compact (dense_local_kernel)
constexpr uint32_t kSigC5 = sig_group(2, false) | sig_group(3, false) << 4 | sig_group(4, false) << 8 |
                            sig_group(5, false) << 12;
constexpr uint32_t kL4CountShift = 20;
constexpr uint32_t kL4BytesMask = (1u << kL4CountShift) - 1;
constexpr uint32_t kL4ByteLimit = 1u << kL4CountShift;
constexpr uint32_t kL4ExtraBytes = 64 * 4 + kMaxSpillWindows * 4;  // dummies + spill counters
GA_HD uint64_t ip_entry(uint32_t ip, uint32_t slot, uint32_t api) {
  return (uint64_t)ip | ((uint64_t)slot << 32) | ((uint64_t)(api & 1) << 53);
}

// Sparse table slots are interleaved: k0 k1 k2 cnt byt (40 bytes), so an insert's CAS /
// publish / adds touch one or two lines, and a segment of slots is one contiguous run
// that the wide-key fold loads into LDS with coalesced reads.
constexpr uint32_t kSparseSlotWords = 5;
// Sparse group-by key: k0 = occ | group<<59 | sub<<53 | s_slot1<<32 | s_ip
//                      k1 = s_port17<<47 | d_port17<<30 | d_slot1<<9
//                      k2 = d_ip<<32 | dns_id
// sub: bits 5..3 reason or flag index, bits 2..1 traffic direction, bit 0 side (local).
constexpr uint64_t kKeyOcc = 1ULL << 63;
constexpr uint64_t kKeyPending = ~0ULL;  // k2 before publication
GA_HD uint64_t key0(uint32_t group, uint32_t sub, uint32_t s_slot1, uint32_t s_ip) {
  return kKeyOcc | ((uint64_t)group << 59) | ((uint64_t)sub << 53) | ((uint64_t)s_slot1 << 32) |
         (uint64_t)s_ip;
}
GA_HD uint64_t key1(uint32_t s_port17, uint32_t d_port17, uint32_t d_slot1) {
  return ((uint64_t)s_port17 << 47) | ((uint64_t)d_port17 << 30) | ((uint64_t)d_slot1 << 9);
}
GA_HD uint64_t key2(uint32_t d_ip, uint32_t dns_id) { return ((uint64_t)d_ip << 32) | dns_id; }
GA_HD uint32_t key_group(uint64_t k0) { return (uint32_t)(k0 >> 59) & 15u; }
GA_HD uint32_t key_sub(uint64_t k0) { return (uint32_t)(k0 >> 53) & 63u; }
GA_HD uint32_t key_s_slot1(uint64_t k0) { return (uint32_t)(k0 >> 32) & ((1u << 21) - 1); }
GA_HD uint32_t key_s_ip(uint64_t k0) { return (uint32_t)k0; }
GA_HD uint32_t key_s_port17(uint64_t k1) { return (uint32_t)(k1 >> 47) & 0x1FFFFu; }
GA_HD uint32_t key_d_port17(uint64_t k1) { return (uint32_t)(k1 >> 30) & 0x1FFFFu; }
GA_HD uint32_t key_d_slot1(uint64_t k1) { return (uint32_t)(k1 >> 9) & ((1u << 21) - 1); }
GA_HD uint32_t key_d_ip(uint64_t k2) { return (uint32_t)(k2 >> 32); }
GA_HD uint32_t key_dns(uint64_t k2) { return (uint32_t)k2; }
GA_HD uint64_t key_hash(uint64_t k0, uint64_t k1, uint64_t k2) {
  return fmix64(k0 ^ fmix64(k1 ^ fmix64(k2 ^ 0x243F6A8885A308D3ULL)));
}
constexpr uint32_t kSparseMaxProbe = 1u << 16;
// compact table segments: 2^13 (key, count) slots = 128 KiB, folded in LDS
constexpr uint32_t kSparseSegLog2 = 13, kSparseMaxSegLists = 4096;
// Wide-key table segments (192-bit keys): 2^12 slots of 40 bytes = the 160 KiB LDS of one
// fold workgroup.  Probing wraps inside the segment, so a segment is folded alone
// (sparse_fold_wide_kernel); tables of up to 2^24 slots (4096 segments) take the
// per-segment lists, bigger ones probe the whole table with memory-side atomics.
constexpr uint32_t kWideSegLog2 = 12, kWideMaxLog2 = kWideSegLog2 + 12;
// A wide list entry: k0 k1 k2 and home << 52 | count << 40 | bytes -- home = the key's slot
// in its segment (key_hash & (2^kWideSegLog2 - 1)), so the fold does not hash the key again;
// updates whose count or bytes do not fit the fields go to the table directly
constexpr uint32_t kWideEntryWords = 4, kWideCountShift = 40, kWideHomeShift = 52;
static_assert(kWideHomeShift + kWideSegLog2 == 64, "home field fills the word");
// Narrow entries (plans with no port option and no DNS family, e.g. C1 / C4 remote): the
// key's port fields (k1 bits 30-63) and DNS id (k2 bits 0-31) are zero, so k1 and k2 pack
// into one word d_slot1 << 32 | d_ip -- 24 bytes an entry instead of 32 (GPUAGG_FLAG_NARROW_ENTRIES:
// the 24-byte entries are written as partial 32-byte sectors, so they win only while the
// lists stay small -- C1 -3 % per step, C4 remote +6 %, profiles/round6/exp/r6z6_*, r6fin2_d_*)
constexpr uint32_t kWideNarrowWords = 3;
GA_HD uint64_t wide_pack12(uint64_t k1, uint64_t k2) { return ((k1 >> 9) << 32) | (k2 >> 32); }
GA_HD uint64_t wide_unpack1(uint64_t n) { return (n >> 32) << 9; }
GA_HD uint64_t wide_unpack2(uint64_t n) { return (n & 0xFFFFFFFFULL) << 32; }
constexpr int kSparseEntryWords = 5;  // k0 k1 k2 count bytes

// ---- sketches ---------------------------------------------
constexpr uint64_t kCmsSeed = 0x5EED5EED5EED5EEDULL;
constexpr uint64_t kHllSeed = 0xA5A5A5A5DEADBEEFULL;
GA_HD uint64_t cms_base(uint32_t src, uint32_t dst, uint32_t ports, uint32_t proto) {
  const uint64_t lo = (uint64_t)src | ((uint64_t)dst << 32);
  const uint64_t hi = (uint64_t)ports | ((uint64_t)proto << 32);
  return fmix64(lo ^ fmix64(hi ^ kCmsSeed));
}
// Row r's column: double hashing of the 64-bit base (Kirsch & Mitzenmacher, "Less hashing,
// same performance"): h1 + r*h2 with h1, h2 the base's halves (h2 odd), so a record costs
// two 64-bit mixes, not one per row.
GA_HD uint32_t cms_col(uint64_t base, uint32_t row, uint32_t wmask) {
  const uint32_t h1 = (uint32_t)base, h2 = (uint32_t)(base >> 32) | 1u;
  return (h1 + row * h2) & wmask;
}
GA_HD uint64_t hll_hash(uint32_t dst) { return fmix64((uint64_t)dst ^ kHllSeed); }

}  // namespace gpuagg
