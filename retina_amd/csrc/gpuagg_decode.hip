// On-GPU decode of the producers' raw perf records into the SoA record columns
// (include/gpuagg.h "Raw perf records").
//
//  * packet_decode_kernel: struct packet of the packetparser program (72 bytes,
//    pkg/plugin/conntrack/_cprog/conntrack.c:34-49; Go mirror packetparserPacket,
//    packetparser_bpfel_x86.go:45-69), decoded as packetParser.processRecord does
//    (packetparser_linux.go:571-631).
//  * drop_decode_kernel: struct packet of the dropreason program (32 bytes,
//    pkg/plugin/dropreason/_cprog/drop_reason.c:39-54; kprobePacket,
//    kprobe_bpfel_x86.go:33-44), decoded as dropReason.processRecord does
//    (dropreason_linux.go:345-386).
//
// Both are HBM-streaming kernels: every raw byte is read once and the five u32
// columns are written once (packet: 72 B in + 20 B out per record; drop: 32 + 20).
// The 72-byte records are not 16-byte aligned per record, so a workgroup stages a
// tile of kTile records through LDS with coalesced dwordx4 loads and every lane then
// reads its record's six useful dwords from LDS (stride 18 dwords: 2-way bank
// conflicts at most).  The 32-byte drop records are two aligned dwordx4 loads per lane.
#include <hip/hip_runtime.h>

#include "gpuagg_internal.h"
#include "gpuagg_launch.h"

namespace gpuagg {
namespace {

constexpr uint32_t kDecodeThreads = 256;
constexpr uint32_t kTile = 512;                       // records per LDS tile
constexpr uint32_t kPacketWords = 18;                 // 72 bytes
constexpr uint32_t kTileVec = kTile * kPacketWords / 4;  // uint4 per tile (2304)

__device__ __forceinline__ uint32_t bswap16(uint32_t x) { return ((x & 0xFFu) << 8) | ((x >> 8) & 0xFFu); }

// utils.HostToNetShort on both ports (utils_linux.go:65-70), packed sport | dport << 16
// as flow.L4 carries them.
__device__ __forceinline__ uint32_t swap_ports(uint32_t w) { return bswap16(w & 0xFFFFu) | (bswap16(w >> 16) << 16); }

struct DecodeOut {
  uint32_t *src, *dst, *bytes, *meta, *ports, *dns;
  unsigned long long *out_of_range;
  uint32_t *tcp_id;  // latency columns, or null
  uint64_t *time_ns;
  uint64_t time_offset;
};

// Out-of-range rows never come from the eBPF programs: one atomic per lane that saw any.
__device__ __forceinline__ void count_out_of_range(uint32_t cnt, unsigned long long *ctr) {
  if (cnt) atomicAdd(ctr, (unsigned long long)cnt);
}

// One record of struct packet (dwords w[0..17]) -> columns.
//   w2 bytes (skb->len)        -> RetinaMetadata.Bytes  (AddPacketSize, :608)
//   w3/w4 src/dst ip           -> Int2ip(LE) as-is       (:585-586)
//   w5 src|dst port (LE u16)   -> HostToNetShort each    (:580-581)
//   w10 obs | tdir<<8 | proto<<16 | flags<<24
//   w11 is_reply (bool byte)   -> IsReply = byte != 0    (:600)
// meta: proto, verdict FORWARDED (:592), TrafficDirection = tdir (:603), TCP flags for
// TCP only (AddTCPFlags, flow_utils.go:136-149; bits FIN..URG, types_linux.go:22-31).
// A traffic direction above 3 does not fit the 2-bit field (conntrack.c only emits
// 0..2): the row is counted in out_of_range and gets verdict kVerdictUnencodable, which
// no metric consumes, rather than a wrong label (the sketches still see its 5-tuple).
__device__ __forceinline__ void packet_fields(const uint32_t *w, size_t i, const DecodeOut &o, bool &bad) {
  const uint32_t w10 = w[10], w11 = w[11];
  const uint32_t obs = w10 & 0xFFu, tdir = (w10 >> 8) & 0xFFu, proto = (w10 >> 16) & 0xFFu, flags = w10 >> 24;
  const uint32_t tcp_flags = proto == 6u ? (flags & 0x3Fu) : 0u;
  bad = tdir > 3u;
  // observation point (ToFlow, flow_utils.go:72-92) in bits 30-31: only 2 (FROM_NETWORK)
  // and 3 (TO_NETWORK) are read (latency), other points are written as 0
  const uint32_t meta = proto | ((bad ? kVerdictUnencodable : kVerdictForwarded) << 8) | ((tdir & 3u) << 16) |
                        (tcp_flags << 21) | ((w11 & 0xFFu) ? (1u << 27) : 0u) | ((obs <= 3u ? obs : 0u) << 30);
  o.src[i] = w[3];
  o.dst[i] = w[4];
  o.bytes[i] = w[2];
  o.meta[i] = meta;
  if (o.ports) o.ports[i] = swap_ports(w[5]);
  if (o.dns) o.dns[i] = 0xFFFFFFFFu;
  // TcpId: TSval (w8) on TO_NETWORK, TSecr (w9) on FROM_NETWORK (:622-628); t_nsec (w0-1)
  if (o.tcp_id) o.tcp_id[i] = obs == 3u ? w[8] : obs == 2u ? w[9] : 0u;
  if (o.time_ns) o.time_ns[i] = ((uint64_t)w[0] | ((uint64_t)w[1] << 32)) + o.time_offset;
}

__global__ __launch_bounds__(kDecodeThreads) void packet_decode_kernel(const uint4 *raw, size_t n,
                                                                       DecodeOut o) {
  __shared__ uint4 tile[kTileVec];
  const uint32_t *tw = (const uint32_t *)tile;
  const size_t ntiles = (n + kTile - 1) / kTile;
  uint32_t n_bad = 0;
  for (size_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const size_t r0 = t * kTile;
    const uint32_t nrec = (uint32_t)(n - r0 < kTile ? n - r0 : kTile);
    if (nrec == kTile) {
      const uint4 *g = raw + t * kTileVec;
#pragma unroll
      for (uint32_t k = 0; k < kTileVec / kDecodeThreads; ++k)  // 9 coalesced dwordx4 per lane
        tile[threadIdx.x + k * kDecodeThreads] = g[threadIdx.x + k * kDecodeThreads];
    } else {
      // partial last tile: dword loads up to the end of the batch
      const uint32_t *g = (const uint32_t *)raw + r0 * kPacketWords;
      uint32_t *tl = (uint32_t *)tile;
      for (uint32_t k = threadIdx.x; k < nrec * kPacketWords; k += kDecodeThreads) tl[k] = g[k];
    }
    __syncthreads();
    for (uint32_t r = threadIdx.x; r < nrec; r += kDecodeThreads) {
      const uint32_t *w = tw + r * kPacketWords;
      bool bad;
      packet_fields(w, r0 + r, o, bad);
      n_bad += bad;
    }
    __syncthreads();
  }
  count_out_of_range(n_bad, o.out_of_range);
}

// One struct packet of dropreason (dwords d[0..7]):
//   d0/d1 src/dst ip, d2 src|dst port, d3 skb_len, d4 return_val,
//   d5 drop_type | proto << 16 | in_filtermap << 24, d6-7 ts
// -> ToFlow(obs 2 => INGRESS, DROPPED) (:358-368), IsReply nil (:374), AddDropReason
// (drop_type, :379), AddPacketSize(skb_len) (:382).  No TCP flags.  drop_type above 7
// does not fit the 3-bit field (drop_reason.h's enum is 0..6): counted, and the row gets
// verdict kVerdictUnencodable like an out-of-range packet row.
__global__ __launch_bounds__(kDecodeThreads) void drop_decode_kernel(const uint4 *raw, size_t n,
                                                                     DecodeOut o) {
  uint32_t n_bad = 0;
  for (size_t i = (size_t)blockIdx.x * kDecodeThreads + threadIdx.x; i < n;
       i += (size_t)gridDim.x * kDecodeThreads) {
    const uint4 a = raw[2 * i], b = raw[2 * i + 1];
    const uint32_t drop_type = b.y & 0xFFFFu, proto = (b.y >> 16) & 0xFFu;
    const bool bad = drop_type > 7u;
    n_bad += bad;
    o.src[i] = a.x;
    o.dst[i] = a.y;
    o.bytes[i] = a.w;
    o.meta[i] = proto | ((bad ? kVerdictUnencodable : kVerdictDropped) << 8) | (1u << 16) |
                ((drop_type & 7u) << 18) | (2u << 30);  // ToFlow(obs 2): FROM_NETWORK
    if (o.ports) o.ports[i] = swap_ports(a.z);
    if (o.dns) o.dns[i] = 0xFFFFFFFFu;
    if (o.tcp_id) o.tcp_id[i] = 0u;  // dropreason sets no TcpId
    if (o.time_ns) o.time_ns[i] = ((uint64_t)b.z | ((uint64_t)b.w << 32)) + o.time_offset;
  }
  count_out_of_range(n_bad, o.out_of_range);
}

}  // namespace

hipError_t launch_decode(const DecodeArgs &a, hipStream_t st) {
  if (a.n == 0) return hipSuccess;
  const DecodeOut o{a.out.src_ip, a.out.dst_ip, a.out.bytes, a.out.meta, a.out.ports, a.out.dns_id,
                    (unsigned long long *)a.out_of_range, a.out.tcp_id, a.out.time_ns, a.time_offset};
  const uint32_t cap = a.n_cu * 8u;  // enough resident workgroups to cover HBM latency
  if (a.kind == kRawPacket) {
    const size_t tiles = (a.n + kTile - 1) / kTile;
    const uint32_t blocks = (uint32_t)(tiles < cap ? tiles : cap);
    hipLaunchKernelGGL(packet_decode_kernel, dim3(blocks), dim3(kDecodeThreads), 0, st,
                       (const uint4 *)a.raw, a.n, o);
  } else {
    const size_t need = (a.n + kDecodeThreads - 1) / kDecodeThreads;
    const uint32_t blocks = (uint32_t)(need < cap ? need : cap);
    hipLaunchKernelGGL(drop_decode_kernel, dim3(blocks), dim3(kDecodeThreads), 0, st,
                       (const uint4 *)a.raw, a.n, o);
  }
  return hipGetLastError();
}

}  // namespace gpuagg
