// Hubble-mode L3/L4 enrichment on the GPU (row (f)-4): per flow record, the source and
// destination endpoints from an image of the ipcache and the summary of
// pkg/hubble/parser/layer34/parser_linux.go (or seven/ for DNS flows) as codes.
//
// Reference, per flow (one goroutine): Parser._decode (parser_linux.go:64-93) sends
// L3/L4 flows to layer34.Decode (:30-57) and L7 flows to seven.Decode; both replace
// Source / Destination with epDecoder.Decode (common/decoder_linux.go:32-60): identity =
// ipcache.LookupByIP or World, PodName / Namespace from the ipcache's K8s metadata.
// decodeSummary (:59-84): DROPPED -> "Drop Reason: ..." ; TCP with flags -> "TCP Flags: .."
// ; UDP -> "UDP"; DNS (seven, :117-146) -> the query / answer summary.
//
// Here the ipcache is an open-addressed table of 16-byte entries (ip, identity, K8s
// metadata id, 0) in HBM (a few MB at most, L2-resident); one lane per record, the
// strings are rendered by the host from the codes (oracle/hubble.py render_summary).
// HBM-bound: 12-16 B read + 24 B written per record.
#include <hip/hip_runtime.h>

#include "gpuagg_internal.h"
#include "gpuagg_launch.h"

namespace gpuagg {

__device__ __forceinline__ uint2 ipc_lookup(const HubbleArgs &a, uint32_t ip) {
  uint32_t h = ip_h1(ip, a.seed) & a.mask;
  for (uint32_t p = 0; p <= a.max_probe; ++p, h = (h + 1) & a.mask) {
    const uint4 e = a.table[h];
    if (e.x == ip) return make_uint2(e.y, e.z);
    if (e.x == kIpcEmpty) break;
  }
  return make_uint2(kIdentityWorld, kIpcNoMeta);  // LookupByIP miss: World, no metadata
}

__global__ __launch_bounds__(256) void hubble_decode_kernel(HubbleArgs a) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < a.n; i += (size_t)gridDim.x * blockDim.x) {
    const uint2 s = ipc_lookup(a, a.src[i]), d = ipc_lookup(a, a.dst[i]);
    a.o_sid[i] = s.x;
    a.o_did[i] = d.x;
    a.o_smeta[i] = s.y;
    a.o_dmeta[i] = d.y;
    const uint32_t m = a.meta[i], proto = meta_proto(m), verdict0 = meta_verdict(m);
    const uint32_t verdict = verdict0 == 0u ? kVerdictForwarded : verdict0;  // ToFlow (flow_utils.go:94-96)
    uint32_t kind = kSummaryNone, arg = 0;
    if (verdict == kVerdictDns) {  // L7: seven.Parser (DNS summary from the dictionary)
      kind = kSummaryDns;
      arg = (a.dns ? a.dns[i] & 0x3FFFFFFFu : 0u) | (meta_dnstype(m) << 30);
    } else if (verdict == kVerdictDropped) {
      kind = kSummaryDrop;
      arg = meta_reason(m);
    } else if (proto == 6) {  // flags exist on forwarded / retransmitted TCP flows
      if (verdict == kVerdictForwarded || verdict == kVerdictRetrans) {
        kind = kSummaryTcp;
        arg = meta_flags(m);
      }
    } else if (proto == 17) {
      kind = kSummaryUdp;
    }
    a.o_kind[i] = kind;
    a.o_arg[i] = arg;
  }
}

hipError_t launch_hubble(const HubbleArgs &a, uint32_t n_cu, hipStream_t st) {
  if (a.n == 0) return hipSuccess;
  const size_t need = (a.n + 255) / 256;
  const uint32_t blocks = (uint32_t)(need < (size_t)n_cu * 16 ? need : (size_t)n_cu * 16);
  hipLaunchKernelGGL(hubble_decode_kernel, dim3(blocks), dim3(256), 0, st, a);
  return hipGetLastError();
}

}  // namespace gpuagg
