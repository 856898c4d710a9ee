"""Vectorised decode of the producers' raw perf records (TEST INFRASTRUCTURE ONLY).

numpy restatement of the two decoders the engine runs on the GPU
(retina_amd/csrc/gpuagg_decode.hip), producing the SoA column batch of
``oracle/records.py``.  It is pinned to the per-record restatements
``oracle.decode_packet`` / ``oracle.decode_drop`` (tests/test_decode_oracle.py:
every decoded row replays to the same flow.Flow fields), which follow:

* packetparser: struct packet (pkg/plugin/conntrack/_cprog/conntrack.c:34-49,
  Go mirror packetparser_bpfel_x86.go:45-69), packetParser.processRecord
  (pkg/plugin/packetparser/packetparser_linux.go:571-631);
* dropreason: struct packet (pkg/plugin/dropreason/_cprog/drop_reason.c:39-54,
  kprobePacket kprobe_bpfel_x86.go:33-44), dropReason.processRecord
  (pkg/plugin/dropreason/dropreason_linux.go:345-386).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may import this.
"""

from __future__ import annotations

from typing import Tuple

import numpy as np

from . import records as R

PACKET_SIZE, DROP_SIZE = 72, 32

# little-endian field offsets of struct packet (packetparser), conntrack.c:34-49
PACKET_DTYPE = np.dtype({
    "names": ["t_nsec", "bytes", "src_ip", "dst_ip", "src_port", "dst_port", "seq", "ack_num",
              "tsval", "tsecr", "obs", "tdir", "proto", "flags", "is_reply",
              "bytes_fwd", "bytes_rep", "pkts_fwd", "pkts_rep"],
    "formats": ["<u8", "<u4", "<u4", "<u4", "<u2", "<u2", "<u4", "<u4", "<u4", "<u4",
                "u1", "u1", "u1", "u1", "u1", "<u8", "<u8", "<u4", "<u4"],
    "offsets": [0, 8, 12, 16, 20, 22, 24, 28, 32, 36, 40, 41, 42, 43, 44, 48, 56, 64, 68],
    "itemsize": PACKET_SIZE})

# struct packet (dropreason), drop_reason.c:39-54
DROP_DTYPE = np.dtype({
    "names": ["src_ip", "dst_ip", "src_port", "dst_port", "skb_len", "return_val", "drop_type",
              "proto", "in_filtermap", "ts"],
    "formats": ["<u4", "<u4", "<u2", "<u2", "<u4", "<u4", "<u2", "u1", "u1", "<u8"],
    "offsets": [0, 4, 8, 10, 12, 16, 20, 22, 23, 24],
    "itemsize": DROP_SIZE})


def _swap16(x: np.ndarray) -> np.ndarray:
    """utils.HostToNetShort (utils_linux.go:65-70)."""
    x = x.astype(np.uint32)
    return ((x & 0xFF) << 8) | (x >> 8)


def decode_packets(raw: np.ndarray) -> Tuple[R.Batch, np.ndarray]:
    """Raw packetparser records -> (column batch, out-of-range mask).

    verdict FORWARDED (:592), TrafficDirection = traffic_direction (:603), IsReply
    (:600), AddPacketSize(bytes) (:608), AddTCPFlags for TCP only (:612-620 with
    flow_utils.go:136-149).  traffic_direction > 3 does not fit the meta word: the row
    gets verdict 255 (consumed by no metric) and is flagged."""
    r = np.frombuffer(np.ascontiguousarray(raw).view(np.uint8).tobytes(), PACKET_DTYPE)
    u = np.uint32
    proto = r["proto"].astype(u)
    tdir = r["tdir"].astype(u)
    flags = np.where(proto == 6, r["flags"].astype(u) & u(0x3F), u(0))
    bad = tdir > 3
    obs = r["obs"].astype(u)
    meta = R.pack_meta_np(proto, np.where(bad, u(255), u(1)), tdir, 0, flags, (r["is_reply"] != 0).astype(u), 0,
                          obs)
    ports = _swap16(r["src_port"]) | (_swap16(r["dst_port"]) << u(16))
    # TcpId: TSval on TO_NETWORK (3), TSecr on FROM_NETWORK (2) (:622-628)
    tcp_id = np.where(obs == 3, r["tsval"], np.where(obs == 2, r["tsecr"], 0)).astype(u)
    b = R.Batch(r["src_ip"].astype(u), r["dst_ip"].astype(u), r["bytes"].astype(u), meta, ports,
                np.full(len(r), 0xFFFFFFFF, u), tcp_id, r["t_nsec"].astype(np.uint64))
    return b, bad


def decode_drops(raw: np.ndarray) -> Tuple[R.Batch, np.ndarray]:
    """Raw dropreason records -> (column batch, out-of-range mask).

    ToFlow(obs 2 -> INGRESS, DROPPED) (:358-368), AddDropReason(drop_type) (:379),
    AddPacketSize(skb_len) (:382); no TCP flags, IsReply nil.  drop_type > 7 gets
    verdict 255 and is flagged."""
    r = np.frombuffer(np.ascontiguousarray(raw).view(np.uint8).tobytes(), DROP_DTYPE)
    u = np.uint32
    proto = r["proto"].astype(u)
    dt = r["drop_type"].astype(u)
    bad = dt > 7
    meta = R.pack_meta_np(proto, np.where(bad, u(255), u(2)), 1, dt, 0, 0, 0, 2)  # ToFlow(obs 2)
    ports = _swap16(r["src_port"]) | (_swap16(r["dst_port"]) << u(16))
    b = R.Batch(r["src_ip"].astype(u), r["dst_ip"].astype(u), r["skb_len"].astype(u), meta, ports,
                np.full(len(r), 0xFFFFFFFF, u), np.zeros(len(r), u), r["ts"].astype(np.uint64))
    return b, bad
