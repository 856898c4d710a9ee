"""Round-6 ablations of dense_lds_kernel (timing only; results are wrong):
   nospill   records of spilled groups are not queued (no SpillQ pushes / flushes)
   noflush   no end-of-kernel store of the workgroup's bins (staged or atomic)
   noatomic  the forward bins are read (ds_read) instead of added (ds_add_rtn)
   nolookup  slots from a hash of the IP instead of the LDS image reads
usage: patch_abl.py SRC_DIR WHAT[,WHAT...]"""
import sys

src, what = sys.argv[1], sys.argv[2].split(",")
p = src + "/gpuagg_kernels.hip"
s = open(p).read()


def rep(old, new, count=1):
    global s
    assert s.count(old) >= 1, old
    s = s.replace(old, new, count)


k0 = s.index("__global__ __launch_bounds__(1024) void dense_lds_kernel(KArgs a)")
head, body = s[:k0], s[k0:]
s = body
if "noqflush" in what:  # records are queued, the full queue is dropped
    rep("""        if (full) {
          q_flush(true);""", """        if (full) {
          if (a.n == 3) q_flush(true);""")
if "nospill" in what:
    rep("      l4_records<NG, SIG, 4, 1>(G, l4, ds, by, me, ss, sd);\n",
        "      l4_records<NG, SIG, 4, 1>(G, l4, ds, by, me, ss, sd);\n      if (a.n) continue;\n")
if "noflush" in what:
    rep("  if (a.stage_a) {\n    // staged flush", "  if (a.n == 3) {\n    // staged flush")
    rep("  } else {\n    // flush group by group", "  } else if (a.n == 5) {\n    // flush group by group")
if "nolookup" in what:
    rep("      iv.lookup8(ip, act, sl);",
        "#pragma unroll\n      for (int q = 0; q < 8; ++q) sl[q] = act ? ((ip[q] * 2654435761u) >> 16) % 10000u : kIplNoSlot;")
body = s
s = head
if "nostore" in what:  # spill_put reserves and returns without the store
    rep("""      spill[mul_u24(w, spill_cap) + pos] = entry(bin, nbytes);
      return;
    }
    atomicAdd(&d.cnt[bin], 1ULL);""", """      if (pos == 0xFFFFFFFFu) spill[mul_u24(w, spill_cap) + pos] = entry(bin, nbytes);
      return;
    }
    atomicAdd(&d.cnt[bin], 1ULL);""")
if "noatomic" in what:
    rep("          od[k] = atomicAdd(&l4.bins[vd[k] ? bd[k] : l4.dummy], add);\n"
        "          os[k] = atomicAdd(&l4.bins[vs[k] ? bs[k] : l4.dummy], add);",
        "          od[k] = l4.bins[vd[k] ? bd[k] : l4.dummy] + (add & 1u);\n"
        "          os[k] = l4.bins[vs[k] ? bs[k] : l4.dummy] + (add & 1u);")
s = s + body
open(p, "w").write(s)
