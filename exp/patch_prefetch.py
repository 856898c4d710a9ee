"""Experiment: for_each_record loads the next step's record columns one step ahead."""
import sys

p = sys.argv[1] + "/gpuagg_kernels.hip"
s = open(p).read()
old_loop = """    for (uint64_t vblk = v0; kRounds ? vblk < vend : vblk + wave0 < vend; vblk += blockDim.x) {
      const uint64_t vw = vblk + wave0;
      const bool act = vw + lane < vend;
      const uint64_t v = act ? vw + lane : vlast;
      const uint4 vs = rec_ld(&s4[v]), vd = rec_ld(&d4[v]), vm = rec_ld(&m4[v]);
      const uint4 vb = need_bytes ? b4[v] : make_uint4(0, 0, 0, 0);
      const uint4 vp = need_ports ? p4[v] : make_uint4(0, 0, 0, 0);
      const uint4 vq = need_dns ? rec_ld(&q4[v]) : make_uint4(0, 0, 0, 0);
"""
new_loop = """    uint4 ns, nd, nm, nb, np_, nq;
    auto ldn = [&](uint64_t vn) {
      const uint64_t v = vn < vend ? vn : vlast;
      ns = rec_ld(&s4[v]); nd = rec_ld(&d4[v]); nm = rec_ld(&m4[v]);
      nb = need_bytes ? b4[v] : make_uint4(0, 0, 0, 0);
      np_ = need_ports ? p4[v] : make_uint4(0, 0, 0, 0);
      nq = need_dns ? rec_ld(&q4[v]) : make_uint4(0, 0, 0, 0);
    };
    ldn(v0 + wave0 + lane);
    for (uint64_t vblk = v0; kRounds ? vblk < vend : vblk + wave0 < vend; vblk += blockDim.x) {
      const uint64_t vw = vblk + wave0;
      const bool act = vw + lane < vend;
      const uint4 vs = ns, vd = nd, vm = nm, vb = nb, vp = np_, vq = nq;
      ldn(vw + blockDim.x + lane);
"""
assert old_loop in s
s = s.replace(old_loop, new_loop)
open(p, "w").write(s)
