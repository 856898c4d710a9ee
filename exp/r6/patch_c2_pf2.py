"""Experiment (round 6): dense_lds_kernel keeps TWO steps of record loads in flight (A/B
register sets, loop unrolled by 2) instead of one."""
import sys

p = sys.argv[1] + "/gpuagg_kernels.hip"
s = open(p).read()
a = s.index("    uint64_t vl = vwave + lane < vend ? vwave + lane : vlast;\n    uint4 ns = rec_ld(&s4[vl])")
b = s.index("    tail = start + (vn << 2);", a)
body_start = s.index("      const uint32_t ip[8] = {vs.x", a)
body_end = s.index("\n    }\n", body_start)  # end of the for loop body
body = s[body_start:body_end].replace("        continue;\n", "        return;\n")
new = """    auto step = [&](uint64_t vw, const uint4 vs, const uint4 vd, const uint4 vb, const uint4 vm) {
      const bool act = vw + lane < vend;
""" + body + """
    };
    const uint64_t W = blockDim.x;
    auto cl = [&](uint64_t v) { return v < vend ? v : vlast; };
    uint64_t vl = cl(vwave + lane);
    uint4 as = rec_ld(&s4[vl]), ad = rec_ld(&d4[vl]), ab = rec_ld(&b4[vl]), am = rec_ld(&m4[vl]);
    vl = cl(vwave + W + lane);
    uint4 bs = rec_ld(&s4[vl]), bd = rec_ld(&d4[vl]), bb = rec_ld(&b4[vl]), bm = rec_ld(&m4[vl]);
    for (uint64_t vw = vwave; vw < vend; vw += 2 * W) {
      {
        const uint4 xs = as, xd = ad, xb = ab, xm = am;
        vl = cl(vw + 2 * W + lane);
        as = rec_ld(&s4[vl]);
        ad = rec_ld(&d4[vl]);
        ab = rec_ld(&b4[vl]);
        am = rec_ld(&m4[vl]);
        step(vw, xs, xd, xb, xm);
      }
      if (vw + W >= vend) break;
      {
        const uint4 xs = bs, xd = bd, xb = bb, xm = bm;
        vl = cl(vw + 3 * W + lane);
        bs = rec_ld(&s4[vl]);
        bd = rec_ld(&d4[vl]);
        bb = rec_ld(&b4[vl]);
        bm = rec_ld(&m4[vl]);
        step(vw + W, xs, xd, xb, xm);
      }
    }
"""
s = s[:a] + new + s[b:]
open(p, "w").write(s)
