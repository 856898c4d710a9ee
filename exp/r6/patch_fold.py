"""Round-6 ablations of sparse_fold_wide_kernel (timing only; results are wrong):
   noins   list entries are loaded but not inserted (XOR-folded into a register)
   nolist  the lists are not read (segment load + store only)
   noseg   the segment is zero-filled in LDS instead of loaded, and not stored back
usage: patch_fold.py SRC_DIR WHAT[,WHAT...]"""
import sys

src, what = sys.argv[1], sys.argv[2].split(",")
p = src + "/gpuagg_kernels.hip"
s = open(p).read()
k0 = s.index("void sparse_fold_wide_kernel(")
k1 = s.index("// Dense local-context fast path", k0)
head, body, tail = s[:k0], s[k0:k1], s[k1:]


def rep(old, new):
    global body
    assert body.count(old) == 1, old
    body = body.replace(old, new)


if "noins" in what:
    rep("  auto ins = [&](const ulonglong2 &a0, const ulonglong2 &a1) {\n    insert(",
        "  unsigned long long acc = 0;\n  auto ins = [&](const ulonglong2 &a0, const ulonglong2 &a1) {\n"
        "    acc ^= a0.x ^ a0.y ^ a1.x ^ a1.y;\n    if (acc == 0x5A5A5A5A5A5A5A5AULL) insert(")
if "nolist" in what:
    rep("for (uint32_t l0 = 0; l0 < n_lists; l0 += lists_per_round) {",
        "for (uint32_t l0 = 0; l0 < (s.mask == 7u ? n_lists : 0u); l0 += lists_per_round) {")
if "noseg" in what:
    rep("for (int q = 0; q < 4; ++q) v[q] = g[j0 + q * blockDim.x];",
        "for (int q = 0; q < 4; ++q) v[q] = s.mask == 7u ? g[j0 + q * blockDim.x] : 0ULL;")
    rep("    seg[f * N + slot] = g[j0];", "    seg[f * N + slot] = 0ULL;")
    rep("    g[j] = seg[f * N + slot];", "    if (s.mask == 7u) g[j] = seg[f * N + slot];")
open(p, "w").write(head + body + tail)
