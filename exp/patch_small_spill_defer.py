"""Experiment: defer the spill folds of small spill-only launches (C2/C4 plans at <= 2^16
records per workgroup, e.g. the Go plugin's 2^20-record batches) across up to 16 launches,
as compact-list plans already do.  In production geometry the C2 fold (spill_window_kernel
+ stage_reduce_kernel, 0.026 ms) costs more per launch than the tier-1 kernel (0.016 ms).
Not yet run on a GPU: apply with exp/variant.py, then tests -k deferred,parity and the
`production` object of bench.py --config c2."""
import sys

p = sys.argv[1] + "/gpuagg_runtime.cpp"
s = open(p).read()
old = "    // Only plans with compact-key lists defer: their fold pays a fixed pass over the\n    // group-by table.  Spill-only plans (C2, C4) fold per batch -- their fold is\n    // proportional to the entries, and appending past earlier launches' entries measured\n    // ~2 % slower in the tier-1 kernel (profiles/round2/r4f_*).\n    const bool lists = sp_lists;\n    const bool defer = c->defer_folds && lists;\n    // Wide lists (192-bit keys) are folded when the device says so: every launch's fold\n    // skips itself until some list is half full (sparse_fold_wide_kernel), so the host keeps\n    // appending without a record budget -- under skew the LDS hot-key cache absorbs most\n    // updates and a budget that assumes one entry per record folded ~5x too often.\n    const bool fold_cond = defer && !c->sv.compact;\n"
new = "    // Plans with compact-key lists always defer: their fold pays a fixed pass over the\n    // group-by table.  Spill-only plans (C2, C4) defer only small launches (at most\n    // kMaxRecordsPerBlock / kDeferLaunches records per workgroup, e.g. the Go plugin's 2^20\n    // records): there the spill fold's fixed pass over the windows cost more than the\n    // tier-1 kernel itself; at full-size launches appending past earlier launches' entries\n    // measured ~2 % slower in the tier-1 kernel (profiles/round2/r4f_*), so they fold per batch.\n    const bool small_spill = c->dense_len > a.lds_bins && a.chunk * kDeferLaunches <= kMaxRecordsPerBlock;\n    const bool lists = sp_lists || small_spill;\n    const bool defer = c->defer_folds && lists;\n    // Wide lists (192-bit keys) are folded when the device says so: every launch's fold\n    // skips itself until some list is half full (sparse_fold_wide_kernel), so the host keeps\n    // appending without a record budget -- under skew the LDS hot-key cache absorbs most\n    // updates and a budget that assumes one entry per record folded ~5x too often.\n    const bool fold_cond = defer && sp_lists && !c->sv.compact;\n"
assert old in s
open(p, "w").write(s.replace(old, new))
