"""Diagnostic: phase times of gpuagg_snapshot / render_text on stderr when GA_TR is set."""
import sys

p = sys.argv[1] + "/gpuagg_runtime.cpp"
s = open(p).read()


def rep(old, new):
    global s
    assert old in s, old
    s = s.replace(old, new, 1)


rep('''  // canonical slot attributes per option mask (cached until the slots change)''', '''  auto T1 = std::chrono::steady_clock::now();
  auto L2 = [&](const char *w) { if (getenv("GA_TR")) fprintf(stderr, "    rs %s %.1f\\n", w, std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - T1).count()); };
  // canonical slot attributes per option mask (cached until the slots change)''')
rep('''  // items: one per (counter, view), partitioned by key hash''', '''  L2("canon");
  // items: one per (counter, view), partitioned by key hash''')
rep('''  for (int e : err)
    if (e) return fail(c, e, "snapshot: a group-by''', '''  L2("items");
  for (int e : err)
    if (e) return fail(c, e, "snapshot: a group-by''')
rep('''  // concatenate the partitions
''', '''  L2("agg+arena");
  // concatenate the partitions
''')
rep('''    std::vector<char> &ar = r->arenas[p];
    std::vector<uint32_t> &tk = r->toks[p];''', '''    if (p == 0) L2("agg0");
    std::vector<char> &ar = r->arenas[p];
    std::vector<uint32_t> &tk = r->toks[p];''')
rep('''  int rc = gpuagg_sync(c);
  if (rc) return rc;

  // dense counters''', '''  auto TT0 = std::chrono::steady_clock::now();
  int rc = gpuagg_sync(c);
  if (rc) return rc;
  if (getenv("GA_TR")) fprintf(stderr, "  synced %.1f\\n", std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - TT0).count());

  // dense counters''')
rep('''  auto *r = new gpuagg_result();
  r->dropped = c->stats.sparse_dropped;''', '''  if (getenv("GA_TR")) fprintf(stderr, "  copied %.1f nent %zu\\n", std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - TT0).count(), nent);
  auto *r = new gpuagg_result();
  r->dropped = c->stats.sparse_dropped;''')
rep('''      sort_family(r, F, idx, j.T, perms[f]);''', '''      auto a0 = std::chrono::steady_clock::now(); sort_family(r, F, idx, j.T, perms[f]); if (getenv("GA_TR")) fprintf(stderr, "   sort n=%zu nl=%zu %.1f\\n", n, nl, std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a0).count());''')
rep('''  uint64_t N = 0;
  for (Job &j : jobs) {''', '''  auto W0 = std::chrono::steady_clock::now();
  uint64_t N = 0;
  for (Job &j : jobs) {''')
rep('''  r->text_done = true;
}''', '''  r->text_done = true;
  if (getenv("GA_TR")) fprintf(stderr, "   write %.1f\\n", std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - W0).count());
}''')
open(p, "w").write(s)
