"""Probe: C3's deferred sketch folds with cms_fold_kernel on a second stream beside the
HLL split + fold (they touch disjoint state), joined back before the call returns."""
import sys

p = sys.argv[1] + "/gpuagg_kernels.hip"
s = open(p).read()


def rep(old, new):
    global s
    assert old in s, old
    s = s.replace(old, new, 1)


rep("""  if (a.nwin && a.cms_depth) {
    names += names.empty() ? "cms_fold_kernel" : "+cms_fold_kernel";""", """  static hipStream_t side = nullptr;
  static hipEvent_t fork_ev = nullptr, join_ev = nullptr;
  const bool fork = a.nwin && a.cms_depth && a.hll_nsup && a.hll_p;
  hipStream_t cst = st;
  if (fork) {
    if (!side) {
      hipStreamCreateWithFlags(&side, hipStreamNonBlocking);
      hipEventCreateWithFlags(&fork_ev, hipEventDisableTiming);
      hipEventCreateWithFlags(&join_ev, hipEventDisableTiming);
    }
    hipEventRecord(fork_ev, st);
    hipStreamWaitEvent(side, fork_ev, 0);
    cst = side;
  }
  if (a.nwin && a.cms_depth) {
    names += names.empty() ? "cms_fold_kernel" : "+cms_fold_kernel";""")
rep("""    hipLaunchKernelGGL(cms_fold_kernel, dim3(a.fold_blocks), dim3(1024), lds, st, k, a.blocks);""",
    """    hipLaunchKernelGGL(cms_fold_kernel, dim3(a.fold_blocks), dim3(1024), lds, cst, k, a.blocks);""")
rep("""    hipLaunchKernelGGL(hll_fold_kernel, dim3(a.hll_nwin), dim3(1024), lds, st, k);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  if (kernels) *kernels = names;""", """    hipLaunchKernelGGL(hll_fold_kernel, dim3(a.hll_nwin), dim3(1024), lds, st, k);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  if (fork) {
    hipEventRecord(join_ev, side);
    hipStreamWaitEvent(st, join_ev, 0);
  }
  if (kernels) *kernels = names;""")
open(p, "w").write(s)
