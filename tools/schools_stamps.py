#!/usr/bin/env python3
"""Where the fused 8-schools kernel's time goes: a DIAGNOSTIC build of libstark_hip.so whose
nuts.hip carries s_memtime stamps (MI355X guide, DVFS give-back item 6: stamps in a separate
build, their values only in a buffer of their own).  The product source is not changed: this
script writes an instrumented copy of stark_amd/csrc to tools/_bin/stamp_src, builds it into
tools/_bin/stamp_lib (`build`), and on the GPU box (`run`) runs tools/bench_schools.py's
configuration on it and prints, per chain-step, the cycles spent in: the gradient
(schools_lpgrad), consume() in total, and inside on_leaf: the leaf's own bookkeeping, the
sub-tree merge loop, the push of a pending sub-tree, the top-level completion, and
end_transition (which starts the next transition).  Stamps add their own cycles (≈ 10 %).

usage: tools/schools_stamps.py build | run"""
import ctypes
import os
import re
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "stark_amd", "csrc")
OUT = os.path.join(ROOT, "tools", "_bin", "stamp_src")
LIB = os.path.join(ROOT, "tools", "_bin", "stamp_lib")
REGIONS = ["gradient", "consume", "leaf_pre", "merge_loop", "push", "top_level", "end_transition", "steps"]


def instrument(s):
    def sub(old, new, count=1):
        nonlocal s
        assert s.count(old) >= count, old
        s = s.replace(old, new)
    sub("namespace stk {\n", "namespace stk {\n__device__ unsigned long long stk_stamp_acc[8192 * 8];\n"
        "__device__ __forceinline__ unsigned long long stamp() { return __builtin_amdgcn_s_memtime(); }\n", 1)
    # per-chain accumulators in NutsChain
    sub("  uint32_t nleap = 0, ndiv = 0;", "  uint32_t nleap = 0, ndiv = 0;\n  unsigned long long stp[8] = {0, 0, 0, 0, 0, 0, 0, 0};\n"
        "  __device__ __forceinline__ bool endt(int pause_at) {\n"
        "    const unsigned long long t = stamp();\n    const bool r = end_transition(pause_at);\n"
        "    stp[6] += stamp() - t;\n    return r;\n  }")
    body_start = s.index("  __device__ __forceinline__ bool on_leaf(")
    body_end = s.index("  // Consume the evaluation requested last step.")
    leaf = s[body_start:body_end]
    leaf = leaf.replace("    finish_leapfrog(lp, glp);\n    ++nleap;", "    const unsigned long long tl0 = stamp();\n    finish_leapfrog(lp, glp);\n    ++nleap;", 1)
    leaf = leaf.replace("    bool stop = IV(I_DIV) != 0;\n", "    stp[2] += stamp() - tl0;\n    bool stop = IV(I_DIV) != 0;\n", 1)
    leaf = leaf.replace("    int j = 0;\n", "    const unsigned long long tm0 = stamp();\n    int j = 0;\n", 1)
    leaf = leaf.replace("    if (!stop && j < depth) {\n", "    stp[3] += stamp() - tm0;\n    if (!stop && j < depth) {\n      const unsigned long long tp0 = stamp();\n", 1)
    leaf = leaf.replace("      begin_leapfrog(IV(I_DIR) * S(S_EPS));\n      return true;\n    }",
                        "      begin_leapfrog(IV(I_DIR) * S(S_EPS));\n      stp[4] += stamp() - tp0;\n      return true;\n    }", 1)
    leaf = leaf.replace("      // the top-level sub-tree of this depth is complete and valid\n",
                        "      // the top-level sub-tree of this depth is complete and valid\n      const unsigned long long tt0 = stamp();\n", 1)
    leaf = leaf.replace("      if (!stop) {\n        begin_subtree();\n        return true;\n      }\n    }\n    return end_transition(pause_at);",
                        "      stp[5] += stamp() - tt0;\n      if (!stop) {\n        begin_subtree();\n        return true;\n      }\n    }\n    return endt(pause_at);", 1)
    assert leaf.count("stamp()") == 8, leaf.count("stamp()")
    s = s[:body_start] + leaf + s[body_end:]
    # the fused loop
    sub("        const double lp = schools_lpgrad<NCH, SEG, true>(yc, isc, ch.q, glp, lane, ch.D, mtab, &ch.mk);\n        ++steps;\n        req = ch.consume(lp, glp, pause_at);",
        "        const unsigned long long t0 = stamp();\n"
        "        const double lp = schools_lpgrad<NCH, SEG, true>(yc, isc, ch.q, glp, lane, ch.D, mtab, &ch.mk);\n"
        "        const unsigned long long t1 = stamp();\n        ++steps;\n        req = ch.consume(lp, glp, pause_at);\n"
        "        ch.stp[0] += t1 - t0;\n        ch.stp[1] += stamp() - t1;\n        ch.stp[7] += 1;")
    sub("      ch.save();\n      ch.flush_counts();\n      if (req) ch.st(A.qeval + (size_t)gid * A.Dp, ch.q);",
        "      ch.save();\n      ch.flush_counts();\n      if (lane == 0 && gid < 8192)\n"
        "        for (int i = 0; i < 8; ++i) stk_stamp_acc[(size_t)gid * 8 + i] += ch.stp[i];\n"
        "      if (req) ch.st(A.qeval + (size_t)gid * A.Dp, ch.q);")
    # nuts.hip is compiled twice (nuts.o, and nuts_fused4.o for the 4-chains-per-wave kernel):
    # the export lives in the second, whose accumulators the 8-schools run fills
    s += ("\n#ifdef STK_NUTS_FUSED4_TU\nextern \"C\" __attribute__((visibility(\"default\"))) int stk_debug_stamps(unsigned long long* out, int n) {\n"
          "  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(stk::stk_stamp_acc), sizeof(unsigned long long) * n);\n}\n#endif\n")
    return s


def build():
    if os.path.exists(OUT):
        shutil.rmtree(OUT)
    shutil.copytree(SRC, OUT, ignore=shutil.ignore_patterns("*.o"))
    p = os.path.join(OUT, "nuts.hip")
    text = instrument(open(p).read())
    open(p, "w").write(text)
    mk = open(os.path.join(OUT, "Makefile")).read().replace("../../include/stark_hip.h", os.path.join(ROOT, "include", "stark_hip.h"))
    open(os.path.join(OUT, "Makefile"), "w").write(mk)
    for f in os.listdir(OUT):
        if f.endswith((".hip", ".h")):
            q = os.path.join(OUT, f)
            t = open(q).read().replace('"../../include/stark_hip.h"', '"%s"' % os.path.join(ROOT, "include", "stark_hip.h"))
            open(q, "w").write(t)
    subprocess.run(["make", "-s", "-j8", "-C", OUT, "OUT=" + LIB], check=True)
    shutil.rmtree(os.path.join(LIB, "obj"), ignore_errors=True)
    print("built", os.path.join(LIB, "libstark_hip.so"))


def run():
    os.environ["STARK_HIP_LIB"] = os.path.join(LIB, "libstark_hip.so")
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    sys.path.insert(0, ROOT)
    import numpy as np
    import bench_schools
    from stark_amd import _lib
    line = bench_schools.run()
    lib = _lib.load()
    buf = (ctypes.c_ulonglong * (8192 * 8))()
    assert lib.stk_debug_stamps(buf, 8192 * 8) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(8192, 8)[:line["config"]["chains"]].astype(np.float64)
    tot = a.sum(0)
    steps = tot[7]
    out = {"grads_per_sec": line["value"], "chain_steps": steps,
           "cycles_per_chain_step": {r: tot[i] / steps for i, r in enumerate(REGIONS[:7])}}
    import json
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
