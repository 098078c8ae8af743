#!/usr/bin/env python3
"""Writes tools/_bin/s16_old.hip: a committed k_sweep16 and its logit_resid4 (git REF, default
HEAD), renamed k_sweep16_old / logit_resid4_old, which tools/sweep16_ab.hip times as its "s16-old"
arm against the working tree's kernel.

usage: tools/make_s16_old.py [REF]   (then rebuild tools/_bin/sweep16_ab)"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def show(ref, path):
    return subprocess.run(["git", "-C", ROOT, "show", f"{ref}:{path}"], capture_output=True, text=True,
                          check=True).stdout


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "HEAD"
    src = show(ref, "stark_amd/csrc/sweep16.hip")
    com = show(ref, "stark_amd/csrc/sweep_common.h")
    i = src.index("template <int FAM, int KF,")
    j = src.index("\n}\n", i) + 3
    k = src[i:j].replace("void k_sweep16(SweepArgs A)", "void k_sweep16_old(SweepArgs A)")
    k = k.replace("logit_resid4(", "logit_resid4_old(")
    a = com.index("__device__ __forceinline__ double logit_resid4(")
    b = com.index("\n}\n", a) + 3
    r = com[a:b].replace("logit_resid4(", "logit_resid4_old(")
    os.makedirs(os.path.join(ROOT, "tools", "_bin"), exist_ok=True)
    with open(os.path.join(ROOT, "tools", "_bin", "s16_old.hip"), "w") as f:
        f.write(f"// {ref}'s k_sweep16 and logit_resid4, renamed (tools/make_s16_old.py)\nnamespace stk {{\n{r}{k}}}"
                "  // namespace stk\n")


if __name__ == "__main__":
    main()
