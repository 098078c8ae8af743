#!/usr/bin/env python3
"""A/B of the fused 8-schools kernel (BASELINE configs[1], tools/bench_schools.py's run: 4096
chains, 1000 + 1000): the library built from a git revision (default HEAD) against the working
tree's, alternating runs in fresh processes so box drift hits both arms, and whether the two
arms' draws agree (posterior means, min ESS, divergences, leapfrogs: a change that only moves
work must leave them bit-identical).

usage: tools/schools_ab.py build [REV]     (here: tools/_bin/ab_base, tools/_bin/ab_new)
       tools/schools_ab.py run [rounds]    (on the GPU box; prints one JSON line)"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tools", "_bin")
ARMS = ("ab_base", "ab_new")


def build(rev="HEAD"):
    src = os.path.join(BIN, "ab_base_src")
    subprocess.run(["rm", "-rf", src], check=True)
    os.makedirs(src)
    tar = subprocess.run(["git", "-C", ROOT, "archive", rev, "stark_amd/csrc", "include"], check=True,
                         capture_output=True).stdout
    subprocess.run(["tar", "-x", "-C", src], input=tar, check=True)
    for arm, csrc in (("ab_base", os.path.join(src, "stark_amd", "csrc")), ("ab_new", os.path.join(ROOT, "stark_amd", "csrc"))):
        out = os.path.join(BIN, arm)
        subprocess.run(["make", "-s", "-j8", "-C", csrc, f"OUT={out}"], check=True)
    print("built", [os.path.join(BIN, a, "libstark_hip.so") for a in ARMS])


def run(rounds=3):
    res = {a: [] for a in ARMS}
    for r in range(rounds):
        for a in (ARMS if r % 2 == 0 else ARMS[::-1]):
            env = dict(os.environ, STARK_HIP_LIB=os.path.join(BIN, a, "libstark_hip.so"))
            p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "bench_schools.py")], env=env,
                               capture_output=True, text=True, timeout=300)
            if p.returncode != 0:
                sys.exit(p.stderr[-2000:])
            ln = json.loads(p.stdout.strip().splitlines()[-1])
            res[a].append(ln)
            print(f"[schools_ab] round {r} {a}: {ln['value'] / 1e6:.1f}M grads/s", file=sys.stderr, flush=True)
    key = ("posterior_mean_mu_tau", "min_ess", "divergent", "leapfrogs_per_transition")
    out = {a: {"value_M": sorted(x["value"] / 1e6 for x in v), "median_M": sorted(x["value"] / 1e6 for x in v)[len(v) // 2],
               "whole_run_M": [x["grad_evals_per_sec_whole_run"] / 1e6 for x in v]} for a, v in res.items()}
    out["draws_identical"] = all(res[ARMS[0]][0][k] == res[a][i][k] for a in ARMS for i in range(rounds) for k in key)
    out["ratio_new_over_base"] = out["ab_new"]["median_M"] / out["ab_base"]["median_M"]
    print(json.dumps(out))


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build(*(sys.argv[2:3]))
    else:
        run(int(sys.argv[2]) if len(sys.argv) > 2 else 3)
