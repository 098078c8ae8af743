#!/usr/bin/env python3
"""A/B of whole library builds on the bench's own workloads: each arm is libstark_hip.so built
from the working tree (or a git revision) with extra compiler flags on chosen source files;
the arms run alternately in fresh processes (STARK_HIP_LIB) so box drift hits every arm, and
each workload reports whether the arms' results are bit-identical.

  workloads  schools   tools/bench_schools.py (configs[1]: 4096 chains, 1000 + 1000): grads/s,
                       identical = posterior means, min ESS, divergences, leapfrogs agree
             sweep16   bench.py --throughput-only (configs[3]: 8 x 1.25e7 rows, d = 100, 16
                       chains): k_sweep16's ms per launch (HIP events), identical = grads agree
             sweep16lin  the same at configs[2]'s shape (linear, 8 x 1.25e6 rows, d = 50)
             fulldata  tools/bench_fulldata.py --steps 6 (configs[4] at 1e7 rows): pass F + B ms

usage: tools/lib_ab.py build NAME [--rev REV] [--flags FILE=FLAGS ...]   (here; -> tools/_bin/ab_NAME; no
       --flags: the tree's Makefile)
       tools/lib_ab.py run --arms A,B[,C] --work schools|sweep16|fulldata [--rounds R]   (GPU box)"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tools", "_bin")
SRCS = ["capi.hip", "nuts.hip", "nuts_fused4.hip", "sweep.hip", "sweep16.hip", "datagen.hip", "combine.hip"]
BASE_FLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-fvisibility=hidden"]


def build(name, rev=None, flags=()):
    out = os.path.join(BIN, f"ab_{name}")
    os.makedirs(out, exist_ok=True)
    csrc = os.path.join(ROOT, "stark_amd", "csrc")
    if rev:
        src = os.path.join(BIN, f"ab_{name}_src")
        subprocess.run(["rm", "-rf", src], check=True)
        os.makedirs(src)
        tar = subprocess.run(["git", "-C", ROOT, "archive", rev, "stark_amd/csrc", "include"], check=True,
                             capture_output=True).stdout
        subprocess.run(["tar", "-x", "-C", src], input=tar, check=True)
        csrc = os.path.join(src, "stark_amd", "csrc")
    extra = {}
    for f in flags:
        k, v = f.split("=", 1)
        extra[k] = v.split()
    if not extra:        # the tree's own Makefile (its per-file flags)
        subprocess.run(["make", "-s", "-j8", "-C", csrc, f"OUT={out}"], check=True)
        json.dump({"rev": rev or "working tree", "flags": "Makefile"}, open(os.path.join(out, "arm.json"), "w"))
        print("built", os.path.join(out, "libstark_hip.so"), "with the Makefile")
        return
    procs, objs = [], []
    for s in SRCS:
        o = os.path.join(out, s.replace(".hip", ".o"))
        objs.append(o)
        procs.append(subprocess.Popen(["/opt/rocm/bin/hipcc", *BASE_FLAGS, *extra.get(s, []), "-c",
                                       os.path.join(csrc, s), "-o", o]))
    if any(p.wait() for p in procs):
        sys.exit("build failed")
    subprocess.run(["/opt/rocm/bin/hipcc", "-shared", "--offload-arch=gfx950", "-o",
                    os.path.join(out, "libstark_hip.so"), *objs], check=True)
    json.dump({"rev": rev or "working tree", "flags": extra}, open(os.path.join(out, "arm.json"), "w"))
    print("built", os.path.join(out, "libstark_hip.so"), extra)


def one(arm, work):
    env = dict(os.environ, STARK_HIP_LIB=os.path.join(BIN, f"ab_{arm}", "libstark_hip.so"))
    if work == "schools":
        cmd = [sys.executable, os.path.join(ROOT, "tools", "bench_schools.py")]
    elif work == "sweep16":
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--throughput-only", "--steps", "200", "--warmup", "10"]
    elif work == "sweep16lin":
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--throughput-only", "--family", "linear", "--rows", "1e7",
               "--d", "50", "--steps", "2000", "--warmup", "50"]
    else:
        cmd = [sys.executable, os.path.join(ROOT, "tools", "bench_fulldata.py"), "--rows-per-gpu", "1e7", "--steps", "6",
               "--warmup", "2"]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=400)
    if p.returncode != 0:
        sys.exit(p.stderr[-2000:])
    ln = json.loads(p.stdout.strip().splitlines()[-1])
    if work == "schools":
        return ln["value"] / 1e6, [ln[k] for k in ("posterior_mean_mu_tau", "min_ess", "divergent", "leapfrogs_per_transition")]
    if work in ("sweep16", "sweep16lin"):
        return ln["roofline"]["avg_launch_ms"], [round(ln["value"] * ln["ms_per_step"])]
    return ln["roofline"]["avg_launch_ms"], [ln.get("chains_sha16_per_rank")]


def run(arms, work, rounds):
    res = {a: [] for a in arms}
    ident = {}
    for r in range(rounds):
        for a in (arms if r % 2 == 0 else arms[::-1]):
            v, key = one(a, work)
            res[a].append(v)
            ident.setdefault(a, key)
            print(f"[lib_ab] {work} round {r} {a}: {v:.4f}", file=sys.stderr, flush=True)
    med = {a: sorted(v)[len(v) // 2] for a, v in res.items()}
    out = {"work": work, "unit": "M grads/s" if work == "schools" else "ms per launch",
           "arms": {a: {"values": res[a], "median": med[a],
                        "build": json.load(open(os.path.join(BIN, f"ab_{a}", "arm.json")))} for a in arms},
           "ratio_vs_first": {a: med[a] / med[arms[0]] for a in arms},
           "identical_to_first": {a: ident[a] == ident[arms[0]] for a in arms}}
    print(json.dumps(out))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("cmd", choices=["build", "run"])
    p.add_argument("name", nargs="?")
    p.add_argument("--rev", default=None)
    p.add_argument("--flags", nargs="*", default=[])
    p.add_argument("--arms", default="")
    p.add_argument("--work", default="schools", choices=["schools", "sweep16", "sweep16lin", "fulldata"])
    p.add_argument("--rounds", type=int, default=3)
    a = p.parse_args()
    if a.cmd == "build":
        build(a.name, a.rev, a.flags)
    else:
        run(a.arms.split(","), a.work, a.rounds)


if __name__ == "__main__":
    main()
