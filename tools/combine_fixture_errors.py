#!/usr/bin/env python3
"""Max relative error of the GPU combine against the reference-run fixtures (tests/golden/
combine_ref.npz: the reference's own consensus_avg and final solve, P = 11, 53, 102), next to
cond(sum W): how close the kernels are to the north_star's flat 1e-12."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from stark_amd import engine  # noqa: E402
from stark_amd.stark import consensus_avg  # noqa: E402

g = np.load(os.path.join(ROOT, "tests", "golden", "combine_ref.npz"))
ctx = engine.Context(0)
out = {}
for P in (11, 53, 102):
    f1, f2 = g[f"P{P}_f1"], g[f"P{P}_f2"]
    sw, swt = consensus_avg(2)(f1, f2)
    fin, _ = engine.consensus([f1, f2], ctx)
    rel = lambda a, b: float(np.abs(a - b).max() / np.abs(b).max())
    out[P] = {"cond_sumW": float(np.linalg.cond(g[f"P{P}_sumW"])), "sumW": rel(sw, g[f"P{P}_sumW"]),
              "sumWtheta": rel(swt, g[f"P{P}_sumWtheta"]), "final": rel(fin, g[f"P{P}_final"])}
print(json.dumps(out))
