"""Compare the per-replica results two scripts/bench_ising.py --dump runs wrote (e.g. 1 rank against 2 ranks):
replica r's episode length, final order parameter and Q-table digest, bit for bit, over the whole replica range.

    python scripts/compare_ising_dumps.py DIR_A DIR_B"""
import glob
import json
import os
import sys

import numpy as np


def load(d):
    parts = sorted((np.load(f) for f in glob.glob(os.path.join(d, "rank*.npz"))), key=lambda z: int(z["first"]))
    first = 0
    out = {"steps": [], "final_order": [], "q_sha": []}
    for z in parts:
        assert int(z["first"]) == first, (d, int(z["first"]), first)
        first += len(z["steps"])
        for k in out:
            out[k].append(z[k])
    return {k: np.concatenate(v) for k, v in out.items()}, len(parts)


a, na = load(sys.argv[1])
b, nb = load(sys.argv[2])
same = (len(a["steps"]) == len(b["steps"]) and np.array_equal(a["steps"], b["steps"]) and
        a["final_order"].tobytes() == b["final_order"].tobytes() and np.array_equal(a["q_sha"], b["q_sha"]))
print(json.dumps({"replicas": len(a["steps"]), "ranks": [na, nb], "identical": bool(same)}))
sys.exit(0 if same else 1)
