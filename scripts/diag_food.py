"""Diagnostic: the first step where an engine library departs from the reference build on a rules-test scenario
(tests/test_rules_gpu.py's turn / food mode config), with the differing fields' details.

    python scripts/diag_food.py LIB [turn food minimap big seed]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mean-field-multi-agent-reinforcement-learning_amd", "python"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import numpy as np  # noqa: E402
import common  # noqa: E402
import test_rules_gpu as tr  # noqa: E402

lib = sys.argv[1]
turn, food, minimap, big, seed = (int(x) for x in (sys.argv[2:7] if len(sys.argv) > 6 else (0, 1, 1, 0, 13)))
cfg = tr._mode_config(16, bool(turn), bool(food), bool(minimap), big=bool(big))
ref = tr._play(common.REF_LIB, cfg, 16, (14, 30), seed, 60, 6)
got = tr._play(lib, tr._mode_config(16, bool(turn), bool(food), bool(minimap), big=bool(big)), 16, (14, 30), seed, 60, 6)
names = ["view0", "feat0", "view1", "feat1", "rew0", "alive0", "pos0", "id0", "rew1", "alive1", "pos1", "id1", "done"]
for t, (a, b) in enumerate(zip(got, ref)):
    bad = [k for k, (x, y) in enumerate(zip(a, b)) if x.shape != y.shape or x.tobytes() != y.tobytes()]
    if not bad:
        continue
    print("first difference at step %d: fields %s" % (t, [names[k] for k in bad]))
    for k in bad:
        x, y = a[k], b[k]
        if x.shape != y.shape:
            print("  %s shapes %s vs %s" % (names[k], x.shape, y.shape))
            continue
        d = np.argwhere(x != y)
        print("  %s: %d elements differ, first %s" % (names[k], len(d), d[:6].tolist()))
        for idx in d[:6]:
            print("    at %s: got %r ref %r" % (tuple(idx), x[tuple(idx)], y[tuple(idx)]))
    if t > 0:
        pa, pb = got[t - 1], ref[t - 1]
        print("  (step %d identical; ids0 %s)" % (t - 1, pb[7][:20].tolist()))
    break
else:
    print("no difference over %d steps" % len(ref))
