"""Loader for the committed golden fixtures (no pickle: allow_pickle=False)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    d = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    arrays = {k: d[k] for k in d.files if k != "__meta__"}
    meta = json.loads(bytes(d["__meta__"]).decode())
    return arrays, meta


E2E_CASES = ["readme", "readme_wide", "uniform_1d", "mixed_50d", "many_dists",
             "many_dists_pw", "quniform_ties", "nested"]
