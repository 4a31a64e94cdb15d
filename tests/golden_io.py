"""Shared loader for the golden fixtures written by tests/golden/make_golden.py."""
import glob
import json
import os

import numpy as np

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def golden_names():
    with open(os.path.join(GOLDEN_DIR, "MANIFEST.json")) as f:
        return json.load(f)["cases"]


def load_golden(name):
    z = np.load(os.path.join(GOLDEN_DIR, name + ".npz"), allow_pickle=False)
    meta = json.loads(str(z["meta"]))
    ev = {k[3:]: z[k] for k in z.files if k.startswith("ev_")}
    return dict(meta=meta, data=z["data"], pdf=z["pdf"], domain=z["domain"], evidence=ev)
