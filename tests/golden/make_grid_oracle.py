"""Oracle-generated fixture for the full configs[4] plan shape (10 x 10 grid,
d = N = 64, 100 factors, 99 evidence columns) with peaked CPDs whose fp32
products stay finite.  The training data and evidence are regenerated in the
test from the same seeds (tests/helpers.py grid_data / sample_evidence), so
the fixture holds only the expected [64, 64] marginals and the target domain.
The expected values come from oracle/ref_infer.py (itself pinned against the
reference-generated goldens); the oracle needs ~40 s for this case, too slow
for the GPU test, hence the fixture.  Run from the repo root:
    python tests/golden/make_grid_oracle.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from helpers import grid_data, sample_evidence  # noqa: E402
from oracle.ref_infer import OracleBN  # noqa: E402

GRID_ARGS = dict(S=60000, seed=3, side=10, d=64, keep=0.995, noise=0)
Q, EV_SEED, N = 64, 5, 64


def main():
    data, cols, edges = grid_data(**GRID_ARGS)
    target, names = cols[-1], cols[:-1]
    ev = sample_evidence(data, cols, names, Q, EV_SEED)
    ref, dom = OracleBN(edges, cols, data).infer(target, ev, N)
    out = os.path.join(ROOT, "tests", "golden", "grid10_d64_peaked_oracle.npz")
    np.savez_compressed(out, pdf=np.asarray(ref, np.float32), domain=np.asarray(dom, np.float32))
    print(out, np.isfinite(ref).all(), float((np.asarray(ref) > 0).mean()))


if __name__ == "__main__":
    main()
