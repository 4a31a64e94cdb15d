"""Oracle fixture for configs[4] AT ITS BENCHMARKED SIZE: tools/bench_grid.py's
headline batch (10 x 10 grid, d = N = 64, peaked CPDs fitted on
grid_data(400 000, 3, keep 0.995, noise 0), 65 536 queries drawn with
sample_evidence seed 0).  The oracle needs ~2 s per query on this plan, so
the fixture holds the UNnormalised rows (bayesian_network.py:269-295, before
the :296 division) of a fixed row set -- every 1 638th row (40 rows), the
first and last 128-query block (k_query_slots' block of L = 8 lanes per
query), and the batch's argmax row, found once by the HIP path (argv[1];
tests/test_gpu_parity.py asserts the GPU's argmax is still that row, and the
oracle's value there is the max of every fixture row).  Data and evidence are
regenerated in the test from the same seeds.  Run from the repo root:

    python tests/golden/make_grid_bench_oracle.py <argmax_row>
"""
import multiprocessing as mp
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from helpers import grid_data, sample_evidence  # noqa: E402
from oracle.ref_infer import OracleBN  # noqa: E402

GRID_ARGS = dict(S=400_000, seed=3, side=10, d=64, keep=0.995, noise=0)
Q, EV_SEED, N, BLOCK = 65536, 0, 64, 128
_ORA = _EV = _TARGET = None


def fixture_rows(argmax_row: int) -> np.ndarray:
    rows = list(np.arange(0, Q, Q // 40)[:40]) + list(range(BLOCK)) + list(range(Q - BLOCK, Q)) + [argmax_row]
    return np.unique(np.asarray(rows, np.int64))


def _raw(chunk):
    sub = {k: v[chunk] for k, v in _EV.items()}
    return _ORA.infer_raw(_TARGET, sub, N)[0]


def main():
    global _ORA, _EV, _TARGET
    argmax_row = int(sys.argv[1])
    data, cols, edges = grid_data(**GRID_ARGS)
    _TARGET, names = cols[-1], cols[:-1]
    _EV = sample_evidence(data, cols, names, Q, EV_SEED)
    _ORA = OracleBN(edges, cols, data)  # fitted once; the forked workers share it
    rows = fixture_rows(argmax_row)
    chunks = np.array_split(rows, 8)
    with mp.get_context("fork").Pool(7) as pool:
        raw = np.concatenate(pool.map(_raw, chunks))
    _, dom = _ORA.infer_raw(_TARGET, {k: v[:1] for k, v in _EV.items()}, N)
    out = os.path.join(ROOT, "tests", "golden", "grid10_d64_bench65536_oracle.npz")
    np.savez_compressed(out, rows=rows, raw=raw.astype(np.float32), domain=np.asarray(dom[:1], np.float32),
                        argmax_row=np.int64(argmax_row))
    print(out, raw.shape, float(raw.max()), int(rows[np.argmax(raw.max(1))]))


if __name__ == "__main__":
    main()
