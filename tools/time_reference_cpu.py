"""Time the REFERENCE's own BayesianNetwork.infer on CPU for the bench workload
(BASELINE configs[1]) on a bounded query sample.  Runs only where
/root/reference exists (this container); the GPU box uses bench.py's oracle
port instead.  Usage: python tools/time_reference_cpu.py [n_queries] [threads] [processes]
(processes > 1: the sample split into one chunk per process, each running the
reference with one torch thread -- the layout of bench.py's parallel port;
per-chunk normalisation does not change the work)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

import torch  # noqa: E402

from helpers import chain_data, sample_evidence  # noqa: E402
from make_golden import _load_reference  # noqa: E402


_BN = None


def _chunk(ev):
    import contextlib
    import io

    with contextlib.redirect_stdout(io.StringIO()):
        _BN.infer("X19", ev, N_max=32)
    return True


def main():
    global _BN
    q = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    th = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    procs = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    torch.set_num_threads(th)
    import networkx as nx
    import pandas as pd

    BN = _load_reference()
    n, d = 20, 32
    data, cols, edges = chain_data(n, d, 200_000, 3, stay=0.8)
    dag = nx.DiGraph()
    dag.add_nodes_from(cols)
    dag.add_edges_from(edges)
    bn = BN(dag, pd.DataFrame(data, columns=cols), {"estimator_name": "brute_force"},
            {"inference_obj": "exact"}, device="cpu")
    ev = sample_evidence(data, cols, [c for c in cols if c != "X19"], q, seed=1000)
    ev = {k: torch.tensor(v) for k, v in ev.items()}
    import contextlib
    import io

    with contextlib.redirect_stdout(io.StringIO()):
        bn.infer("X19", {k: v[:8] for k, v in ev.items()}, N_max=d)
        if procs > 1:
            import multiprocessing as mp

            _BN = bn
            cuts = [q * i // procs for i in range(procs + 1)]
            jobs = [{k: v[cuts[i]:cuts[i + 1]] for k, v in ev.items()} for i in range(procs)]
            with mp.get_context("fork").Pool(procs) as pool:
                pool.map(_chunk, [{k: v[:8] for k, v in ev.items()}] * procs, chunksize=1)
                t0 = time.perf_counter()
                pool.map(_chunk, jobs, chunksize=1)
                t = time.perf_counter() - t0
        else:
            t0 = time.perf_counter()
            bn.infer("X19", ev, N_max=d)
            t = time.perf_counter() - t0
    print(f"reference BayesianNetwork.infer, chain20 d32, {q} queries, {th} torch threads x {procs} processes: "
          f"{t:.3f} s -> {q / t:.1f} queries/s")


if __name__ == "__main__":
    main()
