"""Child process of tests/test_gpu_diag.py and tests/test_native_abi.py.

Diagnostic kernel-selection switches (CBN_NO_STAGED, CBN_PARAM_GENERIC, ...)
count only when libcbn_amd.so is loaded with CBN_DIAG=1 (cbn_diag_enabled,
include/cbn_amd.h), so a test that toggles them needs a process started with
the environment it is testing.  Prints one JSON line.

    python tests/diag_child.py enabled   # no GPU: cbn_diag_enabled()
    python tests/diag_child.py flags     # configs[1]-shaped plan's cbn_plan_flags
    python tests/diag_child.py generic   # NN [16] rows: fast kernel vs CBN_PARAM_GENERIC
    python tests/diag_child.py gridfull  # configs[4] bench batch: k_query_slots vs k_query_fast (CBN_NO_SLOTS)
    python tests/diag_child.py gridcoal  # k_query_slots' coalesced index phase vs the per-lane one (CBN_SLOTS_NO_COAL)
"""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)


def main(mode: str):
    from continuousbayesiannetwork_amd import _native

    lib = _native.load()
    res = {"diag": int(lib.cbn_diag_enabled())}
    if mode == "enabled":
        print(json.dumps(res))
        return
    import numpy as np
    import torch

    from continuousbayesiannetwork_amd import BayesianNetwork
    from helpers import chain_data, make_bn, mixed_dag_data, param_config, sample_evidence

    dev = torch.device("cuda:0")
    if mode == "flags":
        # BASELINE configs[1]'s plan shape: 20-node chain, d = 32, evidence on X0..X18, N = 32
        data, cols, edges = chain_data(20, 32, 20000, 21, stay=0.8)
        bn = make_bn(BayesianNetwork, edges, cols, data, device=dev)
        ev = {k: torch.tensor(v, device=dev) for k, v in sample_evidence(data, cols, cols[:19], 1024, 5).items()}
        bn.infer("X19", ev, N_max=32)
        res["flags"] = [int(lib.cbn_plan_flags(p.handle)) for p in bn.engine._plans.values()]
    elif mode == "generic":
        data, cols, edges = mixed_dag_data(3000, 4, n=12, unit=True)
        model = {"hidden_dims": [16], "activation": "tanh"}
        names = [cols[-2], cols[5], cols[2]]
        ev = {k: torch.tensor(v, device=dev) for k, v in sample_evidence(data, cols, names, 500, 3).items()}
        bn = make_bn(BayesianNetwork, edges, cols, data, device=dev, estimator="neural_network",
                     config=param_config("neural_network", n_epochs=10, model=model))
        os.environ["CBN_PARAM_PARTS"] = "1"  # one factor range per wave: the generic kernel's product order
        outs, flags = [], []
        for generic in (False, True):
            if generic:  # read at plan creation: drop the cached plan
                os.environ["CBN_PARAM_GENERIC"] = "1"
                bn.engine.invalidate()
            random.seed(4)
            outs.append(bn.infer(cols[-1], ev, N_max=8)[0].cpu().numpy())
        res["equal"] = bool(np.array_equal(outs[0], outs[1], equal_nan=True))
        res["finite"] = int(np.isfinite(outs[0]).sum())
    elif mode == "gridfull":
        # tools/bench_grid.py's headline batch (BASELINE configs[4], 65 536 queries)
        from helpers import grid_data

        data, cols, edges = grid_data(400_000, 3, side=10, d=64, keep=0.995, noise=0)
        target, names = cols[-1], cols[:-1]
        ev = {k: torch.tensor(v, device=dev) for k, v in sample_evidence(data, cols, names, 65536, 0).items()}
        bn = make_bn(BayesianNetwork, edges, cols, data, device=dev)
        outs, flags = [], []
        for no_slots in (False, True):
            if no_slots:  # read at plan creation: drop the cached plan
                os.environ["CBN_NO_SLOTS"] = "1"
                bn.engine.invalidate()
            outs.append(bn.infer(target, ev, N_max=64)[0].cpu().numpy())
            flags += [int(lib.cbn_plan_flags(p.handle)) for p in bn.engine._plans.values()]
        res["flags"] = flags
        res["equal"] = bool(np.array_equal(outs[0], outs[1], equal_nan=True))
        res["nonzero_rows"] = int((outs[0] > 0).any(1).sum())
    elif mode == "gridcoal":
        # >= 3 block rounds (the raw launch + scale path): coalesced index phase
        # vs the per-lane loads, ragged batch, and a column view that is not
        # 16-B aligned (the coalesced phase declines it)
        from helpers import grid_data

        data, cols, edges = grid_data(100000, 7, side=5, d=64, keep=0.995, noise=0)
        target, names = cols[-1], cols[:-1]
        ev = {k: torch.tensor(v, device=dev) for k, v in sample_evidence(data, cols, names, 200003, 3).items()}
        bn = make_bn(BayesianNetwork, edges, cols, data, device=dev)
        outs = []
        for no_coal in (False, True):
            os.environ["CBN_SLOTS_NO_COAL"] = "1" if no_coal else "0"
            if not no_coal:
                os.environ.pop("CBN_SLOTS_NO_COAL")
            outs.append(bn.infer(target, ev, N_max=64)[0].cpu().numpy())
        off = {k: torch.cat([torch.zeros((1, 1), device=dev), v])[1:] for k, v in ev.items()}  # 4-B offset views
        outs.append(bn.infer(target, off, N_max=64)[0].cpu().numpy())
        res["flags"] = [int(lib.cbn_plan_flags(p.handle)) for p in bn.engine._plans.values()]
        res["equal"] = bool(np.array_equal(outs[0], outs[1], equal_nan=True))
        res["equal_unaligned"] = bool(np.array_equal(outs[0], outs[2], equal_nan=True))
        res["nonzero_rows"] = int((outs[0] > 0).any(1).sum())
        rows = np.append(np.arange(0, 200003, 5003)[:40], [200002, int(np.argmax(outs[0].max(1)))])
        np.save(os.environ["CBN_CHILD_OUT"], outs[0][rows])
        res["rows"] = rows.tolist()
    print(json.dumps(res))


if __name__ == "__main__":
    main(sys.argv[1])
