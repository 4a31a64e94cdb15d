"""CPU oracle: restatement of the reference's batched inference path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module, and only as the
checker / the CPU baseline -- never as the product path.

It restates, with numpy (plus torch CPU for the two reference helpers whose
float32 semantics are torch-specific: ``torch.linspace(...).round()`` and the
tensor-valued ``random.uniform``), the algorithm of:

* ``cbn/parameter_learning/brute_force.py:17-53``   BruteForce._fit
* ``cbn/parameter_learning/brute_force.py:172-244`` BruteForce._get_prob
* ``cbn/base/node.py:45-110``   Node.fit (domain bookkeeping in ``info``)
* ``cbn/base/node.py:115-204``  Node.get_prob
* ``cbn/base/node.py:206-284``  Node._setup_parents_query
* ``cbn/base/node.py:286-333``  Node.sample_domain
* ``cbn/base/node.py:335-375``  Node._batched_meshgrid_combinations
* ``cbn/base/bayesian_network.py:86-102``  get_ancestors
* ``cbn/base/bayesian_network.py:176-206`` get_pdf
* ``cbn/base/bayesian_network.py:208-305`` infer (factor product / mean-out / max-normalise)
* ``cbn/parameter_learning/linear_regression.py:78-96``   LinearRegression._get_prob
* ``cbn/parameter_learning/logistIc_regression.py:67-98`` LogisticRegression._get_prob
* ``cbn/parameter_learning/neural_network.py:43-52, 95-124`` NeuralNetwork._build_nn / _get_prob

The parametric estimators are restated for inference only: their fitted
parameters are inputs (the reference's training loop -- torch autograd + Adam --
is not restated), taken from the reference-generated fixtures or from the
model under test.

Parity of this oracle is pinned against golden vectors produced by running the
reference itself (``tests/golden/make_golden.py`` -> ``tests/golden/*.npz``).
The matching in ``bf_get_prob`` is the reference's O(rows x n_mle) equality
scan, deliberately: this module is the reference algorithm, not a fast path.
"""
from __future__ import annotations

import random
from typing import Dict, List, Optional, Sequence, Tuple

import networkx as nx
import numpy as np
import torch

EPS = np.float32(1e-10)  # brute_force.py:240


# --------------------------------------------------------------------------
# BruteForce estimator (brute_force.py)
# --------------------------------------------------------------------------
class OracleBruteForce:
    """brute_force.py:8-271 restated on numpy float32."""

    def __init__(self):
        self.mle = None  # [n_unique, k+2] float32: parents..., node, prob

    def fit(self, node_data: np.ndarray, parents_data: Optional[np.ndarray]):
        # brute_force.py:23-53
        node_data = np.asarray(node_data, np.float32).reshape(-1, 1)
        if parents_data is not None:
            pd_ = np.asarray(parents_data, np.float32).T  # [S, k]
            all_data = np.concatenate([pd_, node_data], axis=1)
        else:
            all_data = node_data
        rows, counts = np.unique(all_data, axis=0, return_counts=True)
        probs = counts.astype(np.float32) / np.float32(counts.sum())
        mle = np.empty((rows.shape[0], rows.shape[1] + 1), np.float32)
        mle[:, :-1] = rows
        mle[:, -1] = probs
        self.mle = mle

    def get_prob(self, points: np.ndarray, query: Optional[np.ndarray] = None) -> np.ndarray:
        """brute_force.py:172-244.  points [Qr, V]; query [Qr, k, 1] or None."""
        points = np.asarray(points, np.float32)
        mle_data = self.mle[:, :-1]
        mle_probs = self.mle[:, -1]
        if query is None:
            # brute_force.py:192-201: marginal P(node_value)
            node_values = mle_data[:, -1]
            out = np.zeros_like(points)
            for i in range(points.shape[0]):
                for j in range(points.shape[1]):
                    m = node_values == points[i, j]
                    out[i, j] = mle_probs[m].sum(dtype=np.float32) if m.any() else 0.0
            return out
        query = np.asarray(query, np.float32)
        nq, k, _ = query.shape
        nv = points.shape[1]
        pq = np.broadcast_to(query[:, None, :, 0], (nq, nv, k))
        full = np.concatenate([pq, points[:, :, None]], axis=-1).reshape(-1, k + 1)
        joint_m = (full[:, None, :] == mle_data[None, :, :]).all(-1)
        joint = (joint_m * mle_probs[None, :]).sum(-1, dtype=np.float32)
        par_m = (full[:, None, :-1] == mle_data[None, :, :-1]).all(-1)
        par = (par_m * mle_probs[None, :]).sum(-1, dtype=np.float32)
        pdf = joint / (par + EPS)
        return pdf.reshape(nq, nv).astype(np.float32)


# --------------------------------------------------------------------------
# Parametric estimators (linear_regression.py / logistIc_regression.py /
# neural_network.py), inference only
# --------------------------------------------------------------------------
def _act(name: str, x: np.ndarray) -> np.ndarray:
    """activation_map of neural_network.py:10-18 (torch formulas, float32)."""
    x = x.astype(np.float32)
    if name == "tanh":
        return np.tanh(x)
    if name == "relu":
        return np.where(x > 0, x, np.float32(0)).astype(np.float32)
    if name == "sigmoid":
        return (np.float32(1) / (np.float32(1) + np.exp(-x))).astype(np.float32)
    if name == "leakyrelu":
        return np.where(x > 0, x, x * np.float32(0.01)).astype(np.float32)
    if name == "gelu":
        import math
        erf = np.vectorize(math.erf, otypes=[np.float64])
        return (x * np.float32(0.5) * (np.float32(1) + erf(x * np.float32(0.7071067811865476)).astype(np.float32))
                ).astype(np.float32)
    if name == "elu":
        return np.where(x > 0, x, np.expm1(x)).astype(np.float32)
    raise KeyError(name)


class OracleParametric:
    """Inference-time restatement of the three parametric estimators.

    ``layers`` = [(W [out, in], b [out]), ...] (nn.Linear), ``act`` = the
    activation between layers, ``log_scale`` = log_sigma (``family`` "gauss",
    LinearRegression) or log_scale ("logistic": LogisticRegression,
    NeuralNetwork).  ``root_bias_only``: LinearRegression's query-free mean is
    its bias (linear_regression.py:84-89); the logistic models evaluate on a
    ones input (logistIc_regression.py:83-86, neural_network.py:111-114).
    """

    def __init__(self, family: str, layers, log_scale: float, act: Optional[str] = None,
                 root_bias_only: bool = False):
        self.family = family
        self.layers = [(np.asarray(W, np.float32), np.asarray(b, np.float32)) for W, b in layers]
        self.log_scale = np.float32(log_scale)
        self.act = act
        self.root_bias_only = root_bias_only

    def fit(self, node_data, parents_data):
        pass  # parameters are given

    def mu(self, q: np.ndarray) -> np.ndarray:
        h = q.astype(np.float32)
        for i, (W, b) in enumerate(self.layers):
            h = (h @ W.T + b).astype(np.float32)
            if i < len(self.layers) - 1:
                h = _act(self.act, h)
        return h

    def get_prob(self, points: np.ndarray, query: Optional[np.ndarray] = None) -> np.ndarray:
        x = np.asarray(points, np.float32)
        if query is not None:
            mu = self.mu(np.asarray(query, np.float32)[..., 0])  # [n, 1]
        elif self.root_bias_only:
            mu = (np.zeros((x.shape[0], 1), np.float32) + self.layers[-1][1]).astype(np.float32)
        else:
            mu = self.mu(np.ones((x.shape[0], 1), np.float32))
        # the reference's scale is torch.exp of the fp32 log-scale parameter
        # (linear_regression.py:91, neural_network.py:120); numpy's float32 exp
        # can differ by an ulp, which (x - mu) / s amplifies by t^2 in the density
        s = np.float32(torch.exp(torch.tensor(self.log_scale, dtype=torch.float32)).item())
        if self.family == "gauss":
            norm = (np.float32(1) / (s * np.sqrt(np.float32(2 * np.pi)))).astype(np.float32)
            t = ((x - mu) / s).astype(np.float32)
            return (norm * np.exp(np.float32(-0.5) * t ** 2)).astype(np.float32)
        d = ((x - mu) / s).astype(np.float32)
        e = np.exp(-d).astype(np.float32)
        return (e / (s * (np.float32(1) + e) ** 2)).astype(np.float32)


# --------------------------------------------------------------------------
# Node (node.py)
# --------------------------------------------------------------------------
class OracleNode:
    def __init__(self, name: str, parents: Sequence[str], est=None):
        self.name = name
        self.parents = sorted(parents)  # node.py:65
        self.est = est if est is not None else OracleBruteForce()
        self.info: Dict[str, list] = {}

    def fit(self, node_data: np.ndarray, parents_data: Optional[np.ndarray]):
        # node.py:45-110 (kind flag is not used on the inference path)
        node_data = np.asarray(node_data, np.float32)
        self.est.fit(node_data, parents_data)
        self.info[self.name] = [np.float32(node_data.min()), np.float32(node_data.max()),
                                np.unique(node_data)]
        if parents_data is not None and len(self.parents) > 0:
            parents_data = np.asarray(parents_data, np.float32)
            for i, p in enumerate(self.parents):
                self.info[p] = [np.float32(parents_data[i].min()),
                                np.float32(parents_data[i].max()),
                                np.unique(parents_data[i])]

    def sample_domain(self, node: str, N: int) -> np.ndarray:
        """node.py:286-333, including the N > cardinality random fill.

        The random fill consumes Python's global ``random`` exactly as the
        reference does: ``random.uniform(min_tensor, max_tensor)`` evaluates
        ``a + (b - a) * random.random()`` on 0-dim float32 tensors, and the
        ``candidate not in existing`` test is always true for a tensor
        candidate (tensor hashing is by identity).
        """
        mn, mx, dom = self.info[node]
        card = dom.shape[0]
        if N < card:
            idx = torch.linspace(start=0, end=card - 1, steps=N).round().long().numpy()
            return dom[idx]
        if N == card:
            return dom.copy()
        need = N - card
        a = torch.tensor(mn, dtype=torch.float32)
        b = torch.tensor(mx, dtype=torch.float32)
        new = [float(a + (b - a) * random.random()) for _ in range(need)]
        out = np.concatenate([dom, np.asarray(new, np.float32)])
        return np.sort(out, kind="stable").astype(np.float32)

    @staticmethod
    def _meshgrid(points: np.ndarray) -> np.ndarray:
        """node.py:335-375: [nq, k, N] -> [nq, k, N**k], 'ij' order."""
        nq, k, n = points.shape
        out = np.empty((nq, k, n ** k), np.float32)
        for m in range(nq):
            grids = np.meshgrid(*[points[m, i] for i in range(k)], indexing="ij")
            out[m] = np.stack(grids, 0).reshape(k, -1)
        return out

    def get_prob(self, query: Dict[str, np.ndarray], N: int):
        """node.py:115-204.  query values are [Q, 1] float arrays."""
        query = dict(query)
        nq = next(iter(query.values())).shape[0] if query else 1
        query.pop(self.name, None)  # node.py:140 (never a parent of itself)
        pq, _ = self._setup_parents_query(query, N)
        combos = pq.shape[2] if pq is not None else 0
        dom = np.broadcast_to(self.sample_domain(self.name, N)[None, :], (nq, N))
        nv = dom.shape[1]
        k = len(self.parents)
        parent_dims = [N if combos > 1 else 1 for _ in self.parents]
        if k > 0:
            pdfs = np.empty((nq, combos, nv), np.float32)
            if combos > 1:
                npq = np.transpose(pq, (2, 1, 0))  # [combos, k, n_start]
                for i in range(npq.shape[2]):
                    q = npq[:, :, i, None]
                    d = np.broadcast_to(dom[i][None, :], (combos, nv))
                    pdfs[i] = self.est.get_prob(d, q)
            else:
                for i in range(combos):
                    pdfs[:, i, :] = self.est.get_prob(dom, pq[:, :, i, None])
        else:
            pdfs = self.est.get_prob(dom)
        return pdfs.reshape([nq] + parent_dims + [nv]), dom

    def _setup_parents_query(self, query: Dict[str, np.ndarray], N: int):
        """node.py:206-284."""
        feats = sorted(query.keys())
        k = len(self.parents)
        if feats:
            n0 = query[feats[0]].shape[0]
            assert all(f in self.parents for f in feats)
            if feats == self.parents:
                q = np.zeros((n0, k, 1), np.float32)
                for i, p in enumerate(self.parents):
                    _check_width(query[p], 1, f"[{n0}, 1]")  # node.py:233-234 (a copy into [Q, 1])
                    q[:, i, :] = np.asarray(query[p], np.float32)
                return q, q
            pts = np.empty((n0, k, N), np.float32)
            for i, p in enumerate(self.parents):
                if p in feats:
                    _check_width(query[p], N, f"[-1, {N}]")  # node.py:246-248 (.expand(-1, N))
                    pts[:, i, :] = np.broadcast_to(np.asarray(query[p], np.float32), (n0, N))
                else:
                    pts[:, i, :] = self.sample_domain(p, N)[None, :]
            return self._meshgrid(pts), pts
        if k > 0:
            pts = np.empty((1, k, N), np.float32)
            for i, p in enumerate(self.parents):
                pts[:, i, :] = self.sample_domain(p, N)[None, :]
            return self._meshgrid(pts), pts
        return None, None


def _check_width(col: np.ndarray, target: int, shape: str):
    """torch's broadcast error for an evidence column whose width is neither 1
    nor ``target`` (the reference raises it from node.py:234 / :246-248)."""
    k = col.shape[1]
    if k != 1 and k != target:
        raise RuntimeError(f"The expanded size of the tensor ({target}) must match the existing size ({k}) at "
                           f"non-singleton dimension 1.  Target sizes: {shape}.  Tensor sizes: [{col.shape[0]}, {k}]")


# --------------------------------------------------------------------------
# BayesianNetwork.infer (bayesian_network.py)
# --------------------------------------------------------------------------
class OracleBN:
    def __init__(self, edges: Sequence[Tuple[str, str]], columns: Sequence[str],
                 data: np.ndarray, nodes: Optional[Sequence[str]] = None, estimators: Optional[Dict] = None):
        """``data`` is [S, n_columns] float32, columns named by ``columns``.

        ``nodes`` fixes the DAG node insertion order (bayesian_network.py:31-32
        iterates ``dag.nodes``); default: the columns order.  ``estimators``:
        node -> fitted OracleParametric (default: BruteForce fitted on data).
        """
        self.dag = nx.DiGraph()
        self.dag.add_nodes_from(list(nodes) if nodes is not None else list(columns))
        self.dag.add_edges_from(edges)
        col = {c: i for i, c in enumerate(columns)}
        self.nodes: Dict[str, OracleNode] = {}
        for n in self.dag.nodes:
            parents = sorted(self.dag.predecessors(n))
            nd = OracleNode(n, parents, (estimators or {}).get(n))
            pdata = np.stack([data[:, col[p]] for p in parents], 0) if parents else None
            nd.fit(data[:, col[n]], pdata)
            self.nodes[n] = nd

    def ancestors(self, target: str) -> List[str]:
        """bayesian_network.py:86-102."""
        anc = nx.ancestors(self.dag, target)
        order = list(nx.topological_sort(self.dag.subgraph(anc | {target})))
        order.remove(target)
        return order

    def infer(self, target: str, evidence: Optional[Dict[str, np.ndarray]], N_max: int = 16):
        """bayesian_network.py:208-305.  Returns (pdf [Q, N], domain [Qt, N])."""
        raw, dom = self.infer_raw(target, evidence, N_max)
        out = raw / raw.max()
        return out.astype(np.float32), dom

    def infer_raw(self, target: str, evidence: Optional[Dict[str, np.ndarray]], N_max: int = 16):
        """bayesian_network.py:208-295: the factor product before the global-max
        division of :296 (used to check the sharded normalisation)."""
        order = self.ancestors(target) + [target]
        factors = {}
        tdom = None
        for n in order:
            parents = sorted(self.dag.predecessors(n))
            q = {f: v for f, v in (evidence or {}).items() if f in parents}
            pdf, dom = self.nodes[n].get_prob(q, N_max)
            factors[n] = pdf
            if n == target:
                tdom = dom
        if evidence:
            nq = next(iter(evidence.values())).shape[0]
        else:
            nq = 1
        ns = self.nodes[target].sample_domain(target, N_max).shape[0]
        out = np.ones((nq, ns), np.float32)
        for n, pdf in factors.items():
            if pdf.ndim > 2:
                dims = tuple(range(1, pdf.ndim - 1))
            else:
                dims = (1,)
            # torch.mean's CPU reduction is cascaded (error ~ a few ulp for any
            # count); numpy's float32 mean over several axes accumulates
            # sequentially (error ~ count x ulp: 1e-3 at 4^10 combos), so the
            # mean is accumulated in float64 and rounded once
            x = pdf.astype(np.float32).mean(axis=dims, dtype=np.float64).astype(np.float32)
            out = (out * x).astype(np.float32)
        if out.size == 0:
            raise RuntimeError("max(): Expected reduction dim to be specified for input.numel() == 0.")
        if out.shape != tdom.shape:
            raise AssertionError("pdf and domain must have same shape.")
        return out, np.ascontiguousarray(tdom)
