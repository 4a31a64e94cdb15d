"""Node: one variable, its parents and its probability estimator.

Mirrors cbn/base/node.py (constructor, ``fit`` validation, the ``info`` domain
bookkeeping, ``sample_domain`` including its random padding, ``get_prob`` output
shapes).  The per-query Python loops of the reference (node.py:178-193 and the
meshgrid loop at :360-373) are replaced by one batched evaluation on the device.
"""
from __future__ import annotations

import random
from typing import Dict, List, Tuple

import torch

from . import BASE_MAX_CARDINALITY, KEY_CONTINUOUS, KEY_DISCRETE, KEY_MAX_CARDINALITY_FOR_DISCRETE
from ..utils import choose_probability_estimator

# Source of the uniform draws sample_domain consumes for N > |domain|
# (node.py:313-317: random.uniform -> random.random()).  None: Python's global
# ``random``, as the reference.  distributed.shared_draws installs a callable
# n -> n floats so that every rank of a sharded call uses rank 0's draws.
_DRAWS = [None]


def uniforms(n: int) -> list:
    """The next n ``random.random()`` values of this process's draw source."""
    src = _DRAWS[0]
    return [random.random() for _ in range(n)] if src is None else src(n)


class Node:
    def __init__(self, node_name: str, estimator_name: str, parameter_learning_config: Dict,
                 parents_names: List[str] = None, **kwargs):
        self.node_name = node_name
        self.parameter_learning_config = parameter_learning_config
        self.parents_names = parents_names if parents_names else []
        self.device = kwargs.get("device", "cuda" if torch.cuda.is_available() else "cpu")
        self.max_cardinality_for_discrete_domain = kwargs.get(
            KEY_MAX_CARDINALITY_FOR_DISCRETE, BASE_MAX_CARDINALITY)
        self.plot_prob = kwargs.get("plot_prob", False)
        self.fixed_dtype = kwargs.get("fixed_dtype", torch.float32)
        self.estimator = choose_probability_estimator(estimator_name, parameter_learning_config, **kwargs)
        self.info = {}

    # -------------------------------------------------------------- fit ----
    def fit(self, node_data: torch.Tensor, parents_data: torch.Tensor = None, **kwargs):
        """node.py:45-110.  node_data [n_samples]; parents_data [n_parents, n_samples]."""
        if len(self.parents_names) > 0:
            if parents_data is not None:
                if len(self.parents_names) != parents_data.shape[0]:
                    raise ValueError(
                        f"number of parents features in input ({parents_data.shape[0]}) is not equal to "
                        f"number of parents node set ({len(self.parents_names)})")
                start = self.parents_names
                self.parents_names = sorted(self.parents_names)
                parents_data = parents_data[[start.index(v) for v in self.parents_names]]
            else:
                raise ValueError(
                    f"parents data is empty; should be [{node_data.shape[0], len(self.parents_names)}]")
        elif parents_data is not None:
            raise ValueError("there are no parents for which setting data.")

        self.estimator.fit(node_data, parents_data)

        uniq = torch.unique(node_data)
        self.info[self.node_name] = [
            torch.min(node_data), torch.max(node_data),
            KEY_CONTINUOUS if len(uniq) > self.max_cardinality_for_discrete_domain else KEY_DISCRETE,
            uniq,
        ]
        if parents_data is not None and len(self.parents_names) > 0:
            uniq_cols = torch.unique(parents_data, dim=1)
            for i, parent in enumerate(self.parents_names):
                self.info[parent] = [
                    torch.min(parents_data[i]), torch.max(parents_data[i]),
                    KEY_CONTINUOUS if len(uniq_cols[i]) > self.max_cardinality_for_discrete_domain
                    else KEY_DISCRETE,
                    torch.unique(uniq_cols[i]),
                ]

    def sample(self, N: int, **kwargs) -> torch.Tensor:
        return self.estimator.sample(N, **kwargs)

    # ----------------------------------------------------------- domains ---
    def sample_domain(self, node: str, N: int = 1024) -> torch.Tensor:
        """node.py:286-333: N evaluation points of ``node``'s domain.

        N < |domain|: ``linspace`` index subsample; N == |domain|: the domain;
        N > |domain|: the domain plus N-|domain| values drawn with Python's
        global ``random`` as ``min + (max - min) * random.random()`` in float32
        (``random.uniform`` on the 0-dim tensors kept in ``info``), then sorted.
        """
        min_value, max_value, _, domain_values = self.info[node]
        card = domain_values.shape[0]
        if N < card:
            idx = torch.linspace(start=0, end=card - 1, steps=N).round().long()
            return domain_values[idx.to(domain_values.device)]
        if N == card:
            return domain_values
        out, _ = self._sample_points(node, N)
        return out.to(domain_values.device)

    def _sample_points(self, node: str, N: int) -> Tuple[torch.Tensor, bool]:
        """sample_domain's points, consuming ``random`` identically; for
        N > |domain| they are built on the host ((points, True)) -- the engine
        maps a redrawn plan's points to domain indices there and uploads only
        the indices -- otherwise (sample_domain(node, N), False)."""
        min_value, max_value, _, domain_values = self.info[node]
        card = domain_values.shape[0]
        if N <= card:
            return self.sample_domain(node, N), False
        needed = N - card
        # host copies of min, max - min and the domain, cached per info entry:
        # device reads on every redraw would be a stream sync per node per call
        cache = self.__dict__.setdefault("_span_cache", {})
        hit = cache.get(node)
        if hit is None or hit[0] is not min_value or hit[1] is not max_value or hit[2] is not domain_values:
            lo = min_value.detach().to("cpu", torch.float32)
            hit = cache[node] = (min_value, max_value, domain_values, lo,
                                 max_value.detach().to("cpu", torch.float32) - lo, domain_values.detach().cpu())
        lo, span, host_dom = hit[3], hit[4], hit[5]
        # lo + span * r on 0-dim float32 tensors (random.uniform): r is rounded to
        # float32 first, then one float32 multiply and one add -- vectorised
        new_values = lo + span * torch.tensor(uniforms(needed), dtype=torch.float64).to(torch.float32)
        out = torch.cat([host_dom, new_values.to(dtype=host_dom.dtype)])
        out, _ = torch.sort(out)
        return out, True

    @staticmethod
    def sample_domain_is_deterministic(info_entry, N: int) -> bool:
        return N <= info_entry[3].shape[0]

    # -------------------------------------------------------------- prob ---
    def get_prob(self, query: Dict[str, torch.Tensor], N: int = 1024
                 ) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        """node.py:115-204.

        :return: pdf [n_queries, d_0..d_{k-1}, N] (d_i = N when some parent is
                 unobserved, else 1), target domains [n_queries, N], parents'
                 evaluation points.
        """
        if query:
            n_queries = next(iter(query.values())).shape[0]
            for feat, tensor in query.items():
                assert tensor.shape[0] == n_queries, ValueError("n_queries must be equal for all features.")
                assert tensor.dim() == 2, ValueError("Each query tensor must be of dimension 2.")
        else:
            n_queries = 1
        node_query = query.pop(self.node_name, None)
        parents_query, parents_domains = self._setup_parents_query(query, N)
        combos = parents_query.shape[2] if parents_query is not None else 0
        if node_query is None:
            target_node_domains = self.sample_domain(self.node_name, N).unsqueeze(0).expand(n_queries, -1)
        else:
            target_node_domains = node_query
        n_samples_node = target_node_domains.shape[1]
        k = len(self.parents_names)
        parent_dims = [N if combos > 1 else 1 for _ in self.parents_names]
        if k > 0:
            if combos > 1:
                n_start = parents_query.shape[0]
                pdfs = self._eval_grid(parents_query, target_node_domains[:n_start])
            else:
                pdfs = self.estimator.get_prob(target_node_domains, parents_query[:, :, 0, None]).unsqueeze(1)
        else:
            pdfs = self.estimator.get_prob(target_node_domains)
        pdfs = pdfs.reshape([n_queries] + parent_dims + [n_samples_node])
        if self.plot_prob:
            self._plot_pdfs(pdfs, target_node_domains, parents_domains)
        return pdfs, target_node_domains, parents_domains

    def _eval_grid(self, parents_query: torch.Tensor, domains: torch.Tensor) -> torch.Tensor:
        """pdf[i, c, v] = P(domains[i, v] | parents_query[i, :, c]) for all i at once."""
        n_start, k, combos = parents_query.shape
        nv = domains.shape[1]
        if hasattr(self.estimator, "eval_grid"):  # parametric estimators: one kernel call
            return self.estimator.eval_grid(parents_query, domains)
        if hasattr(self.estimator, "eval_points"):
            pts = torch.empty((n_start, combos, nv, k + 1), dtype=torch.float32, device=parents_query.device)
            pts[..., :k] = parents_query.permute(0, 2, 1).unsqueeze(2).to(torch.float32)
            pts[..., k] = domains.unsqueeze(1).to(device=pts.device, dtype=torch.float32)
            return self.estimator.eval_points(pts.view(-1, k + 1)).view(n_start, combos, nv)
        out = torch.empty((n_start, combos, nv), dtype=self.fixed_dtype, device=self.device)
        q_all = parents_query.permute(2, 1, 0)
        for i in range(n_start):
            out[i] = self.estimator.get_prob(domains[i].unsqueeze(0).expand(combos, -1), q_all[:, :, i, None])
        return out

    def _setup_parents_query(self, query: Dict[str, torch.Tensor], N: int):
        """node.py:206-284."""
        query_features = sorted(query.keys())
        query = {key: query[key] for key in query_features}
        k = len(self.parents_names)
        if len(query_features) > 0:
            n0 = query[query_features[0]].shape[0]
            assert all(f in self.parents_names for f in query_features), \
                ValueError("You have specified parent features that don't exist")
            if query_features == self.parents_names:
                new_query = torch.zeros((n0, k, 1), device=self.device)
                for i, parent in enumerate(self.parents_names):
                    new_query[:, i, :] = query[parent]
                return new_query, new_query
            pts = torch.empty((n0, k, N), device=self.device, dtype=self.fixed_dtype)
            for i, parent in enumerate(self.parents_names):
                if parent in query_features:
                    pts[:, i, :] = query[parent].expand(-1, N)
                else:
                    pts[:, i, :] = self.sample_domain(parent, N).unsqueeze(0).expand(n0, -1)
            return self._batched_meshgrid_combinations(pts), pts
        if k > 0:
            pts = torch.empty((1, k, N), device=self.device, dtype=self.fixed_dtype)
            for i, parent in enumerate(self.parents_names):
                pts[:, i, :] = self.sample_domain(parent, N).unsqueeze(0)
            return self._batched_meshgrid_combinations(pts), pts
        return None, None

    def _batched_meshgrid_combinations(self, input_tensor: torch.Tensor, indexing: str = "ij") -> torch.Tensor:
        """node.py:335-375, vectorised: [nq, k, N] -> [nq, k, N**k] ('ij' order)."""
        nq, k, n = input_tensor.shape
        flat = torch.arange(n ** k, device=input_tensor.device)
        axes = list(range(k)) if indexing == "ij" else ([1, 0] + list(range(2, k)) if k >= 2 else [0])
        digits = []
        for i in range(k):
            pos = axes.index(i)
            digits.append((flat // (n ** (k - 1 - pos))) % n)
        idx = torch.stack(digits, 0).unsqueeze(0).expand(nq, -1, -1)
        return torch.gather(input_tensor.to(self.fixed_dtype), 2, idx)

    # ------------------------------------------------------------ save -----
    def save_node(self, path: str):
        self.estimator.save_model(path)

    def load_node(self, path: str):
        self.estimator.load_model(path)

    def _plot_pdfs(self, pdfs, node_domains, parents_domains=None):
        """Marginal / conditional plots (node.py:526-628), reduced to one figure per query."""
        import matplotlib.pyplot as plt

        p = pdfs.detach().cpu().numpy()
        d = node_domains.detach().cpu().numpy()
        for q in range(p.shape[0]):
            y = p[q].reshape(-1, p.shape[-1]).sum(0)
            y = y / y.sum() if y.sum() > 0 else y
            plt.figure(dpi=150)
            plt.plot(d[q], y)
            plt.xlabel(f"Domain of {self.node_name}")
            plt.ylabel("PDF")
            plt.title(f"Query {q} - P({self.node_name}|{','.join(self.parents_names)})")
            plt.grid(True)
            plt.show()
