"""BruteForce (discrete maximum-likelihood) estimator on MI355X.

Mirrors cbn/parameter_learning/brute_force.py (same class name, constructor,
``fit`` / ``get_prob`` / ``sample`` semantics and error behaviour).  What
changes is the representation: the reference keeps the unique
``[parents..., node, prob]`` rows (``mle_tensor``, :55-66) and answers every
``get_prob`` with two equality scans over all rows (:240-254, O(points x rows)).
Here ``fit`` also compiles the rows into a dense conditional table
``cpd[parent idx..., node idx] = joint / (parent marginal + 1e-10)`` by the HIP
kernels ``k_cpd_scatter`` / ``k_cpd_normalize`` (``cbn_bf_cpd_build``), and
``get_prob`` maps each value to its domain index by binary search and gathers
(``cbn_bf_cpd_eval``).  Values absent from the fitted domain give 0, exactly the
reference's ``0 / (0 + 1e-10)``.

The dense table is compiled lazily on first device use, so the host logic can
be exercised without a GPU; every evaluation requires the HIP library.
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Optional

import torch

from .. import _native
from ..base.parameter_learning import BaseParameterLearningEstimator

MAX_DENSE_CELLS = 1 << 28  # 1 GiB of fp32 per CPD


class BruteForce(BaseParameterLearningEstimator):
    def __init__(self, config: Dict, **kwargs):
        super().__init__(config=config, **kwargs)
        self.mle_tensor = None
        self.domains: Optional[List[torch.Tensor]] = None  # sorted values per column
        self.cpd: Optional[torch.Tensor] = None  # dense [card_parents..., card_node]
        self.node_marginal: Optional[torch.Tensor] = None  # [card_node]
        self._rows = None
        self._probs = None
        self._setup_model(config, **kwargs)

    def _setup_model(self, config: Dict = None, **kwargs):
        pass

    # -------------------------------------------------------------- fit ----
    def _fit(self, node_data: torch.Tensor, parents_data: torch.Tensor = None):
        """brute_force.py:30-66: unique rows + empirical probabilities."""
        node_data = node_data.view(-1, 1)
        if parents_data is not None:
            parents_data = parents_data.T
            all_data = torch.empty((node_data.shape[0], parents_data.shape[1] + 1),
                                   dtype=node_data.dtype, device=node_data.device)
            all_data[:, :-1] = parents_data
            all_data[:, -1] = node_data.squeeze(-1)
        else:
            all_data = node_data
        unique_rows, counts = torch.unique(all_data, dim=0, return_counts=True)
        probs = counts.float() / counts.sum()
        self.mle_tensor = torch.empty((unique_rows.shape[0], unique_rows.shape[1] + 1),
                                      dtype=unique_rows.dtype, device=self.device)
        self.mle_tensor[:, :-1] = unique_rows
        self.mle_tensor[:, -1] = probs
        self._rows = self.mle_tensor[:, :-1].to(torch.float32)
        self._probs = self.mle_tensor[:, -1].to(torch.float32).contiguous()
        self.domains = [torch.unique(self._rows[:, c]).contiguous() for c in range(self._rows.shape[1])]
        self.cpd = None
        self.node_marginal = None

    @property
    def cards(self) -> List[int]:
        return [int(d.numel()) for d in self.domains]

    def compiled(self):
        """Dense CPD on the device (built once per fit by the HIP kernels)."""
        assert self.mle_tensor is not None, "MLE tensor not fitted yet. Call _fit() first."
        if self.cpd is not None:
            return self.cpd
        dev = _native.require_gpu(self.mle_tensor.device)
        lib = _native.load()
        cards = self.cards
        n_cells = 1
        for c in cards:
            n_cells *= c
        if n_cells > MAX_DENSE_CELLS:
            raise _native.NativeError(
                f"BruteForce dense CPD would hold {n_cells} cells (> {MAX_DENSE_CELLS}); "
                "this estimator targets discrete domains")
        with torch.cuda.device(dev):
            cell = torch.zeros(self._rows.shape[0], dtype=torch.int64, device=dev)
            stride = 1
            idx_last = None
            for c in range(len(cards) - 1, -1, -1):
                idx = torch.searchsorted(self.domains[c], self._rows[:, c].contiguous())
                if c == len(cards) - 1:
                    idx_last = idx
                cell += idx * stride
                stride *= cards[c]
            cell32 = cell.to(torch.int32).contiguous()
            cpd = torch.empty(n_cells, dtype=torch.float32, device=dev)
            n_pcells = n_cells // cards[-1]
            _native.check(lib.cbn_bf_cpd_build(_native.ptr(cell32), _native.ptr(self._probs),
                                               cell32.numel(), n_pcells, cards[-1],
                                               1 if len(cards) > 1 else 0, _native.ptr(cpd),
                                               _native.stream_ptr(dev)), "cbn_bf_cpd_build")
            # P(node value) over all rows: the query=None case of brute_force.py:205-214
            marg = torch.zeros(cards[-1], dtype=torch.float32, device=dev)
            marg.index_add_(0, idx_last, self._probs)
        self.cpd = cpd.view(*cards)
        self.node_marginal = marg
        return self.cpd

    # ------------------------------------------------------------- eval ----
    def eval_points(self, points: torch.Tensor, table: Optional[torch.Tensor] = None,
                    domains: Optional[List[torch.Tensor]] = None) -> torch.Tensor:
        """cpd at float points [n, n_cols] (columns = parents..., node)."""
        cpd = self.compiled() if table is None else table
        domains = self.domains if domains is None else domains
        dev = cpd.device
        lib = _native.load()
        pts = points.to(device=dev, dtype=torch.float32).contiguous()
        n_cols = len(domains)
        assert pts.dim() == 2 and pts.shape[1] == n_cols
        out = torch.empty(pts.shape[0], dtype=torch.float32, device=dev)
        dom_ptrs = (ctypes.c_void_p * n_cols)(*[d.data_ptr() for d in domains])
        card_arr = (ctypes.c_int32 * n_cols)(*[int(d.numel()) for d in domains])
        with torch.cuda.device(dev):
            _native.check(lib.cbn_bf_cpd_eval(_native.ptr(cpd.contiguous()), n_cols, dom_ptrs, card_arr,
                                              _native.ptr(pts), pts.shape[0], _native.ptr(out),
                                              _native.stream_ptr(dev)), "cbn_bf_cpd_eval")
        return out

    def _get_prob(self, point_to_evaluate: torch.Tensor, query: torch.Tensor = None):
        """brute_force.py:185-257 semantics, evaluated by table lookup."""
        assert self.mle_tensor is not None, "MLE tensor not fitted yet. Call _fit() first."
        n_node_values = point_to_evaluate.shape[1]
        if query is None:
            self.compiled()
            pts = point_to_evaluate.reshape(-1, 1)
            out = self.eval_points(pts, table=self.node_marginal, domains=[self.domains[-1]])
            return out.view(point_to_evaluate.shape).to(point_to_evaluate.dtype)
        assert query.dim() == 3 and query.shape[-1] == 1, \
            f"Query must be [n_queries, n_parents, 1]. Got {query.shape}."
        n_queries, n_parents, _ = query.shape
        if point_to_evaluate.shape[0] != n_queries:
            raise ValueError(
                f"'point_to_evaluate' first dimension must match number of queries. "
                f"Got {point_to_evaluate.shape[0]}, expected {n_queries}.")
        dev = self.mle_tensor.device
        pq = query.squeeze(-1).to(device=dev, dtype=torch.float32)
        full = torch.empty((n_queries, n_node_values, n_parents + 1), dtype=torch.float32, device=dev)
        full[:, :, :-1] = pq.unsqueeze(1)
        full[:, :, -1] = point_to_evaluate.to(device=dev, dtype=torch.float32)
        return self.eval_points(full.view(-1, n_parents + 1)).view(n_queries, n_node_values)

    def _sample(self, N: int, **kwargs):
        """brute_force.py:259-278: N rows drawn from the empirical joint."""
        assert self.mle_tensor is not None, "MLE tensor not fitted yet. Call _fit() first."
        probs = self.mle_tensor[:, -1]
        indices = torch.multinomial(probs, N, replacement=True)
        return self.mle_tensor[indices, :-1]

    def save_model(self, path: str):
        raise NotImplementedError

    def load_model(self, path: str):
        raise NotImplementedError
