"""BruteForce (discrete maximum-likelihood) estimator on MI355X.

Mirrors cbn/parameter_learning/brute_force.py (same class name, constructor,
``fit`` / ``get_prob`` / ``sample`` semantics and error behaviour).  What
changes is the representation: the reference keeps the unique
``[parents..., node, prob]`` rows (``mle_tensor``, :55-66) and answers every
``get_prob`` with two equality scans over all rows (:227-241, O(points x rows)).
Here ``fit`` also compiles the rows into a dense conditional table
``cpd[parent idx..., node idx] = joint / (parent marginal + 1e-10)`` by the HIP
kernels ``k_cpd_scatter`` / ``k_cpd_normalize`` (``cbn_bf_cpd_build``), and
``get_prob`` maps each value to its domain index by binary search and gathers
(``cbn_bf_cpd_eval``).  Values absent from the fitted domain give 0, exactly the
reference's ``0 / (0 + 1e-10)``.

When the dense table would exceed ``dense_limit`` cells (continuous or
high-cardinality columns: the table is prod(cards) while the reference only
stores the U unique rows), ``fit`` compiles a SPARSE CPD instead: the U
conditionals keyed by their mixed-radix domain index in an open-addressing
hash table of 2^ceil(log2 2U) slots (``cbn_hash_build``), evaluated by
``cbn_cpd_ref_eval`` and by direct inference plans (csrc/cbn_direct.hip).  The
key is an int64, so the product of the column cardinalities must stay below
2^62 (e.g. four columns of ~60 000 distinct values, or five of ~6 000); a
larger node raises NotImplementedError when it is first evaluated.

The table is compiled lazily on first device use, so the host logic can be
exercised without a GPU; every evaluation requires the HIP library.
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Optional

import torch

from .. import _native
from ..base.parameter_learning import BaseParameterLearningEstimator

MAX_DENSE_CELLS = 1 << 24  # 64 MiB of fp32 per dense CPD; larger CPDs are hashed
MAX_KEY_CELLS = 1 << 62  # hashed CPDs: mixed-radix int64 keys over the columns' domain indices


def sparse_conditionals(cell: torch.Tensor, probs: torch.Tensor, card_node: int, conditional: bool) -> torch.Tensor:
    """Value of each unique row of a hashed CPD (cell = mixed-radix domain
    index, node column last): joint / (parent marginal + 1e-10), the sums of
    brute_force.py:227-241 over the rows sharing the row's parent values; the
    root case (:192-201) keeps the joint."""
    if not conditional:
        return probs.clone()
    pcell = torch.div(cell, card_node, rounding_mode="floor")
    _, inv = torch.unique(pcell, return_inverse=True)
    # summed in fp64 and rounded once (k_cpd_normalize's convention: within an
    # ulp of the exact marginal, and independent of the atomics' order)
    pmarg = torch.zeros(int(inv.max()) + 1 if inv.numel() else 0, dtype=torch.float64, device=probs.device)
    pmarg.index_add_(0, inv, probs.double())
    return probs / (pmarg.float()[inv] + 1e-10)


def hash_capacity(n: int) -> int:
    """Slots of the open-addressing table for n keys: power of two >= 2n (load <= 1/2)."""
    cap = 2
    while cap < 2 * n:
        cap *= 2
    return cap


class BruteForce(BaseParameterLearningEstimator):
    def __init__(self, config: Dict, **kwargs):
        super().__init__(config=config, **kwargs)
        self.mle_tensor = None
        self.domains: Optional[List[torch.Tensor]] = None  # sorted values per column
        self.cpd: Optional[torch.Tensor] = None  # dense [card_parents..., card_node]
        self.node_marginal: Optional[torch.Tensor] = None  # [card_node]
        self._rows = None
        self._probs = None
        # dense CPD above this many cells -> hashed unique rows (sparse)
        self.dense_limit = int(kwargs.get("dense_limit", config.get("dense_limit", MAX_DENSE_CELLS)
                                          if isinstance(config, dict) else MAX_DENSE_CELLS))
        self.sparse = False
        self.hash_keys: Optional[torch.Tensor] = None  # int64 [capacity], -1 empty
        self.hash_vals: Optional[torch.Tensor] = None  # float32 [capacity]
        self._compiled = False
        self._setup_model(config, **kwargs)

    def _setup_model(self, config: Dict = None, **kwargs):
        pass

    # -------------------------------------------------------------- fit ----
    def _fit(self, node_data: torch.Tensor, parents_data: torch.Tensor = None):
        """brute_force.py:17-53: unique rows + empirical probabilities."""
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
        self.hash_keys = self.hash_vals = None
        self.sparse = False
        self._compiled = False

    @property
    def cards(self) -> List[int]:
        return [int(d.numel()) for d in self.domains]

    def n_cells(self) -> int:
        n = 1
        for c in self.cards:
            n *= c
        return n

    def compiled(self):
        """The device CPD, built once per fit by the HIP kernels: the dense
        table (returned), or -- above ``dense_limit`` cells -- the hashed
        unique rows (``self.sparse``; returns None)."""
        assert self.mle_tensor is not None, "MLE tensor not fitted yet. Call _fit() first."
        if self._compiled:
            return self.cpd
        cards = self.cards
        n_cells = self.n_cells()
        if n_cells >= MAX_KEY_CELLS:
            # the hashed CPD keys a row by its mixed-radix domain index in an
            # int64 (the direct plans add free-parent terms to a precomputed
            # partial key): beyond 2^62 cells that index no longer fits
            raise NotImplementedError(
                f"BruteForce CPD over {len(cards)} columns with {n_cells:.3e} value combinations (cards {cards}): "
                f"hashed CPD keys are mixed-radix int64 indices, limited to < 2^62 combinations")
        dev = _native.require_gpu(self.mle_tensor.device)
        lib = _native.load()
        with torch.cuda.device(dev):
            rows = self._rows.to(dev)
            probs = self._probs.to(dev)
            cell = torch.zeros(rows.shape[0], dtype=torch.int64, device=dev)
            stride = 1
            idx_last = None
            for c in range(len(cards) - 1, -1, -1):
                idx = torch.searchsorted(self.domains[c].to(dev), rows[:, c].contiguous())
                if c == len(cards) - 1:
                    idx_last = idx
                cell += idx * stride
                stride *= cards[c]
            # P(node value) over all rows: the query=None case of brute_force.py:192-201
            # (fp64, rounded once: see sparse_conditionals)
            marg = torch.zeros(cards[-1], dtype=torch.float64, device=dev)
            marg.index_add_(0, idx_last, probs.double())
            marg = marg.float()
            if n_cells <= self.dense_limit:
                cell32 = cell.to(torch.int32).contiguous()
                cpd = torch.empty(n_cells, dtype=torch.float32, device=dev)
                n_pcells = n_cells // cards[-1]
                _native.check(lib.cbn_bf_cpd_build(_native.ptr(cell32), _native.ptr(probs),
                                                   cell32.numel(), n_pcells, cards[-1],
                                                   1 if len(cards) > 1 else 0, _native.ptr(cpd),
                                                   _native.stream_ptr(dev)), "cbn_bf_cpd_build")
                self.cpd = cpd.view(*cards)
            else:
                self._build_sparse(lib, dev, cell, probs, cards[-1], len(cards) > 1)
        self.node_marginal = marg
        self._compiled = True
        return self.cpd

    def _build_sparse(self, lib, dev, cell: torch.Tensor, probs: torch.Tensor, card_node: int, conditional: bool):
        """Hashed CPD: value of unique row u = joint_u / (sum of joint over the
        rows sharing u's parent values + 1e-10) (brute_force.py:227-241), the
        root case without the division (:192-201)."""
        vals = sparse_conditionals(cell, probs, card_node, conditional)
        n = cell.numel()
        cap = hash_capacity(n)
        keys = torch.empty(cap, dtype=torch.int64, device=dev)
        tvals = torch.empty(cap, dtype=torch.float32, device=dev)
        cell = cell.contiguous()
        vals = vals.contiguous()
        _native.check(lib.cbn_hash_build(_native.ptr(cell), _native.ptr(vals), n, _native.ptr(keys),
                                          _native.ptr(tvals), cap, _native.stream_ptr(dev)), "cbn_hash_build")
        self.sparse = True
        self.cpd = None
        self.hash_keys, self.hash_vals = keys, tvals

    def cpd_ref(self):
        """(cbn_cpd_ref, host arrays it points into) of the compiled CPD."""
        self.compiled()
        n = len(self.domains)
        doms = (ctypes.c_void_p * n)(*[d.data_ptr() for d in self.domains])
        cards = (ctypes.c_int32 * n)(*self.cards)
        r = _native.CpdRef()
        r.n_cols = n
        r.domains = ctypes.cast(doms, ctypes.POINTER(ctypes.c_void_p))
        r.cards = ctypes.cast(cards, ctypes.POINTER(ctypes.c_int32))
        if self.sparse:
            r.keys, r.vals, r.capacity = self.hash_keys.data_ptr(), self.hash_vals.data_ptr(), self.hash_keys.numel()
        else:
            r.dense = self.cpd.data_ptr()
        return r, (doms, cards)

    # ------------------------------------------------------------- eval ----
    def eval_points(self, points: torch.Tensor, table: Optional[torch.Tensor] = None,
                    domains: Optional[List[torch.Tensor]] = None) -> torch.Tensor:
        """cpd at float points [n, n_cols] (columns = parents..., node)."""
        cpd = self.compiled() if table is None else table
        domains = self.domains if domains is None else domains
        dev = self.hash_keys.device if cpd is None else cpd.device
        lib = _native.load()
        pts = points.to(device=dev, dtype=torch.float32).contiguous()
        n_cols = len(domains)
        assert pts.dim() == 2 and pts.shape[1] == n_cols
        out = torch.empty(pts.shape[0], dtype=torch.float32, device=dev)
        with torch.cuda.device(dev):
            if table is None and (self.sparse or n_cols > _native.CBN_MAX_PARENTS + 1):
                ref, _keep = self.cpd_ref()
                _native.check(lib.cbn_cpd_ref_eval(ctypes.byref(ref), _native.ptr(pts), pts.shape[0],
                                                   _native.ptr(out), _native.stream_ptr(dev)), "cbn_cpd_ref_eval")
                return out
            dom_ptrs = (ctypes.c_void_p * n_cols)(*[d.data_ptr() for d in domains])
            card_arr = (ctypes.c_int32 * n_cols)(*[int(d.numel()) for d in domains])
            _native.check(lib.cbn_bf_cpd_eval(_native.ptr(cpd.contiguous()), n_cols, dom_ptrs, card_arr,
                                              _native.ptr(pts), pts.shape[0], _native.ptr(out),
                                              _native.stream_ptr(dev)), "cbn_bf_cpd_eval")
        return out

    def _get_prob(self, point_to_evaluate: torch.Tensor, query: torch.Tensor = None):
        """brute_force.py:172-244 semantics, evaluated by table lookup."""
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
        """brute_force.py:246-265: N rows drawn from the empirical joint."""
        assert self.mle_tensor is not None, "MLE tensor not fitted yet. Call _fit() first."
        probs = self.mle_tensor[:, -1]
        indices = torch.multinomial(probs, N, replacement=True)
        return self.mle_tensor[indices, :-1]

    def save_model(self, path: str):
        raise NotImplementedError

    def load_model(self, path: str):
        raise NotImplementedError
