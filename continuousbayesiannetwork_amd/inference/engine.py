"""Batched inference engine behind ``BayesianNetwork.infer``.

Reference path (cbn/base/bayesian_network.py:208-305): for every ancestor of the
target (topological order, target last) build the per-query pdf tensor
``[n_queries, d_0..d_{k-1}, N]`` with Node.get_prob, average it over the
parent axes, multiply the averages into ``out_pdf`` and divide by the global
max.  This engine computes the same numbers in three launches:

  1. ``k_build_tables``  -- every factor's mean over its unobserved parents as a
     small table (indexed by the observed parents' domain indices),
  2. ``k_query<max>``     -- per query/value product of the gathered table rows,
     folded into the global max,
  3. ``k_query<write>``   -- the same product divided by the max, written out.

Host work per call is one dict walk and one C call; the plan (descriptors,
sample-domain index arrays, device image) is cached per
(target, observed parent columns, N_max) when every sample domain is
deterministic (N_max <= |domain|).  When the reference would draw random
padding values (node.py:302-333) the plan is rebuilt on every call, consuming
Python's ``random`` in the reference's order, so results stay identical.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from .. import _native
from .._native import CBN_FACTOR_QUERY, CBN_FACTOR_SCALAR, CBN_FACTOR_SHARED, CBN_MAX_EVIDENCE, CBN_MAX_PARENTS
from ..base.parameter_learning import GENERATION


def domain_index(values: torch.Tensor, domain: torch.Tensor) -> torch.Tensor:
    """int32 index of each value in the sorted ``domain``; -1 when absent."""
    values = values.to(device=domain.device, dtype=domain.dtype).contiguous()
    i = torch.searchsorted(domain, values).clamp_(max=domain.numel() - 1)
    return torch.where(domain[i] == values, i, torch.full_like(i, -1)).to(torch.int32)


@dataclass
class FactorSpec:
    """Host-side description of one factor (also used by the CPU tests)."""
    node: str
    kind: int
    parents: List[str]
    observed: List[str]
    free_samples: Dict[str, torch.Tensor]
    node_samples: torch.Tensor


@dataclass
class Plan:
    target: str
    n_samples: int
    order: List[str]
    factors: List[FactorSpec]
    slots: List[str]
    target_domain: torch.Tensor
    target_observed: bool
    deterministic: bool
    handle: Optional[ctypes.c_void_p] = None
    keep: list = field(default_factory=list)
    max_bits: Optional[torch.Tensor] = None
    tables_built: bool = False
    direct: bool = False  # factors evaluated from the CPDs (cbn_plan_create_direct)
    # BruteForce plans read their sample points through device index arrays
    # (per factor: node [N], parents [k, N]; views of idx_flat) that the plan
    # only points at: a plan whose domains are redrawn every call
    # (N > |domain|) is kept and those arrays are overwritten in place before
    # each call (tables rebuilt)
    reusable: bool = False
    host_doms: Optional[list] = None  # redrawn plans: host copies of each factor's estimator domains
    idx_flat: Optional[torch.Tensor] = None  # every factor's sample-index arrays, one device buffer
    idx_offs: list = field(default_factory=list)  # per factor: (offset in idx_flat, number of parents)
    idx_host: Optional[torch.Tensor] = None  # redrawn plans: host mirror of idx_flat
    redraw: Optional["RedrawProgram"] = None  # redrawn plans: the per-call draws (host_fast.redraw jobs)
    observed: frozenset = frozenset()  # the observed parent columns the plan was built for

    def destroy(self):
        if self.handle is not None and self.handle.value:
            _native.load().cbn_plan_destroy(self.handle)
        self.handle = None
        self.keep = []


def relevant_observed(bn, order: Sequence[str], evidence_keys) -> frozenset:
    keys = set(evidence_keys)
    rel = set()
    for n in order:
        rel.update(p for p in bn.nodes_obj[n].parents_names if p in keys)
    return frozenset(rel)


def build_factor_specs(bn, target: str, observed: frozenset, N: int) -> Tuple[List[str], List[FactorSpec], torch.Tensor, bool]:
    """Walk the factors in the reference's order, calling sample_domain exactly
    where Node.get_prob / BayesianNetwork.infer do (node.py:243-256, 263-276,
    :153-156; bayesian_network.py:265-267)."""
    order = bn.get_ancestors(bn.initial_dag, target)
    order.append(target)
    specs = []
    deterministic = True
    target_dom = None
    for n in order:
        nd = bn.nodes_obj[n]
        parents = list(nd.parents_names)
        obs = [p for p in parents if p in observed]
        free = [p for p in parents if p not in obs] if (parents and obs != parents) else []
        free_samples = {}
        for p in parents:
            if p in free:
                deterministic &= nd.sample_domain_is_deterministic(nd.info[p], N)
                free_samples[p] = nd._sample_points(p, N)[0]  # (redrawn points stay on the host)
        deterministic &= nd.sample_domain_is_deterministic(nd.info[n], N)
        node_samples, on_host = nd._sample_points(n, N)
        kind = CBN_FACTOR_SCALAR if not parents else (CBN_FACTOR_QUERY if obs else CBN_FACTOR_SHARED)
        specs.append(FactorSpec(n, kind, parents, obs, free_samples, node_samples))
        if n == target:
            target_dom = node_samples.to(nd.info[n][3].device) if on_host else node_samples
    # bayesian_network.py:265-267 draws the target domain once more (shape only)
    bn.nodes_obj[target]._sample_points(target, N)
    return order, specs, target_dom, deterministic


def sample_calls(bn, order: Sequence[str], observed: frozenset):
    """The sample_domain calls of one infer, in the reference's order (the walk
    of build_factor_specs, without drawing): (factor index, node, variable,
    parent position or -1 for the node's own points); the final
    (-1, target, target, -1) is bayesian_network.py:265-267's shape-only draw."""
    calls = []
    for f, n in enumerate(order):
        parents = list(bn.nodes_obj[n].parents_names)
        obs = [p for p in parents if p in observed]
        if parents and obs != parents:
            calls += [(f, n, p, i) for i, p in enumerate(parents) if p not in obs]
        calls.append((f, n, n, -1))
    calls.append((-1, order[-1], order[-1], -1))
    return calls


def needs_redraw(bn, order: Sequence[str], observed: frozenset, N: int) -> bool:
    """True when some sample_domain call of the infer draws random padding
    (N > |domain|, node.py:302-333)."""
    return any(N > bn.nodes_obj[n].info[v][3].shape[0] for _, n, v, _ in sample_calls(bn, order, observed))


class RedrawProgram:
    """host_fast.redraw's job tables for a kept plan whose sample domains are
    redrawn on every call: one job per drawing sample_domain call, in the
    reference's order, each writing its sorted points' domain indices into the
    plan's host index mirror (and, for the target's own points, the returned
    target domain).  Built once per plan from the fitted domains (a refit
    drops the plan)."""

    def __init__(self, bn, plan: "Plan", observed: frozenset):
        N = plan.n_samples
        meta, lospan, doms, off = [], [], [], 0
        self.total = 0
        self.target_pts = False
        cache = {}

        def flat(t: torch.Tensor):
            nonlocal off
            key = id(t)
            if key not in cache:
                h = t.detach().to("cpu").contiguous()
                if h.dtype != torch.float32:
                    raise TypeError("redraw program needs float32 domains")
                doms.append(h)
                cache[key] = (off, h.numel(), t)  # (t kept alive: ids stay unique)
                off += h.numel()
            return cache[key][:2]

        for f, n, v, i in sample_calls(bn, plan.order, observed):
            nd = bn.nodes_obj[n]
            mn, mx, _, dom = nd.info[v]
            need = N - dom.shape[0]
            if need <= 0:
                continue  # deterministic: fixed in the plan's index arrays
            lo = mn.detach().to("cpu", torch.float32)
            span = mx.detach().to("cpu", torch.float32) - lo
            soff, slen = flat(dom)
            if f < 0:
                dest, loff, llen, pts = -1, 0, 0, 0
            else:
                est_doms = nd.estimator.domains
                loff, llen = flat(est_doms[-1] if i < 0 else est_doms[i])
                foff, _ = plan.idx_offs[f]
                dest = foff if i < 0 else foff + N * (1 + i)
                pts = 1 if (i < 0 and n == plan.target) else 0
                self.target_pts |= bool(pts)
            meta.append([need, soff, slen, loff, llen, dest, pts])
            lospan.append([float(lo), float(span)])
            self.total += need
        self.meta = torch.tensor(meta, dtype=torch.int64).reshape(-1, 7)
        self.lospan = torch.tensor(lospan, dtype=torch.float32).reshape(-1, 2)
        self.doms = torch.cat(doms) if doms else torch.zeros(1)
        self.pts = torch.empty(N, dtype=torch.float32)


def domain_index_host(values: torch.Tensor, domain: torch.Tensor) -> torch.Tensor:
    """domain_index on host tensors (CPU int32)."""
    values = values.to(dtype=domain.dtype).contiguous()
    i = torch.searchsorted(domain, values).clamp_(max=domain.numel() - 1)
    return torch.where(domain[i] == values, i, torch.full_like(i, -1)).to(torch.int32)


class _FastPath:
    """Everything the hot path needs for one cached (target, evidence keys, N)."""

    __slots__ = ("plan", "device", "first", "ptrs", "max_ptr", "lib", "tdom", "host", "run_fn", "slot_keys",
                 "scale_fn", "host_scale", "words", "redraw", "runner")

    def __init__(self, plan: "Plan", device: torch.device, first_key):
        self.plan = plan
        self.redraw = not plan.deterministic  # a kept plan whose sample domains are redrawn on every call
        self.device = device
        self.first = first_key
        self.ptrs = (ctypes.c_void_p * max(1, len(plan.slots)))()
        self.max_ptr = plan.max_bits.data_ptr()
        self.lib = _native.load()
        self.tdom = {}
        self.host = _native.load_host().run  # native per-call checks + output allocation + cbn_plan_run
        self.run_fn = ctypes.cast(self.lib.cbn_plan_run, ctypes.c_void_p).value
        self.slot_keys = tuple(plan.slots)
        self.host_scale = _native.load_host().scale
        self.scale_fn = ctypes.cast(self.lib.cbn_scale, ctypes.c_void_p).value
        # raw launches: one max word per block of the launch (0: plan has no raw launch)
        nw = self.lib.cbn_plan_max_words(plan.handle)
        self.words = torch.zeros(nw, dtype=torch.int32, device=device) if nw > 0 else None
        self.runner = None  # native Runner of this fast path (InferenceEngine._runner), built on first use


class InferenceEngine:
    """Factor tables depend only on the fitted CPDs and the plan (target,
    observed columns, N) -- never on evidence values -- so by default
    (``cache_tables=True``) each plan's tables are built once by
    ``k_build_tables`` and a call is the two query passes over the evidence.
    A refit (``fit`` / ``update_knowledge``) drops every plan.
    ``cache_tables=False`` re-runs the table build on every call (what the
    reference effectively does: it recomputes every factor per call)."""

    def __init__(self, bn, cache_tables: bool = True):
        self.bn = bn
        self.cache_tables = cache_tables
        self._plans: Dict[tuple, Plan] = {}
        # (target, observed, N, wide columns) -> (base plan, its direct plan for [Q, N] columns)
        self._wide_plans: Dict[tuple, tuple] = {}
        self._orders: Dict[str, List[str]] = {}
        # record HIP events around the two query passes inside the library
        # (bench.py's per-kernel timing; read back with timing())
        self._runner = None  # (target, N, native Runner) of the last fast path (see infer)
        self.timed = False
        # single-launch path (both passes, grid barrier on the max) when the
        # batch fits one round of the resident grid; False forces two launches
        self.fused = True
        self._fast: Dict[tuple, "_FastPath"] = {}
        self._gen = GENERATION[0]  # estimator generation last checked
        self._sig = self._signature()  # this network's estimator states the cached plans were built under
        # bumped whenever cached plans are destroyed: holders of raw plan
        # handles (distributed.ShardedStepper) rebuild when it moved
        self.epoch = 0
        # evaluate every BruteForce factor from its CPD (direct plans) even when
        # the table path could take the plan (tests; the direct path is chosen
        # by itself for hashed CPDs, > 8 parents and oversized tables)
        self.force_direct = False

    def _signature(self):
        if not self.bn.nodes_obj:
            return ()
        return tuple((id(nd.estimator), getattr(nd.estimator, "_stamp", 0)) for nd in self.bn.nodes_obj.values())

    def _check_generation(self):
        """Drop every cached plan when an estimator of THIS network was
        refitted / reloaded / edited (or replaced) since they were built (plans
        hold raw device pointers to the CPDs and packed weights of that
        state); another network's refit leaves them."""
        if GENERATION[0] != self._gen:
            sig = self._signature()
            if sig != self._sig:
                self.invalidate()
                self._sig = sig
            self._gen = GENERATION[0]

    # the per-call flags a runner was built under: changing one drops it
    @property
    def timed(self):
        return self._timed

    @timed.setter
    def timed(self, v):
        if getattr(self, "_timed", None) != v:
            self._runner = None
        self._timed = v

    @property
    def fused(self):
        return self._fused

    @fused.setter
    def fused(self, v):
        if getattr(self, "_fused", None) != v:
            self._runner = None
        self._fused = v

    @property
    def cache_tables(self):
        return self._cache_tables

    @cache_tables.setter
    def cache_tables(self, v):
        if getattr(self, "_cache_tables", None) != v:
            self._runner = None
        self._cache_tables = v

    def invalidate(self):
        self._runner = None
        if self._plans:
            torch.cuda.synchronize()
        self.epoch += 1
        for p in self._plans.values():
            p.destroy()
        for _, wp in self._wide_plans.values():
            wp.destroy()
        self._plans = {}
        self._wide_plans = {}
        self._orders = {}
        self._fast = {}

    def synchronize(self):
        """Wait for this engine's calls on the current device and report a call
        whose single-launch grid barrier timed out (its rows are NaN) NOW, as
        NativeError(CBN_E_TIMEOUT) -- without this, the plan's next call reports
        it.  Not in the reference (its infer has no grid barrier)."""
        torch.cuda.synchronize()
        lib = _native.load()
        for p in self._plans.values():
            if p.handle is not None and p.handle.value:
                _native.check(lib.cbn_plan_check(p.handle), "cbn_plan_check")

    def __del__(self):
        try:
            for p in self._plans.values():
                p.destroy()
            for _, wp in self._wide_plans.values():
                wp.destroy()
        except Exception:
            pass

    # ---------------------------------------------------------------- plan --
    def _materialise(self, plan: Plan, device: torch.device):
        ests = [self.bn.nodes_obj[s.node].estimator for s in plan.factors]
        param = [hasattr(e, "model_desc") for e in ests]
        if all(param):
            return self._materialise_param(plan, device)
        if any(param):
            raise NotImplementedError("a plan mixing BruteForce tables and parametric estimators is not supported "
                                      "(the reference fits one estimator type per network)")
        for spec in plan.factors:
            self.bn.nodes_obj[spec.node].estimator.compiled()
        if self.force_direct or any(self.bn.nodes_obj[s.node].estimator.sparse or len(s.parents) > CBN_MAX_PARENTS
                                    for s in plan.factors):
            return self._materialise_direct(plan, device)
        lib = _native.load()
        descs = (_native.FactorDesc * len(plan.factors))()
        keep = []
        slot_of = {v: i for i, v in enumerate(plan.slots)}
        N = plan.n_samples
        self._alloc_index_arrays(plan, device)
        keep.append(plan.idx_flat)
        with torch.cuda.device(device):
            for f, spec in enumerate(plan.factors):
                est = self.bn.nodes_obj[spec.node].estimator
                cpd = est.compiled()
                doms = est.domains
                # the plan's descriptors point into these: keep them alive with the plan
                keep += [cpd, est.node_marginal, *doms]
                d = descs[f]
                d.kind = spec.kind
                d.n_parents = len(spec.parents)
                d.node_card = int(doms[-1].numel())
                d.cpd = cpd.data_ptr() if spec.kind != CBN_FACTOR_SCALAR else est.node_marginal.data_ptr()
                nidx, pidx = self._index_arrays(plan, f, doms, 0)
                d.node_sample_idx = nidx.data_ptr()
                if pidx is not None:
                    d.parent_sample_idx = pidx.data_ptr()
                for i, p in enumerate(spec.parents):
                    d.parent_card[i] = int(doms[i].numel())
                    if p in spec.observed:
                        d.parent_ev_slot[i] = slot_of[p]
                        d.parent_domain[i] = doms[i].data_ptr()
                    else:
                        d.parent_ev_slot[i] = -1
            handle = ctypes.c_void_p()
            torch.cuda.current_stream(device).synchronize()  # index arrays ready before the D2D copies
            rc = lib.cbn_plan_create(descs, len(plan.factors), N, ctypes.byref(handle))
            if rc == _native.CBN_E_LIMIT:  # factor tables / N beyond the table path: evaluate directly
                return self._materialise_direct(plan, device)
            _native.check(rc, "cbn_plan_create")
        plan.handle = handle
        plan.keep = keep
        plan.reusable = True
        plan.max_bits = torch.zeros(1, dtype=torch.int32, device=device)

    def _materialise_direct(self, plan: Plan, device: torch.device, widths: Optional[Dict[str, int]] = None,
                            share_idx: Optional[Plan] = None):
        """cbn_direct_factor per ancestor (include/cbn_amd.h): each factor is
        evaluated per (query, sample column) from its CPD -- dense or hashed --
        with no per-plan table (nodes with > 8 parents, hashed CPDs of
        continuous / high-cardinality columns, factor tables beyond the
        table path's limits).  Same sample-index conventions as the table path.
        ``widths``: evidence columns taken as [Q, N] (_wide_plan);
        ``share_idx``: a plan of the same factors whose sample-index arrays
        this one reads (free-parent rows only, the same in both conventions)."""
        lib = _native.load()
        descs = (_native.DirectFactor * len(plan.factors))()
        keep = []
        slot_of = {v: i for i, v in enumerate(plan.slots)}
        N = plan.n_samples
        if share_idx is None:
            self._alloc_index_arrays(plan, device)
        else:
            plan.idx_flat, plan.idx_offs = share_idx.idx_flat, share_idx.idx_offs
        keep.append(plan.idx_flat)
        with torch.cuda.device(device):
            for f, spec in enumerate(plan.factors):
                est = self.bn.nodes_obj[spec.node].estimator
                est.compiled()
                doms = est.domains
                k = len(spec.parents)
                if k > _native.CBN_MAX_DIRECT_PARENTS:
                    raise _native.NativeError(f"node {spec.node}: {k} parents > {_native.CBN_MAX_DIRECT_PARENTS}")
                d = descs[f]
                d.kind = spec.kind
                d.n_parents = k
                if spec.kind == CBN_FACTOR_SCALAR:
                    # root: the node marginal (brute_force.py:192-201) as a one-column dense CPD
                    mdoms = (ctypes.c_void_p * 1)(doms[-1].data_ptr())
                    mcards = (ctypes.c_int32 * 1)(int(doms[-1].numel()))
                    ref = _native.CpdRef()
                    ref.n_cols = 1
                    ref.domains = ctypes.cast(mdoms, ctypes.POINTER(ctypes.c_void_p))
                    ref.cards = ctypes.cast(mcards, ctypes.POINTER(ctypes.c_int32))
                    ref.dense = est.node_marginal.data_ptr()
                    host = (mdoms, mcards)
                else:
                    ref, host = est.cpd_ref()
                d.cpd = ref
                keep += [host, est.cpd, est.hash_keys, est.hash_vals, est.node_marginal, *doms]
                if share_idx is None:
                    nidx, pidx = self._index_arrays(plan, f, doms, -1)
                else:
                    nidx, pidx = self._index_views(plan.idx_flat, *plan.idx_offs[f], N)
                d.node_sample_idx = nidx.data_ptr()
                if k:
                    ev = (ctypes.c_int32 * k)(*[slot_of[p] if p in spec.observed else -1 for p in spec.parents])
                    keep.append(ev)
                    d.parent_ev_slot = ctypes.cast(ev, ctypes.POINTER(ctypes.c_int32))
                    d.parent_sample_idx = pidx.data_ptr()
                    if widths:
                        w = (ctypes.c_int32 * k)(*[widths.get(p, 1) if p in spec.observed else 1
                                                   for p in spec.parents])
                        keep.append(w)
                        d.parent_ev_width = ctypes.cast(w, ctypes.POINTER(ctypes.c_int32))
            handle = ctypes.c_void_p()
            torch.cuda.current_stream(device).synchronize()  # index arrays ready before the plan reads them
            _native.check(lib.cbn_plan_create_direct(descs, len(plan.factors), N, ctypes.byref(handle)),
                          "cbn_plan_create_direct")
        plan.handle = handle
        plan.keep = keep
        plan.direct = True
        plan.reusable = True
        plan.max_bits = torch.zeros(1, dtype=torch.int32, device=device)

    def _materialise_param(self, plan: Plan, device: torch.device):
        """cbn_param_factor per ancestor (include/cbn_amd.h): the estimator's
        packed model, the input wiring (evidence slot / free parent sampled at
        sample_domain / constant 1 for roots) and the sample points -- the
        values Node.get_prob evaluates (node.py:152-193)."""
        lib = _native.load()
        descs = (_native.ParamFactor * len(plan.factors))()
        keep = []
        slot_of = {v: i for i, v in enumerate(plan.slots)}
        N = plan.n_samples
        with torch.cuda.device(device):
            for f, spec in enumerate(plan.factors):
                est = self.bn.nodes_obj[spec.node].estimator
                root = not spec.parents
                model, w = est.model_desc(root=root, device=device)
                keep += [w, getattr(model, "_widths_keep", None)]
                d = descs[f]
                d.kind = spec.kind
                d.model = model
                k = int(model.widths[0]) if model.widths else int(model.width[0])
                slots = [_native.CBN_INPUT_ONE] * k
                if not root:
                    if len(spec.parents) != k:
                        raise _native.NativeError(f"node {spec.node}: model has {k} inputs, {len(spec.parents)} parents")
                    samples = torch.zeros((k, N), dtype=torch.float32, device=device)
                    for i, p in enumerate(spec.parents):
                        if p in spec.observed:
                            slots[i] = slot_of[p]
                        else:
                            slots[i] = _native.CBN_INPUT_FREE
                            samples[i] = spec.free_samples[p].to(device=device, dtype=torch.float32)
                    keep.append(samples)
                    d.input_samples = samples.data_ptr()
                if k <= CBN_MAX_PARENTS:
                    for i, v in enumerate(slots):
                        d.input_slot[i] = v
                else:  # more inputs than the fixed array: the input_slots array
                    arr = (ctypes.c_int32 * k)(*slots)
                    keep.append(arr)
                    d.input_slots = ctypes.cast(arr, ctypes.POINTER(ctypes.c_int32))
                ns = spec.node_samples.to(device=device, dtype=torch.float32).contiguous()
                keep.append(ns)
                d.node_samples = ns.data_ptr()
            handle = ctypes.c_void_p()
            torch.cuda.current_stream(device).synchronize()  # sample/weight buffers ready before the D2D copies
            _native.check(lib.cbn_plan_create_param(descs, len(plan.factors), N, ctypes.byref(handle)),
                          "cbn_plan_create_param")
        plan.handle = handle
        plan.keep = keep
        plan.max_bits = torch.zeros(1, dtype=torch.int32, device=device)

    def plan(self, target: str, observed: frozenset, N: int, device) -> Plan:
        self._check_generation()
        key = (target, observed, int(N))
        p = self._plans.get(key)
        if p is not None:
            return p
        q = self._plans.get(("redrawn",) + key)
        if q is not None:
            self._redraw_plan(q)  # this call's draws
            return q
        order, specs, tdom, det = build_factor_specs(self.bn, target, observed, N)
        slots = sorted({o for s in specs for o in s.observed})
        if len(slots) > CBN_MAX_EVIDENCE:
            raise _native.NativeError(f"{len(slots)} observed columns > {CBN_MAX_EVIDENCE}")
        tobs = any(s.observed for s in specs if s.node == target)
        p = Plan(target, int(N), order, specs, slots, tdom, tobs, det)
        p.observed = observed
        self._materialise(p, device)
        if det:
            self._plans[key] = p
        elif p.reusable:
            self._plans[("redrawn",) + key] = p
            p.idx_host = p.idx_flat.cpu()  # host mirror: this call's indices; later calls rewrite the drawn ones
            try:
                p.redraw = RedrawProgram(self.bn, p, observed)
            except TypeError:  # non-float32 domains: later calls re-walk build_factor_specs
                p.redraw = None
        return p

    @staticmethod
    def _alloc_index_arrays(plan: Plan, device):
        """One flat int32 device buffer for every factor's sample-index arrays
        (node [N], parents [k, N]): a redrawn plan refreshes all of them with
        one upload per call."""
        N = plan.n_samples
        plan.idx_offs, off = [], 0
        for spec in plan.factors:
            plan.idx_offs.append((off, len(spec.parents)))
            off += N * (1 + len(spec.parents))
        plan.idx_flat = torch.empty(max(1, off), dtype=torch.int32, device=device)
        plan.idx_host = None

    @staticmethod
    def _index_views(flat: torch.Tensor, off: int, k: int, N: int):
        nidx = flat[off:off + N]
        return nidx, (flat[off + N:off + N * (1 + k)].view(k, N) if k else None)

    def _index_arrays(self, plan: Plan, f: int, doms, pfill: int):
        """Factor f's index arrays (views of plan.idx_flat), filled: the node's
        sample points -> domain index, free parents' likewise, other parent
        rows ``pfill``."""
        spec = plan.factors[f]
        off, k = plan.idx_offs[f]
        nidx, pidx = self._index_views(plan.idx_flat, off, k, plan.n_samples)
        nidx.copy_(domain_index(spec.node_samples, doms[-1]))
        if pidx is not None:
            pidx.fill_(pfill)
            for i, p in enumerate(spec.parents):
                if p in spec.free_samples:
                    pidx[i] = domain_index(spec.free_samples[p], doms[i])
        return nidx, pidx

    def _redraw_plan(self, plan: Plan):
        """This call's redrawn sample points (node.py:302-333) into a kept
        plan: the call's uniforms drawn in the reference's order
        (base.node.uniforms), every drawn domain's sorted points mapped to
        estimator-domain indices in ONE native host call (host_fast.redraw)
        into the plan's host index mirror, then one upload (stream-ordered after
        the plan's earlier launches); the tables / constant rows are rebuilt by
        the next launch."""
        from ..base.node import uniforms

        rd = plan.redraw
        if rd is None:
            return self._refresh_indices_walk(plan)
        _native.load_host().redraw(uniforms(rd.total), rd.meta, rd.lospan, rd.doms, plan.idx_host, rd.pts,
                                   plan.n_samples)
        plan.idx_flat.copy_(plan.idx_host)
        if rd.target_pts:  # a new tensor per call: earlier results keep their domain
            plan.target_domain = rd.pts.to(plan.idx_flat.device)
        plan.tables_built = False

    def _refresh_indices_walk(self, plan: Plan):
        """_redraw_plan for domains the job tables do not take (not float32):
        the draws through build_factor_specs, the index maps per factor."""
        _, specs, tdom, _ = build_factor_specs(self.bn, plan.target, plan.observed, plan.n_samples)
        if plan.host_doms is None:
            plan.host_doms = [[d.detach().cpu() for d in self.bn.nodes_obj[spec.node].estimator.domains]
                              for spec in specs]
        N = plan.n_samples
        for (off, k), spec, hd in zip(plan.idx_offs, specs, plan.host_doms):
            hn, hp = self._index_views(plan.idx_host, off, k, N)
            hn.copy_(domain_index_host(spec.node_samples.cpu(), hd[-1]))
            for i, p in enumerate(spec.parents):
                if p in spec.free_samples:
                    hp[i] = domain_index_host(spec.free_samples[p].cpu(), hd[i])
        plan.idx_flat.copy_(plan.idx_host)
        plan.target_domain = tdom
        plan.tables_built = False

    def redraws(self, target: str, evidence_keys, N_max: int) -> bool:
        """Whether an infer of (target, evidence keys, N) draws random sample
        points (the same answer on every rank of a sharded call)."""
        order = self._order(target)
        return needs_redraw(self.bn, order, relevant_observed(self.bn, order, evidence_keys), N_max)

    # --------------------------------------------------------------- infer --
    def _order(self, target: str) -> List[str]:
        order = self._orders.get(target)
        if order is None:
            order = self._orders[target] = self.bn.get_ancestors(self.bn.initial_dag, target) + [target]
        return order

    @staticmethod
    def check_columns(plan: Plan, evidence):
        """Raise what the reference raises for the plan's evidence columns, in
        the reference's order: per factor (ancestors, target last), the
        dimension / length asserts of Node.get_prob (node.py:127-135), then
        the parents' columns in ``parents_names`` order -- a node whose sorted
        evidence keys equal its ``parents_names`` copies each column into a
        [Q, 1] slot (``new_query[:, i, :] = query[parent]``, :233-234), any
        other node expands it to [Q, N] (``.expand(-1, N)``, :246-248): a
        RuntimeError unless the width is 1 (or N for the expand).

        A width-N column read only through ``.expand`` is accepted by the
        reference as N per-sample values of the observed parent (a per-query
        free parent): those columns are returned (a set, empty when every
        column is [Q, 1]) and run on a direct plan that averages over them
        (``_wide_plan``; cbn_direct_factor.parent_ev_width, ABI 5)."""
        N = plan.n_samples
        wide = set()
        for spec in plan.factors:
            if not spec.observed:
                continue
            cols = [evidence[p] for p in spec.observed]
            n0 = cols[0].shape[0]
            for t in cols:
                assert t.shape[0] == n0, ValueError("n_queries must be equal for all features.")
                assert t.dim() == 2, ValueError("Each query tensor must be of dimension 2.")
            strict = sorted(spec.observed) == list(spec.parents)
            for p in spec.observed:
                t = evidence[p]
                k = t.shape[1]
                if k == 1:
                    continue
                if strict or k != N:
                    target, shape = (1, f"[{n0}, 1]") if strict else (N, f"[-1, {N}]")
                    raise RuntimeError(f"The expanded size of the tensor ({target}) must match the existing size "
                                       f"({k}) at non-singleton dimension 1.  Target sizes: {shape}.  "
                                       f"Tensor sizes: [{t.shape[0]}, {k}]")
                wide.add(p)
        return wide

    def _columns(self, plan: Plan, evidence, n_queries: int, device) -> List[torch.Tensor]:
        cols = []
        for v in plan.slots:
            t = evidence[v]
            assert t.dim() == 2, ValueError("Each query tensor must be of dimension 2.")
            assert t.shape[0] == n_queries, ValueError("n_queries must be equal for all features.")
            if t.shape[1] != 1 and self.check_columns(plan, evidence):  # (raises the reference's errors)
                raise NotImplementedError(
                    "[n_queries, N_max] evidence columns run on a direct plan's raw launch (infer / infer_raw / "
                    "sharded_infer's raw path); the two-pass passes take [n_queries, 1] columns")
            if t.device != device or t.dtype != torch.float32 or not t.is_contiguous():
                t = t.to(device=device, dtype=torch.float32).contiguous()
            cols.append(t)
        return cols

    def call_plan(self, target: str, evidence: Dict[str, torch.Tensor], N_max: int):
        """(plan, fast path) of one call with the call's sample-domain draws made
        -- exactly once per call, in the reference's order: a kept plan whose
        domains are redrawn gets its new points here.  The fast path is None for
        plans rebuilt per call (the caller destroys those after use)."""
        key = (target, tuple(evidence.keys()), N_max)
        if GENERATION[0] != self._gen:
            self._check_generation()
        fp = self._fast.get(key)
        if fp is not None:
            if fp.redraw:
                self._redraw(fp)
            return fp.plan, fp
        device = _native.require_gpu(self.bn.device)
        observed = relevant_observed(self.bn, self._order(target), evidence.keys())
        plan = self.plan(target, observed, N_max, device)
        if plan.deterministic or plan.reusable:
            fp = self._fast[key] = _FastPath(plan, device, next(iter(evidence)) if len(evidence) else None)
            return plan, fp
        return plan, None

    def _redraw(self, fp: "_FastPath"):
        self._redraw_plan(fp.plan)
        fp.tdom.clear()

    def prepare(self, target: str, evidence: Dict[str, torch.Tensor], N_max: int):
        """Plan (this call's draws made) + device evidence columns of one call,
        without launching: (plan, cols, n_queries, target domain, device).  A
        plan rebuilt per call is the caller's to destroy."""
        plan, _ = self.call_plan(target, evidence, N_max)
        return (plan, *self.prepare_plan(plan, evidence))

    def prepare_plan(self, plan: Plan, evidence: Dict[str, torch.Tensor]):
        """Device evidence columns + target domain of one call on ``plan``
        (two-pass sharded path), without launching."""
        device = _native.require_gpu(self.bn.device)
        n_queries = next(iter(evidence.values())).shape[0] if len(evidence) > 0 else 1
        cols = self._columns(plan, evidence, n_queries, device)
        tq = n_queries if plan.target_observed else 1
        return cols, n_queries, plan.target_domain.unsqueeze(0).expand(tq, -1), device

    def infer(self, target: str, evidence: Dict[str, torch.Tensor], N_max: int,
              out: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
        # leanest path: the last fast path's native Runner (csrc/host_fast.cpp)
        # matches the dict's keys itself and launches; None -> the general path
        r = self._runner
        if r is not None and r[0] == target and r[1] == N_max and GENERATION[0] == self._gen:
            res = r[2](evidence, out)
            if type(res) is tuple:
                return res
            if res is not None:
                _native.check(res, "cbn_plan_run")
        # lean path: (target, evidence keys, N) -> cached plan (a kept redrawn
        # plan draws this call's points first)
        key = (target, tuple(evidence.keys()), N_max)  # evidence=None raises AttributeError, as the reference
        if GENERATION[0] != self._gen:
            self._check_generation()
        fp = self._fast.get(key)
        if fp is not None:
            if fp.redraw:
                self._redraw(fp)
            res = self._run_fast(fp, evidence, out)
            if res is not None:
                if not fp.redraw:
                    self._set_runner(fp, key)
                return res
            # conversions / the reference's errors, on the same (already drawn) plan
            n_queries = next(iter(evidence.values())).shape[0] if len(evidence) > 0 else 1
            return self._run(fp.plan, dict(evidence.items()), n_queries, fp.device, out)
        device = _native.require_gpu(self.bn.device)
        items = evidence.items()
        n_queries = next(iter(evidence.values())).shape[0] if len(evidence) > 0 else 1
        observed = relevant_observed(self.bn, self._order(target), evidence.keys())
        plan = self.plan(target, observed, N_max, device)
        try:
            res = self._run(plan, dict(items), n_queries, device, out)
            if plan.deterministic or plan.reusable:
                self._fast[key] = _FastPath(plan, device, next(iter(evidence)) if len(evidence) else None)
            return res
        finally:
            if not plan.deterministic and not plan.reusable:
                torch.cuda.current_stream(device).synchronize()
                plan.destroy()

    def infer_raw(self, target: str, evidence: Dict[str, torch.Tensor], N_max: int,
                  out: Optional[torch.Tensor] = None, words: Optional[torch.Tensor] = None,
                  fp: Optional["_FastPath"] = None):
        """One launch storing this batch's UNnormalised rows (the factor product
        of bayesian_network.py:269-295) and its max word -- the per-rank step of
        the sharded path, which all-reduces the word and then calls the returned
        ``scale(rows, max_bits)`` (the :296 division, in place).

        Returns (rows, target domain, max words int32[W], scale) or None when
        the plan cannot take a raw launch (the caller uses the two-pass
        exchange).  The W words are per-block maxima (all-reduce them with MAX).
        ``words``: a caller-owned int32[W] buffer for them (W =
        ``raw_word_count``); by default the plan's own buffer, which the next
        raw launch of the same plan overwrites.  ``fp``: the fast path
        ``call_plan`` returned for this call (its draws made); by default the
        cached deterministic one (``raw_fast_path``).
        """
        if fp is None:
            fp = self.raw_fast_path(target, evidence, N_max)
        if fp is None:
            return None
        if fp.words is None:
            return self._raw_wide(fp, evidence, out)
        plan = fp.plan
        if words is None:
            words = fp.words
        elif (words.dtype is not torch.int32 or words.device != fp.device or words.numel() != fp.words.numel()
              or not words.is_contiguous()):
            raise ValueError(f"words must be a contiguous int32[{fp.words.numel()}] tensor on {fp.device}")
        built = plan.tables_built
        res = fp.host(fp.run_fn, plan.handle.value, evidence, fp.slot_keys, fp.first, fp.device.index,
                      plan.n_samples, plan.target_observed, words.data_ptr(),
                      self._flags(plan) | _native.CBN_RUN_RAW, out)
        if res is None:  # evidence the native checks reject (dtype, device, layout): convert, launch here
            plan.tables_built = built  # (nothing launched yet)
            wres = self._raw_wide(fp, evidence, out)
            if wres is not None:
                return wres
            res = self._run_raw_converted(fp, evidence, words, out)
        if res is None or (type(res) is int and res == _native.CBN_E_UNSUPPORTED):
            return None
        if type(res) is int:
            _native.check(res, "cbn_plan_run(raw)")
        n = res.shape[0]
        tdom = fp.tdom.get(n)
        if tdom is None:
            tdom = fp.tdom[n] = plan.target_domain.unsqueeze(0).expand(n if plan.target_observed else 1, -1)

        def scale(rows: torch.Tensor, bits: torch.Tensor):
            rc = fp.host_scale(fp.scale_fn, rows, bits.data_ptr(), bits.numel())
            if rc:
                _native.check(rc, "cbn_scale")
            return rows

        return res, tdom, words, scale

    def _run_raw_converted(self, fp: "_FastPath", evidence, words: torch.Tensor, out):
        """Raw launch with the evidence converted to contiguous float32 columns
        on the plan's device (the reference's shape errors raise as in _run);
        None when the batch has no rows or the target is unobserved with > 1."""
        plan = fp.plan
        n = next(iter(evidence.values())).shape[0]
        if n == 0 or (not plan.target_observed and n != 1):
            return None
        cols = self._columns(plan, evidence, n, fp.device)
        if out is None:
            out = torch.empty((n, plan.n_samples), dtype=torch.float32, device=fp.device)
        ptrs = (ctypes.c_void_p * max(1, len(cols)))(*[c.data_ptr() for c in cols])
        with torch.cuda.device(fp.device):
            rc = _native.load().cbn_plan_run(plan.handle, n, ptrs, len(cols), words.data_ptr(), _native.ptr(out),
                                             self._flags(plan) | _native.CBN_RUN_RAW, _native.stream_ptr(fp.device))
        return rc if rc else out  # (converted copies: stream-ordered frees on the launch stream)

    def raw_fast_path(self, target: str, evidence: Dict[str, torch.Tensor], N_max: int) -> Optional["_FastPath"]:
        """The cached fast path of (target, evidence keys, N) when its plan is
        deterministic and takes raw launches (planned here if needed, nothing
        launched, nothing drawn); else None.  Plans whose sample domains are
        redrawn per call go through ``call_plan`` (one draw per call)."""
        key = (target, tuple(evidence.keys()), N_max)
        if GENERATION[0] != self._gen:
            self._check_generation()
        fp = self._fast.get(key)
        if fp is None:
            device = _native.require_gpu(self.bn.device)
            if len(evidence) == 0 or self.redraws(target, evidence.keys(), N_max):
                return None
            observed = relevant_observed(self.bn, self._order(target), evidence.keys())
            plan = self.plan(target, observed, N_max, device)
            fp = self._fast[key] = _FastPath(plan, device, next(iter(evidence)))
        return fp if (fp.words is not None and not fp.redraw) else None

    def raw_flags(self, plan: Plan) -> int:
        return self._flags(plan) | _native.CBN_RUN_RAW

    def raw_word_count(self, target: str, evidence_keys, N_max: int) -> int:
        """W, the number of per-block max words of this (target, evidence keys,
        N) raw launch; 0 when it has none (or no raw launch ran yet)."""
        fp = self._fast.get((target, tuple(evidence_keys), N_max))
        return 0 if fp is None or fp.words is None else int(fp.words.numel())

    def _flags(self, plan: Plan) -> int:
        f = 0
        if not (self.cache_tables and plan.tables_built):
            f |= _native.CBN_RUN_BUILD_TABLES
            plan.tables_built = self.cache_tables
        if self.timed:
            f |= _native.CBN_RUN_TIMED
        if not self.fused:
            f |= _native.CBN_RUN_TWO_PASS
        return f

    def check_status(self):
        """Raise if any fused launch's grid barrier timed out (output invalid)."""
        lib = _native.load()
        st = ctypes.c_int32()
        for p in self._plans.values():
            _native.check(lib.cbn_plan_status(p.handle, ctypes.byref(st)), "status")
            if st.value:
                raise _native.NativeError("a single-launch inference timed out in its grid barrier "
                                          "(not every block was resident); rerun with engine.fused = False")

    def fused_capacity(self, target: str, evidence_keys, N_max: int) -> int:
        fp = self._fast.get((target, tuple(evidence_keys), N_max))
        return int(_native.load().cbn_plan_fused_capacity(fp.plan.handle)) if fp else 0

    def _set_runner(self, fp: "_FastPath", key):
        """Make fp the Runner path of the next calls (deterministic plans whose
        tables are built and whose per-call flags are 0: fused, untimed)."""
        plan = fp.plan
        if self._flags_peek(plan) != 0 or len(key[1]) == 0:
            return
        if fp.runner is None:
            fp.runner = _native.load_host().Runner(fp.run_fn, plan.handle.value, key[1], fp.slot_keys,
                                                   fp.device.index, plan.n_samples, plan.target_observed,
                                                   fp.max_ptr, 0, plan.target_domain)
        self._runner = (key[0], key[2], fp.runner)

    def _flags_peek(self, plan: Plan) -> int:
        """_flags without its side effect (the table-build bookkeeping)."""
        f = 0 if (self.cache_tables and plan.tables_built) else _native.CBN_RUN_BUILD_TABLES
        if self.timed:
            f |= _native.CBN_RUN_TIMED
        if not self.fused:
            f |= _native.CBN_RUN_TWO_PASS
        return f

    def _run_fast(self, fp: "_FastPath", evidence, out):
        """Hot path: no plan lookup, no context managers, no re-validation
        beyond dtype/device/shape of the evidence columns."""
        plan = fp.plan
        built = plan.tables_built
        res = fp.host(fp.run_fn, plan.handle.value, evidence, fp.slot_keys, fp.first, fp.device.index,
                      plan.n_samples, plan.target_observed, fp.max_ptr, self._flags(plan), out)
        if res is None:  # nothing launched: the tables are still to be built by the launch that runs
            plan.tables_built = built
        else:
            if type(res) is int:
                _native.check(res, "cbn_plan_run")
            n = res.shape[0]
            tdom = fp.tdom.get(n)
            if tdom is None:
                tdom = fp.tdom[n] = plan.target_domain.unsqueeze(0).expand(n if plan.target_observed else 1, -1)
            return res, tdom
        n = evidence[fp.first].shape[0] if fp.first is not None else 1
        ptrs = fp.ptrs
        for i, v in enumerate(plan.slots):
            t = evidence[v]
            if (t.dtype is not torch.float32 or t.device != fp.device or t.dim() != 2 or t.shape[0] != n
                    or t.shape[1] != 1 or not t.is_contiguous()):
                return None  # slow path converts / raises the reference's errors
            ptrs[i] = t.data_ptr()
        if n == 0 or (not plan.target_observed and n != 1):
            return None
        if out is None:
            out = torch.empty((n, plan.n_samples), dtype=torch.float32, device=fp.device)
        tdom = fp.tdom.get(n)
        if tdom is None:
            tdom = fp.tdom[n] = plan.target_domain.unsqueeze(0).expand(n if plan.target_observed else 1, -1)
        if torch.cuda.current_device() != fp.device.index:
            torch.cuda.set_device(fp.device)
        rc = fp.lib.cbn_plan_run(plan.handle, n, ptrs, len(plan.slots), fp.max_ptr, out.data_ptr(),
                                 self._flags(plan), torch.cuda.current_stream(fp.device).cuda_stream)
        if rc:
            _native.check(rc, "cbn_plan_run")
        return out, tdom

    def timing(self):
        """(calls, avg max-pass ms, avg write-pass ms) over the timed calls of every cached plan."""
        lib = _native.load()
        n, a, b = ctypes.c_int32(), ctypes.c_float(), ctypes.c_float()
        tot = [0, 0.0, 0.0]
        for p in self._plans.values():
            _native.check(lib.cbn_plan_timing(p.handle, ctypes.byref(n), ctypes.byref(a), ctypes.byref(b)), "timing")
            tot[0] += n.value
            tot[1] += a.value * n.value
            tot[2] += b.value * n.value
        return tot[0], (tot[1] / tot[0] if tot[0] else 0.0), (tot[2] / tot[0] if tot[0] else 0.0)

    def _wide(self, plan: Plan, evidence) -> set:
        """The columns of this call read as [Q, N] per-query sample values
        (check_columns; the reference's shape errors raise here)."""
        for v in plan.slots:
            t = evidence[v]
            if t.dim() == 2 and t.shape[1] != 1:
                return self.check_columns(plan, evidence)
        return set()

    def _wide_plan(self, plan: Plan, wide, device) -> Plan:
        """The direct plan of ``plan`` whose observed parents in ``wide`` take
        [Q, N] columns (node.py:246-248: each query's N values of that parent
        enter the meshgrid like a free parent's samples, node.py:335-375, and
        the factor is their mean).  It shares ``plan``'s sample-index arrays
        (a redrawn plan's draws of this call included; its constant rows are
        then rebuilt per call).  BruteForce networks only."""
        if plan.direct is False and any(hasattr(self.bn.nodes_obj[s.node].estimator, "model_desc")
                                        for s in plan.factors):
            raise NotImplementedError(
                "[n_queries, N_max] evidence columns (per-query sample values, node.py:246-248) are evaluated on "
                "BruteForce networks; the parametric kernels take [n_queries, 1] columns")
        key = (plan.target, plan.observed, plan.n_samples, frozenset(wide))
        wp = self._wide_plans.get(key)
        if wp is not None and wp[0] is plan:
            return wp[1]
        import dataclasses

        wp = dataclasses.replace(plan, handle=None, keep=[], max_bits=None, tables_built=False, direct=False,
                                 redraw=None, idx_host=None)
        self._materialise_direct(wp, device, widths={c: plan.n_samples for c in wide}, share_idx=plan)
        wp.words = torch.zeros(int(_native.load().cbn_plan_max_words(wp.handle)), dtype=torch.int32, device=device)
        old = self._wide_plans.pop(key, None)
        if old is not None:
            torch.cuda.synchronize()
            old[1].destroy()
        self._wide_plans[key] = (plan, wp)
        return wp

    def _run_wide(self, plan: Plan, evidence, wide, n_queries: int, device, out, raw: bool = False):
        """One call with [Q, N] columns on the wide direct plan: raw launch,
        then the global-max division -- or, ``raw``, (rows, target domain, the
        launch's max words) for the caller's exchange and scale."""
        wp = self._wide_plan(plan, wide, device)
        N = plan.n_samples
        cols = []
        for v in plan.slots:
            t = evidence[v]
            if t.device != device or t.dtype != torch.float32 or not t.is_contiguous():
                t = t.to(device=device, dtype=torch.float32).contiguous()
            cols.append(t)
        tq = n_queries if plan.target_observed else 1
        tdom = plan.target_domain.unsqueeze(0).expand(tq, -1)
        if (n_queries, N) != tuple(tdom.shape):
            raise AssertionError("pdf and domain must have same shape.")
        if n_queries == 0:
            raise RuntimeError("max(): Expected reduction dim to be specified for input.numel() == 0.")
        if out is None:
            out = torch.empty((n_queries, N), dtype=torch.float32, device=device)
        flags = _native.CBN_RUN_RAW
        if not wp.tables_built or not plan.deterministic:  # (a redrawn plan's constant rows: this call's draws)
            flags |= _native.CBN_RUN_BUILD_TABLES
            wp.tables_built = True
        ptrs = (ctypes.c_void_p * max(1, len(cols)))(*[c.data_ptr() for c in cols])
        lib = _native.load()
        with torch.cuda.device(device):
            s = _native.stream_ptr(device)
            _native.check(lib.cbn_plan_run(wp.handle, n_queries, ptrs, len(cols), _native.ptr(wp.words),
                                           _native.ptr(out), flags, s), "cbn_plan_run(wide)")
            if raw:
                return out, tdom, wp.words
            _native.check(lib.cbn_scale(_native.ptr(out), n_queries * N, _native.ptr(wp.words), wp.words.numel(), s),
                          "cbn_scale")
        return out, tdom

    def wide_word_count(self, plan: Plan, wide, device) -> int:
        """W of the wide direct plan (an empty shard's zero words must match
        the other ranks' raw launch)."""
        return int(self._wide_plan(plan, wide, device).words.numel())

    def _raw_wide(self, fp: "_FastPath", evidence, out):
        """infer_raw of a call with [Q, N] columns: the wide direct plan's raw
        launch and ITS max words (the same W on every rank, empty shards
        included: ``wide_word_count``); None for any other call."""
        n = next(iter(evidence.values())).shape[0] if len(evidence) else 0
        wide = self._wide(fp.plan, evidence) if n > 0 else None
        if not wide:
            return None
        rows, tdom, words = self._run_wide(fp.plan, evidence, wide, n, fp.device, out, raw=True)
        return rows, tdom, words, self._wide_scale(fp)

    @staticmethod
    def _wide_scale(fp: "_FastPath"):
        def scale(rows: torch.Tensor, bits: torch.Tensor):
            rc = fp.host_scale(fp.scale_fn, rows, bits.data_ptr(), bits.numel())
            if rc:
                _native.check(rc, "cbn_scale")
            return rows
        return scale

    def _run(self, plan: Plan, evidence, n_queries: int, device, out):
        wide = self._wide(plan, evidence)
        if wide:
            return self._run_wide(plan, evidence, wide, n_queries, device, out)
        lib = _native.load()
        N = plan.n_samples
        cols = self._columns(plan, evidence, n_queries, device)
        tq = n_queries if plan.target_observed else 1
        tdom = plan.target_domain.unsqueeze(0).expand(tq, -1)
        if (n_queries, N) != tuple(tdom.shape):
            raise AssertionError("pdf and domain must have same shape.")
        if n_queries == 0:
            raise RuntimeError("max(): Expected reduction dim to be specified for input.numel() == 0.")
        if out is None:
            out = torch.empty((n_queries, N), dtype=torch.float32, device=device)
        ptrs = (ctypes.c_void_p * max(1, len(cols)))(*[c.data_ptr() for c in cols])
        with torch.cuda.device(device):
            _native.check(lib.cbn_plan_run(plan.handle, n_queries, ptrs, len(cols), _native.ptr(plan.max_bits),
                                           _native.ptr(out), self._flags(plan), _native.stream_ptr(device)),
                          "cbn_plan_run")
        return out, tdom

    def _build(self, plan: Plan, stream):
        if self.cache_tables and plan.tables_built:
            return
        _native.check(_native.load().cbn_plan_build_tables(plan.handle, stream), "build_tables")
        plan.tables_built = True

    # ---------------------------------------------- split passes (sharded) --
    def query_max(self, plan: Plan, cols: List[torch.Tensor], n_queries: int, device) -> torch.Tensor:
        lib = _native.load()
        ptrs = (ctypes.c_void_p * max(1, len(cols)))(*[c.data_ptr() for c in cols])
        with torch.cuda.device(device):
            s = _native.stream_ptr(device)
            self._build(plan, s)
            _native.check(lib.cbn_plan_query_max(plan.handle, n_queries, ptrs, len(cols),
                                                 _native.ptr(plan.max_bits), s), "query_max")
        return plan.max_bits

    def query_write(self, plan: Plan, cols: List[torch.Tensor], n_queries: int, max_bits: torch.Tensor,
                    out: torch.Tensor, device):
        lib = _native.load()
        ptrs = (ctypes.c_void_p * max(1, len(cols)))(*[c.data_ptr() for c in cols])
        with torch.cuda.device(device):
            _native.check(lib.cbn_plan_query_write(plan.handle, n_queries, ptrs, len(cols), _native.ptr(max_bits),
                                                   _native.ptr(out), _native.stream_ptr(device)), "query_write")
        return out
