"""Exact inference plugin (cbn/inference/exact.py:6-17; a stub in the reference).

The reference registers ``ExactInference`` under ``INFERENCE_OBJS["exact"]``
(cbn/inference/__init__.py) but its ``_infer`` is empty: the computation lives
in ``BayesianNetwork.infer`` (cbn/base/bayesian_network.py:208-305).  Here the
plugin runs that computation on the network it is attached to, and
``VariableElimination`` -- the name the task's north star uses -- adds the
``query`` entry point.  There is no reference behaviour for ``query`` beyond
``infer``'s, so it is exactly ``infer``.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import torch

from ..base.inference import BaseInference


class ExactInference(BaseInference):
    def __init__(self, config: Dict, **kwargs):
        super().__init__(config=config, **kwargs)
        self.bn = kwargs.get("bn")
        self._setup_model(config, **kwargs)

    def _setup_model(self, config: Dict, **kwargs):
        self.config = dict(config or {})

    def _infer(self, target_node: str, evidence: Dict, do: Dict, **kwargs):
        if self.bn is None:
            raise ValueError("ExactInference needs the BayesianNetwork (bn=...) it runs on")
        return self.bn.infer(target_node, evidence, do, N_max=kwargs.get("N_max", 16))


class VariableElimination(ExactInference):
    """``ExactInference`` with the ``query`` entry point: the normalised
    marginal of ``target_node`` per evidence row and its evaluation points,
    as ``BayesianNetwork.infer`` returns them (bayesian_network.py:208-305)."""

    def query(self, target_node: str, evidence: Optional[Dict[str, torch.Tensor]] = None, N_max: int = 16,
              do: Optional[List[str]] = None):
        return self.infer(target_node, evidence, do, N_max=N_max)
