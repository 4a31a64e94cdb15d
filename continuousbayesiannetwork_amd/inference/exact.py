"""Exact inference plugin (cbn/inference/exact.py:6-17; a stub in the reference)."""
from __future__ import annotations

from typing import Dict

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


VariableElimination = ExactInference
