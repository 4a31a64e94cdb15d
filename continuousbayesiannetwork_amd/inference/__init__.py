"""Inference plugin registry, mirroring cbn/inference/__init__.py:1-3."""
from .exact import ExactInference, VariableElimination

INFERENCE_OBJS = {"exact": ExactInference}
