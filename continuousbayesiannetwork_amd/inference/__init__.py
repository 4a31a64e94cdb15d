"""Inference plugin registry, mirroring cbn/inference/__init__.py:1-3."""
from .exact import ExactInference, VariableElimination

# "exact" mirrors the reference's registry; "variable_elimination" is the same
# plugin with the query() entry point
INFERENCE_OBJS = {"exact": ExactInference, "variable_elimination": VariableElimination}
