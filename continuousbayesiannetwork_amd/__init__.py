"""MI355X-native batched inference for ContinuousBayesianNetwork.

Drop-in for the reference's ``cbn`` inference path: ``BayesianNetwork``,
``Node``, the ``BruteForce`` / ``LinearRegression`` / ``LogisticRegression`` /
``NeuralNetwork`` estimators and the ``exact`` inference plugin keep the
reference's names and call signatures; the batched factor product runs in the
HIP kernels of ``csrc/cbn_infer.hip`` (tables) and ``csrc/cbn_param.hip``
(parametric CPDs) behind the C ABI of ``include/cbn_amd.h``.
"""
from .base.bayesian_network import BayesianNetwork
from .base.node import Node
from .inference import INFERENCE_OBJS, ExactInference, VariableElimination
from .parameter_learning import ESTIMATORS, BruteForce, LinearRegression, LogisticRegression, NeuralNetwork

__all__ = ["BayesianNetwork", "Node", "BruteForce", "LinearRegression", "LogisticRegression", "NeuralNetwork",
           "ESTIMATORS", "INFERENCE_OBJS", "ExactInference", "VariableElimination"]
__version__ = "0.1.0"
