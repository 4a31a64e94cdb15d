"""Estimator registry, mirroring cbn/parameter_learning/__init__.py:7-13.

BruteForce (discrete tables) and the parametric LinearRegression /
LogisticRegression / NeuralNetwork estimators are on the accelerated inference
path.  ``gp_gpytorch`` needs the third-party gpytorch (~=1.14,
requirements.txt), which is not installed in this image: it is registered as a
stub that raises on construction (out of scope).
"""
from .brute_force import BruteForce
from .parametric import LinearRegression, LogisticRegression, NeuralNetwork


class GP_gpytorch:  # noqa: N801  (reference class name, gp_gpytorch.py:39)
    def __init__(self, config, **kwargs):
        raise ImportError("gp_gpytorch needs gpytorch (~=1.14), which is not installed; "
                          "the Gaussian-process estimator is not on the MI355X inference path")


ESTIMATORS = {
    "brute_force": BruteForce,
    "gp_gpytorch": GP_gpytorch,
    "linear_regression": LinearRegression,
    "logistic_regression": LogisticRegression,
    "neural_network": NeuralNetwork,
}
