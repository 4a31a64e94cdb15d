"""Estimator plugin interface, mirroring cbn/base/parameter_learning.py:8-61."""
from abc import ABC, abstractmethod
from typing import Dict

import torch


# Bumped whenever any estimator's fitted state changes (fit, load_model, a
# parameter edit followed by _invalidate): inference plans capture raw device
# pointers to CPDs / packed weights.  One integer compare per call tells an
# engine that SOME estimator changed; it then compares the stamps of its own
# network's estimators and drops its cached plans only if one of them moved.
GENERATION = [0]


def bump_generation(estimator=None):
    GENERATION[0] += 1
    if estimator is not None:
        estimator._stamp = GENERATION[0]


class BaseParameterLearningEstimator(ABC):
    def __init__(self, config: Dict, **kwargs):
        self.estimator_name = config.get("estimator_name")
        self.device = kwargs.get("device", "cuda" if torch.cuda.is_available() else "cpu")
        self.if_log = kwargs.get("log", False)

    @abstractmethod
    def _setup_model(self, config: Dict, **kwargs):
        raise NotImplementedError

    def fit(self, node_data: torch.Tensor, parents_data: torch.Tensor = None):
        """node_data [n_samples]; parents_data [n_parents_features, n_samples]."""
        self._fit(node_data, parents_data)
        bump_generation(self)

    @abstractmethod
    def _fit(self, node_data: torch.Tensor, parents_data: torch.Tensor = None):
        raise NotImplementedError

    def get_prob(self, point_to_evaluate: torch.Tensor, query: torch.Tensor = None) -> torch.Tensor:
        """point_to_evaluate [n_queries, n_values]; query [n_queries, n_features, 1]."""
        return self._get_prob(point_to_evaluate, query)

    @abstractmethod
    def _get_prob(self, point_to_evaluate: torch.Tensor, query: torch.Tensor = None):
        raise NotImplementedError

    def sample(self, N: int, **kwargs) -> torch.Tensor:
        return self._sample(N, **kwargs)

    @abstractmethod
    def _sample(self, N: int, **kwargs) -> torch.Tensor:
        raise NotImplementedError

    def save_model(self, path: str):
        raise NotImplementedError

    def load_model(self, path: str):
        raise NotImplementedError
