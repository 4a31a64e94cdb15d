"""Registry helpers, mirroring cbn/utils.py:16-33."""
from typing import Dict

import torch

from .base.parameter_learning import BaseParameterLearningEstimator


def get_distribution_parameters(dist: torch.distributions.Distribution):
    """cbn/utils.py:4-14."""
    return {key: getattr(dist, key) for key in vars(dist) if not key.startswith("_")}


def choose_probability_estimator(estimator_name: str, config: Dict, **kwargs) -> BaseParameterLearningEstimator:
    from .parameter_learning import ESTIMATORS

    if estimator_name in ESTIMATORS.keys():
        return ESTIMATORS[estimator_name](config, **kwargs)
    raise ValueError(f"Unknown estimator: {estimator_name}")


def choose_inference_obj(inference_name: str, config: Dict, **kwargs):
    """cbn/utils.py:29-33 (a stub returning None in the reference) -> the
    registered inference plugin instance."""
    from .inference import INFERENCE_OBJS

    if inference_name in INFERENCE_OBJS.keys():
        return INFERENCE_OBJS[inference_name](config, **kwargs)
    raise ValueError(f"Unknown inference object: {inference_name}")
