"""Estimator registry, mirroring cbn/parameter_learning/__init__.py:7-13.

Only the discrete BruteForce estimator is on the accelerated inference path
this round; the regression / neural / GP estimators of the reference are listed
in DESIGN.md as the next rows.
"""
from .brute_force import BruteForce

ESTIMATORS = {
    "brute_force": BruteForce,
}
