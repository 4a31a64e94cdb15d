"""Constants of the reference's cbn/base/__init__.py (same names, same values)."""
KEY_CONTINUOUS = "continuous"
KEY_DISCRETE = "discrete"

KEY_MAX_CARDINALITY_FOR_DISCRETE = "max_cardinality_for_discrete_domain"
BASE_MAX_CARDINALITY = 20
