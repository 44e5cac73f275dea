"""Compatibility import path of the native backend (now the package ``engine/native``)."""
from .native import CELL_ID, FORGET_BIAS, ExecutionPlan, Knobs, NativeBackend  # noqa: F401
