"""The native (gfx950 HIP) execution engine: see backend.py."""
from .backend import CELL_ID, NativeBackend  # noqa: F401
from .forward import FORGET_BIAS  # noqa: F401
from .plan import DEBUG_KEYS, ExecutionPlan, Knobs, make_plan  # noqa: F401
