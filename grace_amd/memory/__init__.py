"""Error-feedback memories (GRACE layer L3)."""
from .none import NoneMemory  # noqa: F401
from .residual import ResidualMemory  # noqa: F401
from .efsignsgd import EFSignSGDMemory  # noqa: F401
from .dgc import DgcMemory  # noqa: F401
from .powersgd import PowerSGDMemory  # noqa: F401
