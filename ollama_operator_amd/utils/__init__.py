"""Small shared utilities: roctx tracing (`trace`)."""
from .trace import enabled as roctx_enabled, mark, trace_range

__all__ = ["roctx_enabled", "mark", "trace_range"]
