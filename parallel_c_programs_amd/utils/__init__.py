"""BMP I/O, timers (reference print format), device info, JSON metrics."""
from . import bmp, device, timing  # noqa: F401
from .metrics import emit_metric  # noqa: F401
