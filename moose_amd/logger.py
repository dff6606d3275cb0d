"""``get_logger`` (reference ``pymoose/pymoose/logger.py``); level from ``MOOSEX_LOG``."""
from moose_amd.utils.telemetry import get_logger  # noqa: F401
