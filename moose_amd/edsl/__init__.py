from moose_amd.edsl.base import *  # noqa: F401,F403
from moose_amd.edsl.tracer import trace  # noqa: F401
from moose_amd.edsl.tracer import trace_and_compile  # noqa: F401
