"""Executor-group runtime: launcher (one process per MI355X), worker bootstrap, log streaming,
heartbeat / failure detection, restarts, fault injection."""
from .fault import fault_point  # noqa: F401
from .heartbeat import progress  # noqa: F401
from .launcher import LaunchError, launch  # noqa: F401
