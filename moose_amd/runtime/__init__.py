"""Runtimes (reference ``pymoose/pymoose/runtime.py``): ``LocalMooseRuntime`` simulates
every identity in one process; ``GrpcMooseRuntime`` / ``DistributedMooseRuntime`` run one
worker process per identity."""


def __getattr__(name):
    if name == "LocalMooseRuntime":
        from moose_amd.runtime.local import LocalMooseRuntime

        return LocalMooseRuntime
    if name in ("GrpcMooseRuntime", "DistributedMooseRuntime"):
        from moose_amd.runtime import distributed

        return getattr(distributed, name)
    raise AttributeError(name)
