"""Range tracing for step phases: ROCTx ranges (visible in rocprofv3 traces with
``--marker-trace``) when libroctx64 is loadable, plus torch.profiler ``record_function`` so the
same ranges appear in torch profiles.  Disabled (zero cost) unless ``SPARKMI_TRACE=1`` or
``enable()`` was called.

    with trace.range("fwd"): ...
"""
import contextlib
import ctypes
import os

_enabled = os.environ.get("SPARKMI_TRACE", "0") == "1"
_roctx = None
_tried = False


def _lib():
    global _roctx, _tried
    if _tried:
        return _roctx
    _tried = True
    for name in ("libroctx64.so", "/opt/rocm/lib/libroctx64.so", "librocprofiler-sdk-roctx.so",
                 "/opt/rocm/lib/librocprofiler-sdk-roctx.so"):
        try:
            lib = ctypes.CDLL(name)
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            lib.roctxRangePushA.restype = ctypes.c_int
            lib.roctxRangePop.restype = ctypes.c_int
            lib.roctxMarkA.argtypes = [ctypes.c_char_p]
            _roctx = lib
            break
        except (OSError, AttributeError):
            continue
    return _roctx


def enable(on=True):
    global _enabled
    _enabled = bool(on)


def enabled():
    return _enabled


def available():
    return _lib() is not None


@contextlib.contextmanager
def range(name):  # noqa: A001 - mirrors roctx naming
    if not _enabled:
        yield
        return
    lib = _lib()
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    try:
        import torch
        with torch.profiler.record_function(name):
            yield
    finally:
        if lib is not None:
            lib.roctxRangePop()


def mark(name):
    if _enabled and _lib() is not None:
        _lib().roctxMarkA(name.encode())
