"""Loader for sparkmi's in-tree native extensions.

``sparkmi._C`` holds the HIP/CDNA4 kernels (built for gfx950 by ``tools/build_native.py``);
``sparkmi._runtime`` holds the host C++ runtime (libsvm parser, tokenizer, vocab encoder);
``sparkmi._comm`` the native communication layer (RCCL communicator, xGMI IPC all-reduce),
``sparkmi._io`` the native input pipeline (pinned host ring, threaded gather, async H2D).

torch is imported first on purpose: torch ships its own ``libamdhip64.so.7`` and ``_C``
declares the same SONAME, so the dynamic linker binds ``_C`` to torch's already-loaded HIP
runtime — one runtime, one set of streams, so our launches on
``torch.cuda.current_stream()`` are ordered with torch's own work and captured by
``torch.cuda.graph``.

Policy: on a GPU tensor the HIP kernel is *the* implementation.  If ``_C`` is missing on a
GPU box every op raises (``require()``) instead of silently running an eager fallback, unless
``SPARKMI_ALLOW_REFERENCE=1`` is set explicitly (debugging only).
"""
import importlib
import os
import threading

import torch  # noqa: F401  (must precede _C; see module docstring)

_lock = threading.Lock()
_C = None
_RT = None
_C_err = None
_RT_err = None


def _try_build():
    if os.environ.get("SPARKMI_NO_AUTOBUILD"):
        return
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = os.path.join(root, "tools", "build_native.py")
    if os.path.exists(script) and os.path.isdir(os.path.join(root, "csrc")):
        import subprocess
        import sys
        subprocess.run([sys.executable, script], check=False, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)


def _load(name):
    return importlib.import_module("sparkmi." + name)


def C():
    """The HIP kernel module; raises ImportError with the build error if unavailable."""
    global _C, _C_err
    if _C is not None:
        return _C
    with _lock:
        if _C is None and _C_err is None:
            try:
                _C = _load("_C")
            except ImportError:
                _try_build()
                try:
                    _C = _load("_C")
                except ImportError as e:  # pragma: no cover
                    _C_err = e
    if _C is None:
        raise ImportError(f"sparkmi._C (HIP kernels) unavailable: {_C_err}; run python tools/build_native.py")
    return _C


def RT():
    """The host C++ runtime module."""
    global _RT, _RT_err
    if _RT is not None:
        return _RT
    with _lock:
        if _RT is None and _RT_err is None:
            try:
                _RT = _load("_runtime")
            except ImportError:
                _try_build()
                try:
                    _RT = _load("_runtime")
                except ImportError as e:  # pragma: no cover
                    _RT_err = e
    if _RT is None:
        raise ImportError(f"sparkmi._runtime unavailable: {_RT_err}; run python tools/build_native.py")
    return _RT


_COMM = None
_COMM_err = None


def comm():
    """The native communication module (RCCL communicator + IPC one-shot all-reduce)."""
    global _COMM, _COMM_err
    if _COMM is not None:
        return _COMM
    with _lock:
        if _COMM is None and _COMM_err is None:
            try:
                _COMM = _load("_comm")
            except ImportError:
                _try_build()
                try:
                    _COMM = _load("_comm")
                except ImportError as e:  # pragma: no cover
                    _COMM_err = e
    if _COMM is None:
        raise ImportError(f"sparkmi._comm unavailable: {_COMM_err}; run python tools/build_native.py")
    return _COMM


_IO = None
_IO_err = None


def io():
    """The native input-pipeline module (pinned host ring, threaded gather, async H2D)."""
    global _IO, _IO_err
    if _IO is not None:
        return _IO
    with _lock:
        if _IO is None and _IO_err is None:
            try:
                _IO = _load("_io")
            except ImportError:
                _try_build()
                try:
                    _IO = _load("_io")
                except ImportError as e:  # pragma: no cover
                    _IO_err = e
    if _IO is None:
        raise ImportError(f"sparkmi._io unavailable: {_IO_err}; run python tools/build_native.py")
    return _IO


def has_native():
    try:
        C()
        return True
    except ImportError:
        return False


def has_runtime():
    try:
        RT()
        return True
    except ImportError:
        return False


ALLOW_REFERENCE = os.environ.get("SPARKMI_ALLOW_REFERENCE", "0") == "1"


def use_native(t: torch.Tensor) -> bool:
    """True when ``t`` lives on the GPU: the HIP kernel must run (raises if _C is missing)."""
    if not t.is_cuda:
        return False
    if ALLOW_REFERENCE and not has_native():
        return False
    C()  # raises loudly when missing
    return True


def stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def ptr(t):
    return 0 if t is None else t.data_ptr()
