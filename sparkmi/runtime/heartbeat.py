"""Progress counter of this executor, read by the worker's heartbeat thread
(sparkmi/runtime/worker.py) and advanced by the training loop once per step."""
_progress = [0]


def progress(step=None):
    """Advance (or set) this executor's progress counter."""
    _progress[0] = _progress[0] + 1 if step is None else int(step)


def current():
    return _progress[0]
