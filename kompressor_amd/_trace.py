"""roctx ranges around the codec stages (SURVEY.md §5 tracing): ``KMP_TRACE=1`` brackets every
encode / decode / chunked call and every user callback with a named range, which
``rocprofv3 --marker-trace --kernel-trace`` lines up with the kernels each stage launched.
Off by default: then the wrappers cost one dict lookup."""

import contextlib
import functools
import os

import torch

ENABLED = os.environ.get('KMP_TRACE', '0') not in ('', '0')


@contextlib.contextmanager
def stage(name):
    if not ENABLED:
        yield
        return
    torch.cuda.nvtx.range_push(name)
    try:
        yield
    finally:
        torch.cuda.nvtx.range_pop()


def traced(name):
    """Decorator form of :func:`stage`."""
    def wrap(fn):
        @functools.wraps(fn)
        def inner(*args, **kwargs):
            if not ENABLED:
                return fn(*args, **kwargs)
            with stage(name):
                return fn(*args, **kwargs)
        return inner
    return wrap
