"""tensorpack-style ``arg_scope`` default injection (lib/utils/arg_scope.py:10-88).

``@add_arg_scope`` on a layer class makes its constructor pick up defaults
from the innermost ``with arg_scope([Cls, ...], **defaults)`` block; explicit
constructor keywords win.
"""
import copy
from collections import defaultdict
from contextlib import contextmanager
from functools import wraps

_ArgScopeStack = []


def get_arg_scope():
    if _ArgScopeStack:
        return _ArgScopeStack[-1]
    return defaultdict(dict)


@contextmanager
def arg_scope(layers, **kwargs):
    if not isinstance(layers, (list, tuple)):
        layers = [layers]
    for layer in layers:
        if not getattr(layer, "__arg_scope_enabled__", False):
            raise AssertionError(f"Argscope not supported for {layer}")
    new_scope = copy.copy(get_arg_scope())
    new_scope = defaultdict(dict, {k: dict(v) for k, v in new_scope.items()})
    for layer in layers:
        new_scope[layer.__name__].update(kwargs)
    _ArgScopeStack.append(new_scope)
    try:
        yield
    finally:
        del _ArgScopeStack[-1]


def add_arg_scope(cls):
    original_init = cls.__init__

    @wraps(original_init)
    def wrapped_init(self, *args, **kwargs):
        actual = dict(get_arg_scope()[cls.__name__])
        actual.update(kwargs)
        return original_init(self, *args, **actual)

    cls.__arg_scope_enabled__ = True
    cls.__init__ = wrapped_init
    return cls
