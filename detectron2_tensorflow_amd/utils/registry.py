"""Name -> object registries keyed by config strings (lib/utils/registry.py:1-56)."""


class Registry:
    """Maps ``obj.__name__`` to the registered class/function.

    Usage mirrors the reference: ``@REG.register()`` as a decorator or
    ``REG.register(obj)``; ``REG.get(name)`` raises KeyError for unknown names.
    """

    def __init__(self, name):
        self._name = name
        self._obj_map = {}

    def _do_register(self, name, obj):
        if name in self._obj_map:
            raise KeyError(f"An object named '{name}' was already registered in "
                           f"'{self._name}' registry!")
        self._obj_map[name] = obj

    def register(self, obj=None):
        if obj is None:
            def deco(func_or_class):
                self._do_register(func_or_class.__name__, func_or_class)
                return func_or_class
            return deco
        self._do_register(obj.__name__, obj)
        return obj

    def get(self, name):
        ret = self._obj_map.get(name)
        if ret is None:
            raise KeyError(f"No object named '{name}' found in '{self._name}' registry!")
        return ret

    def __contains__(self, name):
        return name in self._obj_map

    def keys(self):
        return list(self._obj_map)
