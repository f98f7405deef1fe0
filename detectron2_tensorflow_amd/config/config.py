"""A small yacs-compatible CfgNode (yacs is not installed here).

Behaviour of the reference's config object (lib/config/config.py:12-140, on
top of yacs.config.CfgNode):
  * attribute access, ``freeze()`` / ``defrost()``, ``clone()``;
  * ``merge_from_file`` with ``_BASE_`` inheritance (path relative to the
    including file), ``merge_from_list`` ([key, value, ...]),
    ``merge_from_other_cfg``; merging a key absent from the defaults raises
    KeyError (yacs semantics) and values are type-checked against the
    defaults (list/tuple interchangeable, int -> float allowed);
  * string values are decoded with ``ast.literal_eval`` when possible
    (e.g. ``STEPS: (210000, 250000)``);
  * ``!!python/object/apply:eval ["<expr>"]`` (used by
    configs/Base-RetinaNet.yaml:7) is accepted when ``allow_unsafe`` is set,
    but evaluated by a RESTRICTED evaluator (numbers, + - * / ** // %, list /
    tuple literals and list comprehensions over them) — never by ``eval``.
"""
import ast
import copy
import operator
import os

import yaml

BASE_KEY = "_BASE_"


class CfgNode(dict):
    IMMUTABLE = "__immutable__"

    def __init__(self, init_dict=None):
        super().__init__()
        object.__setattr__(self, CfgNode.IMMUTABLE, False)
        for k, v in (init_dict or {}).items():
            self[k] = CfgNode(v) if isinstance(v, dict) and not isinstance(v, CfgNode) else v

    # attribute access ---------------------------------------------------
    def __getattr__(self, name):
        try:
            return self[name]
        except KeyError:
            raise AttributeError(name)

    def __setattr__(self, name, value):
        if self.is_frozen():
            raise AttributeError(f"Attempted to set {name} to {value}, but CfgNode is immutable")
        if name.startswith("COMPUTED_") and name in self and self[name] != value:
            raise KeyError(f"Computed attributed '{name}' already exists with a different value! "
                           f"old={self[name]}, new={value}.")
        self[name] = value

    def __deepcopy__(self, memo):
        out = CfgNode()
        for k, v in self.items():
            dict.__setitem__(out, k, copy.deepcopy(v, memo))
        return out

    # mutability ---------------------------------------------------------
    def freeze(self):
        self._set_immutable(True)

    def defrost(self):
        self._set_immutable(False)

    def is_frozen(self):
        return object.__getattribute__(self, CfgNode.IMMUTABLE)

    def _set_immutable(self, flag):
        object.__setattr__(self, CfgNode.IMMUTABLE, flag)
        for v in self.values():
            if isinstance(v, CfgNode):
                v._set_immutable(flag)

    def clone(self):
        return copy.deepcopy(self)

    # merging ------------------------------------------------------------
    @staticmethod
    def load_yaml_with_base(filename, allow_unsafe=False):
        with open(filename) as f:
            text = f.read()
        try:
            cfg = yaml.safe_load(text)
        except yaml.constructor.ConstructorError:
            if not allow_unsafe:
                raise
            cfg = yaml.load(text, Loader=_RestrictedEvalLoader)
        cfg = cfg or {}

        def merge_a_into_b(a, b):
            for k, v in a.items():
                if isinstance(v, dict) and k in b:
                    if not isinstance(b[k], dict):
                        raise AssertionError(f"Cannot inherit key '{k}' from base!")
                    merge_a_into_b(v, b[k])
                else:
                    b[k] = v

        if BASE_KEY in cfg:
            base = cfg.pop(BASE_KEY)
            if base.startswith("~"):
                base = os.path.expanduser(base)
            if not base.startswith("/"):
                base = os.path.join(os.path.dirname(filename), base)
            base_cfg = CfgNode.load_yaml_with_base(base, allow_unsafe=allow_unsafe)
            merge_a_into_b(cfg, base_cfg)
            return base_cfg
        return cfg

    def merge_from_file(self, cfg_filename, allow_unsafe=True):
        loaded = CfgNode.load_yaml_with_base(cfg_filename, allow_unsafe=allow_unsafe)
        self.merge_from_other_cfg(CfgNode(loaded))

    def merge_from_other_cfg(self, cfg_other):
        if BASE_KEY in cfg_other:
            raise AssertionError(f"The reserved key '{BASE_KEY}' can only be used in files!")
        _merge_a_into_b(cfg_other, self, self, [])

    def merge_from_list(self, cfg_list):
        if len(cfg_list) % 2 != 0:
            raise ValueError(f"Override list has odd length: {cfg_list}")
        if BASE_KEY in set(cfg_list[0::2]):
            raise AssertionError(f"The reserved key '{BASE_KEY}' can only be used in files!")
        root = self
        for full_key, v in zip(cfg_list[0::2], cfg_list[1::2]):
            if root.is_frozen():
                raise AttributeError("CfgNode is immutable")
            d = self
            parts = full_key.split(".")
            for sub in parts[:-1]:
                if sub not in d:
                    raise KeyError(f"Non-existent config key: {full_key}")
                d = d[sub]
            leaf = parts[-1]
            if leaf not in d:
                raise KeyError(f"Non-existent config key: {full_key}")
            value = _decode(v)
            d[leaf] = _coerce(value, d[leaf], full_key)

    def dump(self):
        def plain(x):
            if isinstance(x, dict):
                return {k: plain(v) for k, v in x.items()}
            if isinstance(x, tuple):
                return [plain(v) for v in x]
            return x
        return yaml.safe_dump(plain(self), sort_keys=True)


def _decode(v):
    if isinstance(v, dict):
        return CfgNode(v)
    if isinstance(v, str):
        try:
            return ast.literal_eval(v)
        except (ValueError, SyntaxError):
            return v
    return v


def _coerce(replacement, original, full_key):
    if original is None or replacement is None:
        return replacement
    if type(replacement) == type(original):
        return replacement
    if isinstance(original, (list, tuple)) and isinstance(replacement, (list, tuple)):
        return type(original)(replacement)
    if isinstance(original, float) and isinstance(replacement, int) and not isinstance(replacement, bool):
        return float(replacement)
    if isinstance(original, str) and isinstance(replacement, str):
        return replacement
    raise ValueError(f"Type mismatch ({type(original)} vs. {type(replacement)}) with values "
                     f"({original} vs. {replacement}) for config key: {full_key}")


def _merge_a_into_b(a, b, root, key_list):
    for k, v_ in a.items():
        full_key = ".".join(key_list + [k])
        v = _decode(copy.deepcopy(v_))
        if k in b:
            if isinstance(v, CfgNode) and isinstance(b[k], CfgNode):
                _merge_a_into_b(v, b[k], root, key_list + [k])
            else:
                dict.__setitem__(b, k, _coerce(v, b[k], full_key))
        else:
            raise KeyError(f"Non-existent config key: {full_key}")


# --------------------------------------------------- restricted eval tag
_BINOPS = {ast.Add: operator.add, ast.Sub: operator.sub, ast.Mult: operator.mul,
           ast.Div: operator.truediv, ast.Pow: operator.pow, ast.FloorDiv: operator.floordiv,
           ast.Mod: operator.mod}
_UNOPS = {ast.USub: operator.neg, ast.UAdd: operator.pos}


def restricted_eval(expr):
    """Evaluate a config expression such as
    ``[[x, x * 2**(1.0/3), x * 2**(2.0/3)] for x in [32, 64, 128, 256, 512]]``
    allowing only numeric literals, arithmetic, list/tuple literals and list
    comprehensions (no calls, attributes, subscripts or free names)."""
    tree = ast.parse(expr, mode="eval")

    def ev(node, env):
        if isinstance(node, ast.Expression):
            return ev(node.body, env)
        if isinstance(node, ast.Constant) and isinstance(node.value, (int, float)):
            return node.value
        if isinstance(node, (ast.List, ast.Tuple)):
            vals = [ev(e, env) for e in node.elts]
            return vals if isinstance(node, ast.List) else tuple(vals)
        if isinstance(node, ast.BinOp) and type(node.op) in _BINOPS:
            return _BINOPS[type(node.op)](ev(node.left, env), ev(node.right, env))
        if isinstance(node, ast.UnaryOp) and type(node.op) in _UNOPS:
            return _UNOPS[type(node.op)](ev(node.operand, env))
        if isinstance(node, ast.Name) and node.id in env:
            return env[node.id]
        if isinstance(node, ast.ListComp) and len(node.generators) == 1:
            gen = node.generators[0]
            if gen.ifs or gen.is_async or not isinstance(gen.target, ast.Name):
                raise ValueError("unsupported comprehension in config expression")
            out = []
            for item in ev(gen.iter, env):
                out.append(ev(node.elt, {**env, gen.target.id: item}))
            return out
        raise ValueError(f"disallowed construct in config expression: {ast.dump(node)[:80]}")

    return ev(tree, {})


class _RestrictedEvalLoader(yaml.SafeLoader):
    pass


def _construct_eval(loader, suffix, node):
    args = loader.construct_sequence(node)
    if suffix != "eval" or len(args) != 1 or not isinstance(args[0], str):
        raise yaml.constructor.ConstructorError(None, None, f"unsupported python/object/apply:{suffix}",
                                                node.start_mark)
    return restricted_eval(args[0])


_RestrictedEvalLoader.add_multi_constructor("tag:yaml.org,2002:python/object/apply:", _construct_eval)
