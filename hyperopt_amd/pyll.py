"""A small expression-graph runtime for search spaces (the reference's `pyll`).

Mirrors the parts of hyperopt/pyll/base.py and pyll/stochastic.py that search
spaces and objective expressions use: ``Apply`` / ``Literal`` nodes with
operator overloading (pyll/base.py:231-587), ``as_apply`` (:204-228), the
``scope`` symbol table with ``define``/``define_pure``/``define_info``
(:41-201), ``dfs``/``toposort`` (:681-713), ``rec_eval`` with lazy ``switch``
(:775-934), and the prior samplers (pyll/stochastic.py:36-158).

It is host-side plumbing for the drop-in API; the TPE hot path does not
interpret graphs (hyperopt_amd/tpe.py walks the space level by level and hands
each level to the GPU engine).
"""
from __future__ import annotations

import inspect
import math
import operator

import numpy as np


class PyllImportError(ImportError):
    """A pyll symbol was not defined in the scope."""


class MissingArgument(object):
    """Placeholder for a missing argument."""


class GarbageCollected(object):
    """Marks memo entries that must not be read (Domain.memo_from_config)."""


class SymbolTableEntry(object):
    def __init__(self, table, name, o_len, pure):
        self.table = table
        self.apply_name = name
        self.o_len = o_len
        self.pure = pure

    def __call__(self, *args, **kwargs):
        return self.table._new_apply(self.apply_name, args, kwargs, self.o_len, self.pure)


class SymbolTable(object):
    """Allocates Apply nodes by name; ``_impls`` holds their implementations."""

    def __init__(self):
        self._impls = {
            "list": list, "dict": dict, "range": range, "len": len, "int": int,
            "float": float, "map": map, "max": max, "min": min, "getattr": getattr,
        }

    def _new_apply(self, name, args, kwargs, o_len, pure):
        pos = [as_apply(a) for a in args]
        named = sorted((k, as_apply(v)) for k, v in kwargs.items())
        return Apply(name, pos, named, o_len=o_len, pure=pure)

    def dict(self, *args, **kwargs):
        return self._new_apply("dict", args, kwargs, None, True)

    def int(self, arg):
        return self._new_apply("int", [arg], {}, None, True)

    def float(self, arg):
        return self._new_apply("float", [arg], {}, None, True)

    def len(self, obj):
        return self._new_apply("len", [obj], {}, None, True)

    def list(self, init):
        return self._new_apply("list", [init], {}, None, True)

    def range(self, *args):
        return self._new_apply("range", args, {}, None, True)

    def max(self, *args):
        return self._new_apply("max", args, {}, None, True)

    def min(self, *args):
        return self._new_apply("min", args, {}, None, True)

    def getattr(self, obj, attr, *args):
        return self._new_apply("getattr", (obj, attr) + args, {}, None, True)

    def _define(self, f, o_len, pure):
        name = f.__name__
        setattr(self, name, SymbolTableEntry(self, name, o_len, pure))
        self._impls[name] = f
        return f

    def define(self, f, o_len=None, pure=False):
        """Register ``f`` under its name; raises on redefinition (pyll/base.py:129-135)."""
        if hasattr(self, f.__name__):
            raise ValueError("Cannot override existing symbol", f.__name__)
        return self._define(f, o_len, pure)

    def define_if_new(self, f, o_len=None, pure=False):
        name = f.__name__
        if hasattr(self, name) and self._impls.get(name) is not f:
            raise ValueError("Cannot redefine existing symbol", name)
        return self._define(f, o_len, pure)

    def define_pure(self, f):
        return self.define(f, o_len=None, pure=True)

    def define_info(self, o_len=None, pure=False):
        def wrapper(f):
            return self.define(f, o_len=o_len, pure=pure)

        return wrapper

    def inject(self, *args, **kwargs):
        for a in args:
            self.define_if_new(a)
        for k, v in kwargs.items():
            self._impls[k] = v
            setattr(self, k, SymbolTableEntry(self, k, None, False))

    def undefine(self, f):
        name = f if isinstance(f, str) else f.__name__
        del self._impls[name]
        delattr(self, name)


scope = SymbolTable()


def as_apply(obj):
    """Smart constructor: lists/tuples -> pos_args, dicts -> dict, else Literal."""
    if isinstance(obj, Apply):
        return obj
    if isinstance(obj, tuple):
        return Apply("pos_args", [as_apply(a) for a in obj], [], o_len=len(obj))
    if isinstance(obj, list):
        return Apply("pos_args", [as_apply(a) for a in obj], [], o_len=None)
    if isinstance(obj, dict):
        items = list(obj.items())
        if all(isinstance(k, str) for k, _ in items):
            named = sorted((k, as_apply(v)) for k, v in items)
            return Apply("dict", [], named, o_len=len(named))
        return Apply("dict", [as_apply([as_apply(kv) for kv in items])], [], o_len=None)
    return Literal(obj)


class Apply(object):
    """A function application node."""

    def __init__(self, name, pos_args, named_args, o_len=None, pure=False, define_params=None):
        self.name = name
        self.pos_args = list(pos_args)
        self.named_args = [[k, v] for k, v in named_args]
        self.o_len = o_len
        self.pure = pure
        self.define_params = define_params
        for x in self.pos_args:
            assert isinstance(x, Apply), x
        for _, v in self.named_args:
            assert isinstance(v, Apply), v

    # -- structure ----------------------------------------------------------
    def inputs(self):
        return self.pos_args + [v for _, v in self.named_args]

    @property
    def arg(self):
        """Arguments bound to the implementation's parameter names."""
        binding = dict(self.named_args)
        impl = scope._impls.get(self.name)
        params = []
        if impl is not None:
            try:
                params = list(inspect.signature(impl).parameters.values())
            except (TypeError, ValueError):
                params = []
        pos = list(self.pos_args)
        for p in params:
            if not pos:
                break
            if p.kind == p.VAR_POSITIONAL:
                binding[p.name] = pos
                pos = []
            elif p.kind in (p.POSITIONAL_ONLY, p.POSITIONAL_OR_KEYWORD):
                binding[p.name] = pos.pop(0)
        if pos:
            binding["__pos__"] = pos
        return binding

    def replace_input(self, old, new):
        for i, a in enumerate(self.pos_args):
            if a is old:
                self.pos_args[i] = new
        for kv in self.named_args:
            if kv[1] is old:
                kv[1] = new

    def clone_from_inputs(self, inputs, o_len="same"):
        n = len(self.pos_args)
        return Apply(self.name, inputs[:n],
                     [(k, v) for (k, _), v in zip(self.named_args, inputs[n:])],
                     o_len=self.o_len if o_len == "same" else o_len, pure=self.pure)

    def eval(self, memo=None):
        return rec_eval(self, memo=memo)

    def __str__(self):
        return "%s(%s)" % (self.name, ", ".join(
            [str(a) for a in self.pos_args] + ["%s=%s" % (k, v) for k, v in self.named_args]))

    __repr__ = __str__

    # -- operators (pyll/base.py:459-531) -------------------------------------
    def __add__(self, o):
        return scope.add(self, o)

    def __radd__(self, o):
        return scope.add(o, self)

    def __sub__(self, o):
        return scope.sub(self, o)

    def __rsub__(self, o):
        return scope.sub(o, self)

    def __neg__(self):
        return scope.neg(self)

    def __mul__(self, o):
        return scope.mul(self, o)

    def __rmul__(self, o):
        return scope.mul(o, self)

    def __truediv__(self, o):
        return scope.truediv(self, o)

    def __rtruediv__(self, o):
        return scope.truediv(o, self)

    def __floordiv__(self, o):
        return scope.floordiv(self, o)

    def __rfloordiv__(self, o):
        return scope.floordiv(o, self)

    def __pow__(self, o):
        return scope.pow(self, o)

    def __rpow__(self, o):
        return scope.pow(o, self)

    def __gt__(self, o):
        return scope.gt(self, o)

    def __ge__(self, o):
        return scope.ge(self, o)

    def __lt__(self, o):
        return scope.lt(self, o)

    def __le__(self, o):
        return scope.le(self, o)

    def __getitem__(self, idx):
        if self.o_len is not None and isinstance(idx, int) and idx >= self.o_len:
            raise IndexError()
        return scope.getitem(self, idx)

    def __len__(self):
        if self.o_len is None:
            raise TypeError("len of pyll.Apply either undefined or unknown")
        return self.o_len

    def __call__(self, *args, **kwargs):
        return scope.call(self, args, kwargs)

    # identity-based hashing (nodes are graph vertices)
    __hash__ = object.__hash__

    def __eq__(self, other):  # noqa: D105 -- identity, like the reference's dict keys
        return self is other


class Literal(Apply):
    def __init__(self, obj=None):
        try:
            o_len = len(obj)
        except TypeError:
            o_len = None
        Apply.__init__(self, "literal", [], [], o_len, pure=True)
        self._obj = obj

    @property
    def obj(self):
        return self._obj

    def __str__(self):
        return "Literal{%s}" % (self._obj,)

    __repr__ = __str__


def dfs(aa, seq=None, seqset=None):
    """Post-order (inputs before users) list of the nodes reachable from aa."""
    if seq is None:
        seq, seqset = [], set()
    stack = [(aa, False)]
    while stack:
        node, done = stack.pop()
        if done:
            if id(node) not in seqset:
                seqset.add(id(node))
                seq.append(node)
            continue
        if id(node) in seqset:
            continue
        stack.append((node, True))
        for ii in reversed(node.inputs()):
            if id(ii) not in seqset:
                stack.append((ii, False))
    return seq


def toposort(expr):
    return dfs(expr)


def clone(expr, memo=None):
    memo = {} if memo is None else memo
    for node in dfs(expr):
        if id(node) in memo:
            continue
        if isinstance(node, Literal):
            memo[id(node)] = node
        else:
            memo[id(node)] = node.clone_from_inputs([memo[id(i)] for i in node.inputs()])
    return memo[id(expr)]


def rec_eval(expr, deepcopy_inputs=False, memo=None, max_program_len=100000, memo_gc=False,
             print_trace=False, print_node_on_error=True):
    """Evaluate a graph; ``switch`` evaluates only the chosen branch.

    memo maps nodes (by identity) to values and is copied, as in
    pyll/base.py:775-934.
    """
    node = as_apply(expr)
    vals = {}
    if memo:
        for k, v in memo.items():
            vals[id(k)] = v
    keep = [node]  # keep ids alive
    todo = [node]
    while todo:
        if len(todo) > max_program_len:
            raise RuntimeError("Probably infinite loop in document")
        n = todo.pop()
        if id(n) in vals:
            continue
        if n.name == "switch":
            sel = n.pos_args[0]
            if id(sel) not in vals:
                todo += [n, sel]
                continue
            i = vals[id(sel)]
            try:
                int(i)
            except Exception:
                raise TypeError("switch argument was", i)
            if i != int(i) or i < 0:
                raise ValueError("switch pos must be positive int", i)
            chosen = n.pos_args[int(i) + 1]
            if id(chosen) not in vals:
                todo += [n, chosen]
                continue
            vals[id(n)] = vals[id(chosen)]
            continue
        if isinstance(n, Literal):
            vals[id(n)] = n.obj
            continue
        waiting = [v for v in n.inputs() if id(v) not in vals]
        if waiting:
            todo.append(n)
            todo.extend(waiting)
            continue
        args = [vals[id(v)] for v in n.pos_args]
        kwargs = {k: vals[id(v)] for k, v in n.named_args}
        try:
            fn = scope._impls[n.name]
        except KeyError:
            raise PyllImportError(n.name)
        try:
            rv = fn(*args, **kwargs)
        except Exception:
            if print_node_on_error:
                print("ERROR in rec_eval node", n.name)
            raise
        if isinstance(rv, Apply):
            keep.append(rv)
            rv = rec_eval(rv, memo={k: v for k, v in (memo or {}).items()})
        vals[id(n)] = rv
    return vals[id(node)]


# ---------------------------------------------------------------------------
# pure numeric symbols (pyll/base.py:941-1101)
# ---------------------------------------------------------------------------
@scope.define_pure
def pos_args(*args):
    return args


@scope.define_pure
def identity(obj):
    return obj


for _op in (operator.getitem, operator.add, operator.sub, operator.mul, operator.truediv,
            operator.floordiv, operator.neg, operator.eq, operator.lt, operator.le,
            operator.gt, operator.ge):
    scope.define_pure(_op)


@scope.define_pure
def exp(a):
    return np.exp(a)


@scope.define_pure
def log(a):
    return np.log(a)


@scope.define_pure
def pow(a, b):  # noqa: A001
    return a ** b


@scope.define_pure
def sin(a):
    return np.sin(a)


@scope.define_pure
def cos(a):
    return np.cos(a)


@scope.define_pure
def tan(a):
    return np.tan(a)


@scope.define_pure
def sum(x, axis=None):  # noqa: A001
    return np.sum(x) if axis is None else np.sum(x, axis=axis)


@scope.define_pure
def sqrt(x):
    return np.sqrt(x)


@scope.define_pure
def minimum(x, y):
    return np.minimum(x, y)


@scope.define_pure
def maximum(x, y):
    return np.maximum(x, y)


@scope.define_pure
def asarray(a, dtype=None):
    return np.asarray(a) if dtype is None else np.asarray(a, dtype=dtype)


@scope.define_pure
def str_join(s, seq):
    return s.join(seq)


@scope.define_pure
def repeat(n_times, obj):
    return [obj] * n_times


@scope.define
def call(fn, args=(), kwargs={}):  # noqa: B006
    return fn(*args, **kwargs)


@scope.define
def call_method(obj, methodname, *args, **kwargs):
    return getattr(obj, methodname)(*args, **kwargs)


@scope.define_pure
def call_method_pure(obj, methodname, *args, **kwargs):
    return getattr(obj, methodname)(*args, **kwargs)


@scope.define_pure
def switch(pos, *args):
    return args[pos]


def _kwswitch(kw, **kwargs):
    keys, values = list(zip(*sorted(kwargs.items())))
    match_idx = scope.call_method_pure(keys, "index", kw)
    return scope.switch(match_idx, *values)


scope.kwswitch = _kwswitch


@scope.define_pure
def Raise(etype, *args, **kwargs):  # noqa: N802
    raise etype(*args, **kwargs)


@scope.define
def hyperopt_param(label, obj):
    """Annotates a hyperparameter (pyll_utils.py:72-80)."""
    return obj


# ---------------------------------------------------------------------------
# prior samplers (pyll/stochastic.py:36-158), numpy RandomState
# ---------------------------------------------------------------------------
implicit_stochastic_symbols = set()


def implicit_stochastic(f):
    implicit_stochastic_symbols.add(f.__name__)
    return f


@implicit_stochastic
@scope.define
def uniform(low, high, rng=None, size=()):
    return rng.uniform(low, high, size=size)


@implicit_stochastic
@scope.define
def loguniform(low, high, rng=None, size=()):
    return np.exp(rng.uniform(low, high, size=size))


@implicit_stochastic
@scope.define
def quniform(low, high, q, rng=None, size=()):
    return np.round(rng.uniform(low, high, size=size) / q) * q


@implicit_stochastic
@scope.define
def qloguniform(low, high, q, rng=None, size=()):
    return np.round(np.exp(rng.uniform(low, high, size=size)) / q) * q


@implicit_stochastic
@scope.define
def normal(mu, sigma, rng=None, size=()):
    return rng.normal(mu, sigma, size=size)


@implicit_stochastic
@scope.define
def qnormal(mu, sigma, q, rng=None, size=()):
    return np.round(rng.normal(mu, sigma, size=size) / q) * q


@implicit_stochastic
@scope.define
def lognormal(mu, sigma, rng=None, size=()):
    return np.exp(rng.normal(mu, sigma, size=size))


@implicit_stochastic
@scope.define
def qlognormal(mu, sigma, q, rng=None, size=()):
    return np.round(np.exp(rng.normal(mu, sigma, size=size)) / q) * q


@implicit_stochastic
@scope.define
def randint(low, high=None, rng=None, size=()):
    return rng.randint(low, high, size)


@implicit_stochastic
@scope.define
def categorical(p, rng=None, size=()):
    """Draws i with probability p[i] (pyll/stochastic.py:119-158)."""
    if len(p) == 1 and isinstance(p[0], np.ndarray):
        p = p[0]
    p = np.asarray(p)
    if size == ():
        size = (1,)
    elif isinstance(size, (int, np.number)):
        size = (int(size),)
    else:
        size = tuple(size)
    if size == (0,):
        return np.asarray([])
    n = int(np.prod(size))
    draws = rng.multinomial(n=1, pvals=p, size=n)
    return np.dot(draws, np.arange(len(p))).reshape(size)


def recursive_set_rng_kwarg(expr, rng=None):
    """Make every stochastic node in expr use ``rng`` (pyll/stochastic.py:176-193)."""
    if rng is None:
        rng = np.random.RandomState()
    lrng = as_apply(rng)
    for node in dfs(expr):
        if node.name in implicit_stochastic_symbols:
            for kv in node.named_args:
                if kv[0] == "rng":
                    kv[1] = lrng
                    break
            else:
                node.named_args.append(["rng", lrng])
    return expr


def sample(expr, rng=None, **kwargs):
    """Draw one sample of a stochastic expression."""
    if rng is None:
        rng = np.random.RandomState()
    return rec_eval(recursive_set_rng_kwarg(clone(as_apply(expr)), as_apply(rng)), **kwargs)


_ = math  # keep math importable for user expressions
