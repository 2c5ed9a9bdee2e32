"""``hp.*`` search-space constructors (hyperopt/hp.py, pyll_utils.py:52-132)."""
from functools import wraps

from .pyll import Literal, scope


def validate_label(f):
    @wraps(f)
    def wrapper(label, *args, **kwargs):
        is_str = isinstance(label, (str, bytes))
        is_lit = isinstance(label, Literal) and isinstance(label.obj, (str, bytes))
        if not is_str and not is_lit:
            raise TypeError("require string label")
        return f(label, *args, **kwargs)

    return wrapper


def validate_distribution_range(f):
    # mirrors pyll_utils.py:28-44, including its truthiness test on the bounds
    @wraps(f)
    def wrapper(label, *args, **kwargs):
        lo = args[0] if len(args) > 0 else kwargs.get("low")
        hi = args[1] if len(args) > 1 else kwargs.get("high")
        if lo and hi and not lo < hi:
            raise ValueError("low should be less than high: %s is not smaller than %s" % (lo, hi))
        return f(label, *args, **kwargs)

    return wrapper


@validate_label
def pchoice(label, p_options):
    p, options = list(zip(*p_options))
    ch = scope.hyperopt_param(label, scope.categorical(p))
    return scope.switch(ch, *options)


@validate_label
def choice(label, options):
    ch = scope.hyperopt_param(label, scope.randint(len(options)))
    return scope.switch(ch, *options)


@validate_label
def randint(label, *args, **kwargs):
    return scope.hyperopt_param(label, scope.randint(*args, **kwargs))


@validate_label
@validate_distribution_range
def uniform(label, *args, **kwargs):
    return scope.float(scope.hyperopt_param(label, scope.uniform(*args, **kwargs)))


@validate_label
@validate_distribution_range
def quniform(label, *args, **kwargs):
    return scope.float(scope.hyperopt_param(label, scope.quniform(*args, **kwargs)))


@validate_label
def uniformint(label, *args, **kwargs):
    args += (1.0,)
    return scope.int(quniform(label, *args, **kwargs))


@validate_label
@validate_distribution_range
def loguniform(label, *args, **kwargs):
    return scope.float(scope.hyperopt_param(label, scope.loguniform(*args, **kwargs)))


@validate_label
@validate_distribution_range
def qloguniform(label, *args, **kwargs):
    return scope.float(scope.hyperopt_param(label, scope.qloguniform(*args, **kwargs)))


@validate_label
def normal(label, *args, **kwargs):
    return scope.float(scope.hyperopt_param(label, scope.normal(*args, **kwargs)))


@validate_label
def qnormal(label, *args, **kwargs):
    return scope.float(scope.hyperopt_param(label, scope.qnormal(*args, **kwargs)))


@validate_label
def lognormal(label, *args, **kwargs):
    return scope.float(scope.hyperopt_param(label, scope.lognormal(*args, **kwargs)))


@validate_label
def qlognormal(label, *args, **kwargs):
    return scope.float(scope.hyperopt_param(label, scope.qlognormal(*args, **kwargs)))
