"""Random search (hyperopt/rand.py:15-37) and the startup phase of tpe.suggest.

``suggest`` / ``suggest_batch``: the reference's random-search algorithm on
the host -- every live hyperparameter drawn from its prior with numpy's
RandomState(seed), following the conditional structure of the space (a
choice's branch is only sampled when it is taken).

``suggest_device``: the same prior draws on the GPU (tpe_prior_sample, one
launch for every label of every new trial; Philox keyed by (seed, label,
position in new_ids)), used by tpe.suggest for its first n_startup_jobs
calls (tpe.py:909-911).  The conditional structure is resolved on the host:
a trial keeps the labels its own choices make live.  Same distributions as
pyll/stochastic.py:36-158 (tests/test_gpu_prior.py); the streams differ.
"""
from __future__ import annotations

import ctypes

import numpy as np

from .base import as_domain


def sample_config(domain, rng):
    """{label: value} for the labels live under the sampled choices."""
    decided = {}
    while True:
        live = domain.reachable(decided)
        todo = [lab for lab in live if lab not in decided]
        if not todo:
            return {lab: decided[lab] for lab in live}
        for lab in todo:
            decided[lab] = domain.specs[lab].sample(rng)


def _misc(domain, new_id, config):
    return dict(tid=new_id, cmd=domain.cmd, workdir=domain.workdir,
                idxs={lab: ([new_id] if lab in config else []) for lab in domain.params},
                vals={lab: ([config[lab]] if lab in config else []) for lab in domain.params})


def suggest(new_ids, domain, trials, seed):
    domain = as_domain(domain)
    rng = np.random.RandomState(seed)
    rval = []
    for new_id in new_ids:
        config = sample_config(domain, rng)
        rval.extend(trials.new_trial_docs([new_id], [None], [domain.new_result()],
                                          [_misc(domain, new_id, config)]))
    return rval


def suggest_batch(new_ids, domain, trials, seed):
    domain = as_domain(domain)
    rng = np.random.RandomState(seed)
    idxs = {lab: [] for lab in domain.params}
    vals = {lab: [] for lab in domain.params}
    for new_id in new_ids:
        for lab, v in sample_config(domain, rng).items():
            idxs[lab].append(new_id)
            vals[lab].append(v)
    return idxs, vals


# ---------------------------------------------------------------------------
# device prior draws
# ---------------------------------------------------------------------------
def _prior_table(domain):
    """(labels, tpe_prior records without keys, probability pool), cached on
    the domain (the space does not change)."""
    cached = domain.__dict__.get("_tpe_prior_table")
    if cached is not None:
        return cached
    from . import _lib as L
    labels = list(domain.params)
    rec = np.zeros(len(labels), L.PRIOR_DTYPE)
    pool, off = [], 0
    for j, lab in enumerate(labels):
        kind, a = domain.specs[lab].kind, domain.specs[lab].args
        if kind in ("uniform", "quniform", "loguniform", "qloguniform",
                    "normal", "qnormal", "lognormal", "qlognormal"):
            if kind in ("uniform", "quniform", "loguniform", "qloguniform"):
                code = L.PRIOR_LOGUNIFORM if "log" in kind else L.PRIOR_UNIFORM
            else:
                code = L.PRIOR_LOGNORMAL if "log" in kind else L.PRIOR_NORMAL
            rec[j] = (code, 0, float(a[0]), float(a[1]),
                      float(a[2]) if kind.startswith("q") else 0.0, 0, 0)
        elif kind == "randint":
            lo, hi = (0, int(a[0])) if (len(a) < 2 or a[1] is None) else (int(a[0]), int(a[1]))
            rec[j] = (L.PRIOR_RANDINT, 0, float(lo), float(hi), 0.0, 0, 0)
        else:  # categorical (hp.pchoice): p, possibly 2-D with identical rows
            p = np.asarray(a[0], dtype=np.float64)
            p = p[0] if p.ndim == 2 else p.reshape(-1)
            rec[j] = (L.PRIOR_CATEGORICAL, p.size, 0.0, 0.0, 0.0, off, 0)
            pool.append(p)
            off += p.size
    pool = np.concatenate(pool) if pool else np.zeros(1)
    domain._tpe_prior_table = (labels, rec, pool)
    return domain._tpe_prior_table


def draw_priors(domain, seed, n):
    """n draws of every label's prior on the current GPU: (labels, array of
    shape (len(labels), n)), draw i of label j a function of (seed, label, i)."""
    import torch
    from . import _lib as L
    from .tpe import label_keys
    labels, rec, pool = _prior_table(domain)
    rec = rec.copy()
    rec["key"] = label_keys(seed, labels)
    if n == 0 or not labels:
        return labels, np.zeros((len(labels), n))
    dev = torch.device("cuda", torch.cuda.current_device())
    d_rec = torch.from_numpy(rec.view(np.uint8).copy()).to(dev)
    d_p = torch.from_numpy(pool).to(dev)
    out = torch.empty(len(labels) * n, dtype=torch.float64, device=dev)
    stream = torch.cuda.current_stream(dev)
    L.check(L.load().tpe_prior_sample(d_rec.data_ptr(), rec.ctypes.data_as(ctypes.c_void_p),
                                      len(labels), d_p.data_ptr(), n, 0, out.data_ptr(),
                                      ctypes.c_void_p(stream.cuda_stream)), "tpe_prior_sample")
    return labels, out.cpu().numpy().reshape(len(labels), n)


def _configs(domain, labels, vals):
    """Per new trial, {label: value} of the labels its own choices make live."""
    col = {lab: j for j, lab in enumerate(labels)}
    ints = {lab for lab in labels if domain.specs[lab].kind in ("randint", "categorical")}
    out = []
    for i in range(vals.shape[1]):
        decided = {}
        while True:
            live = domain.reachable(decided)
            todo = [lab for lab in live if lab not in decided]
            if not todo:
                break
            for lab in todo:
                v = vals[col[lab], i]
                decided[lab] = int(round(v)) if lab in ints else float(v)
        out.append({lab: decided[lab] for lab in live})
    return out


def suggest_device(new_ids, domain, trials, seed):
    """rand.suggest with the prior draws made on the GPU (see module doc)."""
    domain = as_domain(domain)
    labels, vals = draw_priors(domain, seed, len(new_ids))
    rval = []
    for new_id, config in zip(new_ids, _configs(domain, labels, vals)):
        rval.extend(trials.new_trial_docs([new_id], [None], [domain.new_result()],
                                          [_misc(domain, new_id, config)]))
    return rval
