"""Random search: the startup path of tpe.suggest (hyperopt/rand.py:15-37).

Draws every live hyperparameter from its prior with numpy's RandomState(seed),
following the conditional structure of the space (a choice's branch is only
sampled when it is taken), and returns new trial documents.
"""
from __future__ import annotations

import numpy as np


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
    rng = np.random.RandomState(seed)
    rval = []
    for new_id in new_ids:
        config = sample_config(domain, rng)
        rval.extend(trials.new_trial_docs([new_id], [None], [domain.new_result()],
                                          [_misc(domain, new_id, config)]))
    return rval


def suggest_batch(new_ids, domain, trials, seed):
    rng = np.random.RandomState(seed)
    idxs = {lab: [] for lab in domain.params}
    vals = {lab: [] for lab in domain.params}
    for new_id in new_ids:
        for lab, v in sample_config(domain, rng).items():
            idxs[lab].append(new_id)
            vals[lab].append(v)
    return idxs, vals
