"""The reference-shaped Domain adapter (hyperopt_amd.base.as_domain): what
lets the reference's own driver plug this package in --
``hyperopt.fmin(fn, space, algo=hyperopt_amd.tpe.suggest)`` hands the algo
its own Domain (fmin.py:268-270, base.py:783-870), whose ``expr`` is a graph
of the reference's pyll nodes.

tests/golden/domain_fixtures.json was made by
tests/golden/make_domain_fixtures.py from the REFERENCE's Domain objects: the
graph of each space (node by node, as data), and the adapter's result on the
real reference Domain (kinds, prior arguments, live labels per decided
choice), cross-checked there against this package's own Domain.  Here the
graph is rebuilt from the JSON with stand-in node objects (no reference code
at run time) and the adapter must give the same result."""
import json
import os

import numpy as np
import pytest

from hyperopt_amd import base as B
from hyperopt_amd import hp
from hyperopt_amd import tpe

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = json.load(open(os.path.join(HERE, "golden", "domain_fixtures.json")))


def _dec(v):
    if isinstance(v, dict):
        t, x = v["t"], v["v"]
        if t == "ndarray":
            return np.asarray(x, dtype=v["dtype"])
        if t == "tuple":
            return tuple(_dec(a) for a in x)
        if t == "list":
            return [_dec(a) for a in x]
        if t == "dict":
            return {_dec(k): _dec(a) for k, a in x}
    return v


class ForeignNode(object):
    """Stand-in for the reference's pyll Apply / Literal (pyll/base.py:232-560)."""

    def __init__(self, rec, nodes):
        self.name, self.o_len, self.pure = rec["name"], rec["o_len"], rec["pure"]
        if self.name == "literal":
            self.obj = _dec(rec["obj"])
            self.pos_args, self.named_args = [], []
        else:
            self.pos_args = [nodes[i] for i in rec["pos"]]
            self.named_args = [[k, nodes[i]] for k, i in rec["named"]]


class ForeignDomain(object):
    """Reference-shaped Domain: expr, params, cmd, workdir, new_result -- no
    ``specs`` / ``reachable``."""

    def __init__(self, fix):
        nodes = []
        for rec in fix["graph"]:
            nodes.append(ForeignNode(rec, nodes))
        self.expr = nodes[-1]
        self.params = {n.pos_args[0].obj: n.pos_args[1] for n in nodes
                       if n.name == "hyperopt_param"}
        self.cmd = tuple(fix["cmd"])
        self.workdir = None
        self.fn = None

    def new_result(self):
        return {"status": "new"}


@pytest.mark.parametrize("name", sorted(FIX))
def test_adapter_matches_the_reference_domain(name):
    fix = FIX[name]
    fd = ForeignDomain(fix)
    dom = B.as_domain(fd)
    assert B.as_domain(fd) is dom  # converted once, cached
    assert B.as_domain(dom) is dom
    assert sorted(dom.params) == sorted(fix["specs"])
    for lab, (kind, args) in fix["specs"].items():
        sp = dom.specs[lab]
        assert sp.kind == kind
        got = tuple(np.asarray(a).tolist() if isinstance(a, np.ndarray) else a for a in sp.args)
        assert got == _dec(args), (lab, got, args)
    for dec, live in fix["reachable"]:
        assert dom.reachable(dict(dec)) == live, (name, dec)
    assert dom.cmd == tuple(fix["cmd"])


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["readme", "nested", "many_dists"])
def test_suggest_through_a_reference_shaped_domain(name):
    """tpe.suggest / rand.suggest_device given the reference-shaped Domain
    (the fmin(algo=hyperopt_amd.tpe.suggest) plug point) return the same
    documents as given this package's own Domain of the same space."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    import sys
    sys.path.insert(0, os.path.join(HERE, "golden"))
    import spaces as SPACES
    fd = ForeignDomain(FIX[name])
    ours = B.Domain(lambda p: 0.0, SPACES.SPACES[name](hp))
    rng = np.random.RandomState(7)
    ta, tb = B.Trials(), B.Trials()
    for it in range(30):
        seed = int(rng.randint(2 ** 31 - 1))
        da = tpe.suggest(ta.new_trial_ids(1), fd, ta, seed, n_EI_candidates=64)
        db = tpe.suggest(tb.new_trial_ids(1), ours, tb, seed, n_EI_candidates=64)
        assert [d["misc"]["vals"] for d in da] == [d["misc"]["vals"] for d in db], it
        assert da[0]["misc"]["cmd"] == fd.cmd
        for t, docs in ((ta, da), (tb, db)):
            loss = float(sum(float(np.sum(v)) for v in docs[0]["misc"]["vals"].values() if v))
            docs[0]["state"] = B.JOB_STATE_DONE
            docs[0]["result"] = {"status": B.STATUS_OK, "loss": loss}
            t.insert_trial_docs(docs)
            t.refresh()
