"""Fixtures for the reference-shaped Domain adapter (hyperopt_amd.base.as_domain).

Run in the build container only (needs /root/reference, loaded exactly as
make_golden.py loads it):

    python tests/golden/make_domain_fixtures.py

For every space of spaces.py it builds the REFERENCE's own Domain
(hyperopt/base.py:783-870, the object hyperopt.fmin passes to its algo,
fmin.py:268-270) and stores, as JSON data:
  * the reference Domain's pyll graph, node by node (name, argument indices,
    o_len, pure, literal values with type tags) -- the graph, not source;
  * the adapter's result on that real reference Domain: every label's prior
    kind and arguments, and the live labels for a set of decided choices;
  * the same from this package's own Domain built with hyperopt_amd.hp --
    the generator asserts that the two agree.
tests/test_domain_adapter.py rebuilds the graph from the JSON with stand-in
node objects and checks the adapter against the recorded results.
"""
from __future__ import annotations

import itertools
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
import spaces as SPACES  # noqa: E402
from make_golden import load_reference  # noqa: E402


def enc(v):
    if isinstance(v, np.ndarray):
        return {"t": "ndarray", "dtype": str(v.dtype), "v": v.tolist()}
    if isinstance(v, np.generic):
        return enc(v.item())
    if isinstance(v, tuple):
        return {"t": "tuple", "v": [enc(x) for x in v]}
    if isinstance(v, list):
        return {"t": "list", "v": [enc(x) for x in v]}
    if isinstance(v, dict):
        return {"t": "dict", "v": [[enc(k), enc(x)] for k, x in v.items()]}
    if v is None or isinstance(v, (bool, int, float, str)):
        return v
    raise TypeError("literal of type %s" % type(v))


def graph(expr):
    """Nodes in post order: {name, pos, named, o_len, pure[, obj]}."""
    order, index, stack = [], {}, [(expr, False)]
    while stack:
        n, done = stack.pop()
        if id(n) in index:
            continue
        if done or n.name == "literal":
            index[id(n)] = len(order)
            rec = {"name": n.name, "o_len": n.o_len, "pure": bool(n.pure)}
            if n.name == "literal":
                rec["obj"] = enc(n.obj)
            else:
                rec["pos"] = [index[id(a)] for a in n.pos_args]
                rec["named"] = [[k, index[id(v)]] for k, v in n.named_args]
            order.append(rec)
            continue
        stack.append((n, True))
        for k in reversed(list(n.pos_args) + [v for _, v in n.named_args]):
            if id(k) not in index:
                stack.append((k, False))
    return order


def spec_record(dom):
    out = {}
    for lab in sorted(dom.specs):
        sp = dom.specs[lab]
        out[lab] = [sp.kind, enc(tuple(np.asarray(a).tolist() if isinstance(a, np.ndarray) else a
                                     for a in sp.args))]
    return out


def decided_sets(dom):
    """Decided-choice combinations to test reachability on: every selector
    label's categories (up to 3 each), plus nothing decided."""
    sel = sorted(lab for lab in dom.specs if dom.specs[lab].kind in ("randint", "categorical"))
    opts = []
    for lab in sel[:3]:
        sp = dom.specs[lab]
        n = len(sp.args[0]) if sp.kind == "categorical" else (
            sp.args[0] if sp.args[1] is None else sp.args[1] - sp.args[0])
        opts.append([(lab, int(i)) for i in range(min(int(n), 3))])
    combos = [{}]
    for c in itertools.product(*opts):
        combos.append(dict(c))
    return combos


def main():
    ref = load_reference()
    sys.path.insert(0, ROOT)
    from hyperopt_amd import base as B
    from hyperopt_amd import hp as our_hp
    out = {}
    for name, build in SPACES.SPACES.items():
        rdom = ref.base.Domain(lambda p: 0.0, build(ref.hp))
        conv = B.as_domain(rdom)
        ours = B.Domain(lambda p: 0.0, build(our_hp))
        assert sorted(conv.params) == sorted(rdom.params) == sorted(ours.params), name
        specs = spec_record(conv)
        assert specs == spec_record(ours), name
        reach = []
        for dec in decided_sets(ours):
            live = conv.reachable(dict(dec))
            assert live == ours.reachable(dict(dec)), (name, dec)
            reach.append([dec, live])
        out[name] = {"graph": graph(rdom.expr), "specs": specs, "reachable": reach,
                     "cmd": list(rdom.cmd)}
        print(name, len(out[name]["graph"]), "nodes,", len(specs), "labels,", len(reach),
              "decided sets")
    with open(os.path.join(HERE, "domain_fixtures.json"), "w") as f:
        json.dump(out, f, indent=0, sort_keys=True)


if __name__ == "__main__":
    main()
