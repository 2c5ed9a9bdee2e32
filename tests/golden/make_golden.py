"""Generate golden vectors by running the REFERENCE hyperopt (read-only, /root/reference).

Run in the build container only (the reference does not exist on the GPU box):

    python tests/golden/make_golden.py

The reference needs three pure-Python modules that are not installed here
(`past.utils.old_div`, `past.builtins.basestring`,
`future.standard_library.install_aliases`).  This script writes tiny stand-ins
for them into a temporary directory (our own code, not reference source) and
puts that directory plus /root/reference on sys.path.  No reference source is
copied; the outputs are data only (inputs and expected outputs), stored as
``.npz`` files with a JSON metadata string, loadable with
``np.load(allow_pickle=False)``.

Tie handling: cases flagged ``stable`` are generated with ``np.argsort``
forced to ``kind="stable"`` while the reference runs (its default sort kind has
host-dependent tie order); all other cases run unpatched.
"""
from __future__ import annotations

import contextlib
import json
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
sys.path.insert(0, HERE)
import spaces as SPACES  # noqa: E402

_SHIMS = {
    "past/__init__.py": "",
    "past/utils.py": (
        "import numbers\n"
        "def old_div(a, b):\n"
        "    if isinstance(a, numbers.Integral) and isinstance(b, numbers.Integral):\n"
        "        return a // b\n"
        "    return a / b\n"),
    "past/builtins.py": "basestring = (str, bytes)\n",
    "future/__init__.py": "",
    "future/standard_library.py": "def install_aliases():\n    pass\n",
}


def load_reference():
    sys.dont_write_bytecode = True  # never write into /root/reference
    shim = tempfile.mkdtemp(prefix="hyperopt_ref_shim_")
    for rel, body in _SHIMS.items():
        path = os.path.join(shim, rel)
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "w") as f:
            f.write(body)
    sys.path[:0] = [shim, REF]
    import hyperopt  # noqa: F401
    import hyperopt.tpe  # noqa: F401
    import hyperopt.rand  # noqa: F401
    assert hyperopt.__file__.startswith(REF), hyperopt.__file__
    return hyperopt


@contextlib.contextmanager
def stable_argsort(enabled=True):
    if not enabled:
        yield
        return
    orig = np.argsort

    def patched(a, axis=-1, kind=None, order=None, **kw):
        return orig(a, axis=axis, kind="stable", order=order)

    np.argsort = patched
    try:
        yield
    finally:
        np.argsort = orig


def save(name, arrays, meta):
    out = dict(arrays)
    out["__meta__"] = np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8)
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes")


# ---------------------------------------------------------------------------
# unit-level vectors
# ---------------------------------------------------------------------------
def gen_units(ho):
    tpe = ho.tpe
    rng = np.random.RandomState(1234)
    arrays, meta = {}, {"numpy": np.__version__, "parzen": [], "split": [], "lpdf": [],
                        "best": [], "cat": []}
    import scipy
    meta["scipy"] = scipy.__version__

    # -- adaptive_parzen_normal (tpe.py:399-467)
    pz = [
        (np.zeros(0), 1.0, 0.0, 1.0, 25, False),
        (np.array([0.3]), 1.0, 0.5, 1.0, 25, False),  # prior after obs
        (np.array([0.7]), 1.0, 0.5, 1.0, 25, False),  # prior before obs
        (np.array([0.5]), 1.0, 0.5, 1.0, 25, False),  # tie, len==1 branch
        (np.array([0.9, 0.1]), 2.5, 0.5, 2.0, 25, False),
        (np.array([0.9, 0.1, 0.4]), 1.0, 0.4, 1.0, 25, False),  # searchsorted tie
        (rng.uniform(-5, 5, 24), 1.0, 0.0, 10.0, 25, False),
        (rng.uniform(-5, 5, 25), 1.0, 0.0, 10.0, 25, False),
        (rng.uniform(-5, 5, 26), 1.0, 0.0, 10.0, 25, False),
        (rng.uniform(-5, 5, 30), 0.01, 0.0, 10.0, 25, False),
        (rng.uniform(-5, 5, 500), 1.0, 0.0, 10.0, 25, False),
        (rng.uniform(-5, 5, 500), 1.0, 0.0, 10.0, 0, False),  # LF disabled
        (rng.normal(0, 2, 3000), 1.0, 0.0, 2.0, 25, False),
        (np.round(rng.uniform(0, 10, 200)), 1.0, 5.0, 10.0, 25, True),  # ties
        (np.round(rng.uniform(0, 3, 80)), 1.0, 1.5, 3.0, 25, True),
        (rng.uniform(-5, 0, 1000), 1.0, -2.5, 5.0, 25, False),
    ]
    for i, (obs, pw, pmu, psig, lf, stable) in enumerate(pz):
        with stable_argsort(stable):
            w, mu, sig = tpe.adaptive_parzen_normal(obs, pw, pmu, psig, LF=lf)
        arrays["parzen%d_obs" % i] = obs
        arrays["parzen%d_w" % i] = w
        arrays["parzen%d_mu" % i] = mu
        arrays["parzen%d_sigma" % i] = sig
        meta["parzen"].append(dict(prior_weight=pw, prior_mu=pmu, prior_sigma=psig,
                                   lf=lf, stable=stable))

    # -- ap_split_trials (tpe.py:623-646)
    sp = []
    for T in (1, 2, 5, 17, 100, 1000, 5000):
        tids = np.arange(T) * 3 + 7
        losses = rng.normal(size=T)
        sp.append((tids, rng.uniform(size=T), tids, losses, 0.25, False))
    tids = np.arange(400)
    losses = np.round(rng.normal(size=400), 1)  # duplicate losses
    losses[::9] = np.inf  # failed / running trials
    sub = tids[rng.uniform(size=400) < 0.6]  # label active on a subset
    sp.append((sub, rng.uniform(size=sub.size), tids, losses, 0.25, True))
    sp.append((tids, rng.uniform(size=400), tids, losses, 0.05, True))
    for i, (oi, ov, li, lv, g, stable) in enumerate(sp):
        with stable_argsort(stable):
            b, a = tpe.ap_split_trials(oi, ov, li, lv, g)
        arrays.update({"split%d_oi" % i: oi, "split%d_ov" % i: ov, "split%d_li" % i: li,
                       "split%d_lv" % i: lv, "split%d_below" % i: np.asarray(b, float),
                       "split%d_above" % i: np.asarray(a, float)})
        meta["split"].append(dict(gamma=g, stable=stable))

    # -- GMM1_lpdf / LGMM1_lpdf (tpe.py:117-180, 265-307)
    lp = []
    mix_u = tpe.adaptive_parzen_normal(rng.uniform(-5, 5, 300), 1.0, 0.0, 10.0)
    cand_u = np.concatenate([rng.uniform(-5, 5, 400), [-5.0, 4.999999, 0.0, 50.0, -1e3]])
    lp.append(("GMM1", mix_u, cand_u, None, None, None))
    lp.append(("GMM1", mix_u, cand_u, -5.0, 5.0, None))
    mix_q = tpe.adaptive_parzen_normal(np.round(rng.uniform(0, 100, 300)), 1.0, 50.0, 100.0)
    cand_q = np.concatenate([np.arange(0, 101, 1.0), [300.0, -400.0]])
    lp.append(("GMM1", mix_q, cand_q, 0.0, 100.0, 1.0))
    lp.append(("GMM1", mix_q, cand_q, None, None, 1.0))
    mix_q3 = tpe.adaptive_parzen_normal(np.round(rng.normal(0, 10, 100) / 2) * 2, 1.0, 0.0, 10.0)
    lp.append(("GMM1", mix_q3, np.arange(-40, 41, 2.0), None, None, 2.0))
    mix_l = tpe.adaptive_parzen_normal(rng.uniform(-5, 0, 300), 1.0, -2.5, 5.0)
    cand_l = np.concatenate([np.exp(rng.uniform(-5, 0, 400)), [np.exp(-5.0), 1.0, 1e-9, 30.0]])
    lp.append(("LGMM1", mix_l, cand_l, None, None, None))
    lp.append(("LGMM1", mix_l, cand_l, -5.0, 0.0, None))
    mix_ql = tpe.adaptive_parzen_normal(np.log(np.maximum(np.round(np.exp(rng.uniform(0, 3, 200)) / 2) * 2,
                                                          np.exp(0.0))), 1.0, 1.5, 3.0)
    lp.append(("LGMM1", mix_ql, np.arange(0, 24, 2.0), 0.0, 3.0, 2.0))
    mix_ql2 = tpe.adaptive_parzen_normal(np.log(np.maximum(np.round(np.exp(rng.normal(0, 1, 100)) / 0.5) * 0.5, 1e-12)), 1.0, 0.0, 1.0)
    lp.append(("LGMM1", mix_ql2, np.arange(0, 20, 0.5), None, None, 0.5))
    for i, (fam, (w, mu, sig), cand, lo, hi, q) in enumerate(lp):
        f = tpe.GMM1_lpdf if fam == "GMM1" else tpe.LGMM1_lpdf
        with np.errstate(all="ignore"):
            out = f(cand, w, mu, sig, low=lo, high=hi, q=q)
        arrays.update({"lpdf%d_w" % i: w, "lpdf%d_mu" % i: mu, "lpdf%d_sigma" % i: sig,
                       "lpdf%d_x" % i: cand, "lpdf%d_out" % i: np.asarray(out, float)})
        meta["lpdf"].append(dict(family=fam, low=lo, high=hi, q=q))

    # -- broadcast_best (tpe.py:649-658)
    bb = [
        (np.array([1.0, 2.0, 3.0]), np.array([0.0, 1.0, 1.0]), np.array([0.0, 0.0, 0.0])),
        (np.array([1.0, 2.0, 3.0]), np.array([0.0, np.nan, 1.0]), np.array([0.0, 0.0, 0.0])),
        (np.array([1.0, 2.0, 3.0, 4.0]), np.array([-np.inf, 0.0, -np.inf, 5.0]),
         np.array([-np.inf, 1.0, 0.0, 5.0])),
        (np.arange(6.0), np.array([1.0, 3.0, 3.0, 2.0, 3.0, 0.0]), np.zeros(6)),
    ]
    for i, (s, b, a) in enumerate(bb):
        with np.errstate(invalid="ignore"):
            out = ho.pyll.scope._impls["broadcast_best"](s, b, a)
        arrays.update({"best%d_s" % i: s, "best%d_b" % i: b, "best%d_a" % i: a,
                       "best%d_out" % i: np.asarray(out, float)})
        meta["best"].append({})

    # -- randint / categorical posteriors (tpe.py:578-615, pyll/base.py:1053-1060)
    pyll = ho.pyll
    cats = [
        ("randint", (10,), rng.randint(0, 10, 7)),
        ("randint", (10,), rng.randint(0, 10, 60)),  # > LF: ramp weights
        ("randint", (12, 25), rng.randint(12, 25, 90)),
        ("randint", (3,), np.zeros(0, int)),
        ("categorical", ([0.1, 0.3, 0.6],), rng.randint(0, 3, 45)),
        ("categorical", ([0.25, 0.25, 0.5],), np.array([2, 2, 0, 1, 2])),
    ]
    for i, (kind, args, obs) in enumerate(cats):
        fn = tpe.adaptive_parzen_samplers[kind]
        for pw in (1.0, 2.5):
            if kind == "randint":
                post = fn(pyll.as_apply(obs), pw, *args, size=5, rng=np.random.RandomState(0))
            else:
                post = fn(pyll.as_apply(obs), pw, pyll.as_apply(np.asarray(args[0])), size=5,
                          rng=np.random.RandomState(0))
            p = pyll.rec_eval(post.pos_args[0])
            arrays["cat%d_pw%g_p" % (i, pw)] = np.asarray(p, float)
        arrays["cat%d_obs" % i] = obs
        meta["cat"].append(dict(kind=kind, args=[list(a) if isinstance(a, list) else a for a in args]))

    save("units", arrays, meta)


# ---------------------------------------------------------------------------
# end-to-end: the reference's own posterior on its own candidates
# ---------------------------------------------------------------------------
def _flatten(x):
    if isinstance(x, dict):
        for k in sorted(x):
            yield from _flatten(x[k])
    elif isinstance(x, (list, tuple)):
        for v in x:
            yield from _flatten(v)
    else:
        yield x


def make_objective(seed, fail_every=0, round_to=None):
    rng = np.random.RandomState(seed)
    state = {"i": 0}

    def fn(point):
        state["i"] += 1
        leaves = [float(v) for v in _flatten(point)
                  if isinstance(v, (int, float, np.number)) and not isinstance(v, bool)]
        loss = float(np.sum(np.sin(1.3 * np.asarray(leaves)))) + 0.1 * rng.randn()
        if round_to is not None:
            loss = round(loss, round_to)
        if fail_every and state["i"] % fail_every == 0:
            return {"status": "fail"}
        return {"loss": loss, "status": "ok"}

    return fn


def capture_suggest(ho, domain, trials, seed, n_ei, prior_weight, gamma):
    """Evaluate the reference posterior graph (tpe.py:864-942) and capture every
    label's candidates, both log-likelihood vectors and both posteriors."""
    tpe, pyll = ho.tpe, ho.pyll
    observed, observed_loss, posterior = tpe.build_posterior_wrapper(domain, prior_weight, gamma)
    best_docs, best_loss = {}, {}
    for doc in trials.trials:  # tpe.py:876-890
        tid = doc["misc"].get("from_tid", doc["tid"])
        loss = doc["result"].get("loss")
        loss = float("inf") if loss is None else float(loss)
        best_loss.setdefault(tid, loss)
        if loss <= best_loss[tid]:
            best_loss[tid] = loss
            best_docs[tid] = doc
    tid_docs = sorted(best_docs.items())
    losses = [best_loss[t] for t, _ in tid_docs]
    tids, docs = list(zip(*tid_docs))
    first_new_id = max(tids) + 1
    fake0 = max(max(tids), first_new_id) + 2
    fake_ids = list(range(fake0, fake0 + n_ei))
    memo = {domain.s_new_ids: fake_ids, domain.s_rng: np.random.RandomState(seed),
            observed_loss["idxs"]: list(tids), observed_loss["vals"]: losses}
    oi, ov = ho.base.miscs_to_idxs_vals([d["misc"] for d in docs],
                                        keys=list(domain.params.keys()))
    memo[observed["idxs"]] = oi
    memo[observed["vals"]] = ov
    post_idxs, post_vals = posterior
    labels = sorted(post_vals)
    nodes = [post_idxs, post_vals]
    for lab in labels:
        bb = post_vals[lab]
        s, bl, al = bb.pos_args
        nodes.append([s, bl, al, list(bl.pos_args[1:4]), list(al.pos_args[1:4])])
    with np.errstate(all="ignore"):
        out = pyll.rec_eval(nodes, memo=memo, print_node_on_error=False)
    pidx, pval = out[0], out[1]
    res = {}
    for lab, (s, bl, al, bpar, apar) in zip(labels, out[2:]):
        s = np.asarray(s)
        r = dict(samples=s, below_llik=np.asarray(bl, float), above_llik=np.asarray(al, float),
                 below=[np.asarray(v, float) for v in bpar if np.ndim(v) >= 1],
                 above=[np.asarray(v, float) for v in apar if np.ndim(v) >= 1],
                 n=int(len(pidx[lab])))
        if s.size:
            with np.errstate(invalid="ignore"):
                best = int(np.argmax(r["below_llik"] - r["above_llik"]))
            assert list(pval[lab]) == [s[best]] * len(s)
            r["best"] = best
        res[lab] = r
    return res, tids, losses, oi, ov


E2E = [
    # name, space, T, n_ei, seed, gamma, prior_weight, fail_every, round_to, stable
    ("readme", "readme", 60, 24, 11, 0.25, 1.0, 0, None, False),
    ("readme_wide", "readme", 80, 512, 12, 0.25, 1.0, 7, None, False),
    ("uniform_1d", "uniform_1d", 2000, 4096, 13, 0.25, 1.0, 0, None, False),
    ("mixed_50d", "mixed_50d", 400, 256, 14, 0.25, 1.0, 0, None, True),
    ("many_dists", "many_dists", 200, 128, 15, 0.25, 1.0, 0, None, True),
    ("many_dists_pw", "many_dists", 120, 64, 16, 0.1, 2.5, 9, None, True),
    ("quniform_ties", "quniform_ties", 300, 128, 17, 0.25, 1.0, 0, 1, True),
    ("nested", "nested", 300, 64, 18, 0.25, 1.0, 11, None, True),
]


def gen_e2e(ho):
    for name, space_name, T, n_ei, seed, gamma, pw, fail_every, round_to, stable in E2E:
        space = SPACES.SPACES[space_name](ho.hp)
        trials = ho.Trials()
        ho.fmin(make_objective(seed, fail_every, round_to), space, algo=ho.rand.suggest,
                max_evals=T, trials=trials, rstate=np.random.RandomState(seed),
                show_progressbar=False)
        domain = ho.base.Domain(lambda x: x, space)
        with stable_argsort(stable):
            res, tids, losses, oi, ov = capture_suggest(ho, domain, trials, seed + 1000,
                                                        n_ei, pw, gamma)
        arrays = {"hist_tids": np.asarray(tids, np.int64),
                  "hist_losses": np.asarray(losses, float)}
        meta = dict(space=space_name, T=T, n_ei=n_ei, gamma=gamma, prior_weight=pw,
                    stable=stable, labels={}, numpy=np.__version__, specs={})
        for lab, node in domain.params.items():
            args = [np.asarray(ho.pyll.rec_eval(a)).tolist() for a in node.pos_args]
            kw = {k: np.asarray(ho.pyll.rec_eval(a)).tolist() for k, a in node.named_args}
            meta["specs"][lab] = dict(kind=node.name, args=args, kwargs=kw)
        for lab in sorted(oi):
            arrays["obs_idxs/" + lab] = np.asarray(oi[lab], np.int64)
            arrays["obs_vals/" + lab] = np.asarray(ov[lab], float)
        for lab, r in res.items():
            arrays["cand/" + lab] = r["samples"].astype(float)
            arrays["bl/" + lab] = r["below_llik"]
            arrays["al/" + lab] = r["above_llik"]
            for j, v in enumerate(r["below"]):
                arrays["bpost%d/%s" % (j, lab)] = v
            for j, v in enumerate(r["above"]):
                arrays["apost%d/%s" % (j, lab)] = v
            meta["labels"][lab] = dict(n=r["n"], best=r.get("best"),
                                       n_post=len(r["below"]))
        save("e2e_" + name, arrays, meta)


if __name__ == "__main__":
    ho = load_reference()
    gen_units(ho)
    gen_e2e(ho)
