"""Search spaces shared by the golden generator (reference hp) and the tests (our hp).

Each builder takes the `hp` module (and `scope`, for arithmetic helpers) so the
same space can be instantiated against /root/reference's hyperopt when fixtures
are generated and against ``hyperopt_amd`` when they are checked.
"""


def readme(hp):
    # README.md example space (config C1)
    return hp.choice("a", [("case 1", 1 + hp.lognormal("c1", 0, 1)),
                           ("case 2", hp.uniform("c2", -10, 10))])


def uniform_1d(hp):
    # config C2 (scaled down in the fixture)
    return {"x": hp.uniform("x", -5, 5)}


def mixed_50d(hp):
    # config C3 kinds: 10 x uniform/loguniform/quniform/normal/choice(8)
    sp = {}
    for i in range(10):
        sp["u%d" % i] = hp.uniform("u%d" % i, -5, 5)
        sp["lu%d" % i] = hp.loguniform("lu%d" % i, -5, 0)
        sp["qu%d" % i] = hp.quniform("qu%d" % i, 0, 100, 1)
        sp["n%d" % i] = hp.normal("n%d" % i, 0, 2)
        sp["c%d" % i] = hp.choice("c%d" % i, list(range(8)))
    return sp


def many_dists(hp):
    # every hp kind (reference tests/test_domains.py:160-175)
    return {
        "a": hp.choice("a", [0, 1, 2]),
        "b": hp.randint("b", 10),
        "bb": hp.randint("bb", 12, 25),
        "c": hp.uniform("c", 4, 7),
        "d": hp.loguniform("d", -2, 0),
        "e": hp.quniform("e", 0, 10, 3),
        "f": hp.qloguniform("f", 0, 3, 2),
        "g": hp.normal("g", 4, 7),
        "h": hp.lognormal("h", -2, 2),
        "i": hp.qnormal("i", 0, 10, 2),
        "j": hp.qlognormal("j", 0, 2, 1),
        "k": hp.pchoice("k", [(0.1, 0), (0.3, 1), (0.6, 2)]),
    }


def quniform_ties(hp):
    return {"q": hp.quniform("q", 0, 10, 1), "u": hp.uniform("u", 0, 1)}


def nested(hp):
    # three-level conditional space (config C5 shape, scaled down)
    return hp.choice("root", [
        {"kind": "lin", "lr": hp.loguniform("lin_lr", -7, 0)},
        {"kind": "tree",
         "depth": hp.quniform("tree_depth", 1, 12, 1),
         "split": hp.choice("tree_split", [
             {"crit": "gini", "w": hp.uniform("gini_w", 0, 1)},
             {"crit": "ent", "w": hp.normal("ent_w", 0, 1),
              "s": hp.qlognormal("ent_s", 0, 1, 0.5)},
         ])},
        {"kind": "nn", "units": hp.qloguniform("nn_units", 2, 7, 1),
         "drop": hp.uniform("nn_drop", 0, 0.7)},
    ])


SPACES = {
    "readme": readme,
    "uniform_1d": uniform_1d,
    "mixed_50d": mixed_50d,
    "many_dists": many_dists,
    "quniform_ties": quniform_ties,
    "nested": nested,
}
