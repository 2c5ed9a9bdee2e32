"""Round-4 diagnostics: the band tiles of one label (tile_cap shrunk), and the
tpe_table error-bound fields of C3-like labels."""
import numpy as np
import torch
import hyperopt_amd.engine as E
from hyperopt_amd import _lib as L
from oracle import tpe_oracle as O

T = 10_000
gens = {"uniform": ((-5.0, 5.0), lambda r, n: r.uniform(-5, 5, n)),
        "loguniform": ((-5.0, 0.0), lambda r, n: np.exp(r.uniform(-5, 0, n))),
        "normal": ((0.0, 2.0), lambda r, n: r.normal(0, 2, n)),
        "lognormal": ((0.0, 1.0), lambda r, n: np.exp(r.normal(0, 1, n)))}
for kind, (args, gen) in gens.items():
    rng = np.random.RandomState(41)
    obs = gen(rng, T)
    losses = rng.normal(size=T)
    below, above = O.ap_split_trials(np.arange(T), obs, np.arange(T), losses, 0.25)
    for cap in (64, 1):
        E.BAND_TILE_CAP = cap
        eng = E.Engine()
        w = E.LabelWork(kind, kind, args, below, above, n_cand=1 << 22, key=77)
        r, = eng.run([w], precision=32)
        ctl = eng._bufs["band_ctl"]
        n_t = 1024
        h = ctl[:16 * n_t].cpu().numpy().view(np.uint32).reshape(n_t, 4)
        lo = h[:, 0].view(np.float32)
        hi = h[:, 1].view(np.float32)
        n = h[:, 2]
        G = lo.max()
        rel = ~(hi < G)
        tab = eng._bufs["tables"][:L.TABLE_DTYPE.itemsize].cpu().numpy().view(L.TABLE_DTYPE)[0]
        print(kind, "cap", cap, "G", G, "relevant tiles", int(rel.sum()), "full", int((n == 0xFFFFFFFF).sum()),
              "full&rel", int(((n == 0xFFFFFFFF) & rel).sum()),
              "entries(rel)", int(n[rel & (n != 0xFFFFFFFF)].sum()), "n_scored", r.n_scored,
              "overflows", getattr(eng, "band_overflows", 0))
        print("   table: nb %d items %d ab %.3f eps_mix %.3e eps_cubic %.3e slope %.3e" % (
            tab["nb"], tab["build_items"], tab["build_ab"], tab["eps_mix"], tab["eps_cubic"],
            tab["slope"]), "stats", eng.last_table_stats)
E.BAND_TILE_CAP = 64
