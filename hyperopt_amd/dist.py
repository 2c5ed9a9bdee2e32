"""Multi-GPU partition of one suggest level and the cross-rank max-loc combine.

One process per GPU (torch.distributed; backend "nccl" is RCCL on ROCm).
A level's work is a set of (label, candidate range) units.  The labels of a
level are independent (build_posterior fits and scores each label alone,
tpe.py:697-746) and so are a label's candidates (i.i.d. rows of the N x M
score, tpe.py:153-158), so ``plan_units`` deals the level out as:

  * labels >= ranks: whole labels, balanced by a per-kind cost (label
    sharding: a rank fits, builds the tables of and scores only its own
    labels, so no per-label work is replicated);
  * labels <  ranks: every label split into c = ceil(ranks / labels)
    contiguous candidate ranges (candidate sharding, the C2 / C5 shapes).

Candidates are drawn with counter-based Philox keyed by the label and the
GLOBAL candidate index, so a unit's candidates do not depend on which rank
draws them or how many ranks there are.  The per-label winners are exchanged
once per level: every rank contributes an n_labels x 32-byte ``tpe_best``
array (index -1 where it scored nothing of that label), an all-gather moves
them (latency-bound: well under a microsecond of xGMI bandwidth), and
``tpe_best_combine`` applies np.argmax's rule (first max, NaN wins) on the
device.  Reference: the argmax of tpe.py:649-658 over all candidates.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib as L


def world():
    """(rank, world_size) if torch.distributed is initialised, else (0, 1)."""
    try:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            return dist.get_rank(), dist.get_world_size()
    except Exception:
        pass
    return 0, 1


SHARD_ALIGN = 4096  # one scorer tile (256 threads x 16 candidates)


def shard(n_total, rank, world_size):
    """Contiguous [start, start+count) share of n_total global candidate indices.

    Shares are rounded up to whole scorer tiles (SHARD_ALIGN candidates) when
    every rank gets at least one, else to multiples of 4 (one Philox call of
    the categorical sampler), so shard starts fall on tile / pair boundaries.
    The kernels give the same candidates at any start (odd ones included);
    alignment only keeps every rank on the fast paired-draw path."""
    per = (n_total + world_size - 1) // world_size
    a = SHARD_ALIGN if per >= SHARD_ALIGN else 4
    per = (per + a - 1) // a * a
    start = min(rank * per, n_total)
    return start, max(0, min(per, n_total - start))


# relative per-label cost of a level's kernels by kind (C3 group times at 2^22
# candidates per label: table build + score ~26 us, lattice ~19 us,
# categorical fit + score ~10 us per label)
UNIT_COST = {"table": 1.0, "quant": 0.75, "cat": 0.4}


def kind_class(kind):
    if kind in ("randint", "categorical"):
        return "cat"
    return "quant" if kind.startswith("q") else "table"


def plan_units(kinds, n_total, world_size):
    """Deal one level's labels (``kinds``: prior name per label) over
    ``world_size`` ranks.  Returns one list per rank of (label position,
    candidate start, candidate count) units; every candidate of every label
    is in exactly one unit.  Deterministic (every rank computes the same
    plan)."""
    n = len(kinds)
    ws = max(int(world_size), 1)
    out = [[] for _ in range(ws)]
    if n == 0:
        return out
    if ws == 1:
        out[0] = [(i, 0, n_total) for i in range(n)]
        return out
    if n >= ws:
        # longest-processing-time-first over whole labels; ties by label
        # position and rank so the plan is the same everywhere
        order = sorted(range(n), key=lambda i: (-UNIT_COST[kind_class(kinds[i])], i))
        load = [0.0] * ws
        for i in order:
            r = min(range(ws), key=lambda q: (load[q], q))
            load[r] += UNIT_COST[kind_class(kinds[i])]
            out[r].append((i, 0, n_total))
        for units in out:
            units.sort()
        return out
    c = (ws + n - 1) // n  # candidate shards per label
    r = 0
    for i in range(n):
        for j in range(c):
            start, count = shard(n_total, j, c)
            if count:
                out[r % ws].append((i, start, count))
            r += 1
    return out


def comm_ptr(group=None):
    """The ncclComm_t address behind torch's RCCL process group (for
    Engine.run(exchange=...)), or None (gloo, or a torch without the
    accessor): the level's cross-rank argmax then stays on the host path."""
    try:
        import torch
        import torch.distributed as dist
        if dist.get_backend(group) != "nccl":
            return None
        pg = group if group is not None else dist.distributed_c10d._get_default_group()
        be = pg._get_backend(torch.device("cuda", torch.cuda.current_device()))
        ptr = int(be._comm_ptr())
        return ptr or None
    except Exception:
        return None


def empty_records(n):
    rec = np.zeros(n, L.BEST_DTYPE)
    rec["index"] = -1
    return rec


def gather_best(n_labels, local, group=None):
    """Cross-rank winners of a level.  ``local``: list of (label position,
    LabelResult) this rank scored (several units of one label are folded
    first).  Returns n_labels (score, index, value, n_scored) tuples that are
    the same on every rank."""
    rec = empty_records(n_labels)
    for i, r in local:
        cur = rec[i]
        if better(r.score, r.index, cur["score"], cur["index"]):
            rec[i] = (r.score, r.index, r.value, cur["n_scored"] + r.n_scored)
        else:
            rec[i]["n_scored"] = cur["n_scored"] + r.n_scored
    rank, ws = world()
    if ws > 1:
        rec = _allgather_combine(rec, ws, group)
    return [(float(x["score"]), int(x["index"]), float(x["value"]), int(x["n_scored"]))
            for x in rec]


def _allgather_combine(rec, ws, group=None):
    import torch
    import torch.distributed as dist
    raw = rec.view(np.uint8)
    if dist.get_backend(group) == "nccl":
        dev = torch.device("cuda", torch.cuda.current_device())
        src = torch.from_numpy(raw.copy()).to(dev)
        gathered = torch.empty(ws * raw.size, dtype=torch.uint8, device=dev)
        dist.all_gather_into_tensor(gathered, src, group=group)
        return _combine_on_device(gathered, ws, rec.size, dev)
    src = torch.from_numpy(raw.copy())
    bufs = [torch.empty_like(src) for _ in range(ws)]
    dist.all_gather(bufs, src, group=group)
    return combine_host(np.stack([b.numpy() for b in bufs]))


def combine_device(sets, stream=None):
    """Combine ``sets`` ((n_sets, n_labels) BEST_DTYPE records, e.g. one row
    per rank) on the device with ``tpe_best_combine`` (np.argmax rules: first
    max, NaN wins; n_scored summed).  Returns (n_labels,) BEST_DTYPE."""
    import torch
    sets = np.ascontiguousarray(np.asarray(sets).view(L.BEST_DTYPE))
    if sets.ndim == 1:
        sets = sets[None]
    n_sets, n_labels = sets.shape
    dev = torch.device("cuda", torch.cuda.current_device())
    src = torch.from_numpy(sets.view(np.uint8).reshape(-1).copy()).to(dev)
    return _combine_on_device(src, n_sets, n_labels, dev, stream)


def _combine_on_device(src, n_sets, n_labels, dev, stream=None):
    import torch
    out = torch.empty(n_labels * L.BEST_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    st = stream if stream is not None else torch.cuda.current_stream(dev)
    L.check(L.load().tpe_best_combine(src.data_ptr(), n_sets, n_labels, out.data_ptr(),
                                      ctypes.c_void_p(st.cuda_stream)), "tpe_best_combine")
    with torch.cuda.stream(st):
        host = out.cpu().numpy()
    return host.view(L.BEST_DTYPE).copy()


def better(sa, ia, sb, ib):
    """np.argmax order on (score, index) pairs; index < 0 is empty."""
    if ib < 0:
        return ia >= 0
    if ia < 0:
        return False
    na, nb = sa != sa, sb != sb
    if na or nb:
        return ia < ib if (na and nb) else na
    if sa != sb:
        return sa > sb
    return ia < ib


def combine_host(records):
    """Combine gathered best records on the host (gloo / CPU tests only)."""
    sets = np.asarray(records).view(L.BEST_DTYPE)
    out = sets[0].copy()
    for s in sets[1:]:
        for k in range(out.size):
            owed = out["n_scored"][k] < 0 or s["n_scored"][k] < 0  # (an inexact record)
            out["n_scored"][k] = -1 if owed else out["n_scored"][k] + s["n_scored"][k]
            if better(s["score"][k], s["index"][k], out["score"][k], out["index"][k]):
                n = out["n_scored"][k]
                out[k] = s[k]
                out["n_scored"][k] = n
    return out


def allreduce_best(results, group=None):
    """Replace each LabelResult's winner by the global winner over all ranks
    (every rank scored a candidate range of every label)."""
    rank, ws = world()
    if ws == 1 or not results:
        return results
    rec = np.zeros(len(results), L.BEST_DTYPE)
    for k, r in enumerate(results):
        rec[k] = (r.score, r.index, r.value, r.n_scored)
    comb = _allgather_combine(rec, ws, group)
    for k, r in enumerate(results):
        r.score = float(comb["score"][k])
        r.index = int(comb["index"][k])
        r.value = float(comb["value"][k])
        r.n_scored = int(comb["n_scored"][k])
    return results


def settle_exchange(combined, local_exact, exchange):
    """The exact-argmax rule of a label-sharded level's exchange.  A rank
    whose band overflowed (more near-ties than its band tiles hold) sends its
    fp32 winner with n_scored = -1; the combine propagates the -1 (a label
    owed an exact decision), so ``combined`` -- the same records on every
    rank -- shows it to EVERY rank at once.  Then every rank, together and in
    the same order, runs ``exchange`` once more on ``local_exact()`` (its
    records after the exact re-score of its overflowed jobs): no rank leaves
    the level early, none takes the inexact winner, and a level without an
    overflow costs nothing extra.  ``exchange(records) -> combined records``
    is the collective (the engine's RCCL max-loc, or an all-gather + combine
    on gloo)."""
    if not (np.asarray(combined)["n_scored"] < 0).any():
        return combined
    exact = local_exact()
    if (np.asarray(exact)["n_scored"] < 0).any():
        raise L.TpeHipError("settle_exchange: a local record is still inexact")
    out = exchange(exact)
    if (np.asarray(out)["n_scored"] < 0).any():
        raise L.TpeHipError("settle_exchange: the second exchange is still inexact")
    return out

