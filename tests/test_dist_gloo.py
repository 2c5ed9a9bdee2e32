"""Multi-process (world_size 2, gloo on CPU) coverage of the cross-rank argmax
combine and candidate sharding used by tpe.suggest / bench.py at N > 1."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from hyperopt_amd import dist as hdist
from hyperopt_amd import _lib as L
from hyperopt_amd.engine import LabelResult


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # per-rank winners for 4 labels: rank 1 wins label 0 (score), ties on
    # label 1 (lower global index wins), NaN on label 2 wins, label 3 empty on
    # rank 0
    local = {
        0: [(1.0, 5, 0.1), (2.0, 7, 0.2), (3.0, 1, 0.3), (0.0, -1, 0.0)],
        1: [(4.0, 105, 1.1), (2.0, 3, 1.2), (float("nan"), 150, 1.3), (-1.0, 120, 1.4)],
    }[rank]
    res = [LabelResult("l%d" % k, i, v, s, 100) for k, (s, i, v) in enumerate(local)]
    hdist.allreduce_best(res)
    q.put((rank, [(r.score, r.index, r.value, r.n_scored) for r in res]))
    start, count = hdist.shard(1000, rank, world)
    q.put((rank, ("shard", start, count)))
    dist.destroy_process_group()


def test_allreduce_best_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(4)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    best = {r: v for r, v in out if not (isinstance(v, tuple) and v[0] == "shard")}
    shards = sorted(v[1:] for r, v in out if isinstance(v, tuple) and v[0] == "shard")
    assert shards == [(0, 500), (500, 500)]
    for r in (0, 1):
        b = best[r]
        assert b[0][:3] == (4.0, 105, 1.1)
        assert b[1][:3] == (2.0, 3, 1.2)
        assert np.isnan(b[2][0]) and b[2][1:3] == (150, 1.3)
        assert b[3][:3] == (-1.0, 120, 1.4)
        assert all(x[3] == 200 for x in b)


def test_better_matches_numpy_argmax():
    rng = np.random.RandomState(0)
    for _ in range(200):
        s = rng.choice([0.0, 1.0, 2.0, np.nan], size=7)
        best = -1
        for i, v in enumerate(s):
            if best < 0 or hdist.better(v, i, s[best], best):
                best = i
        with np.errstate(invalid="ignore"):
            assert best == int(np.argmax(s))


def test_shard_covers_range():
    for n in (0, 1, 7, 24, 1 << 20):
        for ws in (1, 2, 3, 8):
            parts = [hdist.shard(n, r, ws) for r in range(ws)]
            assert sum(c for _, c in parts) == n
            pos = 0
            for s, c in parts:
                if c:
                    assert s == pos
                pos += c


def test_combine_host_records():
    a = np.zeros(2, L.BEST_DTYPE)
    b = np.zeros(2, L.BEST_DTYPE)
    a[0] = (1.0, 4, 0.5, 10)
    b[0] = (1.0, 2, 0.7, 10)
    a[1] = (0.0, -1, 0.0, 0)
    b[1] = (-3.0, 9, 0.9, 10)
    out = hdist.combine_host(np.stack([a.view(np.uint8), b.view(np.uint8)]))
    assert out[0]["index"] == 2 and out[0]["n_scored"] == 20
    assert out[1]["index"] == 9


def _unit_worker(rank, world, port, q):
    """Label-sharded level: each rank 'scores' only its units (synthetic
    winners derived from the unit) and gather_best combines them."""
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    kinds = ["uniform", "randint", "quniform", "normal", "loguniform"]
    units = hdist.plan_units(kinds, 1000, world)[rank]
    local = []
    for i, start, count in units:
        # winner of a unit: global index start + (7 * i) % count, score by label;
        # label 1 is a NaN label whose first NaN must win
        idx = start + (7 * i) % count
        score = float("nan") if i == 1 else float(i)
        local.append((i, LabelResult("l%d" % i, idx, 0.5 * idx, score, count)))
    best = hdist.gather_best(len(kinds), local)
    q.put((rank, best))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gather_best_label_sharded_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_unit_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # every rank agrees, and each label's winner is its unit's (whole labels:
    # 5 labels >= ranks, so each label lives on one rank)
    for r in range(1, world):
        assert [tuple(np.nan_to_num(b)) for b in out[r]] == \
               [tuple(np.nan_to_num(b)) for b in out[0]]
    for i, (score, index, value, n) in enumerate(out[0]):
        assert n == 1000 and index == (7 * i) % 1000 and value == 0.5 * index
        assert (np.isnan(score) if i == 1 else score == float(i))


def test_plan_units_partition():
    kinds = ["uniform"] * 10 + ["loguniform"] * 10 + ["quniform"] * 10 + ["normal"] * 10 + \
            ["randint"] * 10
    for n_total in (1, 24, 4097, 1 << 22):
        for ws in (1, 2, 3, 4, 7, 8, 64):
            for ks in (kinds, kinds[:3], kinds[:1], []):
                plan = hdist.plan_units(ks, n_total, ws)
                assert len(plan) == ws
                assert plan == hdist.plan_units(ks, n_total, ws)  # deterministic
                cover = {}
                for units in plan:
                    for i, s, c in units:
                        cover.setdefault(i, []).append((s, c))
                assert sorted(cover) == list(range(len(ks)))
                for i, parts in cover.items():
                    parts.sort()
                    pos = 0
                    for s, c in parts:
                        assert s == pos and c > 0
                        pos += c
                    assert pos == n_total
    # C3 on 8 ranks: whole labels, the costliest rank within one table label
    # of the mean
    plan = hdist.plan_units(kinds, 1 << 22, 8)
    cost = [sum(hdist.UNIT_COST[hdist.kind_class(kinds[i])] for i, _, _ in u) for u in plan]
    mean = sum(cost) / 8
    assert max(cost) - mean <= 1.0
    assert all(c == 1 << 22 for u in plan for _, _, c in u)


def _empty_rank_worker(rank, world, port, q):
    """A one-label level with n_EI = 24 on 4 ranks: the plan leaves rank 3
    without units; it must still join the winners' all-gather
    (tpe.suggest skips the engine for it) so the other ranks do not hang."""
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    units = hdist.plan_units(["uniform"], 24, world)[rank]
    local = [(i, LabelResult("x", start + 1, 0.1 * (start + 1), float(start), count))
             for i, start, count in units]
    q.put((rank, len(units), hdist.gather_best(1, local)))
    dist.destroy_process_group()


def test_rank_without_units_joins_the_gather():
    world = 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_empty_rank_worker, args=(r, world, port, q))
             for r in range(world)]
    for p in procs:
        p.start()
    out = {r: (n, best) for r, n, best in (q.get(timeout=120) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [out[r][0] for r in range(world)] == [1, 1, 1, 0]
    for r in range(world):  # the highest-scoring shard (start 16) wins everywhere
        assert out[r][1] == [(16.0, 17, 0.1 * 17, 24)]


def _overflow_worker(rank, world, port, q):
    """a band overflow on ONE rank of a label-sharded level.  Rank
    1's first record for label 0 is its fp32 winner with n_scored = -1 (its
    band tiles overflowed; BAND_TILE_CAP shrunk to 0 gives exactly this on the
    GPU).  The combine shows the -1 to every rank, every rank settles with a
    second exchange of its exact records, and all end on the same exact
    winner -- no rank leaves early, nobody takes the inexact one."""
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    calls = [0]

    def exchange(rec):
        calls[0] += 1
        return hdist._allgather_combine(rec, world)

    first = hdist.empty_records(3)
    exact = hdist.empty_records(3)
    if rank == 0:
        first[0] = exact[0] = (2.0, 10, 0.5, 100)
        first[1] = exact[1] = (1.0, 11, 0.6, 100)
    else:
        first[0] = (2.5, 110, 1.5, -1)       # fp32 winner, owed an exact decision
        exact[0] = (1.9999, 117, 1.7, 100)   # the exact re-score picks another candidate
        first[1] = exact[1] = (0.5, 111, 1.6, 100)
        first[2] = exact[2] = (3.0, 112, 1.8, 100)
    combined = exchange(first)
    owed = bool(combined["n_scored"][0] < 0)
    settled = hdist.settle_exchange(combined, lambda: exact, exchange)
    # a level without an overflow settles at once (no second collective)
    clean = exchange(exact)
    n_before = calls[0]
    again = hdist.settle_exchange(clean, lambda: exact, exchange)
    q.put((rank, owed, settled.tolist(), again.tolist(), calls[0] - n_before))
    dist.destroy_process_group()


def test_band_overflow_on_one_rank_settles_everywhere():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_overflow_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {r: rest for r, *rest in (q.get(timeout=120) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        owed, settled, again, extra = out[r]
        assert owed  # every rank saw the -1
        assert settled == out[0][1]  # the same records everywhere
        assert settled[0][:3] == (2.0, 10, 0.5) and settled[0][3] == 200  # exact winner
        assert settled[1][:3] == (1.0, 11, 0.6) and settled[2][:3] == (3.0, 112, 1.8)
        assert again == settled and extra == 0
