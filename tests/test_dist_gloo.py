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
