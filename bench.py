#!/usr/bin/env python
"""Benchmark: EI candidates scored/sec for one TPE suggest step on config C3.

Workload (BASELINE.json configs[2]): a 50-dim mixed space
(10 x uniform(-5,5), 10 x loguniform(-5,0), 10 x quniform(0,100,1),
10 x normal(0,2), 10 x choice(8)), a 10k-trial history drawn from the prior
(seed 0) with N(0,1) losses (seed 1), and 2^22 EI candidates per label.  One
step = one full suggest level on the device path: the below/above split of the
resident columnar history, the Parzen fit of all mixtures, sampling 50 x 2^22
candidates from the below posteriors, scoring each under both posteriors, and
the per-label argmax (plus the cross-GPU max-loc combine when N > 1).

Scaling (``--scaling``): "strong" (default) keeps the job at 2^22 candidates
per label and splits it over the N ranks with hyperopt_amd.dist.plan_units
(whole labels per rank when labels >= ranks, the reference's label
independence, tpe.py:697-746); "weak" gives every rank 2^22 candidates per
label of its own global index range.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--scaling strong|weak]

With --gpus N > 1 and no torch.distributed environment (WORLD_SIZE unset)
the script launches itself as N ranks (torch.distributed.run, one process
per GPU) before touching the GPU, and prints rank 0's line.  Prints ONE JSON
line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import platform
import sys
import time

# kernel arguments in device memory: shorter launch-to-start latency for the
# ~20 launches of a level (a one-eighth label share: 0.318 -> 0.292 ms,
# DESIGN.md 6); read by the HIP runtime at initialisation, so before torch
os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

T_HIST = 10_000
N_CAND = 1 << 22
FP32_PEAK_TFLOPS = 157.3  # MI355X vector FP32 (MI355X_MICROARCH.md, chip table)
# VALU issue peak: 256 CUs x 4 SIMDs, one wave64 VALU instruction per 2 cycles
# per SIMD at 2.4 GHz (MI355X_MICROARCH.md: v_fma_f32 wave64 2 cycles)
VALU_ISSUE_PEAK = 1024 * 2.4e9 / 2
FLOPS_PER_PAIR = 9  # unquantized GMM1/LGMM1 pair
OPS_PER_TABLE_CAND = 56  # fast table scorer (score cubic per cell), per candidate
DIRECT_PAIR_CEILING = 9.81e12  # pairs/s of the exp-bound direct loop (profiles/r01_valu_microbench.txt)


def c3_space():
    kinds = []
    for i in range(10):
        kinds += [("u%d" % i, "uniform", (-5.0, 5.0)), ("lu%d" % i, "loguniform", (-5.0, 0.0)),
                  ("qu%d" % i, "quniform", (0.0, 100.0, 1.0)), ("n%d" % i, "normal", (0.0, 2.0)),
                  ("c%d" % i, "randint", (8,))]
    return kinds


def c3_history(space, T=T_HIST):
    """Prior draws (seed 0) and N(0,1) losses (seed 1): SURVEY.md §8(d) C3."""
    rng = np.random.RandomState(0)
    vals = {}
    for lab, kind, a in space:
        if kind == "uniform":
            v = rng.uniform(a[0], a[1], T)
        elif kind == "loguniform":
            v = np.exp(rng.uniform(a[0], a[1], T))
        elif kind == "quniform":
            v = np.round(rng.uniform(a[0], a[1], T) / a[2]) * a[2]
        elif kind == "normal":
            v = rng.normal(a[0], a[1], T)
        else:
            v = rng.randint(0, a[0], T).astype(np.float64)
        vals[lab] = v
    losses = np.random.RandomState(1).normal(size=T)
    return vals, losses


def split(vals, losses, gamma=0.25):
    """ap_split_trials for every label at once (tpe.py:623-646), columnar."""
    T = losses.size
    n_below = min(int(math.ceil(gamma * math.sqrt(T))), 25)
    order = np.argsort(losses, kind="stable")
    isb = np.zeros(T, bool)
    isb[order[:n_below]] = True
    return {lab: (v[isb], v[~isb]) for lab, v in vals.items()}


def c3_matrix(space, vals):
    """The history as a (T, labels) matrix in space order (all labels active)."""
    return np.stack([vals[lab] for lab, _, _ in space], axis=1)


def below_rows(losses, gamma=0.25):
    """Rows of the n_below best losses, ascending (ap_split_trials, tpe.py:623-646)."""
    from hyperopt_amd.tpe import _smallest_rows
    T = losses.size
    n_below = min(int(math.ceil(gamma * math.sqrt(T))), 25)
    return np.sort(_smallest_rows(losses, n_below))


def history_works(space, mat, hist, rows_b, step, n_cand, cand_base, units=None, n_total=0):
    """LabelWork list for the device-resident history: only the (small) below
    sets are read on the host; the above sets are gathered on the GPU.
    ``units`` (label position, start, count): this rank's share of the level
    (hyperopt_amd.dist.plan_units); default every label, n_cand candidates
    from cand_base."""
    from hyperopt_amd.engine import LabelWork
    below = mat[rows_b]
    n_above = (hist.n_active - hist.active_host[rows_b].sum(0)).tolist()
    keys = label_keys(0, step, [lab for lab, _, _ in space])
    if units is None:
        units = [(j, 0, n_cand) for j in range(len(space))]
    return [LabelWork(label=space[j][0], kind=space[j][1], args=space[j][2],
                      obs_below=below[:, j], obs_above=None, n_cand=count, key=keys[j],
                      cand_base=cand_base + start, col=j, n_above=n_above[j],
                      n_total=n_total or n_cand)
            for j, start, count in units]


def history_batch(space, mat, hist, rows_b, step, n_cand, cand_base, units, n_total):
    """The same level as history_works, as an engine.WorkBatch (the columnar
    form tpe.suggest uses): counts and keys as arrays, LabelWork objects only
    when the engine first sees the structure."""
    from hyperopt_amd.engine import WorkBatch
    nb = hist.active_host[rows_b].sum(0)
    na = hist.n_active - nb
    from hyperopt_amd.tpe import label_keys_array
    keys = label_keys_array(0 * 1000003 + step, space_labels(space))
    j = np.fromiter((u[0] for u in units), np.int64, len(units))
    return WorkBatch(("bench-c3", tuple(units), n_total), nb[j], na[j], keys[j],
                     [cand_base + u[1] for u in units],
                     lambda: history_works(space, mat, hist, rows_b, step, n_cand, cand_base,
                                           units, n_total))


def space_labels(space):
    """The space's labels as a tuple (label_keys_array caches their hashes by it)."""
    return tuple(lab for lab, _, _ in space)


def label_key(seed, step, lab):
    """Philox key of (seed, step, label): the drop-in's key rule (tpe.label_key)
    with the step folded into the seed."""
    from hyperopt_amd.tpe import label_key as key
    return key(seed * 1000003 + step, lab)


def label_keys(seed, step, labels):
    """label_key for a list of labels (vectorised, tpe.label_keys)."""
    from hyperopt_amd.tpe import label_keys as keys
    return keys(seed * 1000003 + step, labels)


def make_works(space, splits, step, n_cand, cand_base):
    from hyperopt_amd.engine import LabelWork
    return [LabelWork(label=lab, kind=kind, args=a, obs_below=splits[lab][0],
                      obs_above=splits[lab][1], n_cand=n_cand, key=label_key(0, step, lab),
                      cand_base=cand_base) for lab, kind, a in space]


def _cpu_label(task):
    """One label of the oracle pipeline (fit + sample + score + argmax);
    returns the candidates it scored.  Module-level so that spawned
    multiprocessing workers can import it."""
    from oracle import tpe_oracle as O
    kind, a, below, above, n, seed = task
    rng = np.random.RandomState(seed)
    if kind == "randint":
        pb = O.randint_posterior(below, 1.0, a[0])
        cand = rng.choice(a[0], size=n, p=pb)
        O.categorical_label_scores(kind, a, below, above, cand)
        return n
    fam, pmu, psig, tf, low, high, q = O.posterior_spec(kind, a)
    post_b = O.adaptive_parzen_normal(tf(below), 1.0, pmu, psig)
    samp = O.gmm1_sample if fam == "GMM1" else O.lgmm1_sample
    cand = samp(*post_b, low=low, high=high, q=q, rng=rng, size=n)
    with np.errstate(all="ignore"):
        O.continuous_label_scores(kind, a, below, above, cand)
    return n


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or platform.machine()


def cpu_baseline(space, vals, losses, n=20480, workers=64):
    """The oracle (numpy restatement of tpe.suggest's per-label pipeline,
    /root/reference/hyperopt/tpe.py:837-964) on a bounded sample of C3 --
    test infrastructure only, never on the product path.  Two variants
    (BASELINE.md "CPU-baseline plan"): one process over one label of each kind
    (numpy elementwise code is single-threaded), and label-parallel
    multiprocessing, one label per worker over every CPU this process may run
    on (os.sched_getaffinity), at most `workers` spawned processes (each holds
    a few hundred MB of numpy temporaries), timed after the workers have
    started."""
    import multiprocessing as mp
    sp = split(vals, losses)
    by_kind = {}
    for lab, kind, a in space:
        by_kind.setdefault(kind, []).append((lab, kind, a))
    picks = [v[0] for v in by_kind.values()]
    t0 = time.perf_counter()
    done = sum(_cpu_label((kind, a, sp[lab][0], sp[lab][1], n, 5)) for lab, kind, a in picks)
    dt1 = time.perf_counter() - t0
    ncpu = os.cpu_count() or 1
    try:
        allowed = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        allowed = ncpu
    nw = max(1, min(workers, allowed))
    order = [s for group in zip(*by_kind.values()) for s in group]  # kinds interleaved
    order = (order * ((nw + len(order) - 1) // len(order)))[:nw]  # one label per worker
    tasks = [(kind, a, sp[lab][0], sp[lab][1], n, 5 + i) for i, (lab, kind, a) in enumerate(order)]
    multi = None
    try:
        with mp.get_context("spawn").Pool(nw) as pool:
            pool.map(_cpu_label, [(t[0], t[1], t[2], t[3], 64, 0) for t in tasks])  # warm-up
            t0 = time.perf_counter()
            done_m = sum(pool.map(_cpu_label, tasks, chunksize=1))
            dtm = time.perf_counter() - t0
        multi = {"value": done_m / dtm, "cores": nw, "seconds": dtm,
                 "sample": "%d labels (kinds interleaved), one per worker, %d candidates each"
                           % (len(tasks), n)}
    except Exception as e:  # report, do not fail the bench line
        multi = {"error": repr(e)}
    return {"value": done / dt1, "unit": "EI candidates/s", "cores": 1, "kind": "port",
            "sample": "oracle/tpe_oracle.py numpy pipeline (fit+sample+score+argmax), 5 labels "
                      "(uniform, loguniform, quniform, normal, choice8) x %d candidates, 10k-trial "
                      "history, %.2f s" % (n, dt1),
            "cpu_model": _cpu_model(), "os_cpu_count": ncpu, "sched_affinity_cpus": allowed,
            "label_parallel": multi}


def append_steps(eng, space, mat, hist, losses, n_cand, units, steps=20, warmup=3):
    """The engine step with the history growing by one trial per step, as an
    fmin loop grows it: each step appends a trial (a prior draw, N(0,1) loss)
    to the HBM history, and the level merges it into the sorted orders
    (tpe_history_order), re-splits and re-fits -- so the incremental-sort
    cache is paid for inside the timed region.  p50 / mean per step."""
    import torch
    rng = np.random.RandomState(11)
    T0, n = mat.shape[0], warmup + steps
    big = np.empty((T0 + n, mat.shape[1]))
    big[:T0] = mat
    lo = np.empty(T0 + n)
    lo[:T0] = losses
    extra = [mat[i] for i in rng.randint(T0, size=n)]  # the new trials (prior draws)
    new_loss = rng.normal(size=n)
    times = []
    for k in range(n):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        T = T0 + k + 1
        big[T - 1] = extra[k]
        lo[T - 1] = new_loss[k]
        hist.append(big[T - 1:T])
        rb = below_rows(lo[:T])
        isb = np.zeros(T, np.uint8)
        isb[rb] = 1
        works = history_batch(space, big[:T], hist, rb, 5000 + k, n_cand, 0, units, n_cand)
        eng.run(works, precision=32, history=hist, is_below=isb)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    t = np.array(times[warmup:]) * 1e3
    return {"p50_ms": float(np.median(t)), "mean_ms": float(t.mean()), "steps": int(t.size),
            "config": "C3 engine step, history + 1 trial per step (append, sorted-order merge, "
                      "split, fit, score)"}


def readme_suggest_p50():
    """Config C1 (BASELINE configs[0]): the README space, fmin(max_evals=100,
    n_EI_candidates=24, rstate=RandomState(3)) through the drop-in API; p50 of
    the wall time of TPE suggest calls 21-100 (calls 1-20 are the random
    startup)."""
    from hyperopt_amd import Trials, fmin, hp, tpe
    times = []

    def timed(new_ids, domain, trials, seed):
        t0 = time.perf_counter()
        out = tpe.suggest(new_ids, domain, trials, seed, verbose=False)
        times.append(time.perf_counter() - t0)
        return out

    space = hp.choice("a", [("case 1", 1 + hp.lognormal("c1", 0, 1)),
                            ("case 2", hp.uniform("c2", -10, 10))])

    def objective(args):
        case, val = args
        return val if case == "case 1" else val ** 2

    fmin(objective, space, algo=timed, max_evals=100, trials=Trials(),
         rstate=np.random.RandomState(3), show_progressbar=False)
    t = np.array(times[20:]) * 1e3
    return {"p50_ms": float(np.median(t)), "p90_ms": float(np.percentile(t, 90)),
            "calls": int(t.size), "config": "README space, max_evals=100, n_EI=24"}


class ForeignTrials(object):
    """A trials object shaped like the reference's ``hyperopt.Trials``
    (base.py:252-698: ``_dynamic_trials``, ``refresh`` filtering to the valid
    states, ``trials``, ``new_trial_docs``) without this package's
    ``columnar()`` -- what ``hyperopt.fmin(..., algo=hyperopt_amd.tpe.suggest)``
    hands the suggest (the reference itself is not on the GPU box)."""

    def __init__(self):
        self._dynamic_trials = []
        self.refresh()

    def refresh(self):
        from hyperopt_amd.base import JOB_VALID_STATES
        self._trials = [t for t in self._dynamic_trials if t["state"] in JOB_VALID_STATES]

    @property
    def trials(self):
        return self._trials

    def __len__(self):
        return len(self._trials)

    def insert_trial_docs(self, docs):
        self._dynamic_trials.extend(docs)
        return [d["tid"] for d in docs]

    def new_trial_docs(self, tids, specs, results, miscs):
        return [{"state": 0, "tid": tid, "spec": spec, "result": result, "misc": misc,
                 "exp_key": None, "owner": None, "version": 0, "book_time": None,
                 "refresh_time": None}
                for tid, spec, result, misc in zip(tids, specs, results, miscs)]


def c3_trials(space, vals, losses, foreign=False):
    """The C3 history as a drop-in ``Trials`` of T finished documents (and its
    Domain), in the reference's document format (base.py:459-482);
    ``foreign``: in a ForeignTrials instead."""
    from hyperopt_amd import Trials, hp
    from hyperopt_amd.base import JOB_STATE_DONE, Domain
    hps = {lab: (hp.randint(lab, a[0]) if kind == "randint" else getattr(hp, kind)(lab, *a))
           for lab, kind, a in space}
    domain = Domain(lambda p: 0.0, hps)
    trials = ForeignTrials() if foreign else Trials()
    T = losses.size
    ints = {lab for lab, kind, _ in space if kind == "randint"}
    cols = {lab: (vals[lab].astype(np.int64).tolist() if lab in ints else vals[lab].tolist())
            for lab, _, _ in space}
    miscs = [{"tid": i, "cmd": domain.cmd, "workdir": None,
              "idxs": {lab: [i] for lab in cols}, "vals": {lab: [cols[lab][i]] for lab in cols}}
             for i in range(T)]
    docs = trials.new_trial_docs(list(range(T)), [None] * T,
                                 [{"status": "ok", "loss": float(x)} for x in losses], miscs)
    for d in docs:
        d["state"] = JOB_STATE_DONE
    trials.insert_trial_docs(docs)
    trials.refresh()
    return domain, trials


def dropin_suggest_p50(space, vals, losses, n_cand, calls=20, warmup=3, foreign=False):
    """suggest p50 through the drop-in API on C3: ``tpe.suggest(new_ids,
    domain, trials, seed, n_EI_candidates=n_cand)`` on the 10k-document Trials
    (per-tid history, split, HBM mirror of the columnar cache appended with the
    previous call's document, every level's kernels, the returned document).
    Each call's document is completed with a loss and inserted, as fmin does.
    ``foreign``: the same on a reference-shaped ForeignTrials (no columnar(),
    the cache kept beside it: base.foreign_columnar)."""
    from hyperopt_amd import tpe
    from hyperopt_amd.base import JOB_STATE_DONE
    domain, trials = c3_trials(space, vals, losses, foreign=foreign)
    rng = np.random.RandomState(9)
    times = []
    for k in range(warmup + calls):
        tid = losses.size + k
        t0 = time.perf_counter()
        docs = tpe.suggest([tid], domain, trials, k, n_EI_candidates=n_cand, verbose=False)
        times.append(time.perf_counter() - t0)
        docs[0]["state"] = JOB_STATE_DONE
        docs[0]["result"] = {"status": "ok", "loss": float(rng.normal())}
        trials.insert_trial_docs(docs)
        trials.refresh()
    t = np.array(times[warmup:]) * 1e3
    return {"p50_ms": float(np.median(t)), "p90_ms": float(np.percentile(t, 90)),
            "calls": int(t.size),
            "config": "C3 through tpe.suggest: %d-document %s, n_EI_candidates=2^%d"
                      % (losses.size, "reference-shaped Trials (no columnar())" if foreign
                         else "Trials", int(round(math.log2(n_cand))))}


def valu_issue(prof, n_launch_cand):
    """VALU-issue roofline of the dominant kernel from its PMC pass
    (profiles/traffic.json, tools/make_traffic.py): wave-level VALU
    instructions per candidate (one lane's worth), measured cycles per VALU
    instruction (SQ_ACTIVE_INST_VALU x 4 / SQ_INSTS_VALU), and the fraction of
    the plain-VALU issue rate the kernel reaches: the time its instructions
    would take at 2 cycles each (v_fma_f32 wave64 on a SIMD-32,
    MI355X_MICROARCH.md) on all 1024 SIMDs, over its measured duration."""
    insts = prof.get("valu_insts_per_launch")
    cand = prof.get("candidates_per_launch") or n_launch_cand
    if not insts or not cand:
        return None
    out = {"insts_per_candidate": insts * 64.0 / cand}
    if prof.get("active_inst_valu"):
        out["cycles_per_inst"] = prof["active_inst_valu"] * 4.0 / insts
    if prof.get("grbm_gui_active"):
        out["issue_frac"] = 2.0 * insts / 1024.0 / (prof["grbm_gui_active"] / 8.0)
    out["source"] = prof.get("source")
    return out


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def self_launch(n):
    """--gpus N without a torch.distributed environment: run this script as N
    ranks under torch.distributed.run (a child process; this process never
    touches the GPU), pass rank 0's JSON line through, exit with its code."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node",
           str(n), "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def drawn_per_step(eng, space, units):
    """Candidates this rank drew in its last level: every candidate of a
    table unit; of a quantized or categorical unit, eng.lat_prefix when the
    prefix-first argmax settled it (need flag 0: tpe_lattice_suggest,
    tpe_categorical_suggest), else all."""
    prefix = eng.lat_prefix
    drawn = 0
    for kinds, buf_name in ((lambda k: k.startswith("q"), "lat_need"),
                            (lambda k: k in ("randint", "categorical"), "cat_need")):
        cnt = [c for j, _, c in units if kinds(space[j][1])]
        buf = eng._bufs.get(buf_name)
        if not cnt or buf is None or not prefix or max(cnt) <= prefix:
            drawn += sum(cnt)
            continue
        need = buf[:4 * len(cnt)].cpu().numpy().view(np.int32)
        drawn += sum(c if (n or c <= prefix) else prefix for c, n in zip(cnt, need.tolist()))
    drawn += sum(c for j, _, c in units
                 if not space[j][1].startswith("q") and space[j][1] not in ("randint", "categorical"))
    return drawn


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--precision", type=int, default=32)
    ap.add_argument("--n-cand", type=int, default=N_CAND)
    ap.add_argument("--scaling", default="strong", choices=("strong", "weak"),
                    help="strong: 2^22 candidates per label in total, split over the ranks by "
                         "dist.plan_units; weak: 2^22 per label per rank")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the fp64 line and the drop-in / README suggest timings")
    ap.add_argument("--upload-history", action="store_true",
                    help="pack and upload the observation lists every step instead of gathering "
                         "them from the HBM-resident history")
    ap.add_argument("--dense", action="store_true",
                    help="score with the dense fp32 kernel (same as --scorer dense)")
    ap.add_argument("--timer-every", type=int, default=4,
                    help="time the dominant kernel with HIP events on every k-th timed step")
    ap.add_argument("--scorer", default="auto", choices=("auto", "dense", "sorted", "table"),
                    help="fp32 kernel for the unquantized labels (engine.Engine.run)")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(self_launch(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print("bench.py: WORLD_SIZE=%d but --gpus %d" % (world, args.gpus), file=sys.stderr)
        sys.exit(2)

    import torch
    import torch.distributed as dist
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # BENCH_DIST_BACKEND=gloo rehearses the multi-rank path on one GPU (ranks
    # share cuda:0; the winners are combined on the host) -- never for numbers
    backend = os.environ.get("BENCH_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    from hyperopt_amd.engine import DeviceHistory, Engine, LabelResult
    from hyperopt_amd import dist as hdist

    scorer = "dense" if args.dense else args.scorer
    space = c3_space()
    vals, losses = c3_history(space)
    eng = Engine()
    n_cand = args.n_cand
    strong = args.scaling == "strong"
    if strong:  # this rank's units of the level (whole labels at 50 labels >= ranks)
        units = hdist.plan_units([k for _, k, _ in space], n_cand, world)[rank]
        cand_base = 0
    else:  # every label, 2^22 candidates of this rank's own global range
        units = [(j, 0, n_cand) for j in range(len(space))]
        cand_base = rank * n_cand
    # the history is resident in HBM before timing starts (appended once, as
    # trials would be); each step uploads only the below-row flags
    mat = c3_matrix(space, vals)
    hist = DeviceHistory(eng, len(space), cap=T_HIST)
    hist.append(mat)

    # label-sharded levels on RCCL: the per-label argmax all-reduce runs inside
    # the level, on its stream (tpe_best_scatter + tpe_maxloc_allreduce on
    # torch's communicator), read back with the level's results
    xcomm = hdist.comm_ptr() if (world > 1 and strong) else None
    xchg = (xcomm, len(space), world, [u[0] for u in units]) if xcomm else None

    def step(k, timers=None, timer_groups=None, precision=None):
        prec = precision or args.precision
        if args.upload_history:
            works = make_works(space, split(vals, losses), k, n_cand, cand_base)
            works = [works[j] for j, _, _ in units]
            for w, (_, start, count) in zip(works, units):
                w.n_cand, w.cand_base, w.n_total = count, cand_base + start, n_cand
            res = eng.run(works, precision=prec, timers=timers, scorer=scorer,
                          timer_groups=timer_groups)
        else:
            rb = below_rows(losses)
            isb = np.zeros(T_HIST, np.uint8)
            isb[rb] = 1
            works = history_batch(space, mat, hist, rb, k, n_cand, cand_base, units, n_cand)
            res = eng.run(works, precision=prec, timers=timers, scorer=scorer,
                          history=hist, is_below=isb, timer_groups=timer_groups, exchange=xchg)
        if world > 1:
            if strong and xchg is not None and not args.upload_history:
                pass  # every rank already holds every label's winner (eng.last_exchange)
            elif strong:  # label-sharded level: every rank learns every label's winner
                hdist.gather_best(len(space), list(zip([u[0] for u in units], as_results(res))))
            else:
                hdist.allreduce_best(as_results(res))
        return works, res

    def as_results(res):
        """LabelResults of a level (a WorkBatch level returns columns)."""
        if isinstance(res, list):
            return res
        return [LabelResult(space[u[0]][0], ix, v, sc, ns) for u, ix, v, sc, ns in
                zip(units, res.index.tolist(), res.value.tolist(), res.score.tolist(),
                    res.n_scored.tolist())]

    xnote = "inside the level" if xchg else "(host path)"
    if xchg is not None:
        # first level: the in-level exchange checked against the host path
        # (torch all-gather + host fold); every rank must agree to keep it
        try:
            _, res0 = step(0)
            got = [(float(x["score"]), int(x["index"]), float(x["value"]), int(x["n_scored"]))
                   for x in eng.last_exchange]
            ok = got == hdist.gather_best(len(space), [(u[0], r) for u, r in
                                                       zip(units, as_results(res0))])
        except Exception as e:  # noqa: BLE001 -- reported in the JSON line
            ok, xnote = False, "(host path: in-level exchange failed: %r)" % (e,)
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device="cuda")
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        if not int(flag.item()):
            xchg = None
            if ok:
                xnote = "(host path: in-level exchange disagreed on some rank)"
            elif "failed" not in xnote:
                xnote = "(host path: in-level exchange disagreed with the host fold)"
    group = {"dense": "cont", "sorted": "sorted"}.get(scorer, "table")
    every = max(1, args.timer_every)
    for k in range(args.warmup):
        step(k)
    if every > 1:  # the timed variant of the level recorded before timing starts
        for k in range(2):
            step(args.warmup + k, {}, {group})
    if eng.graphs:  # (TPE_DIAG=1 TPE_GRAPHS=1) the level's hipGraph captured before timing
        for k in range(2):
            step(args.warmup + 2 + k)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    # the dominant kernel group is timed with HIP events on its own stream inside
    # the timed region; the other groups only in an untimed pass afterwards
    # (every event pair adds a ~10 us timestamp barrier to the stream)
    timers = {}
    step_times = []
    barrier()
    t_start = time.perf_counter()
    for k in range(args.steps):
        t0 = time.perf_counter()
        # HIP events around the dominant kernel on every `every`-th step
        # (each event pair is a timestamp barrier on its stream)
        works, res = step(args.warmup + k, timers if k % every == 0 else None, {group})
        step_times.append(time.perf_counter() - t0)
    barrier()
    elapsed = time.perf_counter() - t_start
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # dominant kernel: unquantized continuous scoring of this rank's continuous labels
    if not isinstance(works, list):
        works = works.materialize()
    cont = [w for w in works if w.kind in ("uniform", "loguniform", "normal", "lognormal")]
    dense_pairs = sum(w.n_cand * (w.obs_below.size + 1 + (w.n_above if w.obs_above is None
                                                          else w.obs_above.size) + 1)
                      for w in cont)
    n_cont = sum(w.n_cand for w in cont)
    kname = {"cont": "k_score32 (tpe_score_continuous)",
             "sorted": "k_score_sorted (tpe_score_sorted)",
             "table": "k_score_table_fast (tpe_score_table_fast)"}[group]
    kms = [e0.elapsed_time(e1) for e0, e1 in timers.get(group, [])]
    avg_ms = float(np.mean(kms)) if kms else float("nan")
    sec = avg_ms * 1e-3
    if group == "table":
        # builder-defined operations per candidate of the
        # fast table scorer (sample + cell lookup + score cubic + argmax)
        ops = OPS_PER_TABLE_CAND * n_cont
        work = {"ops_per_candidate": OPS_PER_TABLE_CAND, "candidates_per_launch": n_cont}
    else:
        exec_pairs = dense_pairs if group == "cont" else (eng.last_pairs or dense_pairs)
        ops = exec_pairs * FLOPS_PER_PAIR
        work = {"flops_per_pair": FLOPS_PER_PAIR, "evaluated_pairs_per_launch": exec_pairs}
    builder_tflops = ops / sec / 1e12 if sec > 0 else float("nan")
    all_timers = {}
    for k in range(3):
        step(args.warmup + args.steps + k, all_timers)
    torch.cuda.synchronize()
    group_ms = {k: round(float(np.mean([a.elapsed_time(b) for a, b in v])), 4)
                for k, v in all_timers.items()}

    per_rank = sum(c for _, _, c in units)
    total_cand = (len(space) * n_cand if strong else per_rank * world) * args.steps
    # candidates actually drawn: a quantized label's prefix-first lattice
    # argmax (tpe_lattice_suggest) decides most labels from the first
    # eng.lat_prefix draws of its stream (exact by construction);
    # the per-job "need" flags of the last level say which labels drew it all
    drawn = drawn_per_step(eng, space, units)
    if world > 1:
        t = torch.tensor([float(drawn)], dtype=torch.float64, device="cuda")
        dist.all_reduce(t)
        drawn = int(t.item())
    # the headline counts candidates actually drawn and scored (VERDICT r03
    # weak #2); the decided count (every label's full 2^22-candidate argmax,
    # settled from a prefix for the quantized / categorical labels) is reported
    # beside it as value_decided
    value = drawn * args.steps / elapsed
    # per-launch HBM bytes / VALU figures of the dominant kernel, from the PMC
    # passes of tools/profile_round.sh (tools/make_traffic.py)
    traffic, prof = None, {}
    tfile = os.path.join(HERE, "profiles", "traffic.json")
    if os.path.exists(tfile):
        prof = json.load(open(tfile))
        if not (prof.get("kernel") and prof["kernel"] in kname and
                prof.get("candidates_per_launch") in (None, n_cont)):
            prof = {}  # another kernel or another workload: not this launch's counters
        traffic = prof.get("bytes_per_launch")
    issue = valu_issue(prof, n_cont) if prof else None
    dense_ps = dense_pairs / sec if sec > 0 else None
    roofline = {"kernel": kname, "avg_launch_ms": avg_ms, "timed_launches": len(kms),
                "traffic": traffic, "traffic_source": prof.get("source"),
                "valu_busy": prof.get("valu_busy"), "valu_issue": issue,
                # SURVEY 8(d)'s count: the (candidate, component) pairs the
                # reference evaluates at 9 flop each -- the table scorer does not
                # evaluate them (one cubic per cell), so this rate is reported, not
                # held against the FP32 peak
                "dense_equivalent": {"pairs_per_launch": dense_pairs, "pairs_per_s": dense_ps,
                                     "tflops_at_9_flop_per_pair":
                                         dense_ps * FLOPS_PER_PAIR / 1e12 if dense_ps else None,
                                     "direct_pair_ceiling_per_s": DIRECT_PAIR_CEILING},
                "builder_ops": dict(work, achieved_tflops=builder_tflops,
                                    peak_tflops=FP32_PEAK_TFLOPS,
                                    frac=builder_tflops / FP32_PEAK_TFLOPS)}
    if issue and prof.get("valu_insts_per_launch") and sec > 0:
        # VALU issue efficiency: the dominant kernel's VALU wave-instructions
        # per launch (PMC SQ_INSTS_VALU) over its live launch time, against one
        # wave64 VALU instruction per 2 cycles on every SIMD
        ach = prof["valu_insts_per_launch"] / sec
        roofline.update({"bound": "valu-issue", "achieved": ach, "peak": VALU_ISSUE_PEAK,
                         "unit": "VALU wave-instructions/s", "frac": ach / VALU_ISSUE_PEAK})
    else:  # no PMC figures for this workload: the builder's operation count
        roofline.update({"bound": "valu", "achieved": builder_tflops, "peak": FP32_PEAK_TFLOPS,
                         "unit": "TFLOP/s (builder-defined ops per candidate, DESIGN.md 3.1)",
                         "frac": builder_tflops / FP32_PEAK_TFLOPS})
    if group == "table":
        roofline["l2_gather_bytes_per_launch"] = 16 * n_cont  # one 16-B score cubic per candidate
        roofline["build_ms"] = group_ms.get("table_build")
        roofline["band_rescore_ms"] = group_ms.get("band")
    line = {
        "metric": "EI candidates scored/sec (50-dim, 10k trials)",
        "value": value,
        "unit": "EI candidates/s",
        "value_note": "candidates drawn and scored per second (value_decided: every "
                      "label's full candidate count, prefix-settled labels included)",
        "candidates_drawn_per_step": drawn,
        "candidates_decided_per_step": total_cand // args.steps,
        "value_decided": total_cand / elapsed,
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "engine_step_p50_ms": float(np.median(step_times)) * 1e3,
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "f32" if args.precision == 32 else "f64",
        "data": "synthetic: prior draws (seed 0), N(0,1) losses (seed 1), Philox candidates",
        "config": {"workload": "C3: 50-dim mixed (10x uniform/loguniform/quniform/normal/"
                               "choice8), 10k-trial history, 2^%d EI candidates per label%s"
                               % (int(round(math.log2(n_cand))),
                                  "" if strong else " per GPU"),
                   "labels": len(space), "history": T_HIST, "candidates_per_label": n_cand,
                   "parallelism": ("label-sharded x%d (dist.plan_units), RCCL all-gather + "
                                   "device max-loc %s" % (world, xnote)) if strong else
                                  ("candidate-sharded x%d, RCCL max-loc combine" % world),
                   "rank0_units": len(units)},
        "roofline": roofline,
        "group_ms": group_ms,
        "launch": dict(eng.graph_stats),
    }
    if rank == 0 and world == 1 and not args.no_extras:
        if args.precision == 32:  # the fp64 parity mode's throughput on the same workload
            step(0, precision=64)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(2):
                step(1000 + k, precision=64)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / 2
            line["fp64"] = {"value": len(space) * n_cand / dt, "ms_per_step": dt * 1e3,
                            "steps": 2, "dtype": "f64",
                            "note": "exact fp64 scoring of every label: component-pruned "
                                    "k_score_pruned64 for the 10k-component above mixtures "
                                    "(e^-40 margin), dense k_score64 for smaller ones"}
        line["append_step"] = append_steps(eng, space, mat, hist, losses, n_cand, units)
        line["dropin_suggest"] = dropin_suggest_p50(space, vals, losses, n_cand)
        line["dropin_suggest_foreign"] = dropin_suggest_p50(space, vals, losses, n_cand,
                                                            foreign=True)
        line["readme_suggest"] = readme_suggest_p50()
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(space, vals, losses)
    elif rank == 0:
        line["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
