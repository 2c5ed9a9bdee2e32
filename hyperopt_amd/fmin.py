"""fmin driver (hyperopt/fmin.py): the caller of ``algo`` (tpe.suggest).

Same control flow as the reference: FMinIter.run asks ``algo(new_ids,
domain, trials, rstate.randint(2**31 - 1))`` for new trial documents
(fmin.py:262-270), inserts them, evaluates them serially (fmin.py:158-187)
and repeats until max_evals / timeout / loss_threshold / early stop.
"""
from __future__ import annotations

import functools
import logging
import os
import sys
import time
from contextlib import contextmanager
from timeit import default_timer as timer

import numpy as np

from . import base, pyll

logger = logging.getLogger(__name__)


def generate_trial(tid, space):
    variables = space.keys()
    return {"state": base.JOB_STATE_NEW, "tid": tid, "spec": None, "result": {"status": "new"},
            "misc": {"tid": tid, "cmd": ("domain_attachment", "FMinIter_Domain"),
                     "workdir": None, "idxs": {v: [tid] for v in variables},
                     "vals": {k: [v] for k, v in space.items()}},
            "exp_key": None, "owner": None, "version": 0, "book_time": None,
            "refresh_time": None}


def generate_trials_to_calculate(points):
    """Trials pre-filled with points to evaluate before optimisation (fmin.py:60-76)."""
    trials = base.Trials()
    trials.insert_trial_docs([generate_trial(tid, x) for tid, x in enumerate(points)])
    return trials


def fmin_pass_expr_memo_ctrl(f):
    f.fmin_pass_expr_memo_ctrl = True
    return f


def partial(fn, **kwargs):
    rval = functools.partial(fn, **kwargs)
    if hasattr(fn, "fmin_pass_expr_memo_ctrl"):
        rval.fmin_pass_expr_memo_ctrl = fn.fmin_pass_expr_memo_ctrl
    return rval


class _NoProgress(object):
    postfix = ""

    def update(self, n):
        pass


@contextmanager
def no_progress_callback(initial, total):
    yield _NoProgress()


@contextmanager
def default_callback(initial, total):
    try:
        from tqdm import tqdm
    except ImportError:  # pragma: no cover
        yield _NoProgress()
        return
    with tqdm(total=total, initial=initial, postfix={"best loss": "?"}, disable=False,
              dynamic_ncols=True, unit="trial", file=sys.stdout) as pbar:
        class _P(object):
            @property
            def postfix(self):
                return pbar.postfix

            @postfix.setter
            def postfix(self, v):
                pbar.postfix = v

            def update(self, n):
                pbar.update(n)

        yield _P()


class FMinIter(object):
    """Sequential search loop (fmin.py:103-354)."""

    catch_eval_exceptions = False
    pickle_protocol = -1

    def __init__(self, algo, domain, trials, rstate, asynchronous=None, max_queue_len=1,
                 poll_interval_secs=1.0, max_evals=sys.maxsize, timeout=None,
                 loss_threshold=None, verbose=False, show_progressbar=True, early_stop_fn=None):
        self.algo = algo
        self.domain = domain
        self.trials = trials
        if not show_progressbar or not verbose:
            self.progress_callback = no_progress_callback
        elif show_progressbar is True:
            self.progress_callback = default_callback
        else:
            self.progress_callback = show_progressbar
        self.asynchronous = trials.asynchronous if asynchronous is None else asynchronous
        self.poll_interval_secs = poll_interval_secs
        self.max_queue_len = max_queue_len
        self.max_evals = max_evals
        self.early_stop_fn = early_stop_fn
        self.early_stop_args = []
        self.timeout = timeout
        self.loss_threshold = loss_threshold
        self.start_time = timer()
        self.rstate = rstate
        self.verbose = verbose
        if self.asynchronous:
            import pickle
            trials.attachments["FMinIter_Domain"] = pickle.dumps(domain)

    def serial_evaluate(self, N=-1):
        for trial in self.trials._dynamic_trials:
            if trial["state"] == base.JOB_STATE_NEW:
                trial["state"] = base.JOB_STATE_RUNNING
                now = base.coarse_utcnow()
                trial["book_time"] = now
                trial["refresh_time"] = now
                spec = base.spec_from_misc(trial["misc"])
                ctrl = base.Ctrl(self.trials, current_trial=trial)
                try:
                    result = self.domain.evaluate(spec, ctrl)
                except Exception as e:
                    logger.error("job exception: %s" % str(e))
                    trial["state"] = base.JOB_STATE_ERROR
                    trial["misc"]["error"] = (str(type(e)), str(e))
                    trial["refresh_time"] = base.coarse_utcnow()
                    if not self.catch_eval_exceptions:
                        self.trials.refresh()
                        raise
                else:
                    trial["state"] = base.JOB_STATE_DONE
                    trial["result"] = result
                    trial["refresh_time"] = base.coarse_utcnow()
                N -= 1
                if N == 0:
                    break
        self.trials.refresh()

    @property
    def is_cancelled(self):
        return bool(getattr(self.trials, "_fmin_cancelled", False))

    def block_until_done(self):
        if self.asynchronous:
            unfinished = [base.JOB_STATE_NEW, base.JOB_STATE_RUNNING]
            while self.trials.count_by_state_unsynced(unfinished) > 0:
                time.sleep(self.poll_interval_secs)
            self.trials.refresh()
        else:
            self.serial_evaluate()

    def run(self, N, block_until_done=True):
        trials = self.trials
        n_queued = 0

        def get_queue_len():
            return trials.count_by_state_unsynced(base.JOB_STATE_NEW)

        def get_n_done():
            return trials.count_by_state_unsynced(base.JOB_STATE_DONE)

        def get_n_unfinished():
            return trials.count_by_state_unsynced([base.JOB_STATE_NEW, base.JOB_STATE_RUNNING])

        stopped = False
        initial_n_done = get_n_done()
        with self.progress_callback(initial=initial_n_done, total=self.max_evals) as progress:
            all_done = False
            best_loss = float("inf")
            while ((n_queued < N or (block_until_done and not all_done))
                   and (self.timeout is None or (timer() - self.start_time) < self.timeout)
                   and (self.loss_threshold is None or best_loss >= self.loss_threshold)):
                qlen = get_queue_len()
                while qlen < self.max_queue_len and n_queued < N and not self.is_cancelled:
                    n_to_enqueue = min(self.max_queue_len - qlen, N - n_queued)
                    new_ids = trials.new_trial_ids(n_to_enqueue)
                    trials.refresh()
                    new_trials = self.algo(new_ids, self.domain, trials,
                                           self.rstate.randint(2 ** 31 - 1))
                    assert len(new_ids) >= len(new_trials)
                    if len(new_trials):
                        trials.insert_trial_docs(new_trials)
                        trials.refresh()
                        n_queued += len(new_trials)
                        qlen = get_queue_len()
                    else:
                        stopped = True
                        break
                if self.is_cancelled:
                    break
                if self.asynchronous:
                    time.sleep(self.poll_interval_secs)
                else:
                    self.serial_evaluate()
                trials.refresh()
                if self.early_stop_fn is not None:
                    stop, kwargs = self.early_stop_fn(trials, *self.early_stop_args)
                    self.early_stop_args = kwargs
                    if stop:
                        logger.info("Early stop triggered. Stopping iterations as condition "
                                    "is reach.")
                        stopped = True
                losses = [l for l in trials.losses() if l is not None and not np.isnan(l)]
                if losses:
                    best_loss = min(losses)
                    progress.postfix = "best loss: " + str(best_loss)
                if get_n_unfinished() == 0:
                    all_done = True
                n_done = get_n_done()
                if n_done - initial_n_done > 0:
                    progress.update(n_done - initial_n_done)
                initial_n_done = n_done
                if stopped:
                    break
        if block_until_done:
            self.block_until_done()
            trials.refresh()
            logger.info("Queue empty, exiting run.")
        else:
            qlen = get_queue_len()
            if qlen:
                logger.info("Exiting run, not waiting for %d jobs." % qlen)

    def __iter__(self):
        return self

    def __next__(self):
        self.run(1, block_until_done=self.asynchronous)
        if self.early_stop_fn is not None:
            stop, kwargs = self.early_stop_fn(self.trials, *self.early_stop_args)
            self.early_stop_args = kwargs
            if stop:
                raise StopIteration()
        if len(self.trials) >= self.max_evals:
            raise StopIteration()
        return self.trials

    def exhaust(self):
        n_done = len(self.trials)
        self.run(self.max_evals - n_done, block_until_done=self.asynchronous)
        self.trials.refresh()
        return self


def fmin(fn, space, algo, max_evals=sys.maxsize, timeout=None, loss_threshold=None,
         trials=None, rstate=None, allow_trials_fmin=True, pass_expr_memo_ctrl=None,
         catch_eval_exceptions=False, verbose=True, return_argmin=True, points_to_evaluate=None,
         max_queue_len=1, show_progressbar=True, early_stop_fn=None):
    """Minimize ``fn`` over ``space`` with ``algo`` (fmin.py:357-551)."""
    if rstate is None:
        env_seed = os.environ.get("HYPEROPT_FMIN_SEED", "")
        rstate = np.random.RandomState(int(env_seed)) if env_seed else np.random.RandomState()
    base.validate_timeout(timeout)
    base.validate_loss_threshold(loss_threshold)
    if allow_trials_fmin and hasattr(trials, "fmin"):
        return trials.fmin(fn, space, algo=algo, max_evals=max_evals, timeout=timeout,
                           loss_threshold=loss_threshold, max_queue_len=max_queue_len,
                           rstate=rstate, pass_expr_memo_ctrl=pass_expr_memo_ctrl,
                           verbose=verbose, catch_eval_exceptions=catch_eval_exceptions,
                           return_argmin=return_argmin, show_progressbar=show_progressbar,
                           early_stop_fn=early_stop_fn)
    if trials is None:
        if points_to_evaluate is None:
            trials = base.Trials()
        else:
            assert type(points_to_evaluate) == list
            trials = generate_trials_to_calculate(points_to_evaluate)
    domain = base.Domain(fn, space, pass_expr_memo_ctrl=pass_expr_memo_ctrl)
    rval = FMinIter(algo, domain, trials, max_evals=max_evals, timeout=timeout,
                    loss_threshold=loss_threshold, rstate=rstate, verbose=verbose,
                    max_queue_len=max_queue_len, show_progressbar=show_progressbar,
                    early_stop_fn=early_stop_fn)
    rval.catch_eval_exceptions = catch_eval_exceptions
    rval.exhaust()
    if return_argmin:
        if len(trials.trials) == 0:
            raise Exception("There are no evaluation tasks, cannot return argmin of task losses.")
        return trials.argmin
    if len(trials) > 0:
        return space_eval(space, trials.argmin)
    return None


def space_eval(space, hp_assignment):
    """Point in ``space`` for a {label: value} assignment (fmin.py:554-572)."""
    space = pyll.as_apply(space)
    memo = {}
    for node in pyll.toposort(space):
        if node.name == "hyperopt_param":
            label = node.pos_args[0].obj
            if label in hp_assignment:
                memo[node] = hp_assignment[label]
    return pyll.rec_eval(space, memo=memo)
