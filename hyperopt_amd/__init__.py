"""hyperopt_amd -- MI355X-native Tree-of-Parzen-Estimators suggest engine.

Drop-in for hyperopt's ``fmin`` / ``hp`` / ``Trials`` / ``tpe.suggest`` API;
the TPE hot path (Parzen fit, candidate sampling, EI scoring, argmax) runs as
hand-written HIP kernels for gfx950 (libtpe_hip.so, include/tpe_hip.h).
"""
from . import hp, pyll, rand, tpe  # noqa: F401
from .base import (JOB_STATE_DONE, JOB_STATE_ERROR, JOB_STATE_NEW,  # noqa: F401
                   JOB_STATE_RUNNING, JOB_STATES, STATUS_FAIL, STATUS_NEW, STATUS_OK,
                   STATUS_RUNNING, STATUS_STRINGS, STATUS_SUSPENDED, Ctrl, Domain, Trials,
                   trials_from_docs)
from .exceptions import (AllTrialsFailed, BadSearchSpace, DuplicateLabel,  # noqa: F401
                         InvalidLoss, InvalidResultStatus, InvalidTrial)
from .fmin import (FMinIter, fmin, fmin_pass_expr_memo_ctrl, partial,  # noqa: F401
                   space_eval)

__version__ = "0.1.0"
