"""gprx -- MI355X-native exact SE-ARD Gaussian-process hot path for GPR.jl (host mirror over the
C ABI in include/gprx.h).  Importing this package loads libgprx.so and fails loudly without it."""
from . import _lib
from ._lib import GPRXError, NotPositiveDefinite, DIST_DIRECT, DIST_EXPANDED, OPT_GRAPHS, OPT_LEAF_TILES, OPT_SMALL_N
from .batch import Context, GPBatch, default_context
from .gp import GP, GPE, SEArd, MeanZero, MeanFunction, predict_f, predict_y
from .rollout import predictdynamics, predictdynamicsmin, predictdynamicsmin_batch, rollout_min

__all__ = [
    "Context", "GPBatch", "default_context", "GP", "GPE", "SEArd", "MeanZero", "MeanFunction",
    "predict_f", "predict_y", "GPRXError", "NotPositiveDefinite", "DIST_DIRECT", "DIST_EXPANDED",
    "predictdynamics", "predictdynamicsmin", "predictdynamicsmin_batch", "rollout_min",
]
