"""ORACLE -- test infrastructure only (imported by tests/; never by the product path).

Independent CPU restatement of the optimiser every experiment calls,
    GaussianProcesses.optimize!(gp, LBFGS(linesearch = BackTracking(order = 2)),
                                Optim.Options(time_limit = 10.))
(examples/maximal_coordinates/CPnoise.jl:41 and its 15 siblings; hyperparameter.jl's searches),
written in the structure of the two packages' sources as published -- Optim 1.4.1
(src/multivariate/optimize/optimize.jl: the main loop; solvers/first_order/l_bfgs.jl:
initial_state, update_state!, twoloop!, update_h!; utilities/assess_convergence.jl) and
LineSearches 7.1.1 (src/backtracking.jl) -- [ext: neither package is in the reference tree;
Manifest.toml pins the versions].  It shares no code with the product's restatements
(gpr.jl_amd/gprx/optim.py on the host, k_lbfgs in gprx_lbfgs.hip on the device).

Parity status: UNPINNED with respect to Optim itself (not runnable here: no Julia, no network).
Pinned instead by hand-derived known answers (tests/test_lbfgs_oracle.py: the quadratic-
interpolation backtracking step, the scaleinvH0 scaling of the first two-loop direction, exact
convergence on quadratics) and used to check the device optimiser's iterates (tests/test_gpu.py).

Conventions restated:
  * NLSolversBase call counting: value_gradient!! at the start counts one f and one g call;
    every line-search trial phi(alpha) one f call; update_g! one g call.
  * Options: iterations 1000, g_abstol 1e-8, x/f tolerances 0 (exact repeats), successive_f_tol
    1, allow_f_increases true, time_limit NaN, f_calls_limit 0 (= none; a soft limit checked after
    each iteration, Optim's semantics -- the deterministic evaluation budget of the benchmarks).
  * The objective is get_optim_target's -mll; a failed evaluation is +Inf with a NaN gradient.
  * dot products: sequential sums of products in index order (the order the product kernels use;
    Julia's BLAS ddot block order is not part of any pinned source).
  * LineSearches' `iterfinite` counter starts at 0 (at most iterfinitemax = 52 halvings for
    non-finite trial values), as in LineSearches 7.1.1; both product restatements
    (gprx/optim.py, gprx_lbfgs.hip) start it at 0 too since round 2.
"""
from __future__ import annotations

import math
import time

import numpy as np

EPS = float(np.finfo(np.float64).eps)


def vdot(a, b) -> float:
    s = 0.0
    for i in range(len(a)):
        s += float(a[i]) * float(b[i])
    return s


def _fdiv(a: float, b: float) -> float:
    """IEEE division as Julia does it (x/0 = +-Inf, 0/0 = NaN)."""
    with np.errstate(divide="ignore", invalid="ignore"):
        return float(np.float64(a) / np.float64(b))


def _nanmin(a, b):  # NaNMath.min
    if math.isnan(a):
        return b
    if math.isnan(b):
        return a
    return a if a < b else b


def _nanmax(a, b):  # NaNMath.max
    if math.isnan(a):
        return b
    if math.isnan(b):
        return a
    return a if a > b else b


class LineSearchException(Exception):
    def __init__(self, message, alpha):
        super().__init__(message)
        self.alpha = alpha


def backtracking(phi, alpha_initial, phi_0, dphi_0, c_1=1e-4, rho_hi=0.5, rho_lo=0.1, iterations=1000, order=2):
    """LineSearches.BackTracking(order)(phi, alpha_initial, phi_0, dphi_0) -> (alpha, phi(alpha))."""
    iterfinitemax = -math.log2(EPS)
    iteration = 0
    phix_0, phix_1 = phi_0, phi_0
    alpha_1, alpha_2 = alpha_initial, alpha_initial
    phix_1 = phi(alpha_1)
    iterfinite = 0
    while not math.isfinite(phix_1) and iterfinite < iterfinitemax:
        iterfinite += 1
        alpha_1 = alpha_2
        alpha_2 = alpha_1 / 2
        phix_1 = phi(alpha_2)
    while phix_1 > phi_0 + c_1 * alpha_2 * dphi_0:
        iteration += 1
        if iteration > iterations:
            raise LineSearchException("Linesearch failed to converge", alpha_2)
        if order == 2 or iteration == 1:
            alpha_tmp = _fdiv(-(dphi_0 * alpha_2 ** 2), 2 * (phix_1 - phi_0 - dphi_0 * alpha_2))
        else:
            div = _fdiv(1.0, alpha_1 ** 2 * alpha_2 ** 2 * (alpha_2 - alpha_1))
            a = (alpha_1 ** 2 * (phix_1 - phi_0 - dphi_0 * alpha_2) - alpha_2 ** 2 * (phix_0 - phi_0 - dphi_0 * alpha_1)) * div
            b = (-alpha_1 ** 3 * (phix_1 - phi_0 - dphi_0 * alpha_2) + alpha_2 ** 3 * (phix_0 - phi_0 - dphi_0 * alpha_1)) * div
            if abs(a) <= EPS:
                alpha_tmp = _fdiv(dphi_0, 2 * b)
            else:
                d = max(b * b - 3 * a * dphi_0, 0.0)
                alpha_tmp = _fdiv(-b + math.sqrt(d), 3 * a)
        alpha_tmp = _nanmin(alpha_tmp, alpha_2 * rho_hi)
        alpha_1 = alpha_2
        alpha_2 = _nanmax(alpha_tmp, alpha_2 * rho_lo)
        phix_0, phix_1 = phix_1, phi(alpha_2)
    return alpha_2, phix_1


class Objective:
    """OnceDifferentiable(f, g!, fg!) with NLSolversBase's call counters and value caches."""

    def __init__(self, fg):
        self._fg = fg
        self.f_calls = 0
        self.g_calls = 0
        self.F = math.nan
        self.DF = None
        self.x_f = None
        self.x_df = None

    def value_gradient_bang(self, x):  # value_gradient!!
        self.F, self.DF = self._fg(x)
        self.DF = np.asarray(self.DF, dtype=np.float64)
        self.x_f = self.x_df = x.copy()
        self.f_calls += 1
        self.g_calls += 1

    def value_bang(self, x):  # value! (line-search trial)
        f, g = self._fg(x)
        self.F = float(f)
        self.x_f = x.copy()
        self.f_calls += 1
        return self.F

    def gradient_bang(self, x):  # gradient! (update_g!)
        if self.x_df is None or not np.array_equal(x, self.x_df):
            _, g = self._fg(x)
            self.DF = np.asarray(g, dtype=np.float64)
            self.x_df = x.copy()
            self.g_calls += 1


class LBFGSState:
    def __init__(self, x, m):
        n = x.shape[0]
        self.x = x.copy()
        self.x_previous = x.copy()
        self.g_previous = np.zeros(n)
        self.rho = np.zeros(m)
        self.dx_history = [np.zeros(n) for _ in range(m)]
        self.dg_history = [np.zeros(n) for _ in range(m)]
        self.dx = np.zeros(n)
        self.dg = np.zeros(n)
        self.s = np.zeros(n)
        self.twoloop_alpha = np.zeros(m)
        self.f_x_previous = math.nan
        self.alpha = 1.0
        self.pseudo_iteration = 0


def twoloop(s, gr, rho, dx_history, dg_history, m, pseudo_iteration, alpha, scaleinvH0):
    """Optim's twoloop! (l_bfgs.jl), identity preconditioner; writes s."""
    q = np.array(gr, dtype=np.float64)
    upper = pseudo_iteration - 1
    lower = pseudo_iteration - m
    for index in range(upper, lower - 1, -1):
        if index < 1:
            continue
        i = (index - 1) % m + 1 - 1  # mod1(index, m), 0-based
        alpha[i] = rho[i] * vdot(dx_history[i], q)
        q = q - alpha[i] * dg_history[i]
    if scaleinvH0 and pseudo_iteration > 1:
        pi = (upper - 1) % m
        q = _fdiv(vdot(dx_history[pi], dg_history[pi]), vdot(dg_history[pi], dg_history[pi])) * q
    for index in range(lower, upper + 1):
        if index < 1:
            continue
        i = (index - 1) % m
        beta = rho[i] * vdot(dg_history[i], q)
        q = q + dx_history[i] * (alpha[i] - beta)
    s[:] = -q


def optimize(fg, x0, m=10, alphaguess=1.0, scaleinvH0=True, c_1=1e-4, rho_hi=0.5, rho_lo=0.1, ls_iterations=1000,
             iterations=1000, g_abstol=1e-8, successive_f_tol=1, time_limit=math.nan, f_calls_limit=0) -> dict:
    """Optim.optimize(OnceDifferentiable, x0, LBFGS(m, alphaguess=InitialStatic(alpha),
    linesearch=BackTracking(order=2)), Options(...)).  fg(x) -> (f, g); f may be +Inf with a NaN
    gradient (a failed GP evaluation)."""
    d = Objective(fg)
    x0 = np.asarray(x0, dtype=np.float64)
    state = LBFGSState(x0, m)
    d.value_gradient_bang(state.x)  # initial_state
    t0 = time.time()
    g_converged = max(abs(float(v)) for v in d.DF) <= g_abstol if d.DF.size else True  # initial_convergence
    if any(math.isnan(float(v)) for v in d.DF):
        g_converged = False
    converged = g_converged
    stopped = False
    iteration = 0
    counter_f_tol = 0
    reason = "g_tol" if converged else None
    x_conv = f_conv = False
    while not converged and not stopped and iteration < iterations:
        iteration += 1
        # ---- update_state! (l_bfgs.jl)
        state.pseudo_iteration += 1
        twoloop(state.s, d.DF, state.rho, state.dx_history, state.dg_history, m, state.pseudo_iteration,
                state.twoloop_alpha, scaleinvH0)
        state.g_previous = d.DF.copy()
        # perform_linesearch!
        dphi_0 = vdot(d.DF, state.s)
        if dphi_0 >= 0.0:  # reset_search_direction!
            state.pseudo_iteration = 1
            state.s = -d.DF
            dphi_0 = vdot(d.DF, state.s)
        phi_0 = d.F
        state.alpha = alphaguess  # InitialStatic
        state.f_x_previous = phi_0
        state.x_previous = state.x.copy()
        xs, ss = state.x.copy(), state.s.copy()
        try:
            state.alpha, _ = backtracking(lambda a: d.value_bang(xs + a * ss), state.alpha, phi_0, dphi_0, c_1, rho_hi,
                                          rho_lo, ls_iterations)
            ls_success = True
        except LineSearchException as ex:
            state.alpha = ex.alpha
            ls_success = False
        state.dx = state.alpha * state.s
        state.x = state.x + state.dx
        if not ls_success:
            reason = "linesearch"
            break
        d.gradient_bang(state.x)  # update_g!
        # ---- assess_convergence (x_abstol = x_reltol = f_abstol = f_reltol = 0)
        with np.errstate(invalid="ignore"):
            xch = np.abs(state.x - state.x_previous)
            x_conv = (not np.any(np.isnan(xch))) and float(np.max(xch)) <= 0.0
            f_conv = abs(d.F - state.f_x_previous) <= 0.0
            gres = np.abs(d.DF)
            g_converged = (not np.any(np.isnan(gres))) and float(np.max(gres)) <= g_abstol
        counter_f_tol = counter_f_tol + 1 if f_conv else 0
        converged = x_conv or g_converged or counter_f_tol > successive_f_tol
        # ---- update_h!
        state.dg = d.DF - state.g_previous
        rho_iteration = _fdiv(1.0, vdot(state.dx, state.dg))
        if not math.isinf(rho_iteration):
            idx = (state.pseudo_iteration - 1) % m
            state.dx_history[idx] = state.dx.copy()
            state.dg_history[idx] = state.dg.copy()
            state.rho[idx] = rho_iteration
        if converged:
            reason = "g_tol" if g_converged else ("x_tol" if x_conv else "f_tol")
        stopped_by_time_limit = time.time() - t0 > time_limit  # False for NaN
        f_limit_reached = f_calls_limit > 0 and d.f_calls >= f_calls_limit
        if stopped_by_time_limit or f_limit_reached:
            stopped = True
            if not converged:
                reason = "time_limit" if stopped_by_time_limit else "max_evals"
        if d.g_calls > 0 and not np.all(np.isfinite(d.DF)):
            if not converged and not stopped:
                reason = "nan_gradient"
            break
    if reason is None:
        reason = "iterations"
    return dict(minimizer=state.x.copy(), minimum=float(d.F), iterations=iteration, f_calls=d.f_calls,
                g_calls=d.g_calls, converged=bool(converged), stopped_by=reason)
