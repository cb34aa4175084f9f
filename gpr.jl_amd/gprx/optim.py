"""Host-side hyper-parameter optimiser: the call GaussianProcesses.optimize!(gp,
LBFGS(linesearch=BackTracking(order=2)), Optim.Options(time_limit=10.)) made by every experiment
(e.g. examples/maximal_coordinates/CPnoise.jl:41), restated from the published algorithms of
Optim 1.4.1 (LBFGS, m = 10, InitialStatic alpha = 1, scaleinvH0) and LineSearches 7.1.1
(BackTracking, c1 = 1e-4, rho_hi = 0.5, rho_lo = 0.1, quadratic interpolation) -- [ext, not in
the reference tree; Manifest.toml pins the versions].

Each evaluation is one device call (gprx_gp_lml / gprx_gp_lml_grad through GPE).  The objective
follows GaussianProcesses' get_optim_target: minimise -mll; a failed evaluation (not positive
definite, ArgumentError, non-finite hyper-parameters) counts as +Inf and the parameters are
restored.  Convergence follows Optim's assess_convergence with its defaults (g_abstol = 1e-8,
x_abstol = f_abstol = 0, i.e. an exact repeat of x stops, and an exact repeat of f stops once it
has happened on successive_f_tol + 1 = 2 successive iterations; allow_f_increases = true); a
failed line search moves x by the search's last step and stops before the gradient evaluation;
a non-finite gradient after an iteration ends the loop ("Terminated early due to NaN in
gradient").  Calls are counted as NLSolversBase does: the initial value_gradient!! is one f and
one g call, every line-search trial one f call, update_g! one g call.
Besides the reference's wall-clock cap, `max_evals` gives the deterministic evaluation budget
SURVEY.md section 8d asks for: Optim's own Options.f_calls_limit, a soft limit checked after each
iteration (f calls = the initial evaluation + every line-search trial = the device evaluations of
the lock-step driver, whose evaluations all carry the gradient).  The independent restatement in
oracle/lbfgs_oracle.py checks this one.  `gprx.batch.GPBatch.optimize` runs the same algorithm on the
device (k_lbfgs), one lock-step round per batch evaluation.
"""
from __future__ import annotations

import math
import time
from dataclasses import dataclass, field

import numpy as np

from . import _lib as L


@dataclass
class BackTracking:
    order: int = 2
    c_1: float = 1e-4
    rho_hi: float = 0.5
    rho_lo: float = 0.1
    iterations: int = 1000

    def __call__(self, phi, alpha_0: float, phi_0: float, dphi_0: float):
        """LineSearches.BackTracking: returns (alpha, phi(alpha)); raises LineSearchError."""
        return _drive(self.search(alpha_0, phi_0, dphi_0), phi)

    def search(self, alpha_0: float, phi_0: float, dphi_0: float):
        """The same search as a generator: yields each step length to evaluate, receives phi(a),
        returns (alpha, phi(alpha)) -- so a batch of independent searches can share device calls."""
        iterfinitemax = -math.log2(np.finfo(float).eps)
        a1 = a2 = alpha_0
        phix0, phix1 = phi_0, (yield a1)
        it_fin = 0  # LineSearches BackTracking: iterfinite = 0, at most iterfinitemax halvings
        while not math.isfinite(phix1) and it_fin < iterfinitemax:
            it_fin += 1
            a1 = a2
            a2 = a1 / 2
            phix1 = yield a2
        it = 0
        # sufficient decrease and the quadratic model are both anchored at phi(0) = phi_0; phix0
        # (the previous trial value) only enters the cubic model
        while phix1 > phi_0 + self.c_1 * a2 * dphi_0:
            it += 1
            if it > self.iterations:
                raise LineSearchError(a2, phix1)
            if self.order == 2 or it == 1:
                atmp = _div(-(dphi_0 * (a2 * a2)), 2 * (phix1 - phi_0 - dphi_0 * a2))  # Julia: dphi_0 * a2^2
            else:
                div = _div(1.0, a1 * a1 * a2 * a2 * (a2 - a1))
                a = (a1 * a1 * (phix1 - phi_0 - dphi_0 * a2) - a2 * a2 * (phix0 - phi_0 - dphi_0 * a1)) * div
                b = (-a1**3 * (phix1 - phi_0 - dphi_0 * a2) + a2**3 * (phix0 - phi_0 - dphi_0 * a1)) * div
                if abs(a) <= np.finfo(float).eps:
                    atmp = _div(dphi_0, 2 * b)
                else:
                    disc = max(b * b - 3 * a * dphi_0, 0.0)
                    atmp = _div(-b + math.sqrt(disc), 3 * a)
            atmp = _nanmin(atmp, a2 * self.rho_hi)
            a1 = a2
            a2 = _nanmax(atmp, a2 * self.rho_lo)
            phix0, phix1 = phix1, (yield a2)
        return a2, phix1


def _drive(gen, fn):
    """Run a request generator to completion, answering each yielded request with fn(request)."""
    try:
        req = next(gen)
        while True:
            req = gen.send(fn(req))
    except StopIteration as e:
        return e.value


class LineSearchError(Exception):
    def __init__(self, alpha, phi=math.nan):
        super().__init__("line search failed to converge")
        self.alpha = alpha
        self.phi = phi  # phi(alpha): the last value the search evaluated


def _div(a, b) -> float:
    """a / b with IEEE (Julia) semantics: x/0 -> +-Inf, 0/0 -> NaN, never an exception."""
    with np.errstate(divide="ignore", invalid="ignore"):
        return float(np.float64(a) / np.float64(b))


def _dot(a, b) -> float:
    """Sequential sum of products, left to right without fused multiply-adds: the summation order
    of the device optimiser's dot_ (gprx_lbfgs.hip), so host and device iterates agree bit for
    bit.  (Julia's dot is BLAS ddot, whose blocked order is not part of the reference tree.)"""
    s = 0.0
    for u, v in zip(np.asarray(a, dtype=np.float64).tolist(), np.asarray(b, dtype=np.float64).tolist()):
        s += u * v
    return s


def _nanmin(a, b):
    return b if math.isnan(a) else (a if math.isnan(b) else min(a, b))


def _nanmax(a, b):
    return b if math.isnan(a) else (a if math.isnan(b) else max(a, b))


@dataclass
class LBFGS:
    m: int = 10
    linesearch: BackTracking = field(default_factory=lambda: BackTracking(order=2))
    alphaguess: float = 1.0
    scaleinvH0: bool = True


@dataclass
class Options:
    iterations: int = 1000
    g_abstol: float = 1e-8
    time_limit: float = math.nan
    successive_f_tol: int = 1
    max_evals: int | None = None  # Optim's f_calls_limit: a soft limit on f calls;
    # None or <= 0: no limit (Optim's f_calls_limit = 0 default)


@dataclass
class Result:
    minimizer: np.ndarray
    minimum: float
    iterations: int
    f_calls: int
    g_calls: int
    converged: bool
    stopped_by: str


def _twoloop(g, rho, dxh, dgh, m, pseudo_it, scaleinvH0):
    """Optim's twoloop!: s = -H g from the last m (dx, dg) pairs."""
    q = g.copy()
    lower, upper = pseudo_it - m, pseudo_it - 1
    alpha = np.zeros(m)
    for index in range(upper, lower - 1, -1):
        if index < 1:
            continue
        i = (index - 1) % m
        alpha[i] = rho[i] * _dot(dxh[i], q)
        q -= alpha[i] * dgh[i]
    if scaleinvH0 and pseudo_it > 1:
        i = (upper - 1) % m
        s = _div(_dot(dxh[i], dgh[i]), _dot(dgh[i], dgh[i])) * q  # Julia float semantics: x/0 -> Inf/NaN
    else:
        s = q.copy()
    for index in range(lower, upper + 1):
        if index < 1:
            continue
        i = (index - 1) % m
        beta = rho[i] * _dot(dgh[i], s)
        s += dxh[i] * (alpha[i] - beta)
    return -s


def lbfgs_minimize(f, fg, x0, method: LBFGS | None = None, options: Options | None = None) -> Result:
    """Optim.optimize(OnceDifferentiable(f, g!, fg!), x0, LBFGS(...), options).

    f(x) -> value; fg(x) -> (value, gradient).  Values may be +inf (failed evaluations)."""

    def answer(req):
        kind, x = req
        return f(x) if kind == "f" else fg(x)

    return _drive(lbfgs_steps(x0, method, options), answer)


def lbfgs_steps(x0, method: LBFGS | None = None, options: Options | None = None):
    """LBFGS as a request generator: yields ("f", x) or ("fg", x), receives f(x) or (f(x), g(x)),
    returns the Result.  lbfgs_minimize drives one; optimize_batch drives a batch in lock-step."""
    method = method or LBFGS()
    options = options or Options()
    t0 = time.time()
    calls = {"f": 0, "g": 0}

    def budget(kind):
        calls[kind] += 1

    x = np.array(x0, dtype=np.float64)
    n = x.shape[0]
    m = method.m
    dxh = [np.zeros(n) for _ in range(m)]
    dgh = [np.zeros(n) for _ in range(m)]
    rho = np.zeros(m)
    stopped = "iterations"
    it = 0
    fx = math.nan
    converged = False
    counter_f_tol = 0
    budget("f")  # value_gradient!!: one f and one g call
    budget("g")
    fx, g = yield ("fg", x)
    pseudo = 0
    converged = bool(np.max(np.abs(g)) <= options.g_abstol)
    if converged:
        stopped = "g_tol"
    while not converged and it < options.iterations:
        it += 1
        pseudo += 1
        s = _twoloop(g, rho, dxh, dgh, m, pseudo, method.scaleinvH0)
        g_prev = g.copy()
        dphi0 = _dot(g, s)
        if dphi0 >= 0:  # reset_search_direction!
            pseudo = 1
            s = -g
            dphi0 = _dot(g, s)
        ls = method.linesearch.search(method.alphaguess, fx, dphi0)
        try:
            a = next(ls)
            while True:
                budget("f")
                a = ls.send((yield ("f", x + a * s)))
        except StopIteration as e:
            alpha, ls_ok = e.value[0], True
        except LineSearchError as e:
            alpha, ls_ok, ls_phi = e.alpha, False, e.phi
        dx = alpha * s
        x_prev, f_prev = x, fx
        x = x + dx
        if not ls_ok:
            # Optim's update_state! reports the failed search and the loop breaks before
            # update_g!: x has moved, the objective's value cache holds phi(alpha)
            fx = float(ls_phi)
            stopped = "linesearch"
            break
        budget("g")
        fx, g = yield ("fg", x)
        dg = g - g_prev
        denom = _dot(dx, dg)
        r = _div(1.0, denom)
        if not math.isinf(r):
            i = (pseudo - 1) % m
            dxh[i] = dx.copy()
            dgh[i] = dg.copy()
            rho[i] = r
        # assess_convergence with Optim's defaults x_tol = f_tol = 0 (exact repeats) and g_tol;
        # f convergence counts only on successive iterations (Options.successive_f_tol)
        with np.errstate(invalid="ignore"):
            g_conv = bool(np.max(np.abs(g)) <= options.g_abstol)
            x_conv = bool(np.max(np.abs(x - x_prev)) <= 0.0)
            f_conv = bool(abs(fx - f_prev) <= 0.0)
        counter_f_tol = counter_f_tol + 1 if f_conv else 0
        if g_conv:
            converged, stopped = True, "g_tol"
        elif x_conv:
            converged, stopped = True, "x_tol"
        elif counter_f_tol > options.successive_f_tol:
            converged, stopped = True, "f_tol"
        if converged:
            break
        if not math.isnan(options.time_limit) and time.time() - t0 > options.time_limit:
            stopped = "time_limit"
            break
        # Optim: f_limit_reached = f_calls_limit > 0 && f_calls >= f_calls_limit (0 / None: no limit)
        if options.max_evals is not None and options.max_evals > 0 and calls["f"] >= options.max_evals:
            stopped = "max_evals"
            break
        if not np.all(np.isfinite(g)):
            stopped = "nan_gradient"
            break
    return Result(x, float(fx), it, calls["f"], calls["g"], converged, stopped)


def optimize(gp, method: LBFGS | None = None, options: Options | None = None) -> Result:
    """GaussianProcesses.optimize!(gp, method, options): minimise -mll over
    [logσn, logℓ..., logσf]; evaluations that fail count as +Inf (get_optim_target)."""
    init = gp.get_params().copy()

    def safe(hyp, want_grad):
        prev = gp.get_params().copy()
        try:
            if not np.all(np.isfinite(hyp)):
                raise ValueError("non-finite hyperparameters")
            gp.set_params(hyp)
            if want_grad:
                m, dm = gp.update_mll_and_dmll()
                return -m, -np.asarray(dm)
            return -gp.update_mll(), None
        except (L.NotPositiveDefinite, ValueError):
            gp.set_params(prev)
            return math.inf, np.full(hyp.shape[0], math.nan)

    res = lbfgs_minimize(lambda h: safe(h, False)[0], lambda h: safe(h, True), init, method, options)
    try:
        gp.set_params(res.minimizer)
        gp.update_mll()
    except Exception:
        gp.set_params(init)
        gp.update_mll()
        raise
    return res


def optimize_batch(batch, theta0, method: LBFGS | None = None, options: Options | None = None,
                   trace: list | None = None):
    """One LBFGS run per slot of a GPBatch (the per-output GPs of CPnoise.jl:37-43 and the trials
    of examples/parallel/core.jl:28), in lock-step: every round answers all pending requests with
    ONE device evaluation of the whole batch (value + gradient for every slot).  Each slot follows
    exactly the trajectory lbfgs_minimize would give it alone (the requests and their answers are
    the same; only the device calls are shared).  A gradient computed during the line search is
    reused when that point is accepted, within the same round (k_lbfgs does the same).  Failed
    slots answer +Inf as in `optimize`.
    trace: a list that receives one (B, 2n+2) array per round, rows [active, theta(n), mll,
    dmll(n)] -- the layout of GPBatch.optimize's `last_opt_trace` (gprx_batch_set_opt_trace).
    Returns (results, rounds)."""
    theta0 = np.asarray(theta0, dtype=np.float64)
    B, npar = theta0.shape
    gens = [lbfgs_steps(theta0[s], method, options) for s in range(B)]
    results = [None] * B
    pending = [None] * B
    for s in range(B):
        try:
            pending[s] = next(gens[s])
        except StopIteration as e:
            results[s] = e.value
    cache = [None] * B  # (x, f, g) of the slot's last evaluation
    rounds = 0
    while any(p is not None for p in pending):
        todo = []
        th = theta0.copy()
        for s, req in enumerate(pending):
            if req is None:
                continue
            x = req[1]
            if cache[s] is not None and np.array_equal(cache[s][0], x):
                continue
            todo.append(s)
            th[s] = x if np.all(np.isfinite(x)) else theta0[s]
        if todo:
            rounds += 1
            r = batch.run(th, grad=True, predict=False)
            if trace is not None:
                act = np.zeros((B, 1))
                act[todo] = 1.0
                trace.append(np.hstack([act, th, np.asarray(r["mll"])[:, None], np.asarray(r["grad"])]))
            for s in todo:
                x = pending[s][1]
                if r["status"][s] != 0 or not np.all(np.isfinite(x)):
                    cache[s] = (x.copy(), math.inf, np.full(npar, math.nan))
                else:
                    cache[s] = (x.copy(), -float(r["mll"][s]), -np.asarray(r["grad"][s], dtype=np.float64))
        for s, req in enumerate(pending):
            if req is None:
                continue
            # answer from the cache, and keep answering while the slot's next request is its
            # cached point (the accepted line-search point's gradient): one round per new point
            while True:
                x, f, g = cache[s]
                try:
                    req = gens[s].send(f if req[0] == "f" else (f, g.copy()))
                except StopIteration as e:
                    pending[s] = None
                    results[s] = e.value
                    break
                if not np.array_equal(x, req[1]):
                    pending[s] = req
                    break
    return results, rounds


def _same_bits(a, b) -> bool:
    """Bitwise equality of two float arrays (NaN payloads and signed zeros included)."""
    a = np.ascontiguousarray(a, dtype=np.float64)
    b = np.ascontiguousarray(b, dtype=np.float64)
    return a.shape == b.shape and bool(np.array_equal(a.view(np.uint64), b.view(np.uint64)))


def compare_optimisers(res_a, res_b, trace_a=None, trace_b=None) -> dict:
    """Bit-level comparison of two optimiser runs over the same batch (e.g. the device optimiser,
    GPBatch.optimize, against the host lock-step restatement, optimize_batch).  Minimisers and
    minima compare by their bits, so equal NaN minima agree.  With both evaluation traces (rows
    [active, theta(n), mll, dmll(n)] per round) the first differing slot's evaluation sequences
    are walked in order to name the first evaluation where the two runs part: the same theta
    answered differently (the evaluation is not reproducible) or a different theta requested (the
    two optimisers decided differently on equal answers)."""
    B = len(res_a)
    bad = [s for s in range(B)
           if not (_same_bits(res_a[s].minimizer, res_b[s].minimizer)
                   and _same_bits(np.float64(res_a[s].minimum), np.float64(res_b[s].minimum)))]
    out = {"equal": not bad, "slots": B, "n_differ": len(bad)}
    if not bad:
        return out
    s = bad[0]
    a, b = res_a[s], res_b[s]
    with np.errstate(invalid="ignore"):
        dth = float(np.max(np.abs(np.asarray(a.minimizer) - np.asarray(b.minimizer))))
    out.update(first_slot=s, differing_slots=bad[:16], stopped_by=[a.stopped_by, b.stopped_by],
               f_calls=[a.f_calls, b.f_calls], minimum=[a.minimum, b.minimum], max_abs_dtheta=dth,
               nonfinite_minimum=[not math.isfinite(a.minimum), not math.isfinite(b.minimum)])
    if trace_a is None or trace_b is None:
        return out

    def seq(tr):
        tr = np.asarray(tr)
        return [(r, tr[r, s]) for r in range(tr.shape[0]) if tr[r, s, 0] == 1.0]

    sa, sb = seq(trace_a), seq(trace_b)
    n = (np.asarray(trace_a).shape[2] - 2) // 2
    first = None
    for k, ((ra, ea), (rb, eb)) in enumerate(zip(sa, sb)):
        if not _same_bits(ea[1:1 + n], eb[1:1 + n]):
            first = dict(index=k, round=[ra, rb], kind="different theta requested",
                         max_abs_dtheta=float(np.max(np.abs(ea[1:1 + n] - eb[1:1 + n]))))
            break
        if not _same_bits(ea[1 + n:], eb[1 + n:]):
            with np.errstate(invalid="ignore"):
                dm = abs(float(ea[1 + n]) - float(eb[1 + n]))
                dg = float(np.max(np.abs(ea[2 + n:] - eb[2 + n:])))
            first = dict(index=k, round=[ra, rb], kind="same theta answered differently",
                         mll=[float(ea[1 + n]), float(eb[1 + n])], abs_dmll=dm, max_abs_dgrad=dg)
            break
    if first is None and len(sa) != len(sb):
        first = dict(index=min(len(sa), len(sb)), kind="evaluation counts differ", counts=[len(sa), len(sb)])
    out["first_eval_diff"] = first
    out["evaluations"] = [len(sa), len(sb)]
    return out
