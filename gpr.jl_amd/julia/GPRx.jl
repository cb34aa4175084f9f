"""
    GPRx — Julia ccall shim routing GaussianProcesses.jl's exact SE-ARD GP evaluations to the
    MI355X library (libgprx.so, C ABI in include/gprx.h).

Load it after GaussianProcesses (e.g. one `include` in src/GPR.jl, see INTEGRATION.md); the
experiment scripts (examples/noise.jl, examples/hyperparameter.jl) stay textually unchanged:

    GP(X, y, mean, SEArd(...))            -> gprx_gp_create + gprx_gp_lml   (CPnoise.jl:40)
    optimize!(gp, LBFGS(...), Options())  -> gprx_gp_lml / gprx_gp_lml_grad per evaluation
    predict_y(gp, x*)                     -> gprx_gp_predict                 (predictdynamics.jl:13)

plus `GPRx.optimize_all!(gps)`: the loop `for gp in gps; optimize!(gp, LBFGS(linesearch =
BackTracking(order=2)), Optim.Options(time_limit=10.)); end` of CPnoise.jl:37-43 as ONE
gprx_batch_optimize call (device LBFGS, every GP of the trial in lock-step).

Method names follow GaussianProcesses v0.12.4 internals (update_mll!, update_target_and_dtarget!,
predict_f); they are [ext] — confirm against that package's source before shipping.
Not executable in the build container (no Julia runtime).
"""
module GPRx

using GaussianProcesses
using GaussianProcesses: GPE, SEArd, Mean
using LinearAlgebra

const LIB = joinpath(@__DIR__, "..", "lib", "libgprx.so")
const ABI = Cint(3)  # include/gprx.h GPRX_ABI_VERSION these ccall signatures follow
const OK, NOT_PD, INVALID = Cint(0), Cint(1), Cint(2)

function __init__()
    abi = ccall((:gprx_abi_version, LIB), Cint, ())
    abi == ABI || error("gprx: $LIB implements ABI version $abi, GPRx.jl expects $ABI")
end

# one context (HIP stream) per Julia thread; device = thread mod #GPUs (core.jl:28 workers), the
# device count from the library (GPRX_NGPU, if set, caps it, e.g. to leave GPUs to other jobs)
const CTX = Dict{Int,Ptr{Cvoid}}()
function ndevices()
    n = Int(ccall((:gprx_device_count, LIB), Cint, ()))
    n > 0 || error("gprx: no visible GPU")
    haskey(ENV, "GPRX_NGPU") ? clamp(parse(Int, ENV["GPRX_NGPU"]), 1, n) : n
end
const CTX_LOCK = ReentrantLock()
function context()
    tid = Threads.threadid()
    lock(CTX_LOCK) do
        get!(CTX, tid) do
            ngpu = ndevices()
            h = Ref{Ptr{Cvoid}}(C_NULL)
            rc = ccall((:gprx_ctx_create, LIB), Cint, (Cint, Ref{Ptr{Cvoid}}), (tid - 1) % ngpu, h)
            rc == OK || error("gprx_ctx_create failed ($rc)")
            h[]
        end
    end
end

# device handle per GPE; X and y - μ(X) copied once (μ is θ-independent: MeanDynamics has no
# parameters, src/mDynamics.jl:29)
mutable struct Handle
    ptr::Ptr{Cvoid}
end
const HANDLES = WeakKeyDict{Any,Handle}()
const H_LOCK = ReentrantLock()

function handle(gp::GPE)
    lock(H_LOCK) do
        get!(HANDLES, gp) do
            X = Matrix{Float64}(gp.x)                      # d x N column-major, as the ABI
            r = gp.y .- GaussianProcesses.mean(gp.mean, X)
            h = Ref{Ptr{Cvoid}}(C_NULL)
            rc = ccall((:gprx_gp_create, LIB), Cint,
                       (Ptr{Cvoid}, Ptr{Float64}, Cint, Cint, Ptr{Float64}, Ref{Ptr{Cvoid}}),
                       context(), X, size(X, 1), size(X, 2), r, h)
            rc == OK || error("gprx_gp_create failed ($rc)")
            hd = Handle(h[])
            finalizer(x -> ccall((:gprx_gp_destroy, LIB), Cvoid, (Ptr{Cvoid},), x.ptr), hd)
            hd
        end
    end
end

# θ in GaussianProcesses' optimiser order: [logNoise; mean params (none); logℓ...; logσ]
theta(gp::GPE) = Float64[gp.logNoise.value; GaussianProcesses.get_params(gp.kernel)...]

# status -> the exception GaussianProcesses' own path raises; `info` is the 1-based failing pivot
# the ABI reports (LAPACK dpotrf's info, as cholesky! puts it into PosDefException)
function check(rc::Cint, gp, info::Integer=-1)
    rc == NOT_PD && throw(LinearAlgebra.PosDefException(Int(info)))
    rc == INVALID && throw(ArgumentError("gprx: invalid hyperparameters"))
    rc == OK || error("gprx device error ($rc)")
end

# One evaluation of the GP's batch of one (gprx_batch_run: it also reports the failing pivot).
# flags: 1 = gradient.  Afterwards gp.alpha holds K^-1 (y - m(X)) of the device factorisation.
function evaluate!(gp::GPE, flags::Integer)
    b = ccall((:gprx_gp_batch, LIB), Ptr{Cvoid}, (Ptr{Cvoid},), handle(gp).ptr)
    m = Ref{Float64}(0.0)
    g = zeros(length(theta(gp)))
    st, info = Ref{Cint}(0), Ref{Cint}(0)
    rc = ccall((:gprx_batch_run, LIB), Cint,
               (Ptr{Cvoid}, Ptr{Float64}, Cuint, Ref{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64},
                Ref{Cint}, Ref{Cint}),
               b, theta(gp), Cuint(flags), m, g, C_NULL, C_NULL, st, info)
    check(rc, gp, info[])
    a = zeros(length(gp.y))
    check(ccall((:gprx_batch_alpha, LIB), Cint, (Ptr{Cvoid}, Ptr{Float64}), b, a), gp)
    gp.alpha = a
    return m[], g
end

# gp.cK (the host PDMat of K and its Cholesky factor) is not maintained by the device path: the
# factorisation stays in HBM.  Code that reads it (full-covariance prediction, rand, ...) calls
# materialize!(gp) first, which runs GaussianProcesses' own update_cK! / update_mll! on the host
# once at the current hyperparameters (O(N^3) on the CPU, on request only).
function materialize!(gp::GPE)
    invoke(GaussianProcesses.update_mll!, Tuple{GPE}, gp)
    gp
end

# The varargs absorb GaussianProcesses' optional positional arguments (e.g. the precompute buffer
# that optimize! passes to update_target_and_dtarget!) so these methods win dispatch for every
# call form.
function GaussianProcesses.update_mll!(gp::GPE{<:Any,<:Any,<:Mean,<:SEArd}, args...; kwargs...)
    m, _ = evaluate!(gp, 0)
    gp.mll = m
    gp.target = gp.mll
    gp
end

function GaussianProcesses.update_target_and_dtarget!(gp::GPE{<:Any,<:Any,<:Mean,<:SEArd}, args...; kwargs...)
    m, g = evaluate!(gp, 1)
    gp.mll = m
    gp.dmll = g
    gp.target = gp.mll
    gp.dtarget = g
    gp
end

function GaussianProcesses.predict_f(gp::GPE{<:Any,<:Any,<:Mean,<:SEArd}, x::AbstractMatrix; full_cov::Bool=false)
    if full_cov  # the M x M posterior covariance: GaussianProcesses' own host method on gp.cK
        materialize!(gp)
        return invoke(GaussianProcesses.predict_f, Tuple{GPE,AbstractMatrix}, gp, x; full_cov=true)
    end
    xs = Matrix{Float64}(x)
    M = size(xs, 2)
    mu = zeros(M)
    var = zeros(M)
    check(ccall((:gprx_gp_predict, LIB), Cint, (Ptr{Cvoid}, Ptr{Float64}, Cint, Ptr{Float64}, Ptr{Float64}),
                handle(gp).ptr, xs, M, mu, var), gp)
    return mu .+ GaussianProcesses.mean(gp.mean, xs), var   # predict_y adds exp(2 logNoise)
end

# predictdynamicsmin (examples/utils/predictdynamics.jl:30-102) for all test observations of one
# trial in one device launch.  `gps` must be MeanZero GPEs evaluated on this thread's context (the
# experiment's own thread, core.jl:28).  Returns the (q_cur, q̇_last) per coordinate and
# trajectory; the caller builds the CState from q_cur as predictdynamics.jl:48-101 does.
const MECH = Dict("P1" => Cint(1), "P2" => Cint(2), "CP" => Cint(3), "FB" => Cint(4))
function rollout_min(etype::String, gps::Vector{<:GPE}, startobservations::Vector{Vector{Float64}},
                     steps::Integer; usesin::Bool=false, Δt::Real=0.01)
    haskey(MECH, etype) || throw(ArgumentError("Experiment $etype not supported!"))
    all(gp -> gp.mean isa MeanZero, gps) || error("gprx: device rollouts need MeanZero GPs")
    T = length(startobservations)
    nc = etype == "P1" ? 1 : 2
    fin = zeros(2nc, T)
    bs = [ccall((:gprx_gp_batch, LIB), Ptr{Cvoid}, (Ptr{Cvoid},), handle(gp).ptr) for gp in gps]
    rc = ccall((:gprx_rollout_min, LIB), Cint,
               (Ptr{Cvoid}, Cint, Cint, Cdouble, Cint, Cint, Ptr{Ptr{Cvoid}}, Ptr{Cint}, Cint, Ptr{Cint},
                Ptr{Float64}, Ptr{Float64}),
               context(), MECH[etype], Cint(usesin), Float64(Δt), Cint(steps), Cint(1), bs, zeros(Cint, nc),
               Cint(T), zeros(Cint, T), reduce(hcat, startobservations), fin)
    check(rc, gps)
    return [fin[:, t] for t in 1:T]
end

# gprx_opt_options (include/gprx.h): same field order and C layout
struct OptOptions
    m::Cint
    iterations::Cint
    max_evals::Cint
    ls_iterations::Cint
    scaleinvH0::Cint
    refit::Cint
    successive_f_tol::Cint
    g_abstol::Cdouble
    time_limit::Cdouble
    alphaguess::Cdouble
    c_1::Cdouble
    rho_hi::Cdouble
    rho_lo::Cdouble
end
const STOP = ("iterations", "g_tol", "x_tol", "f_tol", "linesearch", "max_evals", "time_limit", "nan_gradient")

# optimize! for every GP of a trial (CPnoise.jl:37-43) in one device call: Optim LBFGS +
# BackTracking(order=2) as k_lbfgs, one lock-step evaluation of all GPs per round.  `time_limit`
# is per call (the reference's 10 s applies to each GP in turn).  Afterwards every GP holds its
# minimiser (set_params! + update_mll!, as optimize! leaves it).  Returns one NamedTuple per GP.
function optimize_all!(gps::Vector{<:GPE}; time_limit::Real=NaN, iterations::Integer=1000,
                       max_evals::Integer=-1, g_abstol::Real=1e-8)
    B = length(gps)
    X1 = Matrix{Float64}(gps[1].x)
    d, N = size(X1)
    shared = all(gp -> gp.x == gps[1].x, gps)
    X = shared ? X1 : reduce(hcat, [Matrix{Float64}(gp.x) for gp in gps])
    Y = reduce(hcat, [gp.y .- GaussianProcesses.mean(gp.mean, Matrix{Float64}(gp.x)) for gp in gps])
    th0 = reduce(hcat, [theta(gp) for gp in gps])          # (d+2) x B: slot b's theta contiguous
    ctx = context()
    b = Ref{Ptr{Cvoid}}(C_NULL)
    rc = ccall((:gprx_batch_create, LIB), Cint, (Ptr{Cvoid}, Cint, Cint, Cint, Cint, Ref{Ptr{Cvoid}}),
               ctx, B, d, N, 0, b)
    rc == OK || error("gprx_batch_create failed ($rc)")
    try
        rc = ccall((:gprx_batch_set_train, LIB), Cint, (Ptr{Cvoid}, Ptr{Float64}, Int64, Ptr{Float64}, Int64, Cint),
                   b[], X, shared ? 0 : d * N, Y, N, 0)
        rc == OK || error("gprx_batch_set_train failed ($rc)")
        o = Ref{OptOptions}()
        ccall((:gprx_opt_defaults, LIB), Cvoid, (Ref{OptOptions},), o)
        o[] = OptOptions(o[].m, iterations, max_evals, o[].ls_iterations, o[].scaleinvH0, 0, o[].successive_f_tol,
                         g_abstol, time_limit, o[].alphaguess, o[].c_1, o[].rho_hi, o[].rho_lo)
        thx = similar(th0)
        fmin = zeros(B)
        its, fc, gc, stp = (zeros(Cint, B) for _ in 1:4)
        rounds = Ref{Cint}(0)
        rc = ccall((:gprx_batch_optimize, LIB), Cint,
                   (Ptr{Cvoid}, Ptr{Float64}, Ref{OptOptions}, Ptr{Float64}, Ptr{Float64}, Ptr{Cint}, Ptr{Cint},
                    Ptr{Cint}, Ptr{Cint}, Ref{Cint}),
                   b[], th0, o, thx, fmin, its, fc, gc, stp, rounds)
        rc == OK || error("gprx_batch_optimize failed ($rc)")
        for (k, gp) in enumerate(gps)   # optimize!: set_params!(gp, minimizer); update_target!(gp)
            GaussianProcesses.set_params!(gp, thx[:, k])
            GaussianProcesses.update_mll!(gp)
        end
        return [(minimizer=thx[:, k], minimum=fmin[k], iterations=Int(its[k]), f_calls=Int(fc[k]),
                 g_calls=Int(gc[k]), converged=(stp[k] & 0x100) != 0, stopped_by=STOP[(stp[k] & 0xff) + 1])
                for k in 1:B]
    finally
        ccall((:gprx_batch_destroy, LIB), Cvoid, (Ptr{Cvoid},), b[])
    end
end

end # module
