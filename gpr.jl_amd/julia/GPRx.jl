"""
    GPRx — Julia ccall shim routing GaussianProcesses.jl's exact SE-ARD GP evaluations to the
    MI355X library (libgprx.so, C ABI in include/gprx.h).

Load it after GaussianProcesses (e.g. one `include` in src/GPR.jl, see INTEGRATION.md); the
experiment scripts (examples/noise.jl, examples/hyperparameter.jl) stay textually unchanged:

    GP(X, y, mean, SEArd(...))            -> gprx_gp_create + gprx_gp_lml   (CPnoise.jl:40)
    optimize!(gp, LBFGS(...), Options())  -> gprx_gp_lml / gprx_gp_lml_grad per evaluation
    predict_y(gp, x*)                     -> gprx_gp_predict                 (predictdynamics.jl:13)

Method names follow GaussianProcesses v0.12.4 internals (update_mll!, update_target_and_dtarget!,
predict_f); they are [ext] — confirm against that package's source before shipping.
Not executable in the build container (no Julia runtime).
"""
module GPRx

using GaussianProcesses
using GaussianProcesses: GPE, SEArd, Mean
using LinearAlgebra

const LIB = joinpath(@__DIR__, "..", "lib", "libgprx.so")
const OK, NOT_PD, INVALID = Cint(0), Cint(1), Cint(2)

# one context (HIP stream) per Julia thread; device = thread mod #GPUs (core.jl:28 workers)
const CTX = Dict{Int,Ptr{Cvoid}}()
const CTX_LOCK = ReentrantLock()
function context()
    tid = Threads.threadid()
    lock(CTX_LOCK) do
        get!(CTX, tid) do
            ngpu = parse(Int, get(ENV, "GPRX_NGPU", "1"))
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

function check(rc::Cint, gp)
    rc == NOT_PD && throw(LinearAlgebra.PosDefException(-1))
    rc == INVALID && throw(ArgumentError("gprx: invalid hyperparameters"))
    rc == OK || error("gprx device error ($rc)")
end

# The varargs absorb GaussianProcesses' optional positional arguments (e.g. the precompute buffer
# that optimize! passes to update_target_and_dtarget!) so these methods win dispatch for every
# call form.
function GaussianProcesses.update_mll!(gp::GPE{<:Any,<:Any,<:Mean,<:SEArd}, args...; kwargs...)
    m = Ref{Float64}(0.0)
    check(ccall((:gprx_gp_lml, LIB), Cint, (Ptr{Cvoid}, Ptr{Float64}, Ref{Float64}),
                handle(gp).ptr, theta(gp), m), gp)
    gp.mll = m[]
    gp.target = gp.mll
    gp
end

function GaussianProcesses.update_target_and_dtarget!(gp::GPE{<:Any,<:Any,<:Mean,<:SEArd}, args...; kwargs...)
    m = Ref{Float64}(0.0)
    g = zeros(length(theta(gp)))
    check(ccall((:gprx_gp_lml_grad, LIB), Cint, (Ptr{Cvoid}, Ptr{Float64}, Ref{Float64}, Ptr{Float64}),
                handle(gp).ptr, theta(gp), m, g), gp)
    gp.mll = m[]
    gp.dmll = g
    gp.target = gp.mll
    gp.dtarget = g
    gp
end

function GaussianProcesses.predict_f(gp::GPE{<:Any,<:Any,<:Mean,<:SEArd}, x::AbstractMatrix; full_cov::Bool=false)
    full_cov && error("gprx: full_cov=true is not provided by the device path")
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

end # module
