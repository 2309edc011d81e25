# iLQRHIP.jl — Julia-side drop-in for aabouman/iLQR.jl's hot path over the C ABI of
# libilqr_hip.so (include/ilqr.h). Not executable in this build environment (no Julia
# toolchain); every ccall below is exercised from Python with the same symbols and the
# same memory layouts by tests/test_gpu_julia_layout.py (tests/julia_layout.py restates
# this file's permutedims conventions on Fortran-ordered arrays).
#
# It keeps the reference's public signatures and error behaviour:
#   fit(x_init, u_init, dynamicsf, immediate_cost, final_cost; x_traj, max_iter, tol)
#                                            -> (x̄, ū)          reference src/forward_pass.jl:148-179
#   backward_pass(x, u, dynamicsf, immediate_cost, final_cost)
#                                            -> (δu, K)         reference src/backward_pass.jl:324-357
#   forward_pass(x, u, x_traj, δu, K, prev_cost, dynamicsf, immediate_cost, final_cost)
#                                            -> (x̄, ū, cost)    reference src/forward_pass.jl:55-93
# and dispatches on the closures:
#   * LinearDynamics / QuadraticCost / QuadraticFinalCost  → ILQR_PROBLEM_LQ (all on the GPU);
#   * TwoLinkDynamics{NU} / TwoLinkCost / TwoLinkFinalCost → ILQR_PROBLEM_TWO_LINK (all on the
#     GPU; these callable structs evaluate test/2_link_example/2_link_helper_functions.jl
#     on the host too, so they ARE the reference's closures);
#   * any other Julia closures → ILQR_PROBLEM_TILES: ForwardDiff on the host produces the
#     per-step derivative tiles exactly as the reference's backward_pass.jl:32-33, 95-99,
#     142-143 do, the Riccati recursion runs on the GPU (ilqr_backward_tiles), and the
#     forward pass rolls the user's closure out on the host (a Julia closure cannot run on
#     the device; this is the reference's own forward_pass.jl:70-87 loop with the line
#     search capped).
# The reference's documented per-step API (docs/src/documentation.md:13-51) with its
# signatures: linearize_dynamics (vector and trajectory forms; ilqr_linearize on the device
# for the LQ / 2-link families), immediate_cost_quadratization, final_cost_quadratization,
# optimal_controller_param, feedback_parameters, step_back.
# New API: `solve!(::iLQRProblem)` (batched LQ, one or several GPUs), the resident
# single-GPU `Solver` (set_problem! / fit! / backward! / forward! / solve!, close: one
# workspace reused by every call — fit / backward_pass / forward_pass run on a cached one),
# the resident multi-GPU `MultiSolver`, `chain_fit` (the RBD family of BASELINE config 5) and
# the floating-base family of the reference's RBD script: `FloatingDynamics` /
# `FloatingCost` / `FloatingFinalCost` (floating_closures(model)), which fit /
# backward_pass / forward_pass / linearize_dynamics dispatch to ilqr_floating_* on a cached
# FloatingSolver, and `floating_fit` (batched).
module iLQRHIP

using ForwardDiff: gradient, jacobian, hessian   # as the reference (src/iLQR.jl:3)
using LinearAlgebra: dot

const libilqr = joinpath(@__DIR__, "..", "lib", "libilqr_hip.so")

const ILQR_OK = Int32(0)
const ILQR_ERR_BAD_DIMS = Int32(1)
const ILQR_ERR_NAN = Int32(5)
const ILQR_ERR_LS_EXHAUSTED = Int32(6)
const ILQR_PROBLEM_LQ = Int32(1)
const ILQR_PROBLEM_TWO_LINK = Int32(2)
const ILQR_PROBLEM_TILES = Int32(3)
const ILQR_TRAJ_NAN = Int32(4)

struct Problem               # ilqr_problem
    kind::Int32
    reserved::Int32
    A::Ptr{Float64}
    B::Ptr{Float64}
    Q::Ptr{Float64}
    R::Ptr{Float64}
    Qf::Ptr{Float64}
end

struct Tiles                 # ilqr_tiles: per-step derivatives of an arbitrary problem
    A::Ptr{Float64}; B::Ptr{Float64}; lx::Ptr{Float64}; lu::Ptr{Float64}; lxx::Ptr{Float64}
    lux::Ptr{Float64}; luu::Ptr{Float64}; lfx::Ptr{Float64}; lfxx::Ptr{Float64}
end

struct History               # ilqr_history: device arrays (max_iter × batch), iteration-major
    cost::Ptr{Float64}; trials::Ptr{Int32}; alpha::Ptr{Float64}; du2::Ptr{Float64}
end

mutable struct Options       # ilqr_options
    max_iter::Int32
    max_trials::Int32
    tol::Float64
    mu::Float64
    alpha0::Float64
    shrink::Float64
end

function default_options()
    o = Options(0, 0, 0.0, 0.0, 0.0, 0.0)
    ccall((:ilqr_default_options, libilqr), Cvoid, (Ref{Options},), o)
    return o
end

"""The reference's line search (forward_pass.jl:70-87) loops forever when no step lowers
the cost; the device stops after `max_trials` halvings and the shim throws this."""
struct LineSearchExhausted <: Exception end

# -- the reference's callbacks, as recognisable callable structs ------------------
struct LinearDynamics{M<:AbstractMatrix}; A::M; B::M; end
(f::LinearDynamics)(x, u) = f.A * x + f.B * u                      # dynamicsf(x, u)
struct QuadraticCost{M<:AbstractMatrix}; Q::M; R::M; end
(l::QuadraticCost)(x, u) = x' * l.Q * x + u' * l.R * u             # immediate_cost(x, u)
struct QuadraticFinalCost{M<:AbstractMatrix}; Qf::M; end
(l::QuadraticFinalCost)(x) = x' * l.Qf * x                         # final_cost(x)

# test/2_link_example/2_link_helper_functions.jl:4-108 with the same expression order
# (the CoriolisMatrix quirk `for k in length(θ)` → k = 2 only, :42-44). NU = 1 is the
# build-defined f(x, [u₁, 0]) of BASELINE configs 1-2 (not reference-pinned).
module TwoLinkConsts
    const l₁ = sqrt(2.) / 2.; const l₂ = sqrt(2.) / 2.
    const r₁ = 0.5 * l₁; const r₂ = 0.5 * l₂
    const m₁ = 1.0; const m₂ = 1.0
    const Iz1 = 1.0 / 12.0 * m₁ * l₁^2; const Iz2 = 1.0 / 12.0 * m₂ * l₂^2
    const α = Iz1 + Iz2 + m₁ * r₁^2 + m₂ * (l₁^2 + r₂^2)
    const β = m₂ * l₁ * r₂
    const δ = Iz2 + m₂ * r₂^2
    const Δt = 0.01
    function ik(x, y)                                               # InverseKinematics (:19-26)
        q₂ = acos((x^2 + y^2 - l₁^2 - l₂^2) / (2 * l₁ * l₂))
        q₁ = atan(y, x) - atan(l₂ * sin(q₂), l₁ + l₂ * cos(q₂))
        return [q₁, q₂]
    end
    const θstar = ik(0.6, -0.5)                                     # target_tool_loc (:16)
end

struct TwoLinkDynamics{NU} end
TwoLinkDynamics(nu::Integer=2) = (nu in (1, 2) || throw(ArgumentError("nu ∈ (1, 2)")); TwoLinkDynamics{nu}())
function _tl_continuous(x, w)
    C = TwoLinkConsts
    c2 = cos(x[2]); s2 = sin(x[2])
    M = [C.α+2*C.β*c2 C.δ+C.β*c2; C.δ+C.β*c2 C.δ]                 # InertiaMatrix (:29-33)
    dM11 = 2 * C.β * -s2; dM12 = C.β * -s2                          # ∂M/∂θ₂ (the nested jacobian, :37)
    Cm = [1/2*dM11*x[4] 1/2*dM12*x[4]; 1/2*dM12*x[4] zero(dM11)]   # CoriolisMatrix, k = 2 only
    acc = -(M \ Cm) * x[3:4] + inv(M) * w                           # :56-66
    return [x[3], x[4], acc[1], acc[2]]
end
function (f::TwoLinkDynamics{NU})(x, u) where {NU}                 # RK4 (:71-78)
    w = NU == 2 ? u : [u[1], zero(eltype(u))]
    Δt = TwoLinkConsts.Δt
    k1 = Δt * _tl_continuous(x, w)
    k2 = Δt * _tl_continuous(x + k1 / 2, w)
    k3 = Δt * _tl_continuous(x + k2 / 2, w)
    k4 = Δt * _tl_continuous(x + k3, w)
    return x + (1 / 6) * (k1 + 2 * k2 + 2 * k3 + k4)
end
struct TwoLinkCost end                                              # immediate_cost (:82-97)
(::TwoLinkCost)(x, u) = sum((TwoLinkConsts.θstar .- x[1:2]) .^ 2) * 1.0 + sum(u .^ 2) * 1.0
struct TwoLinkFinalCost end                                         # final_cost (:100-108)
(::TwoLinkFinalCost)(x) = sum((TwoLinkConsts.θstar .- x[1:2]) .^ 2) * 1.0

function check(st, what)
    st == ILQR_OK && return nothing
    st == ILQR_ERR_BAD_DIMS && throw(AssertionError("N == M+1"))           # backward_pass.jl:329
    st == ILQR_ERR_NAN && throw(AssertionError("!any(isnan, ...)"))        # backward_pass.jl:353, forward_pass.jl:89
    st == ILQR_ERR_LS_EXHAUSTED && throw(LineSearchExhausted())
    error("$what: " * unsafe_string(ccall((:ilqr_status_string, libilqr), Cstring, (Cint,), st)))
end

# a handle bound to device 0 plus the device buffers it owns (freed with it)
mutable struct Handle
    ptr::Ptr{Cvoid}
    bufs::Vector{Ptr{Cvoid}}
end

function Handle(nx, nu, T, batch; device=0)
    r = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:ilqr_create, libilqr), Cint, (Ref{Ptr{Cvoid}}, Cint, Cint, Cint, Cint, Cint),
                r, device, nx, nu, T, batch), "ilqr_create")
    h = Handle(r[], Ptr{Cvoid}[])
    finalizer(close, h)       # a backstop: Solver and the per-call paths close explicitly
    return h
end

"""close(h): free the handle's device buffers and its workspace now (idempotent)."""
function Base.close(h::Handle)
    h.ptr == C_NULL && return nothing
    for p in h.bufs; ccall((:ilqr_free, libilqr), Cint, (Ptr{Cvoid}, Ptr{Cvoid}), h.ptr, p); end
    empty!(h.bufs)
    ccall((:ilqr_destroy, libilqr), Cint, (Ptr{Cvoid},), h.ptr)
    h.ptr = C_NULL
    return nothing
end

# launch schedule of the LQ family (include/ilqr.h: ILQR_SCHED_*)
const ILQR_SCHED_PIPELINED = Int32(1)
const ILQR_SCHED_RING_FORWARD = Int32(2)
const ILQR_SCHED_BACKWARD_WAVE = Int32(4)
const ILQR_SCHED_BACKWARD_BLOCK = Int32(8)
const ILQR_SCHED_FUSED = Int32(16)
const ILQR_SCHED_FORWARD_MFMA = Int32(32)
const ILQR_SCHED_SEQUENTIAL_SEARCH = Int32(64)
set_schedule!(h::Handle, flags::Integer) =
    check(ccall((:ilqr_set_schedule, libilqr), Cint, (Ptr{Cvoid}, Cint), h.ptr, flags), "ilqr_set_schedule")

function alloc(h::Handle, T::Type, n)
    p = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:ilqr_malloc, libilqr), Cint, (Ptr{Cvoid}, Csize_t, Ref{Ptr{Cvoid}}), h.ptr, max(n, 1) * sizeof(T), p), "ilqr_malloc")
    push!(h.bufs, p[])
    return Ptr{T}(p[])
end

function upload(h::Handle, a::Array{T}) where {T}
    p = alloc(h, T, length(a))
    check(ccall((:ilqr_memcpy_h2d, libilqr), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Csize_t),
                h.ptr, p, a, sizeof(a)), "ilqr_memcpy_h2d")
    return p
end

# into an existing device buffer (the resident Solver: no allocation)
function upload!(h::Handle, p::Ptr, a::Array)
    check(ccall((:ilqr_memcpy_h2d, libilqr), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Csize_t),
                h.ptr, p, a, sizeof(a)), "ilqr_memcpy_h2d")
    return p
end

function release!(h::Handle, p::Ptr)
    i = findfirst(==(Ptr{Cvoid}(p)), h.bufs)
    i === nothing && return nothing
    ccall((:ilqr_free, libilqr), Cint, (Ptr{Cvoid}, Ptr{Cvoid}), h.ptr, p)
    deleteat!(h.bufs, i)
    return nothing
end

function download!(h::Handle, a::Array, p::Ptr)
    check(ccall((:ilqr_memcpy_d2h, libilqr), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Csize_t),
                h.ptr, a, p, sizeof(a)), "ilqr_memcpy_d2h")
    return a
end

# -- layouts ------------------------------------------------------------------------
# The reference's per-trajectory matrices are row-per-timestep (x::(N × nx), column-
# major: time fastest). The ABI's trajectory is C row-major (N, nx) = Julia (nx, N):
# permutedims for one trajectory, no copy for batched (nx, N, batch) arrays. A C
# row-major (r, c) matrix is the Julia transpose; K (T, nu, nx) row-major comes back
# as Julia (nx, nu, T) and is permuted to the reference's 𝐊s (T × nu × nx).
to_abi(x::AbstractMatrix) = Array{Float64}(permutedims(x))
from_abi(a::AbstractMatrix) = permutedims(a)
gains_from_abi(K::Array{Float64,3}) = permutedims(K, (3, 2, 1))
gains_to_abi(K::AbstractArray{<:Real,3}) = Array{Float64}(permutedims(K, (3, 2, 1)))
rowmajor(M::AbstractMatrix) = Array{Float64}(permutedims(M))
# batched per-instance matrices (r, c, batch) → C (batch, r, c): each matrix transposed
rowmajor3(A::AbstractArray{<:Real,3}) = Array{Float64}(permutedims(A, (2, 1, 3)))

# -- problem families -----------------------------------------------------------------
const LQTriple = Tuple{LinearDynamics,QuadraticCost,QuadraticFinalCost}
const TwoLinkTriple = Tuple{TwoLinkDynamics,TwoLinkCost,TwoLinkFinalCost}
family(f, l, lf) = (f, l, lf) isa LQTriple ? :lq : (f, l, lf) isa TwoLinkTriple ? :two_link :
                   is_floating(f, l, lf) ? :floating : :tiles

function problem(h::Handle, f::LinearDynamics, l::QuadraticCost, lf::QuadraticFinalCost)
    return Problem(ILQR_PROBLEM_LQ, 0, upload(h, rowmajor(f.A)), upload(h, rowmajor(f.B)),
                   upload(h, rowmajor(l.Q)), upload(h, rowmajor(l.R)), upload(h, rowmajor(lf.Qf)))
end
problem(h::Handle, f::TwoLinkDynamics, l::TwoLinkCost, lf::TwoLinkFinalCost) =
    Problem(ILQR_PROBLEM_TWO_LINK, 0, C_NULL, C_NULL, C_NULL, C_NULL, C_NULL)

nu_of(::TwoLinkDynamics{NU}) where {NU} = NU

# Per-step derivative tiles of arbitrary closures on the host, exactly the reference's
# calls: linearize_dynamics (backward_pass.jl:32-33), immediate_cost_quadratization
# (:95-99; 𝐏 = jacobian of ∂L∂u w.r.t. x, nu × nx) and final_cost_quadratization
# (:142-143). Returned in the ABI's row-major per-step layout (ilqr_tiles).
function derivative_tiles(x::AbstractMatrix, u::AbstractMatrix, f, ℓ, ℓf)
    N, nx = size(x); M, nu = size(u)
    A = zeros(nx, nx, M); B = zeros(nu, nx, M); lx = zeros(nx, M); lu = zeros(nu, M)
    lxx = zeros(nx, nx, M); lux = zeros(nx, nu, M); luu = zeros(nu, nu, M)
    for i in 1:M
        xi = x[i, :]; ui = u[i, :]
        A[:, :, i] = permutedims(jacobian(z -> f(z, ui), xi))          # :32
        B[:, :, i] = permutedims(jacobian(v -> f(xi, v), ui))          # :33
        ∂L∂u(z, v) = gradient(w -> ℓ(z, w), v)
        lx[:, i] = gradient(z -> ℓ(z, ui), xi)                          # :95
        lu[:, i] = ∂L∂u(xi, ui)                                         # :96
        lxx[:, :, i] = permutedims(hessian(z -> ℓ(z, ui), xi))          # :97
        lux[:, :, i] = permutedims(jacobian(z -> ∂L∂u(z, ui), xi))      # :98 (𝐏, nu × nx)
        luu[:, :, i] = permutedims(hessian(v -> ℓ(xi, v), ui))          # :99
    end
    xN = x[N, :]
    lfx = gradient(ℓf, xN)                                              # :142
    lfxx = permutedims(hessian(ℓf, xN))                                 # :143
    return (A=A, B=B, lx=lx, lu=lu, lxx=lxx, lux=lux, luu=luu, lfx=lfx, lfxx=lfxx)
end

# backward_pass on the resident tiles workspace of this shape (TilesSolver, cached): the
# host tiles go into buffers allocated once, so fit_tiles' iterations allocate nothing
# on the device
function backward_tiles_device(x::AbstractMatrix, u::AbstractMatrix, f, ℓ, ℓf)
    N, nx = size(x); M, nu = size(u)
    t = derivative_tiles(x, u, f, ℓ, ℓf)
    return with_cached(TILES_CACHE, () -> TilesSolver(nx, nu, M), (nx, nu, M)) do s
        for (p, a) in ((s.tl.A, t.A), (s.tl.B, t.B), (s.tl.lx, t.lx), (s.tl.lu, t.lu), (s.tl.lxx, t.lxx),
                       (s.tl.lux, t.lux), (s.tl.luu, t.luu), (s.tl.lfx, t.lfx), (s.tl.lfxx, t.lfxx))
            upload!(s.h, p, a)
        end
        check(ccall((:ilqr_backward_tiles, libilqr), Cint,
                    (Ptr{Cvoid}, Ref{Tiles}, Ref{Options}, Ptr{Float64}, Ptr{Float64}, Ptr{Int32}),
                    s.h.ptr, Ref(s.tl), default_options(), s.d, s.K, s.status), "ilqr_backward_tiles")
        (from_abi(download!(s.h, zeros(nu, M), s.d)), gains_from_abi(download!(s.h, zeros(nx, nu, M), s.K)))
    end
end

"""backward_pass(x, u, dynamicsf, immediate_cost, final_cost) -> (δu::T×nu, K::T×nu×nx)"""
function backward_pass(x::AbstractMatrix, u::AbstractMatrix, dynamicsf, immediate_cost, final_cost)
    N, nx = size(x); M, nu = size(u)
    @assert(N == M + 1)                                                 # backward_pass.jl:329
    fam = family(dynamicsf, immediate_cost, final_cost)
    fam == :tiles && return backward_tiles_device(x, u, dynamicsf, immediate_cost, final_cost)
    fam == :floating && return floating_backward(dynamicsf, x, u)
    # the resident solver of this shape (no allocation per call): δu (T × nu), K (T × nu × nx) like 𝐊s
    return with_cached(SOLVER_CACHE, () -> Solver(nx, nu, M, 1), (nx, nu, M)) do s
        backward!(set_problem!(s, dynamicsf, immediate_cost, final_cost), x, u)
    end
end

# total_cost_generator (forward_pass.jl:182-196), for the host rollout of the tiles path
function total_cost(x̄, ū, x_traj, ℓ, ℓf)
    s = 0.
    for i in 1:size(ū, 1)
        s += ℓ(x̄[i, :] - x_traj[i, :], ū[i, :])
    end
    return s + ℓf(x̄[end, :])
end

# forward_pass.jl:55-93 for a closure the device cannot run: the reference's loop on the
# host (it must call the user's Julia dynamicsf), the unbounded search capped at max_trials
function forward_host(x, u, x_traj, δu, K, prev_cost, f, ℓ, ℓf; max_trials=default_options().max_trials)
    N, nx = size(x); M, nu = size(u)
    x̄ = zeros(eltype(x), N, nx); ū = zeros(eltype(u), M, nu)
    x̄[1, :] .= x[1, :]
    α = 1.0; new_cost = 0.0
    for trial in 1:max_trials
        for k in 1:M
            δx = x̄[k, :] - x[k, :]
            ū[k, :] .= u[k, :] + α * δu[k, :] + K[k, :, :] * δx
            x̄[k+1, :] .= f(x̄[k, :], ū[k, :])
        end
        new_cost = total_cost(x̄, ū, x_traj, ℓ, ℓf)
        prev_cost - new_cost > 0 && break
        trial == max_trials && throw(LineSearchExhausted())
        α /= 2
    end
    @assert !any(isnan, ū)                                              # forward_pass.jl:89
    @assert !any(isnan, x̄)                                              # forward_pass.jl:90
    return (x̄, ū, new_cost)
end

"""forward_pass(x, u, x_traj, δu, K, prev_cost, dynamicsf, immediate_cost, final_cost) -> (x̄, ū, new_cost)"""
function forward_pass(x::AbstractMatrix, u::AbstractMatrix, x_traj::AbstractMatrix, δu::AbstractMatrix,
                      K::AbstractArray{<:Real,3}, prev_cost::Real, dynamicsf, immediate_cost, final_cost)
    N, nx = size(x); M, nu = size(u)
    @assert(N == M + 1)                                                 # forward_pass.jl:62
    fam = family(dynamicsf, immediate_cost, final_cost)
    fam == :tiles && return forward_host(x, u, x_traj, δu, K, prev_cost, dynamicsf, immediate_cost, final_cost)
    fam == :floating && return floating_forward(dynamicsf, x, u, x_traj, δu, K, prev_cost)
    return with_cached(SOLVER_CACHE, () -> Solver(nx, nu, M, 1), (nx, nu, M)) do s
        forward!(set_problem!(s, dynamicsf, immediate_cost, final_cost), x, u, x_traj, δu, K, prev_cost)
    end
end

# the reference's per-iteration line (forward_pass.jl:167), from a fit's history
function print_history(cost::AbstractVector, trials::AbstractVector)
    for i in eachindex(trials)
        trials[i] == 0 && break
        println("Iteration: ", i, "\t\tTotal Cost: ", cost[i])
    end
end

"""fit(x_init, u_init, dynamicsf, immediate_cost, final_cost; x_traj, max_iter, tol, verbose) -> (x̄, ū)

verbose = true prints the reference's `Iteration: i  Total Cost: c` line for every
iteration (forward_pass.jl:167), from the device fit's history (ilqr_fit_ex)."""
function fit(x_init::AbstractMatrix, u_init::AbstractMatrix, dynamicsf, immediate_cost, final_cost;
             x_traj=zero(x_init), max_iter::Int64=100, tol::Float64=1e-6, verbose::Bool=false)
    N, nx = size(x_init); M, nu = size(u_init)
    @assert(N == M + 1, "size(x_init)[2] == size(u_init)[1]")          # forward_pass.jl:156
    fam = family(dynamicsf, immediate_cost, final_cost)
    fam == :tiles &&
        return fit_tiles(x_init, u_init, dynamicsf, immediate_cost, final_cost, x_traj, max_iter, tol, verbose)
    fam == :floating && return floating_fit1(dynamicsf, x_init, u_init, x_traj, max_iter, tol, verbose)
    # the resident solver of this shape: an MPC loop calling fit allocates nothing per call;
    # an exhausted line search returns the last iterate (fit_resident!)
    return with_cached(SOLVER_CACHE, () -> Solver(nx, nu, M, 1), (nx, nu, M)) do s
        fit!(set_problem!(s, dynamicsf, immediate_cost, final_cost), x_init, u_init;
             x_traj=x_traj, max_iter=max_iter, tol=tol, verbose=verbose)
    end
end

# fit (forward_pass.jl:148-179) for arbitrary closures: tiles backward on the GPU, host
# rollout; same return semantics (the iterate before the update that met tol, :171)
function fit_tiles(x_init, u_init, f, ℓ, ℓf, x_traj, max_iter, tol, verbose=false)
    x̄ⁱ = x_init; ūⁱ = u_init
    prev_cost = Inf
    for iter in 1:max_iter
        δu, K = backward_tiles_device(x̄ⁱ, ūⁱ, f, ℓ, ℓf)                 # :162
        x̄ⁱ⁺¹, ūⁱ⁺¹, new_cost = try                                      # :163-166
            forward_host(x̄ⁱ, ūⁱ, x_traj, δu, K, prev_cost, f, ℓ, ℓf)
        catch e
            e isa LineSearchExhausted && break     # the reference would loop forever here
            rethrow()
        end
        verbose && println("Iteration: ", iter, "\t\tTotal Cost: ", new_cost)   # :167
        @assert(prev_cost > new_cost); prev_cost = new_cost             # :168
        convert(Float64, sum((ūⁱ⁺¹ - ūⁱ) .^ 2)) <= tol && break          # :171
        x̄ⁱ = x̄ⁱ⁺¹; ūⁱ = ūⁱ⁺¹                                           # :174-175
    end
    return (x̄ⁱ, ūⁱ)
end

"""Batched problem (new API): per-instance A (nx,nx,B) … and trajectories (nx, N, B)."""
struct iLQRProblem
    A::Array{Float64,3}; B::Array{Float64,3}; Q::Array{Float64,3}; R::Array{Float64,3}; Qf::Array{Float64,3}
    x::Array{Float64,3}; u::Array{Float64,3}
end

"""solve!(prob; max_iter, tol, history): fits every instance; overwrites prob.x / prob.u.
history = true returns (prob, h) with h the per-iteration record (ilqr_fit_ex): Julia
arrays (batch, max_iter) `cost`, `trials`, `alpha`, `du2` (include/ilqr.h ilqr_history)."""
function solve!(prob::iLQRProblem; max_iter::Int64=100, tol::Float64=1e-6, history::Bool=false)
    nx, N, nb = size(prob.x); nu = size(prob.u, 1); M = N - 1
    h = Handle(nx, nu, M, nb)
    p = Ref(Problem(ILQR_PROBLEM_LQ, 0, upload(h, rowmajor3(prob.A)), upload(h, rowmajor3(prob.B)),
                    upload(h, rowmajor3(prob.Q)), upload(h, rowmajor3(prob.R)), upload(h, rowmajor3(prob.Qf))))
    o = default_options(); o.max_iter = max_iter; o.tol = tol
    xi = upload(h, prob.x); ui = upload(h, prob.u)                      # (nx, N, B) is the ABI layout as is
    xo = alloc(h, Float64, length(prob.x)); uo = alloc(h, Float64, length(prob.u))
    n = max(max_iter, 1)
    # (max_iter, batch) row-major = Julia (batch, max_iter): no permute on the way back
    hd = history ? (alloc(h, Float64, n * nb), upload(h, zeros(Int32, n * nb)), alloc(h, Float64, n * nb),
                    alloc(h, Float64, n * nb)) : (C_NULL, C_NULL, C_NULL, C_NULL)
    hist = Ref(History(hd...))
    st = ccall((:ilqr_fit_ex, libilqr), Cint,
               (Ptr{Cvoid}, Ref{Problem}, Ref{Options}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64},
                Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Int32}, Ptr{Int32}, Ref{History}),
               h.ptr, p, o, xi, ui, C_NULL, xo, uo, C_NULL, C_NULL, C_NULL, hist)
    st in (ILQR_OK, ILQR_ERR_LS_EXHAUSTED) || check(st, "ilqr_fit")
    download!(h, prob.x, xo); download!(h, prob.u, uo)
    history || return prob
    return prob, (cost=download!(h, zeros(nb, n), hd[1]), trials=download!(h, zeros(Int32, nb, n), hd[2]),
                  alpha=download!(h, zeros(nb, n), hd[3]), du2=download!(h, zeros(nb, n), hd[4]))
end

"""solve!(prob, devices; …): the same over several GPUs of this node in one process
(ilqr_multi_fit: contiguous blocks of instances per device, host arrays in and out)."""
function solve!(prob::iLQRProblem, devices::Vector{Int}; max_iter::Int64=100, tol::Float64=1e-6)
    nx, N, nb = size(prob.x); nu = size(prob.u, 1); M = N - 1
    r = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:ilqr_multi_create, libilqr), Cint,
                (Ref{Ptr{Cvoid}}, Ptr{Cint}, Cint, Cint, Cint, Cint, Cint),
                r, Cint.(devices), length(devices), nx, nu, M, nb), "ilqr_multi_create")
    A, B, Q, R, Qf = rowmajor3(prob.A), rowmajor3(prob.B), rowmajor3(prob.Q), rowmajor3(prob.R), rowmajor3(prob.Qf)
    try
        GC.@preserve A B Q R Qf begin
            p = Ref(Problem(ILQR_PROBLEM_LQ, 0, pointer(A), pointer(B), pointer(Q), pointer(R), pointer(Qf)))
            o = default_options(); o.max_iter = max_iter; o.tol = tol
            xo = similar(prob.x); uo = similar(prob.u)
            st = ccall((:ilqr_multi_fit, libilqr), Cint,
                       (Ptr{Cvoid}, Ref{Problem}, Ref{Options}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64},
                        Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Int32}, Ptr{Int32}),
                       r[], p, o, prob.x, prob.u, C_NULL, xo, uo, C_NULL, C_NULL, C_NULL)
            st in (ILQR_OK, ILQR_ERR_LS_EXHAUSTED) || check(st, "ilqr_multi_fit")
            prob.x .= xo; prob.u .= uo
        end
    finally
        ccall((:ilqr_multi_destroy, libilqr), Cint, (Ptr{Cvoid},), r[])
    end
    return prob
end

"""MultiSolver(prob, devices): a device-resident multi-GPU solver for an MPC loop over
many instances (ilqr_multi_set_problem once: A…Qf stay on their devices; then per call
only x/u go up and the results come down — ilqr_multi_load / ilqr_multi_fit_resident /
ilqr_multi_gather). close(ms) frees it."""
mutable struct MultiSolver
    ptr::Ptr{Cvoid}
    nx::Int; nu::Int; M::Int; nb::Int
end

const ILQR_MULTI_WARM_START = Cint(1)

function MultiSolver(prob::iLQRProblem, devices::Vector{Int})
    nx, N, nb = size(prob.x); nu = size(prob.u, 1); M = N - 1
    r = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:ilqr_multi_create, libilqr), Cint,
                (Ref{Ptr{Cvoid}}, Ptr{Cint}, Cint, Cint, Cint, Cint, Cint),
                r, Cint.(devices), length(devices), nx, nu, M, nb), "ilqr_multi_create")
    ms = MultiSolver(r[], nx, nu, M, nb)
    A, B, Q, R, Qf = rowmajor3(prob.A), rowmajor3(prob.B), rowmajor3(prob.Q), rowmajor3(prob.R), rowmajor3(prob.Qf)
    GC.@preserve A B Q R Qf begin
        p = Ref(Problem(ILQR_PROBLEM_LQ, 0, pointer(A), pointer(B), pointer(Q), pointer(R), pointer(Qf)))
        check(ccall((:ilqr_multi_set_problem, libilqr), Cint, (Ptr{Cvoid}, Ref{Problem}), ms.ptr, p),
              "ilqr_multi_set_problem")
    end
    return ms
end

function Base.close(ms::MultiSolver)
    ms.ptr == C_NULL && return
    ccall((:ilqr_multi_destroy, libilqr), Cint, (Ptr{Cvoid},), ms.ptr)
    ms.ptr = C_NULL
end

"""solve!(ms::MultiSolver, prob; max_iter, tol, warm_start) -> prob: fit every instance
on the resident problem. warm_start = false uploads prob.x / prob.u first (the usual
fit from (x_init, u_init)); true starts from the previous call's results, which never
left the devices. prob.x / prob.u receive the results (ilqr_multi_gather)."""
function solve!(ms::MultiSolver, prob::iLQRProblem; max_iter::Int64=100, tol::Float64=1e-6,
                warm_start::Bool=false)
    size(prob.x) == (ms.nx, ms.M + 1, ms.nb) && size(prob.u) == (ms.nu, ms.M, ms.nb) ||
        throw(AssertionError("problem shape differs from the MultiSolver's"))
    if !warm_start
        check(ccall((:ilqr_multi_load, libilqr), Cint, (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}),
                    ms.ptr, prob.x, prob.u, C_NULL), "ilqr_multi_load")
    end
    o = default_options(); o.max_iter = max_iter; o.tol = tol
    st = ccall((:ilqr_multi_fit_resident, libilqr), Cint, (Ptr{Cvoid}, Ref{Options}, Cint, Ptr{Cvoid}),
               ms.ptr, o, warm_start ? ILQR_MULTI_WARM_START : Cint(0), C_NULL)
    st in (ILQR_OK, ILQR_ERR_LS_EXHAUSTED) || check(st, "ilqr_multi_fit_resident")
    check(ccall((:ilqr_multi_gather, libilqr), Cint,
                (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Int32}, Ptr{Int32}),
                ms.ptr, prob.x, prob.u, C_NULL, C_NULL, C_NULL), "ilqr_multi_gather")
    return prob
end

# -- resident single-device solver ------------------------------------------------------
"""Solver(nx, nu, T, batch; device = 0): one GPU, one ilqr_create workspace, and every
device buffer a call needs — the problem (A, B, Q, R, Qf), the trajectories, x_traj, the
results, the gains — allocated ONCE here and reused by every call (include/ilqr.h: "hot
calls never allocate"), for an MPC loop calling fit over and over (forward_pass.jl:148-179).
The history scratch of verbose fits grows on demand. close(s) frees everything at once;
the finalizer is only a backstop. The functional fit / backward_pass / forward_pass above
run on a cached Solver per shape (with_cached; clear_cache!() closes them)."""
mutable struct Solver
    h::Handle
    nx::Int; nu::Int; M::Int; nb::Int
    kind::Int32
    A::Ptr{Float64}; B::Ptr{Float64}; Q::Ptr{Float64}; R::Ptr{Float64}; Qf::Ptr{Float64}
    x::Ptr{Float64}; u::Ptr{Float64}; xt::Ptr{Float64}; xo::Ptr{Float64}; uo::Ptr{Float64}
    d::Ptr{Float64}; K::Ptr{Float64}; pc::Ptr{Float64}; cost::Ptr{Float64}
    iters::Ptr{Int32}; status::Ptr{Int32}; trials::Ptr{Int32}
    hc::Ptr{Float64}; ht::Ptr{Int32}; hcap::Int
    lA::Ptr{Float64}; lB::Ptr{Float64}   # linearize_dynamics' outputs, allocated on first use
    lock::ReentrantLock      # held by the functional entry points for a whole call (with_cached)
end

function Solver(nx::Integer, nu::Integer, T::Integer, batch::Integer; device::Integer=0)
    h = Handle(nx, nu, T, batch; device=device)
    N = T + 1
    f(n) = alloc(h, Float64, batch * n)
    i(n) = alloc(h, Int32, batch * n)
    return Solver(h, nx, nu, T, batch, Int32(0),
                  f(nx * nx), f(nx * nu), f(nx * nx), f(nu * nu), f(nx * nx),     # A B Q R Qf
                  f(N * nx), f(T * nu), f(N * nx), f(N * nx), f(T * nu),         # x u x_traj x̄ ū
                  f(T * nu), f(T * nu * nx), f(1), f(1),                          # δu K prev_cost cost
                  i(1), i(1), i(1),                                               # iters status trials
                  Ptr{Float64}(C_NULL), Ptr{Int32}(C_NULL), 0,
                  Ptr{Float64}(C_NULL), Ptr{Float64}(C_NULL), ReentrantLock())
end

function ensure_linearize!(s::Solver)
    if s.lA == C_NULL
        s.lA = alloc(s.h, Float64, s.nb * s.M * s.nx * s.nx); s.lB = alloc(s.h, Float64, s.nb * s.M * s.nx * s.nu)
    end
    return s
end

Base.close(s::Solver) = lock(() -> close(s.h), s.lock)

"""TilesSolver(nx, nu, T): the resident workspace of the arbitrary-closure path — a handle
and the device buffers of one trajectory's derivative tiles (ilqr_tiles: A, B, lx, lu,
lxx, lux, luu, lfx, lfxx) and its gains (δu, K, status), allocated once per shape and
reused by every backward_pass / fit iteration (include/ilqr.h: "hot calls never
allocate"). Shapes: every nx ≤ 16, nu ≤ 8 — the reference's RBD caller is 16 × 8 at
T = 1000 (test/RBD_2_link_example/animate_RBD_2_link.jl:8,19-20,31)."""
mutable struct TilesSolver
    h::Handle
    nx::Int; nu::Int; M::Int
    tl::Tiles
    d::Ptr{Float64}; K::Ptr{Float64}; status::Ptr{Int32}
    lock::ReentrantLock
end

function TilesSolver(nx::Integer, nu::Integer, T::Integer; device::Integer=0)
    h = Handle(nx, nu, T, 1; device=device)
    f(n) = alloc(h, Float64, n)
    tl = Tiles(f(T * nx * nx), f(T * nx * nu), f(T * nx), f(T * nu), f(T * nx * nx),   # A B lx lu lxx
               f(T * nu * nx), f(T * nu * nu), f(nx), f(nx * nx))                      # lux luu lfx lfxx
    return TilesSolver(h, nx, nu, T, tl, f(T * nu), f(T * nu * nx), alloc(h, Int32, 1), ReentrantLock())
end

Base.close(s::TilesSolver) = lock(() -> close(s.h), s.lock)

problem_ref(s::Solver) = Ref(s.kind == ILQR_PROBLEM_LQ ? Problem(ILQR_PROBLEM_LQ, 0, s.A, s.B, s.Q, s.R, s.Qf) :
                                                       Problem(s.kind, 0, C_NULL, C_NULL, C_NULL, C_NULL, C_NULL))

"""set_problem!(s, dynamicsf, immediate_cost, final_cost): the problem the next calls
solve — LQ matrices copied into the resident buffers (batch 1: one instance), or the
2-link arm (nothing to copy)."""
function set_problem!(s::Solver, f::LinearDynamics, l::QuadraticCost, lf::QuadraticFinalCost)
    s.nb == 1 || throw(ArgumentError("one instance per call: set_problem!(s, ::iLQRProblem) for batches"))
    upload!(s.h, s.A, rowmajor(f.A)); upload!(s.h, s.B, rowmajor(f.B)); upload!(s.h, s.Q, rowmajor(l.Q))
    upload!(s.h, s.R, rowmajor(l.R)); upload!(s.h, s.Qf, rowmajor(lf.Qf))
    s.kind = ILQR_PROBLEM_LQ
    return s
end
function set_problem!(s::Solver, f::TwoLinkDynamics{NU}, ::TwoLinkCost, ::TwoLinkFinalCost) where {NU}
    (s.nx, s.nu) == (4, NU) || throw(AssertionError("the 2-link arm is (4, $NU), the solver ($(s.nx), $(s.nu))"))
    s.kind = ILQR_PROBLEM_TWO_LINK
    return s
end
function set_problem!(s::Solver, prob::iLQRProblem)
    upload!(s.h, s.A, rowmajor3(prob.A)); upload!(s.h, s.B, rowmajor3(prob.B)); upload!(s.h, s.Q, rowmajor3(prob.Q))
    upload!(s.h, s.R, rowmajor3(prob.R)); upload!(s.h, s.Qf, rowmajor3(prob.Qf))
    s.kind = ILQR_PROBLEM_LQ
    return s
end

function ensure_history!(s::Solver, n::Int)
    if s.hcap < n
        s.hc != C_NULL && (release!(s.h, s.hc); release!(s.h, s.ht))
        s.hc = alloc(s.h, Float64, n * s.nb); s.ht = alloc(s.h, Int32, n * s.nb); s.hcap = n
    end
    upload!(s.h, s.ht, zeros(Int32, n * s.nb))   # rows past the last iteration read as "not run"
    return Ref(History(s.hc, s.ht, C_NULL, C_NULL))
end

# ilqr_fit_ex from the resident (x, u, x_traj) into the resident results
function fit_resident!(s::Solver, max_iter::Int64, tol::Float64, verbose::Bool)
    s.kind == 0 && throw(ArgumentError("set_problem! first"))
    o = default_options(); o.max_iter = max_iter; o.tol = tol
    n = max(max_iter, 1)
    hist = verbose ? ensure_history!(s, n) : Ref(History(C_NULL, C_NULL, C_NULL, C_NULL))
    st = ccall((:ilqr_fit_ex, libilqr), Cint,
               (Ptr{Cvoid}, Ref{Problem}, Ref{Options}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64},
                Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Int32}, Ptr{Int32}, Ref{History}),
               s.h.ptr, problem_ref(s), o, s.x, s.u, s.xt, s.xo, s.uo, s.cost, s.iters, s.status, hist)
    st in (ILQR_OK, ILQR_ERR_LS_EXHAUSTED) || check(st, "ilqr_fit")
    if verbose
        c = download!(s.h, zeros(s.nb, n), s.hc); t = download!(s.h, zeros(Int32, s.nb, n), s.ht)
        for b in 1:s.nb; print_history(c[b, :], t[b, :]); end
    end
    return st
end

"""fit!(s, x_init, u_init; x_traj, max_iter, tol, verbose) -> (x̄, ū): iLQR.fit
(forward_pass.jl:148-179) of one trajectory (reference layout) on the resident solver."""
function fit!(s::Solver, x_init::AbstractMatrix, u_init::AbstractMatrix; x_traj=zero(x_init),
              max_iter::Int64=100, tol::Float64=1e-6, verbose::Bool=false)
    N, nx = size(x_init); M, nu = size(u_init)
    @assert(N == M + 1, "size(x_init)[2] == size(u_init)[1]")          # forward_pass.jl:156
    (nx, nu, M, 1) == (s.nx, s.nu, s.M, s.nb) || throw(AssertionError("shape differs from the Solver's"))
    upload!(s.h, s.x, to_abi(x_init)); upload!(s.h, s.u, to_abi(u_init)); upload!(s.h, s.xt, to_abi(x_traj))
    fit_resident!(s, max_iter, tol, verbose)
    return from_abi(download!(s.h, zeros(nx, N), s.xo)), from_abi(download!(s.h, zeros(nu, M), s.uo))
end

"""solve!(s::Solver, prob; max_iter, tol) -> prob: the batched fit of solve!(prob) on the
resident solver (set_problem!(s, prob) first, or here with set = true)."""
function solve!(s::Solver, prob::iLQRProblem; max_iter::Int64=100, tol::Float64=1e-6, set::Bool=false)
    size(prob.x) == (s.nx, s.M + 1, s.nb) && size(prob.u) == (s.nu, s.M, s.nb) ||
        throw(AssertionError("problem shape differs from the Solver's"))
    set && set_problem!(s, prob)
    upload!(s.h, s.x, prob.x); upload!(s.h, s.u, prob.u)
    st = ccall((:ilqr_fit_ex, libilqr), Cint,
               (Ptr{Cvoid}, Ref{Problem}, Ref{Options}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64},
                Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Int32}, Ptr{Int32}, Ptr{Cvoid}),
               s.h.ptr, problem_ref(s), (o = default_options(); o.max_iter = max_iter; o.tol = tol; o),
               s.x, s.u, C_NULL, s.xo, s.uo, s.cost, s.iters, s.status, C_NULL)
    st in (ILQR_OK, ILQR_ERR_LS_EXHAUSTED) || check(st, "ilqr_fit")
    download!(s.h, prob.x, s.xo); download!(s.h, prob.u, s.uo)
    return prob
end

"""backward!(s, x, u) -> (δu, K): iLQR.backward_pass (backward_pass.jl:324-357) on the
resident solver (one trajectory, reference layout)."""
function backward!(s::Solver, x::AbstractMatrix, u::AbstractMatrix)
    N, nx = size(x); M, nu = size(u)
    @assert(N == M + 1)                                                 # backward_pass.jl:329
    upload!(s.h, s.x, to_abi(x)); upload!(s.h, s.u, to_abi(u))
    check(ccall((:ilqr_backward, libilqr), Cint,
                (Ptr{Cvoid}, Ref{Problem}, Ref{Options}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Int32}),
                s.h.ptr, problem_ref(s), default_options(), s.x, s.u, s.d, s.K, s.status), "ilqr_backward")
    return from_abi(download!(s.h, zeros(nu, M), s.d)), gains_from_abi(download!(s.h, zeros(nx, nu, M), s.K))
end

"""forward!(s, x, u, x_traj, δu, K, prev_cost) -> (x̄, ū, new_cost): iLQR.forward_pass
(forward_pass.jl:55-93) on the resident solver."""
function forward!(s::Solver, x::AbstractMatrix, u::AbstractMatrix, x_traj::AbstractMatrix, δu::AbstractMatrix,
                  K::AbstractArray{<:Real,3}, prev_cost::Real)
    N, nx = size(x); M, nu = size(u)
    @assert(N == M + 1)                                                 # forward_pass.jl:62
    upload!(s.h, s.x, to_abi(x)); upload!(s.h, s.u, to_abi(u)); upload!(s.h, s.xt, to_abi(x_traj))
    upload!(s.h, s.d, to_abi(δu)); upload!(s.h, s.K, gains_to_abi(K)); upload!(s.h, s.pc, Float64[prev_cost])
    check(ccall((:ilqr_forward, libilqr), Cint,
                (Ptr{Cvoid}, Ref{Problem}, Ref{Options}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64},
                 Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64},
                 Ptr{Int32}, Ptr{Int32}),
                s.h.ptr, problem_ref(s), default_options(), s.x, s.u, s.xt, s.d, s.K, s.pc, s.xo, s.uo, s.cost,
                s.trials, s.status), "ilqr_forward")
    return (from_abi(download!(s.h, zeros(nx, N), s.xo)), from_abi(download!(s.h, zeros(nu, M), s.uo)),
            download!(s.h, zeros(1), s.cost)[1])
end

# The functional entry points' workspaces, one per (nx, nu, T) on device 0: Solvers for the
# LQ / 2-link families, TilesSolvers for arbitrary closures. The reference's fit is a pure
# function, so two tasks calling fit with one shape must not share buffers: with_cached
# holds the workspace's lock for the whole call (the second task waits for it), and the
# dictionaries change only under CACHE_LOCK. At most MAX_CACHED shapes per family stay
# resident; a new shape evicts an idle one (its device memory freed at once).
const SOLVER_CACHE = Dict{NTuple{3,Int},Solver}()
const TILES_CACHE = Dict{NTuple{3,Int},TilesSolver}()
const CACHE_LOCK = ReentrantLock()
const MAX_CACHED = 8

function evict_idle!(cache::Dict)
    for (k, c) in cache
        # not one in use (islocked: by any task — trylock alone would succeed on a lock
        # this task already holds, the lock being reentrant)
        if !islocked(c.lock) && trylock(c.lock)
            try
                close(c)
            finally
                unlock(c.lock)
            end
            delete!(cache, k)
            return true
        end
    end
    return false
end

"""with_cached(f, cache, make, key): f(s) on the cached workspace `key` (built by make()
on first use), holding s.lock for the call."""
function with_cached(f, cache::Dict, make, key)
    while true
        s = lock(CACHE_LOCK) do
            c = get(cache, key, nothing)
            if c === nothing || c.h.ptr == C_NULL
                length(cache) >= MAX_CACHED && evict_idle!(cache)
                c = cache[key] = make()
            end
            c
        end
        lock(s.lock)
        try
            s.h.ptr == C_NULL && continue      # evicted between the two locks: take a fresh one
            return f(s)
        finally
            unlock(s.lock)
        end
    end
end

"""clear_cache!(): close the workspaces fit / backward_pass / forward_pass keep per shape."""
function clear_cache!()
    lock(CACHE_LOCK) do
        foreach(close, values(SOLVER_CACHE)); empty!(SOLVER_CACHE)
        foreach(close, values(TILES_CACHE)); empty!(TILES_CACHE)
        foreach(close, values(FLOATING_CACHE)); empty!(FLOATING_CACHE)
        foreach(close, values(CHAIN_CACHE)); empty!(CHAIN_CACHE)
    end
    return nothing
end

# -- the reference's documented per-step API (docs/src/documentation.md:13-51) ------------
"""linearize_dynamics(x, u, dynamicsf) -> (𝐀, 𝐁) (backward_pass.jl:25-40). Vectors: one
point. Matrices with one row per step (test/test_linearize_dynamics.jl:10-14): 𝐀s (T × nx
× nx), 𝐁s (T × nx × nu) with 𝐀s[i, :, :] the Jacobian at (x[i, :], u[i, :]) — on the
device (ilqr_linearize) for the LQ and 2-link families, by ForwardDiff (as the reference)
for any other closure."""
function linearize_dynamics(x::AbstractVector, u::AbstractVector, f)
    As, Bs = linearize_dynamics(reshape(collect(x), 1, :), reshape(collect(u), 1, :), f)
    return As[1, :, :], Bs[1, :, :]
end
function linearize_dynamics(x::AbstractMatrix, u::AbstractMatrix, f)
    M, nu = size(u); nx = size(x, 2)
    size(x, 1) in (M, M + 1) || throw(AssertionError("x has $(size(x, 1)) rows for $M inputs"))
    f isa FloatingDynamics && return floating_linearize(f, x, u)
    fam = f isa LinearDynamics ? :lq : f isa TwoLinkDynamics ? :two_link : :host
    if fam == :host                                                     # ForwardDiff, :32-33
        As = zeros(M, nx, nx); Bs = zeros(M, nx, nu)
        for i in 1:M
            As[i, :, :] = jacobian(z -> f(z, u[i, :]), x[i, :]); Bs[i, :, :] = jacobian(v -> f(x[i, :], v), u[i, :])
        end
        return As, Bs
    end
    xa = size(x, 1) == M ? vcat(x, x[end:end, :]) : x                   # the ABI reads T+1 states
    # on the cached Solver of this shape (with_cached): no handle or buffer per call; the A/B
    # outputs are allocated on its first linearisation
    return with_cached(SOLVER_CACHE, () -> Solver(nx, nu, M, 1), (nx, nu, M)) do s
        fam == :lq ? set_problem!(s, f, QuadraticCost(zero(f.A), zeros(nu, nu)), QuadraticFinalCost(zero(f.A))) :
                     set_problem!(s, f, TwoLinkCost(), TwoLinkFinalCost())
        ensure_linearize!(s)
        upload!(s.h, s.x, to_abi(xa)); upload!(s.h, s.u, to_abi(u))
        check(ccall((:ilqr_linearize, libilqr), Cint,
                    (Ptr{Cvoid}, Ref{Problem}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}),
                    s.h.ptr, problem_ref(s), s.x, s.u, s.lA, s.lB), "ilqr_linearize")
        # (T, nx, nx) row-major = Julia (nx, nx, T), each step transposed → 𝐀s (T × nx × nx)
        (permutedims(download!(s.h, zeros(nx, nx, M), s.lA), (3, 2, 1)),
         permutedims(download!(s.h, zeros(nu, nx, M), s.lB), (3, 2, 1)))
    end
end

"""immediate_cost_quadratization(x, u, immediate_cost) -> (𝑞, 𝐪, 𝐫, 𝐐, 𝐏, 𝐑)
(backward_pass.jl:81-109; 𝐏 = ∂(∇ᵤℓ)/∂x is nu × nx): ForwardDiff on the host, the
reference's own derivatives."""
function immediate_cost_quadratization(x::AbstractVector, u::AbstractVector, ℓ)
    gu(z, v) = gradient(w -> ℓ(z, w), v)
    return (ℓ(x, u), gradient(z -> ℓ(z, u), x), gu(x, u), hessian(z -> ℓ(z, u), x),
            jacobian(z -> gu(z, u), x), hessian(v -> ℓ(x, v), u))
end

"""final_cost_quadratization(x, final_cost) -> (𝑞ₙ, 𝐪ₙ, 𝐐ₙ) (backward_pass.jl:134-153)."""
final_cost_quadratization(x::AbstractVector, ℓf) = (ℓf(x), gradient(ℓf, x), hessian(ℓf, x))

"""optimal_controller_param(𝐀, 𝐁, 𝐫, 𝐏, 𝐑, 𝐬′, 𝐒′) -> (𝐠, 𝐆, 𝐇) (backward_pass.jl:177-186)."""
function optimal_controller_param(A::AbstractMatrix, B::AbstractMatrix, r::AbstractVector, P::AbstractMatrix,
                                  R::AbstractMatrix, s::AbstractVector, S::AbstractMatrix)
    BᵀS = transpose(B) * S
    return (r + transpose(B) * s, P + BᵀS * A, R + BᵀS * B)
end

"""feedback_parameters(𝐠, 𝐆, 𝐇) -> (𝛿𝐮ᶠᶠ, 𝐊) with the fixed H + 0.01 I (backward_pass.jl:207-218)."""
function feedback_parameters(g::AbstractVector, G::AbstractMatrix, H::AbstractMatrix)
    Hμ = H + 0.01 * one(H)
    return (-(Hμ \ g), -(Hμ \ G))
end

"""step_back(𝐀, 𝑞, 𝐪, 𝐐, 𝐠, 𝐆, 𝐇, 𝛿𝐮, 𝐊, 𝑠′, 𝐬′, 𝐒′) -> (𝑠, 𝐬, 𝐒), unregularised 𝐇
(backward_pass.jl:262-273)."""
function step_back(A, q, qv, Q, g, G, H, δu, K, s′, sv′, S′)
    Hδu = H * δu
    Kᵀ, Gᵀ, Aᵀ = transpose(K), transpose(G), transpose(A)
    return (q + s′ + 0.5 * dot(δu, Hδu) + dot(δu, g),
            qv + Aᵀ * sv′ + Kᵀ * Hδu + Kᵀ * g + Gᵀ * δu,
            Q + Aᵀ * S′ * A + Kᵀ * H * K + Kᵀ * G + Gᵀ * K)
end

# -- RBD family (ILQR_PROBLEM_CHAIN): test/RBD_2_link_example with a fixed base --------
const ILQR_F64 = Int32(0)
const ILQR_F32 = Int32(1)
const ILQR_LINEARIZE_DUAL = Int32(0)
const ILQR_LINEARIZE_CENTRAL_FD = Int32(1)

struct Chain                 # ilqr_chain (include/ilqr.h), ILQR_CHAIN_MAX_JOINTS = 8
    n_joints::Int32; nu::Int32; dt::Float64; gravity::NTuple{3,Float64}
    joint_rot::NTuple{72,Float64}; joint_pos::NTuple{24,Float64}; axis::NTuple{24,Float64}
    mass::NTuple{8,Float64}; com::NTuple{24,Float64}; inertia::NTuple{72,Float64}
    target::NTuple{8,Float64}; q_weight::NTuple{8,Float64}; r_weight::NTuple{8,Float64}
    qf_weight::NTuple{8,Float64}
end

const ILQR_CHAIN_DYN_AUTO = Int32(0)         # ilqr_chain_set_dynamics (include/ilqr.h)
const ILQR_CHAIN_DYN_RNEA = Int32(1)
const ILQR_CHAIN_DYN_CLOSED_FORM = Int32(2)
const ILQR_CHAIN_COST_JOINT = Int32(0)       # ilqr_chain_set_simple_costs (include/ilqr.h)
const ILQR_CHAIN_COST_SIMPLE = Int32(1)
const ILQR_CHAIN_COST_SIMPLE_EUCLIDEAN = Int32(2)

"""The pair simple_immediate_cost / simple_final_cost(mechanism, body, point,
final_target, weight) of src/cost_functions.jl on the chain's handle: Σuᵢ² and
weight·Σₖ(p_z − final_targetₖ)² for `point` in the frame of `body` (the link joint
`body` moves, 0-based; −1 the base); euclidean = true takes Σₖ(pₖ − final_targetₖ)²."""
struct SimpleCosts
    body::Int32; point::NTuple{3,Float64}; final_target::NTuple{3,Float64}; weight::Float64
    euclidean::Bool
end
simple_costs(body, point, final_target, weight; euclidean::Bool=false) =
    SimpleCosts(Int32(body), Tuple(Float64.(point)), Tuple(Float64.(final_target)), Float64(weight), euclidean)

"""ChainSolver: one ilqr_chain handle (precision, linearisation, evaluator and costs set at
creation) plus its device buffers — the iterate, the results, the status — allocated once
per (chain, T, batch, element type, linearization, dynamics, costs) and reused by every
chain_fit of that key (CHAIN_CACHE; include/ilqr.h: "hot calls never allocate")."""
mutable struct ChainSolver
    ch::Ptr{Cvoid}           # ilqr_chain_handle
    h::Handle                # device-memory helper (ilqr_malloc / memcpy), closed with it
    x::Ptr{Cvoid}; u::Ptr{Cvoid}; xo::Ptr{Cvoid}; uo::Ptr{Cvoid}; status::Ptr{Int32}
    lock::ReentrantLock
end

function ChainSolver(c::Chain, nx::Integer, nu::Integer, T::Integer, nb::Integer, ::Type{E}, linearization,
                     dynamics, costs::Union{Nothing,SimpleCosts}; device::Integer=0) where {E<:Union{Float32,Float64}}
    r = Ref{Ptr{Cvoid}}(C_NULL)
    dt = E === Float32 ? ILQR_F32 : ILQR_F64
    check(ccall((:ilqr_chain_create, libilqr), Cint,
                (Ref{Ptr{Cvoid}}, Cint, Ref{Chain}, Cint, Cint, Int32, Int32),
                r, device, c, T, nb, dt, linearization), "ilqr_chain_create")
    destroy() = ccall((:ilqr_chain_destroy, libilqr), Cint, (Ptr{Cvoid},), r[])
    try
        check(ccall((:ilqr_chain_set_dynamics, libilqr), Cint, (Ptr{Cvoid}, Int32), r[], dynamics),
              "ilqr_chain_set_dynamics")
        if costs !== nothing
            mode = costs.euclidean ? ILQR_CHAIN_COST_SIMPLE_EUCLIDEAN : ILQR_CHAIN_COST_SIMPLE
            check(ccall((:ilqr_chain_set_simple_costs, libilqr), Cint,
                        (Ptr{Cvoid}, Int32, Int32, Ptr{Float64}, Ptr{Float64}, Float64),
                        r[], mode, costs.body, collect(costs.point), collect(costs.final_target), costs.weight),
                  "ilqr_chain_set_simple_costs")
        end
    catch
        destroy(); rethrow()
    end
    h = Handle(nx, nu, T, 1; device=device)  # device-memory helper only
    a(n) = Ptr{Cvoid}(alloc(h, E, n))
    s = ChainSolver(r[], h, a(nb * (T + 1) * nx), a(nb * T * nu), a(nb * (T + 1) * nx), a(nb * T * nu),
                    alloc(h, Int32, nb), ReentrantLock())
    finalizer(destroy!, s)      # a backstop; close(s) frees everything at once
    return s
end

function destroy!(s::ChainSolver)
    s.ch != C_NULL && (ccall((:ilqr_chain_destroy, libilqr), Cint, (Ptr{Cvoid},), s.ch); s.ch = C_NULL)
    close(s.h)
    return nothing
end
Base.close(s::ChainSolver) = lock(() -> destroy!(s), s.lock)

const CHAIN_CACHE = Dict{Tuple{Chain,Int,Int,DataType,Int32,Int32,Union{Nothing,SimpleCosts}},ChainSolver}()

"""chain_fit(chain, x_init, u_init; max_iter, tol, linearization, dynamics) → (x̄, ū, status)

Batched fit of the chain family; x_init (nx, T+1, batch), u_init (nu, T, batch) as
Array{Float32,3} (fp32, BASELINE config 5) or Array{Float64,3}: the element type picks
the device precision, as the reference's generic Julia code would. `dynamics` picks the
2-joint evaluator (AUTO: the closed form sampled from the Newton-Euler recursion at
creation; RNEA: the recursion itself). `costs = simple_costs(…)` replaces the chain's
joint-space costs with cost_functions.jl's pair (2-joint chains, closed form). The handle
and buffers are cached per (chain, T, batch, element type, options): an MPC loop calling
chain_fit allocates nothing per call (clear_cache!() closes them)."""
function chain_fit(c::Chain, x_init::Array{E,3}, u_init::Array{E,3}; max_iter::Int64=100,
                   tol::Float64=1e-6, linearization=ILQR_LINEARIZE_DUAL,
                   dynamics=ILQR_CHAIN_DYN_AUTO,
                   costs::Union{Nothing,SimpleCosts}=nothing) where {E<:Union{Float32,Float64}}
    nx, N, nb = size(x_init); nu = size(u_init, 1); M = N - 1
    @assert(size(u_init, 2) == M)
    key = (c, M, nb, E, Int32(linearization), Int32(dynamics), costs)
    return with_cached(CHAIN_CACHE, () -> ChainSolver(c, nx, nu, M, nb, E, linearization, dynamics, costs), key) do s
        upload!(s.h, s.x, x_init); upload!(s.h, s.u, u_init)
        o = default_options(); o.max_iter = max_iter; o.tol = tol
        st = ccall((:ilqr_chain_fit, libilqr), Cint,
                   (Ptr{Cvoid}, Ref{Options}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid},
                    Ptr{Int32}, Ptr{Int32}),
                   s.ch, o, s.x, s.u, C_NULL, s.xo, s.uo, C_NULL, C_NULL, s.status)
        st == ILQR_ERR_LS_EXHAUSTED || check(st, "ilqr_chain_fit")
        (download!(s.h, similar(x_init), s.xo), download!(s.h, similar(u_init), s.uo),
         download!(s.h, zeros(Int32, nb), s.status))
    end
end

# -- floating-base RBD family: the reference's RBD script as it runs --------------------
struct FloatingModel          # ilqr_floating (include/ilqr.h), ILQR_FLOATING_MAX_JOINTS = 2
    n_joints::Int32; dt::Float64; gravity::NTuple{3,Float64}
    base_mass::Float64; base_com::NTuple{3,Float64}; base_inertia::NTuple{9,Float64}
    joint_rot::NTuple{18,Float64}; joint_pos::NTuple{6,Float64}; axis::NTuple{6,Float64}
    mass::NTuple{2,Float64}; com::NTuple{6,Float64}; inertia::NTuple{18,Float64}
    target::NTuple{8,Float64}; q_weight::NTuple{8,Float64}; r_weight::NTuple{8,Float64}
    qf_weight::NTuple{8,Float64}
    q_scale::Float64; r_scale::Float64; qf_scale::Float64
end

"""The model behind test/RBD_2_link_example: test/urdf/2Dof_arm.urdf parsed with
`floating = true, gravity = 0` (RBD_helper_functions.jl:7) — a 30 kg base (50·I), two
3 kg links (0.5·I) on joints at (.5, .5, 0) about z and (1, 0, 0) about y — with the
script's Δt, target_pose and cost weights (animate_RBD_2_link.jl:8-10,
RBD_helper_functions.jl:85-116)."""
function rbd_2dof_arm_floating(; target=(0., 0., 0., 5., 1., 2., 1., .3))
    I3 = (1., 0., 0., 0., 1., 0., 0., 0., 1.)
    FloatingModel(Int32(2), 0.01, (0., 0., 0.), 30.0, (0., 0., 0.), 50.0 .* I3,
                  (I3..., I3...), (.5, .5, 0., 1., 0., 0.), (0., 0., 1., 0., 1., 0.),
                  (3.0, 3.0), ntuple(_ -> 0.0, 6), (0.5 .* I3..., 0.5 .* I3...),
                  Tuple(Float64.(target)), (100., 100., 100., 1., 1., 1., 10., 10.),
                  (1., 1., 1., 100., 100., 100., 10., 10.),
                  (100., 100., 100., 1000., 1000., 1000., 10., 10.), 10.0, 1.0, 100000.0)
end

"""FloatingSolver(model, T, batch): one ilqr_floating handle and every device buffer its
calls need — the iterate, x_traj, the results, the gains, the costs and statuses (the
linearisation outputs and the verbose history on first use) — allocated once per
(model, T, batch) and reused (FLOATING_CACHE). fit / backward_pass / forward_pass /
linearize_dynamics with the FloatingDynamics / FloatingCost / FloatingFinalCost callables,
and floating_fit, run on a cached one."""
mutable struct FloatingSolver
    fh::Ptr{Cvoid}           # ilqr_floating_handle
    h::Handle                # device-memory helper (ilqr_malloc / memcpy), closed with it
    nx::Int; nu::Int; M::Int; nb::Int
    x::Ptr{Float64}; u::Ptr{Float64}; xt::Ptr{Float64}; xo::Ptr{Float64}; uo::Ptr{Float64}
    d::Ptr{Float64}; K::Ptr{Float64}; pc::Ptr{Float64}; cost::Ptr{Float64}
    iters::Ptr{Int32}; status::Ptr{Int32}; trials::Ptr{Int32}
    lA::Ptr{Float64}; lB::Ptr{Float64}       # linearize_dynamics' outputs, on first use
    hc::Ptr{Float64}; ht::Ptr{Int32}; hcap::Int
    lock::ReentrantLock
end

function FloatingSolver(m::FloatingModel, T::Integer, batch::Integer; device::Integer=0)
    r = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:ilqr_floating_create, libilqr), Cint, (Ref{Ptr{Cvoid}}, Cint, Ref{FloatingModel}, Cint, Cint),
                r, device, m, T, batch), "ilqr_floating_create")
    nu = 6 + Int(m.n_joints); nx = 2 * nu; N = T + 1
    h = Handle(nx, nu, T, 1; device=device)  # device-memory helper only
    f(n) = alloc(h, Float64, batch * n)
    i(n) = alloc(h, Int32, batch * n)
    s = FloatingSolver(r[], h, nx, nu, T, batch,
                       f(N * nx), f(T * nu), f(N * nx), f(N * nx), f(T * nu),      # x u x_traj x̄ ū
                       f(T * nu), f(T * nu * nx), f(1), f(1),                      # δu K prev_cost cost
                       i(1), i(1), i(1),                                           # iters status trials
                       Ptr{Float64}(C_NULL), Ptr{Float64}(C_NULL), Ptr{Float64}(C_NULL), Ptr{Int32}(C_NULL), 0,
                       ReentrantLock())
    finalizer(destroy!, s)      # a backstop; close(s) frees everything at once
    return s
end

function destroy!(s::FloatingSolver)
    s.fh != C_NULL && (ccall((:ilqr_floating_destroy, libilqr), Cint, (Ptr{Cvoid},), s.fh); s.fh = C_NULL)
    close(s.h)
    return nothing
end
Base.close(s::FloatingSolver) = lock(() -> destroy!(s), s.lock)

const FLOATING_CACHE = Dict{Tuple{FloatingModel,Int,Int},FloatingSolver}()
floating_cached(f, m::FloatingModel, M::Integer, nb::Integer) =
    with_cached(f, FLOATING_CACHE, () -> FloatingSolver(m, M, nb), (m, Int(M), Int(nb)))

# -- the script's closures as callable structs (RBD_helper_functions.jl:48-116) -------------
# fit / backward_pass / forward_pass / linearize_dynamics recognise the triple (family
# :floating) and run ilqr_floating_* on a cached FloatingSolver; called directly they are
# the script's functions: dynamicsf one device RK4 step (a cached T = 1 workspace: the
# script calls it 1000 times to build state_traj, animate_RBD_2_link.jl:23-25), the costs
# plain Julia arithmetic (generic, as ForwardDiff needs them).
struct FloatingDynamics; model::FloatingModel; end
struct FloatingCost; model::FloatingModel; end
struct FloatingFinalCost; model::FloatingModel; end
floating_closures(m::FloatingModel=rbd_2dof_arm_floating()) = (FloatingDynamics(m), FloatingCost(m), FloatingFinalCost(m))
is_floating(f, l, lf) = f isa FloatingDynamics && l isa FloatingCost && lf isa FloatingFinalCost &&
                        f.model == l.model == lf.model

function (f::FloatingDynamics)(x::AbstractVector, u::AbstractVector)            # dynamicsf (:48-79)
    return floating_cached(f.model, 1, 1) do s
        upload!(s.h, s.x, Vector{Float64}(x)); upload!(s.h, s.u, Vector{Float64}(u))
        check(ccall((:ilqr_floating_dynamics, libilqr), Cint,
                    (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Cint), s.fh, s.x, s.u, s.xo, 1),
              "ilqr_floating_dynamics")
        download!(s.h, zeros(s.nx), s.xo)
    end
end
function (l::FloatingCost)(x, u)                                                  # immediate_cost (:85-101)
    m = l.model; q = 6 + Int(m.n_joints)
    δx = [m.target[i] - x[i] for i in 1:q]
    return sum(δx[i] * m.q_weight[i] * δx[i] for i in 1:q) * m.q_scale +
           sum(u[j] * m.r_weight[j] * u[j] for j in 1:q) * m.r_scale
end
function (l::FloatingFinalCost)(x)                                                # final_cost (:107-116)
    m = l.model; q = 6 + Int(m.n_joints)
    δx = [m.target[i] - x[i] for i in 1:q]
    return sum(δx[i] * m.qf_weight[i] * δx[i] for i in 1:q) * m.qf_scale
end

function floating_shape(s::FloatingSolver, nx, nu)
    (nx, nu) == (s.nx, s.nu) || throw(AssertionError("the floating model is ($(s.nx), $(s.nu)), x/u are ($nx, $nu)"))
end

# iLQR.fit (forward_pass.jl:148-179) of one trajectory (reference layout) on the device
function floating_fit1(f::FloatingDynamics, x_init, u_init, x_traj, max_iter, tol, verbose)
    N, nx = size(x_init); M, nu = size(u_init)
    return floating_cached(f.model, M, 1) do s
        floating_shape(s, nx, nu)
        upload!(s.h, s.x, to_abi(x_init)); upload!(s.h, s.u, to_abi(u_init)); upload!(s.h, s.xt, to_abi(x_traj))
        o = default_options(); o.max_iter = max_iter; o.tol = tol
        n = max(max_iter, 1)
        if verbose && s.hcap < n
            s.hc != C_NULL && (release!(s.h, s.hc); release!(s.h, s.ht))
            s.hc = alloc(s.h, Float64, n); s.ht = alloc(s.h, Int32, n); s.hcap = n
        end
        verbose && upload!(s.h, s.ht, zeros(Int32, n))
        hist = verbose ? Ref(History(s.hc, s.ht, C_NULL, C_NULL)) : Ref(History(C_NULL, C_NULL, C_NULL, C_NULL))
        st = ccall((:ilqr_floating_fit_ex, libilqr), Cint,
                   (Ptr{Cvoid}, Ref{Options}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64},
                    Ptr{Float64}, Ptr{Int32}, Ptr{Int32}, Ref{History}),
                   s.fh, o, s.x, s.u, s.xt, s.xo, s.uo, s.cost, s.iters, s.status, hist)
        st in (ILQR_OK, ILQR_ERR_LS_EXHAUSTED) || check(st, "ilqr_floating_fit")
        verbose && print_history(download!(s.h, zeros(n), s.hc), download!(s.h, zeros(Int32, n), s.ht))
        (from_abi(download!(s.h, zeros(nx, N), s.xo)), from_abi(download!(s.h, zeros(nu, M), s.uo)))
    end
end

# iLQR.backward_pass (backward_pass.jl:324-357) → (δu::T×nu, K::T×nu×nx)
function floating_backward(f::FloatingDynamics, x, u)
    N, nx = size(x); M, nu = size(u)
    return floating_cached(f.model, M, 1) do s
        floating_shape(s, nx, nu)
        upload!(s.h, s.x, to_abi(x)); upload!(s.h, s.u, to_abi(u))
        check(ccall((:ilqr_floating_backward, libilqr), Cint,
                    (Ptr{Cvoid}, Ref{Options}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Int32}),
                    s.fh, default_options(), s.x, s.u, s.d, s.K, s.status), "ilqr_floating_backward")
        (from_abi(download!(s.h, zeros(nu, M), s.d)), gains_from_abi(download!(s.h, zeros(nx, nu, M), s.K)))
    end
end

# iLQR.forward_pass (forward_pass.jl:55-93) → (x̄, ū, new_cost)
function floating_forward(f::FloatingDynamics, x, u, x_traj, δu, K, prev_cost)
    N, nx = size(x); M, nu = size(u)
    return floating_cached(f.model, M, 1) do s
        floating_shape(s, nx, nu)
        upload!(s.h, s.x, to_abi(x)); upload!(s.h, s.u, to_abi(u)); upload!(s.h, s.xt, to_abi(x_traj))
        upload!(s.h, s.d, to_abi(δu)); upload!(s.h, s.K, gains_to_abi(K)); upload!(s.h, s.pc, Float64[prev_cost])
        check(ccall((:ilqr_floating_forward, libilqr), Cint,
                    (Ptr{Cvoid}, Ref{Options}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64},
                     Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Int32}, Ptr{Int32}),
                    s.fh, default_options(), s.x, s.u, s.xt, s.d, s.K, s.pc, s.xo, s.uo, s.cost, s.trials, s.status),
              "ilqr_floating_forward")
        (from_abi(download!(s.h, zeros(nx, N), s.xo)), from_abi(download!(s.h, zeros(nu, M), s.uo)),
         download!(s.h, zeros(1), s.cost)[1])
    end
end

# linearize_dynamics (backward_pass.jl:25-40) at every step: the dual-number kernel
function floating_linearize(f::FloatingDynamics, x::AbstractMatrix, u::AbstractMatrix)
    M, nu = size(u); nx = size(x, 2)
    size(x, 1) in (M, M + 1) || throw(AssertionError("x has $(size(x, 1)) rows for $M inputs"))
    xa = size(x, 1) == M ? vcat(x, x[end:end, :]) : x                   # the ABI reads T+1 states
    return floating_cached(f.model, M, 1) do s
        floating_shape(s, nx, nu)
        if s.lA == C_NULL
            s.lA = alloc(s.h, Float64, s.M * s.nx * s.nx); s.lB = alloc(s.h, Float64, s.M * s.nx * s.nu)
        end
        upload!(s.h, s.x, to_abi(xa)); upload!(s.h, s.u, to_abi(u))
        check(ccall((:ilqr_floating_linearize, libilqr), Cint,
                    (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}),
                    s.fh, s.x, s.u, s.lA, s.lB), "ilqr_floating_linearize")
        (permutedims(download!(s.h, zeros(nx, nx, M), s.lA), (3, 2, 1)),
         permutedims(download!(s.h, zeros(nu, nx, M), s.lB), (3, 2, 1)))
    end
end

"""floating_fit(model, x_init, u_init; max_iter, tol) → (x̄, ū, status)

iLQR.fit of the floating-base family on the device (include/ilqr.h ilqr_floating_fit):
x_init (16, T+1, batch) = [MRP; r; θ; ω; v; θ̇], u_init (8, T, batch), as the script's
`state_traj` / `input_traj` transposed (animate_RBD_2_link.jl:19-25); on the cached
FloatingSolver of (model, T, batch)."""
function floating_fit(m::FloatingModel, x_init::Array{Float64,3}, u_init::Array{Float64,3};
                      max_iter::Int64=100, tol::Float64=1e-6)
    nx, N, nb = size(x_init); nu = size(u_init, 1); M = N - 1
    @assert(size(u_init, 2) == M)
    return floating_cached(m, M, nb) do s
        floating_shape(s, nx, nu)
        upload!(s.h, s.x, x_init); upload!(s.h, s.u, u_init)
        o = default_options(); o.max_iter = max_iter; o.tol = tol
        st = ccall((:ilqr_floating_fit, libilqr), Cint,
                   (Ptr{Cvoid}, Ref{Options}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64},
                    Ptr{Float64}, Ptr{Int32}, Ptr{Int32}),
                   s.fh, o, s.x, s.u, C_NULL, s.xo, s.uo, C_NULL, C_NULL, s.status)
        st == ILQR_ERR_LS_EXHAUSTED || check(st, "ilqr_floating_fit")
        (download!(s.h, similar(x_init), s.xo), download!(s.h, similar(u_init), s.uo),
         download!(s.h, zeros(Int32, nb), s.status))
    end
end

end # module
