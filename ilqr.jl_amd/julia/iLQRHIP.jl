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
# New API: `solve!(::iLQRProblem)` (batched LQ, one or several GPUs) and `chain_fit`
# (the RBD family of BASELINE config 5).
module iLQRHIP

using ForwardDiff: gradient, jacobian, hessian   # as the reference (src/iLQR.jl:3)

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
    finalizer(h) do h
        for p in h.bufs; ccall((:ilqr_free, libilqr), Cint, (Ptr{Cvoid}, Ptr{Cvoid}), h.ptr, p); end
        ccall((:ilqr_destroy, libilqr), Cint, (Ptr{Cvoid},), h.ptr)
    end
    return h
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
family(f, l, lf) = (f, l, lf) isa LQTriple ? :lq : (f, l, lf) isa TwoLinkTriple ? :two_link : :tiles

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

function backward_tiles_device(x::AbstractMatrix, u::AbstractMatrix, f, ℓ, ℓf)
    N, nx = size(x); M, nu = size(u)
    h = Handle(nx, nu, M, 1)
    t = derivative_tiles(x, u, f, ℓ, ℓf)
    tl = Ref(Tiles(upload(h, t.A), upload(h, t.B), upload(h, t.lx), upload(h, t.lu), upload(h, t.lxx),
                   upload(h, t.lux), upload(h, t.luu), upload(h, t.lfx), upload(h, t.lfxx)))
    dd = alloc(h, Float64, M * nu); Kd = alloc(h, Float64, M * nu * nx); st = alloc(h, Int32, 1)
    check(ccall((:ilqr_backward_tiles, libilqr), Cint,
                (Ptr{Cvoid}, Ref{Tiles}, Ref{Options}, Ptr{Float64}, Ptr{Float64}, Ptr{Int32}),
                h.ptr, tl, default_options(), dd, Kd, st), "ilqr_backward_tiles")
    return from_abi(download!(h, zeros(nu, M), dd)), gains_from_abi(download!(h, zeros(nx, nu, M), Kd))
end

"""backward_pass(x, u, dynamicsf, immediate_cost, final_cost) -> (δu::T×nu, K::T×nu×nx)"""
function backward_pass(x::AbstractMatrix, u::AbstractMatrix, dynamicsf, immediate_cost, final_cost)
    N, nx = size(x); M, nu = size(u)
    @assert(N == M + 1)                                                 # backward_pass.jl:329
    family(dynamicsf, immediate_cost, final_cost) == :tiles &&
        return backward_tiles_device(x, u, dynamicsf, immediate_cost, final_cost)
    h = Handle(nx, nu, M, 1)
    p = Ref(problem(h, dynamicsf, immediate_cost, final_cost))
    xd = upload(h, to_abi(x)); ud = upload(h, to_abi(u))
    dd = alloc(h, Float64, M * nu); Kd = alloc(h, Float64, M * nu * nx)
    st = alloc(h, Int32, 1)
    check(ccall((:ilqr_backward, libilqr), Cint,
                (Ptr{Cvoid}, Ref{Problem}, Ref{Options}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Int32}),
                h.ptr, p, default_options(), xd, ud, dd, Kd, st), "ilqr_backward")
    du = from_abi(download!(h, zeros(nu, M), dd))                       # (T × nu)
    K = gains_from_abi(download!(h, zeros(nx, nu, M), Kd))              # (T × nu × nx) like 𝐊s
    return du, K
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
    family(dynamicsf, immediate_cost, final_cost) == :tiles &&
        return forward_host(x, u, x_traj, δu, K, prev_cost, dynamicsf, immediate_cost, final_cost)
    h = Handle(nx, nu, M, 1)
    p = Ref(problem(h, dynamicsf, immediate_cost, final_cost))
    xd = upload(h, to_abi(x)); ud = upload(h, to_abi(u)); xt = upload(h, to_abi(x_traj))
    dd = upload(h, to_abi(δu)); Kd = upload(h, gains_to_abi(K))
    pc = upload(h, Float64[prev_cost])
    xo = alloc(h, Float64, N * nx); uo = alloc(h, Float64, M * nu); co = alloc(h, Float64, 1)
    st = alloc(h, Int32, 1)
    check(ccall((:ilqr_forward, libilqr), Cint,
                (Ptr{Cvoid}, Ref{Problem}, Ref{Options}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64},
                 Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64},
                 Ptr{Int32}, Ptr{Int32}),
                h.ptr, p, default_options(), xd, ud, xt, dd, Kd, pc, xo, uo, co, C_NULL, st), "ilqr_forward")
    x̄ = from_abi(download!(h, zeros(nx, N), xo)); ū = from_abi(download!(h, zeros(nu, M), uo))
    return (x̄, ū, download!(h, zeros(1), co)[1])
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
    family(dynamicsf, immediate_cost, final_cost) == :tiles &&
        return fit_tiles(x_init, u_init, dynamicsf, immediate_cost, final_cost, x_traj, max_iter, tol, verbose)
    h = Handle(nx, nu, M, 1)
    p = Ref(problem(h, dynamicsf, immediate_cost, final_cost))
    o = default_options(); o.max_iter = max_iter; o.tol = tol
    xi = upload(h, to_abi(x_init)); ui = upload(h, to_abi(u_init)); xt = upload(h, to_abi(x_traj))
    xo = alloc(h, Float64, N * nx); uo = alloc(h, Float64, M * nu)
    hc = alloc(h, Float64, max_iter); ht = upload(h, zeros(Int32, max(max_iter, 1)))
    hist = Ref(History(hc, ht, C_NULL, C_NULL))
    st = ccall((:ilqr_fit_ex, libilqr), Cint,
               (Ptr{Cvoid}, Ref{Problem}, Ref{Options}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64},
                Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Int32}, Ptr{Int32}, Ref{History}),
               h.ptr, p, o, xi, ui, xt, xo, uo, C_NULL, C_NULL, C_NULL, hist)
    st == ILQR_ERR_LS_EXHAUSTED || check(st, "ilqr_fit")   # exhausted: the last iterate is returned
    verbose && print_history(download!(h, zeros(max_iter), hc), download!(h, zeros(Int32, max(max_iter, 1)), ht))
    return from_abi(download!(h, zeros(nx, N), xo)), from_abi(download!(h, zeros(nu, M), uo))
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

"""chain_fit(chain, x_init, u_init; max_iter, tol, linearization, dynamics) → (x̄, ū, status)

Batched fit of the chain family; x_init (nx, T+1, batch), u_init (nu, T, batch) as
Array{Float32,3} (fp32, BASELINE config 5) or Array{Float64,3}: the element type picks
the device precision, as the reference's generic Julia code would. `dynamics` picks the
2-joint evaluator (AUTO: the closed form sampled from the Newton-Euler recursion at
creation; RNEA: the recursion itself). `costs = simple_costs(…)` replaces the chain's
joint-space costs with cost_functions.jl's pair (2-joint chains, closed form)."""
function chain_fit(c::Chain, x_init::Array{E,3}, u_init::Array{E,3}; max_iter::Int64=100,
                   tol::Float64=1e-6, linearization=ILQR_LINEARIZE_DUAL,
                   dynamics=ILQR_CHAIN_DYN_AUTO,
                   costs::Union{Nothing,SimpleCosts}=nothing) where {E<:Union{Float32,Float64}}
    nx, N, nb = size(x_init); nu = size(u_init, 1); M = N - 1
    @assert(size(u_init, 2) == M)
    r = Ref{Ptr{Cvoid}}(C_NULL)
    dt = E === Float32 ? ILQR_F32 : ILQR_F64
    check(ccall((:ilqr_chain_create, libilqr), Cint,
                (Ref{Ptr{Cvoid}}, Cint, Ref{Chain}, Cint, Cint, Int32, Int32),
                r, 0, c, M, nb, dt, linearization), "ilqr_chain_create")
    check(ccall((:ilqr_chain_set_dynamics, libilqr), Cint, (Ptr{Cvoid}, Int32), r[], dynamics),
          "ilqr_chain_set_dynamics")
    if costs !== nothing
        mode = costs.euclidean ? ILQR_CHAIN_COST_SIMPLE_EUCLIDEAN : ILQR_CHAIN_COST_SIMPLE
        pt = collect(costs.point); tg = collect(costs.final_target)
        check(ccall((:ilqr_chain_set_simple_costs, libilqr), Cint,
                    (Ptr{Cvoid}, Int32, Int32, Ptr{Float64}, Ptr{Float64}, Float64),
                    r[], mode, costs.body, pt, tg, costs.weight), "ilqr_chain_set_simple_costs")
    end
    h = Handle(nx, nu, M, 1)                 # device-memory helper only
    xi = upload(h, x_init); ui = upload(h, u_init)
    xo = alloc(h, E, length(x_init)); uo = alloc(h, E, length(u_init)); sd = alloc(h, Int32, nb)
    o = default_options(); o.max_iter = max_iter; o.tol = tol
    st = ccall((:ilqr_chain_fit, libilqr), Cint,
               (Ptr{Cvoid}, Ref{Options}, Ptr{E}, Ptr{E}, Ptr{E}, Ptr{E}, Ptr{E}, Ptr{E}, Ptr{Int32}, Ptr{Int32}),
               r[], o, xi, ui, C_NULL, xo, uo, C_NULL, C_NULL, sd)
    st == ILQR_ERR_LS_EXHAUSTED || check(st, "ilqr_chain_fit")
    x = download!(h, similar(x_init), xo); u = download!(h, similar(u_init), uo)
    status = download!(h, zeros(Int32, nb), sd)
    ccall((:ilqr_chain_destroy, libilqr), Cint, (Ptr{Cvoid},), r[])
    return x, u, status
end

end # module
