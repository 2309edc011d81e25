# iLQRHIP.jl — Julia-side drop-in for aabouman/iLQR.jl's hot path over the C ABI
# of libilqr_hip.so (include/ilqr.h). Not executable in this build environment (no
# Julia toolchain); the same symbols and layouts are exercised from Python by
# tests/test_gpu_parity.py and tests/test_abi.py.
#
# It keeps the reference's public signatures:
#   fit(x_init, u_init, dynamicsf, immediate_cost, final_cost; x_traj, max_iter, tol)
#                                                     (reference src/forward_pass.jl:148-179)
#   backward_pass(x, u, dynamicsf, immediate_cost, final_cost) -> (δu, K)
#                                                     (reference src/backward_pass.jl:324-357)
#   forward_pass(x, u, x_traj, δu, K, prev_cost, dynamicsf, immediate_cost, final_cost)
#                                                     (reference src/forward_pass.jl:55-93)
# for the LQ problem family, whose closures are the callable structs below, and
# adds a batched `solve!(::iLQRProblem)`.
module iLQRHIP

const libilqr = joinpath(@__DIR__, "..", "lib", "libilqr_hip.so")

const ILQR_OK = Int32(0)
const ILQR_ERR_BAD_DIMS = Int32(1)
const ILQR_ERR_NAN = Int32(5)
const ILQR_ERR_LS_EXHAUSTED = Int32(6)
const ILQR_PROBLEM_LQ = Int32(1)

struct Problem               # ilqr_problem
    kind::Int32
    reserved::Int32
    A::Ptr{Float64}
    B::Ptr{Float64}
    Q::Ptr{Float64}
    R::Ptr{Float64}
    Qf::Ptr{Float64}
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

# -- the reference's callbacks, as recognisable callable structs ------------------
struct LinearDynamics{M<:AbstractMatrix}; A::M; B::M; end
(f::LinearDynamics)(x, u) = f.A * x + f.B * u                      # dynamicsf(x, u)
struct QuadraticCost{M<:AbstractMatrix}; Q::M; R::M; end
(l::QuadraticCost)(x, u) = x' * l.Q * x + u' * l.R * u             # immediate_cost(x, u)
struct QuadraticFinalCost{M<:AbstractMatrix}; Qf::M; end
(l::QuadraticFinalCost)(x) = x' * l.Qf * x                         # final_cost(x)

check(st, what) = st == ILQR_OK ? nothing :
    st == ILQR_ERR_BAD_DIMS ? throw(AssertionError("N == M+1")) :
    error("$what: " * unsafe_string(ccall((:ilqr_status_string, libilqr), Cstring, (Cint,), st)))

# device buffer owned by Julia (freed with the handle)
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
set_schedule!(h::Handle, flags::Integer) =
    check(ccall((:ilqr_set_schedule, libilqr), Cint, (Ptr{Cvoid}, Cint), h.ptr, flags), "ilqr_set_schedule")

function upload(h::Handle, a::Array{Float64})
    p = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:ilqr_malloc, libilqr), Cint, (Ptr{Cvoid}, Csize_t, Ref{Ptr{Cvoid}}), h.ptr, sizeof(a), p), "ilqr_malloc")
    push!(h.bufs, p[])
    check(ccall((:ilqr_memcpy_h2d, libilqr), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Csize_t),
                h.ptr, p[], a, sizeof(a)), "ilqr_memcpy_h2d")
    return Ptr{Float64}(p[])
end

function alloc(h::Handle, T::Type, n)
    p = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:ilqr_malloc, libilqr), Cint, (Ptr{Cvoid}, Csize_t, Ref{Ptr{Cvoid}}), h.ptr, n * sizeof(T), p), "ilqr_malloc")
    push!(h.bufs, p[])
    return Ptr{T}(p[])
end

function download!(h::Handle, a::Array, p::Ptr)
    check(ccall((:ilqr_memcpy_d2h, libilqr), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Csize_t),
                h.ptr, a, p, sizeof(a)), "ilqr_memcpy_d2h")
    return a
end

# Reference layout per trajectory: x (N × nx) rows = time steps. The ABI's
# layout for one trajectory is (nx, N) column-major == permutedims(x).
to_abi(x::AbstractMatrix) = Array{Float64}(permutedims(x))
from_abi(a::AbstractMatrix) = permutedims(a)

function problem(h::Handle, f::LinearDynamics, l::QuadraticCost, lf::QuadraticFinalCost)
    # C row-major (nx, nx) == Julia transpose
    A = upload(h, Array{Float64}(permutedims(f.A))); B = upload(h, Array{Float64}(permutedims(f.B)))
    Q = upload(h, Array{Float64}(permutedims(l.Q))); R = upload(h, Array{Float64}(permutedims(l.R)))
    Qf = upload(h, Array{Float64}(permutedims(lf.Qf)))
    return Problem(ILQR_PROBLEM_LQ, 0, A, B, Q, R, Qf)
end

problem(h::Handle, f, l, lf) =
    throw(ArgumentError("the HIP path runs the LQ family: pass LinearDynamics / QuadraticCost / QuadraticFinalCost"))

"""backward_pass(x, u, dynamicsf, immediate_cost, final_cost) -> (δu::T×nu, K::T×nu×nx)"""
function backward_pass(x::AbstractMatrix, u::AbstractMatrix, dynamicsf, immediate_cost, final_cost)
    N, nx = size(x); M, nu = size(u)
    @assert(N == M + 1)
    h = Handle(nx, nu, M, 1)
    p = Ref(problem(h, dynamicsf, immediate_cost, final_cost))
    xd = upload(h, to_abi(x)); ud = upload(h, to_abi(u))
    dd = alloc(h, Float64, M * nu); Kd = alloc(h, Float64, M * nu * nx)
    st = alloc(h, Int32, 1)
    check(ccall((:ilqr_backward, libilqr), Cint,
                (Ptr{Cvoid}, Ref{Problem}, Ref{Options}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Int32}),
                h.ptr, p, default_options(), xd, ud, dd, Kd, st), "ilqr_backward")
    du = from_abi(download!(h, zeros(nu, M), dd))                     # (T × nu)
    Kabi = download!(h, zeros(nx, nu, M), Kd)                          # C (T, nu, nx) row-major
    K = permutedims(Kabi, (3, 2, 1))                                   # (T × nu × nx) like 𝐊s
    return du, K
end

"""fit(x_init, u_init, dynamicsf, immediate_cost, final_cost; x_traj, max_iter, tol) -> (x̄, ū)"""
function fit(x_init::AbstractMatrix, u_init::AbstractMatrix, dynamicsf, immediate_cost, final_cost;
             x_traj=zero(x_init), max_iter::Int64=100, tol::Float64=1e-6)
    N, nx = size(x_init); M, nu = size(u_init)
    @assert(N == M + 1, "size(x_init)[2] == size(u_init)[1]")
    h = Handle(nx, nu, M, 1)
    p = Ref(problem(h, dynamicsf, immediate_cost, final_cost))
    o = default_options(); o.max_iter = max_iter; o.tol = tol
    xi = upload(h, to_abi(x_init)); ui = upload(h, to_abi(u_init)); xt = upload(h, to_abi(x_traj))
    xo = alloc(h, Float64, N * nx); uo = alloc(h, Float64, M * nu)
    st = ccall((:ilqr_fit, libilqr), Cint,
               (Ptr{Cvoid}, Ref{Problem}, Ref{Options}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64},
                Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Int32}, Ptr{Int32}),
               h.ptr, p, o, xi, ui, xt, xo, uo, C_NULL, C_NULL, C_NULL)
    st == ILQR_ERR_NAN && throw(AssertionError("!any(isnan, ...)"))
    st == ILQR_ERR_LS_EXHAUSTED || check(st, "ilqr_fit")
    return from_abi(download!(h, zeros(nx, N), xo)), from_abi(download!(h, zeros(nu, M), uo))
end

"""Batched problem (new API): per-instance A (nx,nx,B) … and trajectories (nx, N, B)."""
struct iLQRProblem
    A::Array{Float64,3}; B::Array{Float64,3}; Q::Array{Float64,3}; R::Array{Float64,3}; Qf::Array{Float64,3}
    x::Array{Float64,3}; u::Array{Float64,3}
end

"""solve!(prob; max_iter, tol): fits every instance; overwrites prob.x / prob.u."""
function solve!(prob::iLQRProblem; max_iter::Int64=100, tol::Float64=1e-6)
    nx, N, nb = size(prob.x); nu = size(prob.u, 1); M = N - 1
    h = Handle(nx, nu, M, nb)
    # Julia (nx, nx, B) column-major is C (B, nx, nx) with each matrix transposed
    tr(a) = Array{Float64}(permutedims(a, (2, 1, 3)))
    p = Ref(Problem(ILQR_PROBLEM_LQ, 0, upload(h, tr(prob.A)), upload(h, tr(prob.B)), upload(h, tr(prob.Q)),
                    upload(h, tr(prob.R)), upload(h, tr(prob.Qf))))
    o = default_options(); o.max_iter = max_iter; o.tol = tol
    xi = upload(h, prob.x); ui = upload(h, prob.u)
    xo = alloc(h, Float64, length(prob.x)); uo = alloc(h, Float64, length(prob.u))
    st = ccall((:ilqr_fit, libilqr), Cint,
               (Ptr{Cvoid}, Ref{Problem}, Ref{Options}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64},
                Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Int32}, Ptr{Int32}),
               h.ptr, p, o, xi, ui, C_NULL, xo, uo, C_NULL, C_NULL, C_NULL)
    st in (ILQR_OK, ILQR_ERR_LS_EXHAUSTED) || check(st, "ilqr_fit")
    download!(h, prob.x, xo); download!(h, prob.u, uo)
    return prob
end

"""solve!(prob, devices; …): the same over several GPUs of this node in one process
(ilqr_multi_fit: contiguous blocks of instances per device, host arrays in and out)."""
function solve!(prob::iLQRProblem, devices::Vector{Int}; max_iter::Int64=100, tol::Float64=1e-6)
    nx, N, nb = size(prob.x); nu = size(prob.u, 1); M = N - 1
    r = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:ilqr_multi_create, libilqr), Cint,
                (Ref{Ptr{Cvoid}}, Ptr{Cint}, Cint, Cint, Cint, Cint, Cint),
                r, Cint.(devices), length(devices), nx, nu, M, nb), "ilqr_multi_create")
    tr(a) = Array{Float64}(permutedims(a, (2, 1, 3)))
    A, B, Q, R, Qf = tr(prob.A), tr(prob.B), tr(prob.Q), tr(prob.R), tr(prob.Qf)
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

"""chain_fit(chain, x_init, u_init; max_iter, tol, linearization) → (x̄, ū, status)

Batched fit of the chain family; x_init (nx, T+1, batch), u_init (nu, T, batch) as
Array{Float32,3} (fp32, BASELINE config 5) or Array{Float64,3}: the element type picks
the device precision, as the reference's generic Julia code would."""
function chain_fit(c::Chain, x_init::Array{E,3}, u_init::Array{E,3}; max_iter::Int64=100,
                   tol::Float64=1e-6, linearization=ILQR_LINEARIZE_DUAL) where {E<:Union{Float32,Float64}}
    nx, N, nb = size(x_init); nu = size(u_init, 1); M = N - 1
    @assert(size(u_init, 2) == M)
    r = Ref{Ptr{Cvoid}}(C_NULL)
    dt = E === Float32 ? ILQR_F32 : ILQR_F64
    check(ccall((:ilqr_chain_create, libilqr), Cint,
                (Ref{Ptr{Cvoid}}, Cint, Ref{Chain}, Cint, Cint, Int32, Int32),
                r, 0, c, M, nb, dt, linearization), "ilqr_chain_create")
    h = Handle(nx, nu, M, 1)                 # device-memory helper only
    dev(a) = (p = alloc(h, E, length(a));
              check(ccall((:ilqr_memcpy_h2d, libilqr), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Csize_t),
                          h.ptr, p, a, sizeof(a)), "ilqr_memcpy_h2d"); p)
    xi = dev(x_init); ui = dev(u_init)
    xo = alloc(h, E, length(x_init)); uo = alloc(h, E, length(u_init)); sd = alloc(h, Int32, nb)
    o = default_options(); o.max_iter = max_iter; o.tol = tol
    st = ccall((:ilqr_chain_fit, libilqr), Cint,
               (Ptr{Cvoid}, Ref{Options}, Ptr{E}, Ptr{E}, Ptr{E}, Ptr{E}, Ptr{E}, Ptr{E}, Ptr{Int32}, Ptr{Int32}),
               r[], o, xi, ui, C_NULL, xo, uo, C_NULL, C_NULL, sd)
    st == ILQR_ERR_NAN && throw(AssertionError("!any(isnan, ...)"))
    st == ILQR_ERR_LS_EXHAUSTED || check(st, "ilqr_chain_fit")
    x = download!(h, similar(x_init), xo); u = download!(h, similar(u_init), uo)
    status = download!(h, zeros(Int32, nb), sd)
    ccall((:ilqr_chain_destroy, libilqr), Cint, (Ptr{Cvoid},), r[])
    return x, u, status
end

end # module
