// MI355X (gfx950) kernels + C ABI of the RBD problem family (ILQR_PROBLEM_CHAIN):
// a fixed-base serial chain of revolute joints described by a URDF — the
// reference's RigidBodyDynamics.jl example (test/RBD_2_link_example/
// RBD_helper_functions.jl:48-116 on test/urdf/2Dof_arm.urdf; BASELINE.json
// config 5) with a fixed base.
//
// What replaces what:
//  * dynamicsf (:48-79): RK4 of v̇ = M(q) \ (τ − dynamics_bias(q, v)), q̇ = v. The
//    device functor is Featherstone's recursive Newton-Euler (the published
//    algorithm behind RBD.jl's dynamics_bias) for the bias, and M's columns from the
//    same recursion with unit accelerations; everything templated on the scalar
//    (float / double / DualT<N, ·>).
//  * linearize_dynamics (src/backward_pass.jl:25-40, ForwardDiff): forward-mode dual
//    numbers (ILQR_LINEARIZE_DUAL, exact like the reference) or central finite
//    differences (ILQR_LINEARIZE_CENTRAL_FD, what BASELINE config 5 names), one lane
//    per (trajectory, step, direction).
//  * immediate_cost / final_cost (:85-116) on the joint rows: Σ qwᵢ(θ*ᵢ−θᵢ)² + Σ rwₖuₖ²
//    and Σ qfwᵢ(θ*ᵢ−θᵢ)²; their derivatives are the exact constants.
//  * backward_pass / forward_pass / fit: the Riccati recursion (four trajectories per
//    wave on the 4-block f64 MFMA for 2-joint chains, lane per trajectory otherwise)
//    and the RK4 rollout + α-halving line search (a 16-lane group per trajectory,
//    component-parallel Newton-Euler for chains of ≤ 3 joints), in the handle's dtype
//    (fp32 or fp64).
// Layout as the other families (include/ilqr.h): x (B, T+1, nx), u/d (B, T, nu),
// K (B, T, nu, nx), trajectory slowest, nx = 2·n_joints.
#include <hip/hip_runtime.h>
#include <math.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/ilqr.h"
#include "ilqr_internal.h"
#include "ilqr_device.h"
#include "ilqr_math.h"
#include "ilqr_fwd_group.h"

namespace ilqr {
namespace {

// ---------------------------------------------------------------------------
// scalar helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ void vsincos(float x, float& s, float& c) { fast_sincosf(x, s, c); }
__device__ __forceinline__ void vsincos(double x, double& s, double& c) { fast_sincos(x, s, c); }

// Forward-mode dual number over value type V (ForwardDiff.Dual restated).
template <int N, class V>
struct DualT {
  V v;
  V d[N];
  DualT() = default;
  __device__ __forceinline__ DualT(V c) : v(c) {
#pragma unroll
    for (int i = 0; i < N; ++i) d[i] = V(0);
  }
};
template <int N, class V>
__device__ __forceinline__ DualT<N, V> operator+(const DualT<N, V>& a, const DualT<N, V>& b) {
  DualT<N, V> r;
  r.v = a.v + b.v;
#pragma unroll
  for (int i = 0; i < N; ++i) r.d[i] = a.d[i] + b.d[i];
  return r;
}
template <int N, class V>
__device__ __forceinline__ DualT<N, V> operator-(const DualT<N, V>& a, const DualT<N, V>& b) {
  DualT<N, V> r;
  r.v = a.v - b.v;
#pragma unroll
  for (int i = 0; i < N; ++i) r.d[i] = a.d[i] - b.d[i];
  return r;
}
template <int N, class V>
__device__ __forceinline__ DualT<N, V> operator-(const DualT<N, V>& a) {
  DualT<N, V> r;
  r.v = -a.v;
#pragma unroll
  for (int i = 0; i < N; ++i) r.d[i] = -a.d[i];
  return r;
}
template <int N, class V>
__device__ __forceinline__ DualT<N, V> operator*(const DualT<N, V>& a, const DualT<N, V>& b) {
  DualT<N, V> r;
  r.v = a.v * b.v;
#pragma unroll
  for (int i = 0; i < N; ++i) r.d[i] = a.d[i] * b.v + a.v * b.d[i];
  return r;
}
template <int N, class V>
__device__ __forceinline__ DualT<N, V> operator*(V a, const DualT<N, V>& b) {
  DualT<N, V> r;
  r.v = a * b.v;
#pragma unroll
  for (int i = 0; i < N; ++i) r.d[i] = a * b.d[i];
  return r;
}
template <int N, class V>
__device__ __forceinline__ DualT<N, V> operator*(const DualT<N, V>& b, V a) { return a * b; }
template <int N, class V>
__device__ __forceinline__ DualT<N, V> operator+(V a, const DualT<N, V>& b) {
  DualT<N, V> r = b;
  r.v = a + b.v;
  return r;
}
template <int N, class V>
__device__ __forceinline__ DualT<N, V> operator-(V a, const DualT<N, V>& b) {
  DualT<N, V> r = -b;
  r.v = a - b.v;
  return r;
}
template <int N, class V>
__device__ __forceinline__ DualT<N, V> operator/(V a, const DualT<N, V>& b) {
  DualT<N, V> r;  // (a/b)' = −(a/b) b'/b
  r.v = a / b.v;
  const V k = -r.v / b.v;
#pragma unroll
  for (int i = 0; i < N; ++i) r.d[i] = k * b.d[i];
  return r;
}
template <int N, class V>
__device__ __forceinline__ void scs(const DualT<N, V>& a, DualT<N, V>& s, DualT<N, V>& c) {
  V sv, cv;
  vsincos(a.v, sv, cv);
  s.v = sv;
  c.v = cv;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    s.d[i] = cv * a.d[i];
    c.d[i] = -sv * a.d[i];
  }
}
__device__ __forceinline__ void scs(float a, float& s, float& c) { vsincos(a, s, c); }
__device__ __forceinline__ void scs(double a, double& s, double& c) { vsincos(a, s, c); }
// 1/x of the mass-matrix pivots: fp32 by v_rcp_f32 and one Newton step (within an
// ulp of the IEEE quotient; the IEEE division's scale/fixup sequence sat on the
// rollout's dependent chain), fp64 and duals by division
__device__ __forceinline__ float crecip(float x) {
  const float r = __builtin_amdgcn_rcpf(x);
  return fmaf(fmaf(-x, r, 1.0f), r, r);
}
__device__ __forceinline__ double crecip(double x) { return 1.0 / x; }
template <int N, class V>
__device__ __forceinline__ DualT<N, V> crecip(const DualT<N, V>& x) { return V(1) / x; }

// a pair of fp32 evaluations carried together (packed v_pk_* arithmetic)
typedef float F2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void scs(F2 a, F2& s, F2& c) {
  float s0, c0, s1, c1;
  vsincos(a.x, s0, c0);
  vsincos(a.y, s1, c1);
  s = F2{s0, s1};
  c = F2{c0, c1};
}
__device__ __forceinline__ F2 crecip(F2 x) {
  const F2 r = F2{__builtin_amdgcn_rcpf(x.x), __builtin_amdgcn_rcpf(x.y)};
  return (F2(1.0f) - x * r) * r + r;
}

template <class S> struct ValueOf { using type = S; };
template <int N, class V> struct ValueOf<DualT<N, V>> { using type = V; };

// ---------------------------------------------------------------------------
// Chain constants in the kernel's value type (converted from ilqr_chain on the host)
// ---------------------------------------------------------------------------
template <class V, int NJ>
struct ChainK {
  V R0[NJ][9];  // joint frame → parent body frame, row-major
  V R0x[NJ][9];  // R0·[a]×   } so that R0·Rot(a, q) = c·R0 + s·R0x + (1−c)·R0aa
  V R0aa[NJ][9]; // R0·a·aᵀ   } (Rodrigues expanded over the constant factors)
  V p[NJ][3];   // joint origin in the parent body frame
  V ax[NJ][3];  // unit axis (joint = child frame)
  V m[NJ];
  V mc[NJ][3];  // m · COM
  V Io[NJ][9];  // rotational inertia about the body origin
  V g[3];       // gravity
  V dt;
  V tgt[NJ], qw[NJ], rw[NJ], qfw[NJ];  // joint-space cost (RBD_helper_functions.jl:85-116)
};

template <class S>
__device__ __forceinline__ void cross3(const S (&a)[3], const S (&b)[3], S (&o)[3]) {
  o[0] = a[1] * b[2] - a[2] * b[1];
  o[1] = a[2] * b[0] - a[0] * b[2];
  o[2] = a[0] * b[1] - a[1] * b[0];
}
// a × b with a constant
template <class S, class V>
__device__ __forceinline__ void crossc(const V (&a)[3], const S (&b)[3], S (&o)[3]) {
  o[0] = a[1] * b[2] - a[2] * b[1];
  o[1] = a[2] * b[0] - a[0] * b[2];
  o[2] = a[0] * b[1] - a[1] * b[0];
}

// The joint transform R_i = R0_i Rot(a_i, q_i) (joint frame → parent body frame),
// built once per evaluation from (cos q, sin q): 9 × 3 ops, after which each of the
// recursion's 6 coordinate changes per joint is a 3×3 product (9 ops) instead of an
// in-place Rodrigues rotation (≈28). v7; the v6 form rotated every vector.
template <class S, class V, int NJ>
__device__ __forceinline__ void joint_rot(const ChainK<V, NJ>& P, int i, const S& c, const S& s,
                                          S (&R)[9]) {
  const S omc = V(1) - c;
#pragma unroll
  for (int k = 0; k < 9; ++k) R[k] = c * P.R0[i][k] + s * P.R0x[i][k] + omc * P.R0aa[i][k];
}
// parent → child coordinates: w_c = R_iᵀ w_p
template <class S>
__device__ __forceinline__ void to_child(const S (&R)[9], const S (&w)[3], S (&o)[3]) {
#pragma unroll
  for (int r = 0; r < 3; ++r) o[r] = R[r] * w[0] + R[3 + r] * w[1] + R[6 + r] * w[2];
}
// child → parent: w_p = R_i w_c
template <class S>
__device__ __forceinline__ void to_parent(const S (&R)[9], const S (&w)[3], S (&o)[3]) {
#pragma unroll
  for (int r = 0; r < 3; ++r) o[r] = R[3 * r] * w[0] + R[3 * r + 1] * w[1] + R[3 * r + 2] * w[2];
}

// Recursive Newton-Euler: τ = M(q) q̈ + [VEL] C(q, q̇)q̇ + [GRAV] g(q).
// qd is read only when VEL; qdd[i] is the joint acceleration.
// gs scales gravity (the lane-split forward runs the bias and the mass-matrix
// columns as one uniform pass with per-lane q̇, q̈ and gravity; 1 elsewhere, folded)
template <bool VEL, bool GRAV, int NJ, class S, class V>
__device__ __forceinline__ void rnea(const ChainK<V, NJ>& P, const S (&c)[NJ], const S (&s)[NJ],
                                     const S (&qd)[NJ], const S (&qdd)[NJ], S (&tau)[NJ],
                                     V gs = V(1)) {
  S w[3], v[3], al[3], ac[3];
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    w[r] = S(V(0));
    v[r] = S(V(0));
    al[r] = S(V(0));
    ac[r] = S(GRAV ? -P.g[r] * gs : V(0));  // fictitious base acceleration −g
  }
  // joint transforms as 3×3 products of the per-evaluation R_i (in-place Rodrigues
  // rotations measured slower once the linearisation ran one direction per lane,
  // DESIGN.md §4; tools/ablation/restore_alternates.patch)
  S fn[NJ][3], ff[NJ][3], R[NJ][9];
#pragma unroll
  for (int i = 0; i < NJ; ++i) joint_rot(P, i, c[i], s[i], R[i]);
  auto tc = [&](int i, const S (&w)[3], S (&o)[3]) { to_child(R[i], w, o); };
  auto tp = [&](int i, const S (&w)[3], S (&o)[3]) { to_parent(R[i], w, o); };
#pragma unroll
  for (int i = 0; i < NJ; ++i) {
    S t[3], u3[3];
    // spatial motion transform to body i: ω_i = X ω, v_i = X (v − p × ω) (same for accel)
    S wi[3], vi[3], ali[3], aci[3];
    tc(i, w, wi);
    crossc(P.p[i], w, t);
#pragma unroll
    for (int r = 0; r < 3; ++r) u3[r] = v[r] - t[r];
    tc(i, u3, vi);
    tc(i, al, ali);
    crossc(P.p[i], al, t);
#pragma unroll
    for (int r = 0; r < 3; ++r) u3[r] = ac[r] - t[r];
    tc(i, u3, aci);
    if constexpr (VEL) {
      S sq[3];
#pragma unroll
      for (int r = 0; r < 3; ++r) sq[r] = P.ax[i][r] * qd[i];  // S q̇
#pragma unroll
      for (int r = 0; r < 3; ++r) wi[r] = wi[r] + sq[r];
      cross3(wi, sq, t);  // (v ×m S q̇): angular part ω × Sq̇, linear part v × Sq̇
#pragma unroll
      for (int r = 0; r < 3; ++r) ali[r] = ali[r] + t[r];
      cross3(vi, sq, t);
#pragma unroll
      for (int r = 0; r < 3; ++r) aci[r] = aci[r] + t[r];
    }
#pragma unroll
    for (int r = 0; r < 3; ++r) ali[r] = ali[r] + P.ax[i][r] * qdd[i];
    // f = I a + v ×f (I v),  I·(α, a) = (Io α + mc × a, m a − mc × α)
#pragma unroll
    for (int r = 0; r < 3; ++r)
      fn[i][r] = P.Io[i][3 * r] * ali[0] + P.Io[i][3 * r + 1] * ali[1] + P.Io[i][3 * r + 2] * ali[2];
    crossc(P.mc[i], aci, t);
#pragma unroll
    for (int r = 0; r < 3; ++r) fn[i][r] = fn[i][r] + t[r];
    crossc(P.mc[i], ali, t);
#pragma unroll
    for (int r = 0; r < 3; ++r) ff[i][r] = P.m[i] * aci[r] - t[r];
    if constexpr (VEL) {
      S hn[3], hf[3];
#pragma unroll
      for (int r = 0; r < 3; ++r)
        hn[r] = P.Io[i][3 * r] * wi[0] + P.Io[i][3 * r + 1] * wi[1] + P.Io[i][3 * r + 2] * wi[2];
      crossc(P.mc[i], vi, t);
#pragma unroll
      for (int r = 0; r < 3; ++r) hn[r] = hn[r] + t[r];
      crossc(P.mc[i], wi, t);
#pragma unroll
      for (int r = 0; r < 3; ++r) hf[r] = P.m[i] * vi[r] - t[r];
      cross3(wi, hn, t);
#pragma unroll
      for (int r = 0; r < 3; ++r) fn[i][r] = fn[i][r] + t[r];
      cross3(vi, hf, t);
#pragma unroll
      for (int r = 0; r < 3; ++r) fn[i][r] = fn[i][r] + t[r];
      cross3(wi, hf, t);
#pragma unroll
      for (int r = 0; r < 3; ++r) ff[i][r] = ff[i][r] + t[r];
    }
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      w[r] = wi[r];
      v[r] = vi[r];
      al[r] = ali[r];
      ac[r] = aci[r];
    }
  }
#pragma unroll
  for (int i = NJ - 1; i >= 0; --i) {
    tau[i] = P.ax[i][0] * fn[i][0] + P.ax[i][1] * fn[i][1] + P.ax[i][2] * fn[i][2];
    if (i > 0) {
      S pf[3], pn[3], t[3];
      tp(i, ff[i], pf);
      tp(i, fn[i], pn);
      crossc(P.p[i], pf, t);
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        fn[i - 1][r] = fn[i - 1][r] + (pn[r] + t[r]);
        ff[i - 1][r] = ff[i - 1][r] + pf[r];
      }
    }
  }
}

// [q̇; v̇] with v̇ = M \ (τ − bias)  (RBD_helper_functions.jl:61-66).
// nu = NJ drives every joint; nu = 1 drives joint 1 only.
template <int NJ, int NU, class S, class V>
__device__ __forceinline__ void chain_xdot(const ChainK<V, NJ>& P, const S (&x)[2 * NJ],
                                           const S (&u)[NU], S (&xd)[2 * NJ]) {
  S c[NJ], s[NJ];
#pragma unroll
  for (int i = 0; i < NJ; ++i) scs(x[i], s[i], c[i]);
  S zero[NJ], qd[NJ], b[NJ];
#pragma unroll
  for (int i = 0; i < NJ; ++i) {
    zero[i] = S(V(0));
    qd[i] = x[NJ + i];
  }
  rnea<true, true>(P, c, s, qd, zero, b);  // dynamics_bias
  S M[NJ][NJ];
#pragma unroll
  for (int k = 0; k < NJ; ++k) {  // mass_matrix, column k = RNEA(q, 0, e_k)
    S e[NJ], col[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) e[j] = S(V(j == k ? 1 : 0));
    rnea<false, false>(P, c, s, zero, e, col);
#pragma unroll
    for (int i = 0; i < NJ; ++i) M[i][k] = col[i];
  }
  S r[NJ];
#pragma unroll
  for (int i = 0; i < NJ; ++i) r[i] = (i < NU ? u[i < NU ? i : 0] : S(V(0))) - b[i];
  // Gaussian elimination (M is SPD: no pivoting)
#pragma unroll
  for (int k = 0; k < NJ; ++k) {
    const S inv = crecip(M[k][k]);
#pragma unroll
    for (int i = k + 1; i < NJ; ++i) {
      const S l = M[i][k] * inv;
#pragma unroll
      for (int j = k + 1; j < NJ; ++j) M[i][j] = M[i][j] - l * M[k][j];
      r[i] = r[i] - l * r[k];
    }
  }
  S qdd[NJ];
#pragma unroll
  for (int i = NJ - 1; i >= 0; --i) {
    S acc = r[i];
#pragma unroll
    for (int j = i + 1; j < NJ; ++j) acc = acc - M[i][j] * qdd[j];
    qdd[i] = acc * crecip(M[i][i]);
  }
#pragma unroll
  for (int i = 0; i < NJ; ++i) {
    xd[i] = x[NJ + i];
    xd[NJ + i] = qdd[i];
  }
}

// ---------------------------------------------------------------------------
// Component-parallel Newton-Euler (v7 forward): a 16-lane group per trajectory,
// lane 4·role + c. The role picks the pass (0: bias with q̇ and gravity, k+1: M's
// column k), c ∈ {0,1,2} holds component c of every 3-vector (lane 3 of each quad
// computes a copy of component 0 and is never read). Cross products, rotations and
// dot products reach the other components of the same quad through DPP quad
// permutations, so each lane issues about a third of the scalar pass's arithmetic;
// the arithmetic per component is the scalar pass's, in the same order up to the
// association of three-term sums.
// ---------------------------------------------------------------------------
// bound_ctrl set: every source lane of a quad_perm / row_newbcast is valid, so it
// changes nothing but lets the compiler fold the move into a VOP2 consumer
// (v_mul_f32_dpp, v_add_f32_dpp: forward 1,733 → 1,653 instructions)
template <int CTRL, class V>
__device__ __forceinline__ V qperm(V x) {  // quad_perm DPP move
  if constexpr (sizeof(V) == 4) {
    return __builtin_bit_cast(V, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), CTRL, 0xF, 0xF, true));
  } else {
    const u2v p = __builtin_bit_cast(u2v, x);
    const u2v q = {(unsigned)__builtin_amdgcn_mov_dpp((int)p.x, CTRL, 0xF, 0xF, true),
                   (unsigned)__builtin_amdgcn_mov_dpp((int)p.y, CTRL, 0xF, 0xF, true)};
    return __builtin_bit_cast(V, q);
  }
}
constexpr int QP_B0 = 0x00, QP_B1 = 0x55, QP_B2 = 0xAA;  // broadcast component k
constexpr int QP_R1 = 0xC9, QP_R2 = 0xD2;                // component c+1 / c+2 (mod 3)
constexpr int QP_ROWBC = 0x150;                         // row_newbcast:n = 0x150 + n
// lane 4·role (component 0 of that pass) of the row, broadcast to the row
template <class V> __device__ __forceinline__ V rowbc_role(V x, int role) {
  return role == 1 ? qperm<QP_ROWBC + 4>(x) : role == 2 ? qperm<QP_ROWBC + 8>(x) : qperm<QP_ROWBC + 12>(x);
}
template <class V> __device__ __forceinline__ V bc0(V x) { return qperm<QP_B0>(x); }
template <class V> __device__ __forceinline__ V bc1(V x) { return qperm<QP_B1>(x); }
template <class V> __device__ __forceinline__ V bc2(V x) { return qperm<QP_B2>(x); }
template <class V> __device__ __forceinline__ V r1(V x) { return qperm<QP_R1>(x); }
template <class V> __device__ __forceinline__ V r2(V x) { return qperm<QP_R2>(x); }
// (a × b)_c = a_{c+1} b_{c+2} − a_{c+2} b_{c+1}
template <class V> __device__ __forceinline__ V cv_cross(V a, V b) { return r1(a) * r2(b) - r2(a) * r1(b); }
// constant a: the lane holds a1 = a_{c+1}, a2 = a_{c+2}
template <class V> __device__ __forceinline__ V cv_crossc(V a1, V a2, V b) { return a1 * r2(b) - a2 * r1(b); }
// Σ_k m_k w_k with m_k the lane's row (m[c][k]) or column entries
template <class V> __device__ __forceinline__ V cv_mat(V m0, V m1, V m2, V w) {
  return m0 * bc0(w) + m1 * bc1(w) + m2 * bc2(w);
}

template <bool VEL, bool GRAV, int NJ, class V>
__device__ __forceinline__ void rnea_cv(const ChainK<V, NJ>& P, const V (&c)[NJ], const V (&s)[NJ],
                                        const V (&qd)[NJ], const V (&qdd)[NJ], V (&tau)[NJ], V gs,
                                        int cmp) {
  const int c0 = cmp < 3 ? cmp : 0;
  const int c1 = c0 == 2 ? 0 : c0 + 1, c2 = c0 == 0 ? 2 : c0 - 1;
  V w = V(0), v = V(0), al = V(0), ac = GRAV ? -P.g[c0] * gs : V(0);
  V fn[NJ], ff[NJ], Rr[NJ][3], Rc[NJ][3];
#pragma unroll
  for (int i = 0; i < NJ; ++i) {  // row c and column c of R_i = R0 Rot(a, q)
    const V omc = V(1) - c[i];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      Rr[i][k] = c[i] * P.R0[i][3 * c0 + k] + s[i] * P.R0x[i][3 * c0 + k] + omc * P.R0aa[i][3 * c0 + k];
      Rc[i][k] = c[i] * P.R0[i][3 * k + c0] + s[i] * P.R0x[i][3 * k + c0] + omc * P.R0aa[i][3 * k + c0];
    }
  }
#pragma unroll
  for (int i = 0; i < NJ; ++i) {
    const V p1 = P.p[i][c1], p2 = P.p[i][c2], mc1 = P.mc[i][c1], mc2 = P.mc[i][c2];
    const V axc = P.ax[i][c0];
    // to_child: w_c = Σ_k R[k][c] w_k
    V wi = cv_mat(Rc[i][0], Rc[i][1], Rc[i][2], w);
    V vi = cv_mat(Rc[i][0], Rc[i][1], Rc[i][2], v - cv_crossc(p1, p2, w));
    V ali = cv_mat(Rc[i][0], Rc[i][1], Rc[i][2], al);
    V aci = cv_mat(Rc[i][0], Rc[i][1], Rc[i][2], ac - cv_crossc(p1, p2, al));
    if constexpr (VEL) {
      const V sq = axc * qd[i];
      wi = wi + sq;
      ali = ali + cv_cross(wi, sq);
      aci = aci + cv_cross(vi, sq);
    }
    ali = ali + axc * qdd[i];
    fn[i] = cv_mat(P.Io[i][3 * c0], P.Io[i][3 * c0 + 1], P.Io[i][3 * c0 + 2], ali) + cv_crossc(mc1, mc2, aci);
    ff[i] = P.m[i] * aci - cv_crossc(mc1, mc2, ali);
    if constexpr (VEL) {
      const V hn = cv_mat(P.Io[i][3 * c0], P.Io[i][3 * c0 + 1], P.Io[i][3 * c0 + 2], wi) + cv_crossc(mc1, mc2, vi);
      const V hf = P.m[i] * vi - cv_crossc(mc1, mc2, wi);
      fn[i] = fn[i] + cv_cross(wi, hn);
      fn[i] = fn[i] + cv_cross(vi, hf);
      ff[i] = ff[i] + cv_cross(wi, hf);
    }
    w = wi;
    v = vi;
    al = ali;
    ac = aci;
  }
#pragma unroll
  for (int i = NJ - 1; i >= 0; --i) {
    const V pr = P.ax[i][c0] * fn[i];  // S_iᵀ f_i over the three components
    tau[i] = (bc0(pr) + bc1(pr)) + bc2(pr);
    if (i > 0) {
      const V pf = cv_mat(Rr[i][0], Rr[i][1], Rr[i][2], ff[i]);  // to_parent: Σ_k R[c][k] f_k
      const V pn = cv_mat(Rr[i][0], Rr[i][1], Rr[i][2], fn[i]);
      fn[i - 1] = fn[i - 1] + (pn + cv_crossc(P.p[i][c1], P.p[i][c2], pf));
      ff[i - 1] = ff[i - 1] + pf;
    }
  }
}

// chain_xdot over a 16-lane group: role = pass, c = component (see rnea_cv); every
// lane of the group ends with the same [q̇; v̇]
template <int NJ, int NU, class V>
__device__ __forceinline__ void chain_xdot_cv(const ChainK<V, NJ>& P, const V (&x)[2 * NJ],
                                              const V (&u)[NU], V (&xd)[2 * NJ]) {
  static_assert(NJ + 1 <= 4, "one role per pass in a group of 16");
  // lane c of a quad evaluates joint min(c, NJ − 1) and the quad reads joint i from its
  // lane i (bc0/bc1/bc2 below): only joints 0..2 have a broadcast
  static_assert(NJ <= 3, "one sin/cos per lane: a quad holds at most three joints");
  const int l16 = threadIdx.x & 15;
  const int role = l16 >> 2, cmp = l16 & 3;
  V c[NJ], s[NJ], qd[NJ], qdd[NJ], tau[NJ];
  // one sin/cos per lane: lane c of each quad evaluates joint min(c, NJ − 1), and the
  // quad reads joint i's pair from its lane i by DPP quad broadcast (the same bits as
  // evaluating every joint in every lane, at one polynomial pair per lane)
  V ang = x[0];
#pragma unroll
  for (int i = 1; i < NJ; ++i)
    if (cmp >= i) ang = x[i];
  V so, co;
  scs(ang, so, co);
#pragma unroll
  for (int i = 0; i < NJ; ++i) {
    s[i] = i == 0 ? bc0(so) : i == 1 ? bc1(so) : bc2(so);
    c[i] = i == 0 ? bc0(co) : i == 1 ? bc1(co) : bc2(co);
    qd[i] = role == 0 ? x[NJ + i] : V(0);
    qdd[i] = V(role == i + 1 ? 1 : 0);
  }
  rnea_cv<true, true>(P, c, s, qd, qdd, tau, V(role == 0 ? 1 : 0), cmp);
  V b[NJ], M[NJ][NJ];
#pragma unroll
  for (int i = 0; i < NJ; ++i) {
    // the group is a DPP row (16 lanes): row_newbcast:n (gfx90a+) hands lane n of the
    // row to all of it on the VALU, off the LDS crossbar that ds_bpermute goes through
    b[i] = qperm<QP_ROWBC + 0>(tau[i]);
#pragma unroll
    for (int k = 0; k < NJ; ++k) M[i][k] = rowbc_role(tau[i], 1 + k);
  }
  V r[NJ];
#pragma unroll
  for (int i = 0; i < NJ; ++i) r[i] = (i < NU ? u[i < NU ? i : 0] : V(0)) - b[i];
#pragma unroll
  for (int k = 0; k < NJ; ++k) {
    const V inv = crecip(M[k][k]);
#pragma unroll
    for (int i = k + 1; i < NJ; ++i) {
      const V lk = M[i][k] * inv;
#pragma unroll
      for (int j = k + 1; j < NJ; ++j) M[i][j] = M[i][j] - lk * M[k][j];
      r[i] = r[i] - lk * r[k];
    }
  }
  V q2[NJ];
#pragma unroll
  for (int i = NJ - 1; i >= 0; --i) {
    V acc = r[i];
#pragma unroll
    for (int j = i + 1; j < NJ; ++j) acc = acc - M[i][j] * q2[j];
    q2[i] = acc * crecip(M[i][i]);
  }
#pragma unroll
  for (int i = 0; i < NJ; ++i) {
    xd[i] = x[NJ + i];
    xd[NJ + i] = q2[i];
  }
}

// ---------------------------------------------------------------------------
// Closed-form dynamics of a 2-joint fixed-base chain (round 2, the default for the
// iteration kernels of 2-joint chains). M(q) depends on q₂ only (turning the whole
// chain about joint 1's fixed axis preserves its kinetic energy) and is a trigonometric
// polynomial of degree 2 in q₂ (body 2's rotation enters its kinetic energy
// quadratically, every factor affine in cos q₂, sin q₂); the gravity torque ∂V/∂q is
// bilinear in (1, cos q₁, sin q₁) ⊗ (1, cos q₂, sin q₂) (each COM's height is). The
// coefficients are sampled from the recursive Newton-Euler above, in fp64, when the
// handle is created — M at 5 angles, g on a 3×3 grid: the discrete Fourier transform is
// exact for these degrees — and the result is checked against the recursion at random
// states before it is used (chain_trig_check_kernel). The velocity term is the
// Christoffel form of M′ = dM/dq₂: c = q̇₂·M′q̇ − ½ e₂ q̇ᵀM′q̇. The same f(x, u) as the
// recursion (RBD_helper_functions.jl:61-66), ≈60 operations and two sin/cos instead
// of the three Newton-Euler passes; the rounding differs.
// ---------------------------------------------------------------------------
// ---------------------------------------------------------------------------
// cost_functions.jl's task-space final cost (src/cost_functions.jl:5-27, the device side
// of ilqr_chain_set_simple_costs): ℓ_f(x) = w Σ_k (p_k(q) − t_k)² where p is the root-
// frame position of a point fixed on one body. Through two revolute joints each
// coordinate is bilinear in (1, cos q₁, sin q₁) ⊗ (1, cos q₂, sin q₂) (Rodrigues is
// affine in cos, sin of each angle), so the handle stores the coefficients, sampled from
// the kinematics on the 3×3 grid like g's. The reference's reading takes the point's z
// for every k (work_space_traj[end] .- transpose(final_target), :21): the handle then
// stores z's coefficients in all three rows. Lives in device memory (one pointer in the
// kernel arguments; read only when the cost mode is set).
// ---------------------------------------------------------------------------
struct ChainTask {
  double Pc[3][3][3];  // p_k = Σ_ab Pc[k][a][b] φ_a(q₁) φ_b(q₂), φ = (1, cos, sin)
  double t[3];         // final_target
  double w;            // weight
};

// ℓ_f(q) in V (the forward's final cost, forward_pass.jl:192); the sum runs in the
// reference's order: weight · ((e₁² + e₂²) + e₃²) (cost_functions.jl:21-23)
template <class V>
__device__ __forceinline__ V chain_task_cost(const ChainTask* __restrict__ C, V q0, V q1) {
  V s0, c0, s1, c1;
  vsincos(q0, s0, c0);
  vsincos(q1, s1, c1);
  V acc = V(0);
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    V h[3];
#pragma unroll
    for (int a = 0; a < 3; ++a)
      h[a] = (V)C->Pc[k][a][0] + ((V)C->Pc[k][a][1] * c1 + (V)C->Pc[k][a][2] * s1);
    const V e = (h[0] + (h[1] * c0 + h[2] * s0)) - (V)C->t[k];
    acc = acc + e * e;
  }
  return (V)C->w * acc;
}

// ∇ℓ_f and ∇²ℓ_f on (q₁, q₂) in f64 (final_cost_quadratization, backward_pass.jl:134-153):
// 2w Σ_k e_k ∇p_k and 2w Σ_k (∇p_k ∇p_kᵀ + e_k ∇²p_k), e_k = p_k − t_k. H = (H₁₁, H₁₂, H₂₂).
__device__ __forceinline__ void chain_task_quad(const ChainTask* __restrict__ C, double q0, double q1,
                                                double (&g)[2], double (&H)[3]) {
  double s0, c0, s1, c1;
  vsincos(q0, s0, c0);
  vsincos(q1, s1, c1);
  g[0] = g[1] = H[0] = H[1] = H[2] = 0.0;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    double h[3], hd[3], hdd[3];  // φ(q₂), φ′(q₂), φ″(q₂) contracted with the q₂ index
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      const double* r = C->Pc[k][a];
      h[a] = r[0] + (r[1] * c1 + r[2] * s1);
      hd[a] = r[2] * c1 - r[1] * s1;
      hdd[a] = -(r[1] * c1 + r[2] * s1);
    }
    const double p = h[0] + (h[1] * c0 + h[2] * s0);
    const double p0 = h[2] * c0 - h[1] * s0, p1 = hd[0] + (hd[1] * c0 + hd[2] * s0);
    const double p00 = -(h[1] * c0 + h[2] * s0), p01 = hd[2] * c0 - hd[1] * s0;
    const double p11 = hdd[0] + (hdd[1] * c0 + hdd[2] * s0);
    const double e = p - C->t[k];
    g[0] += e * p0;
    g[1] += e * p1;
    H[0] += p0 * p0 + e * p00;
    H[1] += p0 * p1 + e * p01;
    H[2] += p1 * p1 + e * p11;
  }
  const double w2 = 2.0 * C->w;
  g[0] *= w2;
  g[1] *= w2;
  H[0] *= w2;
  H[1] *= w2;
  H[2] *= w2;
}

template <class V>
struct ChainTrig {
  V Mc[3][5];     // M₀₀, M₀₁, M₁₁: a₀ + a₁ cos q₂ + b₁ sin q₂ + a₂ cos 2q₂ + b₂ sin 2q₂
  V Gc[2][3][3];  // g_i = Σ_ab Gc[i][a][b] φ_a(q₁) φ_b(q₂), φ = (1, cos, sin)
  V dt;
  V tgt[2], qw[2], rw[2], qfw[2];  // joint-space cost (as ChainK)
  const ChainTask* task;           // the task-space final cost in place of qfw's, or null
};

// q̈ from sin/cos of both joint angles, q̇ = (w0, w1) and u
template <int NU, class S, class V>
__device__ __forceinline__ void chain_qdd_trig(const ChainTrig<V>& P, const S& s1, const S& c1, const S& s2,
                                               const S& c2, const S& w0, const S& w1, const S (&u)[NU],
                                               S& a0, S& a1) {
  S m[3], dm[3];
#pragma unroll
  for (int e = 0; e < 3; ++e) {
    // M_e = a₀ + a₁ cos + b₁ sin + a₂ cos 2q + b₂ sin 2q and dM_e/dq₂ = b₁ cos − a₁ sin +
    // 2(b₂ cos 2q − a₂ sin 2q) in Horner form in (cos q₂, sin q₂), as chain_qdd_trig2 (the
    // kernel argument holds M's coefficients only: fewer scalar registers than a second table)
    const V a0 = P.Mc[e][0], a1 = P.Mc[e][1], b1 = P.Mc[e][2], a2 = P.Mc[e][3], b2 = P.Mc[e][4];
    m[e] = (a0 - a2) + c2 * ((a1 + (V(2) * a2) * c2) + (V(2) * b2) * s2) + b1 * s2;
    dm[e] = V(-2) * b2 + c2 * ((b1 + (V(4) * b2) * c2) - (V(4) * a2) * s2) - a1 * s2;
  }
  S g[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    S h[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) h[a] = P.Gc[i][a][0] + (P.Gc[i][a][1] * c2 + P.Gc[i][a][2] * s2);
    g[i] = h[0] + (h[1] * c1 + h[2] * s1);
  }
  const S p0 = dm[0] * w0 + dm[1] * w1, p1 = dm[1] * w0 + dm[2] * w1;  // M′q̇
  const S qq = w0 * p0 + w1 * p1;                                      // q̇ᵀM′q̇
  S r0 = u[0] - (w1 * p0 + g[0]);
  S r1 = (w1 * p1 - V(0.5) * qq) + g[1];
  if constexpr (NU > 1) r1 = u[NU - 1] - r1;
  else r1 = -r1;
  const S det = m[0] * m[2] - m[1] * m[1];
  const S id = crecip(det);
  a0 = (m[2] * r0 - m[1] * r1) * id;
  a1 = (m[0] * r1 - m[1] * r0) * id;
}

template <int NU, class S, class V>
__device__ __forceinline__ void chain_xdot_trig(const ChainTrig<V>& P, const S (&x)[4], const S (&u)[NU],
                                                S (&xd)[4]) {
  S s1, c1, s2, c2;
  scs(x[0], s1, c1);
  scs(x[1], s2, c2);
  xd[0] = x[2];
  xd[1] = x[3];
  chain_qdd_trig<NU>(P, s1, c1, s2, c2, x[2], x[3], u, xd[2], xd[3]);
}

// One RK4 step of the closed form without a branch (the forward's fast path, as the
// 2-link's rk4_roll): stage 1 reduces both angles, stages 2-4 shift their sin/cos by
// h = ½k₁, ½k₂, k₃ (|h| ≤ 1/8); `bad` flags |h| > 1/8 or an angle past the reduction's
// range, and the caller redoes the rollout on chain_rk4 (NaN: not flagged, NaN either way)
// sin/cos of both joint angles carried from step to step (the forward group's carry): the
// step's stage 1 reads them and leaves those of the new state by the stages' angle shift
template <class V>
struct ChainCarry {
  V s[2], c[2];
};

template <int NU, class V>
__device__ __forceinline__ void chain_trig_rk4_fast(const ChainTrig<V>& P, const V (&x)[4], const V (&u)[NU],
                                                    V (&out)[4], bool& bad, ChainCarry<V>& cy) {
  const V h = V(0.5);
  V s1, c1, s2, c2, a0, a1;
  const V s10 = cy.s[0], c10 = cy.c[0], s20 = cy.s[1], c20 = cy.c[1];
  chain_qdd_trig<NU>(P, s10, c10, s20, c20, x[2], x[3], u, a0, a1);
  const V k10 = P.dt * x[2], k11 = P.dt * x[3], k12 = P.dt * a0, k13 = P.dt * a1;
  V y2 = x[2] + h * k12, y3 = x[3] + h * k13;
  sincos_shift_t(s10, c10, h * k10, s1, c1);
  sincos_shift_t(s20, c20, h * k11, s2, c2);
  chain_qdd_trig<NU>(P, s1, c1, s2, c2, y2, y3, u, a0, a1);
  const V k20 = P.dt * y2, k21 = P.dt * y3, k22 = P.dt * a0, k23 = P.dt * a1;
  y2 = x[2] + h * k22;
  y3 = x[3] + h * k23;
  sincos_shift_t(s10, c10, h * k20, s1, c1);
  sincos_shift_t(s20, c20, h * k21, s2, c2);
  chain_qdd_trig<NU>(P, s1, c1, s2, c2, y2, y3, u, a0, a1);
  const V k30 = P.dt * y2, k31 = P.dt * y3, k32 = P.dt * a0, k33 = P.dt * a1;
  y2 = x[2] + k32;
  y3 = x[3] + k33;
  sincos_shift_t(s10, c10, k30, s1, c1);
  sincos_shift_t(s20, c20, k31, s2, c2);
  chain_qdd_trig<NU>(P, s1, c1, s2, c2, y2, y3, u, a0, a1);
  const V k40 = P.dt * y2, k41 = P.dt * y3, k42 = P.dt * a0, k43 = P.dt * a1;
  const V sixth = V(1) / V(6);
  out[0] = x[0] + sixth * (((k10 + V(2) * k20) + V(2) * k30) + k40);
  out[1] = x[1] + sixth * (((k11 + V(2) * k21) + V(2) * k31) + k41);
  out[2] = x[2] + sixth * (((k12 + V(2) * k22) + V(2) * k32) + k42);
  out[3] = x[3] + sixth * (((k13 + V(2) * k23) + V(2) * k33) + k43);
  const V h0 = out[0] - x[0], h1 = out[1] - x[1];
  sincos_shift_t(s10, c10, h0, cy.s[0], cy.c[0]);
  sincos_shift_t(s20, c20, h1, cy.s[1], cy.c[1]);
  const V hm = fmax(fmax(fmax(fabs(k10), fabs(k11)), fmax(fabs(k20), fabs(k21))),
                    V(2) * fmax(fmax(fabs(k30), fabs(k31)), fmax(fabs(h0), fabs(h1))));
  bad |= ((int)(hm > V(0.25)) | (int)(fabs(x[0]) > ReducedRange<V>::v) | (int)(fabs(x[1]) > ReducedRange<V>::v)) != 0;
}

// ---------------------------------------------------------------------------
// The fp32 fast step with the two joints packed (v_pk_* arithmetic on (joint 1,
// joint 2) pairs: the angle reductions and shifts, M's diagonal, g, M′q̇, the solve and
// the RK4 glue), the configuration BASELINE config 5 runs. The formulas of
// chain_trig_rk4_fast per component (FMA contraction may place roundings differently).
// ---------------------------------------------------------------------------
__device__ __forceinline__ F2 f2fma(F2 a, F2 b, F2 c) { return __builtin_elementwise_fma(a, b, c); }

// sincos_shift_t (fp32) on both components
__device__ __forceinline__ void sincos2_shift(F2 s0, F2 c0, F2 h, F2& s, F2& c) {
  const F2 z = h * h;
  const F2 sh = f2fma(h * z, f2fma(z, F2(1.0f / 120.0f), F2(-1.0f / 6.0f)), h);
  const F2 ch = f2fma(z, f2fma(z, F2(1.0f / 24.0f), F2(-0.5f)), F2(1.0f));
  s = f2fma(s0, ch, c0 * sh);
  c = f2fma(c0, ch, -(s0 * sh));
}

// q̈ (both joints) from packed sin/cos (joint 1, joint 2), q̇ and u
template <int NU>
__device__ __forceinline__ F2 chain_qdd_trig2(const ChainTrig<float>& P, F2 sn, F2 cs, F2 w, const float (&u)[NU]) {
  const float s2 = sn.y, c2 = cs.y;
  // M's entries a₀ + a₁ cos q₂ + b₁ sin q₂ + a₂ cos 2q₂ + b₂ sin 2q₂ and their derivatives
  // b₁ cos − a₁ sin + 2(b₂ cos 2q − a₂ sin 2q), in Horner form in (cos q₂, sin q₂):
  // k₀ + c·(k₁ + k₂ c + k₃ s) + k₄ s, with M: (a₀ − a₂, a₁, 2a₂, 2b₂, b₁) and
  // dM: (−2b₂, b₁, 4b₂, −4a₂, −a₁) (loop-invariant coefficient pairs)
  auto horner = [&](F2 k0, F2 k1, F2 k2, F2 k3, F2 k4) {
    const F2 in = f2fma(k3, F2(s2), f2fma(k2, F2(c2), k1));
    return f2fma(k4, F2(s2), f2fma(in, F2(c2), k0));
  };
  auto a0 = [&](int e) { return P.Mc[e][0]; };
  auto a1 = [&](int e) { return P.Mc[e][1]; };
  auto b1 = [&](int e) { return P.Mc[e][2]; };
  auto a2 = [&](int e) { return P.Mc[e][3]; };
  auto b2 = [&](int e) { return P.Mc[e][4]; };
  // (M₀₀, M₁₁), (M₀₁, dM₀₁/dq₂), (dM₀₀, dM₁₁) as pairs
  const F2 md = horner(F2{a0(0) - a2(0), a0(2) - a2(2)}, F2{a1(0), a1(2)}, F2{2.0f * a2(0), 2.0f * a2(2)},
                       F2{2.0f * b2(0), 2.0f * b2(2)}, F2{b1(0), b1(2)});
  const F2 mo = horner(F2{a0(1) - a2(1), -2.0f * b2(1)}, F2{a1(1), b1(1)}, F2{2.0f * a2(1), 4.0f * b2(1)},
                       F2{2.0f * b2(1), -4.0f * a2(1)}, F2{b1(1), -a1(1)});
  const F2 dmd = horner(F2{-2.0f * b2(0), -2.0f * b2(2)}, F2{b1(0), b1(2)}, F2{4.0f * b2(0), 4.0f * b2(2)},
                        F2{-4.0f * a2(0), -4.0f * a2(2)}, F2{-a1(0), -a1(2)});
  // g (both components): h_a = G[·][a][0] + G[·][a][1] cos q₂ + G[·][a][2] sin q₂
  F2 h[3];
#pragma unroll
  for (int a = 0; a < 3; ++a)
    h[a] = F2{P.Gc[0][a][0], P.Gc[1][a][0]} +
           (F2{P.Gc[0][a][1], P.Gc[1][a][1]} * c2 + F2{P.Gc[0][a][2], P.Gc[1][a][2]} * s2);
  const F2 g = h[0] + (h[1] * cs.x + h[2] * sn.x);
  // M′q̇ = (dM₀₀ w₀ + dM₀₁ w₁, dM₀₁ w₀ + dM₁₁ w₁), packed
  const F2 p = f2fma(F2{mo.y, mo.y}, w.yx, dmd * w);
  const float qq = w.x * p.x + w.y * p.y;
  const F2 t = f2fma(F2{w.y, w.y}, p, g);  // (w₁p₀ + g₀, w₁p₁ + g₁)
  const float r0 = u[0] - t.x;
  float r1 = t.y - 0.5f * qq;
  if constexpr (NU > 1) r1 = u[NU - 1] - r1;
  else r1 = -r1;
  const float det = md.x * md.y - mo.x * mo.x;
  const float id = crecip(det);
  // M⁻¹r = (M₁₁ r₀ − M₀₁ r₁, M₀₀ r₁ − M₀₁ r₀) / det, packed
  const F2 r{r0, r1};
  return (md.yx * r - F2{mo.x, mo.x} * r.yx) * id;
}

template <int NU>
__device__ __forceinline__ void chain_trig_rk4_fast2(const ChainTrig<float>& P, const float (&x)[4],
                                                     const float (&u)[NU], float (&out)[4], bool& bad,
                                                     ChainCarry<float>& cy) {
  const F2 q{x[0], x[1]}, w{x[2], x[3]};
  const float dt = P.dt;
  const F2 s0{cy.s[0], cy.s[1]}, c0{cy.c[0], cy.c[1]};
  F2 sn, cs;
  F2 a = chain_qdd_trig2<NU>(P, s0, c0, w, u);
  const F2 k1p = dt * w, k1v = dt * a;
  F2 y = w + 0.5f * k1v;
  sincos2_shift(s0, c0, 0.5f * k1p, sn, cs);
  a = chain_qdd_trig2<NU>(P, sn, cs, y, u);
  const F2 k2p = dt * y, k2v = dt * a;
  y = w + 0.5f * k2v;
  sincos2_shift(s0, c0, 0.5f * k2p, sn, cs);
  a = chain_qdd_trig2<NU>(P, sn, cs, y, u);
  const F2 k3p = dt * y, k3v = dt * a;
  y = w + k3v;
  sincos2_shift(s0, c0, k3p, sn, cs);
  a = chain_qdd_trig2<NU>(P, sn, cs, y, u);
  const F2 k4p = dt * y, k4v = dt * a;
  const float sixth = 1.0f / 6.0f;
  const F2 op = q + sixth * (((k1p + 2.0f * k2p) + 2.0f * k3p) + k4p);
  const F2 ov = w + sixth * (((k1v + 2.0f * k2v) + 2.0f * k3v) + k4v);
  out[0] = op.x; out[1] = op.y; out[2] = ov.x; out[3] = ov.y;
  const F2 hq = op - q;  // the carry: sin/cos of the new angles
  F2 sq, cq;
  sincos2_shift(s0, c0, hq, sq, cq);
  cy.s[0] = sq.x; cy.s[1] = sq.y; cy.c[0] = cq.x; cy.c[1] = cq.y;
  const F2 m1 = __builtin_elementwise_max(__builtin_elementwise_abs(k1p), __builtin_elementwise_abs(k2p));
  const F2 m2 = __builtin_elementwise_max(__builtin_elementwise_max(m1, 2.0f * __builtin_elementwise_abs(k3p)),
                                          2.0f * __builtin_elementwise_abs(hq));
  const float hm = fmaxf(m2.x, m2.y);
  bad |= ((int)(hm > 0.25f) | (int)(fabsf(x[0]) > 8192.0f) | (int)(fabsf(x[1]) > 8192.0f)) != 0;
}

// the chain's closed form as a model of the shared forward group (ilqr_fwd_group.h)
template <class V_, int NU_>
struct ChainTrigModel {
  using V = V_;
  static constexpr int NU = NU_;
  static constexpr bool HAS_FAST = true;
  static constexpr bool HAS_CARRY = true;
  using Carry = ChainCarry<V>;
  ChainTrig<V> P;
  __device__ __forceinline__ Carry carry_init(const V (&x)[4]) const {
    Carry k;
    sincos_red_t(x[0], k.s[0], k.c[0]);
    sincos_red_t(x[1], k.s[1], k.c[1]);
    return k;
  }
  __device__ __forceinline__ void rk4_fast(const V (&x)[4], const V (&u)[NU], V (&o)[4], bool& bad,
                                           Carry& k) const {
    // fp32: the joints packed (v_pk_* pairs)
    if constexpr (std::is_same_v<V, float>) chain_trig_rk4_fast2<NU>(P, x, u, o, bad, k);
    else chain_trig_rk4_fast<NU>(P, x, u, o, bad, k);
  }
  __device__ __forceinline__ void rk4_robust(const V (&x)[4], const V (&u)[NU], V (&o)[4]) const;
  // ℓ(x̄ₖ − x_trajₖ, ūₖ) on the joints (forward_pass.jl:187-190; RBD_helper_functions.jl:85-99)
  __device__ __forceinline__ V stage_cost(const V (&xb)[4], const V (&xt)[4], V xtw, const V (&ub)[NU]) const {
    V lk = V(0);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const V e = P.tgt[i] - fma(-xtw, xt[i], xb[i]);
      lk = fma(P.qw[i] * e, e, lk);
    }
#pragma unroll
    for (int a = 0; a < NU; ++a) lk = fma(P.rw[a] * ub[a], ub[a], lk);
    return lk;
  }
  // final_cost(x̄_N) on the raw state (:192; RBD_helper_functions.jl:105-116)
  __device__ __forceinline__ V final_cost(const V (&xb)[4]) const {
    if (P.task) return chain_task_cost<V>(P.task, xb[0], xb[1]);  // cost_functions.jl:16-24
    V lf = V(0);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const V e = P.tgt[i] - xb[i];
      lf = fma(P.qfw[i] * e, e, lf);
    }
    return lf;
  }
};

// RK4 (RBD_helper_functions.jl:70-78) on either parameter set: ChainK (the recursion;
// SPLIT = the 16-lane component-parallel form) or ChainTrig (closed form, 2 joints)
template <int NJ, int NU, bool SPLIT = false, class S, class PK>
__device__ __forceinline__ void chain_rk4(const PK& P, const S (&x)[2 * NJ],
                                          const S (&u)[NU], S (&out)[2 * NJ]) {
  constexpr int NX = 2 * NJ;
  using V = decltype(P.dt);
  auto xdot = [](const PK& Pc, const S (&xx)[2 * NJ], const S (&uu)[NU], S (&o)[2 * NJ]) {
    if constexpr (std::is_same_v<PK, ChainTrig<V>>)
      chain_xdot_trig<NU>(Pc, xx, uu, o);
    else if constexpr (SPLIT)
      chain_xdot_cv<NJ, NU>(Pc, xx, uu, o);
    else
      chain_xdot<NJ, NU>(Pc, xx, uu, o);
  };
  S k1[NX], k2[NX], k3[NX], k4[NX], y[NX];
  const V h = V(0.5);
  xdot(P, x, u, k1);
#pragma unroll
  for (int i = 0; i < NX; ++i) {
    k1[i] = P.dt * k1[i];
    y[i] = x[i] + h * k1[i];
  }
  xdot(P, y, u, k2);
#pragma unroll
  for (int i = 0; i < NX; ++i) {
    k2[i] = P.dt * k2[i];
    y[i] = x[i] + h * k2[i];
  }
  xdot(P, y, u, k3);
#pragma unroll
  for (int i = 0; i < NX; ++i) {
    k3[i] = P.dt * k3[i];
    y[i] = x[i] + k3[i];
  }
  xdot(P, y, u, k4);
#pragma unroll
  for (int i = 0; i < NX; ++i) {
    k4[i] = P.dt * k4[i];
    out[i] = x[i] + (V(1) / V(6)) * (((k1[i] + V(2) * k2[i]) + V(2) * k3[i]) + k4[i]);
  }
}

template <class V_, int NU_>
__device__ __forceinline__ void ChainTrigModel<V_, NU_>::rk4_robust(const V (&x)[4], const V (&u)[NU],
                                                                   V (&o)[4]) const {
  chain_rk4<2, NU>(P, x, u, o);
}

// ---------------------------------------------------------------------------
// f(x, u) for n points (a rollout primitive and the dynamics parity test)
// ---------------------------------------------------------------------------
template <class V, int NJ, int NU, class PK = ChainK<V, NJ>>
__global__ __launch_bounds__(256) void chain_dynamics_kernel(PK P, int n,
                                                             const V* __restrict__ x,
                                                             const V* __restrict__ u,
                                                             V* __restrict__ xo) {
  constexpr int NX = 2 * NJ;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  V xs[NX], us[NU], o[NX];
#pragma unroll
  for (int k = 0; k < NX; ++k) xs[k] = x[(size_t)i * NX + k];
#pragma unroll
  for (int k = 0; k < NU; ++k) us[k] = u[(size_t)i * NU + k];
  chain_rk4<NJ, NU>(P, xs, us, o);
#pragma unroll
  for (int k = 0; k < NX; ++k) xo[(size_t)i * NX + k] = o[k];
}

// The central-difference pair f(z + h e_k), f(z − h e_k) of the fp32 closed form in one
// packed RK4 (F2 = (+, −)): stage 1 takes both angles' sin/cos in full, stages 2-4 shift
// them by ½k₁, ½k₂, k₃ (sincos2_shift, |h| ≤ 1/8) instead of reducing the stage's angle
// again. `bad` flags a larger shift; the caller then evaluates the pair on chain_rk4.
template <int NU>
__device__ __forceinline__ void chain_trig_rk4_pm(const ChainTrig<float>& P, const F2 (&x)[4], const F2 (&u)[NU],
                                                  F2 (&out)[4], bool& bad) {
  const float dt = P.dt;
  F2 s10, c10, s20, c20, s1, c1, s2, c2, a0, a1;
  scs(x[0], s10, c10);
  scs(x[1], s20, c20);
  chain_qdd_trig<NU>(P, s10, c10, s20, c20, x[2], x[3], u, a0, a1);
  const F2 k10 = dt * x[2], k11 = dt * x[3], k12 = dt * a0, k13 = dt * a1;
  F2 y2 = x[2] + 0.5f * k12, y3 = x[3] + 0.5f * k13;
  sincos2_shift(s10, c10, 0.5f * k10, s1, c1);
  sincos2_shift(s20, c20, 0.5f * k11, s2, c2);
  chain_qdd_trig<NU>(P, s1, c1, s2, c2, y2, y3, u, a0, a1);
  const F2 k20 = dt * y2, k21 = dt * y3, k22 = dt * a0, k23 = dt * a1;
  y2 = x[2] + 0.5f * k22;
  y3 = x[3] + 0.5f * k23;
  sincos2_shift(s10, c10, 0.5f * k20, s1, c1);
  sincos2_shift(s20, c20, 0.5f * k21, s2, c2);
  chain_qdd_trig<NU>(P, s1, c1, s2, c2, y2, y3, u, a0, a1);
  const F2 k30 = dt * y2, k31 = dt * y3, k32 = dt * a0, k33 = dt * a1;
  y2 = x[2] + k32;
  y3 = x[3] + k33;
  sincos2_shift(s10, c10, k30, s1, c1);
  sincos2_shift(s20, c20, k31, s2, c2);
  chain_qdd_trig<NU>(P, s1, c1, s2, c2, y2, y3, u, a0, a1);
  const F2 k40 = dt * y2, k41 = dt * y3, k42 = dt * a0, k43 = dt * a1;
  const float sixth = 1.0f / 6.0f;
  out[0] = x[0] + sixth * (((k10 + 2.0f * k20) + 2.0f * k30) + k40);
  out[1] = x[1] + sixth * (((k11 + 2.0f * k21) + 2.0f * k31) + k41);
  out[2] = x[2] + sixth * (((k12 + 2.0f * k22) + 2.0f * k32) + k42);
  out[3] = x[3] + sixth * (((k13 + 2.0f * k23) + 2.0f * k33) + k43);
  const F2 m1 = __builtin_elementwise_max(
      __builtin_elementwise_max(__builtin_elementwise_abs(k10), __builtin_elementwise_abs(k11)),
      __builtin_elementwise_max(__builtin_elementwise_abs(k20), __builtin_elementwise_abs(k21)));
  const F2 m2 = __builtin_elementwise_max(
      m1, 2.0f * __builtin_elementwise_max(__builtin_elementwise_abs(k30), __builtin_elementwise_abs(k31)));
  bad |= fmaxf(m2.x, m2.y) > 0.25f;
}

// ---------------------------------------------------------------------------
// Linearisation record per (b, t): [A | B] (NX × (NX+NU), row-major), x_t, u_t
// ---------------------------------------------------------------------------
template <int NJ, int NU>
struct Rec {
  static constexpr int NX = 2 * NJ;
  static constexpr int NJAC = NX * (NX + NU);
  static constexpr int N = NJAC + NX + NU;
};

// One lane per (b, t, direction k): lane g = (b·T + t)·ND + k, so a record's ND
// columns come from ND adjacent lanes and a block writes a contiguous run of records.
// (v7 ran one lane per (b, t) over all ND directions: 3,200 waves at B=2048, T=100 on a
// 3-wave/SIMD occupancy — a second, nearly empty round on 32 CUs.)
// occupancy asked of the linearisation: central differences, the ±h pair packed
// (one packed evaluation), at 3 waves/SIMD (168 VGPRs; config 5 2,208 it/s against 2,175
// at 2 waves, 1,962 at 4 where it spills, and 2,163 unpacked at 4 waves); the dual
// kernel at 2 (256 VGPRs, ~150 spilled, still faster than 1 wave with 300 registers:
// config 5 dual 1,710 → 1,908 it/s)
constexpr int CHAIN_FD_WAVES = 3, CHAIN_DUAL_WAVES = 2;
template <class V, int NJ, int NU, int LIN, class PK = ChainK<V, NJ>>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(LIN == ILQR_LINEARIZE_CENTRAL_FD ? CHAIN_FD_WAVES : CHAIN_DUAL_WAVES))) void chain_linearize_kernel(PK P, int B, int T,
                                                              const V* __restrict__ x,
                                                              const V* __restrict__ u,
                                                              const int32_t* __restrict__ status,
                                                              V* __restrict__ J) {
  constexpr int NX = 2 * NJ, ND = NX + NU, NR = Rec<NJ, NU>::N;
  const size_t g = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (g >= (size_t)B * T * ND) return;
  const int bt = (int)(g / ND);
  const int kd = (int)(g - (size_t)bt * ND);
  const int b = bt / T, t = bt - b * T;
  if (status && status[b] != ILQR_TRAJ_OK) return;
  const V* xb = x + ((size_t)b * (T + 1) + t) * NX;
  const V* ub = u + ((size_t)b * T + t) * NU;
  V* Jt = J + ((size_t)b * T + t) * NR;
  V z[ND];
#pragma unroll
  for (int k = 0; k < NX; ++k) z[k] = xb[k];
#pragma unroll
  for (int k = 0; k < NU; ++k) z[NX + k] = ub[k];
  if constexpr (LIN == ILQR_LINEARIZE_DUAL) {
    // the reference's two ForwardDiff.jacobian calls, one direction per lane (this
    // lane's column k of [A | B]; a pass carrying all ND directions would spill:
    // ≈4.6 KB of scratch per lane)
    constexpr int DC = 1;
    using D = DualT<DC, V>;
    {
      const int k0 = kd;
      D xs[NX], us[NU], o[NX];
#pragma unroll
      for (int k = 0; k < ND; ++k) {
        D v(z[k]);
#pragma unroll
        for (int c = 0; c < DC; ++c) v.d[c] = (k == k0 + c) ? V(1) : V(0);
        if (k < NX) xs[k] = v; else us[k - NX] = v;
      }
      chain_rk4<NJ, NU>(P, xs, us, o);
#pragma unroll
      for (int i = 0; i < NX; ++i)
#pragma unroll
        for (int c = 0; c < DC; ++c)
          if (k0 + c < ND) Jt[i * ND + k0 + c] = o[i].d[c];
    }
  } else {
    // central differences, step h = ε^(1/3)·max(1, |z_k|), divided by the step actually taken
    const V cbe = sizeof(V) == 4 ? V(4.921566e-3) : V(6.0554544523933395e-6);
    {
      const int k = kd;
      V zk = z[0];
#pragma unroll
      for (int j = 1; j < ND; ++j)
        if (j == k) zk = z[j];
      const V h = cbe * fmax(V(1), fabs(zk));
      V xp[NX], up[NU], xm[NX], um[NU], fp[NX], fm[NX];
#pragma unroll
      for (int j = 0; j < NX; ++j) xp[j] = xm[j] = z[j];
#pragma unroll
      for (int j = 0; j < NU; ++j) up[j] = um[j] = z[NX + j];
      V zp = zk + h, zm = zk - h;
#pragma unroll
      for (int j = 0; j < NX; ++j)
        if (j == k) { xp[j] = zp; xm[j] = zm; }
#pragma unroll
      for (int j = 0; j < NU; ++j)
        if (NX + j == k) { up[j] = zp; um[j] = zm; }
      if constexpr (sizeof(V) == 4) {
        // f(z + h e_k) and f(z − h e_k) run the same instruction stream: one packed
        // evaluation (v_pk_* on the pair)
        F2 x2[NX], u2[NU], f2[NX];
#pragma unroll
        for (int j = 0; j < NX; ++j) x2[j] = F2{(float)xp[j], (float)xm[j]};
#pragma unroll
        for (int j = 0; j < NU; ++j) u2[j] = F2{(float)up[j], (float)um[j]};
        if constexpr (std::is_same_v<PK, ChainTrig<float>>) {
          bool bad = false;
          chain_trig_rk4_pm<NU>(P, x2, u2, f2, bad);
          if (bad) chain_rk4<NJ, NU>(P, x2, u2, f2);
        } else {
          chain_rk4<NJ, NU>(P, x2, u2, f2);
        }
#pragma unroll
        for (int j = 0; j < NX; ++j) { fp[j] = f2[j].x; fm[j] = f2[j].y; }
      } else {
        chain_rk4<NJ, NU>(P, xp, up, fp);
        chain_rk4<NJ, NU>(P, xm, um, fm);
      }
      const V inv = V(1) / (zp - zm);
#pragma unroll
      for (int i = 0; i < NX; ++i) Jt[i * ND + k] = (fp[i] - fm[i]) * inv;
    }
  }
  V zd = z[0];
#pragma unroll
  for (int j = 1; j < ND; ++j)
    if (j == kd) zd = z[j];
  Jt[Rec<NJ, NU>::NJAC + kd] = zd;
}

// record → separate A (B,T,NX,NX), B (B,T,NX,NU) tiles (ilqr_chain_linearize)
template <class V, int NJ, int NU>
__global__ __launch_bounds__(256) void chain_unpack_kernel(int B, int T, const V* __restrict__ J,
                                                           V* __restrict__ A, V* __restrict__ Bm) {
  constexpr int NX = 2 * NJ, ND = NX + NU, NR = Rec<NJ, NU>::N;
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (size_t)B * T) return;
  const V* Jt = J + i * NR;
#pragma unroll
  for (int r = 0; r < NX; ++r) {
#pragma unroll
    for (int k = 0; k < NX; ++k) A[i * NX * NX + r * NX + k] = Jt[r * ND + k];
#pragma unroll
    for (int k = 0; k < NU; ++k) Bm[i * NX * NU + r * NU + k] = Jt[r * ND + NX + k];
  }
}

// ---------------------------------------------------------------------------
// Riccati recursion (src/backward_pass.jl:324-357), one lane per trajectory
// ---------------------------------------------------------------------------
template <class V, int NJ, int NU>
__device__ bool chain_backward_lane(const ChainK<V, NJ>& P, int b, int T, const V* __restrict__ x,
                                    const V* __restrict__ J, V* __restrict__ dg,
                                    V* __restrict__ Kg, V mu) {
  constexpr int NX = 2 * NJ, ND = NX + NU, NR = Rec<NJ, NU>::N, NJAC = Rec<NJ, NU>::NJAC;
  const V* xN = x + ((size_t)b * (T + 1) + T) * NX;
  // final_cost_quadratization (:134-153): ∇ℓ_f = −2 qfw (θ* − θ), ∇²ℓ_f = diag(2 qfw, 0)
  V S[NX][NX], s[NX];
#pragma unroll
  for (int i = 0; i < NX; ++i) {
#pragma unroll
    for (int j = 0; j < NX; ++j) S[i][j] = V(0);
    s[i] = V(0);
  }
#pragma unroll
  for (int i = 0; i < NJ; ++i) {
    S[i][i] = V(2) * P.qfw[i];
    s[i] = V(-2) * P.qfw[i] * (P.tgt[i] - xN[i]);
  }
  bool bad = false;
  const V* Jb = J + (size_t)b * T * NR;
  V rec[2][NR];
  auto load = [&](int t, V (&r)[NR]) {
    const V* Jt = Jb + (size_t)(t > 0 ? t : 0) * NR;
#pragma unroll
    for (int k = 0; k < NR; ++k) r[k] = Jt[k];
  };
  auto step = [&](int t, const V (&F)[NR]) {
    // Y = S F, sF = sᵀF  (optimal_controller_param :181-183)
    V Y[NX][ND], sF[ND];
#pragma unroll
    for (int i = 0; i < NX; ++i)
#pragma unroll
      for (int k = 0; k < ND; ++k) {
        V acc = V(0);
#pragma unroll
        for (int j = 0; j < NX; ++j) acc = fma(S[i][j], F[j * ND + k], acc);
        Y[i][k] = acc;
      }
#pragma unroll
    for (int k = 0; k < ND; ++k) {
      V acc = V(0);
#pragma unroll
      for (int j = 0; j < NX; ++j) acc = fma(s[j], F[j * ND + k], acc);
      sF[k] = acc;
    }
    auto Z = [&](int a, int c) {
      V acc = V(0);
#pragma unroll
      for (int j = 0; j < NX; ++j) acc = fma(F[j * ND + a], Y[j][c], acc);
      return acc;
    };
    // immediate_cost_quadratization (:81-109): lx = −2qw(θ*−θ), lu = 2 rw u,
    // lxx = diag(2qw, 0), luu = diag(2rw), lux = 0
    V G[NU][NX], H[NU][NU], g[NU];
#pragma unroll
    for (int a = 0; a < NU; ++a) {
#pragma unroll
      for (int c = 0; c < NX; ++c) G[a][c] = Z(NX + a, c);
#pragma unroll
      for (int c = 0; c < NU; ++c) H[a][c] = Z(NX + a, NX + c) + (a == c ? V(2) * P.rw[a] : V(0));
      g[a] = V(2) * P.rw[a] * F[NJAC + NX + a] + sF[NX + a];
    }
    // feedback_parameters (:207-218): H + μI = L D Lᵀ (unit lower L); δu = −H⁻¹g, K = −H⁻¹G
    V L[NU][NU], D[NU], iD[NU];
#pragma unroll
    for (int i = 0; i < NU; ++i) {
#pragma unroll
      for (int j = 0; j < i; ++j) {
        V acc = H[i][j];
#pragma unroll
        for (int k = 0; k < j; ++k) acc = acc - L[i][k] * L[j][k] * D[k];
        L[i][j] = acc * iD[j];
      }
      V acc = H[i][i] + mu;
#pragma unroll
      for (int k = 0; k < i; ++k) acc = acc - L[i][k] * L[i][k] * D[k];
      D[i] = acc;
      iD[i] = V(1) / acc;
    }
    auto solve = [&](const V (&r)[NU], V (&z)[NU]) {  // z = −(H + μI)⁻¹ r
      V y[NU], w[NU];
#pragma unroll
      for (int i = 0; i < NU; ++i) {
        V acc = r[i];
#pragma unroll
        for (int k = 0; k < i; ++k) acc = acc - L[i][k] * y[k];
        y[i] = acc;
      }
#pragma unroll
      for (int i = NU - 1; i >= 0; --i) {
        V acc = y[i] * iD[i];
#pragma unroll
        for (int k = i + 1; k < NU; ++k) acc = acc - L[k][i] * w[k];
        w[i] = acc;
      }
#pragma unroll
      for (int i = 0; i < NU; ++i) z[i] = -w[i];
    };
    V K[NU][NX], d[NU];
#pragma unroll
    for (int c = 0; c < NX; ++c) {
      V r[NU], z[NU];
#pragma unroll
      for (int a = 0; a < NU; ++a) r[a] = G[a][c];
      solve(r, z);
#pragma unroll
      for (int a = 0; a < NU; ++a) K[a][c] = z[a];
    }
    solve(g, d);
    V* Kt = Kg + ((size_t)b * T + t) * NU * NX;
    V* dt = dg + ((size_t)b * T + t) * NU;
#pragma unroll
    for (int a = 0; a < NU; ++a) {
      dt[a] = d[a];
      bad |= d[a] != d[a];
#pragma unroll
      for (int c = 0; c < NX; ++c) {
        Kt[a * NX + c] = K[a][c];
        bad |= K[a][c] != K[a][c];
      }
    }
    // step_back (:262-273), exact rewrite with W = (H+2μI)[K|d] = −[G|g] + μ[K|d]
    V WK[NU][NX], Wd[NU];
#pragma unroll
    for (int a = 0; a < NU; ++a) {
#pragma unroll
      for (int c = 0; c < NX; ++c) WK[a][c] = fma(mu, K[a][c], -G[a][c]);
      Wd[a] = fma(mu, d[a], -g[a]);
    }
    V Sn[NX][NX], sn[NX];
#pragma unroll
    for (int i = 0; i < NX; ++i) {
#pragma unroll
      for (int j = i; j < NX; ++j) {
        V acc = Z(i, j);
        if (i == j && i < NJ) acc += V(2) * P.qw[i];
#pragma unroll
        for (int a = 0; a < NU; ++a) acc = fma(-K[a][i], WK[a][j], acc);
        Sn[i][j] = acc;
        Sn[j][i] = acc;
      }
      V acc = sF[i];
      if (i < NJ) acc += V(-2) * P.qw[i] * (P.tgt[i] - F[NJAC + i]);
#pragma unroll
      for (int a = 0; a < NU; ++a) acc = fma(-K[a][i], Wd[a], acc);
      sn[i] = acc;
    }
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      s[i] = sn[i];
#pragma unroll
      for (int j = 0; j < NX; ++j) S[i][j] = Sn[i][j];
    }
  };
  load(T - 1, rec[0]);
  int t = T - 1;
  for (; t >= 1; t -= 2) {  // one step of prefetch
    load(t - 1, rec[1]);
    step(t, rec[0]);
    load(t - 2, rec[0]);
    step(t - 1, rec[1]);
  }
  if (t == 0) step(0, rec[0]);
  return bad;
}

// ---------------------------------------------------------------------------
// Forward rollout + line search (src/forward_pass.jl:55-93), one lane per trajectory
// ---------------------------------------------------------------------------
template <class V>
struct ChainFwdOut {
  V cost;
  int trials;
  int accepted;
};

template <class V, int NJ, int NU, bool SPLIT = false, class PK = ChainK<V, NJ>>
__device__ ChainFwdOut<V> chain_forward_lane(const PK& P, int b, int T,
                                             const V* __restrict__ x, const V* __restrict__ u,
                                             const V* __restrict__ xtraj, const V* __restrict__ dg,
                                             const V* __restrict__ Kg, V prev_cost,
                                             V* __restrict__ xnew, V* __restrict__ unew, V* du2_out,
                                             const LSParams& ls) {
  constexpr int NX = 2 * NJ;
  const bool writer = !SPLIT || (threadIdx.x & 15) == 0;  // SPLIT: one lane of the group stores
  const V* xb0 = x + (size_t)b * (T + 1) * NX;
  const V* ub0 = u + (size_t)b * T * NU;
  const V* xt0 = (xtraj ? xtraj : x) + (size_t)b * (T + 1) * NX;
  const V xtw = xtraj ? V(1) : V(0);  // x_traj = NULL means zeros (forward_pass.jl:151)
  const V* d0 = dg + (size_t)b * T * NU;
  const V* K0 = Kg + (size_t)b * T * NU * NX;
  V* xo = xnew + (size_t)b * (T + 1) * NX;
  V* uo = unew + (size_t)b * T * NU;

  V alpha = V(ls.alpha0);
  ChainFwdOut<V> out{V(0), 0, 0};
  V du2 = V(0);
  for (int trial = 1; trial <= ls.max_trials; ++trial) {
    V xb[NX];
#pragma unroll
    for (int i = 0; i < NX; ++i) xb[i] = xb0[i];  // x̄₁ = x₁ (:65)
    V cost = V(0);
    du2 = V(0);
    // step t's inputs (x_t, x_traj_t, K_t, u_t, δu_t) are loaded during step t − 1: a
    // step is a few µs of dependent dynamics, so the loads land off the critical path
    struct In { V xk[NX], xtk[NJ], K[NU * NX], u[NU], d[NU]; };
    auto load = [&](int t, In& in) {
#pragma unroll
      for (int i = 0; i < NX; ++i) in.xk[i] = xb0[(size_t)t * NX + i];
#pragma unroll
      for (int i = 0; i < NJ; ++i) in.xtk[i] = xt0[(size_t)t * NX + i];
#pragma unroll
      for (int k = 0; k < NU * NX; ++k) in.K[k] = K0[(size_t)t * NU * NX + k];
#pragma unroll
      for (int a = 0; a < NU; ++a) {
        in.u[a] = ub0[(size_t)t * NU + a];
        in.d[a] = d0[(size_t)t * NU + a];
      }
    };
    In cur;
    load(0, cur);
    for (int t = 0; t < T; ++t) {
      In nxt;
      load(t + 1 < T ? t + 1 : t, nxt);
      V dx[NX];
#pragma unroll
      for (int i = 0; i < NX; ++i) dx[i] = xb[i] - cur.xk[i];  // δx (:72)
      V ubar[NU];
#pragma unroll
      for (int a = 0; a < NU; ++a) {  // ūₖ = uₖ + α δuₖ + Kₖ δx (:73)
        V kdx = V(0);
#pragma unroll
        for (int i = 0; i < NX; ++i) kdx = fma(cur.K[a * NX + i], dx[i], kdx);
        const V uk = cur.u[a];
        ubar[a] = fma(alpha, cur.d[a], uk) + kdx;
        const V e = ubar[a] - uk;
        du2 = fma(e, e, du2);
      }
      // ℓ(x̄ₖ − x_trajₖ, ūₖ) (:187-190; RBD_helper_functions.jl:85-99 on the joints)
      V lk = V(0);
#pragma unroll
      for (int i = 0; i < NJ; ++i) {
        const V e = P.tgt[i] - fma(-xtw, cur.xtk[i], xb[i]);
        lk = fma(P.qw[i] * e, e, lk);
      }
#pragma unroll
      for (int a = 0; a < NU; ++a) lk = fma(P.rw[a] * ubar[a], ubar[a], lk);
      cost += lk;
#pragma unroll
      for (int i = 0; i < NX; ++i)
        if (writer) xo[(size_t)t * NX + i] = xb[i];
#pragma unroll
      for (int a = 0; a < NU; ++a)
        if (writer) uo[(size_t)t * NU + a] = ubar[a];
      V xn[NX];
      chain_rk4<NJ, NU, SPLIT>(P, xb, ubar, xn);  // x̄ₖ₊₁ = f(x̄ₖ, ūₖ) (:74)
#pragma unroll
      for (int i = 0; i < NX; ++i) xb[i] = xn[i];
      cur = nxt;
    }
#pragma unroll
    for (int i = 0; i < NX; ++i)
      if (writer) xo[(size_t)T * NX + i] = xb[i];
    // final_cost(x̄_N) on the raw state (:192; RBD_helper_functions.jl:105-116)
    V lf = V(0);
#pragma unroll
    for (int i = 0; i < NJ; ++i) {
      const V e = P.tgt[i] - xb[i];
      lf = fma(P.qfw[i] * e, e, lf);
    }
    cost += lf;
    out.trials = trial;
    out.cost = cost;
    if (prev_cost - cost > V(0)) {  // (:77-80); NaN compares false → keep searching
      out.accepted = 1;
      break;
    }
    alpha *= V(ls.shrink);  // (:82)
  }
  if (du2_out) *du2_out = du2;
  return out;
}

template <class V>
struct ChainIter {
  const V* x;
  const V* u;
  const V* xtraj;
  V* xnew;
  V* unew;
  V* K;
  V* d;
  const V* prev_cost;
  V* new_cost;
  V* du2;
  int32_t* trials;
  int32_t* status;
  int32_t* res_parity;
  int32_t* iters;
  int parity;
  int iter;
};

// ---------------------------------------------------------------------------
// Riccati recursion of the 2-joint chain (nx = 4, nu ≤ 2) on the 4-block f64 MFMA,
// four trajectories per wave: the 2-link family's tl_backward4_wave (ilqr_twolink.hip,
// DESIGN.md §4) with the chain's weighted joint-space cost (RBD_helper_functions.jl:
// 85-116: lxx = diag(2qw, 0), luu = diag(2rw), lx = −2qw(θ* − θ), lu = 2rw·u, final
// diag(2qfw, 0) and −2qfw(θ* − θ_N)). The recursion runs in f64 whatever V is (the
// fp32 family's records and gains are converted at the load/store): one rounding of
// the gains to fp32 instead of fp32 arithmetic throughout.
template <class V>
__device__ __forceinline__ double ch_ld(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  if constexpr (sizeof(V) == 4)
    return (double)__builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
  else
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0));
}
template <class V>
__device__ __forceinline__ void ch_st(double v, __amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  if constexpr (sizeof(V) == 4)
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, (float)v), r, voff, soff, 0);
  else
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, v), r, voff, soff, 0);
}
__device__ __forceinline__ double ch_mf(double a, double b, double c) {  // c + aᵀb
  return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ double ch_mfn(double a, double b, double c) {  // c − aᵀb
  return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 1);
}
constexpr int CH_BW4_PF = 4;  // record prefetch depth (steps)

template <class V, int NU>
__device__ unsigned chain_backward4_wave(const ChainK<V, 2>& P, int b0, int B, unsigned active, int T,
                                         const V* __restrict__ x, const V* __restrict__ J,
                                         V* __restrict__ dg, V* __restrict__ Kg, double mu,
                                         double* lds, const ChainTask* task) {
  constexpr int NJ = 2, NX = 4, ND = NX + NU, NR = Rec<NJ, NU>::N, NJAC = Rec<NJ, NU>::NJAC;
  constexpr uint32_t DEAD = 0x80000000u, W = sizeof(V);
  b0 = __builtin_amdgcn_readfirstlane(b0);
  const int l = threadIdx.x & 63;
  const int rho = l >> 4, beta = (l >> 2) & 3, kap = l & 3;
  const int b = b0 + beta;
  const bool live = b < B && ((active >> beta) & 1u);
  const int bc = b < B ? b : B - 1;
  const int nslot = B - b0 < 4 ? B - b0 : 4;
  const bool rj = rho < NJ, ru = rho < NU;
  const int jr = rj ? rho : 0;
  const double tg = (double)P.tgt[jr], qw2 = 2.0 * (double)P.qw[jr], qfw2 = 2.0 * (double)P.qfw[jr];
  const double rw2 = ru ? 2.0 * (double)P.rw[rho < NU ? rho : 0] : 0.0;
  const double lxx = (rho == kap && rj) ? qw2 : 0.0;
  const double luu = (rho == kap && ru) ? rw2 : 0.0;
  double S = (rho == kap && rj) ? qfw2 : 0.0;
  const double xT = (double)x[((size_t)bc * (T + 1) + T) * NX + jr];
  double s = rj ? -qfw2 * (tg - xT) : 0.0;
  if (task) {  // the task-space final cost (cost_functions.jl:16-24): ∇ℓ_f, ∇²ℓ_f on the q rows
    const size_t o = ((size_t)bc * (T + 1) + T) * NX;
    double g[2], H[3];
    chain_task_quad(task, (double)x[o], (double)x[o + 1], g, H);
    const double h0 = jr == 0 ? H[0] : H[1], h1 = jr == 0 ? H[1] : H[2];
    S = (rj && kap < NJ) ? (kap == 0 ? h0 : h1) : 0.0;
    s = rj ? (jr == 0 ? g[0] : g[1]) : 0.0;
  }

  const auto rJ = buffer_rsrc(const_cast<V*>(J) + (size_t)b0 * T * NR, (uint32_t)(nslot * T * NR * W));
  const uint32_t base = (uint32_t)(beta * T * NR * W);
  const uint32_t oA = base + (uint32_t)((rho * ND + kap) * W);
  const uint32_t oB = kap < NU ? base + (uint32_t)((rho * ND + NX + kap) * W) : DEAD;
  const uint32_t oT = rj ? base + (uint32_t)((NJAC + rho) * W) : DEAD;
  const uint32_t oU = ru ? base + (uint32_t)((NJAC + NX + rho) * W) : DEAD;
  const auto rK = buffer_rsrc(Kg + (size_t)b0 * T * NU * NX, (uint32_t)(nslot * T * NU * NX * W));
  const auto rD = buffer_rsrc(dg + (size_t)b0 * T * NU, (uint32_t)(nslot * T * NU * W));
  const uint32_t kv = (live && ru) ? (uint32_t)((beta * T * NU * NX + rho * NX + kap) * W) : DEAD;
  const uint32_t dv = (live && ru && kap == 0) ? (uint32_t)((beta * T * NU + rho) * W) : DEAD;
  const double Id = rho == kap ? 1.0 : 0.0;  // the identity block
  double* Hl = lds + beta * 16;

  constexpr int PF = CH_BW4_PF;
  // the ring holds the records' raw words: an fp32 record converted at the load would
  // make the step that issued it wait for it (the conversion consumes the load), which
  // defeats the prefetch — the conversion happens at the use, PF steps later
  using Raw = std::conditional_t<sizeof(V) == 4, uint32_t, double>;
  Raw rA[PF], rB[PF], rT[PF], rU[PF];
  auto ld = [&](uint32_t off, int t) -> Raw {
    if constexpr (sizeof(V) == 4)
      return __builtin_amdgcn_raw_buffer_load_b32(rJ, off, (uint32_t)(t * NR * W), 0);
    else
      return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rJ, off, (uint32_t)(t * NR * W), 0));
  };
  auto cv = [](Raw r) -> double {
    asm volatile("" : "+v"(r));  // the conversion stays at the use
    if constexpr (sizeof(V) == 4) return (double)__builtin_bit_cast(float, r);
    else return r;
  };
#pragma unroll
  for (int k = 0; k < PF; ++k) {
    const int tk = T - 1 - k > 0 ? T - 1 - k : 0;
    rA[k] = ld(oA, tk); rB[k] = ld(oB, tk); rT[k] = ld(oT, tk); rU[k] = ld(oU, tk);
  }
  __builtin_amdgcn_s_waitcnt(0);
  double Kl = 0.0, dl = 0.0;
  auto step = [&](int t, int k) {
    const double A = cv(rA[k]), Bm = cv(rB[k]), th = cv(rT[k]), uu = cv(rU[k]);
    const int tn = t - PF > 0 ? t - PF : 0;
    rA[k] = ld(oA, tn); rB[k] = ld(oB, tn); rT[k] = ld(oT, tn); rU[k] = ld(oU, tn);
    const double lx = rj ? -qw2 * (tg - th) : 0.0;
    const double lu = rw2 * uu;
    const double Y0 = ch_mf(S, A, 0.0);
    const double Z = ch_mf(A, Y0, lxx);                           // lxx + AᵀSA
    const double G = ch_mf(Bm, Y0, 0.0);                          // BᵀSA
    const double gx = ch_mf(A, s, lx), gu = ch_mf(Bm, s, lu);     // lx + Aᵀs, lu + Bᵀs
    double K, d;
    if constexpr (NU == 2) {
      const double Y1 = ch_mf(S, Bm, 0.0);
      const double H = ch_mf(Bm, Y1, luu);                        // luu + BᵀSB
      Hl[rho * 4 + kap] = H;
      wave_lds_fence();
      const double h00 = Hl[0], h10 = Hl[4], h11 = Hl[5];
      wave_lds_fence();
      // (H + μI)⁻¹ of the 2×2 u block by its adjugate (H = luu + O(Δt²)BᵀSB)
      const double a00 = h00 + mu, a11 = h11 + mu;
      const double idet = rcp<2>(fma(a00, a11, -h10 * h10));
      const bool in2 = rho < 2 && kap < 2;
      const double Hi = !in2 ? 0.0 : (rho != kap ? -h10 : (rho == 0 ? a11 : a00)) * idet;
      K = ch_mfn(Hi, G, 0.0);
      d = ch_mfn(Hi, gu, 0.0);
    } else {
      // 1×1 H in every lane of the slot from B's column replicated over κ (a quad
      // broadcast): no LDS hand-off, and the gains are VALU products (ilqr_twolink.hip)
      const double Br = dpp_quad_bcast0(Bm);
      const double Y1 = ch_mf(S, Br, 0.0);                        // S·b, replicated
      const double H = ch_mf(Br, Y1, 2.0 * (double)P.rw[0]);      // luu + bᵀSb everywhere
      const double hi = rcp<2>(H + mu);
      K = -(hi * G);
      d = -(hi * gu);
      (void)Hl; (void)luu;
    }
    // wave-uniform soffset (a per-lane one makes each store a readfirstlane waterfall
    // loop); a DEAD voffset stays out of range whatever the step
    ch_st<V>(K, rK, kv, (uint32_t)(t * NU * NX * W));
    ch_st<V>(d, rD, dv, (uint32_t)(t * NU * W));
    const double Wk = fma(mu, K, -G), Wd = fma(mu, d, -gu);
    const double Sf = ch_mfn(K, Wk, Z);
    // Sfᵀ on the MFMA (ch_mf(Sf, I, 0), exact): its ≈50-cycle result instead of a
    // ds_bpermute round trip on the recursion's chain
    const double Sm = ch_mf(Sf, Id, 0.0);
    S = rho <= kap ? Sf : Sm;                                      // upper triangle, mirrored
    s = ch_mfn(K, Wd, gx);
    Kl = K; dl = d;
  };
  int t = T - 1;
  for (; t >= PF - 1; t -= PF) {
#pragma unroll
    for (int k = 0; k < PF; ++k) step(t - k, k);
  }
#pragma unroll
  for (int k = 0; k < PF - 1; ++k)
    if (t - k >= 0) step(t - k, k);
  const unsigned long long nb = __ballot(__builtin_isnan(Kl) || __builtin_isnan(dl));
  unsigned r = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) r |= (nb & ((0xFull << (4 * q)) * 0x0001000100010001ull)) ? (1u << q) : 0u;
  return r;
}

constexpr int CH_WG = 64;

template <class V, int NJ, int NU>
__global__ __launch_bounds__(CH_WG) void chain_backward_kernel(ChainK<V, NJ> P, int B, int T,
                                                               const V* __restrict__ x,
                                                               const V* __restrict__ J,
                                                               V* __restrict__ d, V* __restrict__ K,
                                                               int32_t* __restrict__ status, V mu) {
  const int b = blockIdx.x * CH_WG + threadIdx.x;
  if (b >= B) return;
  const bool nan = chain_backward_lane<V, NJ, NU>(P, b, T, x, J, d, K, mu);
  if (status) status[b] = nan ? ILQR_TRAJ_NAN : ILQR_TRAJ_OK;
}

// lanes per trajectory of the forward kernels: a 16-lane group (one DPP row) running
// the component-parallel Newton-Euler (chain_xdot_cv)
constexpr int CH_FW_LANES = 16;

// four trajectories per wave, four waves per workgroup (2-joint chains)
template <class V, int NU>
__global__ __launch_bounds__(256) void chain_backward4_kernel(ChainK<V, 2> P, int B, int T,
                                                              const V* __restrict__ x,
                                                              const V* __restrict__ J,
                                                              V* __restrict__ d, V* __restrict__ K,
                                                              int32_t* __restrict__ status, V mu,
                                                              const ChainTask* task) {
  __shared__ double lds[4 * 64];
  const int w = threadIdx.x >> 6;
  const int b0 = (blockIdx.x * 4 + w) * 4;
  if (b0 >= B) return;
  const unsigned nan = chain_backward4_wave<V, NU>(P, b0, B, 0xFu, T, x, J, d, K, (double)mu, lds + w * 64, task);
  const int l = threadIdx.x & 63;
  if (status && l < 4 && b0 + l < B) status[b0 + l] = ((nan >> l) & 1u) ? ILQR_TRAJ_NAN : ILQR_TRAJ_OK;
}

template <class V, int NJ, int NU>
__global__ __launch_bounds__(CH_WG) void chain_forward_kernel(
    ChainK<V, NJ> P, int B, int T, const V* __restrict__ x, const V* __restrict__ u,
    const V* __restrict__ xtraj, const V* __restrict__ d, const V* __restrict__ K,
    const V* __restrict__ prev_cost, V* __restrict__ xnew, V* __restrict__ unew,
    V* __restrict__ new_cost, int32_t* __restrict__ trials, int32_t* __restrict__ status,
    LSParams ls) {
  constexpr int NX = 2 * NJ;
  __shared__ ChainK<V, NJ> Ps;  // constants in LDS (see chain_iter_forward_kernel)
  for (int i = threadIdx.x; i < (int)(sizeof(ChainK<V, NJ>) / 4); i += CH_WG)
    reinterpret_cast<uint32_t*>(&Ps)[i] = reinterpret_cast<const uint32_t*>(&P)[i];
  __syncthreads();
  const int b = (blockIdx.x * CH_WG + threadIdx.x) / CH_FW_LANES;
  if (b >= B) return;  // the whole lane group
  const V pc = prev_cost ? prev_cost[b] : V(INFINITY);
  const ChainFwdOut<V> r =
      chain_forward_lane<V, NJ, NU, true>(Ps, b, T, x, u, xtraj, d, K, pc, xnew, unew, nullptr, ls);
  if ((threadIdx.x & 15) != 0) return;
  if (!r.accepted) {  // exhausted (the reference would loop forever): return the inputs
    for (int i = 0; i < (T + 1) * NX; ++i) xnew[(size_t)b * (T + 1) * NX + i] = x[(size_t)b * (T + 1) * NX + i];
    for (int i = 0; i < T * NU; ++i) unew[(size_t)b * T * NU + i] = u[(size_t)b * T * NU + i];
  }
  new_cost[b] = r.cost;
  if (trials) trials[b] = r.trials;
  if (status) status[b] = r.accepted ? ILQR_TRAJ_OK
                                     : (r.cost != r.cost ? ILQR_TRAJ_NAN : ILQR_TRAJ_LS_EXHAUSTED);
}

template <class V, int NJ, int NU>
__global__ __launch_bounds__(CH_WG) void chain_iter_backward_kernel(ChainK<V, NJ> P, int B, int T,
                                                                    ChainIter<V> a, const V* J, V mu) {
  const int b = blockIdx.x * CH_WG + threadIdx.x;
  if (b >= B || a.status[b] != ILQR_TRAJ_OK) return;
  if (chain_backward_lane<V, NJ, NU>(P, b, T, a.x, J, a.d, a.K, mu)) {
    a.status[b] = ILQR_TRAJ_NAN;  // reference: AssertionError at backward_pass.jl:353
    if (a.res_parity) a.res_parity[b] = a.parity;
  }
}

// fit iteration, backward part, 2-joint chains: slots whose status is not OK are
// computed on and never stored
template <class V, int NU>
__global__ __launch_bounds__(256) void chain_iter_backward4_kernel(ChainK<V, 2> P, int B, int T,
                                                                   ChainIter<V> a, const V* J, V mu,
                                                                   const ChainTask* task) {
  __shared__ double lds[4 * 64];
  const int w = threadIdx.x >> 6;
  const int b0 = (blockIdx.x * 4 + w) * 4;
  if (b0 >= B) return;
  unsigned active = 0;
  for (int q = 0; q < 4; ++q)
    if (b0 + q < B && a.status[b0 + q] == ILQR_TRAJ_OK) active |= 1u << q;
  if (active == 0) return;
  const unsigned nan =
      chain_backward4_wave<V, NU>(P, b0, B, active, T, a.x, J, a.d, a.K, (double)mu, lds + w * 64, task) &
      active;
  const int l = threadIdx.x & 63;
  if (l < 4 && ((nan >> l) & 1u)) {
    a.status[b0 + l] = ILQR_TRAJ_NAN;  // reference: AssertionError at backward_pass.jl:353
    if (a.res_parity) a.res_parity[b0 + l] = a.parity;
  }
}

template <class V, int NJ, int NU>
__global__ __launch_bounds__(CH_WG) void chain_iter_forward_kernel(ChainK<V, NJ> P, int B, int T,
                                                                   ChainIter<V> a, LSParams ls) {
  // the chain constants go to LDS: as a kernel argument they overflow the SGPR file
  // (~210 SGPRs spilled to VGPR lanes at every use)
  __shared__ ChainK<V, NJ> Ps;
  static_assert(sizeof(ChainK<V, NJ>) % 4 == 0, "dword copy");
  for (int i = threadIdx.x; i < (int)(sizeof(ChainK<V, NJ>) / 4); i += CH_WG)
    reinterpret_cast<uint32_t*>(&Ps)[i] = reinterpret_cast<const uint32_t*>(&P)[i];
  __syncthreads();
  const int b = (blockIdx.x * CH_WG + threadIdx.x) / CH_FW_LANES;
  if (b >= B || a.status[b] != ILQR_TRAJ_OK) return;  // the whole lane group
  V du2 = V(0);
  const V pc = a.prev_cost ? a.prev_cost[b] : V(INFINITY);
  const ChainFwdOut<V> r = chain_forward_lane<V, NJ, NU, true>(Ps, b, T, a.x, a.u, a.xtraj, a.d,
                                                               a.K, pc, a.xnew, a.unew, &du2, ls);
  if ((threadIdx.x & 15) != 0) return;
  if (a.trials) a.trials[b] = r.trials;
  if (a.du2) a.du2[b] = du2;
  if (a.iters) a.iters[b] = a.iter;
  if (!r.accepted) {
    a.status[b] = (r.cost != r.cost) ? ILQR_TRAJ_NAN : ILQR_TRAJ_LS_EXHAUSTED;
    if (a.res_parity) a.res_parity[b] = a.parity;
  } else {
    a.new_cost[b] = r.cost;                // prev_cost = new_cost (:168)
    if ((double)du2 <= ls.tol) {           // (:171) break BEFORE the update
      a.status[b] = ILQR_TRAJ_CONVERGED;
      if (a.res_parity) a.res_parity[b] = a.parity;
    }
  }
}

// ---------------------------------------------------------------------------
// Closed-form dynamics (ChainTrig): coefficient samples, the check against the
// recursion, and the forward kernels (one lane per trajectory: the closed form has
// nothing for a 16-lane group to split)
// ---------------------------------------------------------------------------
constexpr int CH_TRIG_SAMPLES = 15 + 18;  // M at 5 angles (3 entries), g on 3×3 (2 entries)
__global__ void chain_trig_sample_kernel(ChainK<double, 2> P, double* __restrict__ out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const double two_pi = 6.283185307179586476925286766559;
  const double zero[2] = {0.0, 0.0}, e0[2] = {1.0, 0.0}, e1[2] = {0.0, 1.0};
  for (int k = 0; k < 5; ++k) {  // M(q₂ = 2πk/5); M does not depend on q₁
    double c[2] = {1.0, 0.0}, sn[2] = {0.0, 0.0};
    sincos(two_pi * k / 5.0, &sn[1], &c[1]);
    double m0[2], m1[2];
    rnea<false, false>(P, c, sn, zero, e0, m0);
    rnea<false, false>(P, c, sn, zero, e1, m1);
    out[3 * k] = m0[0];
    out[3 * k + 1] = 0.5 * (m1[0] + m0[1]);  // symmetric up to rounding
    out[3 * k + 2] = m1[1];
  }
  for (int a = 0; a < 3; ++a)
    for (int b = 0; b < 3; ++b) {  // g(q₁ = 2πa/3, q₂ = 2πb/3)
      double c[2], sn[2], g[2];
      sincos(two_pi * a / 3.0, &sn[0], &c[0]);
      sincos(two_pi * b / 3.0, &sn[1], &c[1]);
      rnea<false, true>(P, c, sn, zero, zero, g);
      out[15 + 2 * (3 * a + b)] = g[0];
      out[15 + 2 * (3 * a + b) + 1] = g[1];
    }
}

// |f_trig − f_rnea| / max(1, |f_rnea|) at n pseudo-random states and torques (fp64)
__global__ void chain_trig_check_kernel(ChainK<double, 2> P, ChainTrig<double> Q, int n,
                                        double* __restrict__ err) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t h = 0x9E3779B9u * (uint32_t)(i + 1);
  auto rnd = [&](double lo, double hi) {
    h ^= h << 13; h ^= h >> 17; h ^= h << 5;
    return lo + (hi - lo) * ((h & 0xFFFFFF) / 16777216.0);
  };
  double x[4] = {rnd(-4, 4), rnd(-4, 4), rnd(-6, 6), rnd(-6, 6)}, u[2] = {rnd(-3, 3), rnd(-3, 3)};
  double a[4], b[4];
  chain_xdot<2, 2>(P, x, u, a);
  chain_xdot_trig<2>(Q, x, u, b);
  double e = 0.0, m = 1.0;
  for (int k = 0; k < 4; ++k) {
    e = fmax(e, fabs(a[k] - b[k]));
    m = fmax(m, fabs(a[k]));
  }
  err[i] = e / m;
}

// L line-search candidates per trajectory (ilqr_fwd_group.h), W waves per workgroup
template <class V, int NU, int L, int W>
__global__ __launch_bounds__(64 * W) void chain_forward_trig_kernel(
    ChainTrig<V> P, int B, int T, const V* __restrict__ x, const V* __restrict__ u,
    const V* __restrict__ xtraj, const V* __restrict__ d, const V* __restrict__ K,
    const V* __restrict__ prev_cost, V* __restrict__ xnew, V* __restrict__ unew,
    V* __restrict__ new_cost, int32_t* __restrict__ trials, int32_t* __restrict__ status,
    LSParams ls) {
  constexpr int NX = 4;
  const int b = (blockIdx.x * 64 * W + threadIdx.x) / L;
  if (b >= B) return;
  const V pc = prev_cost ? prev_cost[b] : V(INFINITY);
  const ChainTrigModel<V, NU> m{P};
  const FgOut<V> r = fwd_group<ChainTrigModel<V, NU>, L>(m, b, B, T, x, u, xtraj, d, K, pc, xnew, unew, ls);
  if (!r.owner) return;
  if (!r.accepted) {  // exhausted (the reference would loop forever): return the inputs
    for (int i = 0; i < (T + 1) * NX; ++i) xnew[(size_t)b * (T + 1) * NX + i] = x[(size_t)b * (T + 1) * NX + i];
    for (int i = 0; i < T * NU; ++i) unew[(size_t)b * T * NU + i] = u[(size_t)b * T * NU + i];
  }
  new_cost[b] = r.cost;
  if (trials) trials[b] = r.trials;
  if (status) status[b] = r.accepted ? ILQR_TRAJ_OK
                                     : (r.cost != r.cost ? ILQR_TRAJ_NAN : ILQR_TRAJ_LS_EXHAUSTED);
}

template <class V, int NU, int L, int W>
__global__ __launch_bounds__(64 * W) void chain_iter_forward_trig_kernel(ChainTrig<V> P, int B, int T,
                                                                         ChainIter<V> a, LSParams ls) {
  const int b = (blockIdx.x * 64 * W + threadIdx.x) / L;
  if (b >= B || a.status[b] != ILQR_TRAJ_OK) return;
  const V pc = a.prev_cost ? a.prev_cost[b] : V(INFINITY);
  const ChainTrigModel<V, NU> m{P};
  const FgOut<V> r = fwd_group<ChainTrigModel<V, NU>, L>(m, b, B, T, a.x, a.u, a.xtraj, a.d, a.K, pc, a.xnew,
                                                          a.unew, ls, a.res_parity == nullptr);
  if (!r.owner) return;
  if (a.trials) a.trials[b] = r.trials;
  if (a.du2) a.du2[b] = r.du2;
  if (a.iters) a.iters[b] = a.iter;
  if (!r.accepted) {
    a.status[b] = (r.cost != r.cost) ? ILQR_TRAJ_NAN : ILQR_TRAJ_LS_EXHAUSTED;
    if (a.res_parity) a.res_parity[b] = a.parity;
  } else {
    a.new_cost[b] = r.cost;             // prev_cost = new_cost (:168)
    if ((double)r.du2 <= ls.tol) {      // (:171) break BEFORE the update
      a.status[b] = ILQR_TRAJ_CONVERGED;
      if (a.res_parity) a.res_parity[b] = a.parity;
    }
  }
}

// The end of a chain fit (the LQ driver's gather_kernel for V = float / double): x_out[b]
// = the buffer res_parity[b] names — x0 / x1 the handle's, PARITY_INPUT the caller's
// x_init, PARITY_OUT nothing to copy (the last iteration wrote x_out) — with
// final_parity for still-running trajectories, whose status becomes MAX_ITER; cost /
// iterations / status copied out (each may be null); the call-status bits (1 NaN,
// 2 exhausted search) OR-ed into dflags[0] by the trajectories that set one. One block
// per trajectory: status is read by every thread before thread 0 rewrites it.
template <class V>
__global__ __launch_bounds__(256) void chain_gather_kernel(int B, int nxe, int nue, const V* xin, const V* uin,
                                                           const V* x0, const V* u0, const V* x1, const V* u1,
                                                           const int32_t* res_parity, int32_t* status,
                                                           int final_parity, const V* fit_cost,
                                                           const int32_t* fit_iters, V* x_out, V* u_out,
                                                           V* cost_out, int32_t* iters_out, int32_t* status_out,
                                                           int32_t* dflags) {
  const int b = blockIdx.y;
  if (b >= B) return;
  const int32_t st0 = status[b];
  const bool running = st0 == ILQR_TRAJ_OK;
  const int par = running ? final_parity : res_parity[b];
  if (par != PARITY_OUT) {
    const V* xs = (par == PARITY_INPUT ? xin : (par ? x1 : x0)) + (size_t)b * nxe;
    const V* us = (par == PARITY_INPUT ? uin : (par ? u1 : u0)) + (size_t)b * nue;
    for (int i = threadIdx.x; i < nxe + nue; i += 256) {
      if (i < nxe) x_out[(size_t)b * nxe + i] = xs[i];
      else u_out[(size_t)b * nue + (i - nxe)] = us[i - nxe];
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const int32_t st = running ? ILQR_TRAJ_MAX_ITER : st0;
    status[b] = st;
    if (status_out) status_out[b] = st;
    if (cost_out) cost_out[b] = fit_cost[b];
    if (iters_out) iters_out[b] = fit_iters[b];
    const int f = (st == ILQR_TRAJ_NAN ? 1 : 0) | (st == ILQR_TRAJ_LS_EXHAUSTED ? 2 : 0);
    if (f) __hip_atomic_fetch_or(dflags, f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// fit's per-trajectory state (forward_pass.jl:159): prev_cost = +Inf, status OK, result
// "the input" (iteration 1 reads x_init / u_init in place), iterations 0 — one launch
template <class V>
__global__ void chain_fit_init_kernel(int B, V* prev_cost, int32_t* status, int32_t* res_parity, int32_t* iters) {
  const int b = blockIdx.x * 256 + threadIdx.x;
  if (b >= B) return;
  prev_cost[b] = V(INFINITY);
  status[b] = ILQR_TRAJ_OK;
  res_parity[b] = PARITY_INPUT;
  iters[b] = 0;
}

}  // namespace
}  // namespace ilqr

// ---------------------------------------------------------------------------
// Host side: the chain handle and its C ABI (include/ilqr.h, ilqr_chain_*)
// ---------------------------------------------------------------------------
struct ilqr_chain_handle {
  int device = 0;
  int nj = 0, nu = 0, T = 0, batch = 0;
  int dtype = ILQR_F64;
  int lin = ILQR_LINEARIZE_DUAL;
  ilqr_chain chain{};
  hipStream_t stream = nullptr;
  void* xbuf[2] = {nullptr, nullptr};
  void* ubuf[2] = {nullptr, nullptr};
  void* K = nullptr;
  void* d = nullptr;
  void* J = nullptr;
  void* prev_cost = nullptr;
  void* du2 = nullptr;
  int32_t* trials = nullptr;
  int32_t* status = nullptr;
  int32_t* res_parity = nullptr;
  int32_t* iters = nullptr;
  // the fit driver's host-mapped words ([0], [1] running counts of the poll, [2] the
  // call status tagged with the fit's number), their device alias, the gather's device
  // call-status word, the poll's events
  int32_t* host_words = nullptr;
  ilqr::HostWait host_wait;  // the end-of-fit wait (wait_host_seq)
  ilqr::HostWait poll_wait;  // the per-iteration convergence polls (wait_event)
  int32_t* dev_words = nullptr;
  int32_t* dev_flags = nullptr;
  hipEvent_t ev_poll[2] = {nullptr, nullptr};
  uint32_t fit_seq = 0;
  // closed-form dynamics of 2-joint chains (ilqr_chain_set_dynamics): available once
  // sampled and checked against the recursion at creation, used unless RNEA is asked for
  bool trig_ok = false;
  int32_t dyn_mode = ILQR_CHAIN_DYN_AUTO;
  double trig_err = 0.0;  // the check's max relative error
  ilqr::ChainTrig<double> trig{};
  bool use_trig() const { return trig_ok && dyn_mode != ILQR_CHAIN_DYN_RNEA; }
  // cost_functions.jl's factories (ilqr_chain_set_simple_costs): the mode, the chain's
  // joint-space weights as created (restored by ILQR_CHAIN_COST_JOINT) and the
  // task-space final cost's coefficients in device memory
  int32_t cost_mode = ILQR_CHAIN_COST_JOINT;
  ilqr_chain created{};
  ilqr::ChainTask* task_dev = nullptr;
  const ilqr::ChainTask* task() const { return cost_mode == ILQR_CHAIN_COST_JOINT ? nullptr : task_dev; }
};

namespace {

thread_local std::string g_chain_error;

ilqr_status chain_hip_fail(hipError_t e, const char* what) {
  g_chain_error = std::string(what) + ": " + hipGetErrorString(e);
  return ILQR_ERR_HIP;
}

#define CH_TRY(expr)                                         \
  do {                                                       \
    hipError_t e_ = (expr);                                  \
    if (e_ != hipSuccess) return chain_hip_fail(e_, #expr);  \
  } while (0)

template <class V, int NJ>
ilqr::ChainK<V, NJ> chain_consts(const ilqr_chain& c) {
  ilqr::ChainK<V, NJ> P{};
  for (int i = 0; i < NJ; ++i) {
    for (int k = 0; k < 9; ++k) P.R0[i][k] = (V)c.joint_rot[i][k];
    {  // R0·[a]× and R0·a·aᵀ in fp64, then rounded (joint_rot)
      const double* R0 = c.joint_rot[i];
      const double* a = c.axis[i];
      const double ax[9] = {0.0, -a[2], a[1], a[2], 0.0, -a[0], -a[1], a[0], 0.0};
      for (int r = 0; r < 3; ++r)
        for (int k = 0; k < 3; ++k) {
          double x = 0.0, y = 0.0;
          for (int j = 0; j < 3; ++j) {
            x += R0[3 * r + j] * ax[3 * j + k];
            y += R0[3 * r + j] * a[j] * a[k];
          }
          P.R0x[i][3 * r + k] = (V)x;
          P.R0aa[i][3 * r + k] = (V)y;
        }
    }
    for (int k = 0; k < 3; ++k) {
      P.p[i][k] = (V)c.joint_pos[i][k];
      P.ax[i][k] = (V)c.axis[i][k];
      P.mc[i][k] = (V)(c.mass[i] * c.com[i][k]);
    }
    P.m[i] = (V)c.mass[i];
    // Io = Ic + m(|c|²1 − c cᵀ): rotational inertia about the body origin (fp64 first)
    const double* cm = c.com[i];
    const double cc = cm[0] * cm[0] + cm[1] * cm[1] + cm[2] * cm[2];
    for (int r = 0; r < 3; ++r)
      for (int k = 0; k < 3; ++k)
        P.Io[i][3 * r + k] =
            (V)(c.inertia[i][3 * r + k] + c.mass[i] * ((r == k ? cc : 0.0) - cm[r] * cm[k]));
    P.tgt[i] = (V)c.target[i];
    P.qw[i] = (V)c.q_weight[i];
    P.rw[i] = (V)c.r_weight[i];
    P.qfw[i] = (V)c.qf_weight[i];
  }
  for (int k = 0; k < 3; ++k) P.g[k] = (V)c.gravity[k];
  P.dt = (V)c.dt;
  return P;
}

// ChainTrig<V> from the fp64 coefficients and the chain's cost
template <class V>
ilqr::ChainTrig<V> trig_consts(const ilqr_chain_handle* h) {
  ilqr::ChainTrig<V> Q{};
  const ilqr::ChainTrig<double>& D = h->trig;
  for (int e = 0; e < 3; ++e) {
    for (int k = 0; k < 5; ++k) Q.Mc[e][k] = (V)D.Mc[e][k];
  }
  for (int i = 0; i < 2; ++i)
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b) Q.Gc[i][a][b] = (V)D.Gc[i][a][b];
  const ilqr_chain& c = h->chain;
  for (int i = 0; i < 2; ++i) {
    Q.tgt[i] = (V)c.target[i];
    Q.qw[i] = (V)c.q_weight[i];
    Q.rw[i] = (V)c.r_weight[i];
    Q.qfw[i] = (V)c.qf_weight[i];
  }
  Q.dt = (V)c.dt;
  Q.task = h->task();
  return Q;
}

// Samples M and g with the recursion (fp64, on the device), takes their discrete
// Fourier coefficients (exact for M's degree 2 in q₂ and g's degree 1 in each angle:
// 5 and 3 points), and checks f against the recursion at 256 random states. Leaves
// trig_ok false when the check fails (the recursion is then used).
hipError_t chain_trig_build(ilqr_chain_handle* h) {
  h->trig_ok = false;
  if (h->nj != 2) return hipSuccess;
  const auto P = chain_consts<double, 2>(h->chain);
  constexpr int NCHK = 256;
  double* dev = nullptr;
  hipError_t e = hipMalloc(&dev, sizeof(double) * (ilqr::CH_TRIG_SAMPLES + NCHK));
  if (e != hipSuccess) return e;
  double smp[ilqr::CH_TRIG_SAMPLES], err[NCHK];
  ilqr::chain_trig_sample_kernel<<<1, 64>>>(P, dev);
  e = hipGetLastError();
  if (e == hipSuccess) e = hipMemcpy(smp, dev, sizeof(smp), hipMemcpyDeviceToHost);
  if (e == hipSuccess) {
    ilqr::ChainTrig<double>& D = h->trig;
    const double two_pi = 6.283185307179586476925286766559;
    for (int en = 0; en < 3; ++en) {  // a₀ + a₁ cos + b₁ sin + a₂ cos 2 + b₂ sin 2 from 5 samples
      double a0 = 0, a1 = 0, b1 = 0, a2 = 0, b2 = 0;
      for (int k = 0; k < 5; ++k) {
        const double f = smp[3 * k + en], t = two_pi * k / 5.0;
        a0 += f;
        a1 += f * std::cos(t);
        b1 += f * std::sin(t);
        a2 += f * std::cos(2 * t);
        b2 += f * std::sin(2 * t);
      }
      D.Mc[en][0] = a0 / 5;
      D.Mc[en][1] = 2 * a1 / 5;
      D.Mc[en][2] = 2 * b1 / 5;
      D.Mc[en][3] = 2 * a2 / 5;
      D.Mc[en][4] = 2 * b2 / 5;
    }
    for (int i = 0; i < 2; ++i) {  // 2-D transform on the 3×3 grid: φ = (1, cos, sin)
      for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b) {
          double acc = 0.0;
          for (int ka = 0; ka < 3; ++ka)
            for (int kb = 0; kb < 3; ++kb) {
              const double ta = two_pi * ka / 3.0, tb = two_pi * kb / 3.0;
              const double fa = a == 0 ? 1.0 / 3 : (a == 1 ? 2.0 / 3 * std::cos(ta) : 2.0 / 3 * std::sin(ta));
              const double fb = b == 0 ? 1.0 / 3 : (b == 1 ? 2.0 / 3 * std::cos(tb) : 2.0 / 3 * std::sin(tb));
              acc += smp[15 + 2 * (3 * ka + kb) + i] * fa * fb;
            }
          D.Gc[i][a][b] = acc;
        }
    }
    D.dt = h->chain.dt;
    ilqr::chain_trig_check_kernel<<<NCHK / 64, 64>>>(P, D, NCHK, dev + ilqr::CH_TRIG_SAMPLES);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpy(err, dev + ilqr::CH_TRIG_SAMPLES, sizeof(err), hipMemcpyDeviceToHost);
  (void)hipFree(dev);
  if (e != hipSuccess) return e;
  double m = 0.0;
  for (double v : err) m = std::isnan(v) ? INFINITY : std::max(m, v);
  h->trig_err = m;
  h->trig_ok = m < 1e-9;
  return hipSuccess;
}

// transform_to_root(state, body) * point (RigidBodyDynamics.jl; cost_functions.jl:20): the
// root-frame position of a point given in body `body`'s frame (−1 = the fixed base) at
// joint angles q, composing x_parent = p_i + R0_i·Rot(a_i, q_i)·x_child down the chain (fp64)
void chain_point_position(const ilqr_chain& c, int body, const double pt[3], const double* q,
                          double out[3]) {
  double w[3] = {pt[0], pt[1], pt[2]};
  for (int i = body; i >= 0; --i) {
    const double* a = c.axis[i];
    const double cq = std::cos(q[i]), sq = std::sin(q[i]);
    const double adw = a[0] * w[0] + a[1] * w[1] + a[2] * w[2];
    const double axw[3] = {a[1] * w[2] - a[2] * w[1], a[2] * w[0] - a[0] * w[2], a[0] * w[1] - a[1] * w[0]};
    double r[3];
    for (int k = 0; k < 3; ++k) r[k] = cq * w[k] + sq * axw[k] + (1.0 - cq) * adw * a[k];
    for (int k = 0; k < 3; ++k)
      w[k] = c.joint_pos[i][k] +
             (c.joint_rot[i][3 * k] * r[0] + c.joint_rot[i][3 * k + 1] * r[1] + c.joint_rot[i][3 * k + 2] * r[2]);
  }
  for (int k = 0; k < 3; ++k) out[k] = w[k];
}

// The task cost's coefficients: p sampled on the 3×3 grid of (q₁, q₂) and transformed
// like g's (exact for the bilinear form), then checked against the kinematics at 64
// pseudo-random angles. Returns the check's max deviation relative to the point's reach.
double chain_task_build(const ilqr_chain& c, int body, const double pt[3], const double tgt[3],
                        double weight, bool literal, ilqr::ChainTask& C) {
  const double two_pi = 6.283185307179586476925286766559;
  double smp[3][3][3];  // [ka][kb][coordinate]
  for (int ka = 0; ka < 3; ++ka)
    for (int kb = 0; kb < 3; ++kb) {
      const double q[2] = {two_pi * ka / 3.0, two_pi * kb / 3.0};
      chain_point_position(c, body, pt, q, smp[ka][kb]);
    }
  double P[3][3][3];
  for (int k = 0; k < 3; ++k)
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b) {
        double acc = 0.0;
        for (int ka = 0; ka < 3; ++ka)
          for (int kb = 0; kb < 3; ++kb) {
            const double ta = two_pi * ka / 3.0, tb = two_pi * kb / 3.0;
            const double fa = a == 0 ? 1.0 / 3 : (a == 1 ? 2.0 / 3 * std::cos(ta) : 2.0 / 3 * std::sin(ta));
            const double fb = b == 0 ? 1.0 / 3 : (b == 1 ? 2.0 / 3 * std::cos(tb) : 2.0 / 3 * std::sin(tb));
            acc += smp[ka][kb][k] * fa * fb;
          }
        P[k][a][b] = acc;
      }
  for (int k = 0; k < 3; ++k)
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b) C.Pc[k][a][b] = P[literal ? 2 : k][a][b];
  for (int k = 0; k < 3; ++k) C.t[k] = tgt[k];
  C.w = weight;
  double err = 0.0, reach = 1.0;
  uint64_t st = 0x9E3779B97F4A7C15ull;
  for (int n = 0; n < 64; ++n) {
    double q[2];
    for (double& v : q) {
      st = st * 6364136223846793005ull + 1442695040888963407ull;
      v = ((double)(st >> 11) * (1.0 / 9007199254740992.0) - 0.5) * 4.0 * two_pi;
    }
    double ref[3];
    chain_point_position(c, body, pt, q, ref);
    const double c0 = std::cos(q[0]), s0 = std::sin(q[0]), c1 = std::cos(q[1]), s1 = std::sin(q[1]);
    const double f0[3] = {1.0, c0, s0}, f1[3] = {1.0, c1, s1};
    for (int k = 0; k < 3; ++k) {
      double v = 0.0;
      for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b) v += P[k][a][b] * f0[a] * f1[b];
      err = std::max(err, std::fabs(v - ref[k]));
      reach = std::max(reach, std::fabs(ref[k]));
    }
  }
  return err / reach;
}

ilqr::LSParams chain_ls(const ilqr_options* o) {
  ilqr_options def;
  ilqr_default_options(&def);
  if (!o) o = &def;
  return ilqr::LSParams{o->mu, o->alpha0, o->shrink, o->tol, o->max_trials};
}

ilqr_status chain_check_options(const ilqr_options* o) {
  if (!o) return ILQR_OK;
  if (o->max_trials < 1 || o->max_iter < 0) return ILQR_ERR_BAD_ARG;
  if (!(o->shrink > 0.0 && o->shrink < 1.0) || !(o->alpha0 > 0.0) || std::isnan(o->mu))
    return ILQR_ERR_BAD_ARG;
  return ILQR_OK;
}

size_t vsize(const ilqr_chain_handle* h) { return h->dtype == ILQR_F32 ? 4 : 8; }

// Typed operations of one (V, NJ, NU) instantiation.
template <class V, int NJ, int NU>
struct ChainOps {
  static constexpr int NX = 2 * NJ;
  using Value = V;
  using Iter = ilqr::ChainIter<V>;

  static hipError_t linearize(ilqr_chain_handle* h, const V* x, const V* u, const int32_t* st) {
    const auto P = chain_consts<V, NJ>(h->chain);
    const size_t lanes = (size_t)h->batch * h->T * (NX + NU);
    const dim3 grid((unsigned)((lanes + 255) / 256));
    if constexpr (NJ == 2) {
      if (h->use_trig()) {
        const auto Q = trig_consts<V>(h);
        using TK = ilqr::ChainTrig<V>;
        if (h->lin == ILQR_LINEARIZE_DUAL)
          ilqr::chain_linearize_kernel<V, NJ, NU, ILQR_LINEARIZE_DUAL, TK>
              <<<grid, 256, 0, h->stream>>>(Q, h->batch, h->T, x, u, st, (V*)h->J);
        else
          ilqr::chain_linearize_kernel<V, NJ, NU, ILQR_LINEARIZE_CENTRAL_FD, TK>
              <<<grid, 256, 0, h->stream>>>(Q, h->batch, h->T, x, u, st, (V*)h->J);
        return hipGetLastError();
      }
    }
    if (h->lin == ILQR_LINEARIZE_DUAL)
      ilqr::chain_linearize_kernel<V, NJ, NU, ILQR_LINEARIZE_DUAL>
          <<<grid, 256, 0, h->stream>>>(P, h->batch, h->T, x, u, st, (V*)h->J);
    else
      ilqr::chain_linearize_kernel<V, NJ, NU, ILQR_LINEARIZE_CENTRAL_FD>
          <<<grid, 256, 0, h->stream>>>(P, h->batch, h->T, x, u, st, (V*)h->J);
    return hipGetLastError();
  }
  static hipError_t unpack(ilqr_chain_handle* h, V* A, V* Bm) {
    const size_t n = (size_t)h->batch * h->T;
    ilqr::chain_unpack_kernel<V, NJ, NU><<<(unsigned)((n + 255) / 256), 256, 0, h->stream>>>(
        h->batch, h->T, (const V*)h->J, A, Bm);
    return hipGetLastError();
  }
  static hipError_t backward(ilqr_chain_handle* h, const V* x, const V* u, V* d, V* K,
                             int32_t* st, double mu) {
    hipError_t e = linearize(h, x, u, nullptr);
    if (e != hipSuccess) return e;
    const auto P = chain_consts<V, NJ>(h->chain);
    if constexpr (NJ == 2) {  // four trajectories per wave on the f64 MFMA
      ilqr::chain_backward4_kernel<V, NU><<<(h->batch + 15) / 16, 256, 0, h->stream>>>(
          P, h->batch, h->T, x, (const V*)h->J, d, K, st, (V)mu, h->task());
      return hipGetLastError();
    }
    ilqr::chain_backward_kernel<V, NJ, NU><<<(h->batch + ilqr::CH_WG - 1) / ilqr::CH_WG, ilqr::CH_WG,
                                             0, h->stream>>>(P, h->batch, h->T, x, (const V*)h->J,
                                                             d, K, st, (V)mu);
    return hipGetLastError();
  }
  static hipError_t forward(ilqr_chain_handle* h, const V* x, const V* u, const V* xt, const V* d,
                            const V* K, const V* pc, V* xn, V* un, V* nc, int32_t* tr,
                            int32_t* st, const ilqr::LSParams& ls) {
    if constexpr (NJ == 2) {
      if (h->use_trig()) {
        if (!ilqr::fg_fits<V>(h->T)) return hipErrorInvalidValue;
        const auto Q = trig_consts<V>(h);
        const int B = h->batch;
        const int L = ilqr::fg_lanes(B);
        if (L == 32)
          ilqr::chain_forward_trig_kernel<V, NU, 32, 1><<<(32 * B + 63) / 64, 64, 0, h->stream>>>(
              Q, B, h->T, x, u, xt, d, K, pc, xn, un, nc, tr, st, ls);
        else if (L == 4)
          ilqr::chain_forward_trig_kernel<V, NU, 4, 1><<<(4 * B + 63) / 64, 64, 0, h->stream>>>(
              Q, B, h->T, x, u, xt, d, K, pc, xn, un, nc, tr, st, ls);
        else
          ilqr::chain_forward_trig_kernel<V, NU, 1, 4><<<(B + 255) / 256, 256, 0, h->stream>>>(
              Q, B, h->T, x, u, xt, d, K, pc, xn, un, nc, tr, st, ls);
        return hipGetLastError();
      }
    }
    const auto P = chain_consts<V, NJ>(h->chain);
    ilqr::chain_forward_kernel<V, NJ, NU><<<(h->batch * ilqr::CH_FW_LANES + ilqr::CH_WG - 1) / ilqr::CH_WG, ilqr::CH_WG,
                                            0, h->stream>>>(P, h->batch, h->T, x, u, xt, d, K, pc,
                                                            xn, un, nc, tr, st, ls);
    return hipGetLastError();
  }
  static hipError_t iteration(ilqr_chain_handle* h, const Iter& a, const ilqr::LSParams& ls) {
    hipError_t e = linearize(h, a.x, a.u, a.status);
    if (e != hipSuccess) return e;
    const auto P = chain_consts<V, NJ>(h->chain);
    if constexpr (NJ == 2) {
      ilqr::chain_iter_backward4_kernel<V, NU>
          <<<(h->batch + 15) / 16, 256, 0, h->stream>>>(P, h->batch, h->T, a, (const V*)h->J, (V)ls.mu,
                                                         h->task());
    } else {
      const int g = (h->batch + ilqr::CH_WG - 1) / ilqr::CH_WG;
      ilqr::chain_iter_backward_kernel<V, NJ, NU>
          <<<g, ilqr::CH_WG, 0, h->stream>>>(P, h->batch, h->T, a, (const V*)h->J, (V)ls.mu);
    }
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if constexpr (NJ == 2) {
      if (h->use_trig()) {
        if (!ilqr::fg_fits<V>(h->T)) return hipErrorInvalidValue;
        const auto Q = trig_consts<V>(h);
        const int B = h->batch;
        const int L = ilqr::fg_lanes(B, a.iter >= 2);  // a fit past its first iteration
        if (L == 32)
          ilqr::chain_iter_forward_trig_kernel<V, NU, 32, 1><<<(32 * B + 63) / 64, 64, 0, h->stream>>>(Q, B, h->T, a, ls);
        else if (L == 4)
          ilqr::chain_iter_forward_trig_kernel<V, NU, 4, 1><<<(4 * B + 63) / 64, 64, 0, h->stream>>>(Q, B, h->T, a, ls);
        else
          ilqr::chain_iter_forward_trig_kernel<V, NU, 1, 4><<<(B + 255) / 256, 256, 0, h->stream>>>(Q, B, h->T, a, ls);
        return hipGetLastError();
      }
    }
    const int gf = (h->batch * ilqr::CH_FW_LANES + ilqr::CH_WG - 1) / ilqr::CH_WG;
    ilqr::chain_iter_forward_kernel<V, NJ, NU><<<gf, ilqr::CH_WG, 0, h->stream>>>(P, h->batch, h->T,
                                                                                 a, ls);
    return hipGetLastError();
  }
  static hipError_t dynamics(ilqr_chain_handle* h, const V* x, const V* u, V* xo, int n) {
    if constexpr (NJ == 2) {
      if (h->use_trig()) {
        ilqr::chain_dynamics_kernel<V, NJ, NU, ilqr::ChainTrig<V>>
            <<<(n + 255) / 256, 256, 0, h->stream>>>(trig_consts<V>(h), n, x, u, xo);
        return hipGetLastError();
      }
    }
    const auto P = chain_consts<V, NJ>(h->chain);
    ilqr::chain_dynamics_kernel<V, NJ, NU><<<(n + 255) / 256, 256, 0, h->stream>>>(P, n, x, u, xo);
    return hipGetLastError();
  }
};

// (n_joints, nu) shapes with compiled kernels: the iLQR iteration for the 2-DoF arm
// (nu = 2 every joint driven, nu = 1 joint 1 only); dynamics also for the 6-DoF arm.
bool iter_supported(int nj, int nu) { return nj == 2 && (nu == 1 || nu == 2); }
bool dyn_supported(int nj, int nu) { return iter_supported(nj, nu) || (nj == 6 && nu == 6); }

template <class V, class Fn>
hipError_t dispatch(const ilqr_chain_handle* h, Fn&& fn) {
  if (h->nj == 2 && h->nu == 2) return fn(ChainOps<V, 2, 2>{});
  if (h->nj == 2 && h->nu == 1) return fn(ChainOps<V, 2, 1>{});
  return hipErrorInvalidValue;
}
template <class Fn>
hipError_t dispatch_any(const ilqr_chain_handle* h, Fn&& fn) {
  if (h->dtype == ILQR_F32) return dispatch<float>(h, fn);
  return dispatch<double>(h, fn);
}

template <class V>
ilqr::ChainIter<V> iter_args(const ilqr_chain_handle* h, const void* x, const void* u,
                             const void* xt, void* xn, void* un, const void* pc, void* nc,
                             void* du2, int32_t* tr, int32_t* st) {
  ilqr::ChainIter<V> a{};
  a.x = (const V*)x;
  a.u = (const V*)u;
  a.xtraj = (const V*)xt;
  a.xnew = (V*)xn;
  a.unew = (V*)un;
  a.K = (V*)h->K;
  a.d = (V*)h->d;
  a.prev_cost = (const V*)pc;
  a.new_cost = (V*)nc;
  a.du2 = (V*)du2;
  a.trials = tr;
  a.status = st;
  return a;
}

// Reduce per-trajectory status to the call status (host copy, synchronising):
// ilqr_chain_backward / ilqr_chain_forward
ilqr_status chain_fold_status(ilqr_chain_handle* h, const int32_t* dev_status) {
  std::vector<int32_t> st(h->batch);
  CH_TRY(hipMemcpyAsync(st.data(), dev_status, sizeof(int32_t) * h->batch, hipMemcpyDeviceToHost,
                        h->stream));
  CH_TRY(hipStreamSynchronize(h->stream));
  bool nan = false, ls = false;
  for (int32_t s : st) {
    nan |= s == ILQR_TRAJ_NAN;
    ls |= s == ILQR_TRAJ_LS_EXHAUSTED;
  }
  return nan ? ILQR_ERR_NAN : (ls ? ILQR_ERR_LS_EXHAUSTED : ILQR_OK);
}

template <class V>
ilqr_status chain_fit_t(ilqr_chain_handle* h, const ilqr_options* o, const void* x_init,
                        const void* u_init, const void* x_traj, void* x_out, void* u_out,
                        void* cost, int32_t* iters, int32_t* status, const ilqr_history* hist) {
  // The LQ fit driver's structure (ilqr_abi.cpp ilqr_fit_ex, DESIGN.md §4 fit driver):
  // iteration 1 reads x_init / u_init in place (no copy-in), the last iteration writes
  // x_out / u_out directly unless they overlap an input, a tol ≥ 0 fit stops enqueueing
  // once every trajectory has stopped (the running count one iteration behind), and the
  // call ends with one gather + a one-thread launch that publishes the call status to a
  // host-mapped word the host spins on (no status copy, no host fold).
  const size_t B = (size_t)h->batch, nx = 2 * (size_t)h->nj;
  const size_t nxe = (h->T + 1) * nx, nue = (size_t)h->T * h->nu;
  hipStream_t s = h->stream;
  const ilqr::LSParams ls = chain_ls(o);
  const int max_iter = o ? o->max_iter : 100;
  const unsigned g = (unsigned)((B + 255) / 256);
  ilqr::chain_fit_init_kernel<V><<<g, 256, 0, s>>>(h->batch, (V*)h->prev_cost, h->status, h->res_parity, h->iters);
  CH_TRY(hipGetLastError());
  volatile int32_t* flags = h->host_words + 2;
  *flags = 0;
  const size_t xb = sizeof(V) * B * nxe, ub = sizeof(V) * B * nue;
  auto overlap = [](const void* p, size_t np, const void* q, size_t nq) {
    const char *a = (const char*)p, *b = (const char*)q;
    return q && a < b + nq && b < a + np;
  };
  const bool direct = max_iter > 0 && !overlap(x_out, xb, x_init, xb) && !overlap(x_out, xb, x_traj, xb) &&
                      !overlap(x_out, xb, u_init, ub) && !overlap(u_out, ub, u_init, ub) &&
                      !overlap(u_out, ub, x_init, xb) && !overlap(u_out, ub, x_traj, xb);
  const bool poll = ls.tol >= 0.0 && max_iter > 2;
  int enqueued = 0, waited = 0;  // iterations (the end-of-fit wait's units)
  for (int it = 1; it <= max_iter; ++it) {  // forward_pass.jl:161
    const int par = (it - 1) & 1;
    const bool last = direct && it == max_iter;
    auto a = iter_args<V>(h, it == 1 ? x_init : h->xbuf[par], it == 1 ? u_init : h->ubuf[par], x_traj,
                          last ? x_out : h->xbuf[par ^ 1], last ? u_out : h->ubuf[par ^ 1], h->prev_cost,
                          h->prev_cost, h->du2, h->trials, h->status);
    a.res_parity = h->res_parity;
    a.iters = h->iters;
    a.parity = it == 1 ? ilqr::PARITY_INPUT : par;  // where the input x̄ⁱ, ūⁱ lie (:174-175)
    a.iter = it;
    CH_TRY(dispatch<V>(h, [&](auto ops) { return decltype(ops)::iteration(h, a, ls); }));
    enqueued = it;
    if (hist)  // the per-iteration record (ilqr_history)
      CH_TRY(ilqr::launch_record_history(h->batch, it, h->status, h->iters, h->trials, h->prev_cost, h->du2,
                                         sizeof(V) == 4, ls.alpha0, ls.shrink, hist->cost, hist->trials,
                                         hist->alpha, hist->du2, s));
    if (!poll || it == max_iter) continue;
    CH_TRY(ilqr::launch_count_running(h->batch, h->status, h->dev_words + (it & 1), s));
    CH_TRY(hipEventRecord(h->ev_poll[it & 1], s));
    if (it >= 2) {  // iteration it−1's count, read while iteration it runs (:171's break)
      CH_TRY(ilqr::wait_event(h->ev_poll[(it - 1) & 1], &h->poll_wait));
      waited = it - 1;
      if (__atomic_load_n(h->host_words + ((it - 1) & 1), __ATOMIC_ACQUIRE) == 0) break;
    }
  }
  // still-running trajectories (max_iter reached) return the last accepted iterate
  const int final_parity =
      max_iter == 0 ? ilqr::PARITY_INPUT : (direct ? ilqr::PARITY_OUT : (max_iter & 1));
  ilqr::chain_gather_kernel<V><<<dim3(1, h->batch), 256, 0, s>>>(
      h->batch, (int)nxe, (int)nue, (const V*)x_init, (const V*)u_init, (const V*)h->xbuf[0],
      (const V*)h->ubuf[0], (const V*)h->xbuf[1], (const V*)h->ubuf[1], h->res_parity, h->status, final_parity,
      (const V*)h->prev_cost, h->iters, (V*)x_out, (V*)u_out, (V*)cost, iters, status, h->dev_flags);
  CH_TRY(hipGetLastError());
  uint32_t seq = (++h->fit_seq) & 0x3fffffffu;
  if (seq == 0) seq = h->fit_seq = 1;  // 0 is the word's cleared value
  CH_TRY(ilqr::launch_publish_flags(h->dev_flags, h->dev_words + 2, seq, s));
  CH_TRY(ilqr::wait_host_seq(h->host_words + 2, seq, enqueued - waited, s, &h->host_wait));
  const int32_t f = __atomic_load_n(h->host_words + 2, __ATOMIC_ACQUIRE);
  return (f & 1) ? ILQR_ERR_NAN : ((f & 2) ? ILQR_ERR_LS_EXHAUSTED : ILQR_OK);
}

}  // namespace

extern "C" {

int ilqr_chain_supported(int n_joints, int nu) { return iter_supported(n_joints, nu) ? 1 : 0; }

const char* ilqr_chain_last_error(void) { return g_chain_error.c_str(); }

ilqr_status ilqr_chain_create(ilqr_chain_handle** out, int device, const ilqr_chain* chain, int T,
                              int batch, int32_t dtype, int32_t linearization) {
  if (!out || !chain) return ILQR_ERR_BAD_ARG;
  *out = nullptr;
  if (T <= 0 || batch <= 0 || chain->n_joints <= 0 || chain->nu <= 0) return ILQR_ERR_BAD_DIMS;
  if (chain->n_joints > ILQR_CHAIN_MAX_JOINTS || !(chain->nu == chain->n_joints || chain->nu == 1))
    return ILQR_ERR_BAD_DIMS;
  if (dtype != ILQR_F32 && dtype != ILQR_F64) return ILQR_ERR_BAD_ARG;
  if (linearization != ILQR_LINEARIZE_DUAL && linearization != ILQR_LINEARIZE_CENTRAL_FD)
    return ILQR_ERR_BAD_ARG;
  if (!(chain->dt > 0.0)) return ILQR_ERR_BAD_ARG;
  if (!dyn_supported(chain->n_joints, chain->nu)) return ILQR_ERR_UNSUPPORTED;
  CH_TRY(hipSetDevice(device));
  auto* h = new ilqr_chain_handle;
  h->device = device;
  h->nj = chain->n_joints;
  h->nu = chain->nu;
  h->T = T;
  h->batch = batch;
  h->dtype = dtype;
  h->lin = linearization;
  h->chain = *chain;
  h->created = *chain;
  const size_t w = vsize(h), B = (size_t)batch, nx = 2 * (size_t)h->nj, nu = (size_t)h->nu;
  hipError_t e = hipSuccess;
  if (iter_supported(h->nj, h->nu)) {  // dynamics-only shapes need no workspace
    for (int i = 0; i < 2 && e == hipSuccess; ++i) {
      e = hipMalloc(&h->xbuf[i], w * B * (T + 1) * nx);
      if (e == hipSuccess) e = hipMalloc(&h->ubuf[i], w * B * T * nu);
    }
    if (e == hipSuccess) e = hipMalloc(&h->K, w * B * T * nu * nx);
    if (e == hipSuccess) e = hipMalloc(&h->d, w * B * T * nu);
    if (e == hipSuccess) e = hipMalloc(&h->J, w * B * T * (nx * (nx + nu) + nx + nu));
    if (e == hipSuccess) e = hipMalloc(&h->prev_cost, w * B);
    if (e == hipSuccess) e = hipMalloc(&h->du2, w * B);
    if (e == hipSuccess) e = hipMalloc(&h->trials, sizeof(int32_t) * B);
    if (e == hipSuccess) e = hipMalloc(&h->status, sizeof(int32_t) * B);
    if (e == hipSuccess) e = hipMalloc(&h->res_parity, sizeof(int32_t) * B);
    if (e == hipSuccess) e = hipMalloc(&h->iters, sizeof(int32_t) * B);
    if (e == hipSuccess)
      e = hipHostMalloc(&h->host_words, sizeof(int32_t) * 4, hipHostMallocMapped | hipHostMallocCoherent);
    if (e == hipSuccess) e = hipHostGetDevicePointer((void**)&h->dev_words, h->host_words, 0);
    if (e == hipSuccess) e = hipMalloc(&h->dev_flags, sizeof(int32_t) * 2);
    if (e == hipSuccess) e = hipMemset(h->dev_flags, 0, sizeof(int32_t) * 2);
    for (int c = 0; c < 2 && e == hipSuccess; ++c) e = hipEventCreateWithFlags(&h->ev_poll[c], hipEventDisableTiming);
  }
  if (e != hipSuccess) {
    ilqr_chain_destroy(h);
    return chain_hip_fail(e, "ilqr_chain_create: hipMalloc");
  }
  if (iter_supported(h->nj, h->nu) && (e = chain_trig_build(h)) != hipSuccess) {
    ilqr_chain_destroy(h);
    return chain_hip_fail(e, "ilqr_chain_create: closed-form dynamics");
  }
  *out = h;
  return ILQR_OK;
}

ilqr_status ilqr_chain_set_dynamics(ilqr_chain_handle* h, int32_t mode) {
  if (!h) return ILQR_ERR_BAD_ARG;
  if (mode != ILQR_CHAIN_DYN_AUTO && mode != ILQR_CHAIN_DYN_RNEA && mode != ILQR_CHAIN_DYN_CLOSED_FORM)
    return ILQR_ERR_BAD_ARG;
  if (mode == ILQR_CHAIN_DYN_CLOSED_FORM && !h->trig_ok) return ILQR_ERR_UNSUPPORTED;
  // the task-space final cost is evaluated by the closed-form forward only
  if (mode == ILQR_CHAIN_DYN_RNEA && h->cost_mode != ILQR_CHAIN_COST_JOINT) return ILQR_ERR_UNSUPPORTED;
  h->dyn_mode = mode;
  return ILQR_OK;
}

ilqr_status ilqr_chain_set_simple_costs(ilqr_chain_handle* h, int32_t mode, int32_t body,
                                        const double* point, const double* final_target,
                                        double weight) {
  if (!h) return ILQR_ERR_BAD_ARG;
  if (mode != ILQR_CHAIN_COST_JOINT && mode != ILQR_CHAIN_COST_SIMPLE &&
      mode != ILQR_CHAIN_COST_SIMPLE_EUCLIDEAN)
    return ILQR_ERR_BAD_ARG;
  if (mode == ILQR_CHAIN_COST_JOINT) {  // the joint-space costs the handle was created with
    if (h->cost_mode != ILQR_CHAIN_COST_JOINT) {
      CH_TRY(hipStreamSynchronize(h->stream));  // launches in flight still read the old cost
      h->chain = h->created;
      h->cost_mode = ILQR_CHAIN_COST_JOINT;
    }
    return ILQR_OK;
  }
  if (!point || !final_target || !std::isfinite(weight)) return ILQR_ERR_BAD_ARG;
  if (body < -1 || body >= h->nj) return ILQR_ERR_BAD_ARG;
  for (int k = 0; k < 3; ++k)
    if (!std::isfinite(point[k]) || !std::isfinite(final_target[k])) return ILQR_ERR_BAD_ARG;
  if (!iter_supported(h->nj, h->nu) || !h->use_trig()) {
    g_chain_error = "ilqr_chain_set_simple_costs: needs a 2-joint chain on the closed-form dynamics";
    return ILQR_ERR_UNSUPPORTED;
  }
  ilqr::ChainTask C{};
  const double err =
      chain_task_build(h->created, body, point, final_target, weight, mode == ILQR_CHAIN_COST_SIMPLE, C);
  if (!(err < 1e-12)) {
    g_chain_error = "ilqr_chain_set_simple_costs: the point's coordinates are not bilinear in "
                    "(cos, sin) of the joint angles (kinematics check failed)";
    return ILQR_ERR_UNSUPPORTED;
  }
  CH_TRY(hipSetDevice(h->device));
  CH_TRY(hipStreamSynchronize(h->stream));
  if (!h->task_dev) CH_TRY(hipMalloc(&h->task_dev, sizeof(ilqr::ChainTask)));
  CH_TRY(hipMemcpy(h->task_dev, &C, sizeof(C), hipMemcpyHostToDevice));
  // simple_immediate_cost = Σ uᵢ² (cost_functions.jl:45-51): q_weight 0, r_weight 1
  h->chain = h->created;
  for (int i = 0; i < ILQR_CHAIN_MAX_JOINTS; ++i) {
    h->chain.q_weight[i] = 0.0;
    h->chain.r_weight[i] = 1.0;
    h->chain.qf_weight[i] = 0.0;
  }
  h->cost_mode = mode;
  return ILQR_OK;
}

int32_t ilqr_chain_get_cost_mode(const ilqr_chain_handle* h) { return h ? h->cost_mode : -1; }

int32_t ilqr_chain_get_dynamics(const ilqr_chain_handle* h) {
  if (!h) return -1;
  return h->use_trig() ? ILQR_CHAIN_DYN_CLOSED_FORM : ILQR_CHAIN_DYN_RNEA;
}

double ilqr_chain_closed_form_error(const ilqr_chain_handle* h) { return h ? h->trig_err : -1.0; }

ilqr_status ilqr_chain_destroy(ilqr_chain_handle* h) {
  if (!h) return ILQR_OK;
  (void)hipSetDevice(h->device);
  for (int i = 0; i < 2; ++i) {
    (void)hipFree(h->xbuf[i]);
    (void)hipFree(h->ubuf[i]);
  }
  for (void* p : {h->K, h->d, h->J, h->prev_cost, h->du2}) (void)hipFree(p);
  for (int32_t* p : {h->trials, h->status, h->res_parity, h->iters, h->dev_flags}) (void)hipFree(p);
  if (h->host_words) (void)hipHostFree(h->host_words);
  for (hipEvent_t ev : h->ev_poll)
    if (ev) (void)hipEventDestroy(ev);
  (void)hipFree(h->task_dev);
  delete h;
  return ILQR_OK;
}

ilqr_status ilqr_chain_set_stream(ilqr_chain_handle* h, void* s) {
  if (!h) return ILQR_ERR_BAD_ARG;
  h->stream = (hipStream_t)s;
  return ILQR_OK;
}

ilqr_status ilqr_chain_dynamics(ilqr_chain_handle* h, const void* x, const void* u, void* x_next,
                                int n) {
  if (!h || !x || !u || !x_next) return ILQR_ERR_BAD_ARG;
  if (n <= 0) return ILQR_ERR_BAD_DIMS;
  CH_TRY(hipSetDevice(h->device));
  auto fn = [&](auto ops) {
    using O = decltype(ops);
    using V = typename O::Value;
    return O::dynamics(h, (const V*)x, (const V*)u, (V*)x_next, n);
  };
  hipError_t e;
  if (h->nj == 6) {
    e = h->dtype == ILQR_F32 ? fn(ChainOps<float, 6, 6>{}) : fn(ChainOps<double, 6, 6>{});
  } else {
    e = dispatch_any(h, fn);
  }
  CH_TRY(e);
  return ILQR_OK;
}

ilqr_status ilqr_chain_linearize(ilqr_chain_handle* h, const void* x, const void* u, void* A,
                                 void* B) {
  if (!h || !x || !u || !A || !B) return ILQR_ERR_BAD_ARG;
  if (!iter_supported(h->nj, h->nu)) return ILQR_ERR_UNSUPPORTED;
  CH_TRY(hipSetDevice(h->device));
  CH_TRY(dispatch_any(h, [&](auto ops) {
    using O = decltype(ops);
    using V = typename O::Value;
    hipError_t e = O::linearize(h, (const V*)x, (const V*)u, nullptr);
    return e != hipSuccess ? e : O::unpack(h, (V*)A, (V*)B);
  }));
  return ILQR_OK;
}

ilqr_status ilqr_chain_backward(ilqr_chain_handle* h, const ilqr_options* o, const void* x,
                                const void* u, void* d, void* K, int32_t* status) {
  if (!h || !x || !u || !d || !K) return ILQR_ERR_BAD_ARG;
  if (!iter_supported(h->nj, h->nu)) return ILQR_ERR_UNSUPPORTED;
  ilqr_status st = chain_check_options(o);
  if (st != ILQR_OK) return st;
  CH_TRY(hipSetDevice(h->device));
  const double mu = chain_ls(o).mu;
  CH_TRY(dispatch_any(h, [&](auto ops) {
    using O = decltype(ops);
    using V = typename O::Value;
    return O::backward(h, (const V*)x, (const V*)u, (V*)d, (V*)K, status, mu);
  }));
  return status ? chain_fold_status(h, status) : ILQR_OK;
}

ilqr_status ilqr_chain_forward(ilqr_chain_handle* h, const ilqr_options* o, const void* x,
                               const void* u, const void* x_traj, const void* d, const void* K,
                               const void* prev_cost, void* x_new, void* u_new, void* new_cost,
                               int32_t* trials, int32_t* status) {
  if (!h || !x || !u || !d || !K || !prev_cost || !x_new || !u_new || !new_cost)
    return ILQR_ERR_BAD_ARG;
  if (!iter_supported(h->nj, h->nu)) return ILQR_ERR_UNSUPPORTED;
  ilqr_status st = chain_check_options(o);
  if (st != ILQR_OK) return st;
  CH_TRY(hipSetDevice(h->device));
  const ilqr::LSParams ls = chain_ls(o);
  CH_TRY(dispatch_any(h, [&](auto ops) {
    using O = decltype(ops);
    using V = typename O::Value;
    return O::forward(h, (const V*)x, (const V*)u, (const V*)x_traj, (const V*)d, (const V*)K,
                      (const V*)prev_cost, (V*)x_new, (V*)u_new, (V*)new_cost, trials, status, ls);
  }));
  return status ? chain_fold_status(h, status) : ILQR_OK;
}

ilqr_status ilqr_chain_iterate(ilqr_chain_handle* h, const ilqr_options* o, const void* x,
                               const void* u, const void* x_traj, void* x_new, void* u_new,
                               const void* prev_cost, void* new_cost, void* du2, int32_t* trials,
                               int32_t* status) {
  if (!h || !x || !u || !x_new || !u_new || !new_cost || !status) return ILQR_ERR_BAD_ARG;
  if (!iter_supported(h->nj, h->nu)) return ILQR_ERR_UNSUPPORTED;
  ilqr_status st = chain_check_options(o);
  if (st != ILQR_OK) return st;
  CH_TRY(hipSetDevice(h->device));
  const ilqr::LSParams ls = chain_ls(o);
  CH_TRY(dispatch_any(h, [&](auto ops) {
    using O = decltype(ops);
    using V = typename O::Value;
    const auto a = iter_args<V>(h, x, u, x_traj, x_new, u_new, prev_cost, new_cost, du2, trials,
                                status);
    return O::iteration(h, a, ls);
  }));
  return ILQR_OK;
}

ilqr_status ilqr_chain_fit(ilqr_chain_handle* h, const ilqr_options* o, const void* x_init,
                           const void* u_init, const void* x_traj, void* x_out, void* u_out,
                           void* cost, int32_t* iters, int32_t* status) {
  return ilqr_chain_fit_ex(h, o, x_init, u_init, x_traj, x_out, u_out, cost, iters, status, nullptr);
}

ilqr_status ilqr_chain_fit_ex(ilqr_chain_handle* h, const ilqr_options* o, const void* x_init,
                              const void* u_init, const void* x_traj, void* x_out, void* u_out,
                              void* cost, int32_t* iters, int32_t* status, const ilqr_history* hist) {
  if (!h || !x_init || !u_init || !x_out || !u_out) return ILQR_ERR_BAD_ARG;
  if (hist && !hist->cost && !hist->trials && !hist->alpha && !hist->du2) hist = nullptr;
  if (!iter_supported(h->nj, h->nu)) return ILQR_ERR_UNSUPPORTED;
  ilqr_status st = chain_check_options(o);
  if (st != ILQR_OK) return st;
  CH_TRY(hipSetDevice(h->device));
  if (h->dtype == ILQR_F32)
    return chain_fit_t<float>(h, o, x_init, u_init, x_traj, x_out, u_out, cost, iters, status, hist);
  return chain_fit_t<double>(h, o, x_init, u_init, x_traj, x_out, u_out, cost, iters, status, hist);
}

ilqr_status ilqr_chain_sync(ilqr_chain_handle* h) {
  if (!h) return ILQR_ERR_BAD_ARG;
  CH_TRY(hipStreamSynchronize(h->stream));
  return ILQR_OK;
}

}  // extern "C"
