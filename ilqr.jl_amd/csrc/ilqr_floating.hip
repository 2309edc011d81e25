// Floating-base RBD family (include/ilqr.h ilqr_floating_*): the reference's RBD example
// as its script runs it — test/RBD_2_link_example/RBD_helper_functions.jl:48-116 on
// test/urdf/2Dof_arm.urdf parsed with `floating = true, gravity = 0` (:7), fitted by
// animate_RBD_2_link.jl:31 at nx = 16, nu = 8, T = 1000. Every piece of an iteration
// runs on the device:
//   * fb_linearize_kernel: linearize_dynamics (backward_pass.jl:25-40) at every (b, t),
//     one lane per (point, input direction), the RK4 step in forward-mode duals
//     (ForwardDiff's algorithm, one partial per lane: exact like ForwardDiff), plus the
//     costs' derivative tiles (:81-109, :134-153) in closed form — the costs are
//     diagonal weighted squares (:85-116);
//   * the Riccati recursion: the wide tiles kernel (ilqr_tiles.hip, nx ≤ 16, nu ≤ 8);
//   * fb_forward_kernel: forward_pass (forward_pass.jl:55-93) — 4 to 64 line-search
//     trials of a trajectory at once, one per lane, each RK4 step split over the four
//     waves of a workgroup, the first accepted trial kept (bit for bit the sequential
//     search's choice: every trial is independent of the others); each
//     trial stores its x̄, ū as it rolls out (trial 1 into x̄, ū, the others into a
//     per-lane slot), so an accepted later trial is taken from its slot, never rolled
//     out again;
//   * fb_update_kernel / fb_take_kernel: fit's bookkeeping (:161-178) and the accepted
//     trial's move into the iterate.
//
// Dynamics (RigidBodyDynamics.jl is absent; restated with Featherstone's algorithms in
// body coordinates, angular first, as tests/closures.py rbd_floating_arm): the base is a
// free body with twist (ω, v) in its own frame; joint i turns child body i about axis aᵢ
// at the origin pᵢ of its parent; M(q) by the composite-rigid-body algorithm, the bias by
// recursive Newton-Euler at q̈ = 0 (zero gravity, as the script parses the URDF);
// q̇ = [pdot_from_w(p, ω); v; θ̇] exactly as RBD_helper_functions.jl:66 writes it.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/ilqr.h"
#include "ilqr_internal.h"

namespace ilqr {
namespace {

constexpr int FB_NJ = 2;             // joints (the reference's arm)
constexpr int FB_NQ = 6 + FB_NJ;     // pose coordinates in the cost: p (3), r (3), θ
constexpr int FB_NX = 2 * FB_NQ;     // 16
constexpr int FB_NU = FB_NQ;         // 8: base torque, base force, joint torques
constexpr int FB_CAND = 4;           // line-search trials per trajectory per round (large batches)

// forward-mode dual with one partial (one input direction per lane)
struct D1 {
  double v, d;
  __device__ D1() = default;
  __device__ constexpr D1(double a) : v(a), d(0.0) {}
  __device__ constexpr D1(double a, double b) : v(a), d(b) {}
};
// The dual operators contract freely across one another once inlined (the file is built
// with -ffp-contract=on, for the double path's sake: fb_rk_next): the linearisation's
// products and sums fuse as they did before (−14 % per launch otherwise).
#define FB_DUAL_CONTRACT _Pragma("clang fp contract(fast)")
__device__ __forceinline__ D1 operator+(D1 a, D1 b) {
  FB_DUAL_CONTRACT
  return D1(a.v + b.v, a.d + b.d);
}
__device__ __forceinline__ D1 operator-(D1 a, D1 b) {
  FB_DUAL_CONTRACT
  return D1(a.v - b.v, a.d - b.d);
}
__device__ __forceinline__ D1 operator-(D1 a) { return D1(-a.v, -a.d); }
__device__ __forceinline__ D1 operator*(D1 a, D1 b) {
  FB_DUAL_CONTRACT
  return D1(a.v * b.v, fma(a.v, b.d, a.d * b.v));
}
__device__ __forceinline__ D1 operator*(double a, D1 b) {
  FB_DUAL_CONTRACT
  return D1(a * b.v, a * b.d);
}
__device__ __forceinline__ D1 operator*(D1 b, double a) {
  FB_DUAL_CONTRACT
  return D1(a * b.v, a * b.d);
}
__device__ __forceinline__ D1 operator/(D1 a, D1 b) {
  FB_DUAL_CONTRACT
  const double q = a.v / b.v;
  return D1(q, (a.d - q * b.d) / b.v);
}
__device__ __forceinline__ void sincos_s(double a, double& s, double& c) { sincos(a, &s, &c); }
__device__ __forceinline__ void sincos_s(D1 a, D1& s, D1& c) {
  FB_DUAL_CONTRACT
  double sv, cv;
  sincos(a.v, &sv, &cv);
  s = D1(sv, a.d * cv);
  c = D1(cv, -a.d * sv);
}

// the model, by value in the kernel arguments (fp64, prepared on the host)
struct FbModel {
  double dt;
  // bodies 0 (base) .. NJ: mass, h = m·c (first moment), Io = inertia about the body origin
  double m[FB_NJ + 1];
  double h[FB_NJ + 1][3];
  double Io[FB_NJ + 1][9];
  // joint i (parent body i → child body i+1): R0 (joint frame → parent), R0·[a×], R0·a·aᵀ,
  // origin p in the parent frame, axis a
  double R0[FB_NJ][9], R0x[FB_NJ][9], R0aa[FB_NJ][9];
  double p[FB_NJ][3], ax[FB_NJ][3];
  // costs (RBD_helper_functions.jl:85-116): ℓ = qs·Σ qwᵢ(tgtᵢ − xᵢ)² + rs·Σ rwⱼ uⱼ²,
  // ℓ_f = qfs·Σ qfwᵢ(tgtᵢ − xᵢ)², and the derivative coefficients −2·qs·qw, 2·qs·qw, …
  double tgt[FB_NQ], qw[FB_NQ], rw[FB_NU], qfw[FB_NQ];
  double qs, rs, qfs;
  double gx[FB_NQ], hx[FB_NQ], gu[FB_NU], hu[FB_NU], gf[FB_NQ], hf[FB_NQ];
};

// joint i's child→parent rotation Rc = R0·Rot(a, θ) = c·(R0 − R0aaᵀ) + s·R0[a×] + R0aaᵀ
template <class S>
__device__ __forceinline__ void joint_rot(const FbModel& P, int i, S c, S s, S (&Rc)[9]) {
#pragma unroll
  for (int k = 0; k < 9; ++k) Rc[k] = c * (P.R0[i][k] - P.R0aa[i][k]) + s * P.R0x[i][k] + P.R0aa[i][k];
}
// Rcᵀ·a (parent → child)
template <class S>
__device__ __forceinline__ void rot_t(const S (&R)[9], const S (&a)[3], S (&o)[3]) {
  o[0] = R[0] * a[0] + R[3] * a[1] + R[6] * a[2];
  o[1] = R[1] * a[0] + R[4] * a[1] + R[7] * a[2];
  o[2] = R[2] * a[0] + R[5] * a[1] + R[8] * a[2];
}
// Rc·a (child → parent)
template <class S>
__device__ __forceinline__ void rot(const S (&R)[9], const S (&a)[3], S (&o)[3]) {
  o[0] = R[0] * a[0] + R[1] * a[1] + R[2] * a[2];
  o[1] = R[3] * a[0] + R[4] * a[1] + R[5] * a[2];
  o[2] = R[6] * a[0] + R[7] * a[1] + R[8] * a[2];
}

// mixed-type helpers: the model's constants stay double (no dual promotion)
template <class S, class A, class B>
__device__ __forceinline__ void crossm(const A (&a)[3], const B (&b)[3], S (&o)[3]) {
  o[0] = a[1] * b[2] - a[2] * b[1];
  o[1] = a[2] * b[0] - a[0] * b[2];
  o[2] = a[0] * b[1] - a[1] * b[0];
}
template <class S, class A>
__device__ __forceinline__ S dotm(const A (&a)[3], const S (&b)[3]) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
}

// continuous dynamics ẋ = [pdot_from_w(p, ω); v; θ̇; M \ (u − bias)] (RBD_helper_functions.jl:50-69),
// in four pieces that fb_xdot composes and the two-wave forward splits between its
// waves (same operations either way, so the same bits):
//   fb_rots   the joints' rotations from θ;
//   fb_bias   the bias (base moment and force, joint torques) by recursive Newton-Euler
//             at q̈ = 0 — independent of u; b = u − bias;
//   fb_mass   M by the composite-rigid-body algorithm kept in blocks — the base's 6×6
//             composite inertia M₀₀, the base-joint columns M₀ⱼ and the joint block Mⱼⱼ —
//             and what M v̇ = b needs of it: M₀₀⁻¹ in closed form (w = I_c⁻¹(n − c × f),
//             v = f/m + c × w, I_c the composite's inertia about its COM c), Y = M₀₀⁻¹M₀ⱼ
//             and the joint block's Schur complement;
//   fb_solve  v̇ from b through that complement, and the kinematics.
// No 8 × 8 matrix is ever held.
template <class S>
__device__ __forceinline__ void fb_rots(const FbModel& P, const S (&x)[FB_NX], S (&R)[FB_NJ][9]) {
#pragma unroll
  for (int i = 0; i < FB_NJ; ++i) {
    S s, c;
    sincos_s(x[6 + i], s, c);
    joint_rot(P, i, c, s, R[i]);
  }
}

// The bias in pieces (the forward splits them over waves; fb_bias composes them — the
// same expressions either way, so the same bits under -ffp-contract=on):
//   fb_outward<N>     the outward pass through joints 0..N−1: bodies 0..N's twists and
//                     velocity-product accelerations;
//   fb_body_force     body i's own force I·a + v ×* (I·v);
//   fb_transmit       across joint i−1: τ_{i−1} and the force in body i−1's frame.
template <class S>
struct FbMotion {
  S vw[FB_NJ + 1][3], vv[FB_NJ + 1][3], aw[FB_NJ + 1][3], av[FB_NJ + 1][3];
};
// outward: v_{i+1} = X v_i + s q̇, a_{i+1} = X a_i + v_{i+1} × (s q̇) (a₀ = 0); reads x[8..15]
template <int NJO, class S>
__device__ __forceinline__ void fb_outward(const FbModel& P, const S (&R)[FB_NJ][9], const S (&x)[FB_NX],
                                           FbMotion<S>& M) {
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    M.vw[0][k] = x[8 + k];
    M.vv[0][k] = x[11 + k];
    M.aw[0][k] = 0.0;
    M.av[0][k] = 0.0;
  }
#pragma unroll
  for (int i = 0; i < NJO; ++i) {
    S pw[3], t[3], sw[3], c1[3], c2[3];
    crossm(P.p[i], M.vw[i], pw);
#pragma unroll
    for (int k = 0; k < 3; ++k) t[k] = M.vv[i][k] - pw[k];
    rot_t(R[i], M.vw[i], M.vw[i + 1]);
    rot_t(R[i], t, M.vv[i + 1]);
    const S qd = x[14 + i];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      sw[k] = P.ax[i][k] * qd;
      M.vw[i + 1][k] = M.vw[i + 1][k] + sw[k];
    }
    if (i == 0) {  // a₀ = 0
#pragma unroll
      for (int k = 0; k < 3; ++k) M.aw[1][k] = M.av[1][k] = 0.0;
    } else {
      crossm(P.p[i], M.aw[i], pw);
#pragma unroll
      for (int k = 0; k < 3; ++k) t[k] = M.av[i][k] - pw[k];
      rot_t(R[i], M.aw[i], M.aw[i + 1]);
      rot_t(R[i], t, M.av[i + 1]);
    }
    crossm(M.vw[i + 1], sw, c1);
    crossm(M.vv[i + 1], sw, c2);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      M.aw[i + 1][k] = M.aw[i + 1][k] + c1[k];
      M.av[i + 1][k] = M.av[i + 1][k] + c2[k];
    }
  }
}
// body i's own force: I·(w, v) = (Io w + h × v, m v − h × w), f = I a + v ×* (I v)
template <class S>
__device__ __forceinline__ void fb_body_force(const FbModel& P, int i, const FbMotion<S>& M, S (&bn)[3],
                                              S (&bf)[3]) {
  S pn[3], pf[3], an[3], af[3], t1[3], t2[3];
  crossm(P.h[i], M.vv[i], t1);
  crossm(P.h[i], M.vw[i], t2);
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    pn[r] = P.Io[i][3 * r] * M.vw[i][0] + P.Io[i][3 * r + 1] * M.vw[i][1] + P.Io[i][3 * r + 2] * M.vw[i][2] + t1[r];
    pf[r] = P.m[i] * M.vv[i][r] - t2[r];
  }
  crossm(P.h[i], M.av[i], t1);
  crossm(P.h[i], M.aw[i], t2);
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    an[r] = P.Io[i][3 * r] * M.aw[i][0] + P.Io[i][3 * r + 1] * M.aw[i][1] + P.Io[i][3 * r + 2] * M.aw[i][2] + t1[r];
    af[r] = P.m[i] * M.av[i][r] - t2[r];
  }
  S c1[3], c2[3], c3[3];
  crossm(M.vw[i], pn, c1);
  crossm(M.vv[i], pf, c2);
  crossm(M.vw[i], pf, c3);
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    bn[k] = an[k] + (c1[k] + c2[k]);
    bf[k] = af[k] + c3[k];
  }
}
// τ_{i−1} and the force across joint i−1 (i > 0): f' = Rc f, n' = Rc n + p × f'
template <class S>
__device__ __forceinline__ void fb_transmit(const FbModel& P, const S (&R)[FB_NJ][9], int i, const S (&bn)[3],
                                            const S (&bf)[3], S& tau, S (&fn)[3], S (&ff)[3]) {
  tau = dotm(P.ax[i - 1], bn);
  S rn[3], pfx[3];
  rot(R[i - 1], bf, ff);
  rot(R[i - 1], bn, rn);
  crossm(P.p[i - 1], ff, pfx);
#pragma unroll
  for (int k = 0; k < 3; ++k) fn[k] = rn[k] + pfx[k];
}

template <class S>
__device__ __forceinline__ void fb_bias(const FbModel& P, const S (&R)[FB_NJ][9], const S (&x)[FB_NX],
                                        S (&q)[FB_NU]) {
  // --- bias, recursive Newton-Euler at q̈ = 0, zero gravity (:65) -----------------------
  FbMotion<S> M;
  fb_outward<FB_NJ>(P, R, x, M);
  // inward: f_i = I_i a_i + v_i ×* (I_i v_i) + X_{i+1}ᵀ f_{i+1}, τ_i = s_iᵀ f_i
  S fn[3], ff[3], tau[FB_NJ];
#pragma unroll
  for (int i = FB_NJ; i >= 0; --i) {
    S bn[3], bf[3];
    fb_body_force(P, i, M, bn, bf);
    if (i < FB_NJ) {
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        bn[k] = bn[k] + fn[k];
        bf[k] = bf[k] + ff[k];
      }
    }
    if (i > 0) {
      fb_transmit(P, R, i, bn, bf, tau[i - 1], fn, ff);
    } else {
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        fn[k] = bn[k];
        ff[k] = bf[k];
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    q[k] = fn[k];
    q[3 + k] = ff[k];
  }
#pragma unroll
  for (int j = 0; j < FB_NJ; ++j) q[6 + j] = tau[j];
}

// M's blocks reduced to what the solve needs (fb_mass → fb_solve)
template <class S>
struct FbSchur {
  S cc[3];                     // the composite's COM c
  double minv;                 // 1 / total mass
  S d0i, d1i, d2i, l10, l20, l21;  // LDLᵀ of I_c
  S Mb[FB_NJ][6];              // base-joint columns M₀ⱼ
  S Y[FB_NJ][6];               // M₀₀⁻¹ M₀ⱼ
  S Sc[FB_NJ][FB_NJ];          // Mⱼⱼ − M₀ⱼᵀ Y
  // M₀₀⁻¹(n, f) = (w, f/m + c × w), w = I_c⁻¹(n − c × f)
  __device__ __forceinline__ void m00inv(const S (&g)[6], S (&o)[6]) const {
    S cf[3], r[3];
    const S fv[3] = {g[3], g[4], g[5]};
    crossm(cc, fv, cf);
#pragma unroll
    for (int k = 0; k < 3; ++k) r[k] = g[k] - cf[k];
    r[1] = r[1] - l10 * r[0];
    r[2] = r[2] - l20 * r[0] - l21 * r[1];
    r[0] = r[0] * d0i;
    r[1] = r[1] * d1i;
    r[2] = r[2] * d2i;
    r[1] = r[1] - l21 * r[2];
    r[0] = r[0] - l10 * r[1] - l20 * r[2];
    S cw[3];
    crossm(cc, r, cw);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      o[k] = r[k];
      o[3 + k] = fv[k] * minv + cw[k];
    }
  }
};

// M in two pieces (the forward's waves hand the first to the second; fb_mass composes them):
//   fb_crba   the composite-rigid-body recursion, tip to base: the base's composite
//             (m, h, Io), the joint block Mⱼⱼ and the base-joint columns M₀ⱼ;
//   fb_schur  M₀₀⁻¹ in closed form, Y = M₀₀⁻¹M₀ⱼ and the joint block's Schur complement.
template <class S>
struct FbCrba {
  S cI[9];
  S ch[3];
  double cm;
  S Mjj[FB_NJ][FB_NJ];
  S Mb[FB_NJ][6];
};
template <class S>
__device__ __forceinline__ void fb_crba(const FbModel& P, const S (&R)[FB_NJ][9], FbCrba<S>& C) {
  // --- M, composite-rigid-body algorithm (:61), tip to base ------------------------------
  // composite of bodies k..NJ in body k's frame: (m, h, Io)
  double cm = P.m[FB_NJ];
  S ch[3], cI[9];
#pragma unroll
  for (int k = 0; k < 3; ++k) ch[k] = P.h[FB_NJ][k];
#pragma unroll
  for (int k = 0; k < 9; ++k) cI[k] = P.Io[FB_NJ][k];
  S Mjj[FB_NJ][FB_NJ];  // joint block
#pragma unroll
  for (int j = FB_NJ - 1; j >= 0; --j) {
    // F = C_{j+1} s_j = (Io a, −h × a) in body j+1's frame; M_jj = aᵀ n
    S n[3], f[3], t[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) n[r] = cI[3 * r] * P.ax[j][0] + cI[3 * r + 1] * P.ax[j][1] + cI[3 * r + 2] * P.ax[j][2];
    crossm(ch, P.ax[j], t);
#pragma unroll
    for (int r = 0; r < 3; ++r) f[r] = -t[r];
    Mjj[j][j] = dotm(P.ax[j], n);
#pragma unroll
    for (int i = j; i >= 0; --i) {  // across joint i into body i: M_{i-1, j} = a_{i-1}ᵀ n
      S rn[3], fo[3], pfx[3];
      rot(R[i], f, fo);
      rot(R[i], n, rn);
      crossm(P.p[i], fo, pfx);
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        n[k] = rn[k] + pfx[k];
        f[k] = fo[k];
      }
      if (i > 0) Mjj[i - 1][j] = Mjj[j][i - 1] = dotm(P.ax[i - 1], n);
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      C.Mb[j][k] = n[k];
      C.Mb[j][3 + k] = f[k];
    }
    // composite of body j: own inertia + the child composite moved across joint j:
    // h' = Rc h, Io' = Rc Io Rcᵀ + m(|p|²1 − p pᵀ) + 2(p·h')1 − p h'ᵀ − h' pᵀ, h'' = h' + m p
    S hp[3], RI[9];
    rot(R[j], ch, hp);
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int k = 0; k < 3; ++k) RI[3 * r + k] = R[j][3 * r] * cI[k] + R[j][3 * r + 1] * cI[3 + k] + R[j][3 * r + 2] * cI[6 + k];
    const double* pj = P.p[j];
    const double pp = pj[0] * pj[0] + pj[1] * pj[1] + pj[2] * pj[2];
    const S ph = dotm(P.p[j], hp);
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int k = r; k < 3; ++k) {
        S e = RI[3 * r] * R[j][3 * k] + RI[3 * r + 1] * R[j][3 * k + 1] + RI[3 * r + 2] * R[j][3 * k + 2];
        e = e - cm * (pj[r] * pj[k]) - pj[r] * hp[k] - hp[r] * pj[k];
        if (r == k) e = e + (cm * pp + 2.0 * ph);
        cI[3 * r + k] = P.Io[j][3 * r + k] + e;
        if (k != r) cI[3 * k + r] = cI[3 * r + k];
      }
#pragma unroll
    for (int k = 0; k < 3; ++k) ch[k] = P.h[j][k] + (hp[k] + cm * pj[k]);
    cm = P.m[j] + cm;
  }
#pragma unroll
  for (int k = 0; k < 9; ++k) C.cI[k] = cI[k];
#pragma unroll
  for (int k = 0; k < 3; ++k) C.ch[k] = ch[k];
  C.cm = cm;
#pragma unroll
  for (int i = 0; i < FB_NJ; ++i)
#pragma unroll
    for (int j = 0; j < FB_NJ; ++j) C.Mjj[i][j] = Mjj[i][j];
}

template <class S>
__device__ __forceinline__ void fb_schur(const FbCrba<S>& C, FbSchur<S>& F) {
  const double cm = C.cm;
#pragma unroll
  for (int j = 0; j < FB_NJ; ++j)
#pragma unroll
    for (int k = 0; k < 6; ++k) F.Mb[j][k] = C.Mb[j][k];
  // --- M₀₀⁻¹ and the Schur complement of M₀₀ ---------------------------------------------
  // M₀₀ = [[Io, [h×]], [[h×]ᵀ, m1]]: with c = h/m and I_c = Io − m(|c|²1 − c cᵀ),
  // M₀₀⁻¹(n, f) = (w, f/m + c × w), w = I_c⁻¹(n − c × f)
  F.minv = 1.0 / cm;
#pragma unroll
  for (int k = 0; k < 3; ++k) F.cc[k] = C.ch[k] * F.minv;
  S Ic[6];  // I_c lower triangle: 00, 10, 11, 20, 21, 22
  {
    const S c2 = dotm(F.cc, F.cc);
    auto ent = [&](int r, int k) { return C.cI[3 * r + k] - cm * ((r == k ? c2 : S(0.0)) - F.cc[r] * F.cc[k]); };
    Ic[0] = ent(0, 0);
    Ic[1] = ent(1, 0);
    Ic[2] = ent(1, 1);
    Ic[3] = ent(2, 0);
    Ic[4] = ent(2, 1);
    Ic[5] = ent(2, 2);
  }
  // LDLᵀ of I_c: l10, l20, l21 and 1/d
  F.d0i = S(1.0) / Ic[0];
  F.l10 = Ic[1] * F.d0i;
  F.l20 = Ic[3] * F.d0i;
  const S d1 = Ic[2] - F.l10 * Ic[1];
  F.d1i = S(1.0) / d1;
  F.l21 = (Ic[4] - F.l20 * Ic[1]) * F.d1i;
  F.d2i = S(1.0) / (Ic[5] - F.l20 * Ic[3] - F.l21 * (F.l21 * d1));
#pragma unroll
  for (int j = 0; j < FB_NJ; ++j) F.m00inv(F.Mb[j], F.Y[j]);
  // the joint block's Schur complement Mⱼⱼ − M₀ⱼᵀ Y (2 × 2)
#pragma unroll
  for (int i = 0; i < FB_NJ; ++i)
#pragma unroll
    for (int j = 0; j < FB_NJ; ++j) {
      S e = C.Mjj[i][j];
#pragma unroll
      for (int k = 0; k < 6; ++k) e = e - F.Mb[i][k] * F.Y[j][k];
      F.Sc[i][j] = e;
    }
}

template <class S>
__device__ __forceinline__ void fb_mass(const FbModel& P, const S (&R)[FB_NJ][9], FbSchur<S>& F) {
  FbCrba<S> C;
  fb_crba(P, R, C);
  fb_schur(C, F);
}


// fb_solve in two pieces (the forward's waves split them; fb_solve composes them):
//   fb_accel  M v̇ = b, the velocities' rates ẋ[8..15];
//   fb_kin    the kinematics ẋ[0..7] from the state alone, no solve.
template <class S>
__device__ __forceinline__ void fb_accel(const FbSchur<S>& F, const S (&b)[FB_NU], S (&xd)[FB_NX]) {
  // --- M v̇ = b: y₀ = M₀₀⁻¹ b₀, then (Mⱼⱼ − M₀ⱼᵀ Y) v̇ⱼ = bⱼ − M₀ⱼᵀ y₀ ------------------------
  S y0[6];
  {
    const S g[6] = {b[0], b[1], b[2], b[3], b[4], b[5]};
    F.m00inv(g, y0);
  }
  S rj[FB_NJ];
#pragma unroll
  for (int i = 0; i < FB_NJ; ++i) {
    S acc = b[6 + i];
#pragma unroll
    for (int k = 0; k < 6; ++k) acc = acc - F.Mb[i][k] * y0[k];
    rj[i] = acc;
  }
  static_assert(FB_NJ == 2, "the joint block's solve is written for two joints");
  const S det = F.Sc[0][0] * F.Sc[1][1] - F.Sc[0][1] * F.Sc[1][0];
  const S q0 = (rj[0] * F.Sc[1][1] - F.Sc[0][1] * rj[1]) / det;
  const S q1 = (F.Sc[0][0] * rj[1] - F.Sc[1][0] * rj[0]) / det;
#pragma unroll
  for (int k = 0; k < 6; ++k) xd[8 + k] = y0[k] - (F.Y[0][k] * q0 + F.Y[1][k] * q1);
  xd[14] = q0;
  xd[15] = q1;
}
template <class S>
__device__ __forceinline__ void fb_kin(const S (&x)[FB_NX], S (&xd)[FB_NX]) {
  // --- kinematics (:66): q̇ = [pdot_from_w(p, ω); v; θ̇] ----------------------------------
  const S pv[3] = {x[0], x[1], x[2]};
  const S w0[3] = {x[8], x[9], x[10]};
  S pxw[3];
  crossm(pv, w0, pxw);
  const S pp = dotm(pv, pv);
  const S pw = dotm(pv, w0);
#pragma unroll
  for (int k = 0; k < 3; ++k) xd[k] = 0.25 * (((1.0 - pp) * w0[k] + 2.0 * pxw[k]) + (2.0 * pw) * pv[k]);
#pragma unroll
  for (int k = 0; k < 3; ++k) xd[3 + k] = x[11 + k];
#pragma unroll
  for (int j = 0; j < FB_NJ; ++j) xd[6 + j] = x[14 + j];
}
template <class S>
__device__ __forceinline__ void fb_solve(const FbSchur<S>& F, const S (&b)[FB_NU], const S (&x)[FB_NX],
                                         S (&xd)[FB_NX]) {
  fb_accel(F, b, xd);
  fb_kin(x, xd);
}

template <class S>
__device__ void fb_xdot(const FbModel& P, const S (&x)[FB_NX], const S (&u)[FB_NU], S (&xd)[FB_NX]) {
  S R[FB_NJ][9];
  fb_rots(P, x, R);
  S b[FB_NU];
  fb_bias(P, R, x, b);
#pragma unroll
  for (int k = 0; k < FB_NU; ++k) b[k] = u[k] - b[k];
  FbSchur<S> F;
  fb_mass(P, R, F);
  fb_solve(F, b, x, xd);
}

// dynamicsf: RK4 of fb_xdot (RBD_helper_functions.jl:71-78): kᵢ = Δt·f(·),
// x + (1/6)·(((k₁ + 2k₂) + 2k₃) + k₄); the stages as a loop (one copy of the dynamics)
template <class S>
__device__ void fb_step(const FbModel& P, const S (&x)[FB_NX], const S (&u)[FB_NU], S (&xo)[FB_NX]) {
  S k[FB_NX], acc[FB_NX], xs[FB_NX];
#pragma unroll
  for (int i = 0; i < FB_NX; ++i) xs[i] = x[i];
#pragma unroll 1
  for (int st = 0; st < 4; ++st) {
    // the model's constants are re-read (scalar loads) in every stage instead of being
    // hoisted into ~200 vector registers
    asm volatile("" ::: "memory");
    fb_xdot(P, xs, u, k);
    const double w = (st == 0 || st == 3) ? 1.0 : 2.0;
    const double c = st == 2 ? 1.0 : 0.5;
#pragma unroll
    for (int i = 0; i < FB_NX; ++i) {
      k[i] = P.dt * k[i];
      acc[i] = st == 0 ? k[i] : acc[i] + w * k[i];
      xs[i] = x[i] + k[i] * c;
    }
  }
#pragma unroll
  for (int i = 0; i < FB_NX; ++i) xo[i] = x[i] + (1.0 / 6.0) * acc[i];
}

// ℓ(x − x_traj, u) and ℓ_f(x) (RBD_helper_functions.jl:85-116): the weighted squares summed
// as numpy sums eight terms (((0+1)+(2+3))+((4+5)+(6+7))), then scaled
__device__ __forceinline__ double sum8(const double (&t)[8]) {
  return ((t[0] + t[1]) + (t[2] + t[3])) + ((t[4] + t[5]) + (t[6] + t[7]));
}
__device__ __forceinline__ double stage_cost(const FbModel& P, const double (&e)[FB_NQ], const double (&u)[FB_NU]) {
  double a[8], b[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const double d = P.tgt[i] - e[i];
    a[i] = (d * P.qw[i]) * d;
    b[i] = (u[i] * P.rw[i]) * u[i];
  }
  return sum8(a) * P.qs + sum8(b) * P.rs;
}
__device__ __forceinline__ double final_cost(const FbModel& P, const double (&x)[FB_NX]) {
  double a[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const double d = P.tgt[i] - x[i];
    a[i] = (d * P.qfw[i]) * d;
  }
  return sum8(a) * P.qfs;
}

__global__ __launch_bounds__(256) void fb_dynamics_kernel(const FbModel* __restrict__ Pm, int n, const double* __restrict__ x,
                                                          const double* __restrict__ u, double* __restrict__ xo) {
  const FbModel& P = *Pm;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double xs[FB_NX], us[FB_NU], y[FB_NX];
#pragma unroll
  for (int k = 0; k < FB_NX; ++k) xs[k] = x[(size_t)i * FB_NX + k];
#pragma unroll
  for (int k = 0; k < FB_NU; ++k) us[k] = u[(size_t)i * FB_NU + k];
  fb_step(P, xs, us, y);
#pragma unroll
  for (int k = 0; k < FB_NX; ++k) xo[(size_t)i * FB_NX + k] = y[k];
}

// Derivative tiles at every (b, t): lane (point, dir) seeds input direction dir (x 0..15,
// u 16..23) and writes column dir of A or B; lane dir = 0 also writes the cost tiles, and
// the final point's lane the terminal ones. Trajectories whose status is set are skipped.
// The base position r = x[3..5] enters neither ẋ (:66: ṙ = v) nor anything else (the
// family has no gravity), so its three columns of A are the unit columns the dual
// rollout would return for finite inputs; lane dir = 0 writes them and no lane seeds r:
// FB_LIN_DIRS lanes per point.
constexpr int FB_LIN_DIRS = FB_NX + FB_NU - 3;
__global__ __launch_bounds__(256) void fb_linearize_kernel(const FbModel* __restrict__ Pm, int B, int T, const double* __restrict__ x,
                                                           const double* __restrict__ u,
                                                           const int32_t* __restrict__ status,
                                                           double* __restrict__ A, double* __restrict__ Bm,
                                                           double* __restrict__ lx, double* __restrict__ lu,
                                                           double* __restrict__ lxx, double* __restrict__ luu,
                                                           double* __restrict__ lfx, double* __restrict__ lfxx) {
  constexpr int ND = FB_LIN_DIRS;
  const FbModel& P = *Pm;
  const size_t lane = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (lane >= (size_t)B * T * ND) return;
  const int ld = (int)(lane % ND);
  const int dir = ld < 3 ? ld : ld + 3;  // directions 3..5 (r) are not seeded
  const size_t pt = lane / ND;  // b·T + t
  const int b = (int)(pt / T);
  const int t = (int)(pt % T);
  if (status && status[b] != ILQR_TRAJ_OK) return;
  const double* xp = x + ((size_t)b * (T + 1) + t) * FB_NX;
  const double* up = u + pt * FB_NU;
  D1 xs[FB_NX], us[FB_NU], y[FB_NX];
#pragma unroll
  for (int k = 0; k < FB_NX; ++k) xs[k] = D1(xp[k], k == dir ? 1.0 : 0.0);
#pragma unroll
  for (int k = 0; k < FB_NU; ++k) us[k] = D1(up[k], k + FB_NX == dir ? 1.0 : 0.0);
  fb_step(P, xs, us, y);
  if (dir < FB_NX) {
#pragma unroll
    for (int i = 0; i < FB_NX; ++i) A[(pt * FB_NX + i) * FB_NX + dir] = y[i].d;
  } else {
#pragma unroll
    for (int i = 0; i < FB_NX; ++i) Bm[(pt * FB_NX + i) * FB_NU + (dir - FB_NX)] = y[i].d;
  }
  if (dir != 0) return;
#pragma unroll
  for (int i = 0; i < FB_NX; ++i)
#pragma unroll
    for (int c = 3; c < 6; ++c) A[(pt * FB_NX + i) * FB_NX + c] = i == c ? 1.0 : 0.0;
  // cost tiles (:95-99): lx = −2qs·qw·(tgt − x), lxx = diag(2qs·qw), lu = 2rs·rw·u, luu = diag(2rs·rw)
  for (int i = 0; i < FB_NX; ++i) {
    lx[pt * FB_NX + i] = i < FB_NQ ? P.gx[i] * (P.tgt[i] - xp[i]) : 0.0;
    for (int k = 0; k < FB_NX; ++k) lxx[(pt * FB_NX + i) * FB_NX + k] = (i == k && i < FB_NQ) ? P.hx[i] : 0.0;
  }
  for (int j = 0; j < FB_NU; ++j) {
    lu[pt * FB_NU + j] = P.gu[j] * up[j];
    for (int k = 0; k < FB_NU; ++k) luu[(pt * FB_NU + j) * FB_NU + k] = j == k ? P.hu[j] : 0.0;
  }
  if (t == T - 1) {  // (:142-143) at x_N
    const double* xN = x + ((size_t)b * (T + 1) + T) * FB_NX;
    for (int i = 0; i < FB_NX; ++i) {
      lfx[(size_t)b * FB_NX + i] = i < FB_NQ ? P.gf[i] * (P.tgt[i] - xN[i]) : 0.0;
      for (int k = 0; k < FB_NX; ++k)
        lfxx[((size_t)b * FB_NX + i) * FB_NX + k] = (i == k && i < FB_NQ) ? P.hf[i] : 0.0;
    }
  }
}

struct FbFwd {
  const double* x;
  const double* u;
  const double* xtraj;  // nullable
  const double* d;
  const double* K;
  const double* prev_cost;
  double* xn;
  double* un;
  double* new_cost;
  double* du2;
  int32_t* trials;
  int32_t* fstatus;        // out: 0 accepted, LS_EXHAUSTED, NAN
  const int32_t* status;   // in: trajectories with a set status are skipped (nullable)
  double* slots;           // (B, cand, (T+1)·nx + T·nu): trials j > 1, slot (j − 1) mod cand
  double alpha0, shrink;
  int max_trials;
};

// One trial's rollout (forward_pass.jl:65-76) → cost, Σ(ū − u)², and whether every
// ū = u + α·δu equals u (then every later, smaller α rolls out the same); stores x̄
// into xn, ū into un as it goes.
//
// The two-barrier rollout (ILQR_FB_LOOKAHEAD=0, rounds 5-6; the pipelined one below is the
// product) runs on three waves (fb_forward_kernel): a workgroup of three waves holds the same
// 64 (trajectory, trial) lanes and splits each step between them —
//   wave 0 (mass):    the mass blocks and their factors (fb_mass) of every RK4 stage, from
//                     the stage's joint angles;
//   wave 1 (main):    the bias of every stage (fb_bias: independent of u), then
//                     b = ū − bias, the solve and the stage update (fb_solve), storing x̄;
//   wave 2 (control): the step's ūₜ = uₜ + α·δuₜ + Kₜ(x̄ₜ − xₜ), its cost and Σ(ū − u)²,
//                     storing ū — beside stage 1's mass and bias.
// Per stage waves 0 and 2 hand the factors and ū to wave 1 through LDS, and wave 1 hands
// back the next stage's angles (the next step's state at the last stage), between two
// workgroup barriers. One wave alone issues a VALU instruction every 4 cycles at best,
// so a lane's step (≈7,800 instructions on one wave) is bound by its wave's issue; the
// three waves issue side by side. Same operations as fb_step: the same bits.
constexpr int FB_SCHUR_N = (int)(sizeof(FbSchur<double>) / sizeof(double));
static_assert(sizeof(FbSchur<double>) == FB_SCHUR_N * sizeof(double), "FbSchur<double> is doubles only");
constexpr int FB_CRBA_N = (int)(sizeof(FbCrba<double>) / sizeof(double));
static_assert(sizeof(FbCrba<double>) == FB_CRBA_N * sizeof(double), "FbCrba<double> is doubles only");
#ifndef ILQR_FB_LOOKAHEAD
#define ILQR_FB_LOOKAHEAD 1
#endif
#if !ILQR_FB_LOOKAHEAD
constexpr int FB_XU = FB_SCHUR_N;            // ū (8)
constexpr int FB_XX = FB_SCHUR_N + FB_NU;    // the stage's state (angles; all 16 at a step's end)
struct FbXch {
  double v[FB_XX + FB_NX][64];  // value-major: lane l's k-th value at v[k][l]
};
#endif
constexpr int FB_FWD_WAVES = ILQR_FB_LOOKAHEAD ? 4 : 3;

// every wave reaches it: its LDS writes done (lgkmcnt only — the rollout's global stores
// stay in flight), then the workgroup barrier
__device__ __forceinline__ void fb_lds_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt((15) | (7 << 4) | (0 << 8) | (3 << 14));
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Trace build (ILQR_FB_TRACE, never the product): per role, the ticks of the 100 MHz
// counter each wave of workgroup 0 spends working between barriers, waiting at them and
// polling its sequence words, summed over rollouts (ilqr_debug_fb_trace).
#ifdef ILQR_FB_TRACE
__device__ unsigned long long g_fbt[4][8];
#define FBT_DECL uint64_t fbt_prev = __builtin_amdgcn_s_memrealtime(), fbt_work = 0, fbt_wait = 0, fbt_poll = 0, fbt_n = 0, fbt_mark = fbt_prev, fbt_sub[4] = {0, 0, 0, 0};
#define FBT_BAR()                                           \
  do {                                                      \
    const uint64_t a_ = __builtin_amdgcn_s_memrealtime();   \
    fb_lds_barrier();                                       \
    const uint64_t b_ = __builtin_amdgcn_s_memrealtime();   \
    fbt_work += a_ - fbt_prev;                              \
    fbt_wait += b_ - a_;                                    \
    fbt_prev = fbt_mark = b_;                               \
    ++fbt_n;                                                \
  } while (0)
#define FBT_POLL_BEGIN const uint64_t p0_ = __builtin_amdgcn_s_memrealtime();
#define FBT_POLL_END fbt_poll += __builtin_amdgcn_s_memrealtime() - p0_;
// phase k's end (k < 4): the doubles of v computed before the mark (sub-phase ticks)
#define FBT_MARK(k, v)                                                               \
  do {                                                                               \
    const double* m_ = reinterpret_cast<const double*>(&(v));                       \
    for (int i_ = 0; i_ < (int)(sizeof(v) / sizeof(double)); ++i_) asm volatile("" ::"v"(m_[i_])); \
    const uint64_t t_ = __builtin_amdgcn_s_memrealtime();                            \
    fbt_sub[k] += t_ - fbt_mark;                                                     \
    fbt_mark = t_;                                                                   \
  } while (0)
#define FBT_FLUSH                                           \
  if (blockIdx.x == 0 && lane == 0) {                       \
    atomicAdd(&g_fbt[role][0], (unsigned long long)fbt_work); \
    atomicAdd(&g_fbt[role][1], (unsigned long long)fbt_wait); \
    atomicAdd(&g_fbt[role][2], (unsigned long long)fbt_poll); \
    atomicAdd(&g_fbt[role][3], (unsigned long long)fbt_n);    \
    for (int k_ = 0; k_ < 4; ++k_) atomicAdd(&g_fbt[role][4 + k_], (unsigned long long)fbt_sub[k_]); \
  }
#else
#define FBT_DECL
#define FBT_BAR() fb_lds_barrier()
#define FBT_POLL_BEGIN
#define FBT_POLL_END
#define FBT_MARK(k, v)
#define FBT_FLUSH
#endif

#if ILQR_FB_LOOKAHEAD
// LDS writes done (lgkmcnt only), no barrier
__device__ __forceinline__ void fb_lds_wait() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt((15) | (7 << 4) | (0 << 8) | (3 << 14));
  asm volatile("" ::: "memory");
}

// RK4's bookkeeping of one component at stage st (fb_step's loop body, the same
// expressions): k = Δt·ẋ, the sum k₁ + 2k₂ + 2k₃ + k₄ and the next stage's value (the
// step's result at st = 3). Waves 0, 1 and 3 of fb_rollout3 all run it on the joint
// angles and must agree to the bit (the rotations of waves 0 and 3 are the stored
// angles'): this file is built with -ffp-contract=on, so an FMA forms within one
// expression only, never by the surrounding code.
__device__ __forceinline__ double fb_rk_next(int st, double dt, double xd, double xb, double& acc) {
  const double k = dt * xd;
  const double w = (st == 0 || st == 3) ? 1.0 : 2.0;
  const double c = st == 2 ? 1.0 : 0.5;
  acc = st == 0 ? k : acc + w * k;
  return st < 3 ? xb + k * c : xb + (1.0 / 6.0) * acc;
}

// Four waves pipelined by one RK4 stage. A stage's mass blocks depend on its joint
// angles only, and the angles of stage s + 1 on stage s's state alone — θ̇ enters
// q̇ = [·; ·; θ̇] as it is (fb_solve's kinematics), the solve only moves the velocities —
// so waves 0 and 3 compute stage s + 1's rotations and mass while wave 1 works on stage s:
//   wave 0 (mass):    from stage s's θ̇ (and its own running RK4 sum of the angle) joint
//                     1's angle of stage s + 1 and its rotation, then (joint 0's from wave
//                     3, behind a per-lane sequence word) the CRBA (fb_crba), into buffer
//                     (s + 1) & 1;
//   wave 3 (joint 0): the same for joint 0's angle and rotation; then stage s's factors
//                     (fb_schur of wave 0's CRBA of the stage before), to wave 1 behind a
//                     second sequence word, and the kinematics: stage s + 1's positions
//                     and angles from stage s's (fb_kin + RK4; the step's state at its end);
//   wave 1 (main):    stage s's bias from its velocities and the rotations of buffer s & 1,
//                     b = ū − bias, the solve for the velocities' rates (fb_accel) with the
//                     factors and their stage update; stage s + 1's velocities into the
//                     state buffer (s + 1) & 1;
//   wave 2 (control): at a step's start, ūₜ from x̄ₜ, its cost and Σ(ū − u)², storing ū,
//                     and ūₜ to wave 1 through LDS behind a per-lane sequence word (wave 1
//                     waits on it once a step, after its bias — ūₜ is in by then).
// One workgroup barrier a stage (stage s's inputs ready); a buffer a wave reads behind a
// barrier is written by the others in the stage before, one behind a sequence word in
// the same stage. The split follows tools/fb_trace.py's per-wave ticks: with fb_mass
// and the kinematics on waves 0 and 1 (round 6's first pipeline) wave 0's rotation +
// mass took ≈ 1.90 µs a stage and wave 1's bias + solve + update 1.81 µs, while wave 3
// idled 1.27 µs of its 1.93. The one-stage-per-two-barriers rollout
// (ILQR_FB_LOOKAHEAD=0) ran the rotations + bias beside the rotations + mass, then the
// solve. Same operations, and the file built with -ffp-contract=on: the same bits
// (DESIGN.md §4).
constexpr int FB_IN_N = FB_NU * FB_NX + 2 * FB_NU + 2 * FB_NX;  // a step's K, u, δu, x, x_traj
constexpr int FB_IN_S = FB_IN_N + 2;  // row stride: 16 rows' same element in distinct bank pairs
template <int CAND>
__device__ double fb_rollout3(const FbModel& P, const FbFwd& a, int b, int T, double alpha, double* __restrict__ xn,
                              double* __restrict__ un, double& du2, bool& same, int role, int lane, bool run) {
  struct Pipe {
    double in[64 / CAND][FB_IN_S];  // wave 2's copy of its trajectories' step inputs
    double C[2][FB_CRBA_N][64];    // value-major: lane l's k-th value at [k][l]
    double F[FB_SCHUR_N][64];      // wave 1's stage's factors
    double R[2][FB_NJ * 9][64];
    double xs[2][FB_NX][64];       // velocities (8-15) every stage; all 16 at a step's start
    double u[FB_NU][64];
    int32_t useq[64];              // t + 1 once ūₜ is in u
    int32_t fseq[64];              // s + 1 once stage s's factors are in F (wave 3 → wave 1)
    int32_t pseq[64];              // t once x̄ₜ's positions and angles are in xs (wave 3 → 2)
    double out[3][64];
  };
  __shared__ Pipe X;  // named here: see the exchange of the two-barrier rollout below
  FBT_DECL
  const double* x = a.x + (size_t)b * (T + 1) * FB_NX;
  const int S = 4 * T;
  // the hand-off words start at 0 (the words of the previous rollout, or garbage at the
  // kernel's start, are behind this barrier)
  if (role == 3) {
    __hip_atomic_store(&X.fseq[lane], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __hip_atomic_store(&X.pseq[lane], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  FBT_BAR();
  if (role == 0) {  // mass: the joints' angles and rotations, the CRBA — one stage ahead
    double th[FB_NJ], xb[FB_NJ], acc[FB_NJ];
#pragma unroll
    for (int q = 0; q < FB_NJ; ++q) th[q] = xb[q] = x[6 + q];
    for (int s = 0; s <= S; ++s) {
      if (s > 0) {  // stage s's angles from stage s − 1's θ̇
        const int st = (s - 1) & 3;
#pragma unroll
        for (int q = 0; q < FB_NJ; ++q) {
          th[q] = fb_rk_next(st, P.dt, X.xs[(s - 1) & 1][14 + q][lane], xb[q], acc[q]);
          if (st == 3) xb[q] = th[q];
        }
      }
      if (s < S) {
        asm volatile("" ::: "memory");  // the model's constants re-read per stage (fb_step)
        double xa[FB_NX], R[FB_NJ][9];
#pragma unroll
        for (int q = 0; q < FB_NJ; ++q) xa[6 + q] = th[q];
        fb_rots(P, xa, R);  // reads the angles only
#pragma unroll
        for (int k = 0; k < FB_NJ * 9; ++k) X.R[s & 1][k][lane] = R[k / 9][k % 9];
        FBT_MARK(0, R);
        FbCrba<double> C;  // fb_mass's first piece (wave 3 runs the second)
        fb_crba(P, R, C);
        const double* c = reinterpret_cast<const double*>(&C);
#pragma unroll
        for (int k = 0; k < FB_CRBA_N; ++k) X.C[s & 1][k][lane] = c[k];
        FBT_MARK(1, C);
      }
      FBT_BAR();  // stage s's inputs ready
    }
  } else if (role == 3) {
    // the factors of stage s − 1 (fb_schur of wave 0's CRBA, to wave 1 behind a sequence
    // word), then the kinematics: the positions and angles of stage s from stage s − 1's
    // velocities (the step's state at its end)
    double th[FB_NJ], xb[FB_NJ], acc[FB_NJ];
#pragma unroll
    for (int q = 0; q < FB_NJ; ++q) th[q] = xb[q] = x[6 + q];
    double pos[6], pb[6], pacc[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) pos[k] = pb[k] = x[k];
    FBT_BAR();  // stage 0's rotations and CRBA ready
    for (int s = 1; s <= S; ++s) {
      const int st = (s - 1) & 3;
      asm volatile("" ::: "memory");  // the model's constants re-read per stage (fb_step)
      {
        FbCrba<double> C;
        double* c = reinterpret_cast<double*>(&C);
#pragma unroll
        for (int k = 0; k < FB_CRBA_N; ++k) c[k] = X.C[(s - 1) & 1][k][lane];
        FbSchur<double> F;
        fb_schur(C, F);
        const double* f = reinterpret_cast<const double*>(&F);
#pragma unroll
        for (int k = 0; k < FB_SCHUR_N; ++k) X.F[k][lane] = f[k];
        fb_lds_wait();  // the factors written before their sequence word
        __hip_atomic_store(&X.fseq[lane], s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        FBT_MARK(0, F);
      }
      double xv[FB_NX], xd[FB_NX];
#pragma unroll
      for (int k = 0; k < 6; ++k) xv[k] = pos[k];
      xv[6] = xv[7] = 0.0;  // not read by fb_kin
#pragma unroll
      for (int k = 8; k < FB_NX; ++k) xv[k] = X.xs[(s - 1) & 1][k][lane];
      fb_kin(xv, xd);
#pragma unroll
      for (int k = 0; k < 6; ++k) pos[k] = fb_rk_next(st, P.dt, xd[k], pb[k], pacc[k]);
#pragma unroll
      for (int q = 0; q < FB_NJ; ++q) th[q] = fb_rk_next(st, P.dt, xv[14 + q], xb[q], acc[q]);
      if (st == 3) {  // the step's end: x_{t+1}'s positions and angles
        double* xo = xn + (size_t)(s >> 2) * FB_NX;
#pragma unroll
        for (int k = 0; k < 6; ++k) {
          pb[k] = pos[k];
          X.xs[0][k][lane] = pos[k];
          if (run) xo[k] = pos[k];
        }
#pragma unroll
        for (int q = 0; q < FB_NJ; ++q) {
          xb[q] = th[q];
          X.xs[0][6 + q][lane] = th[q];
          if (run) xo[6 + q] = th[q];
        }
        fb_lds_wait();  // written before their sequence word
        __hip_atomic_store(&X.pseq[lane], s >> 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      FBT_MARK(1, pos);
      FBT_BAR();  // stage s − 1's factors ready
    }
  } else if (role == 2) {  // control: ūₜ (:72-73), its cost (:187-190), Σ(ū − u)²
    const double* u = a.u + (size_t)b * T * FB_NU;
    const double* xt = a.xtraj ? a.xtraj + (size_t)b * (T + 1) * FB_NX : nullptr;
    const double* d = a.d + (size_t)b * T * FB_NU;
    const double* K = a.K + (size_t)b * T * FB_NU * FB_NX;
    // step tn's K, u, δu, x, x_traj of this lane's trajectory into its row of X.in, the
    // trajectory's CAND lanes a share each — one stage after ūₜ₋₁, so that ūₜ reads LDS
    // only: wave 1 needs it right after its bias, about 2,000 cycles after x̄ₜ is known,
    // and a step's loads from beyond L2 (the batch's K: 1 MB a trajectory at T = 1000)
    // took longer
    constexpr int NK = FB_NU * FB_NX, PER = (FB_IN_N + CAND - 1) / CAND;
    const int c = lane % CAND;
    double* row = X.in[lane / CAND];
    auto stage_in = [&](size_t tn) {
      double v[PER];
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const int e = c + i * CAND;
        double w = 0.0;
        if (e < NK)
          w = K[tn * NK + e];
        else if (e < NK + FB_NU)
          w = u[tn * FB_NU + (e - NK)];
        else if (e < NK + 2 * FB_NU)
          w = d[tn * FB_NU + (e - NK - FB_NU)];
        else if (e < NK + 2 * FB_NU + FB_NX)
          w = x[tn * FB_NX + (e - NK - 2 * FB_NU)];
        else if (e < FB_IN_N && xt)
          w = xt[tn * FB_NX + (e - NK - 2 * FB_NU - FB_NX)];
        v[i] = w;
      }
#pragma unroll
      for (int i = 0; i < PER; ++i)
        if (c + i * CAND < FB_IN_N) row[c + i * CAND] = v[i];
    };
    const double* rK = row;
    const double* ru = row + NK;
    const double* rd = ru + FB_NU;
    const double* rx = rd + FB_NU;
    const double* rxt = rx + FB_NX;
    double xb[FB_NX];
    double cost = 0.0, s2 = 0.0;
    bool eq = true;
    // Kₜ(x̄ₜ − xₜ): each row's sum in k order, the eight rows side by side. Its first half
    // (k < 8: the positions and angles, wave 3's, known mid-way through the step's last
    // stage) runs in that stage; after the barrier only the velocities' half is left
    double kd[FB_NU];
    auto kd_lo = [&]() {
#pragma unroll
      for (int j = 0; j < FB_NU; ++j) kd[j] = 0.0;
#pragma unroll
      for (int k = 0; k < FB_NX / 2; ++k) {
        const double dxk = X.xs[0][k][lane] - rx[k];
#pragma unroll
        for (int j = 0; j < FB_NU; ++j) kd[j] = fma(rK[j * FB_NX + k], dxk, kd[j]);
      }
    };
    __hip_atomic_store(&X.useq[lane], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    stage_in(0);
    FBT_BAR();
    kd_lo();
    for (int t = 0; t < T; ++t) {
#pragma unroll
      for (int k = 0; k < FB_NX; ++k) xb[k] = X.xs[0][k][lane];  // x̄ₜ (x̄₁ = x₁, :65)
      double ub[FB_NU];
#pragma unroll
      for (int k = FB_NX / 2; k < FB_NX; ++k) {
        const double dxk = xb[k] - rx[k];
#pragma unroll
        for (int j = 0; j < FB_NU; ++j) kd[j] = fma(rK[j * FB_NX + k], dxk, kd[j]);
      }
#pragma unroll
      for (int j = 0; j < FB_NU; ++j) {
        const double uj = ru[j];
        const double ua = uj + alpha * rd[j];
        eq = eq && ua == uj;
        ub[j] = ua + kd[j];
        const double e = ub[j] - uj;
        s2 = fma(e, e, s2);
      }
      // ūₜ to wave 1 after every read of the row (a store between them would order the
      // reads one row of K at a time)
#pragma unroll
      for (int j = 0; j < FB_NU; ++j) X.u[j][lane] = ub[j];
      fb_lds_wait();  // ūₜ written before its sequence word
      __hip_atomic_store(&X.useq[lane], t + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      FBT_MARK(0, ub);
#pragma unroll
      for (int j = 0; j < FB_NU; ++j)
        if (run) un[(size_t)t * FB_NU + j] = ub[j];
      double ev[FB_NQ];
#pragma unroll
      for (int k = 0; k < FB_NQ; ++k) ev[k] = xt ? xb[k] - rxt[k] : xb[k];
      cost = cost + stage_cost(P, ev, ub);
      FBT_MARK(1, cost);
      FBT_BAR();
      if (t + 1 < T) stage_in((size_t)(t + 1));
      FBT_MARK(2, cost);
      FBT_BAR();
      FBT_BAR();
      if (t + 1 < T) {  // x̄ₜ₊₁'s first half from wave 3, then its part of Kₜ₊₁(x̄ₜ₊₁ − xₜ₊₁)
        while (__hip_atomic_load(&X.pseq[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != t + 1)
          __builtin_amdgcn_s_sleep(1);
        asm volatile("" ::: "memory");
        kd_lo();
        FBT_MARK(3, kd);
      }
      FBT_BAR();
    }
#pragma unroll
    for (int k = 0; k < FB_NX; ++k) xb[k] = X.xs[0][k][lane];  // x̄_N
    cost = cost + final_cost(P, xb);  // :192 (raw x̄_N)
    X.out[0][lane] = cost;  // the outcome to waves 0 and 1
    X.out[1][lane] = s2;
    X.out[2][lane] = eq ? 1.0 : 0.0;
  } else {  // main: bias, solve, the velocities' stage update
    double xb[FB_NX], xs[FB_NX], acc[FB_NX], ub[FB_NU];
#pragma unroll
    for (int k = 0; k < FB_NX; ++k) {
      xb[k] = x[k];
      xs[k] = xb[k];
      if (run) xn[k] = xb[k];
      X.xs[0][k][lane] = xb[k];
    }
    FBT_BAR();
    for (int s = 0; s < S; ++s) {
      const int t = s >> 2, st = s & 3;
      asm volatile("" ::: "memory");
      double R[FB_NJ][9];
#pragma unroll
      for (int i = 0; i < FB_NJ; ++i)
#pragma unroll
        for (int k = 0; k < 9; ++k) R[i][k] = X.R[s & 1][9 * i + k][lane];
      double bb[FB_NU];
      fb_bias(P, R, xs, bb);
      FBT_MARK(0, bb);
      // the bias before the waits (else the compiler sinks it behind them)
#pragma unroll
      for (int j = 0; j < FB_NU; ++j) asm volatile("" ::"v"(bb[j]));
      FBT_POLL_BEGIN
      if (st == 0)
        while (__hip_atomic_load(&X.useq[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != t + 1)
          __builtin_amdgcn_s_sleep(1);
      FBT_MARK(3, bb);
      while (__hip_atomic_load(&X.fseq[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != s + 1)
        __builtin_amdgcn_s_sleep(1);
      FBT_POLL_END
      asm volatile("" ::: "memory");
      if (st == 0) {
#pragma unroll
        for (int j = 0; j < FB_NU; ++j) ub[j] = X.u[j][lane];
      }
#pragma unroll
      for (int j = 0; j < FB_NU; ++j) bb[j] = ub[j] - bb[j];
      FbSchur<double> F;
      double* f = reinterpret_cast<double*>(&F);
#pragma unroll
      for (int k = 0; k < FB_SCHUR_N; ++k) f[k] = X.F[k][lane];
      double k[FB_NX];
      fb_accel(F, bb, k);
      FBT_MARK(1, k);
      // the velocities (wave 3 keeps the positions and angles)
#pragma unroll
      for (int i = 8; i < FB_NX; ++i) {
        xs[i] = fb_rk_next(st, P.dt, k[i], xb[i], acc[i]);
        X.xs[(s + 1) & 1][i][lane] = xs[i];
      }
      if (st == 3) {
#pragma unroll
        for (int i = 8; i < FB_NX; ++i) {
          xb[i] = xs[i];
          if (run) xn[(size_t)(t + 1) * FB_NX + i] = xs[i];
        }
      }
      FBT_MARK(2, xs);
      FBT_BAR();  // stage s + 1's velocities ready
    }
  }
  FBT_BAR();
  const double cost = X.out[0][lane];
  du2 = X.out[1][lane];
  same = X.out[2][lane] != 0.0;
  FBT_BAR();  // read before the next rollout writes
  FBT_FLUSH
  return cost;
}
#else
template <int CAND>
__device__ double fb_rollout3(const FbModel& P, const FbFwd& a, int b, int T, double alpha, double* __restrict__ xn,
                              double* __restrict__ un, double& du2, bool& same, int role, int lane, bool run) {
  // the workgroup's exchange, named here rather than passed by reference: through a
  // reference the compiler lost its address space in some instantiations and read it
  // with flat loads, whose waits cover the global loads in flight too
  __shared__ FbXch X;
  const double* x = a.x + (size_t)b * (T + 1) * FB_NX;
  if (role == 0) {  // mass: angles in, factors out, four times a step
    double th[FB_NX];  // only th[6], th[7] (the joint angles) are read by fb_rots
#pragma unroll
    for (int k = 0; k < FB_NX; ++k) th[k] = k == 6 || k == 7 ? x[k] : 0.0;
    for (int t = 0; t < T; ++t) {
#pragma unroll 1
      for (int st = 0; st < 4; ++st) {
        asm volatile("" ::: "memory");  // the model's constants re-read per stage (fb_step)
        double R[FB_NJ][9];
        fb_rots(P, th, R);
        FbSchur<double> F;
        fb_mass(P, R, F);
        const double* f = reinterpret_cast<const double*>(&F);
#pragma unroll
        for (int k = 0; k < FB_SCHUR_N; ++k) X.v[k][lane] = f[k];
        fb_lds_barrier();
        fb_lds_barrier();
        th[6] = X.v[FB_XX + 6][lane];
        th[7] = X.v[FB_XX + 7][lane];
      }
    }
  } else if (role == 2) {  // control: ūₜ (:72-73), its cost (:187-190), Σ(ū − u)²
    const double* u = a.u + (size_t)b * T * FB_NU;
    const double* xt = a.xtraj ? a.xtraj + (size_t)b * (T + 1) * FB_NX : nullptr;
    const double* d = a.d + (size_t)b * T * FB_NU;
    const double* K = a.K + (size_t)b * T * FB_NU * FB_NX;
    double xb[FB_NX];
#pragma unroll
    for (int k = 0; k < FB_NX; ++k) xb[k] = x[k];  // x̄₁ = x₁ (:65)
    double cost = 0.0, s2 = 0.0;
    bool eq = true;
    for (int t = 0; t < T; ++t) {
      double dx[FB_NX], ub[FB_NU];
#pragma unroll
      for (int k = 0; k < FB_NX; ++k) dx[k] = xb[k] - x[(size_t)t * FB_NX + k];
#pragma unroll
      for (int j = 0; j < FB_NU; ++j) {
        const double uj = u[(size_t)t * FB_NU + j];
        const double ua = uj + alpha * d[(size_t)t * FB_NU + j];
        eq = eq && ua == uj;
        double kd = 0.0;
#pragma unroll
        for (int k = 0; k < FB_NX; ++k) kd = fma(K[((size_t)t * FB_NU + j) * FB_NX + k], dx[k], kd);
        ub[j] = ua + kd;
        X.v[FB_XU + j][lane] = ub[j];
        const double e = ub[j] - uj;
        s2 = fma(e, e, s2);
      }
#pragma unroll
      for (int j = 0; j < FB_NU; ++j)
        if (run) un[(size_t)t * FB_NU + j] = ub[j];
      double ev[FB_NQ];
#pragma unroll
      for (int k = 0; k < FB_NQ; ++k) ev[k] = xt ? xb[k] - xt[(size_t)t * FB_NX + k] : xb[k];
      cost = cost + stage_cost(P, ev, ub);
#pragma unroll 1
      for (int st = 0; st < 4; ++st) {
        fb_lds_barrier();
        fb_lds_barrier();
      }
#pragma unroll
      for (int k = 0; k < FB_NX; ++k) xb[k] = X.v[FB_XX + k][lane];  // x̄ₜ₊₁
    }
    cost = cost + final_cost(P, xb);  // :192 (raw x̄_N)
    X.v[0][lane] = cost;  // the outcome to waves 0 and 1
    X.v[1][lane] = s2;
    X.v[2][lane] = eq ? 1.0 : 0.0;
  } else {  // main: bias, solve, stage update
    double xb[FB_NX];
#pragma unroll
    for (int k = 0; k < FB_NX; ++k) {
      xb[k] = x[k];
      if (run) xn[k] = xb[k];
    }
    for (int t = 0; t < T; ++t) {
      double xs[FB_NX], acc[FB_NX], ub[FB_NU];
#pragma unroll
      for (int i = 0; i < FB_NX; ++i) xs[i] = xb[i];
#pragma unroll 1
      for (int st = 0; st < 4; ++st) {
        asm volatile("" ::: "memory");
        double R[FB_NJ][9];
        fb_rots(P, xs, R);
        double bb[FB_NU];
        fb_bias(P, R, xs, bb);
        // the bias is complete before the barrier (else the compiler sinks it past the
        // barrier, behind wave 0's mass, into the serial part of the stage)
#pragma unroll
        for (int j = 0; j < FB_NU; ++j) asm volatile("" ::"v"(bb[j]));
        fb_lds_barrier();
        if (st == 0) {
#pragma unroll
          for (int j = 0; j < FB_NU; ++j) ub[j] = X.v[FB_XU + j][lane];
        }
#pragma unroll
        for (int j = 0; j < FB_NU; ++j) bb[j] = ub[j] - bb[j];
        FbSchur<double> F;
        double* f = reinterpret_cast<double*>(&F);
#pragma unroll
        for (int k = 0; k < FB_SCHUR_N; ++k) f[k] = X.v[k][lane];
        double k[FB_NX];
        fb_solve(F, bb, xs, k);
        const double w = (st == 0 || st == 3) ? 1.0 : 2.0;
        const double c = st == 2 ? 1.0 : 0.5;
#pragma unroll
        for (int i = 0; i < FB_NX; ++i) {
          k[i] = P.dt * k[i];
          acc[i] = st == 0 ? k[i] : acc[i] + w * k[i];
          xs[i] = st < 3 ? xb[i] + k[i] * c : xb[i] + (1.0 / 6.0) * acc[i];
        }
        if (st < 3) {
          X.v[FB_XX + 6][lane] = xs[6];
          X.v[FB_XX + 7][lane] = xs[7];
        } else {
#pragma unroll
          for (int i = 0; i < FB_NX; ++i) X.v[FB_XX + i][lane] = xs[i];
        }
        fb_lds_barrier();
      }
#pragma unroll
      for (int k = 0; k < FB_NX; ++k) {
        xb[k] = xs[k];
        if (run) xn[(size_t)(t + 1) * FB_NX + k] = xb[k];
      }
    }
  }
  fb_lds_barrier();
  const double cost = X.v[0][lane];
  du2 = X.v[1][lane];
  same = X.v[2][lane] != 0.0;
  fb_lds_barrier();  // read before the next rollout writes
  return cost;
}
#endif  // ILQR_FB_LOOKAHEAD

// forward_pass for every trajectory: CAND consecutive lanes roll out trials
// j, j+1, … at once; the first accepted trial (prev_cost − cost > 0, :77-80) is the
// sequential search's; a rejected trial whose ū all equal u ends the search (every later
// trial rolls out identically), as does max_trials (the reference loops unbounded).
// CAND (fb_cand): 4 lanes a trajectory for large batches; small batches, whose waves
// would otherwise run a few live lanes, spend the idle ones on further trials (16 or 64
// a round) — same choice, fewer rounds for a long search. Trial j's α is α₀ multiplied
// by shrink j − 1 times in order, the reference's repeated `α *= shrink` (:82).
template <int CAND>
__global__ __launch_bounds__(64 * FB_FWD_WAVES) void fb_forward_kernel(const FbModel* __restrict__ Pm, int B, int T, FbFwd a) {
  static_assert(CAND == 4 || CAND == 16 || CAND == 64, "a trajectory's lanes sit in one wave");
  const FbModel& P = *Pm;
  const int role = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // the waves of fb_rollout3
  const int lane = threadIdx.x & 63;
  const int c = lane % CAND;
  const int b = (blockIdx.x * 64 + lane) / CAND;
  const bool live = b < B && !(a.status && a.status[b] != ILQR_TRAJ_OK);
  const double pc = live ? a.prev_cost[b] : 0.0;
  int done_trial = 0;     // accepted trial (> 0), or −(last trial) when the search ended
  double done_cost = NAN, done_du2 = 0.0;
  double alpha = a.alpha0;  // trial c + 1's
  for (int k = 0; k < c; ++k) alpha *= a.shrink;
  const size_t nxe = (size_t)(T + 1) * FB_NX, nue = (size_t)T * FB_NU;
  double* slot = a.slots + ((size_t)b * CAND + c) * (nxe + nue);
  for (int j0 = 1; j0 <= a.max_trials; j0 += CAND) {
    const int j = j0 + c;
    const bool run = live && done_trial == 0 && j <= a.max_trials;
    double cost = NAN, du2 = 0.0;
    bool same = false;
    // a trajectory's lanes enter the rollout together when any of them runs (its first:
    // j0 ≤ max_trials): wave 2 loads the trajectory's step inputs a share a lane; the
    // lanes past max_trials roll out without storing, their outcome unused
    if (live && done_trial == 0 && j0 <= a.max_trials) {
      double* xo = j == 1 ? a.xn + (size_t)b * nxe : slot;
      double* uo = j == 1 ? a.un + (size_t)b * nue : slot + nxe;
      double d2 = 0.0;
      bool sm = false;
      const double cs = fb_rollout3<CAND>(P, a, b, T, alpha, xo, uo, d2, sm, role, lane, run);
      if (run) {
        cost = cs;
        du2 = d2;
        same = sm;
      }
    }
    const bool acc = run && (pc - cost > 0.0);
    // the trajectory's lanes agree on the outcome: the smallest accepted j, else whether a
    // rejected trial with ū = u ended the search, else the round's last trial
    const uint64_t accm = __ballot(acc), endm = __ballot(run && !acc && same), runm = __ballot(run);
    const int g0 = (lane / CAND) * CAND;
    constexpr uint64_t gm = CAND == 64 ? ~0ull : (1ull << CAND) - 1;
    const uint64_t ga = (accm >> g0) & gm;
    const uint64_t ge = (endm >> g0) & gm;
    const uint64_t gr = (runm >> g0) & gm;
    // the first accepted lane, the first ending lane, the last lane that ran (every lane
    // takes part in the shuffles)
    const int ca = ga ? __builtin_ctzll(ga) : CAND;
    const int ce = ge ? __builtin_ctzll(ge) : CAND;
    const int cl = gr ? 63 - __builtin_clzll(gr) : 0;
    const int pick = ca < CAND && ca <= ce ? ca : (ce < CAND ? ce : cl);
    const double pcost = __shfl(cost, g0 + pick, 64);
    const double pdu2 = __shfl(du2, g0 + pick, 64);
    if (live && done_trial == 0 && gr) {
      if (ca < CAND && ca <= ce) {
        done_trial = j0 + ca;
      } else if (ce < CAND || j0 + cl >= a.max_trials) {
        done_trial = -(ce < CAND ? a.max_trials : j0 + cl);
      }
      done_cost = pcost;
      done_du2 = pdu2;
    }
    for (int k = 0; k < CAND; ++k) alpha *= a.shrink;  // trial j + CAND's
    if (!__any(live && done_trial == 0)) break;
  }
  // trial 1 stored its rollout into xn/un from waves 1 (x̄) and 2 (ū) with plain global
  // stores, and fb_lds_barrier waits for LDS only: a workgroup release/acquire barrier
  // orders those stores before the copy below writes the same words from other lanes
  // (every wave of the block leaves the loop after the same round: the roles run each
  // rollout together)
  __syncthreads();
  if (live && done_trial <= 0) {  // no trial accepted: x̄, ū = the inputs, as the closure path
    const size_t c2 = (size_t)(FB_FWD_WAVES * c + role);
    for (size_t i = c2; i < nxe; i += FB_FWD_WAVES * CAND) a.xn[(size_t)b * nxe + i] = a.x[(size_t)b * nxe + i];
    for (size_t i = c2; i < nue; i += FB_FWD_WAVES * CAND) a.un[(size_t)b * nue + i] = a.u[(size_t)b * nue + i];
  }
  if (live && c == 0 && role == 0) {
    const bool acc = done_trial > 0;
    a.trials[b] = acc ? done_trial : a.max_trials;
    a.new_cost[b] = done_cost;
    a.du2[b] = done_du2;
    a.fstatus[b] = acc ? ILQR_TRAJ_OK : (done_cost != done_cost ? ILQR_TRAJ_NAN : ILQR_TRAJ_LS_EXHAUSTED);
  }
}

// fit's bookkeeping for one iteration (forward_pass.jl:161-178): a trajectory whose
// backward met a NaN stops (status NAN); an exhausted or NaN search stops; an accepted
// one takes prev_cost = cost (:168), converges when Σ(ū − u)² ≤ tol (:171, returning the
// iterate it started from) or moves to x̄, ū (:174-175).
__global__ __launch_bounds__(256) void fb_update_kernel(int B, int T, int it, double tol, const int32_t* __restrict__ bst,
                                                        const int32_t* __restrict__ fst, const double* __restrict__ cost,
                                                        const double* __restrict__ du2, int32_t* __restrict__ status,
                                                        int32_t* __restrict__ iters, double* __restrict__ prev_cost,
                                                        int32_t* __restrict__ move) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  move[b] = 0;
  if (status[b] != ILQR_TRAJ_OK) return;
  if (bst[b] == ILQR_TRAJ_NAN) {
    status[b] = ILQR_TRAJ_NAN;
    return;
  }
  iters[b] = it;
  if (fst[b] != ILQR_TRAJ_OK) {
    status[b] = fst[b];
    return;
  }
  prev_cost[b] = cost[b];
  if (tol >= 0.0 && du2[b] <= tol) {
    status[b] = ILQR_TRAJ_CONVERGED;
    return;
  }
  move[b] = 1;
}

// the accepted trial's x̄, ū into (x, u): trial 1 from (xn, un), trial j > 1 from its
// slot. fit (move ≠ null): the trajectories that move, into the iterate; forward_pass
// (move = null): every accepted j > 1, into (xn, un) = (x, u) here
__global__ __launch_bounds__(256) void fb_take_kernel(int B, int T, int cand, const int32_t* __restrict__ move,
                                                      const int32_t* __restrict__ fst,
                                                      const int32_t* __restrict__ trials,
                                                      const double* __restrict__ xn, const double* __restrict__ un,
                                                      const double* __restrict__ slots, double* __restrict__ x,
                                                      double* __restrict__ u) {
  const size_t nx = (size_t)(T + 1) * FB_NX, nu = (size_t)T * FB_NU;
  for (int b = blockIdx.y; b < B; b += gridDim.y) {
    const int j = trials[b];
    if (move ? !move[b] : (fst[b] != ILQR_TRAJ_OK || j <= 1)) continue;
    const double* sx = xn + (size_t)b * nx;
    const double* su = un + (size_t)b * nu;
    if (j > 1) {
      sx = slots + ((size_t)b * cand + (j - 1) % cand) * (nx + nu);
      su = sx + nx;
    }
    for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nx + nu; i += (size_t)gridDim.x * blockDim.x) {
      if (i < nx)
        x[(size_t)b * nx + i] = sx[i];
      else
        u[(size_t)b * nu + (i - nx)] = su[i - nx];
    }
  }
}

__global__ void fb_finish_kernel(int B, int32_t* __restrict__ status, int32_t* __restrict__ flags) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  if (status[b] == ILQR_TRAJ_OK) status[b] = ILQR_TRAJ_MAX_ITER;
  if (status[b] == ILQR_TRAJ_NAN) atomicOr(flags, 1);
  if (status[b] == ILQR_TRAJ_LS_EXHAUSTED) atomicOr(flags, 2);
}

__global__ void fb_count_kernel(int B, const int32_t* __restrict__ status, int32_t* __restrict__ out) {
  __shared__ int n;
  if (threadIdx.x == 0) n = 0;
  __syncthreads();
  int k = 0;
  for (int b = threadIdx.x; b < B; b += blockDim.x) k += status[b] == ILQR_TRAJ_OK;
  atomicAdd(&n, k);
  __syncthreads();
  if (threadIdx.x == 0) *out = n;
}

}  // namespace
}  // namespace ilqr

// ---------------------------------------------------------------------------------
// Host side: the handle and its C ABI
// ---------------------------------------------------------------------------------
struct ilqr_floating_handle {
  int device = 0, T = 0, batch = 0;
  ilqr::FbModel model{};
  ilqr::FbModel* model_dev = nullptr;
  hipStream_t stream = nullptr;
  double *x = nullptr, *u = nullptr, *xn = nullptr, *un = nullptr;
  double *d = nullptr, *K = nullptr;
  double *A = nullptr, *Bm = nullptr, *lx = nullptr, *lu = nullptr, *lxx = nullptr, *luu = nullptr;
  double *lfx = nullptr, *lfxx = nullptr;
  double *prev_cost = nullptr, *cost = nullptr, *du2 = nullptr;
  int32_t *trials = nullptr, *status = nullptr, *fstatus = nullptr, *bstatus = nullptr;
  int32_t *iters = nullptr, *move = nullptr, *words = nullptr;
  double* slots = nullptr;  // the line search's trial slots (FbFwd::slots), cand per trajectory
  int cand = 4;             // line-search lanes per trajectory (fb_cand)
};

namespace {

thread_local std::string g_fb_error;

ilqr_status fb_fail(hipError_t e, const char* what) {
  g_fb_error = std::string(what) + ": " + hipGetErrorString(e);
  return ILQR_ERR_HIP;
}

#define FB_TRY(expr)                                    \
  do {                                                  \
    hipError_t e_ = (expr);                             \
    if (e_ != hipSuccess) return fb_fail(e_, #expr);    \
  } while (0)

// the model from the ABI description (fp64 products formed on the host)
bool fb_model(const ilqr_floating* m, ilqr::FbModel& P) {
  using namespace ilqr;
  P = FbModel{};
  P.dt = m->dt;
  auto body = [&](int i, double mass, const double* com, const double* Ic) {
    P.m[i] = mass;
    const double cc = com[0] * com[0] + com[1] * com[1] + com[2] * com[2];
    for (int k = 0; k < 3; ++k) P.h[i][k] = mass * com[k];
    for (int r = 0; r < 3; ++r)
      for (int k = 0; k < 3; ++k) P.Io[i][3 * r + k] = Ic[3 * r + k] + mass * ((r == k ? cc : 0.0) - com[r] * com[k]);
  };
  body(0, m->base_mass, m->base_com, m->base_inertia);
  for (int j = 0; j < FB_NJ; ++j) {
    body(j + 1, m->mass[j], m->com[j], m->inertia[j]);
    const double* R0 = m->joint_rot[j];
    const double* a = m->axis[j];
    const double na = std::sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
    if (!(na > 0.0)) return false;
    const double an[3] = {a[0] / na, a[1] / na, a[2] / na};
    const double ax[9] = {0.0, -an[2], an[1], an[2], 0.0, -an[0], -an[1], an[0], 0.0};
    for (int r = 0; r < 3; ++r)
      for (int k = 0; k < 3; ++k) {
        double s = 0.0, t = 0.0;
        for (int q = 0; q < 3; ++q) {
          s += R0[3 * r + q] * ax[3 * q + k];
          t += R0[3 * r + q] * an[q] * an[k];
        }
        P.R0[j][3 * r + k] = R0[3 * r + k];
        P.R0x[j][3 * r + k] = s;
        P.R0aa[j][3 * r + k] = t;
      }
    for (int k = 0; k < 3; ++k) {
      P.p[j][k] = m->joint_pos[j][k];
      P.ax[j][k] = an[k];
    }
  }
  P.qs = m->q_scale;
  P.rs = m->r_scale;
  P.qfs = m->qf_scale;
  for (int i = 0; i < FB_NQ; ++i) {
    P.tgt[i] = m->target[i];
    P.qw[i] = m->q_weight[i];
    P.rw[i] = m->r_weight[i];
    P.qfw[i] = m->qf_weight[i];
    // derivative coefficients as the closed forms write them: −(2·qs·qw)·(tgt − x), …
    P.gx[i] = -(2.0 * P.qs) * P.qw[i];
    P.hx[i] = (2.0 * P.qs) * P.qw[i];
    P.gu[i] = (2.0 * P.rs) * P.rw[i];
    P.hu[i] = (2.0 * P.rs) * P.rw[i];
    P.gf[i] = -(2.0 * P.qfs) * P.qfw[i];
    P.hf[i] = (2.0 * P.qfs) * P.qfw[i];
  }
  return true;
}

// line-search lanes per trajectory: the most (64, 16 or 4) with which the launch still
// has at most one workgroup per CU (B·CAND ≤ 256·64) — a round of trials costs one
// rollout's latency whatever its width, so idle CUs take further trials (5-iteration
// fits from the script's start, profiles/r06/floating_cand_fit_r06.log: B = 256 13.25 →
// 12.91 ms per iteration with 64 against 16, B = 1024 22.9 → 22.2 ms with 16 against 4)
// — and whose trial slots (B·CAND rollouts) stay within 4 GiB
int fb_cand(int B, int T) {
  if (const char* e = std::getenv("ILQR_FB_CAND")) {  // A/B measurement override: 4, 16 or 64
    const int c = std::atoi(e);
    if (c == 4 || c == 16 || c == 64) return c;
  }
  const size_t slot = 8 * ((size_t)(T + 1) * ilqr::FB_NX + (size_t)T * ilqr::FB_NU);
  for (int c : {64, 16})
    if ((size_t)B * c <= 256 * 64 && (size_t)B * c * slot <= (size_t(4) << 30)) return c;
  return ilqr::FB_CAND;
}

ilqr::LSParams fb_ls(const ilqr_options* o) {
  ilqr_options def;
  ilqr_default_options(&def);
  if (!o) o = &def;
  return ilqr::LSParams{o->mu, o->alpha0, o->shrink, o->tol, o->max_trials};
}

ilqr_status fb_check_options(const ilqr_options* o) {
  if (!o) return ILQR_OK;
  if (o->max_trials < 1 || o->max_iter < 0) return ILQR_ERR_BAD_ARG;
  if (!(o->shrink > 0.0 && o->shrink < 1.0) || !(o->alpha0 > 0.0) || std::isnan(o->mu)) return ILQR_ERR_BAD_ARG;
  return ILQR_OK;
}

// per-trajectory status → the call status (host copy, synchronising)
ilqr_status fb_fold(ilqr_floating_handle* h, const int32_t* dev_status) {
  std::vector<int32_t> st(h->batch);
  FB_TRY(hipMemcpyAsync(st.data(), dev_status, sizeof(int32_t) * h->batch, hipMemcpyDeviceToHost, h->stream));
  FB_TRY(hipStreamSynchronize(h->stream));
  bool nan = false, ls = false;
  for (int32_t s : st) {
    nan |= s == ILQR_TRAJ_NAN;
    ls |= s == ILQR_TRAJ_LS_EXHAUSTED;
  }
  return nan ? ILQR_ERR_NAN : (ls ? ILQR_ERR_LS_EXHAUSTED : ILQR_OK);
}

// fb_take_kernel over the batch: one row of blocks per trajectory, ≤ 64 blocks along it
hipError_t fb_take(ilqr_floating_handle* h, const int32_t* move, const int32_t* fst, const int32_t* trials,
                   const double* xn, const double* un, double* x, double* u) {
  const size_t n = (size_t)(h->T + 1) * ilqr::FB_NX + (size_t)h->T * ilqr::FB_NU;
  const unsigned gx = (unsigned)((n + 255) / 256 < 64 ? (n + 255) / 256 : 64);
  ilqr::fb_take_kernel<<<dim3(gx, (unsigned)(h->batch < 65535 ? h->batch : 65535)), 256, 0, h->stream>>>(
      h->batch, h->T, h->cand, move, fst, trials, xn, un, h->slots, x, u);
  return hipGetLastError();
}

// the forward over the batch at the handle's lanes per trajectory
hipError_t fb_forward(ilqr_floating_handle* h, const ilqr::FbFwd& fa) {
  const unsigned th = 64 * ilqr::FB_FWD_WAVES, g = (unsigned)(((size_t)h->batch * h->cand + 63) / 64);
  if (h->cand == 64)
    ilqr::fb_forward_kernel<64><<<g, th, 0, h->stream>>>(h->model_dev, h->batch, h->T, fa);
  else if (h->cand == 16)
    ilqr::fb_forward_kernel<16><<<g, th, 0, h->stream>>>(h->model_dev, h->batch, h->T, fa);
  else
    ilqr::fb_forward_kernel<4><<<g, th, 0, h->stream>>>(h->model_dev, h->batch, h->T, fa);
  return hipGetLastError();
}

hipError_t fb_linearize(ilqr_floating_handle* h, const double* x, const double* u, const int32_t* st) {
  const size_t lanes = (size_t)h->batch * h->T * ilqr::FB_LIN_DIRS;
  ilqr::fb_linearize_kernel<<<(unsigned)((lanes + 255) / 256), 256, 0, h->stream>>>(
      h->model_dev, h->batch, h->T, x, u, st, h->A, h->Bm, h->lx, h->lu, h->lxx, h->luu, h->lfx, h->lfxx);
  return hipGetLastError();
}

}  // namespace

extern "C" {

int ilqr_floating_supported(int n_joints) { return n_joints == ilqr::FB_NJ ? 1 : 0; }

const char* ilqr_floating_last_error(void) { return g_fb_error.c_str(); }

ilqr_status ilqr_floating_create(ilqr_floating_handle** out, int device, const ilqr_floating* m, int T,
                                 int batch) {
  if (!out || !m) return ILQR_ERR_BAD_ARG;
  *out = nullptr;
  if (T <= 0 || batch <= 0) return ILQR_ERR_BAD_DIMS;
  if (!ilqr_floating_supported(m->n_joints)) {
    g_fb_error = "ilqr_floating_create: n_joints must be 2 (the reference's 2Dof_arm)";
    return ILQR_ERR_UNSUPPORTED;
  }
  if (!(m->dt > 0.0) || !(m->base_mass > 0.0)) return ILQR_ERR_BAD_ARG;
  if (m->gravity[0] != 0.0 || m->gravity[1] != 0.0 || m->gravity[2] != 0.0) {
    g_fb_error = "ilqr_floating_create: gravity must be zero (the reference parses the URDF with gravity = 0)";
    return ILQR_ERR_UNSUPPORTED;
  }
  ilqr::FbModel model;
  if (!fb_model(m, model)) return ILQR_ERR_BAD_ARG;
  FB_TRY(hipSetDevice(device));  // before the handle exists: a failure leaks nothing
  auto* h = new ilqr_floating_handle;
  h->model = model;
  h->device = device;
  h->T = T;
  h->batch = batch;
  const size_t B = (size_t)batch, nx = ilqr::FB_NX, nu = ilqr::FB_NU, P = B * T;
  hipError_t e = hipSuccess;
  auto alloc = [&](auto** p, size_t bytes) {
    if (e == hipSuccess) e = hipMalloc((void**)p, bytes);
  };
  alloc(&h->x, 8 * B * (T + 1) * nx);
  alloc(&h->u, 8 * P * nu);
  alloc(&h->xn, 8 * B * (T + 1) * nx);
  alloc(&h->un, 8 * P * nu);
  alloc(&h->d, 8 * P * nu);
  alloc(&h->K, 8 * P * nu * nx);
  alloc(&h->A, 8 * P * nx * nx);
  alloc(&h->Bm, 8 * P * nx * nu);
  alloc(&h->lx, 8 * P * nx);
  alloc(&h->lu, 8 * P * nu);
  alloc(&h->lxx, 8 * P * nx * nx);
  alloc(&h->luu, 8 * P * nu * nu);
  alloc(&h->lfx, 8 * B * nx);
  alloc(&h->lfxx, 8 * B * nx * nx);
  alloc(&h->prev_cost, 8 * B);
  alloc(&h->cost, 8 * B);
  alloc(&h->du2, 8 * B);
  alloc(&h->trials, 4 * B);
  alloc(&h->status, 4 * B);
  alloc(&h->fstatus, 4 * B);
  alloc(&h->bstatus, 4 * B);
  alloc(&h->iters, 4 * B);
  alloc(&h->move, 4 * B);
  alloc(&h->words, 4 * 4);
  h->cand = fb_cand(batch, T);
  alloc(&h->slots, 8 * B * h->cand * ((T + 1) * nx + (size_t)T * nu));
  alloc(&h->model_dev, sizeof(ilqr::FbModel));
  if (e == hipSuccess) e = hipMemcpy(h->model_dev, &h->model, sizeof(ilqr::FbModel), hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    ilqr_floating_destroy(h);
    return fb_fail(e, "ilqr_floating_create: hipMalloc");
  }
  *out = h;
  return ILQR_OK;
}

ilqr_status ilqr_floating_destroy(ilqr_floating_handle* h) {
  if (!h) return ILQR_OK;
  (void)hipSetDevice(h->device);
  for (double* p : {h->x, h->u, h->xn, h->un, h->d, h->K, h->A, h->Bm, h->lx, h->lu, h->lxx, h->luu, h->lfx,
                    h->lfxx, h->prev_cost, h->cost, h->du2, h->slots})
    (void)hipFree(p);
  for (int32_t* p : {h->trials, h->status, h->fstatus, h->bstatus, h->iters, h->move, h->words}) (void)hipFree(p);
  (void)hipFree(h->model_dev);
  delete h;
  return ILQR_OK;
}

ilqr_status ilqr_floating_set_stream(ilqr_floating_handle* h, void* s) {
  if (!h) return ILQR_ERR_BAD_ARG;
  h->stream = (hipStream_t)s;
  return ILQR_OK;
}

ilqr_status ilqr_floating_sync(ilqr_floating_handle* h) {
  if (!h) return ILQR_ERR_BAD_ARG;
  FB_TRY(hipStreamSynchronize(h->stream));
  return ILQR_OK;
}

ilqr_status ilqr_floating_dynamics(ilqr_floating_handle* h, const double* x, const double* u, double* x_next,
                                   int n) {
  if (!h || !x || !u || !x_next) return ILQR_ERR_BAD_ARG;
  if (n <= 0) return ILQR_ERR_BAD_DIMS;
  FB_TRY(hipSetDevice(h->device));
  ilqr::fb_dynamics_kernel<<<(n + 255) / 256, 256, 0, h->stream>>>(h->model_dev, n, x, u, x_next);
  FB_TRY(hipGetLastError());
  return ILQR_OK;
}

ilqr_status ilqr_floating_linearize(ilqr_floating_handle* h, const double* x, const double* u, double* A,
                                    double* B) {
  if (!h || !x || !u || !A || !B) return ILQR_ERR_BAD_ARG;
  FB_TRY(hipSetDevice(h->device));
  FB_TRY(fb_linearize(h, x, u, nullptr));
  const size_t P = (size_t)h->batch * h->T;
  FB_TRY(hipMemcpyAsync(A, h->A, 8 * P * ilqr::FB_NX * ilqr::FB_NX, hipMemcpyDeviceToDevice, h->stream));
  FB_TRY(hipMemcpyAsync(B, h->Bm, 8 * P * ilqr::FB_NX * ilqr::FB_NU, hipMemcpyDeviceToDevice, h->stream));
  return ILQR_OK;
}

ilqr_status ilqr_floating_backward(ilqr_floating_handle* h, const ilqr_options* o, const double* x,
                                   const double* u, double* d, double* K, int32_t* status) {
  if (!h || !x || !u || !d || !K) return ILQR_ERR_BAD_ARG;
  ilqr_status st = fb_check_options(o);
  if (st != ILQR_OK) return st;
  FB_TRY(hipSetDevice(h->device));
  FB_TRY(fb_linearize(h, x, u, nullptr));
  const ilqr::TileParams tp{h->A, h->Bm, h->lx, h->lu, h->lxx, nullptr, h->luu, h->lfx, h->lfxx};
  int32_t* sd = status ? status : h->bstatus;
  FB_TRY(ilqr::launch_tiles_backward(ilqr::FB_NX, ilqr::FB_NU, tp, h->batch, h->T, d, K, sd, fb_ls(o).mu,
                                     h->stream));
  return fb_fold(h, sd);
}

ilqr_status ilqr_floating_forward(ilqr_floating_handle* h, const ilqr_options* o, const double* x,
                                  const double* u, const double* x_traj, const double* d, const double* K,
                                  const double* prev_cost, double* x_new, double* u_new, double* new_cost,
                                  int32_t* trials, int32_t* status) {
  if (!h || !x || !u || !d || !K || !prev_cost || !x_new || !u_new || !new_cost) return ILQR_ERR_BAD_ARG;
  ilqr_status st = fb_check_options(o);
  if (st != ILQR_OK) return st;
  FB_TRY(hipSetDevice(h->device));
  const ilqr::LSParams ls = fb_ls(o);
  ilqr::FbFwd fa{};
  fa.x = x;
  fa.u = u;
  fa.xtraj = x_traj;
  fa.d = d;
  fa.K = K;
  fa.prev_cost = prev_cost;
  fa.xn = x_new;
  fa.un = u_new;
  fa.new_cost = new_cost;
  fa.du2 = h->du2;
  fa.trials = trials ? trials : h->trials;
  fa.fstatus = status ? status : h->fstatus;
  fa.status = nullptr;
  fa.slots = h->slots;
  fa.alpha0 = ls.alpha0;
  fa.shrink = ls.shrink;
  fa.max_trials = ls.max_trials;
  FB_TRY(fb_forward(h, fa));
  // x̄, ū of a trajectory whose first trial was accepted are written as it rolled out; a
  // later accepted trial is taken from its slot; a search that accepted nothing returns
  // x, u (the closure path's rollout_forward does the same)
  FB_TRY(fb_take(h, nullptr, fa.fstatus, fa.trials, x_new, u_new, x_new, u_new));
  return fb_fold(h, fa.fstatus);
}

ilqr_status ilqr_floating_fit(ilqr_floating_handle* h, const ilqr_options* o, const double* x_init,
                              const double* u_init, const double* x_traj, double* x_out, double* u_out,
                              double* cost, int32_t* iters, int32_t* status) {
  return ilqr_floating_fit_ex(h, o, x_init, u_init, x_traj, x_out, u_out, cost, iters, status, nullptr);
}

ilqr_status ilqr_floating_fit_ex(ilqr_floating_handle* h, const ilqr_options* o, const double* x_init,
                                 const double* u_init, const double* x_traj, double* x_out, double* u_out,
                                 double* cost, int32_t* iters, int32_t* status, const ilqr_history* hist) {
  if (!h || !x_init || !u_init || !x_out || !u_out) return ILQR_ERR_BAD_ARG;
  if (hist && !hist->cost && !hist->trials && !hist->alpha && !hist->du2) hist = nullptr;
  ilqr_status st = fb_check_options(o);
  if (st != ILQR_OK) return st;
  FB_TRY(hipSetDevice(h->device));
  const ilqr::LSParams ls = fb_ls(o);
  const int max_iter = o ? o->max_iter : 100;
  const int B = h->batch, T = h->T;
  const size_t nxe = (size_t)(T + 1) * ilqr::FB_NX, nue = (size_t)T * ilqr::FB_NU;
  hipStream_t s = h->stream;
  FB_TRY(hipMemcpyAsync(h->x, x_init, 8 * B * nxe, hipMemcpyDeviceToDevice, s));
  FB_TRY(hipMemcpyAsync(h->u, u_init, 8 * B * nue, hipMemcpyDeviceToDevice, s));
  FB_TRY(ilqr::launch_fill_f64(h->prev_cost, B, INFINITY, s));  // :159
  FB_TRY(ilqr::launch_fill_i32(h->status, B, ILQR_TRAJ_OK, s));
  FB_TRY(ilqr::launch_fill_i32(h->iters, B, 0, s));
  FB_TRY(hipMemsetAsync(h->words, 0, 4 * 4, s));
  const ilqr::TileParams tp{h->A, h->Bm, h->lx, h->lu, h->lxx, nullptr, h->luu, h->lfx, h->lfxx};
  ilqr::FbFwd fa{};
  fa.x = h->x;
  fa.u = h->u;
  fa.xtraj = x_traj;
  fa.d = h->d;
  fa.K = h->K;
  fa.prev_cost = h->prev_cost;
  fa.xn = h->xn;
  fa.un = h->un;
  fa.new_cost = h->cost;
  fa.du2 = h->du2;
  fa.trials = h->trials;
  fa.fstatus = h->fstatus;
  fa.status = h->status;
  fa.slots = h->slots;
  fa.alpha0 = ls.alpha0;
  fa.shrink = ls.shrink;
  fa.max_trials = ls.max_trials;
  const unsigned g = (unsigned)((B + 255) / 256);
  for (int it = 1; it <= max_iter; ++it) {  // forward_pass.jl:161
    FB_TRY(fb_linearize(h, h->x, h->u, h->status));
    FB_TRY(ilqr::launch_tiles_backward(ilqr::FB_NX, ilqr::FB_NU, tp, B, T, h->d, h->K, h->bstatus, ls.mu, s));
    FB_TRY(fb_forward(h, fa));
    ilqr::fb_update_kernel<<<g, 256, 0, s>>>(B, T, it, ls.tol, h->bstatus, h->fstatus, h->cost, h->du2,
                                             h->status, h->iters, h->prev_cost, h->move);
    FB_TRY(hipGetLastError());
    FB_TRY(fb_take(h, h->move, h->fstatus, h->trials, h->xn, h->un, h->x, h->u));
    if (hist)  // the per-iteration record (ilqr_history), as the other families'
      FB_TRY(ilqr::launch_record_history(B, it, h->status, h->iters, h->trials, h->prev_cost, h->du2, false,
                                         ls.alpha0, ls.shrink, hist->cost, hist->trials, hist->alpha, hist->du2, s));
    if (ls.tol >= 0.0 && it < max_iter) {  // :171's break once every trajectory stopped
      ilqr::fb_count_kernel<<<1, 256, 0, s>>>(B, h->status, h->words);
      FB_TRY(hipGetLastError());
      int32_t running = 0;
      FB_TRY(hipMemcpyAsync(&running, h->words, 4, hipMemcpyDeviceToHost, s));
      FB_TRY(hipStreamSynchronize(s));
      if (running == 0) break;
    }
  }
  ilqr::fb_finish_kernel<<<g, 256, 0, s>>>(B, h->status, h->words + 1);
  FB_TRY(hipGetLastError());
  FB_TRY(hipMemcpyAsync(x_out, h->x, 8 * B * nxe, hipMemcpyDeviceToDevice, s));
  FB_TRY(hipMemcpyAsync(u_out, h->u, 8 * B * nue, hipMemcpyDeviceToDevice, s));
  if (cost) FB_TRY(hipMemcpyAsync(cost, h->prev_cost, 8 * B, hipMemcpyDeviceToDevice, s));
  if (iters) FB_TRY(hipMemcpyAsync(iters, h->iters, 4 * B, hipMemcpyDeviceToDevice, s));
  if (status) FB_TRY(hipMemcpyAsync(status, h->status, 4 * B, hipMemcpyDeviceToDevice, s));
  int32_t flags = 0;
  FB_TRY(hipMemcpyAsync(&flags, h->words + 1, 4, hipMemcpyDeviceToHost, s));
  FB_TRY(hipStreamSynchronize(s));
  return (flags & 1) ? ILQR_ERR_NAN : ((flags & 2) ? ILQR_ERR_LS_EXHAUSTED : ILQR_OK);
}

}  // extern "C"

#ifdef ILQR_FB_TRACE
// the trace build's per-role totals (work, barrier wait, poll wait, barriers), then reset
extern "C" int ilqr_debug_fb_trace(unsigned long long* out) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(ilqr::g_fbt), sizeof(unsigned long long) * 32) != hipSuccess) return -1;
  unsigned long long z[32] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(ilqr::g_fbt), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif
