// MI355X (gfx950) backward pass from caller-supplied derivative tiles
// (ilqr_backward_tiles): the drop-in for backward_pass with
// ARBITRARY closures. The caller evaluates the reference's derivative calls along
// (x, u) — linearize_dynamics (src/backward_pass.jl:25-40), immediate_cost_
// quadratization (:81-109), final_cost_quadratization (:134-153), e.g. with
// ForwardDiff on the host exactly as the reference does — and the device runs the
// rest of backward_pass (:335-357): optimal_controller_param (:177-186),
// feedback_parameters (:207-218) and step_back (:262-273).
//
// Same wave-per-trajectory MFMA recursion as lq_backward_wave (ilqr_lq.hip, DESIGN.md
// §4): the value function Sp = [[S, s], [0, 0]] stays in the accumulator layout of
// v_mfma_f64_16x16x4_f64; per step Y = Spᵀ·F, Z = L + FᵀY, one LDS hand-off of
// [G | H] and g, an LDLᵀ solve per lane and the rank-nu update
// Sp ← [Qxx | lx + Aᵀs] − K_augᵀ (H + 2μI) K_aug. The difference is the data flow:
// F_t = [A_t | B_t], the full cost Hessian L_t = [[lxx, luxᵀ], [lux, luu]] and the
// gradient [lx; lu] are new every step, so the kernel streams 8·(nx(nx+nu) +
// (nx+nu)² + nx + nu) bytes per step from HBM (prefetched one step ahead) and is
// HBM-bound rather than FP64-bound.
#include <hip/hip_runtime.h>
#include <math.h>

#include "ilqr_internal.h"
#include "ilqr_device.h"
#include "../../include/ilqr.h"

namespace ilqr {
namespace {

constexpr int TB_LDS = 96 + 16 * 17;  // doubles of scratch per wave (as the LQ kernel)
constexpr int TB_SYM_EVERY = 4;

template <int NX, int NU>
struct StepTile {
  double fB[(NX + 3) / 4];  // F[4kk+q][c]
  d4 Lc;                    // L[q+4r][c]
  double lv;                // [lx; lu][c]
};

template <int NX, int NU>
__device__ bool tiles_backward_wave(const TileParams& P, int b, int T, double* __restrict__ d_out,
                                    double* __restrict__ K_out, double mu, double* lds) {
  static_assert(NX + NU <= 16 && NX < 16 && NU <= 4, "MFMA tile mapping needs nx+nu <= 16, nu <= 4");
  constexpr int KS = (NX + 3) / 4;
  constexpr int SROW = NX;
  const int l = threadIdx.x & 63;
  const int c = l & 15;
  const int q = l >> 4;
  const bool cx = c < NX;
  const bool cu = c >= NX && c < NX + NU;
  const int ci = cx ? c : 0;
  const int cj = cu ? c - NX : 0;

  const size_t bt = (size_t)b * T;
  const double* A0 = P.A + bt * NX * NX;
  const double* B0 = P.B + bt * NX * NU;
  const double* lx0 = P.lx + bt * NX;
  const double* lu0 = P.lu + bt * NU;
  const double* lxx0 = P.lxx + bt * NX * NX;
  const double* lux0 = P.lux ? P.lux + bt * NU * NX : lxx0;  // NULL: zeros (read with weight 0)
  const double wux = P.lux ? 1.0 : 0.0;
  const double* luu0 = P.luu + bt * NU * NU;

  auto load = [&](int t, StepTile<NX, NU>& s) {
    const double* A = A0 + (size_t)t * NX * NX;
    const double* Bm = B0 + (size_t)t * NX * NU;
    const double* lxx = lxx0 + (size_t)t * NX * NX;
    const double* lux = P.lux ? lux0 + (size_t)t * NU * NX : lxx0;
    const double* luu = luu0 + (size_t)t * NU * NU;
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) {
      const int i = 4 * kk + q;
      const bool ri = i < NX;
      const int ii = ri ? i : 0;
      s.fB[kk] = ldz_async(ri & cx, A + ii * NX + ci, A) + ldz_async(ri & cu, Bm + ii * NU + cj, Bm);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = q + 4 * r;
      const bool rx = i < NX, ru = i >= NX && i < NX + NU;
      const int ix = rx ? i : 0, iu = ru ? i - NX : 0;
      const double xx = ldz_async(rx & cx, lxx + ix * NX + ci, lxx);
      const double xu = ldz_async(rx & cu, lux + cj * NX + ix, lux);  // L[i][NX+j] = 𝐏[j][i]
      const double ux = ldz_async(ru & cx, lux + iu * NX + ci, lux);  // L[NX+j][c] = 𝐏[j][c]
      const double uu = ldz_async(ru & cu, luu + iu * NU + cj, luu);
      s.Lc[r] = xx + wux * (xu + ux) + uu;
    }
    s.lv = ldz_async(cx, lx0 + (size_t)t * NX + ci, lx0) + ldz_async(cu, lu0 + (size_t)t * NU + cj, lu0);
  };

  double* Gl = lds;
  double* gl = lds + 64;
  constexpr int ZERO = 80;
  lds[ZERO] = 0.0;
  int col_at[NU];
#pragma unroll
  for (int j = 0; j < NU; ++j) col_at[j] = cx ? j * 16 + c : (c == SROW ? 64 + NX + j : ZERO);
  const int qq = q < NU ? q : 0;
  const int colq_at = cx ? qq * 16 + c : (c == SROW ? 64 + NX + qq : ZERO);
  int qv_at[KS];
#pragma unroll
  for (int r = 0; r < KS; ++r) qv_at[r] = (c == SROW && q + 4 * r < NX) ? 64 + q + 4 * r : ZERO;

  // terminal value function (:335-336): S = ∇²ℓ_f, s = ∇ℓ_f (column SROW)
  d4 Sp;
  {
    const double* lfxx = P.lfxx + (size_t)b * NX * NX;
    const double* lfx = P.lfx + (size_t)b * NX;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = q + 4 * r;
      const bool rx = i < NX;
      const int ix = rx ? i : 0;
      Sp[r] = ldz_async(rx & cx, lfxx + ix * NX + ci, lfxx) + ldz_async(rx & (c == SROW), lfx + ix, lfx);
    }
  }

  bool nan = false;
  double* Kb = K_out + (size_t)b * T * NU * NX;
  double* db = d_out + (size_t)b * T * NU;
  StepTile<NX, NU> cur, nxt;
  load(T - 1, cur);
  for (int t = T - 1; t >= 0; --t) {
    load(t > 0 ? t - 1 : 0, nxt);  // prefetch

    d4 Y = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) Y = mfma(Sp[kk], cur.fB[kk], Y);
    d4 Z = cur.Lc;  // Z = L + FᵀY: [[lxx + AᵀSA, ·], [lux + BᵀSA, luu + BᵀSB]] (:182-183)
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) Z = mfma(cur.fB[kk], Y[kk], Z);

    // gq[c] = [lx; lu][c] + (Fᵀ s)[c]: lx + Aᵀs (c < NX), g = lu + Bᵀs (:181, :269)
    double part = (q == 0) ? cur.lv : 0.0;
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (r == SROW / 4) part += (q == SROW % 4) ? Y[r] : 0.0;
    const double gq = colsum4(part);

#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = q + 4 * r;
      if (i >= NX && i < NX + NU) Gl[(i - NX) * 16 + c] = Z[r];
    }
    gl[c] = gq;
    double h[NU][NU];
    d4 col = {0.0, 0.0, 0.0, 0.0};
    wave_lds_fence();
#pragma unroll
    for (int i = 0; i < NU; ++i)
#pragma unroll
      for (int k = 0; k <= i; ++k) h[i][k] = Gl[i * 16 + NX + k];
#pragma unroll
    for (int j = 0; j < NU; ++j) col[j] = lds[col_at[j]];
    const double colq = lds[colq_at];
    double qv[KS];
#pragma unroll
    for (int r = 0; r < KS; ++r) qv[r] = lds[qv_at[r]];
    wave_lds_fence();

    // feedback_parameters (:207-218)
    LDLT<NU> f;
    f.factor(h, mu);
    const d4 xs = f.solve(col);
    const double kq = (q < NU) ? -xs[qq] : 0.0;
    const double wk = (q < NU) ? fma(mu, kq, -colq) : 0.0;
    nan |= __builtin_isnan(kq);
    {
      double* dst = cx ? Kb + ((size_t)t * NU + qq) * NX + c : db + (size_t)t * NU + qq;
      if (q < NU && c <= SROW) *dst = kq;
    }

    // step_back (:269-270), exact rewrite
    d4 Cin;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      double v = 0.0;
      if (r < KS) v = cx ? Z[r] : qv[r];
      Cin[r] = (q + 4 * r < NX) ? v : 0.0;
    }
    Sp = mfma(-kq, wk, Cin);
    cur = nxt;

    if ((t % TB_SYM_EVERY) == 0) {
      double* tile = lds + 96;
#pragma unroll
      for (int r = 0; r < 4; ++r) tile[(q + 4 * r) * 17 + c] = Sp[r];
      wave_lds_fence();
#pragma unroll
      for (int r = 0; r < KS; ++r) {
        const int i = q + 4 * r;
        const double other = tile[c * 17 + (i < NX ? i : 0)];
        const double avg = 0.5 * (Sp[r] + other);
        Sp[r] = (i < NX && cx) ? avg : Sp[r];
      }
      wave_lds_fence();
    }
  }
  return __any(nan);
}

template <int NX, int NU>
__global__ __launch_bounds__(256) void tiles_backward_kernel(TileParams P, int B, int T,
                                                             double* __restrict__ d,
                                                             double* __restrict__ K,
                                                             int32_t* __restrict__ status,
                                                             double mu) {
  __shared__ __attribute__((aligned(16))) double lds[4 * TB_LDS];
  const int w = threadIdx.x >> 6;
  const int b = blockIdx.x * 4 + w;
  if (b >= B) return;
  const bool nan = tiles_backward_wave<NX, NU>(P, b, T, d, K, mu, lds + w * TB_LDS);
  if (status && (threadIdx.x & 63) == 0) status[b] = nan ? ILQR_TRAJ_NAN : ILQR_TRAJ_OK;
}

// ---------------------------------------------------------------------------------
// WIDE shapes: nx ≤ 16, nu ≤ 8 (the reference's RBD caller is nx = 16, nu = 8, T = 1000:
// test/RBD_2_link_example/animate_RBD_2_link.jl:8,19-20,31). F = [A | B] no longer fits
// one 16×16 tile beside the value gradient, so the recursion is split over 16×16 tiles
// of v_mfma_f64_16x16x4_f64 (lane 16q + c holds row q + 4r, column c of an accumulator):
//   Y_A = S·A,  Y_B = S·B + s·e₈ᵀ          (B in columns 0..7, s rides in column 8)
//   Z_xx = lxx + AᵀY_A                     (:270's AᵀSA part)
//   Z_xe = [· | lx] + AᵀY_B                (column 8: 𝐪 + Aᵀ𝐬, :269)
//   Z_ux = lux + BᵀY_A = G                 (:182)
//   Z_ue = [luu | lu] + BᵀY_B = [H | g]    (:181, :183)
// one LDS hand-off of G, H, g; every lane factors H + μI (LDLᵀ, 8×8) and solves its
// column of G and g; the exact rank-nu step_back (as the narrow kernel):
//   S ← Z_xx − Kᵀ(H + 2μI)K,  s ← (Z_xe − Kᵀ(H + 2μI)·[· | d]) column 8.
// 28 MFMAs per step. The dimensions are run-time values zero-padded to 16 × 8: padded
// rows/columns of A, B and the cost tiles are zero, so the padded gains are zero and the
// real ones are unchanged (the LDLᵀ pivots of the padding come last and are exactly μ).
// ---------------------------------------------------------------------------------
constexpr int TW_NX = 16, TW_NU = 8;
constexpr int TW_BUF_MIN_B = 64;  // batches from here load their tiles with raw buffer loads
constexpr int TW_LDS = 128 + 128 + 16 * 17;  // G rows, [H | g] rows, symmetrisation tile

__device__ __forceinline__ double pick4(const double (&v)[TW_NU], int q, int base) {
  const double a = (q & 1) ? v[base + 1] : v[base];
  const double b = (q & 1) ? v[base + 3] : v[base + 2];
  return (q & 2) ? b : a;
}

struct WideTile {
  double fA[4];  // A[4kk+q][c]
  double fB[4];  // B[4kk+q][c]
  d4 Lxx;        // lxx[q+4r][c]
  d4 Lux;        // lux[q+4r][c] (rows < nu)
  d4 Lue;        // [luu | lu][q+4r][c]
  d4 Lxe;        // lx[q+4r] in column 8
};

// A step's tiles, zero-padded to 16 × 8, for lane (q, c) of the wide kernel.
//   WideLoads<false> (small batches): ldz_async per element — a lone trajectory's step is
//     a latency chain, and this way it is 4 % faster (B = 1, T = 1000: 2.09 against 2.18 ms);
//   WideLoads<true> (large batches): raw buffer loads — a lane's offset is fixed for the
//     whole recursion (its element, or out of range when its row or column is padding:
//     the bounds check returns 0) and the step moves a scalar offset, so a load is one
//     instruction where ldz_async's address and zero selects and 64-bit address
//     arithmetic were ≈180 VALU instructions a step (B = 4096, T = 100: 1.07 → 0.85 ms).
// The same values either way (profiles/r06/tiles_buf_ab_r06.log: bit-equal gains).
template <bool BUF>
struct WideLoads;
template <>
struct WideLoads<false> {
  const double *A0, *B0, *lx0, *lu0, *lxx0, *lux0, *luu0;
  size_t sxx, sxu, suu;
  int nx, nu, q, c;
  __device__ WideLoads(const TileParams& P, int b, int T, int nx_, int nu_, int q_, int c_)
      : nx(nx_), nu(nu_), q(q_), c(c_) {
    const size_t bt = (size_t)b * T;
    sxx = (size_t)nx * nx;
    sxu = (size_t)nx * nu;
    suu = (size_t)nu * nu;
    A0 = P.A + bt * sxx;
    B0 = P.B + bt * sxu;
    lx0 = P.lx + bt * nx;
    lu0 = P.lu + bt * nu;
    lxx0 = P.lxx + bt * sxx;
    lux0 = P.lux ? P.lux + bt * sxu : nullptr;
    luu0 = P.luu + bt * suu;
  }
  __device__ __forceinline__ void load(int t, WideTile& s) const {
    const bool cx = c < nx, cu = c < nu, c8 = c == 8;
    const double* A = A0 + (size_t)t * sxx;
    const double* Bm = B0 + (size_t)t * sxu;
    const double* lxx = lxx0 + (size_t)t * sxx;
    const double* luu = luu0 + (size_t)t * suu;
    const double* lx = lx0 + (size_t)t * nx;
    const double* lu = lu0 + (size_t)t * nu;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int i = 4 * kk + q;
      const bool ri = i < nx;
      s.fA[kk] = ldz_async(ri & cx, A + i * nx + c, A);
      s.fB[kk] = ldz_async(ri & cu, Bm + i * nu + c, Bm);
      s.Lxx[kk] = ldz_async(ri & cx, lxx + i * nx + c, lxx);
      s.Lxe[kk] = ldz_async(ri & c8, lx + i, lx);
    }
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int i = q + 4 * r;
      const bool ru = i < nu;
      // unconditional (ldz): a load in a branch on lux0 waits for every load in flight at
      // its join — the whole prefetch, at the top of each step
      const double* lux = lux0 ? lux0 + (size_t)t * sxu : A;
      s.Lux[r] = ldz_async((lux0 != nullptr) & ru & cx, lux + i * nx + c, A);
      s.Lue[r] = ldz_async(ru & cu, luu + i * nu + c, luu) + ldz_async(ru & c8, lu + i, lu);
    }
    s.Lux[2] = s.Lux[3] = s.Lue[2] = s.Lue[3] = 0.0;
  }
};
template <>
struct WideLoads<true> {
  __amdgpu_buffer_rsrc_t rA, rB, rXX, rX, rU, rUU, rUX;
  uint32_t oA[4], oB[4], oXe[4], oUX[2], oUU[2], oUe[2];
  uint32_t sxx, sxu, suu, nx, nu;
  __device__ WideLoads(const TileParams& P, int b, int T, int nx_, int nu_, int q, int c)
      : sxx((uint32_t)(nx_ * nx_)), sxu((uint32_t)(nx_ * nu_)), suu((uint32_t)(nu_ * nu_)), nx((uint32_t)nx_),
        nu((uint32_t)nu_) {
    constexpr uint32_t OOR = 0x80000000u;
    const size_t bt = (size_t)b * T;
    auto rsrc = [&](const double* base, size_t n) {
      return buffer_rsrc(const_cast<double*>(uniform_ptr(base)), (uint32_t)(n * sizeof(double)));
    };
    rA = rsrc(P.A + bt * sxx, (size_t)T * sxx);
    rB = rsrc(P.B + bt * sxu, (size_t)T * sxu);
    rXX = rsrc(P.lxx + bt * sxx, (size_t)T * sxx);
    rX = rsrc(P.lx + bt * nx, (size_t)T * nx);
    rU = rsrc(P.lu + bt * nu, (size_t)T * nu);
    rUU = rsrc(P.luu + bt * suu, (size_t)T * suu);
    rUX = P.lux ? rsrc(P.lux + bt * sxu, (size_t)T * sxu) : rsrc(P.A, 0);  // no lux: every load 0
    const bool cx = c < nx_, cu = c < nu_, c8 = c == 8;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int i = 4 * kk + q;
      const bool ri = i < nx_;
      oA[kk] = (ri & cx) ? (uint32_t)(i * nx_ + c) * 8 : OOR;
      oB[kk] = (ri & cu) ? (uint32_t)(i * nu_ + c) * 8 : OOR;
      oXe[kk] = (ri & c8) ? (uint32_t)i * 8 : OOR;
    }
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int i = q + 4 * r;
      const bool ru = i < nu_;
      oUX[r] = (ru & cx) ? (uint32_t)(i * nx_ + c) * 8 : OOR;
      oUU[r] = (ru & cu) ? (uint32_t)(i * nu_ + c) * 8 : OOR;
      oUe[r] = (ru & c8) ? (uint32_t)i * 8 : OOR;
    }
  }
  __device__ static __forceinline__ double ldb(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0));
  }
  __device__ __forceinline__ void load(int t, WideTile& s) const {
    const uint32_t sA = (uint32_t)t * sxx * 8, sB = (uint32_t)t * sxu * 8;
    const uint32_t sX = (uint32_t)t * nx * 8, sU = (uint32_t)t * nu * 8, sUU = (uint32_t)t * suu * 8;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      s.fA[kk] = ldb(rA, oA[kk], sA);
      s.fB[kk] = ldb(rB, oB[kk], sB);
      s.Lxx[kk] = ldb(rXX, oA[kk], sA);
      s.Lxe[kk] = ldb(rX, oXe[kk], sX);
    }
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      s.Lux[r] = ldb(rUX, oUX[r], sB);
      s.Lue[r] = ldb(rUU, oUU[r], sUU) + ldb(rU, oUe[r], sU);
    }
    s.Lux[2] = s.Lux[3] = s.Lue[2] = s.Lue[3] = 0.0;
  }
};

template <bool BUF>
__device__ bool tiles_backward_wide_wave(const TileParams& P, int b, int T, int nx, int nu,
                                         double* __restrict__ d_out, double* __restrict__ K_out,
                                         double mu, double* lds) {
  const int l = threadIdx.x & 63;
  const int c = l & 15;
  const int q = l >> 4;
  const bool cx = c < nx;
  const bool c8 = c == 8;
  const size_t bt = (size_t)b * T;
  const size_t sxx = (size_t)nx * nx;

  WideLoads<BUF> L(P, b, T, nx, nu, q, c);
  auto load = [&](int t, WideTile& s) { L.load(t, s); };

  double* Gl = lds;        // G[j][c], j < 8
  double* Hl = lds + 128;  // [H | g][j][c], j < 8, c ≤ 8
  double* tile = lds + 256;

  // terminal value function (:335-336): S = ∇²ℓ_f, s = ∇ℓ_f (column 8 of Sx)
  d4 S, Sx;
  {
    const double* lfxx = P.lfxx + (size_t)b * sxx;
    const double* lfx = P.lfx + (size_t)b * nx;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = q + 4 * r;
      S[r] = ldz_async((i < nx) & cx, lfxx + i * nx + c, lfxx);
      Sx[r] = ldz_async((i < nx) & c8, lfx + i, lfx);
    }
  }

  bool nan = false;
  double* Kb = K_out + bt * nu * nx;
  double* db = d_out + bt * nu;
  WideTile cur, nxt;
  load(T - 1, cur);
  for (int t = T - 1; t >= 0; --t) {
    load(t > 0 ? t - 1 : 0, nxt);  // prefetch

    // every product as two independent 2-MFMA chains summed by the VALU: the step is a
    // latency chain at small batch (the reference's caller fits ONE trajectory) and a
    // dependent v_mfma_f64_16x16x4 accumulation costs its full latency per link
    const d4 z4 = {0.0, 0.0, 0.0, 0.0};
    d4 YB0;
#pragma unroll
    for (int r = 0; r < 4; ++r) YB0[r] = c8 ? Sx[r] : 0.0;
    const d4 YA = mfma(S[1], cur.fA[1], mfma(S[0], cur.fA[0], z4)) + mfma(S[3], cur.fA[3], mfma(S[2], cur.fA[2], z4));
    const d4 YB = mfma(S[1], cur.fB[1], mfma(S[0], cur.fB[0], YB0)) + mfma(S[3], cur.fB[3], mfma(S[2], cur.fB[2], z4));
    // G and [H | g] first: the hand-off and the factorisation wait for them, the Z_xx and
    // Z_xe chains run in the MFMA pipe meanwhile
    const d4 Zux = mfma(cur.fB[1], YA[1], mfma(cur.fB[0], YA[0], cur.Lux)) +
                   mfma(cur.fB[3], YA[3], mfma(cur.fB[2], YA[2], z4));
    const d4 Zue = mfma(cur.fB[1], YB[1], mfma(cur.fB[0], YB[0], cur.Lue)) +
                   mfma(cur.fB[3], YB[3], mfma(cur.fB[2], YB[2], z4));
    const d4 Zxx = mfma(cur.fA[1], YA[1], mfma(cur.fA[0], YA[0], cur.Lxx)) +
                   mfma(cur.fA[3], YA[3], mfma(cur.fA[2], YA[2], z4));
    const d4 Zxe = mfma(cur.fA[1], YB[1], mfma(cur.fA[0], YB[0], cur.Lxe)) +
                   mfma(cur.fA[3], YB[3], mfma(cur.fA[2], YB[2], z4));

    // hand-off: G (rows q, q+4) and [H | g] (rows q, q+4)
    Gl[q * 16 + c] = Zux[0];
    Gl[(q + 4) * 16 + c] = Zux[1];
    Hl[q * 16 + c] = Zue[0];
    Hl[(q + 4) * 16 + c] = Zue[1];
    wave_lds_fence();
    double h[TW_NU][TW_NU];
#pragma unroll
    for (int i = 0; i < TW_NU; ++i)
#pragma unroll
      for (int k = 0; k <= i; ++k) h[i][k] = Hl[i * 16 + k];
    // rows nu..7 are padding (zero H rows and right-hand sides): give their pivots the
    // value 1 (1 − μ here, + μ in the factor), else a pivot is μ and μ = 0 makes its
    // reciprocal inf, 0·inf = NaN in the padded unknowns, which back-substitution would
    // carry into the real ones
#pragma unroll
    for (int i = 0; i < TW_NU; ++i)
      if (i >= nu) h[i][i] = 1.0 - mu;
    double xs[TW_NU], xd[TW_NU];
#pragma unroll
    for (int j = 0; j < TW_NU; ++j) {
      xs[j] = Gl[j * 16 + c];
      xd[j] = Hl[j * 16 + 8];
    }
    wave_lds_fence();

    // feedback_parameters (:207-218): (H + μI) x = [G[:, c] | g]
    LDLT<TW_NU, 1> f;  // one Newton step on each pivot's v_rcp_f64 (11 ulp)
    f.factor(h, mu);
    f.solve_n(xs);
    f.solve_n(xd);
    const double a0 = pick4(xs, q, 0), a1 = pick4(xs, q, 4);  // −K[q][c], −K[q+4][c]
    const double e0 = pick4(xd, q, 0), e1 = pick4(xd, q, 4);  // −d[q], −d[q+4]
    nan |= __builtin_isnan(a0) | __builtin_isnan(a1) | __builtin_isnan(e0) | __builtin_isnan(e1);
    {
      double* Kt = Kb + (size_t)t * nu * nx;
      double* dt = db + (size_t)t * nu;
      if (cx && q < nu) Kt[q * nx + c] = -a0;
      if (cx && q + 4 < nu) Kt[(q + 4) * nx + c] = -a1;
      if (c == 0 && q < nu) dt[q] = -e0;
      if (c == 0 && q + 4 < nu) dt[q + 4] = -e1;
    }

    // step_back (:269-270), exact rewrite: W = (H + 2μI)K = μK − G, w = μd − g
    const double w0 = fma(-mu, a0, -Zux[0]), w1 = fma(-mu, a1, -Zux[1]);
    const double v0 = c8 ? fma(-mu, e0, -Zue[0]) : 0.0;  // lane (8, q) holds g[q], g[q+4]
    const double v1 = c8 ? fma(-mu, e1, -Zue[1]) : 0.0;
    S = mfma(a1, w1, mfma(a0, w0, Zxx));
    Sx = mfma(a1, v1, mfma(a0, v0, Zxe));
    cur = nxt;

    if ((t % TB_SYM_EVERY) == 0) {
#pragma unroll
      for (int r = 0; r < 4; ++r) tile[(q + 4 * r) * 17 + c] = S[r];
      wave_lds_fence();
#pragma unroll
      for (int r = 0; r < 4; ++r) S[r] = 0.5 * (S[r] + tile[c * 17 + q + 4 * r]);
      wave_lds_fence();
    }
  }
  return __any(nan);
}

template <bool BUF>
__global__ __launch_bounds__(256) void tiles_backward_wide_kernel(TileParams P, int B, int T, int nx,
                                                                  int nu, double* __restrict__ d,
                                                                  double* __restrict__ K,
                                                                  int32_t* __restrict__ status,
                                                                  double mu) {
  __shared__ __attribute__((aligned(16))) double lds[4 * TW_LDS];
  const int w = threadIdx.x >> 6;
  const int b = blockIdx.x * 4 + w;
  if (b >= B) return;
  const bool nan = tiles_backward_wide_wave<BUF>(P, b, T, nx, nu, d, K, mu, lds + w * TW_LDS);
  if (status && (threadIdx.x & 63) == 0) status[b] = nan ? ILQR_TRAJ_NAN : ILQR_TRAJ_OK;
}

bool tiles_narrow(int nx, int nu) { return nx >= 1 && nx <= 12 && nu >= 1 && nu <= 4; }

}  // namespace

// every state dimension 1..12 with 1..4 inputs in one MFMA tile (compiled per shape);
// up to nx = 16, nu = 8 on the tiled wide kernel (run-time dimensions)
bool tiles_supported(int nx, int nu) {
  return tiles_narrow(nx, nu) || (nx >= 1 && nx <= TW_NX && nu >= 1 && nu <= TW_NU);
}

hipError_t launch_tiles_backward(int nx, int nu, const TileParams& p, int B, int T, double* d,
                                 double* K, int32_t* status, double mu, hipStream_t s) {
  const int grid = (B + 3) / 4;
  if (!tiles_narrow(nx, nu)) {
    if (!tiles_supported(nx, nu)) return hipErrorInvalidValue;
    if (B >= TW_BUF_MIN_B)
      tiles_backward_wide_kernel<true><<<grid, 256, 0, s>>>(p, B, T, nx, nu, d, K, status, mu);
    else
      tiles_backward_wide_kernel<false><<<grid, 256, 0, s>>>(p, B, T, nx, nu, d, K, status, mu);
    return hipGetLastError();
  }
#define ILQR_TILES_CASE(NXV, NUV)                                                              \
  if (nx == NXV && nu == NUV) {                                                                \
    tiles_backward_kernel<NXV, NUV><<<grid, 256, 0, s>>>(p, B, T, d, K, status, mu);          \
    return hipGetLastError();                                                                  \
  }
#define ILQR_TILES_NU(NXV) ILQR_TILES_CASE(NXV, 1) ILQR_TILES_CASE(NXV, 2) ILQR_TILES_CASE(NXV, 3) ILQR_TILES_CASE(NXV, 4)
  ILQR_TILES_NU(1) ILQR_TILES_NU(2) ILQR_TILES_NU(3) ILQR_TILES_NU(4) ILQR_TILES_NU(5) ILQR_TILES_NU(6)
  ILQR_TILES_NU(7) ILQR_TILES_NU(8) ILQR_TILES_NU(9) ILQR_TILES_NU(10) ILQR_TILES_NU(11) ILQR_TILES_NU(12)
#undef ILQR_TILES_NU
#undef ILQR_TILES_CASE
  return hipErrorInvalidValue;
}

}  // namespace ilqr
