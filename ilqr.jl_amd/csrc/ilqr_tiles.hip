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
      s.fB[kk] = ldz(ri && cx, A + ii * NX + ci, A) + ldz(ri && cu, Bm + ii * NU + cj, Bm);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = q + 4 * r;
      const bool rx = i < NX, ru = i >= NX && i < NX + NU;
      const int ix = rx ? i : 0, iu = ru ? i - NX : 0;
      const double xx = ldz(rx && cx, lxx + ix * NX + ci, lxx);
      const double xu = ldz(rx && cu, lux + cj * NX + ix, lux);  // L[i][NX+j] = 𝐏[j][i]
      const double ux = ldz(ru && cx, lux + iu * NX + ci, lux);  // L[NX+j][c] = 𝐏[j][c]
      const double uu = ldz(ru && cu, luu + iu * NU + cj, luu);
      s.Lc[r] = xx + wux * (xu + ux) + uu;
    }
    s.lv = ldz(cx, lx0 + (size_t)t * NX + ci, lx0) + ldz(cu, lu0 + (size_t)t * NU + cj, lu0);
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
      Sp[r] = ldz(rx && cx, lfxx + ix * NX + ci, lfxx) + ldz(rx && c == SROW, lfx + ix, lfx);
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

}  // namespace

// every state dimension 1..12 with 1..4 inputs (nx + nu ≤ 16, nu ≤ 4: one MFMA tile)
bool tiles_supported(int nx, int nu) { return nx >= 1 && nx <= 12 && nu >= 1 && nu <= 4; }

hipError_t launch_tiles_backward(int nx, int nu, const TileParams& p, int B, int T, double* d,
                                 double* K, int32_t* status, double mu, hipStream_t s) {
  const int grid = (B + 3) / 4;
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
