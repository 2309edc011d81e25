// (Round 3: the ABL bits / -DILQR_* switches this probe uses exist only in the tree
// tools/archive/ablation/restore_tree.sh restores; build it there.)
// Probe for backward-kernel schedules (not part of the product): times the v7
// four-trajectories-per-wave kernel (lq_backward4_kernel) against the v8 schedule
// variants (lq_backward4_v8_kernel) at B=4096, T=100 on random stable LQ problems,
// checks the variants return v7's bits, and (argv[1] = "quad") their error against the
// symmetrised C oracle on tools/quad256.bin (tools/dump_quad.py).
#include "../ilqr.jl_amd/csrc/ilqr_lq.hip"
#include "../ilqr.jl_amd/csrc/ilqr_bw4.hip"
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <vector>
using namespace ilqr;

// the v8 schedule variants (probe-only: none is faster than v7)
namespace ilqr {
namespace {
// v8 schedule of the same recursion (identical arithmetic, so identical bits): the
// step is one basic block from the S hand-off to the gain solve. The L z branch runs
// first; Y's B column and H go first so that H's LDS round trip overlaps the 27 MFMAs
// of Y's A columns; after the read, the (H + μI) factor's dependent VALU chain shares
// its block with the 41 independent MFMAs of G, Qxx and the gradient, which the
// scheduler interleaves into the factor's latency gaps (v7 issued them before the
// read, leaving the factor to run alone on the critical path).
// SG bits (probe only): 1 = ask the scheduler for explicit VALU/MFMA alternation;
// 2 = record the loop's shader-clock and 100 MHz real-time deltas into clk[0..1].
template <int SG = 0>
__device__ unsigned lq_backward4_wave_v8(const LQParams& P, int b0, int B, unsigned active, int T,
                                         const double* __restrict__ x, const double* __restrict__ u,
                                         double* __restrict__ d_out, double* __restrict__ K_out,
                                         double mu, double* lds, unsigned long long* clk = nullptr) {
  constexpr int NX = 12, NU = 4;
  b0 = __builtin_amdgcn_readfirstlane(b0);
  const int l = threadIdx.x & 63;
  const int rho = l >> 4;
  const int beta = (l >> 2) & 3;
  const int kap = l & 3;
  const int b = b0 + beta;
  const bool live = b < B && ((active >> beta) & 1u);
  const int bc = b < B ? b : B - 1;
  const int nslot = B - b0 < 4 ? B - b0 : 4;

  const double* Ab = P.A + (size_t)bc * NX * NX;
  const double* Bb = P.B + (size_t)bc * NX * NU;
  const double* Qb = P.Q + (size_t)bc * NX * NX;
  const double* Rb = P.R + (size_t)bc * NU * NU;
  const double* Qfb = P.Qf + (size_t)bc * NX * NX;

  double F[3][4], L[3][3];
#pragma unroll
  for (int K = 0; K < 3; ++K) {
    const int r = 4 * K + rho;
#pragma unroll
    for (int J = 0; J < 3; ++J) F[K][J] = Ab[r * NX + 4 * J + kap];
    F[K][3] = Bb[r * NU + kap];
#pragma unroll
    for (int I = 0; I < 3; ++I) L[K][I] = Qb[r * NX + 4 * I + kap] + Qb[(4 * I + kap) * NX + r];
  }
  const double LR = Rb[rho * NU + kap] + Rb[kap * NU + rho];
  const int tr_src = (16 * kap + 4 * beta + rho) * 4;

  double S[3][3], s[3];
  {
    const double* xN = x + ((size_t)bc * (T + 1) + T) * NX;
    double xr[3];
#pragma unroll
    for (int K = 0; K < 3; ++K) {
      const int r = 4 * K + rho;
      xr[K] = xN[r];
#pragma unroll
      for (int I = 0; I < 3; ++I) S[K][I] = Qfb[r * NX + 4 * I + kap] + Qfb[(4 * I + kap) * NX + r];
    }
#pragma unroll
    for (int I = 0; I < 3; ++I) {
      double v = 0.0;
#pragma unroll
      for (int K = 0; K < 3; ++K) v = mf4(S[K][I], xr[K], v);
      s[I] = v;
    }
  }

  const auto rX = buffer_rsrc(const_cast<double*>(x) + (size_t)b0 * (T + 1) * NX, (uint32_t)(nslot * (T + 1) * NX * 8));
  const auto rU = buffer_rsrc(const_cast<double*>(u) + (size_t)b0 * T * NU, (uint32_t)(nslot * T * NU * 8));
  const auto rK = buffer_rsrc(K_out + (size_t)b0 * T * NU * NX, (uint32_t)(nslot * T * NU * NX * 8));
  const auto rD = buffer_rsrc(d_out + (size_t)b0 * T * NU, (uint32_t)(nslot * T * NU * 8));
  const uint32_t DEAD = 0x80000000u;
  const uint32_t kv = live ? (uint32_t)((beta * T * NU * NX + rho * NX + kap) * 8) : DEAD;
  const uint32_t dv = (live && kap == 0) ? (uint32_t)((beta * T * NU + rho) * 8) : DEAD;

  double Lzq[4] = {0.0, 0.0, 0.0, 0.0}, zq[4];
  // z for the next four steps. ZDMA: streamed HBM → LDS by the wave
  // (global_load_lds_dwordx4, two instructions: [slot][step κ][x 12 | u 4]) and read back
  // after an explicit vmcnt wait that lets the 16 gain stores issued since stay in
  // flight. With register loads the compiler's loop-carried vmcnt wait also drained
  // those stores every fourth step (gfx9 counts stores in vmcnt): ≈9 µs per launch.
  constexpr bool ZDMA = (SG & 8) != 0;
  double* const Zl = lds + 64;  // 256 doubles: [β][κ][16]
  const char* zsrc[2];
  {
    const int bz = b0 + (beta < nslot ? beta : nslot - 1);  // absent slots read a present one
    (void)bz;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = 64 * i + l;               // 16-byte chunk: slot c/32, step (c/8)%4, pair c%8
      const int cb = c >> 5, ck = (c >> 3) & 3, cp = c & 7;
      const int bb = b0 + (cb < nslot ? cb : nslot - 1);
      zsrc[i] = cp < 6 ? reinterpret_cast<const char*>(x + (size_t)bb * (T + 1) * NX + 2 * cp)
                       : reinterpret_cast<const char*>(u + (size_t)bb * T * NU + 2 * (cp - 6));
      (void)ck;
    }
  }
  const uint32_t zl_lds = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) double*)Zl;
  auto dma_zq = [&](int t0) {  // steps t0 .. t0-3 (clamped at 0)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = 64 * i + l, ck = (c >> 3) & 3, cp = c & 7;
      const int tz = t0 - ck > 0 ? t0 - ck : 0;
      const char* src = zsrc[i] + (size_t)tz * (cp < 6 ? NX * 8 : NU * 8);
      asm volatile("global_load_lds_dwordx4 %0, off" ::"v"(src), "{m0}"(zl_lds + 1024u * i) : "memory");
    }
  };
  auto load_zq = [&](int t0) {
    if constexpr (ZDMA) {
      dma_zq(t0);
    } else {
      const int tz = t0 - kap > 0 ? t0 - kap : 0;
      const uint32_t xo = (uint32_t)(((beta * (T + 1) + tz) * NX + rho) * 8);
      const uint32_t uo = (uint32_t)(((beta * T + tz) * NU + rho) * 8);
#pragma unroll
      for (int K = 0; K < 3; ++K) zq[K] = buf_ld(rX, xo + 32 * K, 0);
      zq[3] = buf_ld(rU, uo, 0);
    }
  };
  auto read_zq = [&] {  // ZDMA: this lane's z entries of the landed group
    // at most the 16 gain stores of the last four steps are younger than the DMA
    __builtin_amdgcn_s_waitcnt((16 & 15) | (7 << 4) | (15 << 8) | ((16 >> 4) << 14));
    asm volatile("" ::: "memory");
    const double* zr = Zl + beta * 64 + kap * 16;
#pragma unroll
    for (int K = 0; K < 3; ++K) zq[K] = zr[4 * K + rho];
    zq[3] = zr[12 + rho];
  };
  load_zq(T - 1);

  double* Hl = lds + beta * 16;
  double Klast[4];
  __builtin_amdgcn_s_waitcnt(0);
  unsigned long long c0 = 0, r0 = 0;
  if constexpr ((SG & 2) != 0) {
    c0 = __builtin_readcyclecounter();
    r0 = __builtin_amdgcn_s_memrealtime();
  }

  constexpr bool DEFER = (SG & 4) != 0;  // gains stored one step late, off the critical path
  double Kst[4] = {0.0, 0.0, 0.0, 0.0};
  for (int t = T - 1; t >= 0; --t) {
    // L z for steps t .. t-3 (column κ = step t-κ) every fourth step, then the next
    // four steps' z — the step's only branch, ahead of the S-dependent block
    const int j = (T - 1 - t) & 3;
    if constexpr (ZDMA) {
      if (j == 0) read_zq();
    }
    if constexpr (DEFER) {
      if (t < T - 1) {  // step t+1's gains, long computed: no MFMA→store hazard wait
#pragma unroll
        for (int J = 0; J < 3; ++J) buf_st(Kst[J], rK, kv + 32 * J, (uint32_t)((t + 1) * NU * NX * 8));
        buf_st(Kst[3], rD, dv, (uint32_t)((t + 1) * NU * 8));
      }
    }
    if (j == 0) {
#pragma unroll
      for (int I = 0; I < 3; ++I) {
        double v = 0.0;
#pragma unroll
        for (int K = 0; K < 3; ++K) v = mf4(L[K][I], zq[K], v);
        Lzq[I] = v;
      }
      Lzq[3] = mf4(LR, zq[3], 0.0);
      load_zq(t - 4);
    }
    // Y's B column, then H = R + Rᵀ + BᵀSB → LDS
    double Y[3][4];
#pragma unroll
    for (int I = 0; I < 3; ++I) {
      double v = 0.0;
#pragma unroll
      for (int K = 0; K < 3; ++K) v = mf4(S[K][I], F[K][3], v);
      Y[I][3] = v;
    }
    double H = LR;
#pragma unroll
    for (int K = 0; K < 3; ++K) H = mf4(F[K][3], Y[K][3], H);
    Hl[rho * 4 + kap] = H;
    // Y's A columns cover the LDS round trip
#pragma unroll
    for (int J = 0; J < 3; ++J)
#pragma unroll
      for (int I = 0; I < 3; ++I) {
        double v = 0.0;
#pragma unroll
        for (int K = 0; K < 3; ++K) v = mf4(S[K][I], F[K][J], v);
        Y[I][J] = v;
      }
    wave_lds_fence();
    double h[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int k = 0; k <= i; ++k) h[i][k] = Hl[i * 4 + k];
    // (H + μI) = L D Lᵀ in every lane of the slot, M = L⁻¹, this lane's M[ρ][κ], D⁻¹[ρ]
    LDLT<4, 1> f;
    f.factor(h, mu);
    double Mf[4][4];
    Mf[1][0] = -f.l[1][0];
    Mf[2][1] = -f.l[2][1];
    Mf[2][0] = fma(f.l[2][1], f.l[1][0], -f.l[2][0]);
    Mf[3][2] = -f.l[3][2];
    Mf[3][1] = fma(f.l[3][2], f.l[2][1], -f.l[3][1]);
    Mf[3][0] = fma(-f.l[3][2], Mf[2][0], fma(-f.l[3][1], Mf[1][0], -f.l[3][0]));
    double Mn = rho == kap ? 1.0 : 0.0;
#pragma unroll
    for (int i = 1; i < 4; ++i)
#pragma unroll
      for (int jj = 0; jj < i; ++jj) Mn = (rho == i && kap == jj) ? Mf[i][jj] : Mn;
    double dsel = f.dinv[0];
#pragma unroll
    for (int i = 1; i < 4; ++i) dsel = rho == i ? f.dinv[i] : dsel;
    const double Mt = lane_perm(Mn, tr_src), Mnd = Mn * dsel;
    // independent of the factor: the gradient [lx + Aᵀs | lu + Bᵀs], G = BᵀSA, Qxx
    double gv[4];
    {
      const int src = ((l & ~3) | j) * 4;
#pragma unroll
      for (int I = 0; I < 4; ++I) {
        double v = lane_perm(Lzq[I], src);
#pragma unroll
        for (int K = 0; K < 3; ++K) v = mf4(F[K][I], s[K], v);
        gv[I] = v;
      }
    }
    double G[3], Z[3][3];
#pragma unroll
    for (int J = 0; J < 3; ++J) {
      double v = 0.0;
#pragma unroll
      for (int K = 0; K < 3; ++K) v = mf4(F[K][3], Y[K][J], v);
      G[J] = v;
    }
#pragma unroll
    for (int I = 0; I < 3; ++I)
#pragma unroll
      for (int J = I; J < 3; ++J) {
        double v = L[I][J];
#pragma unroll
        for (int K = 0; K < 3; ++K) v = mf4(F[K][I], Y[K][J], v);
        Z[I][J] = v;
      }
    if constexpr ((SG & 1) != 0) {
      // alternate one VALU op with one MFMA through the factor's chain
#pragma unroll
      for (int q = 0; q < 40; ++q) {
        __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      }
    }
    // K_aug = −(D⁻¹M)ᵀ (M [G | g]) (two triangular sweeps as MFMA stages)
    double Kg[4];
#pragma unroll
    for (int J = 0; J < 4; ++J) Kg[J] = mf4n(Mnd, mf4(Mt, J < 3 ? G[J] : gv[3], 0.0), 0.0);
    if constexpr (DEFER) {
#pragma unroll
      for (int J = 0; J < 4; ++J) Kst[J] = Kg[J];
    } else {
#pragma unroll
      for (int J = 0; J < 3; ++J) buf_st(Kg[J], rK, kv + 32 * J, (uint32_t)(t * NU * NX * 8));
      buf_st(Kg[3], rD, dv, (uint32_t)(t * NU * 8));
    }
    // step_back: [S | s] = [Qxx | lx + Aᵀs] − K_augᵀ W, W = μ K_aug − [G | g]
    double W[4];
#pragma unroll
    for (int J = 0; J < 3; ++J) W[J] = fma(mu, Kg[J], -G[J]);
    W[3] = fma(mu, Kg[3], -gv[3]);
#pragma unroll
    for (int I = 0; I < 3; ++I) {
#pragma unroll
      for (int J = I; J < 3; ++J) S[I][J] = mf4n(Kg[I], W[J], Z[I][J]);
      s[I] = mf4n(Kg[I], W[3], gv[I]);
    }
    if ((t % SYM_EVERY) == 0) {
#pragma unroll
      for (int I = 0; I < 3; ++I) S[I][I] = 0.5 * (S[I][I] + lane_perm(S[I][I], tr_src));
    }
#pragma unroll
    for (int I = 0; I < 3; ++I)
#pragma unroll
      for (int J = I + 1; J < 3; ++J) S[J][I] = lane_perm(S[I][J], tr_src);
#pragma unroll
    for (int J = 0; J < 4; ++J) Klast[J] = Kg[J];
  }
  if constexpr (DEFER) {  // step 0's gains
#pragma unroll
    for (int J = 0; J < 3; ++J) buf_st(Kst[J], rK, kv + 32 * J, 0u);
    buf_st(Kst[3], rD, dv, 0u);
  }
  if constexpr ((SG & 2) != 0) {
    __builtin_amdgcn_s_waitcnt(0);
    const unsigned long long c1 = __builtin_readcyclecounter(), r1 = __builtin_amdgcn_s_memrealtime();
    if (clk && l == 0) { clk[0] = c1 - c0; clk[1] = r1 - r0; }
  }
  bool nan = false;
#pragma unroll
  for (int J = 0; J < 4; ++J) nan |= __builtin_isnan(Klast[J]);
  const unsigned long long nb = __ballot(nan);
  unsigned r = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) r |= (nb & slot_lanes(q)) ? (1u << q) : 0u;
  return r;
}

template <int SG = 0>
__global__ __launch_bounds__(256) void lq_backward4_v8_kernel(LQParams P, int B, int T,
                                                              const double* __restrict__ x,
                                                              const double* __restrict__ u,
                                                              double* __restrict__ d,
                                                              double* __restrict__ K,
                                                              int32_t* __restrict__ status, double mu,
                                                              unsigned long long* clk = nullptr) {
  __shared__ __attribute__((aligned(16))) double lds[BW4_WAVES * BW4_LDS];
  const int w = threadIdx.x >> 6;
  const int b0 = (blockIdx.x * BW4_WAVES + w) * BW4_SLOTS;
  if (b0 >= B) return;
  const unsigned nan = lq_backward4_wave_v8<SG>(P, b0, B, 0xFu, T, x, u, d, K, mu, lds + w * BW4_LDS,
                                                clk ? clk + 2 * (b0 / BW4_SLOTS) : nullptr);
  const int l = threadIdx.x & 63;
  if (status && l < BW4_SLOTS && b0 + l < B) status[b0 + l] = ((nan >> l) & 1u) ? ILQR_TRAJ_NAN : ILQR_TRAJ_OK;
}

}  // namespace
}  // namespace ilqr
#define CK(x) do { hipError_t e=(x); if(e!=hipSuccess){printf("err %s line %d\n",hipGetErrorString(e),__LINE__); return 1;} } while(0)

int main(int argc, char** argv) {
  const bool quad = argc > 1 && std::string(argv[1]) == "quad";
  const int B = quad ? 256 : (argc > 1 ? atoi(argv[1]) : 4096), T = 100, n = 12, m = 4;
  std::mt19937_64 g(1);
  std::uniform_real_distribution<double> U(-1, 1);
  auto mk = [&](size_t N, double sc, bool eye, int dim) {
    std::vector<double> v(N);
    for (auto& e : v) e = sc * U(g);
    if (eye) for (size_t b = 0; b < N / (dim * dim); ++b) for (int i = 0; i < dim; ++i) v[b * dim * dim + i * dim + i] += 1.0;
    return v;
  };
  auto A = mk((size_t)B * n * n, 0.02, true, n), Bm = mk((size_t)B * n * m, 0.1, false, 1);
  auto Q = mk((size_t)B * n * n, 0.01, true, n), R = mk((size_t)B * m * m, 0.01, true, m), Qf = mk((size_t)B * n * n, 0.01, true, n);
  auto x = mk((size_t)B * (T + 1) * n, 1.0, false, 1), u = mk((size_t)B * T * m, 0.1, false, 1);
  std::vector<double> Kor((size_t)B * T * m * n), dor((size_t)B * T * m);
  if (quad) {
    FILE* f = fopen("tools/quad256.bin", "rb");
    if (!f) { printf("tools/quad256.bin missing (python tools/dump_quad.py)\n"); return 1; }
    for (auto* v : {&A, &Bm, &Q, &R, &Qf, &x, &u, &Kor, &dor})
      if (fread(v->data(), 8, v->size(), f) != v->size()) { printf("short read\n"); return 1; }
    fclose(f);
  }
  auto up = [&](std::vector<double>& v) { double* p; hipMalloc(&p, v.size() * 8); hipMemcpy(p, v.data(), v.size() * 8, hipMemcpyHostToDevice); return p; };
  LQParams P{up(A), up(Bm), up(Q), up(R), up(Qf)};
  double *xd = up(x), *ud = up(u), *d, *K;
  int32_t* st;
  CK(hipMalloc(&d, (size_t)B * T * m * 8)); CK(hipMalloc(&K, (size_t)B * T * m * n * 8)); CK(hipMalloc(&st, B * 4));
  std::vector<double> K7((size_t)B * T * m * n), d7((size_t)B * T * m), Kv(K7.size()), dv(d7.size());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto time = [&](const char* name, auto launch) -> int {
    for (int i = 0; i < 200; ++i) launch();
    CK(hipDeviceSynchronize());
    const int R = 50;
    CK(hipEventRecord(e0));
    for (int i = 0; i < R; ++i) launch();
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-40s B=%d %8.2f us\n", name, B, 1000.0 * ms / R);
    return 0;
  };
  auto rel = [](const std::vector<double>& a, const std::vector<double>& r, const char* nm) {
    double mx = 0, ref = 0; size_t bad = 0;
    for (size_t i = 0; i < a.size(); ++i) {
      if (a[i] != a[i]) { ++bad; continue; }
      mx = fmax(mx, fabs(a[i] - r[i])); ref = fmax(ref, fabs(r[i]));
    }
    printf("  %s: rel %.3e NaN %zu\n", nm, mx / ref, bad);
  };
  auto v7 = [&] { lq_backward4_kernel<0><<<bw4_grid(B), 256, 0, 0>>>(P, B, T, xd, ud, d, K, st, 0.01); };
  if (time("v7 lq_backward4_kernel", v7)) return 1;
  CK(hipMemcpy(K7.data(), K, K7.size() * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(d7.data(), d, d7.size() * 8, hipMemcpyDeviceToHost));
  if (quad) { rel(K7, Kor, "v7 K vs oracle"); rel(d7, dor, "v7 d vs oracle"); }
  auto check = [&](const char* nm) -> int {
    CK(hipMemcpy(Kv.data(), K, Kv.size() * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(dv.data(), d, dv.size() * 8, hipMemcpyDeviceToHost));
    const bool same = !memcmp(Kv.data(), K7.data(), Kv.size() * 8) && !memcmp(dv.data(), d7.data(), dv.size() * 8);
    printf("  %s: bits %s v7\n", nm, same ? "==" : "!=");
    if (!same) { rel(Kv, K7, "K vs v7"); rel(dv, d7, "d vs v7"); }
    if (quad) { rel(Kv, Kor, "K vs oracle"); rel(dv, dor, "d vs oracle"); }
    return 0;
  };
#define VAR8(SGV, NAME) do { \
    CK(hipMemset(K, 0xff, K7.size() * 8)); CK(hipMemset(d, 0xff, d7.size() * 8)); \
    auto f = [&] { lq_backward4_v8_kernel<SGV><<<bw4_grid(B), 256, 0, 0>>>(P, B, T, xd, ud, d, K, st, 0.01); }; \
    if (time(NAME, f)) return 1; \
    if (check(NAME)) return 1; } while (0)
  for (int rep = 0; rep < 2; ++rep) {
    if (time("v7 lq_backward4_kernel", v7)) return 1;
    VAR8(0, "v8 reordered");
    VAR8(8, "v8 reordered + z via LDS DMA");
  }
  // ablations of the v7 kernel (wrong gains; time only): what each part costs
#define ABLV7(ABLV, NAME) do { \
    auto f = [&] { lq_backward4_kernel<ABLV><<<bw4_grid(B), 256, 0, 0>>>(P, B, T, xd, ud, d, K, st, 0.01); }; \
    if (time(NAME, f)) return 1; } while (0)
  if (!quad) {
    ABLV7(0, "v7 (reference point)");
    ABLV7(1, "v7 - factorisation (ABL 1)");
    ABLV7(2, "v7 - S transposes (ABL 2)");
    ABLV7(4, "v7 - gradient (ABL 4)");
    ABLV7(8, "v7 - gain stores (ABL 8)");
    ABLV7(128, "v7 - diagonal symmetrisation (ABL 128)");
    ABLV7(1 | 2, "v7 - factor - transposes");
    ABLV7(1 | 2 | 4 | 8, "v7 - factor - transposes - grad - stores");
  }
  // cycles per step and the clock, from the waves' own counters
  {
    unsigned long long* clk;
    const int nw = (B + 3) / 4;
    CK(hipMalloc(&clk, 16 * nw));
    for (int i = 0; i < 100; ++i) v7();
    lq_backward4_v8_kernel<10><<<bw4_grid(B), 256, 0, 0>>>(P, B, T, xd, ud, d, K, st, 0.01, clk);
    CK(hipDeviceSynchronize());
    std::vector<unsigned long long> c(2 * nw);
    CK(hipMemcpy(c.data(), clk, 16 * nw, hipMemcpyDeviceToHost));
    double cyc = 0, rt = 0, cmax = 0;
    for (int w = 0; w < nw; ++w) { cyc += c[2 * w]; rt += c[2 * w + 1]; cmax = fmax(cmax, (double)c[2 * w]); }
    cyc /= nw; rt /= nw;
    printf("v8 loop: %.0f shader cycles (max %.0f) = %.1f cycles/step, %.2f us at 100 MHz real time -> %.3f GHz\n",
           cyc, cmax, cyc / T, rt / 100.0, cyc / (rt / 100.0) / 1000.0);
  }
  return 0;
}
