// Device helpers shared by the HIP translation units (gfx950 only). Private header.
#pragma once
#include <hip/hip_runtime.h>

namespace ilqr {
namespace {

typedef double d4 __attribute__((ext_vector_type(4)));
typedef unsigned u2v __attribute__((ext_vector_type(2)));

constexpr int WAVES_PER_WG = 4;   // trajectories per workgroup
constexpr int YT_OFF = 96 + 16 * 17 + 64;  // (the VALU-product variant's Y tile: kept, the LDS size measured)
constexpr int BW_LDS = YT_OFF + 16 * 14;   // doubles of backward scratch per wave: [G|H] rows, g row, zero, S tile, junk row, Y tile
constexpr int SYM_EVERY = 8;          // symmetrise S every this many steps

__device__ __forceinline__ d4 mfma(double a, double b, d4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// all-reduce over lanes {l, l^16} with v_permlane16_swap (gfx950): one instruction
// per dword gives every lane both its own and its partner row's value.
__device__ __forceinline__ double xor16_sum(double v) {
  u2v p = __builtin_bit_cast(u2v, v);
  auto lo = __builtin_amdgcn_permlane16_swap(p.x, p.x, false, false);
  auto hi = __builtin_amdgcn_permlane16_swap(p.y, p.y, false, false);
  u2v a = {lo[0], hi[0]};
  u2v b = {lo[1], hi[1]};
  return __builtin_bit_cast(double, a) + __builtin_bit_cast(double, b);
}
__device__ __forceinline__ double xor32_sum(double v) {
  u2v p = __builtin_bit_cast(u2v, v);
  auto lo = __builtin_amdgcn_permlane32_swap(p.x, p.x, false, false);
  auto hi = __builtin_amdgcn_permlane32_swap(p.y, p.y, false, false);
  u2v a = {lo[0], hi[0]};
  u2v b = {lo[1], hi[1]};
  return __builtin_bit_cast(double, a) + __builtin_bit_cast(double, b);
}
// sum over the four lanes {c, c+16, c+32, c+48} of a column
__device__ __forceinline__ double colsum4(double v) { return xor32_sum(xor16_sum(v)); }

// sum over the 16 lanes of a row (one forward group)
__device__ __forceinline__ double rowsum16(double v) {
#pragma unroll
  for (int m = 8; m >= 1; m >>= 1) v += __shfl_xor(v, m, 16);
  return v;
}

// lane 0 of each quad to the whole quad (DPP quad_perm [0,0,0,0]), a double: in the
// 4-block MFMA layout (lane 16ρ + 4β + κ) the quad is κ = 0..3, so this turns column 0
// of a block into a replicated vector
__device__ __forceinline__ double dpp_quad_bcast0(double x) {
  typedef unsigned u2v_ __attribute__((ext_vector_type(2)));
  const u2v_ p = __builtin_bit_cast(u2v_, x);
  const u2v_ q = {(unsigned)__builtin_amdgcn_mov_dpp((int)p.x, 0x00, 0xF, 0xF, true),
                  (unsigned)__builtin_amdgcn_mov_dpp((int)p.y, 0x00, 0xF, 0xF, true)};
  return __builtin_bit_cast(double, q);
}

// Cross-lane LDS hand-off inside one wave: DS ops of a wave execute in order, so
// only the compiler must be kept from moving LDS accesses across this point.
__device__ __forceinline__ void wave_lds_fence() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// 1/x: v_rcp_f64 (≈2^-24 relative on gfx950) + NEWTON Newton steps. Measured by
// tools/rcp_test.hip: 0 steps 2.5e8 ulp, 1 step 11 ulp, 2 steps 0 ulp. The LQ
// backward's pivots use one step (11 ulp ≈ 2.4e-15 relative: far inside the parity
// tolerances; the factorisation is the kernel's critical path, tools/ablate_bw).
// 64-bit global store without an exec branch: a raw buffer store whose offset is
// pushed out of range (dropped by the hardware bounds check) on inactive lanes.
// a pointer the compiler must treat as wave-uniform (its value is, but divergence
// analysis lost it): both halves through v_readfirstlane
template <class P>
__device__ __forceinline__ P* uniform_ptr(P* p) {
  const uint64_t v = (uint64_t)(uintptr_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return (P*)(uintptr_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buffer_rsrc(void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(base, 0, (int)bytes, 0x00020000);  // gfx9 dword3
}
__device__ __forceinline__ void store_or_drop(double v, __amdgpu_buffer_rsrc_t r, bool ok,
                                              uint32_t byte_off) {
  typedef unsigned u2v_ __attribute__((ext_vector_type(2)));
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v_, v), r,
                                        ok ? byte_off : 0x80000000u, 0, 0);
}

template <int NEWTON = 2>
__device__ __forceinline__ double rcp(double x) {
  double r = __builtin_amdgcn_rcp(x);
#pragma unroll
  for (int i = 0; i < NEWTON; ++i) {
    const double e = fma(-x, r, 1.0);
    r = fma(r, e, r);
  }
  return r;
}

// Load-or-zero without a branch: the address is clamped to `safe` when !ok so
// the load is unconditional (no exec-masked load + vmcnt(0) per element).
__device__ __forceinline__ double ldz(bool ok, const double* p, const double* safe) {
  const double v = *(ok ? p : safe);
  return ok ? v : 0.0;
}

// ldz for loads that must stay in flight (a prefetch): the address is opaque to the
// optimiser, which otherwise may turn the select back into an exec-masked load in a
// branch whose join waits (vmcnt) for every load in flight — the tiles kernels' whole
// prefetch, at the top of each step
__device__ __forceinline__ double ldz_async(bool ok, const double* p, const double* safe) {
  const double* a = ok ? p : safe;
  asm volatile("" : "+v"(a));
  typedef __attribute__((address_space(1))) const double gdouble;  // a global load, not flat
  const double v = *(gdouble*)a;
  return ok ? v : 0.0;
}

// (H + μI) = L D Lᵀ (no pivoting; H symmetric, lower triangle read) and a solve
// with a d4 right-hand side; NU ≤ 4, entries ≥ NU unused.
template <int NU, int NEWTON = 2>
struct LDLT {
  double l[NU][NU];
  double dinv[NU];
  // ADD_MU = false: h already holds H + μI (the caller folded μ into H's accumulator)
  template <bool ADD_MU = true>
  __device__ __forceinline__ void factor(const double (&h)[NU][NU], double mu) {
    double t[NU][NU];  // t[i][k] = L[i][k] · D[k]
#pragma unroll
    for (int k = 0; k < NU; ++k) {
      double dk = ADD_MU ? h[k][k] + mu : h[k][k];
#pragma unroll
      for (int p = 0; p < k; ++p) dk = fma(-l[k][p], t[k][p], dk);
      dinv[k] = rcp<NEWTON>(dk);
#pragma unroll
      for (int i = k + 1; i < NU; ++i) {
        double v = h[i][k];
#pragma unroll
        for (int p = 0; p < k; ++p) v = fma(-l[i][p], t[k][p], v);
        t[i][k] = v;
        l[i][k] = v * dinv[k];
      }
    }
  }
  __device__ __forceinline__ d4 solve(d4 x) const {
#pragma unroll
    for (int i = 0; i < NU; ++i)
#pragma unroll
      for (int p = 0; p < i; ++p) x[i] = fma(-l[i][p], x[p], x[i]);
#pragma unroll
    for (int i = 0; i < NU; ++i) x[i] *= dinv[i];
#pragma unroll
    for (int i = NU - 1; i >= 0; --i)
#pragma unroll
      for (int p = i + 1; p < NU; ++p) x[i] = fma(-l[p][i], x[p], x[i]);
    return x;
  }
  // in place, a right-hand side of NU entries (the wide tiles kernel, NU = 8)
  __device__ __forceinline__ void solve_n(double (&x)[NU]) const {
#pragma unroll
    for (int i = 0; i < NU; ++i)
#pragma unroll
      for (int p = 0; p < i; ++p) x[i] = fma(-l[i][p], x[p], x[i]);
#pragma unroll
    for (int i = 0; i < NU; ++i) x[i] *= dinv[i];
#pragma unroll
    for (int i = NU - 1; i >= 0; --i)
#pragma unroll
      for (int p = i + 1; p < NU; ++p) x[i] = fma(-l[p][i], x[p], x[i]);
  }
};

}  // namespace
}  // namespace ilqr
