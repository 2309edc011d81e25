/*
 * ilqr_ref.c — C restatement of aabouman/iLQR.jl's hot path for the LQ problem
 * family — TEST INFRASTRUCTURE ONLY (checker for the GPU parity tests and the
 * bench's cpu_baseline leg; never linked into the product).
 *
 * The reference is pure Julia (not buildable here: no Julia toolchain), so this
 * is a line-by-line restatement of its algorithm with the LQ callbacks
 *   dynamicsf(x,u) = A x + B u, immediate_cost(x,u) = xᵀQx + uᵀRu, final_cost(x) = xᵀQf x
 * whose ForwardDiff derivatives are exact:
 *   linearize_dynamics            (src/backward_pass.jl:25-40)   → A, B
 *   immediate_cost_quadratization (src/backward_pass.jl:81-109)  → 𝐪=(Q+Qᵀ)x, 𝐫=(R+Rᵀ)u, 𝐐=Q+Qᵀ, 𝐏=0, 𝐑=R+Rᵀ
 *   final_cost_quadratization     (src/backward_pass.jl:134-153) → (Qf+Qfᵀ)x, Qf+Qfᵀ
 *   optimal_controller_param      (src/backward_pass.jl:177-186)
 *   feedback_parameters           (src/backward_pass.jl:207-218) H_reg = H + 0.01 I, `\` = LU w/ partial pivoting
 *   step_back                     (src/backward_pass.jl:262-273) unregularised H
 *   backward_pass                 (src/backward_pass.jl:324-357)
 *   forward_pass                  (src/forward_pass.jl:55-93)    α halving, α on δu only
 *   total_cost                    (src/forward_pass.jl:182-196)  sequential sum, ℓ_f on raw x̄_N
 *   fit                           (src/forward_pass.jl:148-179)  prev_cost=Inf, break before update
 * The reference's unbounded line search is capped at max_trials (status 3).
 * Layout: the ABI's (include/ilqr.h) row-major, trajectory-slowest arrays.
 * OpenMP parallelises over independent trajectories only.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define NMAX 32
#define MMAX 16

/* y[r] = M[r][:] x   (M row-major r×c) */
static void matvec(int r, int c, const double* M, const double* x, double* y) {
  for (int i = 0; i < r; ++i) {
    double s = 0.0;
    for (int k = 0; k < c; ++k) s += M[i * c + k] * x[k];
    y[i] = s;
  }
}
/* y = Mᵀ x  (M row-major r×c, y length c) */
static void matTvec(int r, int c, const double* M, const double* x, double* y) {
  for (int j = 0; j < c; ++j) {
    double s = 0.0;
    for (int k = 0; k < r; ++k) s += M[k * c + j] * x[k];
    y[j] = s;
  }
}
/* C = A(r×k) B(k×c) */
static void matmul(int r, int k, int c, const double* A, const double* B, double* C) {
  for (int i = 0; i < r; ++i)
    for (int j = 0; j < c; ++j) {
      double s = 0.0;
      for (int p = 0; p < k; ++p) s += A[i * k + p] * B[p * c + j];
      C[i * c + j] = s;
    }
}
/* C = Aᵀ(A is k×r) B(k×c) */
static void matTmul(int k, int r, int c, const double* A, const double* B, double* C) {
  for (int i = 0; i < r; ++i)
    for (int j = 0; j < c; ++j) {
      double s = 0.0;
      for (int p = 0; p < k; ++p) s += A[p * r + i] * B[p * c + j];
      C[i * c + j] = s;
    }
}

/* Solve M X = Y in place (M m×m, Y m×c), LU with partial pivoting. Returns 0 if singular. */
static int lu_solve(int m, double* M, int c, double* Y) {
  int piv[MMAX];
  for (int k = 0; k < m; ++k) {
    int p = k;
    double best = fabs(M[k * m + k]);
    for (int i = k + 1; i < m; ++i)
      if (fabs(M[i * m + k]) > best) { best = fabs(M[i * m + k]); p = i; }
    piv[k] = p;
    if (best == 0.0) return 0;
    if (p != k) {
      for (int j = 0; j < m; ++j) { double t = M[k * m + j]; M[k * m + j] = M[p * m + j]; M[p * m + j] = t; }
      for (int j = 0; j < c; ++j) { double t = Y[k * c + j]; Y[k * c + j] = Y[p * c + j]; Y[p * c + j] = t; }
    }
    for (int i = k + 1; i < m; ++i) {
      const double f = M[i * m + k] / M[k * m + k];
      M[i * m + k] = f;
      for (int j = k + 1; j < m; ++j) M[i * m + j] -= f * M[k * m + j];
      for (int j = 0; j < c; ++j) Y[i * c + j] -= f * Y[k * c + j];
    }
  }
  for (int i = m - 1; i >= 0; --i)
    for (int j = 0; j < c; ++j) {
      double s = Y[i * c + j];
      for (int p = i + 1; p < m; ++p) s -= M[i * m + p] * Y[p * c + j];
      Y[i * c + j] = s / M[i * m + i];
    }
  (void)piv;
  return 1;
}

typedef struct {
  int n, m, T;
  const double *A, *B, *Q, *R, *Qf; /* this trajectory's instance */
} lq_t;

/* backward_pass (backward_pass.jl:324-357) for one trajectory. Returns 1 if NaN. */
static int backward_one(const lq_t* P, const double* x, const double* u, double mu, int sym,
                        double* d, double* K) {
  const int n = P->n, m = P->m, T = P->T;
  double S[NMAX * NMAX], s[NMAX], Qs[NMAX * NMAX], Rs[MMAX * MMAX];
  double qv[NMAX], r[MMAX], g[MMAX], G[MMAX * NMAX], H[MMAX * MMAX], Hreg[MMAX * MMAX];
  double BtS[MMAX * NMAX], AtS[NMAX * NMAX], t1[NMAX * NMAX], t2[NMAX], du[MMAX], Ki[MMAX * NMAX];
  double HK[MMAX * NMAX], Hdu[MMAX], Snew[NMAX * NMAX], snew[NMAX];
  int nan = 0;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) Qs[i * n + j] = P->Q[i * n + j] + P->Q[j * n + i];
  for (int i = 0; i < m; ++i)
    for (int j = 0; j < m; ++j) Rs[i * m + j] = P->R[i * m + j] + P->R[j * m + i];
  /* final_cost_quadratization (:134-153) */
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) S[i * n + j] = P->Qf[i * n + j] + P->Qf[j * n + i];
  matvec(n, n, S, x + (size_t)T * n, s);
  for (int t = T - 1; t >= 0; --t) { /* :339 */
    const double* xt = x + (size_t)t * n;
    const double* ut = u + (size_t)t * m;
    /* immediate_cost_quadratization (:81-109) */
    matvec(n, n, Qs, xt, qv);
    matvec(m, m, Rs, ut, r);
    /* optimal_controller_param (:177-186) */
    matTvec(n, m, P->B, s, g);                 /* Bᵀ s */
    for (int i = 0; i < m; ++i) g[i] += r[i];  /* g = r + Bᵀ s */
    matTmul(n, m, n, P->B, S, BtS);            /* Bᵀ S */
    matmul(m, n, n, BtS, P->A, G);             /* G = P + (BᵀS)A, P = 0 */
    matmul(m, n, m, BtS, P->B, H);             /* (BᵀS)B */
    for (int i = 0; i < m * m; ++i) H[i] += Rs[i];
    /* feedback_parameters (:207-218) */
    memcpy(Hreg, H, sizeof(double) * m * m);
    for (int i = 0; i < m; ++i) Hreg[i * m + i] += mu;
    for (int i = 0; i < m; ++i) du[i] = -g[i];
    for (int i = 0; i < m * n; ++i) Ki[i] = -G[i];
    {
      double Hc[MMAX * MMAX];
      memcpy(Hc, Hreg, sizeof(Hc[0]) * m * m);
      if (!lu_solve(m, Hc, 1, du)) nan = 1;
      memcpy(Hc, Hreg, sizeof(Hc[0]) * m * m);
      if (!lu_solve(m, Hc, n, Ki)) nan = 1;
    }
    for (int i = 0; i < m; ++i) d[(size_t)t * m + i] = du[i];
    for (int i = 0; i < m * n; ++i) K[(size_t)t * m * n + i] = Ki[i];
    /* step_back (:262-273), unregularised H */
    matvec(m, m, H, du, Hdu);
    matTvec(n, n, P->A, s, snew);               /* Aᵀ s' */
    for (int i = 0; i < n; ++i) snew[i] += qv[i];
    matTvec(m, n, Ki, Hdu, t2);                 /* Kᵀ H δu */
    for (int i = 0; i < n; ++i) snew[i] += t2[i];
    matTvec(m, n, Ki, g, t2);                   /* Kᵀ g */
    for (int i = 0; i < n; ++i) snew[i] += t2[i];
    matTvec(m, n, G, du, t2);                   /* Gᵀ δu */
    for (int i = 0; i < n; ++i) snew[i] += t2[i];
    matTmul(n, n, n, P->A, S, AtS);             /* Aᵀ S' */
    matmul(n, n, n, AtS, P->A, Snew);           /* Aᵀ S' A */
    for (int i = 0; i < n * n; ++i) Snew[i] += Qs[i];
    matmul(m, m, n, H, Ki, HK);
    matTmul(m, n, n, Ki, HK, t1);               /* Kᵀ H K */
    for (int i = 0; i < n * n; ++i) Snew[i] += t1[i];
    matTmul(m, n, n, Ki, G, t1);                /* Kᵀ G */
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) Snew[i * n + j] += t1[i * n + j] + t1[j * n + i]; /* + Gᵀ K */
    if (sym) /* (S+Sᵀ)/2: identity in exact arithmetic, see ilqr_oracle.backward_pass */
      for (int i = 0; i < n; ++i)
        for (int j = 0; j < i; ++j) {
          const double a = 0.5 * (Snew[i * n + j] + Snew[j * n + i]);
          Snew[i * n + j] = a;
          Snew[j * n + i] = a;
        }
    memcpy(S, Snew, sizeof(double) * n * n);
    memcpy(s, snew, sizeof(double) * n);
  }
  for (int i = 0; i < T * m; ++i) nan |= isnan(d[i]);
  for (int i = 0; i < T * m * n; ++i) nan |= isnan(K[i]);
  return nan;
}

static double stage_cost(const lq_t* P, const double* x, const double* u) {
  double t[NMAX];
  double c = 0.0;
  matvec(P->n, P->n, P->Q, x, t);
  for (int i = 0; i < P->n; ++i) c += x[i] * t[i];
  matvec(P->m, P->m, P->R, u, t);
  double cu = 0.0;
  for (int i = 0; i < P->m; ++i) cu += u[i] * t[i];
  return c + cu;
}

static double final_cost(const lq_t* P, const double* x) {
  double t[NMAX];
  double c = 0.0;
  matvec(P->n, P->n, P->Qf, x, t);
  for (int i = 0; i < P->n; ++i) c += x[i] * t[i];
  return c;
}

/* forward_pass (forward_pass.jl:55-93). Returns trials (>0 accepted, <0 exhausted). */
static int forward_one(const lq_t* P, const double* x, const double* u, const double* xtraj,
                       const double* d, const double* K, double prev_cost, double* xb,
                       double* ub, double* cost_out, int max_trials, double alpha0,
                       double shrink) {
  const int n = P->n, m = P->m, T = P->T;
  double alpha = alpha0;
  double dx[NMAX], e[NMAX], Kdx[MMAX], t1[NMAX], t2[NMAX];
  double new_cost = 0.0;
  for (int trial = 1; trial <= max_trials; ++trial) {
    memcpy(xb, x, sizeof(double) * n); /* :65 */
    for (int k = 0; k < T; ++k) {      /* :71 */
      for (int i = 0; i < n; ++i) dx[i] = xb[(size_t)k * n + i] - x[(size_t)k * n + i];
      matvec(m, n, K + (size_t)k * m * n, dx, Kdx);
      for (int i = 0; i < m; ++i)      /* :73 */
        ub[(size_t)k * m + i] = (u[(size_t)k * m + i] + alpha * d[(size_t)k * m + i]) + Kdx[i];
      matvec(n, n, P->A, xb + (size_t)k * n, t1); /* :74 dynamicsf */
      matvec(n, m, P->B, ub + (size_t)k * m, t2);
      for (int i = 0; i < n; ++i) xb[(size_t)(k + 1) * n + i] = t1[i] + t2[i];
    }
    /* total_cost (:185-193) */
    double acc = 0.0;
    for (int k = 0; k < T; ++k) {
      for (int i = 0; i < n; ++i) e[i] = xb[(size_t)k * n + i] - (xtraj ? xtraj[(size_t)k * n + i] : 0.0);
      acc += stage_cost(P, e, ub + (size_t)k * m);
    }
    acc += final_cost(P, xb + (size_t)T * n);
    new_cost = acc;
    *cost_out = new_cost;
    if (prev_cost - new_cost > 0) return trial; /* :77-80 */
    alpha /= 1.0 / shrink;                     /* :82 α /= 2 */
  }
  return -max_trials;
}

static lq_t instance(int b, int n, int m, int T, const double* A, const double* Bm, const double* Q,
                     const double* R, const double* Qf) {
  lq_t P = {n, m, T, A + (size_t)b * n * n, Bm + (size_t)b * n * m, Q + (size_t)b * n * n,
            R + (size_t)b * m * m, Qf + (size_t)b * n * n};
  return P;
}

static void set_threads(int nthreads) {
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#else
  (void)nthreads;
#endif
}

int oracle_max_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}

/* returns the number of trajectories with NaN gains; status may be NULL */
int oracle_lq_backward(int Bn, int T, int n, int m, const double* A, const double* Bm,
                       const double* Q, const double* R, const double* Qf, const double* x,
                       const double* u, double mu, int sym, double* d, double* K, int* status,
                       int nthreads) {
  if (n > NMAX || m > MMAX) return -1;
  set_threads(nthreads);
  int nans = 0;
#pragma omp parallel for schedule(static) reduction(+ : nans)
  for (int b = 0; b < Bn; ++b) {
    const lq_t P = instance(b, n, m, T, A, Bm, Q, R, Qf);
    const int bad = backward_one(&P, x + (size_t)b * (T + 1) * n, u + (size_t)b * T * m, mu, sym,
                                 d + (size_t)b * T * m, K + (size_t)b * T * m * n);
    if (status) status[b] = bad ? 4 : 0;
    nans += bad;
  }
  return nans;
}

int oracle_lq_forward(int Bn, int T, int n, int m, const double* A, const double* Bm,
                      const double* Q, const double* R, const double* Qf, const double* x,
                      const double* u, const double* xtraj, const double* d, const double* K,
                      const double* prev_cost, double* xnew, double* unew, double* cost,
                      int* trials, int max_trials, double alpha0, double shrink, int nthreads) {
  if (n > NMAX || m > MMAX) return -1;
  set_threads(nthreads);
  int fails = 0;
#pragma omp parallel for schedule(static) reduction(+ : fails)
  for (int b = 0; b < Bn; ++b) {
    const lq_t P = instance(b, n, m, T, A, Bm, Q, R, Qf);
    const int tr = forward_one(&P, x + (size_t)b * (T + 1) * n, u + (size_t)b * T * m,
                               xtraj ? xtraj + (size_t)b * (T + 1) * n : NULL,
                               d + (size_t)b * T * m, K + (size_t)b * T * m * n, prev_cost[b],
                               xnew + (size_t)b * (T + 1) * n, unew + (size_t)b * T * m, &cost[b],
                               max_trials, alpha0, shrink);
    if (trials) trials[b] = tr;
    fails += tr < 0;
  }
  return fails;
}

/* fit (forward_pass.jl:148-179). status: 1 converged, 2 max_iter, 3 LS exhausted, 4 NaN. */
int oracle_lq_fit(int Bn, int T, int n, int m, const double* A, const double* Bm, const double* Q,
                  const double* R, const double* Qf, const double* x_init, const double* u_init,
                  const double* xtraj, int max_iter, double tol, double mu, int sym, int max_trials,
                  double* x_out, double* u_out, double* cost, int* iters, int* status,
                  int nthreads) {
  if (n > NMAX || m > MMAX) return -1;
  set_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 4)
  for (int b = 0; b < Bn; ++b) {
    const lq_t P = instance(b, n, m, T, A, Bm, Q, R, Qf);
    const size_t xs = (size_t)(T + 1) * n, us = (size_t)T * m;
    double* buf = (double*)malloc(sizeof(double) * (2 * xs + 2 * us + us + us * n));
    double *xi = buf, *ui = xi + xs, *xn = ui + us, *un = xn + xs, *d = un + us, *K = d + us;
    memcpy(xi, x_init + b * xs, sizeof(double) * xs);
    memcpy(ui, u_init + b * us, sizeof(double) * us);
    double prev_cost = INFINITY; /* :159 */
    int st = 2, it;
    for (it = 1; it <= max_iter; ++it) { /* :161 */
      if (backward_one(&P, xi, ui, mu, sym, d, K)) { st = 4; break; }
      double nc;
      const int tr = forward_one(&P, xi, ui, xtraj ? xtraj + b * xs : NULL, d, K, prev_cost, xn,
                                 un, &nc, max_trials, 1.0, 0.5);
      if (tr < 0) { st = (nc != nc) ? 4 : 3; break; }
      prev_cost = nc; /* :168 */
      double du2 = 0.0;
      for (size_t i = 0; i < us; ++i) du2 += (un[i] - ui[i]) * (un[i] - ui[i]);
      if (du2 <= tol) { st = 1; break; } /* :171 — break before the update */
      memcpy(xi, xn, sizeof(double) * xs); /* :174-175 */
      memcpy(ui, un, sizeof(double) * us);
    }
    memcpy(x_out + b * xs, xi, sizeof(double) * xs);
    memcpy(u_out + b * us, ui, sizeof(double) * us);
    cost[b] = prev_cost;
    if (iters) iters[b] = it > max_iter ? max_iter : it;
    if (status) status[b] = st;
    free(buf);
  }
  return 0;
}
