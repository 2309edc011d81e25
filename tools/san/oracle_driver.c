/* Host sanitizer driver for the C restatement (oracle/ilqr_ref.c): built with
 * -fsanitize=address,undefined by `make -C oracle SAN=1` and run by tools/san/run_cpu.sh
 * (ASan/UBSan builds of the C++ oracle and runtime). Exercises every entry
 * point on small seeded problems — LQ (12, 4) and a padded-like (5, 2) shape, NaN
 * inputs, unreachable prev_cost (exhausted searches), the 2-link arm (nu 1, 2), tiles,
 * and a 2-joint chain — with OpenMP on, and checks the outputs for consistency (finite
 * where they must be, trial counts in range). Exit 0 on success; a sanitizer finding
 * aborts with its report. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int oracle_max_threads(void);
int oracle_lq_backward(int Bn, int T, int n, int m, const double* A, const double* Bm, const double* Q,
                       const double* R, const double* Qf, const double* x, const double* u, double mu, int sym,
                       double* d, double* K, int* status, int nthreads);
int oracle_lq_forward(int Bn, int T, int n, int m, const double* A, const double* Bm, const double* Q,
                      const double* R, const double* Qf, const double* x, const double* u, const double* xtraj,
                      const double* d, const double* K, const double* prev_cost, double* xnew, double* unew,
                      double* cost, int* trials, int max_trials, double alpha0, double shrink, int nthreads);
int oracle_lq_fit(int Bn, int T, int n, int m, const double* A, const double* Bm, const double* Q, const double* R,
                  const double* Qf, const double* x_init, const double* u_init, const double* xtraj, int max_iter,
                  double tol, double mu, int sym, int max_trials, double* x_out, double* u_out, double* cost,
                  int* iters, int* status, int nthreads);
int oracle_tl_fit(int Bn, int T, int nu, const double* x_init, const double* u_init, const double* xtraj,
                  int max_iter, double tol, double mu, int sym, int max_trials, double* x_out, double* u_out,
                  double* cost, int* iters, int* status, int nthreads, double* hcost, int* htrials,
                  double* hdu2);
int oracle_tiles_backward(int Bn, int T, int n, int m, const double* A, const double* Bm, const double* lx,
                          const double* lu, const double* lxx, const double* lux, const double* luu,
                          const double* lfx, const double* lfxx, double mu, int sym, double* d, double* K,
                          int* status, int nthreads);
int oracle_chain_iterate(int Bn, int T, int nj, int nu, const double* R0, const double* p, const double* ax,
                         const double* mass, const double* com, const double* Ic, const double* grav, double dt,
                         const double* tgt, const double* qw, const double* rw, const double* qfw, const double* x,
                         const double* u, double mu, int sym, int max_trials, double* d, double* K, double* xn,
                         double* un, double* cost, int* trials, int nthreads);

static uint64_t rng = 0x9E3779B97F4A7C15ull;
static double unif(void) { /* xorshift64*, [0, 1) */
  rng ^= rng >> 12; rng ^= rng << 25; rng ^= rng >> 27;
  return (double)((rng * 2685821657736338717ull) >> 11) * (1.0 / 9007199254740992.0);
}
static double* vec(size_t n, double lo, double hi) {
  double* v = (double*)malloc(sizeof(double) * (n ? n : 1));
  for (size_t i = 0; i < n; ++i) v[i] = lo + (hi - lo) * unif();
  return v;
}
static int fails = 0;
#define CHECK(c, ...) do { if (!(c)) { fprintf(stderr, "FAIL: " __VA_ARGS__); fputc('\n', stderr); ++fails; } } while (0)

static void lq_case(int Bn, int T, int n, int m, int nthreads) {
  double *A = vec((size_t)Bn * n * n, -0.05, 0.05), *Bm = vec((size_t)Bn * n * m, -0.1, 0.1);
  double *Q = vec((size_t)Bn * n * n, 0, 0), *R = vec((size_t)Bn * m * m, 0, 0), *Qf = vec((size_t)Bn * n * n, 0, 0);
  for (int b = 0; b < Bn; ++b) {
    for (int i = 0; i < n; ++i) {
      A[(size_t)b * n * n + i * n + i] += 1.0;
      Q[(size_t)b * n * n + i * n + i] = 0.5 + unif();
      Qf[(size_t)b * n * n + i * n + i] = 5.0 + unif();
    }
    for (int i = 0; i < m; ++i) R[(size_t)b * m * m + i * m + i] = 0.05 + 0.1 * unif();
  }
  const size_t xs = (size_t)(T + 1) * n, us = (size_t)T * m;
  double *x = vec(Bn * xs, -1, 1), *u = vec(Bn * us, 0, 0);
  double *d = vec(Bn * us, 0, 0), *K = vec(Bn * us * n, 0, 0), *xt = vec(Bn * xs, -0.1, 0.1);
  double *xn = vec(Bn * xs, 0, 0), *un = vec(Bn * us, 0, 0), *cost = vec(Bn, 0, 0), *pc = vec(Bn, 0, 0);
  int *st = (int*)calloc(Bn, sizeof(int)), *tr = (int*)calloc(Bn, sizeof(int)), *it = (int*)calloc(Bn, sizeof(int));
  x[(size_t)T * n + 3] = NAN; /* trajectory 0 carries a NaN in x_N: status 4 (gains), never a finding */
  int r = oracle_lq_backward(Bn, T, n, m, A, Bm, Q, R, Qf, x, u, 0.01, 1, d, K, st, nthreads);
  CHECK(r >= 1 && st[0] == 4, "lq_backward NaN status (r=%d st0=%d)", r, st[0]);
  for (int b = 0; b < Bn; ++b) pc[b] = (b % 3 == 0) ? -1.0 : INFINITY; /* -1: unreachable */
  oracle_lq_forward(Bn, T, n, m, A, Bm, Q, R, Qf, x, u, xt, d, K, pc, xn, un, cost, tr, 7, 1.0, 0.5, nthreads);
  for (int b = 1; b < Bn; ++b) CHECK(b % 3 == 0 ? tr[b] == -7 : tr[b] == 1, "lq_forward trials b=%d tr=%d", b, tr[b]);
  x[(size_t)T * n + 3] = 0.25;
  oracle_lq_fit(Bn, T, n, m, A, Bm, Q, R, Qf, x, u, NULL, 6, 1e-9, 0.01, 1, 64, xn, un, cost, it, st, nthreads);
  for (int b = 0; b < Bn; ++b) CHECK(isfinite(cost[b]) && it[b] >= 1 && it[b] <= 6, "lq_fit b=%d", b);
  /* tiles backward on the LQ problem's own derivatives */
  double *lx = vec((size_t)Bn * T * n, -1, 1), *lu = vec((size_t)Bn * T * m, -1, 1);
  double *lxx = vec((size_t)Bn * T * n * n, 0, 0), *luu = vec((size_t)Bn * T * m * m, 0, 0);
  double *lfx = vec((size_t)Bn * n, -1, 1), *lfxx = vec((size_t)Bn * n * n, 0, 0);
  double *At = vec((size_t)Bn * T * n * n, 0, 0), *Bt = vec((size_t)Bn * T * n * m, 0, 0);
  for (int b = 0; b < Bn; ++b)
    for (int t = 0; t < T; ++t) {
      memcpy(At + ((size_t)b * T + t) * n * n, A + (size_t)b * n * n, sizeof(double) * n * n);
      memcpy(Bt + ((size_t)b * T + t) * n * m, Bm + (size_t)b * n * m, sizeof(double) * n * m);
      for (int i = 0; i < n; ++i) lxx[((size_t)b * T + t) * n * n + i * n + i] = 2.0;
      for (int i = 0; i < m; ++i) luu[((size_t)b * T + t) * m * m + i * m + i] = 0.2;
    }
  for (int b = 0; b < Bn; ++b)
    for (int i = 0; i < n; ++i) lfxx[(size_t)b * n * n + i * n + i] = 10.0;
  r = oracle_tiles_backward(Bn, T, n, m, At, Bt, lx, lu, lxx, NULL, luu, lfx, lfxx, 0.01, 1, d, K, st, nthreads);
  CHECK(r == 0, "tiles_backward NaNs %d", r);
  void* bufs[] = {A, Bm, Q, R, Qf, x, u, d, K, xt, xn, un, cost, pc, st, tr, it, lx, lu, lxx, luu, lfx, lfxx, At, Bt};
  for (size_t i = 0; i < sizeof(bufs) / sizeof(*bufs); ++i) free(bufs[i]);
}

static void two_link_case(int Bn, int T, int nu, int nthreads) {
  const size_t xs = (size_t)(T + 1) * 4, us = (size_t)T * nu;
  double *x = vec(Bn * xs, 0, 0), *u = vec(Bn * us, 0, 0), *xo = vec(Bn * xs, 0, 0), *uo = vec(Bn * us, 0, 0);
  double* cost = vec(Bn, 0, 0);
  int *it = (int*)calloc(Bn, sizeof(int)), *st = (int*)calloc(Bn, sizeof(int));
  for (int b = 0; b < Bn; ++b)
    for (int t = 0; t <= T; ++t) { x[b * xs + t * 4] = 0.1 * unif(); x[b * xs + t * 4 + 1] = -0.1; }
  oracle_tl_fit(Bn, T, nu, x, u, NULL, 30, 1e-6, 0.01, 1, 64, xo, uo, cost, it, st, nthreads, NULL, NULL, NULL);
  for (int b = 0; b < Bn; ++b) CHECK(st[b] >= 1 && st[b] <= 3, "tl_fit nu=%d b=%d st=%d", nu, b, st[b]);
  free(x); free(u); free(xo); free(uo); free(cost); free(it); free(st);
}

static void chain_case(int Bn, int T, int nthreads) {
  const int nj = 2, nu = 1;
  double R0[18] = {1, 0, 0, 0, 1, 0, 0, 0, 1, 1, 0, 0, 0, 1, 0, 0, 0, 1}, p[6] = {0, 0, 0.1, 0, 0, 0.5};
  double ax[6] = {0, 0, 1, 0, 1, 0}, mass[2] = {3, 3}, com[6] = {0, 0, 0.25, 0, 0, 0.25};
  double Ic[18] = {0}, grav[3] = {0, 0, -9.81}, tgt[2] = {0.5, -0.3}, qw[2] = {1, 1}, rw[1] = {0.01}, qfw[2] = {10, 10};
  for (int j = 0; j < 2; ++j) { Ic[j * 9] = 0.05; Ic[j * 9 + 4] = 0.05; Ic[j * 9 + 8] = 0.01; }
  const size_t xs = (size_t)(T + 1) * 4, us = (size_t)T * nu;
  double *x = vec(Bn * xs, -0.5, 0.5), *u = vec(Bn * us, -0.1, 0.1), *d = vec(Bn * us, 0, 0);
  double *K = vec(Bn * us * 4, 0, 0), *xn = vec(Bn * xs, 0, 0), *un = vec(Bn * us, 0, 0), *cost = vec(Bn, 0, 0);
  int* tr = (int*)calloc(Bn, sizeof(int));
  oracle_chain_iterate(Bn, T, nj, nu, R0, p, ax, mass, com, Ic, grav, 0.01, tgt, qw, rw, qfw, x, u, 0.01, 1, 64, d, K,
                       xn, un, cost, tr, nthreads);
  for (int b = 0; b < Bn; ++b) CHECK(tr[b] != 0, "chain_iterate b=%d", b);
  free(x); free(u); free(d); free(K); free(xn); free(un); free(cost); free(tr);
}

int main(void) {
  const int threads = oracle_max_threads() < 4 ? oracle_max_threads() : 4;
  lq_case(9, 16, 12, 4, threads);
  lq_case(5, 7, 5, 2, 1);
  two_link_case(6, 30, 2, threads);
  two_link_case(3, 20, 1, 1);
  chain_case(4, 20, threads);
  printf("oracle sanitizer driver: %s (%d failed checks)\n", fails ? "FAILED" : "ok", fails);
  return fails ? 1 : 0;
}
