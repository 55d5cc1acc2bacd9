/*
 * nx_cpu.c -- CPU PORT, test infrastructure only (bench.py's all-cores cpu_baseline leg and
 * tests/test_cpu_port.py). Never linked or loaded by the product path.
 *
 * An OpenMP restatement of one full step of the hot path on the host cores, in the device
 * layout (include/nxhip.h): assembly of the symmetric saddle-point system (the reference's
 * forms, /root/reference/src/networks_fenicsx/assembly.py:243-277, pressure rows negated)
 * and a preconditioned MINRES (Paige-Saunders in the form of scipy.sparse.linalg.minres)
 * with the same exact tree Schur-complement preconditioner as the GPU
 * (networks_fenicsx_amd/precond.py derives it; pc_up_model / pc_finish_model are the numpy
 * models this follows). It stands in for the reference's DOLFINx assembly + MUMPS LU
 * (solver.py:58-65, 127), which cannot run in this image: a baseline, not a target.
 *
 * Parallel structure: edges / rows / chains are split over the threads; the junction
 * forest's lower subtrees ("jobs") run one per thread task, the small top part serially.
 * Geometry and element tensors follow the reference mesh generator (mesh.py:269-322) with
 * FMA contraction off (build flag), so the assembled CSR equals the oracle's bit for bit.
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define API __attribute__((visibility("default")))

API int nxc_threads(void) { return omp_get_max_threads(); }
API void nxc_set_threads(int n) { omp_set_num_threads(n > 0 ? n : 1); }

/* ---- pattern: one edge's rows are one contiguous CSR segment (device layout) ---- */
API int64_t nxc_nnz(int N, int64_t E, const int* edge_lm, int64_t B, const int* lm_rowptr) {
  int64_t acc = 0;
  for (int64_t e = 0; e < E; ++e)
    acc += 7 * (int64_t)N + 1 + (edge_lm[2 * e] >= 0) + (edge_lm[2 * e + 1] >= 0);
  return acc + (B > 0 ? lm_rowptr[B] : 0);
}

static void vertex(const double* x0, const double* x1, int k, int N, double invN, double* p) {
  if (k == 0) {
    p[0] = x0[0]; p[1] = x0[1]; p[2] = x0[2];
  } else if (k == N) {
    p[0] = x1[0]; p[1] = x1[1]; p[2] = x1[2];
  } else {  /* numpy: w = k * (1/N); start * (1 - w) + end * w   (mesh.py:275, 290) */
    const double w = (double)k * invN, om = 1.0 - w;
    p[0] = x0[0] * om + x1[0] * w;
    p[1] = x0[1] * om + x1[1] * w;
    p[2] = x0[2] * om + x1[2] * w;
  }
}

static double cell_h(const double* ex, int k, int N, double invN) {
  double a[3], b[3];
  vertex(ex, ex + 3, k, N, invN, a);
  vertex(ex, ex + 3, k + 1, N, invN, b);
  const double d0 = b[0] - a[0], d1 = b[1] - a[1], d2 = b[2] - a[2];
  return sqrt(d0 * d0 + d1 * d1 + d2 * d2);
}

/*
 * Pattern + values + rhs + lumped flux mass in one pass (the pattern is static, but writing
 * it costs the same sweep; the timed baseline passes pattern = 0 and writes values only).
 *   rowptr (n+1), col, val (nnz), rhs (n), dq (E*(N+1))
 */
API void nxc_assemble(int N, int64_t E, const double* edge_x, const int* edge_lm,
                      const double* edge_R, double R_const, const double* edge_bc, double f,
                      int64_t B, const int* lm_rowptr, const int* lm_col, const double* lm_val,
                      int pattern, int* rowptr, int* col, double* val, double* rhs, double* dq) {
  const int64_t per = 2 * (int64_t)N + 1, ned = E * per;
  int64_t* seg = (int64_t*)malloc(sizeof(int64_t) * (size_t)(E + 1));
  seg[0] = 0;
  for (int64_t e = 0; e < E; ++e)
    seg[e + 1] = seg[e] + 7 * (int64_t)N + 1 + (edge_lm[2 * e] >= 0) + (edge_lm[2 * e + 1] >= 0);
  const double invN = 1.0 / (double)N;
#pragma omp parallel
  {
    double* md = (double*)malloc(sizeof(double) * (size_t)N);
    double* mo = (double*)malloc(sizeof(double) * (size_t)N);
    double* hc = (double*)malloc(sizeof(double) * (size_t)N);
#pragma omp for schedule(static)
    for (int64_t e = 0; e < E; ++e) {
      const double* ex = edge_x + 6 * e;
      const double R = edge_R ? edge_R[e] : R_const;
      for (int k = 0; k < N; ++k) {
        const double h = cell_h(ex, k, N, invN);
        hc[k] = h;
        md[k] = R * h / 3.0;
        mo[k] = R * h / 6.0;
      }
      const int ls = edge_lm[2 * e], ld = edge_lm[2 * e + 1];
      const int64_t base = e * per;
      int64_t i = seg[e];
      for (int r = 0; r < (int)per; ++r) {
        const int64_t row = base + r;
        if (pattern) rowptr[row] = (int)i;
#define PUT(c, v)                         \
  do {                                    \
    if (pattern) col[i] = (int)(c);       \
    val[i] = (v);                         \
    ++i;                                  \
  } while (0)
        if (r & 1) {  /* pressure row p_g (negated divergence): +1 at q_g, -1 at q_{g+1} */
          PUT(row - 1, 1.0);
          PUT(row + 1, -1.0);
          rhs[row] = -(f * hc[r / 2]);
        } else {
          const int k = r / 2;
          if (k == 0) {  /* q_0: [q_0, p_0, q_1, (lambda_src)] */
            PUT(row, md[0]);
            PUT(row + 1, 1.0);
            PUT(row + 2, mo[0]);
            if (ls >= 0) PUT(ls, -1.0);
            rhs[row] = edge_bc[2 * e];
          } else if (k == N) {  /* q_N: [q_{N-1}, p_{N-1}, q_N, (lambda_dst)] */
            PUT(row - 2, mo[N - 1]);
            PUT(row - 1, -1.0);
            PUT(row, md[N - 1]);
            if (ld >= 0) PUT(ld, 1.0);
            rhs[row] = edge_bc[2 * e + 1];
          } else {  /* interior q_k: [q_{k-1}, p_{k-1}, q_k, p_k, q_{k+1}] */
            PUT(row - 2, mo[k - 1]);
            PUT(row - 1, -1.0);
            PUT(row, md[k - 1] + md[k]);
            PUT(row + 1, 1.0);
            PUT(row + 2, mo[k]);
            rhs[row] = 0.0;
          }
        }
#undef PUT
      }
      double* d = dq + e * (int64_t)(N + 1);  /* lumped (row-sum) flux mass */
      for (int k = 0; k <= N; ++k) {
        double v;
        if (k < N) {
          v = md[k] + mo[k];
          if (k > 0) v = (mo[k - 1] + md[k - 1]) + v;
        } else {
          v = mo[N - 1] + md[N - 1];
        }
        d[k] = v;
      }
    }
    free(md);
    free(mo);
    free(hc);
  }
  const int64_t nnz_e = seg[E];
#pragma omp parallel for schedule(static)
  for (int64_t b = 0; b < B; ++b) {
    if (pattern) rowptr[ned + b] = (int)(nnz_e + lm_rowptr[b]);
    for (int i = lm_rowptr[b]; i < lm_rowptr[b + 1]; ++i) {
      if (pattern) col[nnz_e + i] = lm_col[i];
      val[nnz_e + i] = lm_val[i];
    }
    rhs[ned + b] = 0.0;
  }
  if (pattern) rowptr[ned + B] = (int)(nnz_e + (B > 0 ? lm_rowptr[B] : 0));
  free(seg);
}

/* ---- the tree preconditioner (single rank; precond.py TreePreconditioner arrays) ---- */
typedef struct {
  int N, exact;
  int64_t n_chains, n_slots;
  int n_jobs, n_top_lvl;
  const int *chain_edge, *chain_flip, *chain_up, *chain_lo;
  const int *slot_lam, *slot_pchain, *slot_parent, *slot_dc_off, *slot_dc;
  const int *job_chain_off, *job_lvl_off, *lvl_slot_off, *top_lvl_off;
  const double* dq;
  double *T, *It, *Ib, *D, *J, *z_slot;
  double *lu;  /* [l_0..l_N | 1/u_0..1/u_N] of T = tridiag(1,4,1), 2 at both ends */
} Pc;

static void chain_rho(const Pc* p, int64_t c, double* rho) {
  const int N = p->N;
  const double* d = p->dq + (int64_t)p->chain_edge[c] * (N + 1);
  if (p->chain_flip[c])
    for (int k = 0; k <= N; ++k) rho[k] = d[N - k];
  else
    memcpy(rho, d, sizeof(double) * (size_t)(N + 1));
}

static inline int64_t cell_dof(const Pc* p, int64_t c, int k) {
  const int N = p->N;
  const int64_t base = (int64_t)p->chain_edge[c] * (2 * N + 1);
  return base + 2 * (p->chain_flip[c] ? N - 1 - k : k) + 1;
}
static inline int64_t q_dof(const Pc* p, int64_t c, int k) {
  const int N = p->N;
  const int64_t base = (int64_t)p->chain_edge[c] * (2 * N + 1);
  return base + 2 * (p->chain_flip[c] ? N - k : k);
}

static void eliminate(const Pc* p, const double* r, int j) {
  const int pcn = p->slot_pchain[j];
  double D = pcn >= 0 ? 1.0 / p->T[pcn] : 0.0;
  double J = r[p->slot_lam[j]] + (pcn >= 0 ? p->Ib[pcn] : 0.0);
  for (int i = p->slot_dc_off[j]; i < p->slot_dc_off[j + 1]; ++i) {
    const int c = p->slot_dc[i];
    const double g = 1.0 / p->T[c];
    J += p->It[c];
    const int lo = p->chain_lo[c];
    if (lo >= 0) {
      D += g * (1.0 - g / p->D[lo]);
      J += g * p->J[lo] / p->D[lo];
    } else {
      D += g;
    }
  }
  p->D[j] = D;
  p->J[j] = J;
}

static void backsub(const Pc* p, double* z, int j) {
  const int par = p->slot_parent[j];
  double num = p->J[j];
  if (par >= 0) num += p->z_slot[par] / p->T[p->slot_pchain[j]];
  const double zj = num / p->D[j];
  p->z_slot[j] = zj;
  z[p->slot_lam[j]] = zj;
}

/* z = P^{-1} r; returns r . z */
static double pc_apply(const Pc* p, const double* r, double* z) {
  const int N = p->N;
#pragma omp parallel
  {
    double* rho = (double*)malloc(sizeof(double) * (size_t)(N + 1));
#pragma omp for schedule(static)
    for (int64_t c = 0; c < p->n_chains; ++c) {  /* chain condensation */
      chain_rho(p, c, rho);
      double T = 0.0, acc = 0.0, sr = 0.0, srd = 0.0;
      for (int k = 0; k <= N; ++k) T += rho[k];
      for (int k = 0; k < N; ++k) {
        acc += rho[k];
        const double rc = r[cell_dof(p, c, k)];
        sr += rc;
        srd += rc * acc;
      }
      const double ib = srd / T;
      p->T[c] = T;
      p->Ib[c] = ib;
      p->It[c] = sr - ib;
    }
    free(rho);
  }
#pragma omp parallel for schedule(dynamic, 1)
  for (int jb = 0; jb < p->n_jobs; ++jb)  /* lower subtrees, deepest level first */
    for (int lv = p->job_lvl_off[jb + 1] - 1; lv >= p->job_lvl_off[jb]; --lv)
      for (int j = p->lvl_slot_off[lv]; j < p->lvl_slot_off[lv + 1]; ++j) eliminate(p, r, j);
  for (int lv = p->n_top_lvl - 1; lv >= 0; --lv)  /* top part */
    for (int j = p->top_lvl_off[lv]; j < p->top_lvl_off[lv + 1]; ++j) eliminate(p, r, j);
  for (int lv = 0; lv < p->n_top_lvl; ++lv)
    for (int j = p->top_lvl_off[lv]; j < p->top_lvl_off[lv + 1]; ++j) backsub(p, z, j);
#pragma omp parallel for schedule(dynamic, 1)
  for (int jb = 0; jb < p->n_jobs; ++jb)
    for (int lv = p->job_lvl_off[jb]; lv < p->job_lvl_off[jb + 1]; ++lv)
      for (int j = p->lvl_slot_off[lv]; j < p->lvl_slot_off[lv + 1]; ++j) backsub(p, z, j);
  double part = 0.0;
#pragma omp parallel reduction(+ : part)
  {
    double* rho = (double*)malloc(sizeof(double) * (size_t)(N + 1));
    double* Dk = (double*)malloc(sizeof(double) * (size_t)N);
    double* suf = (double*)malloc(sizeof(double) * (size_t)(N + 1));
    double* y = (double*)malloc(sizeof(double) * (size_t)(N + 1));
#pragma omp for schedule(static)
    for (int64_t c = 0; c < p->n_chains; ++c) {  /* chain cells and flux block */
      chain_rho(p, c, rho);
      const double T = p->T[c], iT = 1.0 / T;
      const double zt = p->chain_up[c] >= 0 ? p->z_slot[p->chain_up[c]] : 0.0;
      const double zb = p->chain_lo[c] >= 0 ? p->z_slot[p->chain_lo[c]] : 0.0;
      double acc = 0.0;
      for (int k = 0; k < N; ++k) {
        acc += rho[k];
        Dk[k] = acc;
      }
      suf[N] = 0.0;
      for (int k = N - 1; k >= 0; --k) suf[k] = suf[k + 1] + (T - Dk[k]) * r[cell_dof(p, c, k)];
      double pre = 0.0;
      const double mo = rho[0] / 3.0;  /* R h / 6 of the edge */
      for (int k = 0; k < N; ++k) {
        const int64_t dc = cell_dof(p, c, k);
        const double rc = r[dc];
        double zk = zt * (T - Dk[k]) * iT + zb * Dk[k] * iT + Dk[k] * iT * suf[k] +
                    (T - Dk[k]) * iT * pre;
        if (p->exact) zk -= mo * rc;
        pre += Dk[k] * rc;
        z[dc] = zk;
        part += rc * zk;
      }
      if (p->exact) {  /* M_e^{-1} r_q = T^{-1} r_q / mo: Thomas with the fixed pivots */
        const double* l = p->lu;
        const double* iu = p->lu + N + 1;
        for (int k = 0; k <= N; ++k) y[k] = r[q_dof(p, c, k)] - (k ? l[k] * y[k - 1] : 0.0);
        double xk = 0.0;
        for (int k = N; k >= 0; --k) {
          xk = iu[k] * (y[k] - (k < N ? xk : 0.0));
          const int64_t dq_ = q_dof(p, c, k);
          const double zq = xk / mo;
          z[dq_] = zq;
          part += r[dq_] * zq;
        }
      } else {
        for (int k = 0; k <= N; ++k) {
          const int64_t dq_ = q_dof(p, c, k);
          const double zq = r[dq_] / rho[k];
          z[dq_] = zq;
          part += r[dq_] * zq;
        }
      }
    }
    free(rho);
    free(Dk);
    free(suf);
    free(y);
  }
  /* multipliers' share of r . z (owned rows past the edge DoFs) */
  for (int64_t j = 0; j < p->n_slots; ++j) part += r[p->slot_lam[j]] * p->z_slot[j];
  return part;
}

/* ---- direct tree solve (the GPU's kModeDirect sweeps, csrc/nxhip.hip): block LU of
 * [[M, K], [K^T, 0]] -- y = M^{-1} b_q, x_s = S^{-1}(K^T y - b_s), x_q = M^{-1}(b_q - K x_s),
 * the last one recovered conservatively (divergence rows exact) ---- */
static void chain_thomas(const Pc* p, const double* rhs, double* out) {  /* T^{-1} rhs */
  const int N = p->N;
  const double* l = p->lu;
  const double* iu = p->lu + N + 1;
  double yk = 0.0;
  for (int k = 0; k <= N; ++k) {
    yk = rhs[k] - (k ? l[k] * yk : 0.0);
    out[k] = yk;
  }
  double xk = 0.0;
  for (int k = N; k >= 0; --k) {
    xk = iu[k] * (out[k] - (k < N ? xk : 0.0));
    out[k] = xk;
  }
}

/* x = A^{-1} b (owned rows; x also receives the multipliers). mb: scratch of n doubles. */
static void pc_direct(const Pc* p, const double* b, double* x, double* mb, int64_t n) {
  const int N = p->N;
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) mb[i] = -b[i];  /* multiplier rows: -b_lambda */
#pragma omp parallel
  {
    double* rho = (double*)malloc(sizeof(double) * (size_t)(N + 1));
    double* t = (double*)malloc(sizeof(double) * (size_t)(N + 1));
    double* y = (double*)malloc(sizeof(double) * (size_t)(N + 1));
#pragma omp for schedule(static)
    for (int64_t c = 0; c < p->n_chains; ++c) {  /* y, cell inputs w, condensation */
      chain_rho(p, c, rho);
      const double mo = rho[0] / 3.0;
      const int flip = p->chain_flip[c];
      for (int k = 0; k <= N; ++k) t[k] = b[q_dof(p, c, k)];
      chain_thomas(p, t, y);
      for (int k = 0; k <= N; ++k) y[k] /= mo;
      double T = 0.0, acc = 0.0, sr = 0.0, srd = 0.0;
      for (int k = 0; k <= N; ++k) T += rho[k];
      for (int k = 0; k < N; ++k) {
        acc += rho[k];
        const double d = y[k] - y[k + 1];
        const double w = (flip ? -d : d) - b[cell_dof(p, c, k)];
        sr += w;
        srd += w * acc;
      }
      const double ib = srd / T;
      p->T[c] = T;
      p->Ib[c] = ib + (flip ? -y[N] : y[N]);
      p->It[c] = (sr - ib) + (flip ? y[0] : -y[0]);
    }
    free(rho);
    free(t);
    free(y);
  }
#pragma omp parallel for schedule(dynamic, 1)
  for (int jb = 0; jb < p->n_jobs; ++jb)
    for (int lv = p->job_lvl_off[jb + 1] - 1; lv >= p->job_lvl_off[jb]; --lv)
      for (int j = p->lvl_slot_off[lv]; j < p->lvl_slot_off[lv + 1]; ++j) eliminate(p, mb, j);
  for (int lv = p->n_top_lvl - 1; lv >= 0; --lv)
    for (int j = p->top_lvl_off[lv]; j < p->top_lvl_off[lv + 1]; ++j) eliminate(p, mb, j);
  for (int lv = 0; lv < p->n_top_lvl; ++lv)
    for (int j = p->top_lvl_off[lv]; j < p->top_lvl_off[lv + 1]; ++j) backsub(p, x, j);
#pragma omp parallel for schedule(dynamic, 1)
  for (int jb = 0; jb < p->n_jobs; ++jb)
    for (int lv = p->job_lvl_off[jb]; lv < p->job_lvl_off[jb + 1]; ++lv)
      for (int j = p->lvl_slot_off[lv]; j < p->lvl_slot_off[lv + 1]; ++j) backsub(p, x, j);
#pragma omp parallel
  {
    double* rho = (double*)malloc(sizeof(double) * (size_t)(N + 1));
    double* Dk = (double*)malloc(sizeof(double) * (size_t)N);
    double* w = (double*)malloc(sizeof(double) * (size_t)N);
    double* zc = (double*)malloc(sizeof(double) * (size_t)N);
    double* suf = (double*)malloc(sizeof(double) * (size_t)(N + 1));
    double* t = (double*)malloc(sizeof(double) * (size_t)(N + 1));
    double* y = (double*)malloc(sizeof(double) * (size_t)(N + 1));
#pragma omp for schedule(static)
    for (int64_t c = 0; c < p->n_chains; ++c) {  /* cells, then x_q = M^{-1}(b_q - K x_s) */
      chain_rho(p, c, rho);
      const double mo = rho[0] / 3.0;
      const int flip = p->chain_flip[c];
      for (int k = 0; k <= N; ++k) t[k] = b[q_dof(p, c, k)];
      chain_thomas(p, t, y);
      for (int k = 0; k <= N; ++k) y[k] /= mo;
      const double T = p->T[c], iT = 1.0 / T;
      const double zt = p->chain_up[c] >= 0 ? p->z_slot[p->chain_up[c]] : 0.0;
      const double zb = p->chain_lo[c] >= 0 ? p->z_slot[p->chain_lo[c]] : 0.0;
      double acc = 0.0;
      for (int k = 0; k < N; ++k) {
        acc += rho[k];
        Dk[k] = acc;
        const double d = y[k] - y[k + 1];
        w[k] = (flip ? -d : d) - b[cell_dof(p, c, k)];
      }
      suf[N] = 0.0;
      for (int k = N - 1; k >= 0; --k) suf[k] = suf[k + 1] + (T - Dk[k]) * w[k];
      double pre = 0.0;
      for (int k = 0; k < N; ++k) {
        double zk = zt * (T - Dk[k]) * iT + zb * Dk[k] * iT + Dk[k] * iT * suf[k] +
                    (T - Dk[k]) * iT * pre - mo * w[k];
        pre += Dk[k] * w[k];
        zc[k] = zk;
        x[cell_dof(p, c, k)] = zk;
      }
      /* fluxes, conservatively (csrc/nxhip.hip direct_flux_cons): the divergence rows give
       * x_q[k] = q0 - s P_k, P_k = sum_{j<k} b_c[j]; the d-weighted sum of the flux rows
       * gives T q0 = sum_k b_q[k] - s (zb - zt) + s sum_k d_k P_k */
      const double sg = flip ? -1.0 : 1.0;
      double s1 = 0.0, s2 = 0.0, P = 0.0;
      for (int k = 0; k <= N; ++k) {
        s1 += b[q_dof(p, c, k)];
        s2 += rho[k] * P;
        t[k] = P;
        if (k < N) P += b[cell_dof(p, c, k)];
      }
      const double q0 = (s1 - sg * (zb - zt) + sg * s2) / T;
      for (int k = 0; k <= N; ++k) x[q_dof(p, c, k)] = q0 - sg * t[k];
    }
    free(rho); free(Dk); free(w); free(zc); free(suf); free(t); free(y);
  }
}

/* ---- CSR SpMV and vector kernels ---- */
static void spmv(int64_t n, const int* rp, const int* col, const double* val, const double* x,
                 double* y) {
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) {
    double s = 0.0;
    for (int k = rp[i]; k < rp[i + 1]; ++k) s += val[k] * x[col[k]];
    y[i] = s;
  }
}

/*
 * Preconditioned MINRES (scipy.sparse.linalg.minres statement order, shift 0, x0 = 0) with
 * the tree preconditioner above; x (n) out. Returns iterations; *relres = phibar / beta1.
 * pc_* arrays: precond.py TreePreconditioner (single rank).
 */
API int nxc_minres(int64_t n, const int* rp, const int* col, const double* val, const double* b,
                   double rtol, int maxit, int N, const double* dq, int exact, int64_t n_chains,
                   const int* chain_edge, const int* chain_flip, const int* chain_up,
                   const int* chain_lo, int64_t n_slots, const int* slot_lam,
                   const int* slot_pchain, const int* slot_parent, const int* slot_dc_off,
                   const int* slot_dc, int n_jobs, const int* job_chain_off,
                   const int* job_lvl_off, const int* lvl_slot_off, int n_top_lvl,
                   const int* top_lvl_off, double* x, double* relres) {
  Pc p = {N, exact, n_chains, n_slots, n_jobs, n_top_lvl, chain_edge, chain_flip, chain_up,
          chain_lo, slot_lam, slot_pchain, slot_parent, slot_dc_off, slot_dc, job_chain_off,
          job_lvl_off, lvl_slot_off, top_lvl_off, dq, NULL, NULL, NULL, NULL, NULL, NULL, NULL};
  (void)job_chain_off;
  const size_t nc = (size_t)(n_chains > 0 ? n_chains : 1), ns = (size_t)(n_slots > 0 ? n_slots : 1);
  p.T = (double*)malloc(sizeof(double) * nc);
  p.It = (double*)malloc(sizeof(double) * nc);
  p.Ib = (double*)malloc(sizeof(double) * nc);
  p.D = (double*)malloc(sizeof(double) * ns);
  p.J = (double*)malloc(sizeof(double) * ns);
  p.z_slot = (double*)malloc(sizeof(double) * ns);
  p.lu = (double*)malloc(sizeof(double) * 2 * (size_t)(N + 1));
  {
    double u = 2.0;
    p.lu[0] = 0.0;
    p.lu[N + 1] = 1.0 / u;
    for (int k = 1; k <= N; ++k) {
      const double l = 1.0 / u;
      u = (k == N ? 2.0 : 4.0) - l;
      p.lu[k] = l;
      p.lu[N + 1 + k] = 1.0 / u;
    }
  }
  const size_t nb = sizeof(double) * (size_t)(n > 0 ? n : 1);
  /* w1 = w_{k-2}, w2 = w_{k-1} (both zero at the start) */
  double *r1 = malloc(nb), *r2 = malloc(nb), *y = malloc(nb), *v = malloc(nb), *w1 = malloc(nb),
         *w2 = malloc(nb);
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) {
    r1[i] = b[i];
    r2[i] = b[i];
    x[i] = 0.0;
    w1[i] = 0.0;
    w2[i] = 0.0;
  }
  const double bb = pc_apply(&p, r1, y);
  const double beta1 = sqrt(bb);
  double oldb = 0.0, beta = beta1, dbar = 0.0, epsln = 0.0, phibar = beta1, cs = -1.0, sn = 0.0;
  int itn = 0;
  *relres = beta1 > 0.0 ? 1.0 : 0.0;
  while (beta1 > 0.0 && itn < maxit) {
    ++itn;
    const double s = 1.0 / beta;
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) v[i] = s * y[i];
    spmv(n, rp, col, val, v, y);
    double alfa = 0.0;
    const double c1 = itn >= 2 ? beta / oldb : 0.0;
#pragma omp parallel for schedule(static) reduction(+ : alfa)
    for (int64_t i = 0; i < n; ++i) {
      const double t = y[i] - c1 * r1[i];
      y[i] = t;
      alfa += v[i] * t;
    }
    const double c2 = alfa / beta;
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
      const double t = y[i] - c2 * r2[i];
      r1[i] = r2[i];
      r2[i] = t;
    }
    oldb = beta;
    beta = sqrt(pc_apply(&p, r2, y));
    const double oldeps = epsln;
    const double delta = cs * dbar + sn * alfa;
    const double gbar = sn * dbar - cs * alfa;
    epsln = sn * beta;
    dbar = -cs * beta;
    double gamma = hypot(gbar, beta);
    if (gamma < 2.220446049250313e-16) gamma = 2.220446049250313e-16;
    cs = gbar / gamma;
    sn = beta / gamma;
    const double phi = cs * phibar;
    phibar = sn * phibar;
    const double denom = 1.0 / gamma;
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
      const double wn = (v[i] - oldeps * w1[i] - delta * w2[i]) * denom;
      w1[i] = w2[i];
      w2[i] = wn;
      x[i] += phi * wn;
    }
    *relres = phibar / beta1;
    if (*relres <= rtol || beta == 0.0) break;
  }
  free(r1); free(r2); free(y); free(v); free(w1); free(w2);
  free(p.T); free(p.It); free(p.Ib); free(p.D); free(p.J); free(p.z_slot); free(p.lu);
  return itn;
}

/*
 * The direct tree solve on the host (csrc/nxhip.hip kModeDirect, the GPU's default): one
 * pass, the true residual ||b - A x|| / ||b||, one refinement step when it exceeds rtol.
 * Returns the passes run (1 or 2); *relres = the final true residual.
 */
API int nxc_direct(int64_t n, const int* rp, const int* col, const double* val, const double* b,
                   double rtol, int N, const double* dq, int64_t n_chains,
                   const int* chain_edge, const int* chain_flip, const int* chain_up,
                   const int* chain_lo, int64_t n_slots, const int* slot_lam,
                   const int* slot_pchain, const int* slot_parent, const int* slot_dc_off,
                   const int* slot_dc, int n_jobs, const int* job_chain_off,
                   const int* job_lvl_off, const int* lvl_slot_off, int n_top_lvl,
                   const int* top_lvl_off, double* x, double* relres) {
  Pc p = {N, 1, n_chains, n_slots, n_jobs, n_top_lvl, chain_edge, chain_flip, chain_up,
          chain_lo, slot_lam, slot_pchain, slot_parent, slot_dc_off, slot_dc, job_chain_off,
          job_lvl_off, lvl_slot_off, top_lvl_off, dq, NULL, NULL, NULL, NULL, NULL, NULL, NULL};
  const size_t nc = (size_t)(n_chains > 0 ? n_chains : 1), ns = (size_t)(n_slots > 0 ? n_slots : 1);
  p.T = (double*)malloc(sizeof(double) * nc);
  p.It = (double*)malloc(sizeof(double) * nc);
  p.Ib = (double*)malloc(sizeof(double) * nc);
  p.D = (double*)malloc(sizeof(double) * ns);
  p.J = (double*)malloc(sizeof(double) * ns);
  p.z_slot = (double*)malloc(sizeof(double) * ns);
  p.lu = (double*)malloc(sizeof(double) * 2 * (size_t)(N + 1));
  {
    double u = 2.0;
    p.lu[0] = 0.0;
    p.lu[N + 1] = 1.0 / u;
    for (int k = 1; k <= N; ++k) {
      const double l = 1.0 / u;
      u = (k == N ? 2.0 : 4.0) - l;
      p.lu[k] = l;
      p.lu[N + 1 + k] = 1.0 / u;
    }
  }
  const size_t nb = sizeof(double) * (size_t)(n > 0 ? n : 1);
  double *mb = malloc(nb), *r = malloc(nb), *d = malloc(nb);
  int passes = 0;
  for (;;) {
    if (passes == 0) {
      pc_direct(&p, b, x, mb, n);
    } else {  /* refinement: x += A^{-1} (b - A x) */
      pc_direct(&p, r, d, mb, n);
#pragma omp parallel for schedule(static)
      for (int64_t i = 0; i < n; ++i) x[i] += d[i];
    }
    ++passes;
    spmv(n, rp, col, val, x, r);
    double rr = 0.0, bb = 0.0;
#pragma omp parallel for schedule(static) reduction(+ : rr, bb)
    for (int64_t i = 0; i < n; ++i) {
      r[i] = b[i] - r[i];
      rr += r[i] * r[i];
      bb += b[i] * b[i];
    }
    *relres = bb > 0.0 ? sqrt(rr / bb) : sqrt(rr);
    if (*relres <= rtol || passes == 2) break;
  }
  free(mb); free(r); free(d);
  free(p.T); free(p.It); free(p.Ib); free(p.D); free(p.J); free(p.z_slot); free(p.lu);
  return passes;
}
