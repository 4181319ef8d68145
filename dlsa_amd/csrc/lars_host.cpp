// Host LARS / adaptive-lasso path on the LSA quadratic form.
//
// Behavioural spec: dlsa/lsa.py:90-212 (the Python port of R lars.lsa that
// dlsa/dlsa.py:77-80 calls).  The path is a LAR / LASSO homotopy on the
// quadratic loss (b - beta)^T Sigma (b - beta) after the adaptive rescaling
// Sigma <- D Sigma D, b <- sign(b), D = diag|b0| (lsa.py:108-109), with an
// incrementally updated Cholesky factor R of the active Gram block
// (lsa.py:12-32 update, lsa.py:35-80 Givens downdate).  Each knot reports
// RSS_k, BIC = RSS + log(n) dof (the DBIC of the paper) and AIC = RSS + 2 dof
// (lsa.py:190-211).
//
// Reference defects fixed: the intercept branch uses the
// parameter count (lsa.py:100 used the sample size n and raises IndexError);
// the singular back-out keeps the leading block of R (lsa.py:141-142 indexed
// a diagonal).  A knot's "C" vector for the step length is taken over the
// columns that are neither active nor ignored, which is what lsa.py:157-161
// computes whenever no variable has been ignored.
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <immintrin.h>

#include <algorithm>
#include <string>
#include <vector>

#include "../../include/dlsa_hip.h"

namespace dlsa {
void set_error(const std::string& msg);
}

namespace {

// y += alpha x
inline void axpy(
    int n, double alpha, const double* __restrict x, double* __restrict y) {
  for (int i = 0; i < n; ++i) y[i] += alpha * x[i];
}

// sum_i x[i] y[i] with 4 partial sums
inline double dot(
    int n, const double* __restrict x, const double* __restrict y) {
  double s0 = 0, s1 = 0, s2 = 0, s3 = 0;
  int i = 0;
  for (; i + 4 <= n; i += 4) {
    s0 += x[i] * y[i];
    s1 += x[i + 1] * y[i + 1];
    s2 += x[i + 2] * y[i + 2];
    s3 += x[i + 3] * y[i + 3];
  }
  for (; i < n; ++i) s0 += x[i] * y[i];
  return (s0 + s1) + (s2 + s3);
}

// out[j] = Sp[j, 0..n) . w for every j in rows (Sp: row-major, leading dimension ld): four rows per pass share
// each load of w (AVX2 FMA, 2 accumulators per row)
void dots_rows(int n, const double* Sp, size_t ld, const std::vector<int>& rows, const double* w,
               double* out) {
  size_t t = 0;
  const int n8 = n & ~7;
  for (; t + 4 <= rows.size(); t += 4) {
    const double* r0 = Sp + (size_t)rows[t] * ld;
    const double* r1 = Sp + (size_t)rows[t + 1] * ld;
    const double* r2 = Sp + (size_t)rows[t + 2] * ld;
    const double* r3 = Sp + (size_t)rows[t + 3] * ld;
    __m256d a0 = _mm256_setzero_pd(), b0 = _mm256_setzero_pd();
    __m256d a1 = _mm256_setzero_pd(), b1 = _mm256_setzero_pd();
    __m256d a2 = _mm256_setzero_pd(), b2 = _mm256_setzero_pd();
    __m256d a3 = _mm256_setzero_pd(), b3 = _mm256_setzero_pd();
    for (int i = 0; i < n8; i += 8) {
      const __m256d w0 = _mm256_loadu_pd(w + i), w1 = _mm256_loadu_pd(w + i + 4);
      a0 = _mm256_fmadd_pd(_mm256_loadu_pd(r0 + i), w0, a0);
      b0 = _mm256_fmadd_pd(_mm256_loadu_pd(r0 + i + 4), w1, b0);
      a1 = _mm256_fmadd_pd(_mm256_loadu_pd(r1 + i), w0, a1);
      b1 = _mm256_fmadd_pd(_mm256_loadu_pd(r1 + i + 4), w1, b1);
      a2 = _mm256_fmadd_pd(_mm256_loadu_pd(r2 + i), w0, a2);
      b2 = _mm256_fmadd_pd(_mm256_loadu_pd(r2 + i + 4), w1, b2);
      a3 = _mm256_fmadd_pd(_mm256_loadu_pd(r3 + i), w0, a3);
      b3 = _mm256_fmadd_pd(_mm256_loadu_pd(r3 + i + 4), w1, b3);
    }
    double s[4][4];
    _mm256_storeu_pd(s[0], _mm256_add_pd(a0, b0));
    _mm256_storeu_pd(s[1], _mm256_add_pd(a1, b1));
    _mm256_storeu_pd(s[2], _mm256_add_pd(a2, b2));
    _mm256_storeu_pd(s[3], _mm256_add_pd(a3, b3));
    const double* rr[4] = {r0, r1, r2, r3};
    for (int u = 0; u < 4; ++u) {
      double v = (s[u][0] + s[u][1]) + (s[u][2] + s[u][3]);
      for (int i = n8; i < n; ++i) v += rr[u][i] * w[i];
      out[rows[t + u]] = v;
    }
  }
  for (; t < rows.size(); ++t) out[rows[t]] = dot(n, Sp + (size_t)rows[t] * ld, w);
}

struct Chol {
  // upper-triangular R (d x d) stored with leading dimension m, and its
  // transpose lt (row i of lt = column i of R) for the backward solve
  int m = 0, d = 0;
  std::vector<double> r, lt;
  explicit Chol(int m_) : m(m_), d(0), r((size_t)m_ * m_, 0.0), lt((size_t)m_ * m_, 0.0) {}
  // after R changed other than by an appended column (Givens downdate)
  void rebuild_lt() {
    for (int i = 0; i < d; ++i)
      for (int k = 0; k <= i; ++k) lt[(size_t)i * m + k] = r[(size_t)k * m + i];
  }
  double& at(int i, int j) { return r[(size_t)i * m + j]; }
  double at(int i, int j) const { return r[(size_t)i * m + j]; }
  // solve R^T x = b (forward)
  // (column-oriented: row k of R is contiguous; x[i] still subtracts its
  // terms in k order, so the rounding is that of the dot-product form)
  // Four columns per sweep: the block's four entries are finalised in order,
  // then the rest of x takes the four columns' updates in one pass (each
  // element still subtracts them in k order, so the result is bitwise that of
  // the one-column sweep, with a quarter of the dependent store-load chain).
  void solve_rt(const double* b, double* x) const {
    for (int i = 0; i < d; ++i) x[i] = b[i];
    int k = 0;
    for (; k + 4 <= d; k += 4) {
      const double* r0 = &r[(size_t)k * m];
      const double* r1 = r0 + m;
      const double* r2 = r1 + m;
      const double* r3 = r2 + m;
      const double x0 = x[k] / r0[k];
      x[k] = x0;
      x[k + 1] += -x0 * r0[k + 1];
      x[k + 2] += -x0 * r0[k + 2];
      x[k + 3] += -x0 * r0[k + 3];
      const double x1 = x[k + 1] / r1[k + 1];
      x[k + 1] = x1;
      x[k + 2] += -x1 * r1[k + 2];
      x[k + 3] += -x1 * r1[k + 3];
      const double x2 = x[k + 2] / r2[k + 2];
      x[k + 2] = x2;
      x[k + 3] += -x2 * r2[k + 3];
      const double x3 = x[k + 3] / r3[k + 3];
      x[k + 3] = x3;
      for (int j = k + 4; j < d; ++j) {
        double v = x[j];
        v += -x0 * r0[j];
        v += -x1 * r1[j];
        v += -x2 * r2[j];
        v += -x3 * r3[j];
        x[j] = v;
      }
    }
    for (; k < d; ++k) {
      const double xk = x[k] / at(k, k);
      x[k] = xk;
      axpy(d - k - 1, -xk, &r[(size_t)k * m + k + 1], x + k + 1);
    }
  }
  // solve R x = b (backward), column-oriented on lt: x[i] is final once the
  // terms of x[i+1..d) are subtracted; each then updates x[0..i) with one
  // contiguous axpy (no per-row horizontal reduction on the recurrence)
  // (blocked like solve_rt: four columns per sweep, same per-element order)
  void solve_r(const double* b, double* x) const {
    for (int i = 0; i < d; ++i) x[i] = b[i];
    int i = d - 1;
    for (; i >= 3; i -= 4) {
      const double* l0 = &lt[(size_t)i * m];
      const double* l1 = l0 - m;
      const double* l2 = l1 - m;
      const double* l3 = l2 - m;
      const double x0 = x[i] / l0[i];
      x[i] = x0;
      x[i - 1] += -x0 * l0[i - 1];
      x[i - 2] += -x0 * l0[i - 2];
      x[i - 3] += -x0 * l0[i - 3];
      const double x1 = x[i - 1] / l1[i - 1];
      x[i - 1] = x1;
      x[i - 2] += -x1 * l1[i - 2];
      x[i - 3] += -x1 * l1[i - 3];
      const double x2 = x[i - 2] / l2[i - 2];
      x[i - 2] = x2;
      x[i - 3] += -x2 * l2[i - 3];
      const double x3 = x[i - 3] / l3[i - 3];
      x[i - 3] = x3;
      for (int q = 0; q < i - 3; ++q) {
        double v = x[q];
        v += -x0 * l0[q];
        v += -x1 * l1[q];
        v += -x2 * l2[q];
        v += -x3 * l3[q];
        x[q] = v;
      }
    }
    for (; i >= 0; --i) {
      const double* li = &lt[(size_t)i * m];
      const double xi = x[i] / li[i];
      x[i] = xi;
      axpy(i, -xi, li, x);
    }
  }
};

}  // namespace

extern "C" int dlsa_lars_lsa(const double* Sigma0, const double* b0, int32_t P,
                             int32_t intercept, double n, int32_t type, double eps,
                             int32_t max_steps, double* beta_out, double* beta0_out,
                             double* aic, double* bic, int32_t* n_steps) {
  using dlsa::set_error;
  // flush-to-zero / denormals-are-zero for the path: correlations decaying
  // through the subnormal range made steps 10-20x slower (P = 182: 21 ms vs
  // 3 ms at P = 150); values below 2^-1022 do not change any knot, RSS or BIC
  struct FtzScope {
    unsigned int saved;
    FtzScope() : saved(_mm_getcsr()) { _mm_setcsr(saved | 0x8040); }
    ~FtzScope() { _mm_setcsr(saved); }
  } ftz;
  if (!Sigma0 || !b0 || P < 1 + (intercept ? 1 : 0) || !beta_out || !beta0_out || !aic || !bic ||
      !n_steps) {
    set_error("dlsa_lars_lsa: invalid arguments");
    return DLSA_E_INVALID;
  }
  const bool lasso = type == 1;
  if (!(eps > 0)) eps = 2.220446049250313e-16;
  const int ic = intercept ? 1 : 0;
  const int m = P - ic;
  if (max_steps <= 0) max_steps = 8 * m;

  // quadratic form after removing the intercept (Schur complement)
  std::vector<double> Sig((size_t)m * m), b(m), a12(ic ? m : 0);
  double a11 = 1.0, beta0_init = 0.0;
  if (ic) {
    a11 = Sigma0[0];
    for (int i = 0; i < m; ++i) a12[i] = Sigma0[(size_t)(i + 1) * P];
    for (int i = 0; i < m; ++i)
      for (int j = 0; j < m; ++j)
        Sig[(size_t)i * m + j] = Sigma0[(size_t)(i + 1) * P + (j + 1)] - a12[i] * a12[j] / a11;
    for (int i = 0; i < m; ++i) b[i] = b0[i + 1];
    double s = 0;
    for (int i = 0; i < m; ++i) s += a12[i] * b[i];
    beta0_init = s / a11;
  } else {
    for (size_t e = 0; e < (size_t)m * m; ++e) Sig[e] = Sigma0[e];
    for (int i = 0; i < m; ++i) b[i] = b0[i];
  }
  std::vector<double> absb(m), sgnb(m);
  for (int i = 0; i < m; ++i) {
    absb[i] = fabs(b[i]);
    sgnb[i] = (b[i] > 0) - (b[i] < 0);
  }
  for (int i = 0; i < m; ++i)
    for (int j = 0; j < m; ++j) Sig[(size_t)i * m + j] *= absb[i] * absb[j];
  auto S = [&](int i, int j) { return Sig[(size_t)i * m + j]; };

  // SA: the active columns of Sigma, row-major (leading dimension m), column
  // slot[q] holding active variable q.  The equiangular correlations of an
  // inactive row j are then one contiguous dot product SA[j, 0..|A|) . w'
  // (w' = w in slot order), and those of an active column are A * Sign
  // exactly (Sigma_AA w = A Sigma_AA Sigma_AA^-1 Sign): (m - |A|) |A|
  // multiply-adds per knot.  Adding a variable writes one column (its row of
  // the symmetric Sigma); a lasso drop (rare) compacts the kept columns into
  // slots 0..|A|-1 in active order, so slot[q] = q always and every dot
  // product sums in active order (the column swaps of round 2 touched two
  // strided columns per added variable).
  std::vector<double> SA((size_t)m * m, 0.0);
  std::vector<int> slot;
  auto put_col = [&](int s_, int var) {
    const double* src = &Sig[(size_t)var * m];
    for (int i = 0; i < m; ++i) SA[(size_t)i * m + s_] = src[i];
  };

  std::vector<double> Cvec(m, 0.0);
  for (int j = 0; j < m; ++j) {
    double s = 0;
    for (int i = 0; i < m; ++i) s += sgnb[i] * S(i, j);
    Cvec[j] = s;
  }

  const size_t rows = (size_t)max_steps + 1;
  // only the knots reached are written (row k is copied from row k-1 before
  // its update): no memset of the max_steps x m output (16 MB at m = 500, and
  // its page faults, cost more than the path itself)
  memset(beta_out, 0, sizeof(double) * m);
  std::vector<double> Csnap;  // Cvec after each knot (knot 0: beta = 0)
  Csnap.reserve((size_t)std::min<size_t>(rows, 2 * (size_t)m + 2) * m);
  Csnap.insert(Csnap.end(), Cvec.begin(), Cvec.end());
  auto B = [&](int k, int j) -> double& { return beta_out[(size_t)k * m + j]; };

  std::vector<int> active, ignores;
  std::vector<double> Sign;
  std::vector<char> in_active(m, 0), in_ignores(m, 0);
  std::vector<char> drops;  // per active position, from the last lasso step
  bool any_drop = false;
  Chol R(m);
  int rank = 0;
  int k = 0;
  std::vector<double> C, u, Gi1, w, a, wslot;
  bool u_valid = false;
  std::vector<int> inactive;
  std::vector<double> keepm;  // -1.0 (sign bit set) for the columns the step length scans
  while (k < max_steps && (int)active.size() < m) {
    ++k;
    inactive.clear();
    for (int j = 0; j < m; ++j)
      if (!in_active[j]) inactive.push_back(j);
    double Cmax = 0;
    for (int j : inactive) Cmax = std::max(Cmax, fabs(Cvec[j]));
    if (!any_drop) {
      for (int j : inactive) {
        if (!(fabs(Cvec[j]) >= Cmax - eps)) continue;
        // add variable j: extend R by the column [R^-T Sigma_A,j ; rpp]
        const int da = R.d;
        if (da == 0) {
          R.d = 1;
          R.at(0, 0) = sqrt(S(j, j));
          R.lt[0] = R.at(0, 0);
          rank = 1;
        } else {
          std::vector<double> xold(da), rcol(da);
          for (int q = 0; q < da; ++q) xold[q] = S(j, active[q]);
          R.solve_rt(xold.data(), rcol.data());
          double rpp = S(j, j);
          for (int q = 0; q < da; ++q) rpp -= rcol[q] * rcol[q];
          if (rpp <= eps) {
            rpp = eps;
          } else {
            rpp = sqrt(rpp);
            ++rank;
          }
          for (int q = 0; q < da; ++q) R.at(q, da) = rcol[q];
          for (int q = 0; q < da; ++q) R.at(da, q) = 0.0;
          R.at(da, da) = rpp;
          for (int q = 0; q < da; ++q) R.lt[(size_t)da * m + q] = rcol[q];
          R.lt[(size_t)da * m + da] = rpp;
          R.d = da + 1;
        }
        if (rank == (int)active.size()) {  // singular: back out, ignore j
          R.d = (int)active.size();
          ignores.push_back(j);
          in_ignores[j] = 1;
        } else {
          put_col((int)active.size(), j);
          slot.push_back((int)active.size());
          active.push_back(j);
          in_active[j] = 1;
          Sign.push_back((Cvec[j] > 0) - (Cvec[j] < 0));
        }
      }
    }
    const int na = (int)active.size();
    if (na == 0) {  // knot k stays the zero row (as with a pre-zeroed output)
      memset(&B(k, 0), 0, sizeof(double) * m);
      Csnap.resize((size_t)(k + 1) * m, 0.0);
      break;
    }
    // Gi1 = (R^T R)^-1 Sign ; A = 1/sqrt(Sign . Gi1) ; w = A Gi1.
    // u = R^-T Sign is kept across knots: R^T is lower triangular, so adding
    // a variable (a new last row of R^T, a new last entry of Sign) leaves the
    // leading entries of u unchanged and only the new ones are computed, in
    // the forward solve's own order (same rounding); a Givens downdate (lasso
    // drop) rotates R and the whole u is recomputed.
    if (!u_valid || (int)u.size() > na) {
      u.assign(na, 0.0);
      R.solve_rt(Sign.data(), u.data());
      u_valid = true;
    } else {
      for (int i = (int)u.size(); i < na; ++i) {
        double x = Sign[i];
        for (int q = 0; q < i; ++q) x -= R.at(q, i) * u[q];
        u.push_back(x / R.at(i, i));
      }
    }
    Gi1.assign(na, 0.0);
    R.solve_r(u.data(), Gi1.data());
    double sg = 0;
    for (int q = 0; q < na; ++q) sg += Gi1[q] * Sign[q];
    const double A = 1.0 / sqrt(sg);
    w.assign(na, 0.0);
    for (int q = 0; q < na; ++q) w[q] = A * Gi1[q];
    double gamhat = Cmax / A;
    // a = Sigma[:, active] w: the equiangular correlations of every column,
    // used by the step length and by the correlation update (see SA)
    a.resize(m);
    inactive.clear();
    for (int j = 0; j < m; ++j)
      if (!in_active[j]) inactive.push_back(j);
    wslot.assign(na, 0.0);
    for (int q = 0; q < na; ++q) wslot[slot[q]] = w[q];
    dots_rows(na, SA.data(), (size_t)m, inactive, wslot.data(), a.data());
    for (int q = 0; q < na; ++q) a[active[q]] = A * Sign[q];
    if (na < m) {
      // min over the columns neither active nor ignored of the positive step
      // lengths (Cmax -+ c_j) / (A -+ a_j): four columns per AVX2 pass (the same
      // IEEE divisions and an exact min, so the result is that of the scalar
      // loop)
      keepm.resize(m);
      for (int j = 0; j < m; ++j) keepm[j] = (!in_active[j] && !in_ignores[j]) ? -1.0 : 0.0;
      const __m256d vC = _mm256_set1_pd(Cmax), vA = _mm256_set1_pd(A);
      const __m256d veps = _mm256_set1_pd(eps), vinf = _mm256_set1_pd(INFINITY);
      __m256d vg = _mm256_set1_pd(gamhat);
      int j = 0;
      for (; j + 4 <= m; j += 4) {
        const __m256d aj = _mm256_loadu_pd(&a[j]), c = _mm256_loadu_pd(&Cvec[j]);
        const __m256d keepv = _mm256_loadu_pd(&keepm[j]);  // all-ones sign bit where kept
        const __m256d g1 = _mm256_div_pd(_mm256_sub_pd(vC, c), _mm256_sub_pd(vA, aj));
        const __m256d g2 = _mm256_div_pd(_mm256_add_pd(vC, c), _mm256_add_pd(vA, aj));
        const __m256d m1 = _mm256_and_pd(_mm256_cmp_pd(g1, veps, _CMP_GT_OQ), keepv);
        const __m256d m2 = _mm256_and_pd(_mm256_cmp_pd(g2, veps, _CMP_GT_OQ), keepv);
        vg = _mm256_min_pd(vg, _mm256_blendv_pd(vinf, g1, m1));
        vg = _mm256_min_pd(vg, _mm256_blendv_pd(vinf, g2, m2));
      }
      double gv[4];
      _mm256_storeu_pd(gv, vg);
      gamhat = std::min(std::min(gv[0], gv[1]), std::min(gv[2], gv[3]));
      for (; j < m; ++j) {
        if (keepm[j] == 0.0) continue;
        const double aj = a[j];
        const double c = Cvec[j];
        const double g1 = (Cmax - c) / (A - aj), g2 = (Cmax + c) / (A + aj);
        if (g1 > eps) gamhat = std::min(gamhat, g1);
        if (g2 > eps) gamhat = std::min(gamhat, g2);
      }
    }
    any_drop = false;
    drops.assign(na, 0);
    if (lasso) {
      double zmin = gamhat;
      std::vector<double> z1(na);
      for (int q = 0; q < na; ++q) {
        z1[q] = -B(k - 1, active[q]) / w[q];
        if (z1[q] > eps) zmin = std::min(zmin, z1[q]);
      }
      if (zmin < gamhat) {
        gamhat = zmin;
        for (int q = 0; q < na; ++q) drops[q] = z1[q] == zmin;
        any_drop = true;
      }
    }
    for (int j = 0; j < m; ++j) B(k, j) = B(k - 1, j);
    for (int q = 0; q < na; ++q) B(k, active[q]) += gamhat * w[q];
    for (int j = 0; j < m; ++j) Cvec[j] -= gamhat * a[j];
    // Cvec = Sigma (sign b - beta_k): the knot's RSS is dff . Cvec (O(m)
    // instead of an O(m^2) quadratic form per knot at the end)
    Csnap.insert(Csnap.end(), Cvec.begin(), Cvec.end());  // row k
    if (lasso && any_drop) {
      for (int q = na - 1; q >= 0; --q) {
        if (!drops[q]) continue;
        // downdate: delete column q of R, re-triangularise with Givens
        const int d = R.d;
        if (d == 1) {
          R.d = 0;
          continue;
        }
        for (int i = 0; i < d; ++i)
          for (int c = q; c < d - 1; ++c) R.at(i, c) = R.at(i, c + 1);
        for (int i = q + 1; i < d; ++i) {
          const double aa = R.at(i - 1, i - 1), bb = R.at(i, i - 1);
          if (bb == 0) continue;
          double c, s;
          if (!(fabs(bb) > fabs(aa))) {
            const double tau = -bb / aa;
            c = 1 / sqrt(1 + tau * tau);
            s = c * tau;
          } else {
            const double tau = -aa / bb;
            s = 1 / sqrt(1 + tau * tau);
            c = s * tau;
          }
          for (int col = i - 1; col < d - 1; ++col) {
            const double x1 = R.at(i - 1, col), x2 = R.at(i, col);
            R.at(i - 1, col) = c * x1 - s * x2;
            R.at(i, col) = s * x1 + c * x2;
          }
        }
        for (int col = 0; col < d; ++col) R.at(d - 1, col) = 0.0;
        R.d = d - 1;
      }
      rank = R.d;
      R.rebuild_lt();
      u_valid = false;
      std::vector<int> na_active, na_slot;
      std::vector<double> na_sign;
      for (int q = 0; q < na; ++q) {
        if (drops[q]) {
          B(k, active[q]) = 0.0;
          in_active[active[q]] = 0;
        } else {
          na_active.push_back(active[q]);
          na_slot.push_back(slot[q]);
          na_sign.push_back(Sign[q]);
        }
      }
      active.swap(na_active);
      Sign.swap(na_sign);
      // renumber the kept columns' slots in active order (slot[q] = q): the
      // dot products of dots_rows then sum in active order after a drop too,
      // the same order as a run without drops
      {
        const int na2 = (int)active.size();
        std::vector<double> tmp((size_t)m * na2);
        for (int i = 0; i < m; ++i)
          for (int q = 0; q < na2; ++q) tmp[(size_t)i * na2 + q] = SA[(size_t)i * m + na_slot[q]];
        for (int i = 0; i < m; ++i)
          for (int q = 0; q < na2; ++q) SA[(size_t)i * m + q] = tmp[(size_t)i * na2 + q];
        slot.resize(na2);
        for (int q = 0; q < na2; ++q) slot[q] = q;
      }
    }
  }

  const int nst = k + 1;
  *n_steps = nst;
  const double logn = log(n);
  std::vector<double> dff(m);
  for (int s = 0; s < nst; ++s) {
    for (int j = 0; j < m; ++j) dff[j] = sgnb[j] - B(s, j);
    // rss = dff^T Sigma dff = dff . (Sigma dff) = dff . Cvec_s (lsa.py:191-192)
    const double rss = dot(m, dff.data(), &Csnap[(size_t)s * m]);
    int dof = 0;
    double b0s = beta0_init;
    for (int j = 0; j < m; ++j) {
      const double v = B(s, j) * absb[j];
      B(s, j) = v;
      if (fabs(v) > eps) ++dof;
      if (ic) b0s -= a12[j] * v / a11;
    }
    beta0_out[s] = ic ? b0s : 0.0;
    bic[s] = rss + logn * dof;
    aic[s] = rss + 2.0 * dof;
  }
  return DLSA_OK;
}
