// Multitask / derivative-informed fast GPs (num_tasks > 1 or derivative multi-indices) on MI355X.
//
// Reference: fastgps/util.py:275-363 (_FastInverseLogDetCache, num_tasks > 1), abstract_fast_gp.py:
// 173-191 (kernel parts with beta / kappa), fast_gp_lattice.py:267-273, fast_gp_digital_net_b2.py:
// 289-301 (derivative parts), abstract_gp.py:352-474 (predictions).
//
// The transform-domain Gram matrix of T tasks (sorted by n descending, util.py:273) splits into n_min
// independent R x R Hermitian blocks, one per frequency class j < n_min, R = sum_k n_k / n_min:
//   Lambda_j[(k, q), (l, p)] = lams[k, l][q n_min + j]   iff  k <= l and p == q mod (n_l / n_min)
// (conjugate mirror below the diagonal, zero elsewhere).  The reference inverts it by an unpivoted
// complex Schur-complement bordering that grows a dense [R, R, n_min] inverse (util.py:299-323).
// Here each block gets a structured LDL^H that never leaves the coupling pattern (k_mt_ldl), solves
// by substitution (k_mt_solve) and the inverse's entries on that pattern by Takahashi's recurrence
// (k_mt_selinv): O(R T^2) per class, real pivots (the Schur complements of a Hermitian matrix), all
// arrays in the packed layout of the lams [problem][sum_{k<=l} n_k] with the frequency class fastest,
// one thread per (problem, class) so that a wavefront's accesses are contiguous.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "../../include/fgp_hip.h"
#include "fgp_common.h"
#include "fgp_runtime.h"

namespace fgp {

// ------------------------------------------------------------------------------------------------
// derivative kernel parts
// Bernoulli polynomial of any order 1..8: even orders by the u = x (x - 1) form shared with the fit
// kernels (bernoulli()), odd orders B_{2k+1} by Horner's rule in x as qmcpy.kernel_methods.bernoulli_poly.
__device__ __forceinline__ double bernoulli_any(int order, double x) {
  switch (order) {
    case 1: return x - 0.5;
    case 3: return __builtin_fma(__builtin_fma(x, x, -1.5 * x), x, 0.5 * x);
    case 5: {
      double y = x - 2.5;
      y = __builtin_fma(y, x, 5.0 / 3.0);
      y = y * x;
      y = __builtin_fma(y, x, -1.0 / 6.0);
      return y * x;
    }
    case 7: {
      double y = x - 3.5;
      y = __builtin_fma(y, x, 3.5);
      y = y * x;
      y = __builtin_fma(y, x, -7.0 / 6.0);
      y = y * x;
      y = __builtin_fma(y, x, 1.0 / 6.0);
      return y * x;
    }
    default: return bernoulli(order, x);
  }
}

// parts[i][k][p][j] for x_i (i < N) against z_k (k < M), P (beta, kappa) pairs, d dimensions
// (zip: N == M, the pairs (x_i, z_i) only, parts[i][p][j]):
//   lattice: coef[p][j] * B_{order[p][j]}((x_ij - z_kj) mod 1)
//   net:     coef[p][j] * (add[p][j] + omega_{order[p][j]}(xb_ij XOR zb_kj))
__global__ __launch_bounds__(kWG) void k_mt_parts(int family, const void* __restrict__ xv, int64_t xs, int64_t N,
                                                  const void* __restrict__ zv, int64_t zs, int64_t M, int zip, int d, int P,
                                                  const int* __restrict__ order, const double* __restrict__ coef,
                                                  const double* __restrict__ add, int t, double* __restrict__ out) {
  const int64_t e = (int64_t)blockIdx.x * kWG + threadIdx.x;
  if (e >= (zip ? N : N * M)) return;
  const int64_t i = zip ? e : e / M, k = zip ? e : e - i * M;
  double* o = out + e * (int64_t)P * d;
  for (int j = 0; j < d; ++j) {
    if (family == 0) {
      const double delta = mod1(static_cast<const double*>(xv)[i * xs + j] - static_cast<const double*>(zv)[k * zs + j]);
      for (int p = 0; p < P; ++p) o[p * d + j] = coef[p * d + j] * bernoulli_any(order[p * d + j], delta);
    } else {
      const unsigned long long delta = (unsigned long long)(static_cast<const int64_t*>(xv)[i * xs + j] ^
                                                            static_cast<const int64_t*>(zv)[k * zs + j]);
      for (int p = 0; p < P; ++p) {
        const int od = order[p * d + j];
        const double om = od == 1 ? walsh1(delta, t) : walsh_omega(od, delta, t);
        o[p * d + j] = coef[p * d + j] * (add[p * d + j] + om);
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// block layout
struct MtLay {
  int T;                          // active (n > 0) tasks, sorted by n descending
  int R;                          // rows per block
  int64_t nmin;                   // frequency classes
  int64_t L;                      // packed length per problem: sum_{k <= l} n_k
  int64_t n[FGP_MT_MAX_TASKS];
  int rs[FGP_MT_MAX_TASKS];       // first row of task k
  int64_t off[FGP_MT_MAX_TASKS * FGP_MT_MAX_TASKS];   // packed offset of lams[k, l], k <= l
};

__device__ __forceinline__ double2 conj2(double2 a) { return make_double2(a.x, -a.y); }
__device__ __forceinline__ double2 cmul_cj(double2 a, double2 b) {   // conj(a) * b
  return make_double2(__builtin_fma(a.x, b.x, a.y * b.y), __builtin_fma(a.x, b.y, -a.y * b.x));
}

// ------------------------------------------------------------------------------------------------
// Structured LDL^H.  Order the rows task by task (largest n first).  Task k's rows form a DIAGONAL block
// and each row (k, q) couples to exactly one row (l, q mod q_l) of every later task l, so eliminating
// task k leaves that pattern intact (no fill-in):
//   D_k[q]  = Lambda[(k,q),(k,q)]                 (after the updates of the earlier tasks; real)
//   u_kl[q] = Lambda[(k,q),(l,q mod q_l)] / D_k[q]
//   Lambda[(l,p),(m,p mod q_m)] -= sum_{q : q mod q_l = p} conj(u_kl[q]) D_k[q] u_km[q]   (k < l <= m)
// so Lambda = L D L^H with L[(l, q mod q_l), (k, q)] = conj(u_kl[q]), and the factor lives in the packed
// layout of the lams themselves: D on the diagonal entries, u on the coupling entries.  Work per
// frequency class is R T^2 / 2 instead of the R^3 / 3 of a dense factorisation (and the reference's
// bordering, util.py:301-323, which grows a dense [R, R] inverse).  logdet_j = sum log |D|.
__global__ __launch_bounds__(kWG) void k_mt_ldl(const double2* __restrict__ lp, int64_t G, MtLay lay,
                                                double2* __restrict__ fac, double* __restrict__ logdet,
                                                int* __restrict__ info) {
  const int64_t e = (int64_t)blockIdx.x * kWG + threadIdx.x;
  if (e >= G * lay.nmin) return;
  const int64_t g = e / lay.nmin, j = e - g * lay.nmin;
  const int64_t nm = lay.nmin;
  const double2* src = lp + g * lay.L + j;
  double2* F = fac + g * lay.L + j;
  for (int64_t i = 0; i < lay.L / nm; ++i) F[i * nm] = src[i * nm];
  double ld = 0.0;
  bool bad = false;
  for (int k = 0; k < lay.T; ++k) {
    const int qk = (int)(lay.n[k] / nm);
    double2* Dk = F + lay.off[k * FGP_MT_MAX_TASKS + k];
    for (int q = 0; q < qk; ++q) {
      double dq = Dk[(int64_t)q * nm].x;
      if (!(dq > 0.0)) bad = true;
      ld += log(fabs(dq));      // log|S| as the reference's recursion takes it (util.py:299,310)
      Dk[(int64_t)q * nm] = make_double2(dq, 0.0);
      const double idq = 1.0 / dq;
      // updates of the later tasks' blocks (from the unscaled couplings c = D u), then u = c / D
      for (int l = k + 1; l < lay.T; ++l) {
        const int ql = (int)(lay.n[l] / nm);
        const double2 cl = F[lay.off[k * FGP_MT_MAX_TASKS + l] + (int64_t)q * nm];
        const double2 ul = cl * idq;
        for (int m = l; m < lay.T; ++m) {
          const double2 cm = F[lay.off[k * FGP_MT_MAX_TASKS + m] + (int64_t)q * nm];
          double2* t = F + lay.off[l * FGP_MT_MAX_TASKS + m] + (int64_t)(q % ql) * nm;
          *t -= cmul_cj(ul, cm);                       // conj(u_kl) c_km
        }
      }
      for (int l = k + 1; l < lay.T; ++l) {
        double2* c = F + lay.off[k * FGP_MT_MAX_TASKS + l] + (int64_t)q * nm;
        *c = *c * idq;
      }
    }
  }
  logdet[e] = ld;            // a non-positive pivot still counts as log|pivot| (the reference's log|S|); info flags it
  if (bad) info[0] = 1;
}

// out[b] = Lambda_{g(b)}^-1 v[b] (g(b) = b mod G), per frequency class: forward substitution with L,
// scaling by D^-1, back substitution with L^H -- O(R T) per vector and class.  v, out: [B][R nmin]
// (rows of the sorted tasks concatenated, the reference's [..., R, n_min] view, util.py:356-360).
__global__ __launch_bounds__(kWG) void k_mt_solve(const double2* __restrict__ fac, int64_t G, MtLay lay,
                                                  const double2* __restrict__ v, int64_t vs, int64_t B,
                                                  double2* __restrict__ out) {
  const int64_t e = (int64_t)blockIdx.x * kWG + threadIdx.x;
  if (e >= B * lay.nmin) return;
  const int64_t nm = lay.nmin;
  const int64_t b = e / nm, j = e - b * nm, g = b % G;
  const double2* F = fac + g * lay.L + j;
  const double2* vb = v + b * vs + j;
  double2* o = out + b * (int64_t)lay.R * nm + j;
  for (int r = 0; r < lay.R; ++r) o[(int64_t)r * nm] = vb[(int64_t)r * nm];
  for (int k = 0; k < lay.T; ++k) {                    // w = L^-1 v
    const int qk = (int)(lay.n[k] / nm);
    for (int q = 0; q < qk; ++q) {
      const double2 wq = o[(int64_t)(lay.rs[k] + q) * nm];
      for (int l = k + 1; l < lay.T; ++l) {
        const int ql = (int)(lay.n[l] / nm);
        const double2 u = F[lay.off[k * FGP_MT_MAX_TASKS + l] + (int64_t)q * nm];
        o[(int64_t)(lay.rs[l] + q % ql) * nm] -= cmul_cj(u, wq);
      }
    }
  }
  for (int k = 0; k < lay.T; ++k) {                    // w /= D
    const int qk = (int)(lay.n[k] / nm);
    const double2* Dk = F + lay.off[k * FGP_MT_MAX_TASKS + k];
    for (int q = 0; q < qk; ++q) {
      double2* t = o + (int64_t)(lay.rs[k] + q) * nm;
      *t = *t * (1.0 / Dk[(int64_t)q * nm].x);
    }
  }
  for (int k = lay.T - 1; k >= 0; --k) {               // z = L^-H w
    const int qk = (int)(lay.n[k] / nm);
    for (int q = 0; q < qk; ++q) {
      double2 s = o[(int64_t)(lay.rs[k] + q) * nm];
      for (int l = k + 1; l < lay.T; ++l) {
        const int ql = (int)(lay.n[l] / nm);
        const double2 u = F[lay.off[k * FGP_MT_MAX_TASKS + l] + (int64_t)q * nm];
        s -= cmul(u, o[(int64_t)(lay.rs[l] + q % ql) * nm]);
      }
      o[(int64_t)(lay.rs[k] + q) * nm] = s;
    }
  }
}

// Entries of A = Lambda^-1 on the coupling pattern (Takahashi's recurrence Z = D^-1 L^-1 + (I - L^H) Z,
// evaluated on the pattern only, which is closed under it): rows (k, q) from the last task back,
//   Z[(k,q),(m, q mod q_m)] = - sum_{l > k} u_kl[q] Z[(l, q mod q_l), (m, q mod q_m)]     (m > k)
//   Z[(k,q),(k,q)]          = 1 / D_k[q] - sum_{l > k} u_kl[q] conj(Z[(k,q),(l, q mod q_l)])
// written in the packed layout (Z_pack[k][m][q] = Z[(k,q),(m, q mod q_m)]).  These are the entries the
// MLL gradient and post_cubature_var / cov need (A at the first row of every task, class 0).
__device__ __forceinline__ double2 zpat(const double2* Z, const MtLay& lay, int l, int pl, int m, int pm) {
  const int64_t nm = lay.nmin;
  return l <= m ? Z[lay.off[l * FGP_MT_MAX_TASKS + m] + (int64_t)pl * nm]
                : conj2(Z[lay.off[m * FGP_MT_MAX_TASKS + l] + (int64_t)pm * nm]);
}

__global__ __launch_bounds__(kWG) void k_mt_selinv(const double2* __restrict__ fac, int64_t G, MtLay lay,
                                                   double2* __restrict__ zinv) {
  const int64_t e = (int64_t)blockIdx.x * kWG + threadIdx.x;
  if (e >= G * lay.nmin) return;
  const int64_t nm = lay.nmin;
  const int64_t g = e / nm, j = e - g * nm;
  const double2* F = fac + g * lay.L + j;
  double2* Z = zinv + g * lay.L + j;
  for (int k = lay.T - 1; k >= 0; --k) {
    const int qk = (int)(lay.n[k] / nm);
    for (int q = 0; q < qk; ++q) {
      for (int m = k + 1; m < lay.T; ++m) {
        const int pm = q % (int)(lay.n[m] / nm);
        double2 s = make_double2(0.0, 0.0);
        for (int l = k + 1; l < lay.T; ++l) {
          const int pl = q % (int)(lay.n[l] / nm);
          s -= cmul(F[lay.off[k * FGP_MT_MAX_TASKS + l] + (int64_t)q * nm], zpat(Z, lay, l, pl, m, pm));
        }
        Z[lay.off[k * FGP_MT_MAX_TASKS + m] + (int64_t)q * nm] = s;
      }
      double s = 1.0 / F[lay.off[k * FGP_MT_MAX_TASKS + k] + (int64_t)q * nm].x;
      for (int l = k + 1; l < lay.T; ++l) {
        const double2 u = F[lay.off[k * FGP_MT_MAX_TASKS + l] + (int64_t)q * nm];
        const double2 zc = Z[lay.off[k * FGP_MT_MAX_TASKS + l] + (int64_t)q * nm];
        s -= __builtin_fma(u.x, zc.x, u.y * zc.y);     // Re(u conj(z)): the diagonal is real
      }
      Z[lay.off[k * FGP_MT_MAX_TASKS + k] + (int64_t)q * nm] = make_double2(s, 0.0);
    }
  }
}

// Gradient of the MLL data + logdet terms w.r.t. the packed lams (torch's convention for complex
// inputs: dL/dRe + i dL/dIm), with z_b = A y_b, gn[b] = dL/dnorm_b, gl[g] = dL/dlogdet_g and Z the
// selected inverse:
//   coupling entry (r < c):  -2 sum_b gn[b] z_br conj(z_bc) + 2 gl[g] Z_rc
//   diagonal entry:          -sum_b gn[b] |z_br|^2 + gl[g] Z_rr      (real; the imaginary part of a
//                            Hermitian diagonal does not enter)
__global__ __launch_bounds__(kWG) void k_mt_mll_grad(const double2* __restrict__ zinv, const double2* __restrict__ z,
                                                     const double* __restrict__ gn, const double* __restrict__ gl,
                                                     int64_t B, int64_t G, MtLay lay, double2* __restrict__ glp) {
  const int64_t e = (int64_t)blockIdx.x * kWG + threadIdx.x;
  if (e >= G * lay.nmin) return;
  const int64_t g = e / lay.nmin, j = e - g * lay.nmin;
  const int64_t nm = lay.nmin, zs = (int64_t)lay.R * nm;
  const double glg = gl[g];
  const double2* Z = zinv + g * lay.L + j;
  double2* out = glp + g * lay.L + j;
  for (int k = 0; k < lay.T; ++k) {
    const int qk = (int)(lay.n[k] / nm);
    for (int l = k; l < lay.T; ++l) {
      const int ql = (int)(lay.n[l] / nm);
      const int64_t off = lay.off[k * FGP_MT_MAX_TASKS + l];
      for (int q = 0; q < qk; ++q) {
        const int r = lay.rs[k] + q, c = lay.rs[l] + (q % ql);
        double2 w = make_double2(0.0, 0.0);
        for (int64_t b = g; b < B; b += G) {
          const double2 p = cmulc(z[b * zs + (int64_t)r * nm + j], z[b * zs + (int64_t)c * nm + j]);
          w.x = __builtin_fma(gn[b], p.x, w.x);
          w.y = __builtin_fma(gn[b], p.y, w.y);
        }
        const double2 a = Z[off + (int64_t)q * nm];
        double2 gv;
        if (r == c) gv = make_double2(__builtin_fma(glg, a.x, -w.x), 0.0);
        else gv = make_double2(2.0 * __builtin_fma(glg, a.x, -w.x), 2.0 * __builtin_fma(glg, a.y, -w.y));
        out[off + (int64_t)q * nm] = gv;
      }
    }
  }
}

static int make_layout(const fgp_mt_layout* in, MtLay* lay) {
  if (!in) return set_error(kErrInvalid, "multitask: null layout");
  if (in->T < 1 || in->T > FGP_MT_MAX_TASKS) return set_error(kErrUnsupported, "multitask: %d active tasks outside [1, %d]", in->T, FGP_MT_MAX_TASKS);
  *lay = MtLay{};
  lay->T = in->T;
  int64_t nmin = in->n[in->T - 1];
  if (nmin < 1) return set_error(kErrInvalid, "multitask: empty task in the active layout");
  int64_t rows = 0, L = 0;
  for (int k = 0; k < in->T; ++k) {
    const int64_t nk = in->n[k];
    if (nk < 1 || (nk & (nk - 1)) || nk % nmin) return set_error(kErrInvalid, "multitask: n[%d] = %lld", k, (long long)nk);
    if (k > 0 && nk > in->n[k - 1]) return set_error(kErrInvalid, "multitask: tasks not sorted by n descending");
    lay->n[k] = nk;
    lay->rs[k] = (int)rows;
    rows += nk / nmin;
    for (int l = k; l < in->T; ++l) {
      lay->off[k * FGP_MT_MAX_TASKS + l] = L;
      L += nk;
    }
  }
  if (rows > FGP_MT_MAX_ROWS) return set_error(kErrUnsupported, "multitask: %lld block rows > %d (n spread too wide)", (long long)rows, FGP_MT_MAX_ROWS);
  lay->R = (int)rows;
  lay->nmin = nmin;
  lay->L = L;
  return kOk;
}

}  // namespace fgp

using namespace fgp;

extern "C" {

int fgp_mt_parts(int family, const void* x, int64_t x_row_stride, int64_t N, const void* z, int64_t z_row_stride,
                 int64_t M, int zip, int d, int P, const int* order, const double* coef, const double* add, int tbits,
                 double* parts, void* stream) {
  if (family != 0 && family != 1) return set_error(kErrInvalid, "fgp_mt_parts: family %d", family);
  if (N < 0 || M < 0 || d < 1 || d > FGP_MAX_D || P < 1) return set_error(kErrInvalid, "fgp_mt_parts: bad N/M/d/P");
  if (family == 1 && (tbits < 1 || tbits > 63)) return set_error(kErrInvalid, "fgp_mt_parts: t = %d", tbits);
  if (zip && N != M) return set_error(kErrInvalid, "fgp_mt_parts: zip needs N == M");
  if (N == 0 || M == 0) return kOk;
  if (!x || !z || !order || !coef || !parts || (family == 1 && !add)) return set_error(kErrInvalid, "fgp_mt_parts: null pointer");
  const int64_t cnt = zip ? N : N * M;
  k_mt_parts<<<(unsigned)((cnt + kWG - 1) / kWG), kWG, 0, (hipStream_t)stream>>>(family, x, x_row_stride, N, z,
                                                                                   z_row_stride, M, zip, d, P, order,
                                                                                   coef, add, tbits, parts);
  return check_launch("k_mt_parts");
}

int fgp_mt_factor(const fgp_mt_layout* layout, const void* lams, int64_t G, void* factor, double* logdet, int* info,
                  void* stream) {
  MtLay lay;
  int rc = make_layout(layout, &lay);
  if (rc != kOk) return rc;
  if (G < 1) return set_error(kErrInvalid, "fgp_mt_factor: G = %lld", (long long)G);
  if (!lams || !factor || !logdet || !info) return set_error(kErrInvalid, "fgp_mt_factor: null pointer");
  const int64_t cnt = G * lay.nmin;
  k_mt_ldl<<<(unsigned)((cnt + kWG - 1) / kWG), kWG, 0, (hipStream_t)stream>>>(
      static_cast<const double2*>(lams), G, lay, static_cast<double2*>(factor), logdet, info);
  return check_launch("k_mt_ldl");
}

int fgp_mt_solve(const fgp_mt_layout* layout, const void* factor, int64_t G, const void* v, int64_t v_row_stride,
                 int64_t B, void* out, void* stream) {
  MtLay lay;
  int rc = make_layout(layout, &lay);
  if (rc != kOk) return rc;
  if (G < 1 || B < 0) return set_error(kErrInvalid, "fgp_mt_solve: G = %lld, B = %lld", (long long)G, (long long)B);
  if (B == 0) return kOk;
  if (!factor || !v || !out) return set_error(kErrInvalid, "fgp_mt_solve: null pointer");
  if (v_row_stride < (int64_t)lay.R * lay.nmin) return set_error(kErrInvalid, "fgp_mt_solve: row stride < R * nmin");
  const int64_t cnt = B * lay.nmin;
  k_mt_solve<<<(unsigned)((cnt + kWG - 1) / kWG), kWG, 0, (hipStream_t)stream>>>(
      static_cast<const double2*>(factor), G, lay, static_cast<const double2*>(v), v_row_stride, B,
      static_cast<double2*>(out));
  return check_launch("k_mt_solve");
}

int fgp_mt_selinv(const fgp_mt_layout* layout, const void* factor, int64_t G, void* zinv, void* stream) {
  MtLay lay;
  int rc = make_layout(layout, &lay);
  if (rc != kOk) return rc;
  if (G < 1) return set_error(kErrInvalid, "fgp_mt_selinv: G = %lld", (long long)G);
  if (!factor || !zinv) return set_error(kErrInvalid, "fgp_mt_selinv: null pointer");
  const int64_t cnt = G * lay.nmin;
  k_mt_selinv<<<(unsigned)((cnt + kWG - 1) / kWG), kWG, 0, (hipStream_t)stream>>>(
      static_cast<const double2*>(factor), G, lay, static_cast<double2*>(zinv));
  return check_launch("k_mt_selinv");
}

int fgp_mt_mll_grad(const fgp_mt_layout* layout, const void* zinv, const void* z, const double* grad_norm,
                    const double* grad_logdet, int64_t B, int64_t G, void* grad_lams, void* stream) {
  MtLay lay;
  int rc = make_layout(layout, &lay);
  if (rc != kOk) return rc;
  if (G < 1 || B < G || B % G) return set_error(kErrInvalid, "fgp_mt_mll_grad: B = %lld, G = %lld", (long long)B, (long long)G);
  if (!zinv || !z || !grad_norm || !grad_logdet || !grad_lams) return set_error(kErrInvalid, "fgp_mt_mll_grad: null pointer");
  const int64_t cnt = G * lay.nmin;
  k_mt_mll_grad<<<(unsigned)((cnt + kWG - 1) / kWG), kWG, 0, (hipStream_t)stream>>>(
      static_cast<const double2*>(zinv), static_cast<const double2*>(z), grad_norm, grad_logdet, B, G, lay,
      static_cast<double2*>(grad_lams));
  return check_launch("k_mt_mll_grad");
}

}  // extern "C"
