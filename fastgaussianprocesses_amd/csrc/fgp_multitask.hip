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

#include <algorithm>
#include <type_traits>
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
// the factor of class j of problem g (src / F: that problem's packed arrays offset by j); returns the
// class's logdet, *bad set on a non-positive pivot
__device__ __forceinline__ double mt_ldl_class(const double2* __restrict__ src, double2* __restrict__ F, const MtLay& lay,
                                               bool* bad_out) {
  const int64_t nm = lay.nmin;
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
  *bad_out = bad;
  return ld;                 // a non-positive pivot still counts as log|pivot| (the reference's log|S|); info flags it
}

__global__ __launch_bounds__(kWG) void k_mt_ldl(const double2* __restrict__ lp, int64_t G, MtLay lay,
                                                double2* __restrict__ fac, double* __restrict__ logdet,
                                                int* __restrict__ info) {
  const int64_t e = (int64_t)blockIdx.x * kWG + threadIdx.x;
  if (e >= G * lay.nmin) return;
  const int64_t g = e / lay.nmin, j = e - g * lay.nmin;
  bool bad = false;
  logdet[e] = mt_ldl_class(lp + g * lay.L + j, fac + g * lay.L + j, lay, &bad);
  if (bad) info[0] = 1;
}

// out[b] = Lambda_{g(b)}^-1 v[b] (g(b) = b mod G), per frequency class: forward substitution with L,
// scaling by D^-1, back substitution with L^H -- O(R T) per vector and class.  v, out: [B][R nmin]
// (rows of the sorted tasks concatenated, the reference's [..., R, n_min] view, util.py:356-360).
// one vector of class j: F the factor, vb the right-hand side, o the solution (all offset by j)
__device__ __forceinline__ void mt_solve_class(const double2* __restrict__ F, const MtLay& lay, const double2* __restrict__ vb,
                                               double2* __restrict__ o) {
  const int64_t nm = lay.nmin;
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

__global__ __launch_bounds__(kWG) void k_mt_solve(const double2* __restrict__ fac, int64_t G, MtLay lay,
                                                  const double2* __restrict__ v, int64_t vs, int64_t B,
                                                  double2* __restrict__ out) {
  const int64_t e = (int64_t)blockIdx.x * kWG + threadIdx.x;
  if (e >= B * lay.nmin) return;
  const int64_t nm = lay.nmin;
  const int64_t b = e / nm, j = e - b * nm, g = b % G;
  mt_solve_class(fac + g * lay.L + j, lay, v + b * vs + j, out + b * (int64_t)lay.R * nm + j);
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

__device__ __forceinline__ void mt_selinv_class(const double2* __restrict__ F, const MtLay& lay, double2* __restrict__ Z) {
  const int64_t nm = lay.nmin;
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

__global__ __launch_bounds__(kWG) void k_mt_selinv(const double2* __restrict__ fac, int64_t G, MtLay lay,
                                                   double2* __restrict__ zinv) {
  const int64_t e = (int64_t)blockIdx.x * kWG + threadIdx.x;
  if (e >= G * lay.nmin) return;
  const int64_t g = e / lay.nmin, j = e - g * lay.nmin;
  mt_selinv_class(fac + g * lay.L + j, lay, zinv + g * lay.L + j);
}

// Gradient of the MLL data + logdet terms w.r.t. the packed lams (torch's convention for complex
// inputs: dL/dRe + i dL/dIm), with z_b = A y_b, gn[b] = dL/dnorm_b, gl[g] = dL/dlogdet_g and Z the
// selected inverse:
//   coupling entry (r < c):  -2 sum_b gn[b] z_br conj(z_bc) + 2 gl[g] Z_rc
//   diagonal entry:          -sum_b gn[b] |z_br|^2 + gl[g] Z_rr      (real; the imaginary part of a
//                            Hermitian diagonal does not enter)
// class j of problem g: Z, out offset by g L + j; z the solutions [B][R nmin] (not offset); gn(b) per vector
template <typename GN>
__device__ __forceinline__ void mt_grad_class(const double2* __restrict__ Z, const double2* __restrict__ z, GN gn, double glg,
                                              int64_t B, int64_t G, int64_t g, int64_t j, const MtLay& lay,
                                              double2* __restrict__ out) {
  const int64_t nm = lay.nmin, zs = (int64_t)lay.R * nm;
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
          const double gb = gn(b);
          w.x = __builtin_fma(gb, p.x, w.x);
          w.y = __builtin_fma(gb, p.y, w.y);
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

__global__ __launch_bounds__(kWG) void k_mt_mll_grad(const double2* __restrict__ zinv, const double2* __restrict__ z,
                                                     const double* __restrict__ gn, const double* __restrict__ gl,
                                                     int64_t B, int64_t G, MtLay lay, double2* __restrict__ glp) {
  const int64_t e = (int64_t)blockIdx.x * kWG + threadIdx.x;
  if (e >= G * lay.nmin) return;
  const int64_t g = e / lay.nmin, j = e - g * lay.nmin;
  mt_grad_class(zinv + g * lay.L + j, z, [&](int64_t b) { return gn[b]; }, gl[g], B, G, g, j, lay, glp + g * lay.L + j);
}

// ------------------------------------------------------------------------------------------------
// Device-resident fit of a general multitask GP (ABI 14, fgp_mt_fit_run).  One iteration = five launches, each
// over the G problems of a parameter batch (ABI 16) as its y index:
//   k_mtg_lams          packed lams from the pair spectra and the current parameters (thread per entry)
//   k_mtg_factor_grad   per frequency class: structured LDL^H, solves of the B data vectors, selected inverse,
//   / k_mtg_class       dL/dlams (thread per class: mt_ldl_class / mt_solve_class / mt_selinv_class /
//                       mt_grad_class, the generic path's kernels' bodies; or a wave per class when they are few)
//   k_mtg_contract      dL/dlams contracted with dlams/dtheta (thread per entry): block partials of the norm,
//                       logdet, dL/dnoise, dL/draw_scale, dL/draw_l_m; the per-entry dL/dK_task terms
//   k_mtg_reduce        the fixed-order totals of those, a wave per (total, problem)
//   k_mtg_step          one workgroup: loss history, dL/d(task factor / noise) by the chain rule through
//                       K_task = F F^T + diag(v), the problems' gradients summed into their parameter rows,
//                       torch.optim.Rprop on every element
struct MtFit {
  MtLay lay;
  int family, d, B, T_all, rank, dl, vtask_exp, P;
  int G;                          // problems (parameter batch, ABI 16); rows: their parameter rows ([5][G], or NULL)
  const int* rows;
  int l_off, n_off;               // raw offsets of the lengthscale / noise blocks (scale rows at 0)
  int task[FGP_MT_MAX_TASKS];
  int rg_scale, rg_ls, rg_noise, rg_factor, rg_vtask;
  const double2* spec;
  int64_t spec_off[FGP_MT_MAX_TASKS * (FGP_MT_MAX_TASKS + 1) / 2];
  const double2* y;
  double* raw;
  double *prev, *step, *grad, *loss_hist, *raw_hist;
  double gn, gl, logdet_weight, mll_const, eta_minus, eta_plus, step_min, step_max;
  int n_params, f_off, v_off;
  // workspace
  double2 *lams, *fac, *zinv, *glp, *z;
  double *logdet, *dkt, *part, *sums;
  int* info;
  const double2* nug_coef;        // adaptive nugget (ABI 16): [T][2^d] sqrt(n_k) sum_i Phi^{kk}_S[i], or NULL
  int nug_ref;
  int nblk;
};

constexpr int kMtgQ = 4 + FGP_MAX_D;   // norm, logdet, dnoise (/ noise), draw_scale, draw_l[FGP_MAX_D]

// problem g's row of parameter block q (0 scale, 1 lengthscales, 2 noise, 3 task factor, 4 task noise)
__device__ __forceinline__ int mtg_row(const MtFit& m, int q, int g) { return m.rows ? m.rows[q * m.G + g] : 0; }
// raw indices of problem g's parameters
__device__ __forceinline__ int mtg_is(const MtFit& m, int g) { return mtg_row(m, 0, g); }
__device__ __forceinline__ int mtg_il(const MtFit& m, int g, int j) {
  return m.l_off + mtg_row(m, 1, g) * m.dl + (m.dl > 1 ? j : 0);
}
__device__ __forceinline__ int mtg_in(const MtFit& m, int g) { return m.n_off + mtg_row(m, 2, g); }
__device__ __forceinline__ int mtg_if(const MtFit& m, int g) { return m.f_off + mtg_row(m, 3, g) * m.T_all * m.rank; }
__device__ __forceinline__ int mtg_iv(const MtFit& m, int g) { return m.v_off + mtg_row(m, 4, g) * m.T_all; }
__device__ __forceinline__ double mtg_scale(const MtFit& m, int g) { return exp(m.raw[mtg_is(m, g)]); }
__device__ __forceinline__ double mtg_ls(const MtFit& m, int g, int j) { return exp(m.raw[mtg_il(m, g, j)]); }
__device__ __forceinline__ double mtg_noise(const MtFit& m, int g) { return exp(m.raw[mtg_in(m, g)]); }
// K_task[a, b] = sum_r F[a, r] F[b, r] + [a == b] v_a  (util.py:157-162; F identity, v exp / identity)
__device__ __forceinline__ double mtg_kt(const MtFit& m, int g, int a, int b) {
  const int fo = mtg_if(m, g), vo = mtg_iv(m, g);
  double s = 0.0;
  for (int r = 0; r < m.rank; ++r) s += m.raw[fo + a * m.rank + r] * m.raw[fo + b * m.rank + r];
  if (a == b) s += m.vtask_exp ? exp(m.raw[vo + a]) : m.raw[vo + a];
  return s;
}

// entry e of the packed lams -> sorted pair (k, l), its index p and the position i in lams[k, l]
__device__ __forceinline__ void mtg_entry(const MtFit& m, int64_t e, int& k, int& l, int& p, int64_t& i) {
  const MtLay& lay = m.lay;
  k = 0;
  l = 0;
  p = 0;
  for (int kk = 0; kk < lay.T; ++kk)
    for (int ll = kk; ll < lay.T; ++ll) {
      const int64_t o = lay.off[kk * FGP_MT_MAX_TASKS + ll];
      if (e >= o && e < o + lay.n[kk]) {
        k = kk;
        l = ll;
      }
    }
  p = k * lay.T - k * (k - 1) / 2 + (l - k);
  i = e - lay.off[k * FGP_MT_MAX_TASKS + l];
}

// P = sum_S l^S Phi_S[i] of pair p (ascending S) and, with DER, dp[j] = sum_{S containing j} l^S Phi_S[i]
template <int D, bool DER>
__device__ __forceinline__ double2 mtg_poly(const MtFit& m, int p, int64_t nk, int64_t i, const double* lpow,
                                            double2* dp) {
  constexpr int NS = 1 << D;
  const double2* ph = m.spec + m.spec_off[p] + i;
  double2 P = make_double2(0.0, 0.0);
#pragma unroll
  for (int j = 0; j < (DER ? D : 0); ++j) dp[j] = make_double2(0.0, 0.0);
  // S = sh + t in groups of 8: the bits of t resolve at compile time, the higher bits (D > 3) are uniform per group
  // (a fully unrolled 2^6-term loop with its derivative sums spilled hundreds of VGPRs; a plain partial unroll
  // tested every bit per term).  Every sum in ascending S, as before.
  constexpr int U = NS < 8 ? NS : 8;
#pragma unroll 1
  for (int sh = 0; sh < NS; sh += U) {
#pragma unroll
    for (int t = 0; t < U; ++t) {
      const int S = sh + t;
      const double2 f = ph[(int64_t)S * nk];
      const double w = lpow[S];
      P.x = __builtin_fma(w, f.x, P.x);
      P.y = __builtin_fma(w, f.y, P.y);
      if constexpr (DER) {
#pragma unroll
        for (int j = 0; j < D; ++j)
          if (j < 3 ? ((t >> j) & 1) : ((sh >> j) & 1)) {
            dp[j].x = __builtin_fma(w, f.x, dp[j].x);
            dp[j].y = __builtin_fma(w, f.y, dp[j].y);
          }
      }
    }
  }
  return P;
}

template <int D>
__device__ __forceinline__ void mtg_lpow(const MtFit& m, int g, double* lpow) {
  double ls[D];
#pragma unroll
  for (int j = 0; j < D; ++j) ls[j] = mtg_ls(m, g, j);
#pragma unroll
  for (int S = 0; S < (1 << D); ++S) {
    double w = 1.0;
#pragma unroll
    for (int j = 0; j < D; ++j)
      if ((S >> j) & 1) w *= ls[j];
    lpow[S] = w;
  }
}

// The same products for the launch's problem g in LDS (lp: __shared__ [2^D]), the threads < 2^D forming one each
// (mtg_lpow's order) -- every thread of the workgroup then reads them instead of holding 2^D registers
template <int D>
__device__ __forceinline__ void mtg_lpow_lds(const MtFit& m, int g, double* lp) {
  if ((int)threadIdx.x < (1 << D)) {
    const int S = threadIdx.x;
    double w = 1.0;
    for (int j = 0; j < D; ++j)
      if ((S >> j) & 1) w *= mtg_ls(m, g, j);
    lp[S] = w;
  }
  __syncthreads();
}

// The adaptive nugget's ratio of sorted task k (util.py:286-290): r = |A_k| / |A_ref| with A_k = sqrt(n_k) sum_S l^S c_kS
// (the trace of the block's sqrt(n_k) lam over scale), and with DER dr[j] = l_j dr/dl_j (log-lengthscale derivative:
// l_j dA/dl_j = sum_{S containing j} l^S c_S).
template <int D, bool DER>
__device__ __forceinline__ double mtg_nug_ratio(const MtFit& m, int k, const double* lpow, double* dr) {
  constexpr int NS = 1 << D;
  double2 A[2] = {make_double2(0.0, 0.0), make_double2(0.0, 0.0)};
  double2 Aj[2][DER ? D : 1];
  const int kk[2] = {k, m.nug_ref};
#pragma unroll
  for (int u = 0; u < 2; ++u) {
#pragma unroll
    for (int j = 0; j < (DER ? D : 1); ++j) Aj[u][j] = make_double2(0.0, 0.0);
    const double2* c = m.nug_coef + (int64_t)kk[u] * NS;
#pragma unroll 4
    for (int S = 0; S < NS; ++S) {
      const double2 cs = c[S];
      A[u].x = __builtin_fma(lpow[S], cs.x, A[u].x);
      A[u].y = __builtin_fma(lpow[S], cs.y, A[u].y);
      if constexpr (DER) {
#pragma unroll
        for (int j = 0; j < D; ++j)
          if ((S >> j) & 1) {
            Aj[u][j].x = __builtin_fma(lpow[S], cs.x, Aj[u][j].x);
            Aj[u][j].y = __builtin_fma(lpow[S], cs.y, Aj[u][j].y);
          }
      }
    }
  }
  const double a2 = __builtin_fma(A[0].x, A[0].x, A[0].y * A[0].y), b2 = __builtin_fma(A[1].x, A[1].x, A[1].y * A[1].y);
  const double r = sqrt(a2) / sqrt(b2);
  if constexpr (DER) {
#pragma unroll
    for (int j = 0; j < D; ++j) {
      const double ga = __builtin_fma(A[0].x, Aj[0][j].x, A[0].y * Aj[0][j].y) / a2;
      const double gb = __builtin_fma(A[1].x, Aj[1][j].x, A[1].y * Aj[1][j].y) / b2;
      dr[j] = r * (ga - gb);
    }
  }
  return r;
}

// (problem g = the launch's y index: entry / class / block-row g of a parameter batch; 0 when unbatched)
template <int D>
__global__ __launch_bounds__(kWG) void k_mtg_lams(MtFit m) {
  __shared__ double lpow[1 << D];
  const int64_t e = (int64_t)blockIdx.x * kWG + threadIdx.x;
  const int g = blockIdx.y;
  mtg_lpow_lds<D>(m, g, lpow);
  if (e >= m.lay.L) return;
  int k, l, p;
  int64_t i;
  mtg_entry(m, e, k, l, p, i);
  const double2 P = mtg_poly<D, false>(m, p, m.lay.n[k], i, lpow, nullptr);
  const double sc = mtg_scale(m, g), rn = sqrt((double)m.lay.n[l]);
  // lams = K_task (sqrt(n_l) lam + noise [k == l]),  lam = scale P  (util.py:284-298)
  double2 v = make_double2(rn * (sc * P.x), rn * (sc * P.y));
  if (k == l) v.x += m.nug_coef ? mtg_noise(m, g) * mtg_nug_ratio<D, false>(m, k, lpow, nullptr) : mtg_noise(m, g);
  const double kt = mtg_kt(m, g, m.task[k], m.task[l]);
  m.lams[(int64_t)g * m.lay.L + e] = make_double2(v.x * kt, v.y * kt);
}

__global__ __launch_bounds__(kWG) void k_mtg_factor_grad(MtFit m) {
  const int64_t j = (int64_t)blockIdx.x * kWG + threadIdx.x;
  const int g = blockIdx.y;
  const MtLay& lay = m.lay;
  if (j >= lay.nmin) return;
  const int64_t go = (int64_t)g * lay.L, rn = (int64_t)lay.R * lay.nmin, gy = (int64_t)g * m.B * rn;
  bool bad = false;
  m.logdet[(int64_t)g * lay.nmin + j] = mt_ldl_class(m.lams + go + j, m.fac + go + j, lay, &bad);
  if (bad) m.info[0] = 1;
  for (int b = 0; b < m.B; ++b) mt_solve_class(m.fac + go + j, lay, m.y + gy + b * rn + j, m.z + gy + b * rn + j);
  mt_selinv_class(m.fac + go + j, lay, m.zinv + go + j);
  const double gn = m.gn;
  mt_grad_class(m.zinv + go + j, m.z + gy, [&](int64_t) { return gn; }, m.gl, m.B, 1, 0, j, lay, m.glp + go + j);
}

// The same per class with ONE WAVE per (class j, problem g) -- for few classes (G nmin small: the thread per
// class above is then a single dependent chain of global read-modify-writes, ~0.1 us each).  The class's packed
// entries (E = L / nmin), its selected inverse and its B vectors live in LDS; the rows of a task form a diagonal
// block, so every step of the elimination / substitutions / Takahashi recurrence runs over a task's rows (or the
// entries they update) in parallel.  A value is produced by the same operation sequence as in mt_*_class (the
// updates of one target in ascending q, the logdet summed in row order), so both kernels agree bit for bit.
constexpr int kMtcWG = 64;
constexpr int kMtcMaxLds = 60 * 1024;
constexpr int64_t kMtcMaxClasses = 8192;         // G nmin above this: the thread per class has the parallelism

__device__ __forceinline__ double2 mtc_zpat(const double2* Z, const int* oe, int l, int pl, int m, int pm) {
  return l <= m ? Z[oe[l * FGP_MT_MAX_TASKS + m] + pl] : conj2(Z[oe[m * FGP_MT_MAX_TASKS + l] + pm]);
}

__global__ __launch_bounds__(kMtcWG) void k_mtg_class(MtFit m) {
  extern __shared__ double2 sm[];
  __shared__ int oe[FGP_MT_MAX_TASKS * FGP_MT_MAX_TASKS];     // packed offset / nmin of block (k, l)
  __shared__ int qn[FGP_MT_MAX_TASKS], rs[FGP_MT_MAX_TASKS];
  __shared__ int bad;
  const MtLay& lay = m.lay;
  const int t = threadIdx.x, T = lay.T, R = lay.R, B = m.B;
  const int64_t nm = lay.nmin, j = blockIdx.x, g = blockIdx.y;
  const int E = (int)(lay.L / nm);
  double2* F = sm;
  double2* Z = sm + E;
  double2* o = sm + 2 * E;
  double* lg = reinterpret_cast<double*>(o + B * R);       // log |pivot| of every row
  double* ip = lg + R;                                      // 1 / pivot of every row
  constexpr int MT = FGP_MT_MAX_TASKS;
  for (int u = t; u < T * T; u += kMtcWG) {
    const int k = u / T, l = u - k * T;
    oe[k * MT + l] = k <= l ? (int)(lay.off[k * MT + l] / nm) : 0;
  }
  for (int k = t; k < T; k += kMtcWG) {
    qn[k] = (int)(lay.n[k] / nm);
    rs[k] = lay.rs[k];
  }
  if (t == 0) bad = 0;
  const int64_t go = g * lay.L, rn = (int64_t)R * nm, gy = g * B * rn;
  for (int e = t; e < E; e += kMtcWG) F[e] = m.lams[go + e * nm + j];
  for (int u = t; u < B * R; u += kMtcWG) {
    const int b = u / R, r = u - b * R;
    o[u] = m.y[gy + b * rn + (int64_t)r * nm + j];
  }
  __syncthreads();
#if defined(FGP_MTC_EXP_STOP) && FGP_MTC_EXP_STOP == 1
  return;     // timing experiment (tools/build_exp.sh): the load only
#endif
  // LDL^H (mt_ldl_class): pivots of task k, the updates of the later tasks' blocks, the couplings scaled
  for (int k = 0; k < T; ++k) {
    const int qk = qn[k], dk = oe[k * MT + k];
    for (int q = t; q < qk; q += kMtcWG) {
      const double dq = F[dk + q].x;
      if (!(dq > 0.0)) bad = 1;
      lg[rs[k] + q] = log(fabs(dq));
      ip[rs[k] + q] = 1.0 / dq;
      F[dk + q] = make_double2(dq, 0.0);
    }
    __syncthreads();
    int tot = 0;
    for (int l = k + 1; l < T; ++l) tot += (T - l) * qn[l];
    for (int u = t; u < tot; u += kMtcWG) {
      int l = k + 1, mm = l, rem = u;                  // target (l, mm, p)
      for (;; ) {
        if (rem < qn[l]) break;
        rem -= qn[l];
        if (++mm == T) mm = ++l;
      }
      const int ql = qn[l], p = rem;
      double2 acc = F[oe[l * MT + mm] + p];
#pragma unroll 4
      for (int q = p; q < qk; q += ql) {
        const double2 ul = F[oe[k * MT + l] + q] * ip[rs[k] + q];
        acc -= cmul_cj(ul, F[oe[k * MT + mm] + q]);
      }
      F[oe[l * MT + mm] + p] = acc;
    }
    __syncthreads();
    for (int u = t; u < (T - 1 - k) * qk; u += kMtcWG) {
      const int l = k + 1 + u / qk, q = u % qk;
      double2* c = F + oe[k * MT + l] + q;
      *c = *c * ip[rs[k] + q];
    }
    __syncthreads();
  }
  if (t == 0) {
    double ld = 0.0;
    for (int r = 0; r < R; ++r) ld += lg[r];
    m.logdet[g * nm + j] = ld;
    if (bad) m.info[0] = 1;
  }
#if defined(FGP_MTC_EXP_STOP) && FGP_MTC_EXP_STOP == 2
  return;
#endif
  // solves (mt_solve_class): w = L^-1 v by task, w /= D, z = L^-H w by task (backwards)
  for (int k = 0; k < T; ++k) {
    const int qk = qn[k];
    int S = 0;
    for (int l = k + 1; l < T; ++l) S += qn[l];
    for (int u = t; u < B * S; u += kMtcWG) {
      const int b = u / S;
      int l = k + 1, p = u - b * S;
      while (p >= qn[l]) p -= qn[l++];
      const int ql = qn[l];
      double2 acc = o[b * R + rs[l] + p];
#pragma unroll 4
      for (int q = p; q < qk; q += ql) acc -= cmul_cj(F[oe[k * MT + l] + q], o[b * R + rs[k] + q]);
      o[b * R + rs[l] + p] = acc;
    }
    __syncthreads();
  }
  for (int u = t; u < B * R; u += kMtcWG) o[u] = o[u] * ip[u % R];
  __syncthreads();
  for (int k = T - 1; k >= 0; --k) {
    const int qk = qn[k];
    for (int u = t; u < B * qk; u += kMtcWG) {
      const int b = u / qk, q = u - b * qk;
      double2 s = o[b * R + rs[k] + q];
#pragma unroll 4
      for (int l = k + 1; l < T; ++l) s -= cmul(F[oe[k * MT + l] + q], o[b * R + rs[l] + q % qn[l]]);
      o[b * R + rs[k] + q] = s;
    }
    __syncthreads();
  }
#if defined(FGP_MTC_EXP_STOP) && FGP_MTC_EXP_STOP == 3
  return;
#endif
  // selected inverse (mt_selinv_class), task by task from the last: a row's couplings, then its diagonal
  for (int k = T - 1; k >= 0; --k) {
    const int qk = qn[k];
    for (int q = t; q < qk; q += kMtcWG) {
      for (int mm = k + 1; mm < T; ++mm) {
        const int pm = q % qn[mm];
        double2 s = make_double2(0.0, 0.0);
#pragma unroll 4
        for (int l = k + 1; l < T; ++l) s -= cmul(F[oe[k * MT + l] + q], mtc_zpat(Z, oe, l, q % qn[l], mm, pm));
        Z[oe[k * MT + mm] + q] = s;
      }
      double s = ip[rs[k] + q];
      for (int l = k + 1; l < T; ++l) {
        const double2 u = F[oe[k * MT + l] + q], zc = Z[oe[k * MT + l] + q];
        s -= __builtin_fma(u.x, zc.x, u.y * zc.y);
      }
      Z[oe[k * MT + k] + q] = make_double2(s, 0.0);
    }
    __syncthreads();
  }
#if defined(FGP_MTC_EXP_STOP) && FGP_MTC_EXP_STOP == 4
  return;
#endif
  // dL/dlams (mt_grad_class) and the solutions out
  for (int k = 0; k < T; ++k)
    for (int l = k; l < T; ++l)
      for (int q = t; q < qn[k]; q += kMtcWG) {
        const int e = oe[k * MT + l] + q, r = rs[k] + q, c = rs[l] + q % qn[l];
        double2 w = make_double2(0.0, 0.0);
        for (int b = 0; b < B; ++b) {
          const double2 p = cmulc(o[b * R + r], o[b * R + c]);
          w.x = __builtin_fma(m.gn, p.x, w.x);
          w.y = __builtin_fma(m.gn, p.y, w.y);
        }
        const double2 a = Z[e];
        m.glp[go + e * nm + j] = r == c ? make_double2(__builtin_fma(m.gl, a.x, -w.x), 0.0)
                                        : make_double2(2.0 * __builtin_fma(m.gl, a.x, -w.x),
                                                       2.0 * __builtin_fma(m.gl, a.y, -w.y));
      }
  for (int u = t; u < B * R; u += kMtcWG) {
    const int b = u / R, r = u - b * R;
    m.z[gy + b * rn + (int64_t)r * nm + j] = o[u];
  }
}

static int g_mt_class_mode = 0;            // fgp_set_mt_class_kernel

// LDS bytes of k_mtg_class for this layout (0: does not fit)
static size_t mtc_lds(const MtLay& lay, int B) {
  const size_t E = (size_t)(lay.L / lay.nmin);
  const size_t b = (2 * E + (size_t)B * lay.R) * 16 + (size_t)lay.R * 16;
  return b <= (size_t)kMtcMaxLds ? b : 0;
}

template <int D>
__global__ __launch_bounds__(kWG) void k_mtg_contract(MtFit m) {
  __shared__ double red[kWG / 64];
  const int64_t t0 = (int64_t)blockIdx.x * kWG + threadIdx.x, nt = (int64_t)gridDim.x * kWG;
  const int g = blockIdx.y;
  const MtLay& lay = m.lay;
  const int64_t go = (int64_t)g * lay.L, rnm = (int64_t)lay.R * lay.nmin;
  __shared__ double lpow[1 << D];
  mtg_lpow_lds<D>(m, g, lpow);
  const double sc = mtg_scale(m, g);
  double acc[4 + D];
#pragma unroll
  for (int q = 0; q < 4 + D; ++q) acc[q] = 0.0;
  for (int64_t e = t0; e < lay.L; e += nt) {
    int k, l, p;
    int64_t i;
    mtg_entry(m, e, k, l, p, i);
    double2 dp[D];
    const double2 P = mtg_poly<D, true>(m, p, lay.n[k], i, lpow, dp);
    const double rn = sqrt((double)lay.n[l]);
    const double kt = mtg_kt(m, g, m.task[k], m.task[l]);
    const double2 c = m.glp[go + e];       // dL/dRe + i dL/dIm of lams[e]: dL/dtheta = Re(conj(c) dlams/dtheta)
    const double f = kt * rn * sc;
    acc[3] = __builtin_fma(f, __builtin_fma(c.x, P.x, c.y * P.y), acc[3]);             // draw_scale
#pragma unroll
    for (int j = 0; j < D; ++j) acc[4 + j] = __builtin_fma(f, __builtin_fma(c.x, dp[j].x, c.y * dp[j].y), acc[4 + j]);
    double bx = rn * (sc * P.x), by = rn * (sc * P.y);
    if (k == l) {
      if (m.nug_coef) {
        // adaptive nugget noise r_k: d/dnoise = r_k, d/draw_l_j = noise l_j dr_k/dl_j (on the diagonal entries)
        double dr[D];
        const double r = mtg_nug_ratio<D, true>(m, k, lpow, dr);
        const double nz = mtg_noise(m, g);
        bx += nz * r;
        acc[2] = __builtin_fma(kt * r, c.x, acc[2]);                                   // dnoise / noise
#pragma unroll
        for (int j = 0; j < D; ++j) acc[4 + j] = __builtin_fma(kt * c.x, nz * dr[j], acc[4 + j]);
      } else {
        bx += mtg_noise(m, g);
        acc[2] = __builtin_fma(kt, c.x, acc[2]);                                       // dnoise / noise
      }
    }
    m.dkt[go + e] = __builtin_fma(c.x, bx, c.y * by);                                  // dL/dK_task of entry e
  }
  const double2* yg = m.y + (int64_t)g * m.B * rnm;
  const double2* zg = m.z + (int64_t)g * m.B * rnm;
  for (int64_t e = t0; e < (int64_t)m.B * rnm; e += nt) {
    const double2 yv = yg[e], zv = zg[e];
    acc[0] = __builtin_fma(yv.x, zv.x, __builtin_fma(yv.y, zv.y, acc[0]));             // Re(conj(y) z)
  }
  for (int64_t j = t0; j < lay.nmin; j += nt) acc[1] += m.logdet[(int64_t)g * lay.nmin + j];
#pragma unroll
  for (int q = 0; q < 4 + D; ++q) {
    const double s = block_sum(acc[q], red);
    if (threadIdx.x == 0) m.part[((int64_t)g * m.nblk + blockIdx.x) * kMtgQ + q] = s;
  }
}

// the per-problem totals the step needs: sums[g][q] = the workgroup-order sum of block partial q (q < 4 + D) and of
// dL/dK_task over the entries of pair p (q = 4 + D + p).  One wave per total, reproducing block_sum's order
// (thread t's strided sum, the wave butterfly, the four waves added in order) so the totals are those of a
// 256-thread reduction, bit for bit
template <int D>
__global__ __launch_bounds__(kWG) void k_mtg_reduce(MtFit m) {
  const int ln = threadIdx.x & 63, q = (int)blockIdx.x * (kWG / 64) + (threadIdx.x >> 6), g = blockIdx.y;
  if (q >= 4 + D + m.P) return;
  const MtLay& lay = m.lay;
  const double* src;
  int64_t cnt, stride;
  if (q < 4 + D) {
    src = m.part + (int64_t)g * m.nblk * kMtgQ + q;
    cnt = m.nblk;
    stride = kMtgQ;
  } else {
    int k = 0, l = 0;
    for (int kk = 0, p = 0; kk < lay.T; ++kk)
      for (int ll = kk; ll < lay.T; ++ll, ++p)
        if (p == q - 4 - D) {
          k = kk;
          l = ll;
        }
    src = m.dkt + (int64_t)g * lay.L + lay.off[k * FGP_MT_MAX_TASKS + l];
    cnt = lay.n[k];
    stride = 1;
  }
  double tot = 0.0;
#pragma unroll
  for (int w = 0; w < kWG / 64; ++w) {
    double s = 0.0;
    for (int64_t t = w * 64 + ln; t < cnt; t += kWG) s += src[t * stride];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    tot += s;
  }
  if (ln == 0) m.sums[(int64_t)g * (kMtgQ + m.P) + q] = tot;
}

// one element per thread (the elements' sums are chains of LDS reads: latency, hidden by 16 waves)
constexpr int kMtgStepWG = 1024;

template <int D, bool STAGE>
__global__ __launch_bounds__(kMtgStepWG) void k_mtg_step(MtFit m, int iter, int do_update) {
  __shared__ double term[2];
  // LDS: the gradient [n_params]; with STAGE, copies of the raw parameters [n_params], the problems' totals
  // [G][NQs] and their rows [5][G] (the element loops below then run on LDS latency, not a chain of global loads)
  extern __shared__ double grad[];
  const int tid = threadIdx.x, G = m.G, NQs = kMtgQ + m.P;
  const MtLay& lay = m.lay;
  double* sraw = grad + m.n_params;
  double* ssum = sraw + m.n_params;
  int* srows = reinterpret_cast<int*>(ssum + (int64_t)G * NQs);
  if constexpr (STAGE) {
    for (int u = tid; u < m.n_params; u += kMtgStepWG) sraw[u] = m.raw[u];
    for (int u = tid; u < G * NQs; u += kMtgStepWG) ssum[u] = m.sums[u];
    if (m.rows)
      for (int u = tid; u < 5 * G; u += kMtgStepWG) srows[u] = m.rows[u];
    __syncthreads();
  }
  const double* raw = STAGE ? sraw : m.raw;
  const double* sums = STAGE ? ssum : m.sums;
  const int* rw = m.rows ? (STAGE ? srows : m.rows) : nullptr;
  if (tid == 0) {
    double t0 = 0.0, t1 = 0.0;
    for (int g = 0; g < G; ++g) {
      t0 += sums[(int64_t)g * NQs];
      t1 += sums[(int64_t)g * NQs + 1];
    }
    term[0] = t0;
    term[1] = t1;
  }
  auto row = [&](int q, int g) { return rw ? rw[q * G + g] : 0; };
  // element by element: the problems' contributions to the element's parameter row in ascending problem order
  // (pairs ascending within a problem, the (a, .) term of a pair before its (b, .) term) -- the order of a
  // single-threaded pass over the problems
#ifdef FGP_MTG_EXP_NOELEM
  for (int x = tid; x < m.n_params; x += kMtgStepWG) grad[x] = 0.0;   // timing experiment: no element sums
  if (false)
#endif
  for (int x = tid; x < m.n_params; x += kMtgStepWG) {
    double gs = 0.0;
    if (x < m.l_off) {
      for (int g = 0; g < G; ++g)
        if (row(0, g) == x) gs += sums[(int64_t)g * NQs + 3];
    } else if (x < m.n_off) {
      const int rr = (x - m.l_off) / m.dl, j = (x - m.l_off) - rr * m.dl;
      for (int g = 0; g < G; ++g) {
        if (row(1, g) != rr) continue;
        const double* tot = sums + (int64_t)g * NQs;
        if (m.dl > 1) {
          gs += tot[4 + j];
        } else {
          double s = 0.0;
          for (int jj = 0; jj < m.d; ++jj) s += tot[4 + jj];
          gs += s;
        }
      }
    } else if (x < m.f_off) {
      const double nz = exp(raw[x]);
      for (int g = 0; g < G; ++g)
        if (row(2, g) == x - m.n_off) gs += nz * sums[(int64_t)g * NQs + 2];
    } else if (x < m.v_off) {
      // K_task[a, b] = sum_r F[a, r] F[b, r] + [a == b] v_a:  dF[c, r] += g_ab (F[b, r] [a == c] + F[a, r] [b == c])
      const int TR = m.T_all * m.rank, rr = (x - m.f_off) / TR, u = (x - m.f_off) - rr * TR;
      const int c = u / m.rank, r = u - c * m.rank, fo = m.f_off + rr * TR;
      for (int g = 0; g < G; ++g) {
        if (row(3, g) != rr) continue;
        const double* gkt = sums + (int64_t)g * NQs + 4 + D;
        for (int k = 0, p = 0; k < lay.T; ++k) {
          const int a = m.task[k];
#pragma unroll 4
          for (int l = k; l < lay.T; ++l) {
            const int b = m.task[l];
            const double gv = gkt[p + l - k];
            if (a == c) gs += gv * raw[fo + b * m.rank + r];
            if (b == c) gs += gv * raw[fo + a * m.rank + r];
          }
          p += lay.T - k;
        }
      }
    } else {
      const int rr = (x - m.v_off) / m.T_all, c = (x - m.v_off) - rr * m.T_all;
      const double ev = m.vtask_exp ? exp(raw[x]) : 1.0;
      for (int g = 0; g < G; ++g) {
        if (row(4, g) != rr) continue;
        const double* gkt = sums + (int64_t)g * NQs + 4 + D;
        for (int k = 0; k < lay.T; ++k)
          if (m.task[k] == c) {
            const double gv = gkt[k * lay.T - k * (k - 1) / 2];      // the diagonal pair (k, k)
            gs += m.vtask_exp ? gv * ev : gv;
          }
      }
    }
    grad[x] = gs;
  }
  __syncthreads();
  if (tid == 0) {
    const double term2 = m.logdet_weight * term[1];
    double* lh = m.loss_hist + (int64_t)iter * 3;
    lh[0] = 0.5 * (term[0] + term2 + m.mll_const);
    lh[1] = term[0];
    lh[2] = term2;
  }
  for (int q = tid; q < m.n_params; q += kMtgStepWG) {
    const double gp = grad[q];
    m.raw_hist[(int64_t)iter * m.n_params + q] = m.raw[q];
    m.grad[q] = gp;
    int rg;
    if (q < m.l_off) rg = m.rg_scale;
    else if (q < m.n_off) rg = m.rg_ls;
    else if (q < m.f_off) rg = m.rg_noise;
    else if (q < m.v_off) rg = m.rg_factor;
    else rg = m.rg_vtask;
    if (!(do_update && rg)) continue;
    const double prod = gp * m.prev[q];
    const double sgn = prod > 0.0 ? m.eta_plus : (prod < 0.0 ? m.eta_minus : 1.0);
    const double st = fmin(fmax(m.step[q] * sgn, m.step_min), m.step_max);
    m.step[q] = st;
    const double gg = (sgn == m.eta_minus) ? 0.0 : gp;
    const double gs = gg > 0.0 ? 1.0 : (gg < 0.0 ? -1.0 : 0.0);
    m.raw[q] = m.raw[q] + (-1.0) * (gs * st);
    m.prev[q] = gg;
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

static size_t mtg_align(size_t b) { return (b + 255) & ~(size_t)255; }

static int to_mtfit(const fgp_mt_fit_desc* d, MtFit* m, int64_t* work_bytes) {
  if (!d) return set_error(kErrInvalid, "fgp_mt_fit: null desc");
  *m = MtFit{};
  int rc = make_layout(&d->layout, &m->lay);
  if (rc != kOk) return rc;
  if (d->family != 0 && d->family != 1) return set_error(kErrInvalid, "fgp_mt_fit: family %d", d->family);
  if (d->d < 1 || d->d > 6) return set_error(kErrUnsupported, "fgp_mt_fit: d = %d outside [1, 6]", d->d);
  if (d->B < 1) return set_error(kErrInvalid, "fgp_mt_fit: B = %d", d->B);
  if (d->T_all < m->lay.T || d->T_all > FGP_MT_MAX_TASKS || d->rank < 0 || d->rank > FGP_MT_MAX_TASKS)
    return set_error(kErrInvalid, "fgp_mt_fit: T_all = %d, rank = %d", d->T_all, d->rank);
  if (d->dl != 1 && d->dl != d->d) return set_error(kErrInvalid, "fgp_mt_fit: dl = %d", d->dl);
  m->family = d->family;
  m->d = d->d;
  m->B = d->B;
  m->T_all = d->T_all;
  m->rank = d->rank;
  m->dl = d->dl;
  m->vtask_exp = d->vtask_exp;
  m->P = m->lay.T * (m->lay.T + 1) / 2;
  for (int k = 0; k < m->lay.T; ++k) {
    if (d->task[k] < 0 || d->task[k] >= d->T_all) return set_error(kErrInvalid, "fgp_mt_fit: task[%d] = %d", k, d->task[k]);
    m->task[k] = d->task[k];
  }
  for (int p = 0; p < m->P; ++p) m->spec_off[p] = d->spec_off[p];
  m->rg_scale = d->rg_scale;
  m->rg_ls = d->rg_ls;
  m->rg_noise = d->rg_noise;
  m->rg_factor = d->rg_factor;
  m->rg_vtask = d->rg_vtask;
  m->spec = static_cast<const double2*>(d->spectra);
  m->y = static_cast<const double2*>(d->y);
  m->raw = d->raw;
  m->prev = d->rprop_prev;
  m->step = d->rprop_step;
  m->grad = d->grad_out;
  m->loss_hist = d->loss_hist;
  m->raw_hist = d->raw_hist;
  m->gn = d->grad_norm;
  m->gl = d->grad_logdet;
  m->logdet_weight = d->logdet_weight;
  m->mll_const = d->mll_const;
  m->eta_minus = d->eta_minus;
  m->eta_plus = d->eta_plus;
  m->step_min = d->step_min;
  m->step_max = d->step_max;
  // problems of a parameter batch (ABI 16; G = 0: 1) and the row counts of the parameter blocks
  m->nug_coef = static_cast<const double2*>(d->nugget_coef);
  m->nug_ref = d->nugget_ref;
  if (m->nug_coef && (m->nug_ref < 0 || m->nug_ref >= m->lay.T))
    return set_error(kErrInvalid, "fgp_mt_fit: nugget_ref = %d", m->nug_ref);
  m->G = d->G > 0 ? d->G : 1;
  if (m->G > 65535) return set_error(kErrUnsupported, "fgp_mt_fit: G = %d problems > 65535", m->G);
  m->rows = d->rows;
  int nr[5];
  for (int q = 0; q < 5; ++q) nr[q] = d->nrows[q] > 0 ? d->nrows[q] : 1;
  if (m->G > 1 && !m->rows) return set_error(kErrInvalid, "fgp_mt_fit: G = %d problems without parameter rows", m->G);
  m->l_off = nr[0];
  m->n_off = m->l_off + nr[1] * m->dl;
  m->f_off = m->n_off + nr[2];
  m->v_off = m->f_off + nr[3] * m->T_all * m->rank;
  m->n_params = m->v_off + nr[4] * m->T_all;
  if (m->n_params > 8192) return set_error(kErrUnsupported, "fgp_mt_fit: %d parameters > 8192", m->n_params);
  const int64_t G = m->G, L = m->lay.L, rn = (int64_t)m->lay.R * m->lay.nmin;
  const int64_t cover = std::max<int64_t>(std::max<int64_t>(L, (int64_t)m->B * rn), m->lay.nmin);
  m->nblk = (int)std::min<int64_t>(1024, (cover + kWG - 1) / kWG);
  // workspace: lams, fac, zinv, glp [G][L] double2; z [G][B][R nmin] double2; logdet [G][nmin]; dkt [G][L]; part
  // [G][nblk][kMtgQ]; info
  size_t off = 0;
  const size_t o_lams = off; off += mtg_align(16 * (size_t)(G * L));
  const size_t o_fac = off; off += mtg_align(16 * (size_t)(G * L));
  const size_t o_zinv = off; off += mtg_align(16 * (size_t)(G * L));
  const size_t o_glp = off; off += mtg_align(16 * (size_t)(G * L));
  const size_t o_z = off; off += mtg_align(16 * (size_t)(G * m->B * rn));
  const size_t o_ld = off; off += mtg_align(8 * (size_t)(G * m->lay.nmin));
  const size_t o_dkt = off; off += mtg_align(8 * (size_t)(G * L));
  const size_t o_part = off; off += mtg_align(8 * (size_t)(G * m->nblk * kMtgQ));
  const size_t o_sums = off; off += mtg_align(8 * (size_t)(G * (kMtgQ + m->P)));
  const size_t o_info = off; off += 256;
  if (work_bytes) *work_bytes = (int64_t)off;
  char* w = static_cast<char*>(d->work);
  if (w) {
    m->lams = reinterpret_cast<double2*>(w + o_lams);
    m->fac = reinterpret_cast<double2*>(w + o_fac);
    m->zinv = reinterpret_cast<double2*>(w + o_zinv);
    m->glp = reinterpret_cast<double2*>(w + o_glp);
    m->z = reinterpret_cast<double2*>(w + o_z);
    m->logdet = reinterpret_cast<double*>(w + o_ld);
    m->dkt = reinterpret_cast<double*>(w + o_dkt);
    m->part = reinterpret_cast<double*>(w + o_part);
    m->sums = reinterpret_cast<double*>(w + o_sums);
    m->info = reinterpret_cast<int*>(w + o_info);
  }
  return kOk;
}

template <typename Fn>
static int mtg_with_d(int d, Fn&& fn) {
  switch (d) {
    case 1: return fn(std::integral_constant<int, 1>{});
    case 2: return fn(std::integral_constant<int, 2>{});
    case 3: return fn(std::integral_constant<int, 3>{});
    case 4: return fn(std::integral_constant<int, 4>{});
    case 5: return fn(std::integral_constant<int, 5>{});
    default: return fn(std::integral_constant<int, 6>{});
  }
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


int fgp_set_mt_class_kernel(int mode) {
  if (mode < 0 || mode > 2) return set_error(kErrInvalid, "fgp_set_mt_class_kernel: mode %d", mode);
  g_mt_class_mode = mode;
  return kOk;
}

int fgp_mt_fit_nparams(const fgp_mt_fit_desc* desc, int* n_params) {
  MtFit m;
  int rc = to_mtfit(desc, &m, nullptr);
  if (rc != kOk) return rc;
  if (!n_params) return set_error(kErrInvalid, "fgp_mt_fit_nparams: null n_params");
  *n_params = m.n_params;
  return kOk;
}

int fgp_mt_fit_work(const fgp_mt_fit_desc* desc, int64_t* bytes) {
  MtFit m;
  if (!bytes) return set_error(kErrInvalid, "fgp_mt_fit_work: null bytes");
  return to_mtfit(desc, &m, bytes);
}

int fgp_mt_fit_run(const fgp_mt_fit_desc* desc, int iter0, int iters, int final_no_update, void* stream) {
  MtFit m;
  int rc = to_mtfit(desc, &m, nullptr);
  if (rc != kOk) return rc;
  if (!desc->work || !desc->spectra || !desc->y || !desc->raw || !desc->rprop_prev || !desc->rprop_step ||
      !desc->grad_out || !desc->loss_hist || !desc->raw_hist)
    return set_error(kErrInvalid, "fgp_mt_fit_run: null pointer");
  if (iter0 < 0 || iters < 0) return set_error(kErrInvalid, "fgp_mt_fit_run: iter0 / iters");
  hipStream_t st = (hipStream_t)stream;
  const dim3 ge((unsigned)((m.lay.L + kWG - 1) / kWG), (unsigned)m.G), gc((unsigned)((m.lay.nmin + kWG - 1) / kWG), (unsigned)m.G);
  const dim3 gb((unsigned)m.nblk, (unsigned)m.G);
  // the step's LDS: the gradient, and copies of the parameters / totals / rows when they fit beside it
  const size_t shm0 = sizeof(double) * (size_t)m.n_params;
  const size_t shm1 = shm0 * 2 + sizeof(double) * (size_t)m.G * (kMtgQ + m.P) + 20 * (size_t)m.G;
  const int stage = shm1 <= 65536;
  const size_t shm = stage ? shm1 : shm0;
  // one wave per (class, problem) while the classes are few (and the class fits LDS), else a thread per class
  const size_t lds = mtc_lds(m.lay, m.B);
  const bool wave_class = lds > 0 && (g_mt_class_mode == 2 || (g_mt_class_mode == 0 && (int64_t)m.G * m.lay.nmin <= kMtcMaxClasses));
  const dim3 gw((unsigned)m.lay.nmin, (unsigned)m.G);
  return mtg_with_d(m.d, [&](auto dc) {
    constexpr int D = decltype(dc)::value;
    const dim3 gr((unsigned)((4 + D + m.P + kWG / 64 - 1) / (kWG / 64)), (unsigned)m.G);
    for (int it = 0; it < iters; ++it) {
      const int upd = !(final_no_update && it == iters - 1);
      k_mtg_lams<D><<<ge, kWG, 0, st>>>(m);
      if (wave_class) k_mtg_class<<<gw, kMtcWG, lds, st>>>(m);
      else k_mtg_factor_grad<<<gc, kWG, 0, st>>>(m);
      k_mtg_contract<D><<<gb, kWG, 0, st>>>(m);
      k_mtg_reduce<D><<<gr, kWG, 0, st>>>(m);
      if (stage) k_mtg_step<D, true><<<1, kMtgStepWG, shm, st>>>(m, iter0 + it, upd);
      else k_mtg_step<D, false><<<1, kMtgStepWG, shm, st>>>(m, iter0 + it, upd);
      const int r = check_launch("fgp_mt_fit_run");
      if (r != kOk) return r;
    }
    return (int)kOk;
  });
}

}  // extern "C"
