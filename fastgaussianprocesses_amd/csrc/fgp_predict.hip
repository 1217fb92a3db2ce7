// Posterior-mean cross-kernel contraction, matrix-free (FP64 VALU bound), and kernel rows.
//
// Replaces AbstractGP.post_mean (fastgps/abstract_gp.py:352-380), which materialises the [N, n]
// cross-kernel kmat = scale * prod_j(1 + l_j part_j(x_t, xb_i)) (abstract_fast_gp.py:192-196) and
// contracts it with coeffs = K^-1 y (util.py:396-425):
//     pmean[b, t] = sum_i K_g(x_t, xb_i) coeffs[b, i],   g = b mod Gk (per-output hyper-parameters)
// Lattice parts: coef_j B_{2 alpha_j}((x_tj - xb_ij) % 1)   (fast_gp_lattice.py:263-273)
// Net parts:     walsh1(floor((x_tj % 1) 2^t) XOR xb_ij)     (fast_gp_digital_net_b2.py:270-298)
//
// Layout: one thread per test point (lanes = test points, so every train point read from LDS is a
// broadcast), one workgroup per (train chunk, 256 test points); train points + coefficients of the
// chunk are staged through LDS in slabs; per-chunk partial sums are reduced in fixed order by a
// second kernel (bitwise reproducible, no atomics).
#include <cmath>
#include <cstdlib>
#include <type_traits>

#include "fgp_common.h"
#include "fgp_runtime.h"
#include "../../include/fgp_hip.h"

namespace fgp {

constexpr int kPmB = 4;          // outputs per launch
constexpr int kSlab = 256;       // train points per LDS slab
constexpr int kChunk = 1024;     // train points per workgroup (4 slabs)
#ifndef FGP_PM_UNROLL
#define FGP_PM_UNROLL 2          // training points per k_post_mean loop trip (A/B builds: tools/build_exp.sh)
#endif

struct PredSpec {
  int order[FGP_MAX_D];
  double coef[FGP_MAX_D];
};

// Element strides between consecutive problems of a batch of independent GPs (all 0: one problem):
// test points x, training points z ([d][n] per problem), hyper-parameter rows h, coefficients /
// eigenvalue weights c.
struct ProbStrides {
  int64_t x, z, h, c;
};

// ------------------------------------------------------------------------------------------------
// Per-factor arithmetic.  Lattice: even Bernoulli polynomials are polynomials in u = t(t - 1), and
// B_{2a}((x - z) % 1) = B_{2a}(|x - z|) exactly for x, z in [0, 1] (B_{2a}(1 - t) = B_{2a}(t)), so
//   1 + l c B2 = fma(a, u, 1 + a/6)                 a = l c
//   1 + l c B4 = fma(a u, u, 1 - a/30)              (B4 = u^2 - 1/30)
//   1 + l c B6 = fma(a u^2, u - 1/2, 1 + a/42)      (B6 = u^2 (u - 1/2) + 1/42)
//   1 + l c B8 = fma(a u^2, u (u - 4/3) + 2/3, 1 - a/30)
// (identical to the reference's Horner evaluation up to rounding).  Net (order-1 Walsh):
//   1 + l walsh1(delta) = (1 + l) - 3 l 2^(floor(log2 delta) - t)   (= 1 + l when delta = 0)
__device__ __forceinline__ double fac_const(int order, double a) {
  switch (order) {
    case 2: return 1.0 + a * (1.0 / 6.0);
    case 6: return 1.0 + a * (1.0 / 42.0);
    default: return 1.0 - a * (1.0 / 30.0);   // 4, 8
  }
}

__device__ __forceinline__ double lat_factor(int order, double t, double a, double c) {
  const double u = fma(t, t, -t);
  switch (order) {
    case 2: return fma(a, u, c);
    case 4: return fma(a * u, u, c);
    case 6: return fma(a * u * u, u - 0.5, c);
    default: return fma(a * u * u, fma(u, u - 4.0 / 3.0, 2.0 / 3.0), c);
  }
}

__device__ __forceinline__ double net_factor(unsigned long long delta, int tbits, double c1, double c3) {
  if (delta == 0ull) return c1;
  const int fl = 63 - __clzll((long long)delta);
  return c1 - ldexp(c3, fl - tbits);
}

// Net factor of Walsh order ord: order 1 as above (fa = 1 + l, fc = 3 l); orders 2..4
// 1 + l omega_ord(delta) (fa = l; walsh_omega, fgp_common.h)
__device__ __forceinline__ double net_fa(int ord, double l) { return ord <= 1 ? 1.0 + l : l; }
__device__ __forceinline__ double net_factor_o(int ord, unsigned long long delta, int tbits, double fa, double fc) {
  if (ord <= 1) return net_factor(delta, tbits, fa, fc);
  return __builtin_fma(fa, walsh_omega(ord, delta, tbits), 1.0);
}

__device__ __forceinline__ unsigned long long to_bits(double v, int tbits) {
  double r = fmod(v, 1.0);
  if (r != 0.0 && r < 0.0) r += 1.0;                 // torch.remainder(v, 1)
  return (unsigned long long)(long long)floor(r * ldexp(1.0, tbits));
}

// ------------------------------------------------------------------------------------------------
// pmean partials: thread = test point, workgroup = (kChunk train points, 256 test points).
// ORD: uniform Bernoulli order of every dimension (4 = the default alpha = 2) or 0 = per-dim table.
template <int FAM, int D, int NB, int ORD>
__global__ __launch_bounds__(kWG) void k_post_mean(const double* __restrict__ xt, int64_t N, const void* __restrict__ z,
                                                    int64_t n, PredSpec spec, int tbits,
                                                    const double* __restrict__ hyp, int Gk,
                                                    const double* __restrict__ coeffs, int64_t coeff_stride, int B,
                                                    double* __restrict__ partial, int64_t nchunks, ProbStrides ps,
                                                    int64_t chunk) {
  __shared__ double zs[D][kSlab];
  __shared__ double cs[NB][kSlab];
  const int tid = threadIdx.x;
  const int64_t t = (int64_t)blockIdx.y * kWG + tid;
  const bool live = t < N;
  // problem p of a batch of independent GPs (fgp_post_mean_batched); p = 0 otherwise
  const int64_t p = blockIdx.z;
  xt += p * ps.x;
  z = static_cast<const char*>(z) + p * ps.z * 8;
  hyp += p * ps.h;
  coeffs += p * ps.c;
  partial += p * (int64_t)B * N * nchunks;
  double xv[D];
  unsigned long long xbv[D];
#pragma unroll
  for (int j = 0; j < D; ++j) {
    xv[j] = live ? xt[t * D + j] : 0.0;
    if constexpr (FAM == 1) xbv[j] = to_bits(xv[j], tbits);
  }
  double sc[NB], fa[NB][D], fc[NB][D];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const int g = (b < B ? b : 0) % Gk;
    sc[b] = hyp[g * (1 + D)];
#pragma unroll
    for (int j = 0; j < D; ++j) {
      const double l = hyp[g * (1 + D) + 1 + j];
      if constexpr (FAM == 0) {
        const int ord = ORD ? ORD : spec.order[j];
        fa[b][j] = l * spec.coef[j];
        fc[b][j] = fac_const(ord, fa[b][j]);
      } else {
        fa[b][j] = net_fa(spec.order[j], l);   // c1 (order 1) / l
        fc[b][j] = 3.0 * l;                     // c3
      }
    }
  }
  // Folded B4 factors (ORD = 4, every a != 0): 1 + a B4(t) = a (u^2 + c'), c' = (1 - a/30) / a, with
  // prod_j a_j moved into the output scale -- 4 operations per dimension and pair instead of 5 (this
  // kernel is FP64-VALU bound).  a c' = 1 - a/30 = O(1), so the rounding stays at the factor's ulp.
  bool fold = FAM == 0 && ORD == 4;
  double cp[NB][D];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
#pragma unroll
    for (int j = 0; j < D; ++j) {
      fold = fold && fa[b][j] != 0.0;
      cp[b][j] = fc[b][j] / fa[b][j];
    }
  }
  double acc[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) acc[b] = 0.0;
  const int64_t i0 = (int64_t)blockIdx.x * chunk;
  const int64_t i1 = i0 + chunk < n ? i0 + chunk : n;
  auto slabs = [&](auto fold_c) {
    constexpr bool FOLD = decltype(fold_c)::value;
    for (int64_t s0 = i0; s0 < i1; s0 += kSlab) {
      const int cnt = (int)((i1 - s0) < kSlab ? (i1 - s0) : kSlab);
      __syncthreads();
      if (tid < cnt) {
#pragma unroll
        for (int j = 0; j < D; ++j) {
          if constexpr (FAM == 0) zs[j][tid] = static_cast<const double*>(z)[(int64_t)j * n + s0 + tid];
          else zs[j][tid] = __longlong_as_double(static_cast<const long long*>(z)[(int64_t)j * n + s0 + tid]);
        }
#pragma unroll
        for (int b = 0; b < NB; ++b) cs[b][tid] = b < B ? coeffs[(int64_t)b * coeff_stride + s0 + tid] : 0.0;
      }
      __syncthreads();
#pragma unroll FGP_PM_UNROLL
      for (int i = 0; i < cnt; ++i) {
        double p[NB];
#pragma unroll
        for (int b = 0; b < NB; ++b) p[b] = 1.0;
#pragma unroll
        for (int j = 0; j < D; ++j) {
          if constexpr (FAM == 0) {
            const double tj = fabs(xv[j] - zs[j][i]);
            if constexpr (FOLD) {
              const double u = fma(tj, tj, -tj);
#pragma unroll
              for (int b = 0; b < NB; ++b) p[b] *= fma(u, u, cp[b][j]);
            } else {
              const int ord = ORD ? ORD : spec.order[j];
#pragma unroll
              for (int b = 0; b < NB; ++b) p[b] *= lat_factor(ord, tj, fa[b][j], fc[b][j]);
            }
          } else {
            const unsigned long long delta = xbv[j] ^ (unsigned long long)__double_as_longlong(zs[j][i]);
#pragma unroll
            for (int b = 0; b < NB; ++b) p[b] *= net_factor_o(spec.order[j], delta, tbits, fa[b][j], fc[b][j]);
          }
        }
#pragma unroll
        for (int b = 0; b < NB; ++b) acc[b] = fma(p[b], cs[b][i], acc[b]);
      }
    }
  };
  if (FAM == 0 && ORD == 4 && fold) {
    slabs(std::integral_constant<bool, FAM == 0 && ORD == 4>{});
#pragma unroll
    for (int b = 0; b < NB; ++b) {
#pragma unroll
      for (int j = 0; j < D; ++j) sc[b] *= fa[b][j];
    }
  } else {
    slabs(std::integral_constant<bool, false>{});
  }
  if (live) {
#pragma unroll
    for (int b = 0; b < NB; ++b)
      if (b < B) partial[((int64_t)b * N + t) * nchunks + blockIdx.x] = sc[b] * acc[b];
  }
}

// out[b, t] = sum_c partial[(b N + t), c]: one workgroup per output element, fixed reduction tree
__global__ __launch_bounds__(kWG) void k_sum_chunks(const double* __restrict__ partial, int64_t nchunks,
                                                     double* __restrict__ out, int64_t out_stride, int64_t N) {
  __shared__ double red[kWG / 64];
  const int64_t e = blockIdx.x;
  double s = 0.0;
  for (int64_t c = threadIdx.x; c < nchunks; c += kWG) s += partial[e * nchunks + c];
  s = block_sum(s, red);
  if (threadIdx.x == 0) out[(e / N) * out_stride + e % N] = s;
}

// kernel rows: rows[g, t, i] = K_g(x_t, z_i) for g < Gk (the [N, n] matrix the reference builds for
// post_var / post_cov, abstract_gp.py:407-411,452-457); same factor arithmetic as k_post_mean
template <int FAM, int D>
__global__ __launch_bounds__(kWG) void k_kernel_rows(const double* __restrict__ xt, int64_t N, const void* __restrict__ z,
                                                      int64_t n, PredSpec spec, int tbits, const double* __restrict__ hyp,
                                                      int Gk, double* __restrict__ rows) {
  const int64_t i = (int64_t)blockIdx.x * kWG + threadIdx.x;
  const int64_t t = blockIdx.y;
  if (i >= n) return;
  double tv[D];
  unsigned long long dv[D];
#pragma unroll
  for (int j = 0; j < D; ++j) {
    const double v = xt[t * D + j];
    if constexpr (FAM == 0) tv[j] = fabs(v - static_cast<const double*>(z)[(int64_t)j * n + i]);
    else dv[j] = to_bits(v, tbits) ^ (unsigned long long)static_cast<const long long*>(z)[(int64_t)j * n + i];
  }
  for (int g = 0; g < Gk; ++g) {
    double p = 1.0;
#pragma unroll
    for (int j = 0; j < D; ++j) {
      const double l = hyp[g * (1 + D) + 1 + j];
      if constexpr (FAM == 0) {
        const double a = l * spec.coef[j];
        p *= lat_factor(spec.order[j], tv[j], a, fac_const(spec.order[j], a));
      } else {
        p *= net_factor_o(spec.order[j], dv[j], tbits, net_fa(spec.order[j], l), 3.0 * l);
      }
    }
    rows[((int64_t)g * N + t) * n + i] = hyp[g * (1 + D)] * p;
  }
}

// ------------------------------------------------------------------------------------------------
// Posterior variance by Parseval (n > 4096):  with r_t[i] = K(x_t, z_i) and A = 1/ev,
//   sum_i r_t[i] (K^-1 r_t)[i] = Re <r_t, ift(A ft(r_t))> = sum_k Re(A_k) |ft(r_t)_k|^2,
// which equals the reference's sum(t * kmat) with t = ift(A ft(kmat)).real (abstract_gp.py:408-412,
// util.py:338-353) for real r.  One forward transform per test point instead of two, and the kernel
// rows are generated inside the row pass instead of being materialised.
struct QfArgs {
  int log2n, d, tbits, N;
  const double* xt;          // [N][d]
  const void* z;             // [d][n] float64 (lattice) / int64 (net)
  PredSpec spec;
  const double* hyp;         // device [1 + d]: scale, lengthscales
  const double* wa;          // [n] Re(A)
  void* work;                // [P][N][n]
  double* partial;           // [P][N][n / 4096]
  ProbStrides ps;            // per-problem strides of xt, z, hyp, wa (batched GPs; 0 for one problem)
  // lattice training points regenerated in the kernel instead of read from z (natural-order rank-1
  // lattice: x_ij = ((brev_m(i) z_j mod n) / n + shift_j) % 1, shift row of problem p at gshift + p * gss)
  int gen;
  unsigned gz[FGP_MAX_D];
  const double* gshift;
  int64_t gss;
};

template <int P2, typename T>
__global__ __launch_bounds__(kWG) void k_qf_rows(QfArgs q, const double2* __restrict__ tw, const double2* __restrict__ twm) {
  constexpr int N2 = 1 << P2, TL = N2 / 16, RPW = kTile / N2;
  constexpr int FAM = sizeof(T) == 16 ? 0 : 1;
  __shared__ T lds[kTile + kTile / 16];
  __shared__ T red[kWG / 64];
  const int m = q.log2n, m1 = m - P2;
  const int64_t n = (int64_t)1 << m;
  const int64_t tiles = n >> kTileLog;
  const int tg = (int)(blockIdx.x / tiles);           // (problem, test point) row of work
  const int pb = tg / q.N, t = tg % q.N;
  const int row0 = (int)(blockIdx.x % tiles) * RPW;
  const int tid = threadIdx.x;
  const double* xt = q.xt + pb * q.ps.x;
  const double* hyp = q.hyp + pb * q.ps.h;
  const void* zp = static_cast<const char*>(q.z) + pb * q.ps.z * 8;
  double xv[FGP_MAX_D], fa[FGP_MAX_D], fc[FGP_MAX_D];
  unsigned long long xb[FGP_MAX_D];
  const double scale = hyp[0];
#pragma unroll
  for (int j = 0; j < FGP_MAX_D; ++j) {
    xv[j] = j < q.d ? xt[(int64_t)t * q.d + j] : 0.0;
    const double l = j < q.d ? hyp[1 + j] : 0.0;
    if constexpr (FAM == 0) {
      fa[j] = l * q.spec.coef[j];
      fc[j] = fac_const(q.spec.order[j], fa[j]);
    } else {
      xb[j] = to_bits(xv[j], q.tbits);
      fa[j] = net_fa(q.spec.order[j], l);
      fc[j] = 3.0 * l;
    }
  }
  const int64_t base = (int64_t)row0 * N2;
  double kv0[8], kv1[8];
  double sum = 0.0;
  const bool gen = FAM == 0 && q.gen;                // uniform
  const unsigned mask = (unsigned)(n - 1);
  const double inv_n = ldexp(1.0, -m);
  double gsh[FGP_MAX_D];
#pragma unroll
  for (int j = 0; j < FGP_MAX_D; ++j) gsh[j] = (gen && j < q.d) ? q.gshift[pb * q.gss + j] : 0.0;
#pragma unroll 2
  for (int kk = 0; kk < 8; ++kk) {
    const int e = 2 * tid + 512 * kk;
    double p0 = scale, p1 = scale;
    const unsigned br0 = gen ? brev_bits((unsigned)(base + e), m) : 0u, br1 = br0 + (unsigned)(n >> 1);
#pragma unroll
    for (int j = 0; j < FGP_MAX_D; ++j) {
      if (j < q.d) {
        if constexpr (FAM == 0) {
          double2 zv;
          if (gen) {   // brev_m(i + 1) = brev_m(i) + n/2 for even i
            zv = make_double2(lattice_coord(br0, q.gz[j], mask, inv_n, gsh[j]),
                              lattice_coord(br1, q.gz[j], mask, inv_n, gsh[j]));
          } else {
            zv = *reinterpret_cast<const double2*>(static_cast<const double*>(zp) + (int64_t)j * n + base + e);
          }
          p0 *= lat_factor(q.spec.order[j], fabs(xv[j] - zv.x), fa[j], fc[j]);
          p1 *= lat_factor(q.spec.order[j], fabs(xv[j] - zv.y), fa[j], fc[j]);
        } else {
          const longlong2 zv = *reinterpret_cast<const longlong2*>(static_cast<const long long*>(zp) + (int64_t)j * n + base + e);
          p0 *= net_factor_o(q.spec.order[j], xb[j] ^ (unsigned long long)zv.x, q.tbits, fa[j], fc[j]);
          p1 *= net_factor_o(q.spec.order[j], xb[j] ^ (unsigned long long)zv.y, q.tbits, fa[j], fc[j]);
        }
      }
    }
    kv0[kk] = p0;
    kv1[kk] = p1;
    sum += p0 + p1;
  }
  if constexpr (RPW == 1) {
    const double mean = block_sum(sum, (double*)red) * (1.0 / N2);
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      const int e = 2 * tid + 512 * kk;
      if constexpr (FAM == 0) {
        lds[padi(e)] = make_double2(kv0[kk] - mean, 0.0);
        lds[padi(e + 1)] = make_double2(kv1[kk] - mean, 0.0);
      } else {
        lds[padi(e)] = kv0[kk] - mean;
        lds[padi(e + 1)] = kv1[kk] - mean;
      }
    }
    __syncthreads();
    T mt;
    if constexpr (FAM == 0) mt = make_double2(mean, 0.0);
    else mt = mean;
    transform_add_mean<P2, false>(lds, tid, mt, tw);
  } else {
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      const int e = 2 * tid + 512 * kk;
      if constexpr (FAM == 0) {
        lds[padi(e)] = make_double2(kv0[kk], 0.0);
        lds[padi(e + 1)] = make_double2(kv1[kk], 0.0);
      } else {
        lds[padi(e)] = kv0[kk];
        lds[padi(e + 1)] = kv1[kk];
      }
    }
    __syncthreads();
    T* s = lds + (tid / TL) * (N2 + N2 / 16);
    center_transform<P2, false>(s, tid % TL, 1, red, tw);
  }
  T* out = static_cast<T*>(q.work) + (int64_t)tg * n + base;
  if constexpr (FAM == 0 && RPW == 1) {
    const RowTwiddle rt((unsigned)row0, tid, P2, m1, tw, twm);
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int e = tid + k * kWG;
      out[e] = cmul(lds[padi(e)], rt.at(k, P2, m1, tw, twm));
    }
  } else {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int e = tid + k * kWG;
      T v = lds[padi(e)];
      if constexpr (FAM == 0) {
        const unsigned ex = brev_bits((unsigned)(row0 + (e >> P2)), m1) * (unsigned)(e & (N2 - 1));
        v = cmul(v, inter_tw(ex, P2, m1, tw, twm));
      }
      out[e] = v;
    }
  }
}

__device__ __forceinline__ double sqabs(double2 v) { return v.x * v.x + v.y * v.y; }
__device__ __forceinline__ double sqabs(double v) { return v * v; }

template <int P1, typename T>
__global__ __launch_bounds__(kWG) void k_qf_cols(QfArgs q, const double2* __restrict__ tw) {
  constexpr int N1 = 1 << P1, C = kTile / N1, TL = N1 / 16;
  constexpr int PADLEN = N1 + N1 / 16;
  constexpr int CS = (PADLEN % 2 == 0) ? PADLEN + 1 : PADLEN;
  __shared__ T lds[kLds];
  __shared__ T part[ColPart<C>::size];
  __shared__ double redd[kWG / 64];
  const int m = q.log2n;
  const int64_t n = (int64_t)1 << m, N2 = n >> P1;
  const int64_t tiles = n >> kTileLog;
  const int tg = (int)(blockIdx.x / tiles);
  const int blk = (int)(blockIdx.x % tiles);
  const int64_t c0 = (int64_t)blk * C;
  const int tid = threadIdx.x;
  const T* in = static_cast<const T*>(q.work) + (int64_t)tg * n + c0;
  const double* wa = q.wa + (tg / q.N) * q.ps.c;
  const int cl = tid % C, col = tid / TL;
  T v[16];
  T sum = zero_v<T>();
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    v[k] = in[(int64_t)((tid + k * kWG) / C) * N2 + cl];
    sum += v[k];
  }
  column_partials<C>(sum, part);
  const T mean_l = column_total<C>(cl, part) * (1.0 / N1);
  const T mean_t = column_total<C>(col, part) * (1.0 / N1);
#pragma unroll
  for (int k = 0; k < 16; ++k) lds[cl * CS + padi((tid + k * kWG) / C)] = v[k] - mean_l;
  __syncthreads();
  transform_add_mean<P1, false>(lds + col * CS, tid % TL, mean_t, tw);
  const double inv_n = 1.0 / (double)n;
  double acc = 0.0;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int e = tid + k * kWG;
    const int c = e % C, r = e / C;
    acc += sqabs(lds[c * CS + padi(r)]) * inv_n * wa[(int64_t)r * N2 + c0 + c];
  }
  acc = block_sum(acc, redd);
  if (tid == 0) q.partial[(int64_t)tg * tiles + blk] = acc;
}

// ---------------------------------------------------------------- half-length (R2C) quadratic form
// Lattice, n >= 2^17 (as the fit kernels, FGP_R2C=0 selects the full-length ones): the kernel row
// r_t is real, so its spectrum comes from the half-length transform of r_t[:n/2] + i r_t[n/2:]
// (csrc/fgp_nll.hip, k_fwd_rows_r2c / k_fwd_cols_r2c: same engine, same paired column tiles) and
//   sum_k wa_k |ft(r_t)_k|^2 = sum over mirror pairs (k, n/2 - k) of w (wa_k |A0|^2 + wa_{k+n/2} |A1|^2) / n
// with A0, A1 the unnormalised spectrum at k, k + n/2 and w = 2 for a regular pair (its mirror
// frequencies n/2 - k, n - k have the same |.|^2 and, ev being Hermitian, the same wa) and 1 for the
// self-mirrored frequencies.  Per test point: 8n bytes written + 8n + 4n read instead of 32n + 8n.
//
// Row kernel: register-resident half-length row transform of the kernel values of 16 consecutive
// points per half.  With regenerated lattice points (gen) the distance is formed from the lattice index
// directly, delta = (x_t - shift - k/n) % 1 with k = brev_m(i) z_j mod n (k/n exact): one fract instead
// of the generated point's two and |x - z|; it differs from |x_t - x_i| of the materialised points by
// rounding only (the reference's own kmat carries the rounding of its generated points).
template <int D, int ORD>
__device__ __forceinline__ void qf_row16(const QfArgs& q, int64_t n, int64_t i0, const double* xv, const double* cv,
                                         const double* fa, const double* fc, const void* zp, bool gen, double scale,
                                         double* r, double& sum) {
  const int m = q.log2n;
  const unsigned mask = (unsigned)(n - 1);
  const double inv_n = ldexp(1.0, -m);
  if (gen) {
    const unsigned br0 = brev_bits((unsigned)i0, m);
    static_for<0, 16>([&](auto tc) {
      constexpr int t = decltype(tc)::value;
      const unsigned br = br0 | (Brev4<t>::value << (m - 4));
      double pr = scale;
#pragma unroll
      for (int j = 0; j < D; ++j) {
        const double kf = (double)(mul_u24(br, q.gz[j]) & mask);
        const double dl = __builtin_amdgcn_fract(__builtin_fma(-kf, inv_n, cv[j]));
        pr *= lat_factor(ORD ? ORD : q.spec.order[j], dl, fa[j], fc[j]);
      }
      r[t] = pr;
    });
  } else {
#pragma unroll
    for (int t = 0; t < 16; ++t) r[t] = scale;
#pragma unroll
    for (int j = 0; j < D; ++j) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const double2 zv = *reinterpret_cast<const double2*>(static_cast<const double*>(zp) + (int64_t)j * n + i0 + 2 * u);
        r[2 * u] *= lat_factor(ORD ? ORD : q.spec.order[j], fabs(xv[j] - zv.x), fa[j], fc[j]);
        r[2 * u + 1] *= lat_factor(ORD ? ORD : q.spec.order[j], fabs(xv[j] - zv.y), fa[j], fc[j]);
      }
    }
  }
#pragma unroll
  for (int t = 0; t < 16; ++t) sum += r[t];
}

// paired column-tile position of (row u, column k) of the N1 x N2 half-length intermediate
// (the layout of csrc/fgp_nll.hip work_pos_pair)
__device__ __forceinline__ int64_t qf_pos_pair(int64_t u, int64_t k, int P1, int64_t N2) {
  const int CL = kTileLog - P1;
  const int64_t h = N2 >> 1;
  int64_t tile, slot;
  if (k == h) {
    tile = 0;
    slot = (int64_t)1 << (CL - 1);
  } else {
    const int64_t c = k < h ? k : N2 - k;
    tile = c >> (CL - 1);
    slot = (c & ((1 << (CL - 1)) - 1)) + (k > h ? ((int64_t)1 << (CL - 1)) : 0);
  }
  return (tile << kTileLog) + (u << CL) + slot;
}

// ORD: the Bernoulli order of every dimension (4 = the default alpha = 2), 0 = per-dimension orders
template <int D, int ORD>
__global__ __launch_bounds__(kWG) void k_qf_rows_r2c(QfArgs q, const double2* __restrict__ tw, const double2* __restrict__ twm) {
  constexpr int P2 = 12, N2 = 1 << P2;
  __shared__ double ldsd[kTile + kTile / 16];
  __shared__ double2 red[kWG / 64];
  const int mt = q.log2n - 1, m1 = mt - P2;
  const int64_t n = (int64_t)1 << q.log2n, nt = n >> 1;
  const int64_t tiles = nt >> kTileLog;
  const int tg = (int)(blockIdx.x / tiles);           // (problem, test point) row of work
  const int pb = tg / q.N, t = tg % q.N;
  const int row0 = (int)(blockIdx.x % tiles);
  const int tid = threadIdx.x;
  const double* xt = q.xt + pb * q.ps.x;
  const double* hyp = q.hyp + pb * q.ps.h;
  const void* zp = static_cast<const char*>(q.z) + pb * q.ps.z * 8;
  const bool gen = q.gen;
  double xv[D], cv[D], fa[D], fc[D];
  const double scale = hyp[0];
#pragma unroll
  for (int j = 0; j < D; ++j) {
    xv[j] = xt[(int64_t)t * D + j];
    cv[j] = gen ? xv[j] - q.gshift[pb * q.gss + j] : 0.0;
    fa[j] = hyp[1 + j] * q.spec.coef[j];
    fc[j] = fac_const(q.spec.order[j], fa[j]);
  }
  const int64_t base = (int64_t)row0 * N2;
  double lo[16], hi[16];
  double slo = 0.0, shi = 0.0;
  qf_row16<D, ORD>(q, n, base + 16 * tid, xv, cv, fa, fc, zp, gen, scale, lo, slo);
  qf_row16<D, ORD>(q, n, nt + base + 16 * tid, xv, cv, fa, fc, zp, gen, scale, hi, shi);
  double2 v[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) v[k] = make_double2(lo[k], hi[k]);
  const double2 mean = block_sum_t(make_double2(slo, shi), red) * (1.0 / N2);
#pragma unroll
  for (int k = 0; k < 16; ++k) v[k] -= mean;
  fwd_reg_passes<P2, 0, true>(v, ldsd, tid, tw);
  if (tid == 0) v[0] += mean * (double)N2;
  const RowTwiddle rt((unsigned)row0, tid, P2, m1, tw, twm);
  double2* out = static_cast<double2*>(q.work) + (int64_t)tg * n;
#pragma unroll
  for (int k = 0; k < 16; ++k)
    out[qf_pos_pair(row0, tid + k * kWG, m1, N2)] = cmul(v[k], rt.at(k, P2, m1, tw, twm));
}

// column pass at half length + mirror split + weighted Parseval sum; one partial per column tile
template <int P1>
__global__ __launch_bounds__(kWG, 2) void k_qf_cols_r2c(QfArgs q, const double2* __restrict__ tw,
                                                         const double2* __restrict__ twmf) {
  constexpr int N1 = 1 << P1, C = kTile / N1, CS = N1 + 1, HC = C / 2;
  constexpr int RL0 = PassRL<P1, 0>::value, R0 = 1 << RL0;
  constexpr int SL = LastPass<P1>::S, RLL = PassRL<P1, SL>::value, RLAST = 1 << RLL;
  constexpr int JOBS = kTile / 2 / kWG, RSTEP = kWG / HC;
  static_assert(JOBS * RSTEP == N1, "pair jobs cover the tile");
  __shared__ double2 lds[C * CS];
  __shared__ double2 part[ColPart<C>::size];
  __shared__ double redd[kWG / 64];
  const int m = q.log2n;
  const int64_t n = (int64_t)1 << m, nt = n >> 1, N2 = nt >> P1;
  const int64_t tiles = nt >> kTileLog;
  const int tg = (int)(blockIdx.x / tiles);
  const int blk = (int)(blockIdx.x % tiles);
  const int tid = threadIdx.x;
  const int sl = tid % C, tt = tid / C;
  const double2* wk = static_cast<const double2*>(q.work) + (int64_t)tg * n + (int64_t)blk * kTile + sl;
  const double* wa = q.wa + (tg / q.N) * q.ps.c;
  double2* col = lds + sl * CS;
  const int jq = tid % HC, rr0 = tid / HC;
  const bool col0 = blk == 0 && jq == 0;
  const int64_t cp_gen = (int64_t)blk * HC + jq;
  auto job_primary = [&](int j, int& sp, int& rp, int64_t& cp) {
    const int rr = rr0 + RSTEP * j;
    if (!col0) {
      sp = jq; rp = rr; cp = cp_gen;
    } else if (rr < N1 / 2) {
      sp = 0; rp = rr; cp = 0;
    } else {
      sp = HC; rp = rr - N1 / 2; cp = N2 >> 1;
    }
  };
  double w0[JOBS], w1[JOBS];
#pragma unroll
  for (int j = 0; j < JOBS; ++j) {
    int sp, rp;
    int64_t cp;
    job_primary(j, sp, rp, cp);
    const double* wp = wa + cp + (int64_t)rp * N2;
    w0[j] = wp[0];
    w1[j] = wp[nt];
  }
  double2 v[16];
#pragma unroll
  for (int j = 0; j < 16 / R0; ++j)
#pragma unroll
    for (int t = 0; t < R0; ++t) v[j * R0 + t] = wk[pass_pos<P1, 0, RL0>(tt, j, t) * C];
  double2 sum = zero_v<double2>();
#pragma unroll
  for (int k = 0; k < 16; ++k) sum += v[k];
  column_partials<C>(sum, part);
  const double2 mean = column_total<C>(sl, part) * (1.0 / N1);
#pragma unroll
  for (int k = 0; k < 16; ++k) v[k] -= mean;
  fwd_reg_passes<P1, 0, false>(v, col, tt, tw);
  if (tt == 0) v[0] += mean * (double)N1;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 16 / RLAST; ++j)
#pragma unroll
    for (int t = 0; t < RLAST; ++t) col[pass_pos<P1, SL, RLL>(tt, j, t)] = v[j * RLAST + t];
  __syncthreads();
  double acc2 = 0.0, acc1 = 0.0;
  const double2 wcp = twmf[col0 ? 0 : cp_gen];
  auto split = [&](double2 zk, double2 zm, double2 W, double wk0, double wk1) {
    const double2 S = make_double2(zk.x + zm.x, zk.y - zm.y);
    const double2 Dd = make_double2(zk.x - zm.x, zk.y + zm.y);
    const double2 wd = cmul(W, Dd);
    const double2 A0 = make_double2(0.5 * (S.x + wd.y), 0.5 * (S.y - wd.x));
    const double2 A1 = make_double2(0.5 * (S.x - wd.y), 0.5 * (S.y + wd.x));
    return __builtin_fma(wk0, sqabs(A0), wk1 * sqabs(A1));
  };
#pragma unroll 2
  for (int j = 0; j < JOBS; ++j) {
    int sp, rp;
    int64_t cp;
    job_primary(j, sp, rp, cp);
    int ss, rs;
    if (!col0) {
      ss = sp + HC; rs = N1 - 1 - rp;
    } else if (sp == 0) {
      ss = 0; rs = (N1 - rp) & (N1 - 1);
    } else {
      ss = HC; rs = N1 - 1 - rp;
    }
    const bool self = col0 && sp == 0 && rp == 0;
    const double2 wc = col0 ? twmf[cp] : wcp;
    const double2 W = cmul(wc, tw[rp << (24 - m)]);
    const double s = split(lds[sp * CS + rp], lds[ss * CS + rs], W, w0[j], w1[j]);
    if (self) {
      acc1 += s;
      constexpr int rh = N1 / 2;     // second self-mirrored element of column 0 (frequencies n/4, 3n/4)
      const double2 zh = lds[rh];
      acc1 += split(zh, zh, tw[rh << (24 - m)], wa[(int64_t)rh * N2], wa[(int64_t)rh * N2 + nt]);
    } else {
      acc2 += s;
    }
  }
  double acc = __builtin_fma(2.0, acc2, acc1) * (1.0 / (double)n);
  acc = block_sum(acc, redd);
  if (tid == 0) q.partial[(int64_t)tg * tiles + blk] = acc;
}

// Posterior variance of (problem p, test point t) from its quadratic-form partials:
//   out = K(x, x) - sum_c partial[c], negative values set to 0 (abstract_gp.py:407-413), with
//   K(x, x) = scale * prod_j (1 + l_j part0_j), AbstractFastGP._kernel at zero distance.
__global__ __launch_bounds__(kWG) void k_qf_finish(const double* __restrict__ partial, int64_t nchunks,
                                                    const double* __restrict__ hyp, int64_t hps, PredSpec part0,
                                                    int d, int64_t N, double* __restrict__ out) {
  __shared__ double red[kWG / 64];
  const int64_t e = blockIdx.x;
  double s = 0.0;
  for (int64_t c = threadIdx.x; c < nchunks; c += kWG) s += partial[e * nchunks + c];
  s = block_sum(s, red);
  if (threadIdx.x == 0) {
    const double* h = hyp + (e / N) * hps;
    double pr = 1.0;
    for (int j = 0; j < d; ++j) pr *= 1.0 + h[1 + j] * part0.coef[j];
    const double v = h[0] * pr - s;
    out[e] = v < 0.0 ? 0.0 : v;
  }
}

// A = 1 / ev, ev = sqrt(n) lam + noise (util.py:285,292-300), and the coefficient-solve input
// ya = ytilde * A (util.py:341-342 with the cached ytilde); wa = Re(A), the post_var weights.
template <typename T>
__global__ __launch_bounds__(kWG) void k_inv_eig(const T* __restrict__ lam, const T* __restrict__ yt, int64_t yts,
                                                  const double* __restrict__ raw_noise, int64_t nzs, double rootn,
                                                  int log2n, int64_t total, T* __restrict__ ya,
                                                  double* __restrict__ wa) {
  const int64_t e = (int64_t)blockIdx.x * kWG + threadIdx.x;
  if (e >= total) return;
  const int64_t p = e >> log2n, i = e & (((int64_t)1 << log2n) - 1);
  const double noise = exp(raw_noise[p * nzs]);
  const T l = lam[e];
  const T y = yt[p * yts + i];
  if constexpr (sizeof(T) == 16) {
    const double ar = rootn * l.x + noise, ai = rootn * l.y;
    const double inv = 1.0 / (ar * ar + ai * ai);
    const double rr = ar * inv, ri = -ai * inv;
    ya[e] = make_double2(y.x * rr - y.y * ri, y.x * ri + y.y * rr);
    if (wa) wa[e] = rr;
  } else {
    const double a = 1.0 / (rootn * l + noise);
    ya[e] = y * a;
    if (wa) wa[e] = a;
  }
}

template <int FAM, int D>
static void post_mean_d(dim3 grid, hipStream_t st, bool uniform4, int B, const double* xt, int64_t N, const void* z,
                        int64_t n, const PredSpec& spec, int tbits, const double* hyp, int Gk, const double* coeffs,
                        int64_t cstride, double* work, int64_t nchunks, const ProbStrides& ps, int64_t chunk) {
  if (B == 1) {
    if (FAM == 1 || uniform4)
      k_post_mean<FAM, D, 1, 4><<<grid, kWG, 0, st>>>(xt, N, z, n, spec, tbits, hyp, Gk, coeffs, cstride, B, work, nchunks, ps, chunk);
    else
      k_post_mean<FAM, D, 1, 0><<<grid, kWG, 0, st>>>(xt, N, z, n, spec, tbits, hyp, Gk, coeffs, cstride, B, work, nchunks, ps, chunk);
  } else {
    if (FAM == 1 || uniform4)
      k_post_mean<FAM, D, kPmB, 4><<<grid, kWG, 0, st>>>(xt, N, z, n, spec, tbits, hyp, Gk, coeffs, cstride, B, work, nchunks, ps, chunk);
    else
      k_post_mean<FAM, D, kPmB, 0><<<grid, kWG, 0, st>>>(xt, N, z, n, spec, tbits, hyp, Gk, coeffs, cstride, B, work, nchunks, ps, chunk);
  }
}

// The k_post_mean instance post_mean_d launches (for the residency query)
template <int FAM, int D>
static const void* post_mean_kernel(bool uniform4, int B) {
  if (B == 1) return (FAM == 1 || uniform4) ? reinterpret_cast<const void*>(k_post_mean<FAM, D, 1, 4>)
                                            : reinterpret_cast<const void*>(k_post_mean<FAM, D, 1, 0>);
  return (FAM == 1 || uniform4) ? reinterpret_cast<const void*>(k_post_mean<FAM, D, kPmB, 4>)
                                : reinterpret_cast<const void*>(k_post_mean<FAM, D, kPmB, 0>);
}

// Workgroups of a post_mean instance resident at once on the current device (workgroups per CU x CUs), queried
// once per instance and remembered (no query inside a hipGraph capture after the first eager call); 0 if unknown.
static int64_t post_mean_resident(const void* kp) {
  // keyed by (instance, device): devices of one process may differ in CU count / partition mode
  static const void* rk[256];
  static int rdev[256];
  static int64_t rres[256];
  static int nr = 0;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  for (int i = 0; i < nr; ++i)
    if (rk[i] == kp && rdev[i] == dev) return rres[i];
  int per_cu = 0, cus = 0;
  const int64_t res = (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
                       hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kp, kWG, 0) == hipSuccess)
                          ? (int64_t)per_cu * cus : 0;
  if (nr < 256) {
    rk[nr] = kp;
    rdev[nr] = dev;
    rres[nr++] = res;
  }
  return res;
}

// Training points per workgroup of a batched launch: the workgroups of an FP64-VALU-bound launch run in rounds of
// `resident`; with W workgroups the last round is W / resident - floor(W / resident) full, so of the chunks
// {2048, 1024, 512} (whole 256-point slabs; a workgroup's prologue ~1 % of a 512-point chunk) the one whose launch
// fills its rounds best is taken, the larger on a tie (C4: 8 problems x 2^20 points, 5 workgroups per CU:
// 1024 -> 6.4 rounds, 91 % filled; 512 -> 12.8 rounds, 98.5 %).  Unknown residency: kChunk.
template <int FAM>
static int64_t post_mean_chunk(int d, const PredSpec& spec, int64_t n, int64_t N, int64_t P, int B) {
  bool uniform4 = true;
  for (int j = 0; j < d; ++j) uniform4 = uniform4 && spec.order[j] == 4;
  const void* kp = nullptr;
  switch (d) {
#define FGP_C(DD) case DD: kp = post_mean_kernel<FAM, DD>(uniform4, B); break;
    FGP_C(1) FGP_C(2) FGP_C(3) FGP_C(4) FGP_C(5) FGP_C(6) FGP_C(7) FGP_C(8)
#undef FGP_C
    default: return kChunk;
  }
  const int64_t res = post_mean_resident(kp);
  if (res <= 0) return kChunk;
  const int64_t tiles = (N + kWG - 1) / kWG;
  int64_t best = kChunk;
  double best_fill = -1.0;
  for (int64_t c = 2048; c >= 512; c /= 2) {
    const int64_t w = P * tiles * ((n + c - 1) / c);
    const double rounds = (double)w / (double)res;
    const double fill = rounds / std::ceil(rounds);
    if (fill > best_fill + 1e-9) {
      best_fill = fill;
      best = c;
    }
  }
  return best;
}

template <int FAM>
static int launch_post_mean(int d, const double* xt, int64_t N, const void* z, int64_t n, const PredSpec& spec, int tbits,
                            const double* hyp, int Gk, const double* coeffs, int64_t cstride, int B, double* out,
                            int64_t out_stride, double* work, hipStream_t st, int P = 1,
                            ProbStrides ps = ProbStrides{0, 0, 0, 0}, int64_t chunk = kChunk) {
  const int64_t nchunks = (n + chunk - 1) / chunk;
  const dim3 grid((unsigned)nchunks, (unsigned)((N + kWG - 1) / kWG), (unsigned)P);
  bool uniform4 = true;
  for (int j = 0; j < d; ++j) uniform4 = uniform4 && spec.order[j] == 4;
  switch (d) {
#define FGP_C(DD) \
  case DD: post_mean_d<FAM, DD>(grid, st, uniform4, B, xt, N, z, n, spec, tbits, hyp, Gk, coeffs, cstride, work, nchunks, ps, chunk); break;
    FGP_C(1) FGP_C(2) FGP_C(3) FGP_C(4) FGP_C(5) FGP_C(6) FGP_C(7) FGP_C(8)
#undef FGP_C
    default: return set_error(kErrUnsupported, "post_mean: d=%d unsupported", d);
  }
  int rc = check_launch("k_post_mean");
  if (rc != kOk) return rc;
  k_sum_chunks<<<(unsigned)((int64_t)P * B * N), kWG, 0, st>>>(work, nchunks, out, out_stride, N);
  return check_launch("k_sum_chunks");
}

template <int FAM>
static int launch_rows(int d, const double* xt, int64_t N, const void* z, int64_t n, const PredSpec& spec, int tbits,
                       const double* hyp, int Gk, double* rows, hipStream_t st) {
  const dim3 grid((unsigned)((n + kWG - 1) / kWG), (unsigned)N);
  switch (d) {
#define FGP_C(DD) case DD: k_kernel_rows<FAM, DD><<<grid, kWG, 0, st>>>(xt, N, z, n, spec, tbits, hyp, Gk, rows); break;
    FGP_C(1) FGP_C(2) FGP_C(3) FGP_C(4) FGP_C(5) FGP_C(6) FGP_C(7) FGP_C(8)
#undef FGP_C
    default: return set_error(kErrUnsupported, "kernel_rows: d=%d unsupported", d);
  }
  return check_launch("k_kernel_rows");
}

// Lattice: Bernoulli order 2 alpha and coefficient per dimension.  Net: Walsh order alpha per dimension
// (1..4; order = NULL or 0 entries: 1), coefficients unused.
static int make_spec(int family, int d, const int* order, const double* coef, PredSpec& spec) {
  const bool lat = family == FGP_FAMILY_LATTICE;
  for (int j = 0; j < FGP_MAX_D; ++j) {
    if (lat) {
      spec.order[j] = j < d ? order[j] : 0;
      spec.coef[j] = j < d ? coef[j] : 0.0;
      if (j < d && (order[j] < 2 || order[j] > 8 || (order[j] & 1)))
        return set_error(kErrUnsupported, "Bernoulli order %d unsupported", order[j]);
    } else {
      spec.order[j] = (order && j < d && order[j] > 0) ? order[j] : 1;
      spec.coef[j] = 0.0;
      if (spec.order[j] > 4) return set_error(kErrUnsupported, "Walsh order %d unsupported", spec.order[j]);
    }
  }
  return kOk;
}

}  // namespace fgp

using namespace fgp;

extern "C" {

int fgp_post_mean(int family, const double* xt, int64_t N, const void* z, int64_t n, int d, int tbits, const int* order,
                  const double* coef, const double* hyp, int Gk, const double* coeffs, int64_t coeff_stride, int B,
                  double* out, int64_t out_stride, double* work, int64_t chunk, void* stream) {
  if (B > kPmB && Gk == B && N > 0) {
    // every output with its own hyper-parameters (per-output batches, e.g. C5 per-output: 512 outputs): the
    // blocks of kPmB outputs as the problems of ONE launch (blockIdx.z; the arithmetic of one block per launch),
    // the B mod kPmB remaining outputs in a second
    if (N < 0 || n < 1 || d < 1 || d > FGP_MAX_D || chunk < 1 || !xt || !z || !hyp || !coeffs || !out || !work)
      return set_error(kErrInvalid, "fgp_post_mean: bad sizes / null pointer");
    if (out_stride != N) return set_error(kErrInvalid, "fgp_post_mean: B > %d needs out_stride == N", kPmB);
    PredSpec spec;
    int rc = make_spec(family, d, order, coef, spec);
    if (rc != kOk) return rc;
    hipStream_t st = (hipStream_t)stream;
    const int nblk = B / kPmB, rem = B - nblk * kPmB;
    const ProbStrides ps{0, 0, (int64_t)kPmB * (1 + d), (int64_t)kPmB * coeff_stride};
    rc = family == FGP_FAMILY_LATTICE
             ? launch_post_mean<0>(d, xt, N, z, n, spec, tbits, hyp, kPmB, coeffs, coeff_stride, kPmB, out, N, work, st,
                                   nblk, ps, chunk)
             : launch_post_mean<1>(d, xt, N, z, n, spec, tbits, hyp, kPmB, coeffs, coeff_stride, kPmB, out, N, work, st,
                                   nblk, ps, chunk);
    if (rc != kOk || rem == 0) return rc;
    const int b0 = nblk * kPmB;
    return fgp_post_mean(family, xt, N, z, n, d, tbits, order, coef, hyp + (int64_t)b0 * (1 + d), rem,
                         coeffs + (int64_t)b0 * coeff_stride, coeff_stride, rem, out + (int64_t)b0 * N, N, work, chunk,
                         stream);
  }
  if (N < 0 || n < 1 || d < 1 || d > FGP_MAX_D || B < 1 || B > kPmB || Gk < 1 || chunk < 1)
    return set_error(kErrInvalid, "fgp_post_mean: bad sizes (N=%lld n=%lld d=%d B=%d Gk=%d)", (long long)N,
                     (long long)n, d, B, Gk);
  if (N == 0) return kOk;
  if (!xt || !z || !hyp || !coeffs || !out || !work) return set_error(kErrInvalid, "fgp_post_mean: null pointer");
  PredSpec spec;
  int rc = make_spec(family, d, order, coef, spec);
  if (rc != kOk) return rc;
  hipStream_t st = (hipStream_t)stream;
  // chunk = training points per workgroup (work holds ceil(n / chunk) * B * N doubles): small chunks give
  // small problems (n = 2^16, N = 256) enough workgroups to fill the chip
  if (family == FGP_FAMILY_LATTICE)
    return launch_post_mean<0>(d, xt, N, z, n, spec, tbits, hyp, Gk, coeffs, coeff_stride, B, out, out_stride, work, st,
                               1, ProbStrides{0, 0, 0, 0}, chunk);
  return launch_post_mean<1>(d, xt, N, z, n, spec, tbits, hyp, Gk, coeffs, coeff_stride, B, out, out_stride, work, st,
                             1, ProbStrides{0, 0, 0, 0}, chunk);
}

}  // extern "C"

namespace fgp {
// partials per (problem, test point) written by launch_qf: one per column tile of the transform
static int64_t qf_partials(int family, int log2n) {
  const char* r2c_env = getenv("FGP_R2C");
  const bool r2c = family == FGP_FAMILY_LATTICE && log2n >= 17 && !(r2c_env && r2c_env[0] == '0');
  return (int64_t)1 << (log2n - kTileLog - (r2c ? 1 : 0));
}

// quadratic-form partials of P problems x N test points (k_qf_rows + k_qf_cols)
static int launch_qf(int family, const double* xt, int64_t N, const void* z, int log2n, int d, int tbits,
                     const PredSpec& spec, const double* hyp, const double* wa, void* work, double* partial, int64_t P,
                     const ProbStrides& ps, hipStream_t st, const fgp_pred_desc* gdesc = nullptr) {
  const Tables* tb = get_tables(st);
  if (!tb) return set_error(kErrHip, "twiddle table initialisation failed");
  QfArgs q;
  q.log2n = log2n;
  q.d = d;
  q.tbits = tbits;
  q.N = (int)N;
  q.xt = xt;
  q.z = z;
  q.spec = spec;
  q.hyp = hyp;
  q.wa = wa;
  q.work = work;
  q.partial = partial;
  q.ps = ps;
  q.gen = 0;
  q.gshift = nullptr;
  q.gss = 0;
  for (int j = 0; j < FGP_MAX_D; ++j) q.gz[j] = 0u;
  if (gdesc && gdesc->points_gen == FGP_PARTS_LATTICE && family == FGP_FAMILY_LATTICE) {
    const uint64_t zmask = ((uint64_t)1 << log2n) - 1;
    for (int j = 0; j < d; ++j) {
      if (gdesc->gen_z[j] <= 0 || gdesc->gen_z[j] >= ((int64_t)1 << (53 - log2n)))
        return set_error(kErrUnsupported, "generating vector entry %lld outside (0, 2^(53-log2n))",
                         (long long)gdesc->gen_z[j]);
      q.gz[j] = (unsigned)((uint64_t)gdesc->gen_z[j] & zmask);
    }
    if (!gdesc->gen_shift) return set_error(kErrInvalid, "null gen_shift");
    q.gen = 1;
    q.gshift = gdesc->gen_shift;
    q.gss = gdesc->gen_shift_stride;
  }
  int rc;
  const char* r2c_env = getenv("FGP_R2C");
  if (family == FGP_FAMILY_LATTICE && log2n >= 17 && !(r2c_env && r2c_env[0] == '0')) {
    // half-length (R2C) quadratic form: (P N) x (n/2 / 4096) workgroups per pass
    const int mt = log2n - 1, p1 = mt - 12;
    const dim3 grid((unsigned)((P * N) << (mt - kTileLog)));
    bool uniform4 = true;
    for (int j = 0; j < d; ++j) uniform4 = uniform4 && spec.order[j] == 4;
    switch (d) {
#define FGP_C(DD)                                                                          \
  case DD:                                                                                 \
    if (uniform4) k_qf_rows_r2c<DD, 4><<<grid, kWG, 0, st>>>(q, tb->tw4096, tb->twm[mt]);  \
    else k_qf_rows_r2c<DD, 0><<<grid, kWG, 0, st>>>(q, tb->tw4096, tb->twm[mt]);           \
    break;
      FGP_C(1) FGP_C(2) FGP_C(3) FGP_C(4) FGP_C(5) FGP_C(6) FGP_C(7) FGP_C(8)
#undef FGP_C
      default: return set_error(kErrUnsupported, "post_var: d=%d unsupported", d);
    }
    if ((rc = check_launch("k_qf_rows_r2c")) != kOk) return rc;
    switch (p1) {
#define FGP_C(PP) case PP: k_qf_cols_r2c<PP><<<grid, kWG, 0, st>>>(q, tb->tw4096, tb->twm[log2n]); break;
      FGP_C(4) FGP_C(5) FGP_C(6) FGP_C(7) FGP_C(8) FGP_C(9) FGP_C(10) FGP_C(11)
#undef FGP_C
      default: return set_error(kErrInvalid, "bad r2c m1");
    }
    return check_launch("k_qf_cols_r2c");
  }
  const int m2 = split_m2(log2n), m1 = log2n - m2;
  const dim3 grid((unsigned)((P * N) << (log2n - kTileLog)));
  const double2* tw = tb->tw4096;
  const double2* twm = tb->twm[log2n];
  if (family == FGP_FAMILY_LATTICE) {
    switch (m2) {
#define FGP_C(PP) case PP: k_qf_rows<PP, double2><<<grid, kWG, 0, st>>>(q, tw, twm); break;
      FGP_C(9) FGP_C(10) FGP_C(11) FGP_C(12)
#undef FGP_C
    }
  } else {
    switch (m2) {
#define FGP_C(PP) case PP: k_qf_rows<PP, double><<<grid, kWG, 0, st>>>(q, tw, twm); break;
      FGP_C(9) FGP_C(10) FGP_C(11) FGP_C(12)
#undef FGP_C
    }
  }
  if ((rc = check_launch("k_qf_rows")) != kOk) return rc;
  if (family == FGP_FAMILY_LATTICE) {
    switch (m1) {
#define FGP_C(PP) case PP: k_qf_cols<PP, double2><<<grid, kWG, 0, st>>>(q, tw); break;
      FGP_C(4) FGP_C(5) FGP_C(6) FGP_C(7) FGP_C(8) FGP_C(9) FGP_C(10) FGP_C(11) FGP_C(12)
#undef FGP_C
    }
  } else {
    switch (m1) {
#define FGP_C(PP) case PP: k_qf_cols<PP, double><<<grid, kWG, 0, st>>>(q, tw); break;
      FGP_C(4) FGP_C(5) FGP_C(6) FGP_C(7) FGP_C(8) FGP_C(9) FGP_C(10) FGP_C(11) FGP_C(12)
#undef FGP_C
    }
  }
  return check_launch("k_qf_cols");
}
}  // namespace fgp

extern "C" {

int fgp_post_var_qf(int family, const double* xt, int64_t N, const void* z, int log2n, int d, int tbits,
                    const int* order, const double* coef, const double* hyp, const double* wa, void* work,
                    double* partial, double* out, void* stream) {
  if (N < 0 || d < 1 || d > FGP_MAX_D || log2n < 13 || log2n > kMaxLog2N)
    return set_error(kErrInvalid, "fgp_post_var_qf: needs 13 <= log2n <= 24 and 1 <= d <= %d", FGP_MAX_D);
  if (N == 0) return kOk;
  if (!xt || !z || !hyp || !wa || !work || !partial || !out) return set_error(kErrInvalid, "fgp_post_var_qf: null pointer");
  if ((N << (log2n - kTileLog)) >= ((int64_t)1 << 31)) return set_error(kErrUnsupported, "fgp_post_var_qf: N too large");
  PredSpec spec;
  int rc = make_spec(family, d, order, coef, spec);
  if (rc != kOk) return rc;
  hipStream_t st = (hipStream_t)stream;
  rc = launch_qf(family, xt, N, z, log2n, d, tbits, spec, hyp, wa, work, partial, 1, ProbStrides{0, 0, 0, 0}, st);
  if (rc != kOk) return rc;
  k_sum_chunks<<<(unsigned)N, kWG, 0, st>>>(partial, qf_partials(family, log2n), out, N, N);
  return check_launch("k_sum_chunks");
}

int fgp_post_mean_batched(const fgp_pred_desc* pd, const double* xt, int64_t xt_stride, int64_t N, double* out,
                          double* work, void* stream) {
  if (!pd) return set_error(kErrInvalid, "fgp_post_mean_batched: null desc");
  const int d = pd->d;
  if (N < 0 || pd->n < 1 || d < 1 || d > FGP_MAX_D || pd->P < 1 || pd->P > 65535)
    return set_error(kErrInvalid, "fgp_post_mean_batched: bad sizes");
  if (N == 0) return kOk;
  if (!xt || !pd->z || !pd->hyp || !pd->coeffs || !out || !work)
    return set_error(kErrInvalid, "fgp_post_mean_batched: null pointer");
  PredSpec spec;
  int rc = make_spec(pd->family, d, pd->order, pd->coef, spec);
  if (rc != kOk) return rc;
  const ProbStrides ps{xt_stride, pd->z_stride, pd->hyp_stride, pd->coeff_stride};
  hipStream_t st = (hipStream_t)stream;
  if (pd->family == FGP_FAMILY_LATTICE) {
    const int64_t chunk = post_mean_chunk<0>(d, spec, pd->n, N, pd->P, 1);
    return launch_post_mean<0>(d, xt, N, pd->z, pd->n, spec, pd->tbits, pd->hyp, 1, pd->coeffs, pd->n, 1, out, N, work,
                               st, pd->P, ps, chunk);
  }
  const int64_t chunk = post_mean_chunk<1>(d, spec, pd->n, N, pd->P, 1);
  return launch_post_mean<1>(d, xt, N, pd->z, pd->n, spec, pd->tbits, pd->hyp, 1, pd->coeffs, pd->n, 1, out, N, work, st,
                             pd->P, ps, chunk);
}

int fgp_post_mean_batched_work(const fgp_pred_desc* pd, int64_t N, int64_t* work) {
  if (!pd || !work) return set_error(kErrInvalid, "fgp_post_mean_batched_work: null pointer");
  if (N < 0 || pd->n < 1 || pd->d < 1 || pd->d > FGP_MAX_D || pd->P < 1)
    return set_error(kErrInvalid, "fgp_post_mean_batched_work: bad sizes");
  PredSpec spec;
  int rc = make_spec(pd->family, pd->d, pd->order, pd->coef, spec);
  if (rc != kOk) return rc;
  const int64_t chunk = pd->family == FGP_FAMILY_LATTICE ? post_mean_chunk<0>(pd->d, spec, pd->n, N, pd->P, 1)
                                                         : post_mean_chunk<1>(pd->d, spec, pd->n, N, pd->P, 1);
  *work = std::max<int64_t>(1, ((pd->n + chunk - 1) / chunk) * pd->P * N);
  return kOk;
}

int fgp_post_var_batched(const fgp_pred_desc* pd, const double* xt, int64_t xt_stride, int64_t N, const double* part0,
                         double* out, void* work, double* partial, void* stream) {
  if (!pd) return set_error(kErrInvalid, "fgp_post_var_batched: null desc");
  const int d = pd->d;
  int log2n = 0;
  while (((int64_t)1 << log2n) < pd->n) ++log2n;
  if (((int64_t)1 << log2n) != pd->n || N < 0 || d < 1 || d > FGP_MAX_D || log2n < 13 || log2n > kMaxLog2N ||
      pd->P < 1)
    return set_error(kErrInvalid, "fgp_post_var_batched: needs n = 2^m, 13 <= m <= 24, 1 <= d <= %d", FGP_MAX_D);
  if (N == 0) return kOk;
  if (!xt || (!pd->z && pd->points_gen != FGP_PARTS_LATTICE) || !pd->hyp || !pd->wa || !part0 || !out || !work ||
      !partial)
    return set_error(kErrInvalid, "fgp_post_var_batched: null pointer");
  if (((int64_t)pd->P * N << (log2n - kTileLog)) >= ((int64_t)1 << 31))
    return set_error(kErrUnsupported, "fgp_post_var_batched: P * N too large");
  PredSpec spec, p0;
  int rc = make_spec(pd->family, d, pd->order, pd->coef, spec);
  if (rc != kOk) return rc;
  for (int j = 0; j < FGP_MAX_D; ++j) {
    p0.order[j] = 0;
    p0.coef[j] = j < d ? part0[j] : 0.0;
  }
  hipStream_t st = (hipStream_t)stream;
  rc = launch_qf(pd->family, xt, N, pd->z, log2n, d, pd->tbits, spec, pd->hyp, pd->wa, work, partial, pd->P,
                 ProbStrides{xt_stride, pd->z_stride, pd->hyp_stride, pd->wa_stride}, st, pd);
  if (rc != kOk) return rc;
  k_qf_finish<<<(unsigned)((int64_t)pd->P * N), kWG, 0, st>>>(partial, qf_partials(pd->family, log2n), pd->hyp,
                                                               pd->hyp_stride, p0, d, N, out);
  return check_launch("k_qf_finish");
}

int fgp_inv_eig(int family, const void* lam, const void* ytilde, int64_t yt_stride, const double* raw_noise,
                int64_t noise_stride, int64_t P, int log2n, void* ya, double* wa, void* stream) {
  if (P < 1 || log2n < 0 || log2n > kMaxLog2N) return set_error(kErrInvalid, "fgp_inv_eig: bad sizes");
  if (!lam || !ytilde || !raw_noise || !ya) return set_error(kErrInvalid, "fgp_inv_eig: null pointer");
  const int64_t total = P << log2n;
  const double rootn = sqrt((double)((int64_t)1 << log2n));
  hipStream_t st = (hipStream_t)stream;
  const unsigned grid = (unsigned)((total + kWG - 1) / kWG);
  if (family == FGP_FAMILY_LATTICE)
    k_inv_eig<double2><<<grid, kWG, 0, st>>>(static_cast<const double2*>(lam), static_cast<const double2*>(ytilde),
                                              yt_stride, raw_noise, noise_stride, rootn, log2n, total,
                                              static_cast<double2*>(ya), wa);
  else
    k_inv_eig<double><<<grid, kWG, 0, st>>>(static_cast<const double*>(lam), static_cast<const double*>(ytilde),
                                             yt_stride, raw_noise, noise_stride, rootn, log2n, total,
                                             static_cast<double*>(ya), wa);
  return check_launch("k_inv_eig");
}

int fgp_kernel_rows(int family, const double* xt, int64_t N, const void* z, int64_t n, int d, int tbits,
                    const int* order, const double* coef, const double* hyp, int Gk, double* rows, void* stream) {
  if (N < 0 || n < 1 || d < 1 || d > FGP_MAX_D || Gk < 1 || N > 65535)
    return set_error(kErrInvalid, "fgp_kernel_rows: bad sizes");
  if (N == 0) return kOk;
  if (!xt || !z || !hyp || !rows) return set_error(kErrInvalid, "fgp_kernel_rows: null pointer");
  PredSpec spec;
  int rc = make_spec(family, d, order, coef, spec);
  if (rc != kOk) return rc;
  hipStream_t st = (hipStream_t)stream;
  if (family == FGP_FAMILY_LATTICE) return launch_rows<0>(d, xt, N, z, n, spec, tbits, hyp, Gk, rows, st);
  return launch_rows<1>(d, xt, N, z, n, spec, tbits, hyp, Gk, rows, st);
}

}  // extern "C"
