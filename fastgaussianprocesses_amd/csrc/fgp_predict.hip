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

#include "fgp_common.h"
#include "fgp_runtime.h"
#include "../../include/fgp_hip.h"

namespace fgp {

constexpr int kPmB = 4;          // outputs per launch
constexpr int kSlab = 256;       // train points per LDS slab
constexpr int kChunk = 1024;     // train points per workgroup (4 slabs)

struct PredSpec {
  int order[FGP_MAX_D];
  double coef[FGP_MAX_D];
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
                                                    double* __restrict__ partial, int64_t nchunks) {
  __shared__ double zs[D][kSlab];
  __shared__ double cs[NB][kSlab];
  const int tid = threadIdx.x;
  const int64_t t = (int64_t)blockIdx.y * kWG + tid;
  const bool live = t < N;
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
        fa[b][j] = 1.0 + l;   // c1
        fc[b][j] = 3.0 * l;   // c3
      }
    }
  }
  double acc[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) acc[b] = 0.0;
  const int64_t i0 = (int64_t)blockIdx.x * kChunk;
  const int64_t i1 = i0 + kChunk < n ? i0 + kChunk : n;
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
#pragma unroll 2
    for (int i = 0; i < cnt; ++i) {
      double p[NB];
#pragma unroll
      for (int b = 0; b < NB; ++b) p[b] = 1.0;
#pragma unroll
      for (int j = 0; j < D; ++j) {
        if constexpr (FAM == 0) {
          const double tj = fabs(xv[j] - zs[j][i]);
          const int ord = ORD ? ORD : spec.order[j];
#pragma unroll
          for (int b = 0; b < NB; ++b) p[b] *= lat_factor(ord, tj, fa[b][j], fc[b][j]);
        } else {
          const unsigned long long delta = xbv[j] ^ (unsigned long long)__double_as_longlong(zs[j][i]);
#pragma unroll
          for (int b = 0; b < NB; ++b) p[b] *= net_factor(delta, tbits, fa[b][j], fc[b][j]);
        }
      }
#pragma unroll
      for (int b = 0; b < NB; ++b) acc[b] = fma(p[b], cs[b][i], acc[b]);
    }
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
        p *= net_factor(dv[j], tbits, 1.0 + l, 3.0 * l);
      }
    }
    rows[((int64_t)g * N + t) * n + i] = hyp[g * (1 + D)] * p;
  }
}

template <int FAM, int D>
static void post_mean_d(dim3 grid, hipStream_t st, bool uniform4, int B, const double* xt, int64_t N, const void* z,
                        int64_t n, const PredSpec& spec, int tbits, const double* hyp, int Gk, const double* coeffs,
                        int64_t cstride, double* work, int64_t nchunks) {
  if (B == 1) {
    if (FAM == 1 || uniform4)
      k_post_mean<FAM, D, 1, 4><<<grid, kWG, 0, st>>>(xt, N, z, n, spec, tbits, hyp, Gk, coeffs, cstride, B, work, nchunks);
    else
      k_post_mean<FAM, D, 1, 0><<<grid, kWG, 0, st>>>(xt, N, z, n, spec, tbits, hyp, Gk, coeffs, cstride, B, work, nchunks);
  } else {
    if (FAM == 1 || uniform4)
      k_post_mean<FAM, D, kPmB, 4><<<grid, kWG, 0, st>>>(xt, N, z, n, spec, tbits, hyp, Gk, coeffs, cstride, B, work, nchunks);
    else
      k_post_mean<FAM, D, kPmB, 0><<<grid, kWG, 0, st>>>(xt, N, z, n, spec, tbits, hyp, Gk, coeffs, cstride, B, work, nchunks);
  }
}

template <int FAM>
static int launch_post_mean(int d, const double* xt, int64_t N, const void* z, int64_t n, const PredSpec& spec, int tbits,
                            const double* hyp, int Gk, const double* coeffs, int64_t cstride, int B, double* out,
                            int64_t out_stride, double* work, hipStream_t st) {
  const int64_t nchunks = (n + kChunk - 1) / kChunk;
  const dim3 grid((unsigned)nchunks, (unsigned)((N + kWG - 1) / kWG));
  bool uniform4 = true;
  for (int j = 0; j < d; ++j) uniform4 = uniform4 && spec.order[j] == 4;
  switch (d) {
#define FGP_C(DD) \
  case DD: post_mean_d<FAM, DD>(grid, st, uniform4, B, xt, N, z, n, spec, tbits, hyp, Gk, coeffs, cstride, work, nchunks); break;
    FGP_C(1) FGP_C(2) FGP_C(3) FGP_C(4) FGP_C(5) FGP_C(6) FGP_C(7) FGP_C(8)
#undef FGP_C
    default: return set_error(kErrUnsupported, "post_mean: d=%d unsupported", d);
  }
  int rc = check_launch("k_post_mean");
  if (rc != kOk) return rc;
  k_sum_chunks<<<(unsigned)((int64_t)B * N), kWG, 0, st>>>(work, nchunks, out, out_stride, N);
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

static int make_spec(int family, int d, const int* order, const double* coef, PredSpec& spec) {
  for (int j = 0; j < FGP_MAX_D; ++j) {
    spec.order[j] = (family == FGP_FAMILY_LATTICE && j < d) ? order[j] : 0;
    spec.coef[j] = (family == FGP_FAMILY_LATTICE && j < d) ? coef[j] : 0.0;
    if (family == FGP_FAMILY_LATTICE && j < d && (order[j] < 2 || order[j] > 8 || (order[j] & 1)))
      return set_error(kErrUnsupported, "Bernoulli order %d unsupported", order[j]);
  }
  return kOk;
}

}  // namespace fgp

using namespace fgp;

extern "C" {

int fgp_post_mean(int family, const double* xt, int64_t N, const void* z, int64_t n, int d, int tbits, const int* order,
                  const double* coef, const double* hyp, int Gk, const double* coeffs, int64_t coeff_stride, int B,
                  double* out, int64_t out_stride, double* work, int64_t chunk, void* stream) {
  if (N < 0 || n < 1 || d < 1 || d > FGP_MAX_D || B < 1 || B > kPmB || Gk < 1 || chunk < 1)
    return set_error(kErrInvalid, "fgp_post_mean: bad sizes (N=%lld n=%lld d=%d B=%d Gk=%d)", (long long)N,
                     (long long)n, d, B, Gk);
  if (N == 0) return kOk;
  if (!xt || !z || !hyp || !coeffs || !out || !work) return set_error(kErrInvalid, "fgp_post_mean: null pointer");
  PredSpec spec;
  int rc = make_spec(family, d, order, coef, spec);
  if (rc != kOk) return rc;
  hipStream_t st = (hipStream_t)stream;
  (void)chunk;   // fixed at kChunk; work must hold ceil(n / 1024) * B * N doubles
  if (family == FGP_FAMILY_LATTICE)
    return launch_post_mean<0>(d, xt, N, z, n, spec, tbits, hyp, Gk, coeffs, coeff_stride, B, out, out_stride, work, st);
  return launch_post_mean<1>(d, xt, N, z, n, spec, tbits, hyp, Gk, coeffs, coeff_stride, B, out, out_stride, work, st);
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
