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

struct PredSpec {
  int order[FGP_MAX_D];
  double coef[FGP_MAX_D];
};

__device__ __forceinline__ double bern(int order, double x) {
  switch (order) {
    case 2: return (x - 1.0) * x + 1.0 / 6.0;
    case 4: return (((x - 2.0) * x + 1.0) * x + 0.0) * x - 1.0 / 30.0;
    case 6: return (((((x - 3.0) * x + 5.0 / 2.0) * x + 0.0) * x - 1.0 / 2.0) * x + 0.0) * x + 1.0 / 42.0;
    default:
      return (((((((x - 4.0) * x + 14.0 / 3.0) * x + 0.0) * x - 7.0 / 3.0) * x + 0.0) * x + 2.0 / 3.0) * x + 0.0) * x -
             1.0 / 30.0;
  }
}

// (x - z) % 1 for x, z in [0, 1] (torch.remainder semantics on that domain)
__device__ __forceinline__ double mod1_unit(double v) { return v < 0.0 ? v + 1.0 : (v >= 1.0 ? v - 1.0 : v); }

__device__ __forceinline__ double walsh_part(unsigned long long delta, int t) {
  if (delta == 0ull) return 6.0 * (1.0 / 6.0 - 0.0);
  const int fl = 63 - __clzll((long long)delta);
  return 6.0 * (1.0 / 6.0 - ldexp(1.0, fl - t - 1));
}

// FAM 0: lattice (z = float points [d][n]); FAM 1: net (z = int64 points [d][n])
template <int FAM, int D>
__global__ __launch_bounds__(kWG) void k_post_mean(const double* __restrict__ xt, int64_t N, const void* __restrict__ z,
                                                    int64_t n, int64_t chunk, PredSpec spec, int tbits,
                                                    const double* __restrict__ hyp, int Gk, const double* __restrict__ coeffs,
                                                    int64_t coeff_stride, int B, double* __restrict__ partial) {
  __shared__ double zs[D][kSlab];
  __shared__ double cs[kPmB][kSlab];
  const int tid = threadIdx.x;
  const int64_t t = (int64_t)blockIdx.y * kWG + tid;
  const bool live = t < N;
  // test point in registers
  double xv[D];
  unsigned long long xbv[D];
#pragma unroll
  for (int j = 0; j < D; ++j) {
    const double v = live ? xt[t * D + j] : 0.0;
    xv[j] = v;
    if constexpr (FAM == 1) {
      double r = fmod(v, 1.0);
      if (r != 0.0 && r < 0.0) r += 1.0;
      xbv[j] = (unsigned long long)(long long)floor(r * ldexp(1.0, tbits));
    }
  }
  double sc[kPmB], ls[kPmB][D];
#pragma unroll
  for (int b = 0; b < kPmB; ++b) {
    const int g = b < B ? b % Gk : 0;
    sc[b] = hyp[g * (1 + D)];
#pragma unroll
    for (int j = 0; j < D; ++j) ls[b][j] = hyp[g * (1 + D) + 1 + j];
  }
  double acc[kPmB];
#pragma unroll
  for (int b = 0; b < kPmB; ++b) acc[b] = 0.0;
  const int64_t i0 = (int64_t)blockIdx.x * chunk;
  const int64_t i1 = i0 + chunk < n ? i0 + chunk : n;
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
      for (int b = 0; b < kPmB; ++b) cs[b][tid] = b < B ? coeffs[(int64_t)b * coeff_stride + s0 + tid] : 0.0;
    }
    __syncthreads();
    for (int i = 0; i < cnt; ++i) {
      double part[D];
#pragma unroll
      for (int j = 0; j < D; ++j) {
        if constexpr (FAM == 0) {
          part[j] = spec.coef[j] * bern(spec.order[j], mod1_unit(xv[j] - zs[j][i]));
        } else {
          const unsigned long long zb = (unsigned long long)__double_as_longlong(zs[j][i]);
          part[j] = walsh_part(xbv[j] ^ zb, tbits);
        }
      }
#pragma unroll
      for (int b = 0; b < kPmB; ++b) {
        if (b < B) {
          double p = 1.0;
#pragma unroll
          for (int j = 0; j < D; ++j) p *= 1.0 + ls[b][j] * part[j];
          acc[b] += (sc[b] * p) * cs[b][i];
        }
      }
    }
  }
  if (live) {
#pragma unroll
    for (int b = 0; b < kPmB; ++b)
      if (b < B) partial[((int64_t)blockIdx.x * B + b) * N + t] = acc[b];
  }
}

__global__ __launch_bounds__(kWG) void k_sum_chunks(const double* __restrict__ partial, int64_t nchunks, int64_t len,
                                                     double* __restrict__ out, int64_t out_stride, int B, int64_t N) {
  const int64_t e = (int64_t)blockIdx.x * kWG + threadIdx.x;
  if (e >= len) return;
  double s = 0.0;
  for (int64_t c = 0; c < nchunks; ++c) s += partial[c * len + e];
  const int64_t b = e / N, t = e % N;
  out[b * out_stride + t] = s;
}

// kernel rows: rows[g, t, i] = K_g(x_t, z_i) for g < Gk (the [N, n] matrix the reference builds for
// post_var / post_cov, abstract_gp.py:407-411,452-457)
template <int FAM, int D>
__global__ __launch_bounds__(kWG) void k_kernel_rows(const double* __restrict__ xt, int64_t N, const void* __restrict__ z,
                                                      int64_t n, PredSpec spec, int tbits, const double* __restrict__ hyp,
                                                      int Gk, double* __restrict__ rows) {
  const int64_t i = (int64_t)blockIdx.x * kWG + threadIdx.x;
  const int64_t t = blockIdx.y;
  if (i >= n) return;
  double part[D];
#pragma unroll
  for (int j = 0; j < D; ++j) {
    const double v = xt[t * D + j];
    if constexpr (FAM == 0) {
      part[j] = spec.coef[j] * bern(spec.order[j], mod1_unit(v - static_cast<const double*>(z)[(int64_t)j * n + i]));
    } else {
      double r = fmod(v, 1.0);
      if (r != 0.0 && r < 0.0) r += 1.0;
      const unsigned long long xb = (unsigned long long)(long long)floor(r * ldexp(1.0, tbits));
      const unsigned long long zb = (unsigned long long)static_cast<const long long*>(z)[(int64_t)j * n + i];
      part[j] = walsh_part(xb ^ zb, tbits);
    }
  }
  for (int g = 0; g < Gk; ++g) {
    double p = 1.0;
#pragma unroll
    for (int j = 0; j < D; ++j) p *= 1.0 + hyp[g * (1 + D) + 1 + j] * part[j];
    rows[((int64_t)g * N + t) * n + i] = hyp[g * (1 + D)] * p;
  }
}

template <int FAM>
static int launch_post_mean(int d, const double* xt, int64_t N, const void* z, int64_t n, const PredSpec& spec, int tbits,
                            const double* hyp, int Gk, const double* coeffs, int64_t cstride, int B, double* out,
                            int64_t out_stride, double* work, int64_t chunk, hipStream_t st) {
  const int64_t nchunks = (n + chunk - 1) / chunk;
  const dim3 grid((unsigned)nchunks, (unsigned)((N + kWG - 1) / kWG));
  switch (d) {
#define FGP_C(DD)                                                                                                   \
  case DD:                                                                                                          \
    k_post_mean<FAM, DD><<<grid, kWG, 0, st>>>(xt, N, z, n, chunk, spec, tbits, hyp, Gk, coeffs, cstride, B, work); \
    break;
    FGP_C(1) FGP_C(2) FGP_C(3) FGP_C(4) FGP_C(5) FGP_C(6) FGP_C(7) FGP_C(8)
#undef FGP_C
    default: return set_error(kErrUnsupported, "post_mean: d=%d unsupported", d);
  }
  int rc = check_launch("k_post_mean");
  if (rc != kOk) return rc;
  const int64_t len = (int64_t)B * N;
  k_sum_chunks<<<(unsigned)((len + kWG - 1) / kWG), kWG, 0, st>>>(work, nchunks, len, out, out_stride, B, N);
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
  if (family == FGP_FAMILY_LATTICE)
    return launch_post_mean<0>(d, xt, N, z, n, spec, tbits, hyp, Gk, coeffs, coeff_stride, B, out, out_stride, work,
                               chunk, st);
  return launch_post_mean<1>(d, xt, N, z, n, spec, tbits, hyp, Gk, coeffs, coeff_stride, B, out, out_stride, work, chunk,
                             st);
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
