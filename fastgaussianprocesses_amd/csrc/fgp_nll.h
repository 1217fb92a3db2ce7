// Shared declarations of the fused fit kernels (fgp_nll.hip, fgp_nll_re.hip): the launch descriptor,
// hyper-parameter / kernel-part helpers, eigenvalue terms and the intermediate layout.
#pragma once
#include <cmath>
#include <cstdlib>
#include <type_traits>

#include "fgp_common.h"
#include "fgp_runtime.h"
#include "../../include/fgp_hip.h"

namespace fgp {

// an A/B switch of the host code: the environment variable is set and starts with '0'
inline bool getenv_off(const char* name) {
  const char* e = std::getenv(name);
  return e && e[0] == '0';
}

struct Nll {
  int log2n, d, G, nb, nq;
  const double* parts;
  int64_t parts_stride;
  const double* ysq;
  int64_t ysq_stride;
  const double* raw;
  int scale_off, scale_pp, ls_off, ls_pp, ls_pd, noise_off, noise_pp;
  double logdet_weight;
  void* grad_lam;
  void* work;
  double* partials;
  // lattice parts generator (FGP_PARTS_LATTICE); pg = its Bernoulli order (0: parts array)
  int pgen, pg;
  int gorder[FGP_MAX_D];
  double gcoef[FGP_MAX_D];
  unsigned gz[FGP_MAX_D];        // z_j mod n
  const double* gshift;
  int64_t gshift_stride;
  int r2c;                       // lattice, n >= 2^17: half-length (R2C) fit kernels
  int re;                        // ... with regenerated parts: real-even (RE) fit kernels (default)
  unsigned long long* stamps;    // optional device-clock timing of the launch (fgp_nll_desc.stamps)
  // spectral path (fgp_spectral.hip, ABI 11): part-product spectra [G?][2^d][spec_K]
  const double* basis;
  int64_t basis_stride;
  int spec, spec_net;            // spectral fit path (basis != NULL); nets (weight 1, K = n)
  int64_t spec_K, spec_KS, spec_main;  // frequencies per spectrum, 64 x its chunks, frequencies in k blocks
  int spec_kpl, spec_ppw, spec_pg;   // frequencies per lane and block, problems per wave, problem groups
  int spec_tile, spec_pgp, spec_ck;  // LDS-tiled kernel: problem-group slots, frequencies per chunk
  int64_t spec_kw;                   // ... and per workgroup
  int spec_ps, spec_nsl;             // ... over problem slices: problems per slice, slices (1: none)
  int ysq_chunked;                   // ysq in the chunked layout [k / 64][G][64] (spectral path)
  // multitask spectral fit (ABI 12, fgp_spectral.hip k_mt_spec_iter): T tasks (0: off), pair spectra,
  // ytilde, task kernel; mt_F frequencies per chunk, mt_cpb chunks per block
  int mt, mt_F, mt_cpb;
  const void* mt_basis;
  const void* mt_ytilde;
  const double* mt_kt;
  // ... a learned task kernel (ABI 18, GCV / CV): bit 0 / 1 = the factor / task noise require grad (0: mt_kt is the
  // fixed task kernel); F [T][mt_rank] at raw[mt_f_off], the task noise [T] at raw[mt_v_off] (exp when mt_vexp)
  int mt_learn, mt_rank, mt_vexp, mt_f_off, mt_v_off;
  int64_t out_stride;                // fgp_fftbr_real_half: row stride of the half spectra (grad_lam)
  int loss;                          // FGP_LOSS_MLL / GCV / CV (ABI 16; GCV / CV: k_spec_loss_iter + k_spec_loss_step)
  double cv_weight;
};

// Device-clock kernel timing (fgp_nll_desc.stamps; off when NULL -- a uniform branch on a kernel
// argument): plain vector stores of the wall clock into the launch's record [gridDim.x][1 + kWG/64]:
// [b][0] = start of workgroup b (its first wave), [b][1 + w] = end of its wave w.  No atomics (one
// contended address serialises thousands of them and slows the kernel being timed).
constexpr int kStampStride = 1 + kWG / 64;
__device__ __forceinline__ void stamp_begin(const Nll& a) {
#ifdef FGP_EXP_HWID
  // (experiment build, tools/build_exp.sh: the start stamp carries where the workgroup runs -- XCC_ID in bits
  // 56-63, HW_ID's se / sh / cu fields (bits 8-15) in bits 48-55; the clock stays below 2^48)
  if (a.stamps && threadIdx.x == 0) {
    const unsigned hw = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));       // HW_REG_HW_ID
    const unsigned xcc = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (15 << 11));     // HW_REG_XCC_ID
    a.stamps[(int64_t)blockIdx.x * kStampStride] = (unsigned long long)wall_clock64() |
        ((unsigned long long)((hw >> 8) & 0xFF) << 48) | ((unsigned long long)(xcc & 0xFF) << 56);
  }
#else
  if (a.stamps && threadIdx.x == 0) a.stamps[(int64_t)blockIdx.x * kStampStride] = (unsigned long long)wall_clock64();
#endif
}
__device__ __forceinline__ void stamp_end(const Nll& a) {
  if (a.stamps && (threadIdx.x & 63) == 0)
    a.stamps[(int64_t)blockIdx.x * kStampStride + 1 + (threadIdx.x >> 6)] = (unsigned long long)wall_clock64();
}

// threadIdx.x behind an opaque asm: values derived from it cannot be hoisted out of the loop around the call
// site (in the persistent k_spec_tile, the reduction / step addresses of every iteration would otherwise be
// computed once before the iteration loop and held in VGPRs through its chunk loop)
__device__ __forceinline__ int tid_fresh() {
  int t = (int)threadIdx.x;
  asm volatile("" : "+v"(t));
  return t;
}

struct Hyp {
  double scale, noise;
  double ls[FGP_MAX_D];
};

__device__ __forceinline__ void load_hyp(const Nll& a, int g, Hyp& h) {
  h.scale = exp(a.raw[a.scale_off + (a.scale_pp ? g : 0)]);
  h.noise = exp(a.raw[a.noise_off + (a.noise_pp ? g : 0)]);
  const int lb = a.ls_off + (a.ls_pp ? g : 0) * (a.ls_pd ? a.d : 1);
#pragma unroll
  for (int j = 0; j < FGP_MAX_D; ++j) h.ls[j] = (j < a.d) ? exp(a.raw[lb + (a.ls_pd ? j : 0)]) : 0.0;
}

__device__ __forceinline__ double read_lane(double v, int lane) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
  return __hiloint2double(hi, lo);
}

// load_hyp for a problem index g that is uniform over the wave: one exp per parameter, evaluated
// lane-parallel (lane 0 scale, 1 noise, 2 + j lengthscale j) and broadcast, instead of 2 + d
// exps in every lane.  Same libm exp, so the same values as load_hyp.
// hyper-parameters of problem g from the raw vector `raw` (a.raw, or an LDS copy of the parameters a fused
// launch has just stepped): exp per lane, broadcast by v_readlane
__device__ __forceinline__ void load_hyp_wave(const Nll& a, int g, Hyp& h, const double* raw) {
  const int lane = threadIdx.x & 63;
  const int lb = a.ls_off + (a.ls_pp ? g : 0) * (a.ls_pd ? a.d : 1);
  int idx = -1;
  if (lane == 0) idx = a.scale_off + (a.scale_pp ? g : 0);
  else if (lane == 1) idx = a.noise_off + (a.noise_pp ? g : 0);
  else if (lane < 2 + a.d) idx = lb + (a.ls_pd ? lane - 2 : 0);
  const double e = exp(idx >= 0 ? raw[idx] : 0.0);
  h.scale = read_lane(e, 0);
  h.noise = read_lane(e, 1);
#pragma unroll
  for (int j = 0; j < FGP_MAX_D; ++j) h.ls[j] = (j < a.d) ? read_lane(e, 2 + j) : 0.0;
}
__device__ __forceinline__ void load_hyp_wave(const Nll& a, int g, Hyp& h) { load_hyp_wave(a, g, h, a.raw); }

// ------------------------------------------------------------------ parts source (array / generated)
// Per-problem source of the kernel parts: the parts array, or (FGP_PARTS_LATTICE) the lattice point
// x_0 = shift from which the parts of element i are regenerated with fgp_lattice_parts' arithmetic.
struct PSrc {
  const double* pg;
  double sh[FGP_MAX_D];
};

__device__ __forceinline__ void psrc_init(const Nll& a, int g, PSrc& s) {
  s.pg = a.parts + (int64_t)g * a.parts_stride;
#pragma unroll
  for (int j = 0; j < FGP_MAX_D; ++j)
    s.sh[j] = (a.pgen && j < a.d) ? a.gshift[(int64_t)g * a.gshift_stride + j] : 0.0;   // (x_0 = shift)
}

// Lattice part at the natural-order point with bit-reversed index br (dimension with generating
// vector entry zj mod n): the first-column distance is
//   delta = (x_i - x_0) mod 1 = (brev_m(i) z_j mod n) / n      EXACTLY (k / n with k < n = 2^m),
// so it is formed from k directly -- one conversion and one exact scaling -- instead of from the two
// rounded coordinates the host generator produces (x = (k / n + shift) % 1, then torch.remainder(x -
// x_0, 1), the reference's op sequence, fast_gp_lattice.py:263-266).  The two differ by the rounding of
// x (|d delta| <= 2^-53); the exact one is the better approximation of the kernel's argument and costs
// 2 VALU per dimension instead of 6.  The coefficient (-1)^(alpha+1) (2 pi)^(2 alpha) / (2 alpha)! is
// folded into the lengthscale (fold_gen_coef): the fit kernels see part = B_ORD(delta) and l_j coef_j.
template <int ORD>
__device__ __forceinline__ double lattice_gen_part_k(unsigned k, double inv_n) {
  return bernoulli(ORD, (double)k * inv_n);
}

template <int ORD>
__device__ __forceinline__ double lattice_gen_part(unsigned zj, unsigned br, unsigned mask, double inv_n) {
  return lattice_gen_part_k<ORD>(mul_u24(br, zj) & mask, inv_n);
}

template <int ORD>
__device__ __forceinline__ double gen_part(const Nll& a, const PSrc&, int j, unsigned br, unsigned mask,
                                           double inv_n) {
  return lattice_gen_part<ORD>(a.gz[j], br, mask, inv_n);
}

// Generated parts carry no coefficient: fold coef_j into l_j once per thread (k1 factors 1 + (l_j coef_j)
// B_j; the gradient factor scale l_j of grad_factor() then includes coef_j as well).
template <int PG>
__device__ __forceinline__ void fold_gen_coef(const Nll& a, Hyp& h) {
  if constexpr (PG != 0) {
#pragma unroll
    for (int j = 0; j < FGP_MAX_D; ++j) h.ls[j] *= a.gcoef[j];
  }
}

// Dimension count as a compile-time constant (D = 1..8), or D = 0: runtime d, loops run over
// FGP_MAX_D zero-padded dimensions (part 0 and lengthscale 0, so a padded factor 1 + l p is exactly 1).
template <int D> struct Dims { static constexpr int N = D ? D : FGP_MAX_D; };
template <int D> __device__ __forceinline__ bool dim_on(const Nll& a, int j) { return D ? true : j < a.d; }

// Parts source as a compile-time choice: PG = 0 reads the parts array, PG = 2/4/6/8 regenerates the
// lattice parts with Bernoulli order PG (FGP_PARTS_LATTICE, one order for every dimension).
// parts of element i (p[j], zero-padded)
template <int PG, int D>
__device__ __forceinline__ void parts_one(const Nll& a, const PSrc& s, int64_t n, int64_t i, double* p) {
  if constexpr (PG != 0) {
    const int m = a.log2n;
    const unsigned br = brev_bits((unsigned)i, m), mask = (unsigned)(n - 1);
    const double inv_n = ldexp(1.0, -m);
#pragma unroll
    for (int j = 0; j < Dims<D>::N; ++j) p[j] = dim_on<D>(a, j) ? gen_part<PG>(a, s, j, br, mask, inv_n) : 0.0;
  } else {
#pragma unroll
    for (int j = 0; j < Dims<D>::N; ++j) p[j] = dim_on<D>(a, j) ? s.pg[(int64_t)j * n + i] : 0.0;
  }
}

// parts of the consecutive elements (i, i+1), i even: 16-byte loads, or generated (brev_m(i + 1) =
// brev_m(i) + n/2)
template <int PG, int D>
__device__ __forceinline__ void parts_pair(const Nll& a, const PSrc& s, int64_t n, int64_t i, double* p0,
                                           double* p1) {
  if constexpr (PG != 0) {
    const int m = a.log2n;
    const unsigned br = brev_bits((unsigned)i, m), mask = (unsigned)(n - 1);
    const unsigned br1 = br + (unsigned)(n >> 1);
    const double inv_n = ldexp(1.0, -m);
#pragma unroll
    for (int j = 0; j < Dims<D>::N; ++j) {
      p0[j] = dim_on<D>(a, j) ? gen_part<PG>(a, s, j, br, mask, inv_n) : 0.0;
      p1[j] = dim_on<D>(a, j) ? gen_part<PG>(a, s, j, br1, mask, inv_n) : 0.0;
    }
  } else {
#pragma unroll
    for (int j = 0; j < Dims<D>::N; ++j) {
      double2 pv = make_double2(0.0, 0.0);
      if (dim_on<D>(a, j)) pv = *reinterpret_cast<const double2*>(s.pg + (int64_t)j * n + i);
      p0[j] = pv.x;
      p1[j] = pv.y;
    }
  }
}

// k1 = scale prod_j (1 + l_j p_j); padded dimensions multiply by exactly 1
template <int D>
__device__ __forceinline__ double k1_from(const Hyp& h, const double* p) {
  double r = 1.0;
#pragma unroll
  for (int j = 0; j < Dims<D>::N; ++j) r *= __builtin_fma(h.ls[j], p[j], 1.0);
  return h.scale * r;
}

// k1 at the consecutive elements (i, i+1), i even
template <int PG, int D>
__device__ __forceinline__ double2 k1_pair(const Nll& a, const Hyp& h, const PSrc& s, int64_t n, int64_t i) {
  if constexpr (PG == 0) {   // product accumulated as each dimension's 16-byte load arrives
    double r0 = 1.0, r1 = 1.0;
#pragma unroll
    for (int j = 0; j < Dims<D>::N; ++j) {
      if (dim_on<D>(a, j)) {
        const double2 pv = *reinterpret_cast<const double2*>(s.pg + (int64_t)j * n + i);
        r0 *= __builtin_fma(h.ls[j], pv.x, 1.0);
        r1 *= __builtin_fma(h.ls[j], pv.y, 1.0);
      }
    }
    return make_double2(h.scale * r0, h.scale * r1);
  } else {
    double p0[Dims<D>::N], p1[Dims<D>::N];
    parts_pair<PG, D>(a, s, n, i, p0, p1);
    return make_double2(k1_from<D>(h, p0), k1_from<D>(h, p1));
  }
}

// Gradient terms at element i with dL/dk1_i = g:
//   acc[0]   += g prod_m f_m                      (x scale after the reduction  = dL/draw_scale)
//   acc[1+j] += (g p_j) prod_{m != j} f_m        (x scale l_j after the reduction = dL/draw_l_j)
// f_m = 1 + l_m p_m (prefix / suffix products; padded dimensions contribute f = 1, p = 0).
template <int D>
__device__ __forceinline__ void grad_terms_p(const Hyp& h, const double* pj, double gi, double* acc) {
  constexpr int ND = Dims<D>::N;
  double f[ND];
#pragma unroll
  for (int j = 0; j < ND; ++j) f[j] = __builtin_fma(h.ls[j], pj[j], 1.0);
  double suf[ND + 1];
  suf[ND] = 1.0;
#pragma unroll
  for (int j = ND - 1; j >= 0; --j) suf[j] = suf[j + 1] * f[j];
  acc[0] = __builtin_fma(gi, suf[0], acc[0]);
  double pre = 1.0;
#pragma unroll
  for (int j = 0; j < ND; ++j) {
    acc[1 + j] = __builtin_fma(gi * pj[j], pre * suf[j + 1], acc[1 + j]);
    pre *= f[j];
  }
}

// brev_m(i0 + t) for i0 a multiple of 16: brev_m(i0) | brev_4(t) << (m - 4)
template <int T4>
__device__ __forceinline__ unsigned brev_run(unsigned br0, int m) { return br0 | (Brev4<T4>::value << (m - 4)); }

__device__ __forceinline__ double re(double2 v) { return v.x; }
__device__ __forceinline__ double re(double v) { return v; }
template <typename T> __device__ __forceinline__ T real_to_T(double v);
template <> __device__ __forceinline__ double2 real_to_T<double2>(double v) { return make_double2(v, 0.0); }
template <> __device__ __forceinline__ double real_to_T<double>(double v) { return v; }

// k1 at the 16 consecutive elements i0 + t (i0 a multiple of 16) into v[t]; sum accumulates them in
// order t.  Generated parts, or the parts array read as 16-byte pairs.
template <int PG, int D, typename T>
__device__ __forceinline__ void k1_run16(const Nll& a, const Hyp& h, const PSrc& s, int64_t n, int64_t i0, T* v,
                                         double& sum) {
  double r[16];
  if constexpr (PG != 0) {
    const int m = a.log2n;
    const unsigned br0 = brev_bits((unsigned)i0, m), mask = (unsigned)(n - 1);
    const double inv_n = ldexp(1.0, -m);
    static_for<0, 16>([&](auto tc) {
      constexpr int t = decltype(tc)::value;
      const unsigned br = brev_run<t>(br0, m);
      double p[Dims<D>::N];
#pragma unroll
      for (int j = 0; j < Dims<D>::N; ++j) p[j] = dim_on<D>(a, j) ? gen_part<PG>(a, s, j, br, mask, inv_n) : 0.0;
      r[t] = k1_from<D>(h, p);
    });
  } else {
#pragma unroll
    for (int t = 0; t < 16; ++t) r[t] = 1.0;
#pragma unroll
    for (int j = 0; j < Dims<D>::N; ++j) {
      if (dim_on<D>(a, j)) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const double2 pv = *reinterpret_cast<const double2*>(s.pg + (int64_t)j * n + i0 + 2 * u);
          r[2 * u] *= __builtin_fma(h.ls[j], pv.x, 1.0);
          r[2 * u + 1] *= __builtin_fma(h.ls[j], pv.y, 1.0);
        }
      }
    }
#pragma unroll
    for (int t = 0; t < 16; ++t) r[t] = h.scale * r[t];
  }
#pragma unroll
  for (int t = 0; t < 16; ++t) {
    sum += r[t];
    v[t] = real_to_T<T>(r[t]);
  }
}

// Gradient terms of the 16 consecutive elements i0 + t with dL/dk1 = g[t] * gs.  g is the thread's
// private run of 16 values in LDS (stride-17 slots: conflict-free): a rolled loop keeps the register
// footprint of the regenerated parts bounded (fully unrolled, they spill to AGPRs).
template <int PG, int D>
__device__ __forceinline__ void grad_run16(const Nll& a, const Hyp& h, const PSrc& s, int64_t n, int64_t i0,
                                           const double* g, double gs, double* acc) {
  if constexpr (PG != 0) {
    const int m = a.log2n;
    const unsigned br0 = brev_bits((unsigned)i0, m), mask = (unsigned)(n - 1);
    const double inv_n = ldexp(1.0, -m);
#pragma unroll 2
    for (int t = 0; t < 16; ++t) {
      const unsigned br = br0 | ((__builtin_bitreverse32((unsigned)t) >> 28) << (m - 4));
      double p[Dims<D>::N];
#pragma unroll
      for (int j = 0; j < Dims<D>::N; ++j) p[j] = dim_on<D>(a, j) ? gen_part<PG>(a, s, j, br, mask, inv_n) : 0.0;
      grad_terms_p<D>(h, p, g[t] * gs, acc);
    }
  } else {
#pragma unroll 2
    for (int u = 0; u < 8; ++u) {
      double p0[Dims<D>::N], p1[Dims<D>::N];
      parts_pair<PG, D>(a, s, n, i0 + 2 * u, p0, p1);
      grad_terms_p<D>(h, p0, g[2 * u] * gs, acc);
      grad_terms_p<D>(h, p1, g[2 * u + 1] * gs, acc);
    }
  }
}

// factor applied to the reduced gradient partial q (0: scale, 1 + j: scale l_j)
__device__ __forceinline__ double grad_factor(const Hyp& h, int q) {
  return q == 0 ? h.scale : h.scale * h.ls[q - 1];
}

// log|ev| accumulated as a product of frexp mantissas (each in [0.5, 1): 16 factors stay >= 2^-16)
// and a sum of exponents, one log per thread instead of one per frequency:
//   sum_k log|ev_k| = log(prod_k mant_k) + ln 2 sum_k exp_k
struct LogAcc {
  double mant = 1.0;
  int ex = 0;
  __device__ __forceinline__ void add(double v) {   // v > 0 (or 0 / inf / nan: propagate as log would)
    int e;
    mant *= frexp(v, &e);
    ex += e;
  }
  __device__ __forceinline__ double log_sum(double half) const {
    return half * (log(mant) + (double)ex * 0.69314718055994530942);
  }
};

// eigenvalue terms for one frequency: returns dL/dlambda, accumulates norm / log|ev| / dnoise
__device__ __forceinline__ double2 eig_terms(double2 lam, double rootn, double noise, double Y, double w,
                                             double& norm, LogAcc& la, double& dnoise) {
  const double ar = rootn * lam.x + noise, ai = rootn * lam.y;    // ev = sqrt(n) lam + noise
  const double den = ar * ar + ai * ai;
  const double inv = 1.0 / den;
  const double rr = ar * inv, ri = -ai * inv;                      // 1/ev
  norm += Y * rr;
  la.add(den);                                                     // log|ev| = 1/2 log(den)
  // G_e = 1/2 conj(w/ev - Y/ev^2) ; 1/ev^2 = (rr^2 - ri^2, 2 rr ri)
  const double qr = w * rr - Y * (rr * rr - ri * ri);
  const double qi = w * ri - Y * (2.0 * rr * ri);
  const double ger = 0.5 * qr, gei = -0.5 * qi;
  dnoise += ger;
  return make_double2(rootn * ger, rootn * gei);
}
__device__ __forceinline__ double eig_terms(double lam, double rootn, double noise, double Y, double w, double& norm,
                                            LogAcc& la, double& dnoise) {
  const double e = rootn * lam + noise;
  const double r = 1.0 / e;
  norm += Y * r;
  la.add(fabs(e));
  const double ge = 0.5 * (w * r - Y * r * r);
  dnoise += ge;
  return rootn * ge;
}
// 1/2 for the lattice (log of |ev|^2), 1 for nets (log of |ev|)
template <typename T> struct LogHalf { static constexpr double value = sizeof(T) == 16 ? 0.5 : 1.0; };

__device__ __forceinline__ double* part_ptr(const Nll& a, int g, int q, int blk) {
  return a.partials + ((int64_t)g * a.nq + q) * a.nb + blk;
}

// ---------------------------------------------------------------- n > 4096: layout of `work`
// The two-pass intermediate is stored as column tiles [N2 / C][N1][C] (C = kTile / N1 columns, the
// column kernel's tile): element (row u, column k) of the N1 x N2 view at
//   (k / C) kTile + u C + k mod C.
// The column kernel (HBM-bound) then streams one contiguous 64 KB block per workgroup; the row
// kernels (FP64-VALU-bound, with bandwidth to spare) take the strided side: runs of C elements
// (256 B at C = 16) spaced kTile elements apart.
__device__ __forceinline__ int64_t work_pos(int64_t u, int64_t k, int P1) {
  const int CL = kTileLog - P1;
  return ((k >> CL) << kTileLog) + (u << CL) + (k & ((1 << CL) - 1));
}

// Calls fn(std::integral_constant<int, PG>) with the parts source of `a` as a compile-time value
// (generated lattice parts exist only for the complex / lattice instantiations).
template <typename T, typename Fn>
static int with_pg(const Nll& a, Fn&& fn) {
  if constexpr (sizeof(T) == 16) {
    switch (a.pg) {
      case 2: return fn(std::integral_constant<int, 2>{});
      case 4: return fn(std::integral_constant<int, 4>{});
      case 6: return fn(std::integral_constant<int, 6>{});
      case 8: return fn(std::integral_constant<int, 8>{});
      default: break;
    }
  }
  return fn(std::integral_constant<int, 0>{});
}

// Calls fn(std::integral_constant<int, D>{}) with d (1 .. FGP_MAX_D) as a compile-time value.
template <typename Fn>
static void with_d(int d, Fn&& fn) {
  switch (d) {
    case 1: fn(std::integral_constant<int, 1>{}); break;
    case 2: fn(std::integral_constant<int, 2>{}); break;
    case 3: fn(std::integral_constant<int, 3>{}); break;
    case 4: fn(std::integral_constant<int, 4>{}); break;
    case 5: fn(std::integral_constant<int, 5>{}); break;
    case 6: fn(std::integral_constant<int, 6>{}); break;
    case 7: fn(std::integral_constant<int, 7>{}); break;
    default: fn(std::integral_constant<int, 8>{}); break;
  }
}

struct Fit {
  int n_params;
  double* raw;
  double* prev;
  double* step;
  double* grad_out;
  double* loss_hist;
  double* raw_hist;
  int scale_rg, ls_rg, noise_rg;
  double mll_const, eta_minus, eta_plus, step_min, step_max;
  int per_problem;
  int hist_stride, hist_offset;   // loss_hist row stride in problems (0: G) and this desc's first problem
};

// torch.optim.Rprop single-tensor step of parameter p with gradient gp, state in f (raw, prev, step)
__device__ __forceinline__ void rprop_update(const Fit& f, int p, double gp) {
  const double prod = gp * f.prev[p];
  const double sgn = prod > 0.0 ? f.eta_plus : (prod < 0.0 ? f.eta_minus : 1.0);
  const double st = fmin(fmax(f.step[p] * sgn, f.step_min), f.step_max);
  f.step[p] = st;
  const double gg = (sgn == f.eta_minus) ? 0.0 : gp;
  const double gs = gg > 0.0 ? 1.0 : (gg < 0.0 ? -1.0 : 0.0);
  f.raw[p] = f.raw[p] + (-1.0) * (gs * st);
  f.prev[p] = gg;
}

// Per-problem reduction + loss history + Rprop (torch.optim.Rprop single-tensor semantics) by one
// workgroup of NT threads for problem g: k_fit_reduce_step, and the last row-pair workgroup of the
// fused real-even backward kernel (SC1: the partials of that same launch are read with sc1 loads,
// MI355X_MICROARCH.md hand-off row 1).  The kernel is a pure latency chain (it sits between two
// iterations), so every load is issued up front: each thread's partials of all quantities at once, and
// the parameter-owning threads' Rprop state before the reduction.  Per-quantity order of the sum is
// fixed (deterministic).  red: [(4 + FGP_MAX_D) * NT / 64], vals: [4 + FGP_MAX_D] (LDS).
template <int NT, bool SC1>
__device__ __forceinline__ void reduce_step_wg(const Nll& a, const Fit& f, int g, int iter, int do_update, double* red,
                                               double* vals) {
  constexpr int NQ = 4 + FGP_MAX_D, NW = NT / 64;
  const int k = threadIdx.x;
  const int dl = a.ls_pd ? a.d : 1;
  // the parameter thread k owns: 0 scale, 1..dl lengthscales, dl + 1 noise
  int p = 0, rg = 0;
  if (k == 0) {
    p = a.scale_off + (a.scale_pp ? g : 0);
    rg = f.scale_rg;
  } else if (k <= dl) {
    p = a.ls_off + (a.ls_pp ? g : 0) * dl + (k - 1);
    rg = f.ls_rg;
  } else {
    p = a.noise_off + (a.noise_pp ? g : 0);
    rg = f.noise_rg;
  }
  const bool owner = k < 2 + dl;
  double raw_p = 0.0, prev_p = 0.0, step_p = 0.0;
  if (owner) {
    raw_p = f.raw[p];
    prev_p = f.prev[p];
    step_p = f.step[p];
  }
  double s[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) s[q] = 0.0;
  for (int b = k; b < a.nb; b += NT) {
    double v[NQ];   // quantities past nq re-read q = 0 (unused)
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      double* pp = part_ptr(a, g, q < a.nq ? q : 0, b);
      v[q] = SC1 ? __hip_atomic_load(pp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : *pp;
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) s[q] += v[q];
  }
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    double v = s[q];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if ((k & 63) == 0) red[q * NW + (k >> 6)] = v;
  }
  __syncthreads();
  if (k < NQ) {
    double tot = 0.0;
#pragma unroll
    for (int w = 0; w < NW; ++w) tot += red[k * NW + w];
    vals[k] = tot;
  }
  __syncthreads();
  if (k == 0) {
    const double term2 = a.logdet_weight * vals[1];
    double* lh = f.loss_hist + ((int64_t)iter * (f.hist_stride ? f.hist_stride : a.G) + f.hist_offset + g) * 3;
    lh[0] = 0.5 * (vals[0] + term2 + f.mll_const);
    lh[1] = vals[0];
    lh[2] = term2;
  }
  if (!owner) return;
  double gp;
  if (k == 0) {
    gp = vals[3];
  } else if (k <= dl) {
    if (a.ls_pd) {
      gp = vals[4 + (k - 1)];
    } else {
      gp = 0.0;
      for (int j = 0; j < a.d; ++j) gp += vals[4 + j];
    }
  } else {
    gp = exp(raw_p) * vals[2];
  }
  f.raw_hist[(int64_t)iter * f.n_params + p] = raw_p;
  f.grad_out[p] = gp;
  if (!(do_update && rg)) return;
  // torch.optim.Rprop single-tensor semantics (as rprop_update, on the prefetched state)
  const double prod = gp * prev_p;
  const double sgn = prod > 0.0 ? f.eta_plus : (prod < 0.0 ? f.eta_minus : 1.0);
  const double st = fmin(fmax(step_p * sgn, f.step_min), f.step_max);
  f.step[p] = st;
  const double gg = (sgn == f.eta_minus) ? 0.0 : gp;
  const double gs = gg > 0.0 ? 1.0 : (gg < 0.0 ? -1.0 : 0.0);
  f.raw[p] = raw_p + (-1.0) * (gs * st);
  f.prev[p] = gg;
}

// real-even lattice fit kernels (fgp_nll_re.hip): stage 0 forward rows, 1 columns, 2 adjoint rows
int launch_re(const Nll& a, int stage, const Tables* tb, hipStream_t st);
// fused backward + reduction + Rprop of one iteration (per-problem fits): the stage-2 kernel's last
// row-pair workgroup of each problem runs reduce_step_wg.  counters: G zeroed 32-bit words.
// Rprop state (raw parameters, previous gradient, step sizes) of every problem: the fit's own vectors, or one
// of the spectral fused run's two scratch copies (fgp_spectral.hip, deferred step)
struct RpState {
  double* raw;
  double* prev;
  double* step;
};
struct FitFuse {
  Fit f;
  int iter, do_update;
  unsigned* counters;
  // spectral tile kernel (fgp_spectral.hip): the step of iteration iter - 1 is deferred into this launch
  // (pending: every workgroup reduces that iteration's level-1 sums of parity par ^ 1 and steps the
  // parameters from sin; workgroup 0 writes histories and sout); this launch's level-1 sums go to parity par
  int pending, par;
  RpState sin, sout;
  // fgp_handoff_check (a test hook): [kSpecBlocks / kSpecGroup][G nq] XOR words, then checks, mismatches
  unsigned long long* check;
  // persistent k_spec_tile (piters > 0): iterations iter .. iter + piters - 1 AND the last one's step in ONE
  // launch; counters[ng] counts the published group sums, counters[ng + 1] is set when a bounded wait gave up
  int piters;
};
constexpr int kSpecStateMax = 64;                  // Rprop parameters of a persistent k_spec_tile (LDS copies)
// parameters of a spectral fit (the raw vector's length: the noise block is last)
__host__ __device__ __forceinline__ int spec_nparams(const Nll& a) {
  return a.noise_off + (a.noise_pp ? a.G : 1) + (a.mt_learn ? a.mt * (a.mt_rank + 1) : 0);
}
constexpr int kHandoffWords = 32 * 8 * 16;         // XOR words of the check buffer (groups x G x nq, at most)
int launch_re_bwd_fused(const Nll& a, const FitFuse& fz, const Tables* tb, hipStream_t st);

// spectral fit path (fgp_spectral.hip): d <= kSpecMaxD, at most kSpecBlocks k blocks per problem
constexpr int kSpecMaxD = 6;
constexpr int kSpecBlocks = 512;
// frequency k of subset 0 in the chunked spectra of ns subsets ([chunk][subset][64]; subset s at + 64 s)
__host__ __device__ __forceinline__ int64_t spec_pos(int64_t k, int ns) { return (((k >> 6) * ns) << 6) + (k & 63); }
#ifndef FGP_SPEC_RING
#define FGP_SPEC_RING 2
#endif
constexpr int kSpecRing = FGP_SPEC_RING;         // LDS ring depth of the spectral tile kernel (chunks)
#ifndef FGP_SPEC_LDS_KB
#define FGP_SPEC_LDS_KB 80
#endif
constexpr int kSpecLdsMax = FGP_SPEC_LDS_KB * 1024;   // its dynamic LDS per workgroup, at most (80: 2 per CU)
constexpr int kSpecScratch = 256;                  // doubles of the deferred step's totals / parameters (ring slot RING-1)
constexpr int kSpecMaxDma = 6;                     // LDS-DMA wave-instructions per wave and chunk (tile <= 3072 doubles;
                                                   // the per-wave source pointers live in registers)
void spec_geometry(Nll& a, bool allow_tile = true);   // nb and the spec_* fields of a spectral desc
int launch_spec_loss_iter(const Nll& a, hipStream_t st);   // GCV / CV partials (ABI 16)
int launch_spec_loss_step(const Nll& a, const Fit& f, int iter, int do_update, hipStream_t st);
int64_t spec_chunks(bool net, int log2n);          // 64-frequency chunks of the spectra (fgp_spec_basis layout)
// one fit iteration (loss + gradient partials); with fz (tile kernel only) also the reduction + Rprop
int launch_spec_iter(const Nll& a, hipStream_t st, const FitFuse* fz = nullptr);
int launch_spec_reduce_step(const Nll& a, const Fit& f, int iter, int do_update, hipStream_t st);
// the step of one loss over many problems (not per_problem) from the spectral partials, ceil(G / 16) workgroups,
// the shared part in the last arriver; its arrival counter (one word of the partials workspace) must be zero
// before the first launch (each launch leaves it zero)
int launch_spec_step_many(const Nll& a, const Fit& f, int iter, int do_update, hipStream_t st);
unsigned* spec_step_many_counter(const Nll& a);
// the fused spectral run's counters: doubles offset into partials and how many 32-bit counters
int spec_counters_offset(const Nll& a, int64_t* off, int* count);
// the fused spectral run's scratch copies of the Rprop state (parity 0, 1) in the partials workspace
RpState spec_scratch_state(const Nll& a, int par);
// the deferred step of a fused spectral run's last iteration (after its last k_spec_tile launch)
int launch_spec_finish_step(const Nll& a, const FitFuse& fz, hipStream_t st);
// the whole fit of one small spectral problem in one launch (fgp_fit_persist): geometry / applicability, launch
int spec_persist_geometry(const Nll& a, int* W, int* bpw, size_t* shm);
void set_persist_poll_max(long long v);
int persist_giveups(unsigned long long* count, int reset);
int launch_spec_persist(const Nll& a, const Fit& f, int iters, double logtol, int wait_max, unsigned* counter, int* out,
                        hipStream_t st);
int launch_spec_lam(const Nll& a, hipStream_t st);    // lambda of the current parameters into grad_lam
int launch_spec_inv_eig(const Nll& a, double* wa, hipStream_t st);
constexpr int kSpvKpl = 16;   // fgp_spec_post_var: frequencies per lane of a wave's block (64 kSpvKpl per block)
int launch_spec_post_var(const Nll& a, const double2* psi, int N, const double* part0, double* out, double* partial,
                         int nblk, int kpl, hipStream_t st);   // A = 1 / (sqrt(n) lambda + noise), [G][n]
// multitask spectral fit (ABI 12): at most kMtMaxT tasks, kMtF frequencies per chunk
constexpr int kMtMaxT = 8;
constexpr int kMtF = 32;
int launch_mt_spec_iter(const Nll& a, hipStream_t st);
int launch_mt_learn_step(const Nll& a, const Fit& f, int iter, int do_update, hipStream_t st);   // learned task kernel   // loss / gradient partials of one iteration
// lattice spectra of the subsets s0 .. s0 + cnt - 1 (log2n >= 17) by the fused R2C pair: products formed in
// the row kernel, real parts k <= n/2 written by the column kernel (work: 16 n cnt bytes)
struct GenSpec;
// (gen: the lattice parts regenerated in the row kernel instead of read from `parts`)
int spec_basis_r2c(const double* parts, int d, int log2n, int s0, int cnt, double* basis, void* work, hipStream_t st,
                   const GenSpec* gen = nullptr);
// their row length log2 (11) for a transform of 2^log2n, or -1 when no split fits
int re_row_log2(int log2n);

}  // namespace fgp
