// Part-product spectra: the spectral fit path (ABI 11).  See DESIGN.md section 3 "Spectral fit".
//
// The first-column kernel of both families is a multilinear polynomial in the lengthscales:
//   k1 = scale prod_j (1 + l_j part_j) = scale sum_{S subset of {0..d-1}} l^S b_S,
//   l^S = prod_{j in S} l_j,   b_S[i] = prod_{j in S} part_j[i]   (b_{} = 1),
// and ft (fftbr / fwht, AbstractFastGP.ft, abstract_fast_gp.py:197-212) is linear, so at EVERY
// hyper-parameter setting
//   lambda = ft(k1) = scale sum_S l^S Phi_S,   Phi_S = ft(b_S).
// The reference's _LamCaches (util.py:95-112) recomputes ft(k1) after each Rprop step; here the 2^d
// transforms Phi_S run once per point set (fgp_spec_basis) and a fit iteration is, per frequency k, one
// evaluation of the multilinear polynomial P(l) = sum_S l^S Phi_S[k] with its d partial derivatives,
// the eigenvalue terms of util.py:275-370 and the gradient of abstract_gp.py:294 in closed form:
//   dL/draw_scale = sum_k G_k scale P_k,  dL/draw_l_j = sum_k G_k scale l_j dP_k/dl_j,
//   G_k = dL/dlambda_k = sqrt(n) dL/dev_k.
// No transform runs per iteration: the iteration streams 8 2^d bytes of spectra per frequency (read once
// for every problem sharing them) plus Y, and is HBM / Infinity-Cache bound.
// Lattice: k1 is real and even in the natural index (B_2a(1 - x) = B_2a(x)), so every Phi_S is real and
// even, Phi_S[k] = Phi_S[n - k]: only k = 0 .. n/2 are stored and the loss is the folded sum (weight 2 for
// 0 < k < n/2), exactly as the real-even kernels fold it (fgp_nll_re.hip).  Nets: Phi_S (FWHT) real,
// k = 0 .. n-1, weight 1.
#include <algorithm>

#include "fgp_nll.h"

namespace fgp {

// P(l) = sum_{S < 2^D} l^S phi[S] (bit j of S = dimension j) and dp[j] = dP/dl_j, by recursion on the
// top dimension J = D - 1:  P = P0 + l_J P1 (P0 over phi[S], P1 over phi[S + 2^J], S < 2^J), so
//   dP/dl_J = P1,   dP/dl_j = dP0/dl_j + l_J dP1/dl_j  (j < J).
// 2 C(D-1) + D fused multiply-adds (D = 5: 57), O(D^2) live temporaries.  The value alone (dp unused, as
// in k_spec_lam) is the same instruction sequence minus the derivative FMAs: bit-identical P.
template <int D>
__device__ __forceinline__ double mlin(const double* phi, const double* l, double* dp) {
  if constexpr (D == 0) {
    return phi[0];
  } else {
    constexpr int H = 1 << (D - 1);
    double d0[D > 1 ? D - 1 : 1], d1[D > 1 ? D - 1 : 1];
    const double p0 = mlin<D - 1>(phi, l, d0);
    const double p1 = mlin<D - 1>(phi + H, l, d1);
#pragma unroll
    for (int j = 0; j < D - 1; ++j) dp[j] = __builtin_fma(l[D - 1], d1[j], d0[j]);
    dp[D - 1] = p1;
    return __builtin_fma(l[D - 1], p1, p0);
  }
}

// Per-problem accumulators of one lane (its frequencies of one block).
template <int D>
struct SpecAcc {
  double norm = 0.0, dnoise = 0.0, gs = 0.0, mant = 1.0;
  double gl[D];
  int ex = 0;
  __device__ __forceinline__ SpecAcc() {
#pragma unroll
    for (int j = 0; j < D; ++j) gl[j] = 0.0;
  }
};

// One frequency k of problem p: eigenvalue ev = sqrt(n) scale P + noise and its terms (weight w = 1 or 2;
// two: the folded pair k, n - k).  Loss terms as eig_terms (fgp_nll.h): norm += w Y / ev,
// log|ev| (frexp mantissa product + exponent sum), dL/dev = w/2 (wl / ev - Y / ev^2).
template <int D>
__device__ __forceinline__ void spec_terms(const double* phi, const Hyp& h, double rootn, double wl, double Y, bool two,
                                           SpecAcc<D>& acc) {
  double dp[D];
  const double P = mlin<D>(phi, h.ls, dp);
  const double e = __builtin_fma(rootn, h.scale * P, h.noise);
  const double r = 1.0 / e;
  const double w = two ? 2.0 : 1.0;
  acc.norm = __builtin_fma(w * Y, r, acc.norm);
  int ex;
  const double m = frexp(fabs(e), &ex);
  acc.mant *= two ? m * m : m;
  acc.ex += two ? 2 * ex : ex;
  const double ge = (0.5 * w) * r * __builtin_fma(-Y, r, wl);   // dL/dev
  acc.dnoise += ge;
  acc.gs = __builtin_fma(ge, P, acc.gs);
#pragma unroll
  for (int j = 0; j < D; ++j) acc.gl[j] = __builtin_fma(ge, dp[j], acc.gl[j]);
}

// One fit iteration over every problem and frequency: per-block partials of the norm, logdet, dL/dnoise
// and gradient terms in the layout of the transform kernels (part_ptr, fgp_nll.h), so the same
// reduction + Rprop (reduce_step_wg) follows.  Wave task t = (k block kb, problem group pg): the
// PG = ceil(G / PPW) waves of one k block are consecutive (the spectra they share are read from the
// same lines at about the same time: one HBM / Infinity-Cache read, the rest L2 / L1 hits); a wave holds
// PPW problems over its block's 64 kpl frequencies (lane-contiguous, coalesced).  The lattice's last
// frequency k = n/2 (weight 1) is an extra step of lane 0 in the last block.  No barriers, no atomics.
template <int D, int PPW, bool NET>
__global__ __launch_bounds__(kWG) void k_spec_iter(Nll a) {
  constexpr int NS = 1 << D;
  const int lane = threadIdx.x & 63;
  const int task = (int)blockIdx.x * (kWG / 64) + (int)(threadIdx.x >> 6);
  const int kb = task / a.spec_pg, pg = task - kb * a.spec_pg;
  stamp_begin(a);
  if (kb < a.nb) {
    const int g0 = pg * PPW;
    Hyp h[PPW];
    bool on[PPW];
#pragma unroll
    for (int p = 0; p < PPW; ++p) {
      on[p] = g0 + p < a.G;
      load_hyp_wave(a, on[p] ? g0 + p : g0, h[p]);
    }
    const int64_t KS = a.spec_KS, main = a.spec_main;
    const double rootn = sqrt((double)((int64_t)1 << a.log2n)), wl = a.logdet_weight;
    const double* phib = a.basis + (int64_t)g0 * a.basis_stride;   // PPW = 2: shared spectra (stride 0)
    const double* ys[PPW];
#pragma unroll
    for (int p = 0; p < PPW; ++p) ys[p] = a.ysq + (int64_t)(on[p] ? g0 + p : g0) * a.ysq_stride;
    SpecAcc<D> acc[PPW];
    const int64_t kbase = (int64_t)kb * 64 * a.spec_kpl;
    auto step = [&](int64_t k, bool two) {
      double phi[NS];
#pragma unroll
      for (int s = 0; s < NS; ++s) phi[s] = phib[(int64_t)s * KS + k];
      double Y[PPW];
#pragma unroll
      for (int p = 0; p < PPW; ++p) Y[p] = ys[p][k];
#pragma unroll
      for (int p = 0; p < PPW; ++p)
        if (on[p]) spec_terms<D>(phi, h[p], rootn, wl, Y[p], two, acc[p]);
    };
    for (int i = 0; i < a.spec_kpl; ++i) {
      const int64_t k = kbase + lane + 64 * i;
      if (k >= main) break;
      step(k, !NET && k != 0);
    }
    if (!NET && kb == a.nb - 1 && lane == 0) step(main, false);   // k = n/2
    // wave sums (fixed shuffle order: deterministic) and this block's partials
#pragma unroll
    for (int p = 0; p < PPW; ++p) {
      if (!on[p]) continue;
      double v[4 + D];
      v[0] = acc[p].norm;
      v[1] = log(acc[p].mant) + (double)acc[p].ex * 0.69314718055994530942;
      v[2] = acc[p].dnoise;
      v[3] = acc[p].gs;
#pragma unroll
      for (int j = 0; j < D; ++j) v[4 + j] = acc[p].gl[j];
#pragma unroll
      for (int q = 0; q < 4 + D; ++q)
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v[q] += __shfl_xor(v[q], o, 64);
      if (lane == 0) {
        const int g = g0 + p;
        const double gsc = rootn * h[p].scale;   // dL/dlambda = sqrt(n) dL/dev; dlambda/draw_scale = lambda
        v[3] *= gsc;
#pragma unroll
        for (int j = 0; j < D; ++j) v[4 + j] *= gsc * h[p].ls[j];
#pragma unroll
        for (int q = 0; q < 4 + D; ++q) *part_ptr(a, g, q, kb) = v[q];
      }
    }
  }
  stamp_end(a);
}

// Per-problem reduction + loss history + Rprop of problem g by ONE wave: the reduce_step_wg semantics
// (fgp_nll.h: torch.optim.Rprop single-tensor, loss = 1/2 (norm + w logdet + const), histories) with the
// blocks summed lane-strided then by shuffles -- the one order used by both the stage launches
// (k_spec_reduce_step) and the fused last-workgroup step of k_spec_tile, so the two are bit-identical.
// SC1: the partials of the same launch are read with sc1 loads (the producers stored them sc1).
template <bool SC1>
__device__ __forceinline__ void reduce_step_wave(const Nll& a, const Fit& f, int g, int iter, int do_update) {
  constexpr int NQ = 4 + FGP_MAX_D;
  const int lane = threadIdx.x & 63;
  const int dl = a.ls_pd ? a.d : 1;
  int p = 0, rg = 0;
  if (lane == 0) {
    p = a.scale_off + (a.scale_pp ? g : 0);
    rg = f.scale_rg;
  } else if (lane <= dl) {
    p = a.ls_off + (a.ls_pp ? g : 0) * dl + (lane - 1);
    rg = f.ls_rg;
  } else {
    p = a.noise_off + (a.noise_pp ? g : 0);
    rg = f.noise_rg;
  }
  const bool owner = lane < 2 + dl;
  double raw_p = 0.0, prev_p = 0.0, step_p = 0.0;
  if (owner) {
    raw_p = f.raw[p];
    prev_p = f.prev[p];
    step_p = f.step[p];
  }
  double v[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) v[q] = 0.0;
  for (int b = lane; b < a.nb; b += 64) {
    double t[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      if (q < a.nq) {
        double* pp = part_ptr(a, g, q, b);
        t[q] = SC1 ? __hip_atomic_load(pp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : *pp;
      } else {
        t[q] = 0.0;
      }
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) v[q] += t[q];
  }
#pragma unroll
  for (int q = 0; q < NQ; ++q)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v[q] += __shfl_xor(v[q], o, 64);
  if (lane == 0) {
    const double term2 = a.logdet_weight * v[1];
    double* lh = f.loss_hist + ((int64_t)iter * (f.hist_stride ? f.hist_stride : a.G) + f.hist_offset + g) * 3;
    lh[0] = 0.5 * (v[0] + term2 + f.mll_const);
    lh[1] = v[0];
    lh[2] = term2;
  }
  if (!owner) return;
  double gp;
  if (lane == 0) {
    gp = v[3];
  } else if (lane <= dl) {
    if (a.ls_pd) {
      gp = 0.0;
#pragma unroll
      for (int j = 0; j < FGP_MAX_D; ++j) gp = (j == lane - 1) ? v[4 + j] : gp;
    } else {
      gp = 0.0;
#pragma unroll
      for (int j = 0; j < FGP_MAX_D; ++j) gp += (j < a.d) ? v[4 + j] : 0.0;
    }
  } else {
    gp = exp(raw_p) * v[2];
  }
  f.raw_hist[(int64_t)iter * f.n_params + p] = raw_p;
  f.grad_out[p] = gp;
  if (!(do_update && rg)) return;
  const double prod = gp * prev_p;
  const double sgn = prod > 0.0 ? f.eta_plus : (prod < 0.0 ? f.eta_minus : 1.0);
  const double st = fmin(fmax(step_p * sgn, f.step_min), f.step_max);
  f.step[p] = st;
  const double gg = (sgn == f.eta_minus) ? 0.0 : gp;
  const double gs = gg > 0.0 ? 1.0 : (gg < 0.0 ? -1.0 : 0.0);
  f.raw[p] = raw_p + (-1.0) * (gs * st);
  f.prev[p] = gg;
}

// The per-problem step of the spectral path as its own launch (fgp_fit_step, stage-by-stage fits):
// wave w of workgroup b reduces problem 4 b + w.
__global__ __launch_bounds__(kWG) void k_spec_reduce_step(Nll a, Fit f, int iter, int do_update) {
  const int g = (int)blockIdx.x * (kWG / 64) + (int)(threadIdx.x >> 6);
  if (g < a.G) reduce_step_wave<false>(a, f, g, iter, do_update);
}

// One fit iteration when every problem shares ONE set of spectra and the problem groups fit in the four
// waves of a workgroup (PG = ceil(G / PPW) <= 4; the C4 shifts, single GPs) and a chunk's tile is at most
// 24 KB (two buffers: 48 KB of LDS, two workgroups per CU).  The k blocks are those of
// k_spec_iter (nb blocks of B = 64 kpl frequencies, one partial per problem and block, lane l summing
// k = block base + l + 64 i in ascending i): workgroup b owns NBW = 4 / PGP consecutive blocks (PGP = PG
// rounded up to 1, 2 or 4), wave w the block w / PGP for problem group w mod PGP -- so every problem's
// arithmetic, and its partials, are those of k_spec_iter whatever G is (a batch equals its GPs' own fits
// bit for bit).  The spectra and Y stream through a double-buffered LDS tile in chunks of 64 frequencies
// per block: the chunk's (2^d + G) rows x NBW segments are read ONCE from HBM by all 256 threads (16-byte
// loads issued a chunk ahead into registers, so they fly under the previous chunk's compute) instead of
// once per problem group, and each wave reads its segment from LDS (lane-consecutive 8-byte reads:
// conflict-free).  With fz.counters the LAST workgroup to finish (sc1 partials, an agent-scope arrival
// counter: MI355X_MICROARCH.md hand-off row 1, as the real-even backward kernel) runs every problem's
// reduction + Rprop, wave w taking problems w, w + 4, ...
template <int D, int PPW, bool NET>
__global__ __launch_bounds__(kWG, 2) void k_spec_tile(Nll a, FitFuse fz) {
  constexpr int NS = 1 << D, MAXP = 8;              // 16-byte pieces per thread and chunk, at most
  extern __shared__ double lds[];                   // [2][NS + G][NBW][64]
  __shared__ int last_wg;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int PGP = a.spec_pgp, NBW = 4 / PGP, G = a.G;
  const int rows = NS + G, tile = rows * NBW * 64, npieces = tile / 2, rowp = 32 * NBW;
  const int pg = w % PGP, bw = w / PGP;
  const int g0 = pg * PPW;
  const bool active = g0 < G;
  const int64_t B = 64 * (int64_t)a.spec_kpl;       // frequencies per block
  const int blk = (int)blockIdx.x * NBW + bw;
  stamp_begin(a);
  Hyp h[PPW];
  bool on[PPW];
#pragma unroll
  for (int p = 0; p < PPW; ++p) {
    on[p] = g0 + p < G;
    load_hyp_wave(a, on[p] ? g0 + p : 0, h[p]);
  }
  const int64_t KS = a.spec_KS, main = a.spec_main;
  const double rootn = sqrt((double)((int64_t)1 << a.log2n)), wl = a.logdet_weight;
  const int64_t wg_base = (int64_t)blockIdx.x * NBW * B;
  // piece i of chunk c: row i / rowp (spectrum rows, then Y rows), segment (i mod rowp) / 32, 16-byte
  // column i mod 32; LDS offset 2 i (the image is [row][segment][64] in piece order)
  auto src = [&](int i, int c) -> const double2* {
    const int r = i / rowp, rem = i - r * rowp, sg = rem >> 5, col = rem & 31;
    const double* row = r < NS ? a.basis + (int64_t)r * KS : a.ysq + (int64_t)(r - NS) * a.ysq_stride;
    return reinterpret_cast<const double2*>(row + wg_base + sg * B + 64 * (int64_t)c) + col;
  };
  double2 stage[MAXP];
  auto load_chunk = [&](int c) {
#pragma unroll
    for (int j = 0; j < MAXP; ++j) {
      const int i = (int)threadIdx.x + kWG * j;
      if (i < npieces) stage[j] = *src(i, c);
    }
  };
  auto store_chunk = [&](double* buf) {
#pragma unroll
    for (int j = 0; j < MAXP; ++j) {
      const int i = (int)threadIdx.x + kWG * j;
      if (i < npieces) reinterpret_cast<double2*>(buf)[i] = stage[j];
    }
  };
  SpecAcc<D> acc[PPW];
  const int nc = a.spec_kpl;
  load_chunk(0);
  store_chunk(lds);
  __syncthreads();
  for (int c = 0; c < nc; ++c) {
    if (c + 1 < nc) load_chunk(c + 1);
    const double* buf = lds + (c & 1) * tile;
    if (active) {
      double phi[NS];
#pragma unroll
      for (int s = 0; s < NS; ++s) phi[s] = buf[(s * NBW + bw) * 64 + lane];
      const bool two = !NET && (blk != 0 || c != 0 || lane != 0);
#pragma unroll
      for (int p = 0; p < PPW; ++p)
        if (on[p]) spec_terms<D>(phi, h[p], rootn, wl, buf[((NS + g0 + p) * NBW + bw) * 64 + lane], two, acc[p]);
    }
    if (c + 1 < nc) store_chunk(lds + ((c + 1) & 1) * tile);
    __syncthreads();
  }
  if (!NET && active && blk == a.nb - 1 && lane == 0) {   // k = n/2, weight 1 (as k_spec_iter)
    double phi[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) phi[s] = a.basis[(int64_t)s * KS + main];
#pragma unroll
    for (int p = 0; p < PPW; ++p)
      if (on[p]) spec_terms<D>(phi, h[p], rootn, wl, a.ysq[(int64_t)(g0 + p) * a.ysq_stride + main], false, acc[p]);
  }
  // the block's partials (k_spec_iter's values), one storing lane per problem (sc1 when fused)
#pragma unroll
  for (int p = 0; p < PPW; ++p) {
    if (!on[p] || !active) continue;
    double v[4 + D];
    v[0] = acc[p].norm;
    v[1] = log(acc[p].mant) + (double)acc[p].ex * 0.69314718055994530942;
    v[2] = acc[p].dnoise;
    v[3] = acc[p].gs;
#pragma unroll
    for (int j = 0; j < D; ++j) v[4 + j] = acc[p].gl[j];
#pragma unroll
    for (int q = 0; q < 4 + D; ++q)
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) v[q] += __shfl_xor(v[q], o, 64);
    if (lane == 0) {
      const int g = g0 + p;
      const double gsc = rootn * h[p].scale;
      v[3] *= gsc;
#pragma unroll
      for (int j = 0; j < D; ++j) v[4 + j] *= gsc * h[p].ls[j];
#pragma unroll
      for (int q = 0; q < 4 + D; ++q) {
        double* dst = part_ptr(a, g, q, blk);
        if (fz.counters) __hip_atomic_store(dst, v[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else *dst = v[q];
      }
    }
  }
  if (fz.counters) {
    // hand-off: every storing lane's sc1 stores retired (vmcnt) before the workgroup's arrival
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned prev = __hip_atomic_fetch_add(fz.counters, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last_wg = prev == gridDim.x - 1;
    }
    __syncthreads();
    if (last_wg) {
      for (int g = w; g < G; g += kWG / 64) reduce_step_wave<true>(a, fz.f, g, fz.iter, fz.do_update);
      if (threadIdx.x == 0) __hip_atomic_store(fz.counters, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  stamp_end(a);
}

// lambda = scale P (the eigenvalues of the current parameters, fgp_nll_lam): lattice complex128 [G][n]
// (k and its mirror n - k from one evaluation; imaginary parts 0), net float64 [G][n].
template <int D, bool NET>
__global__ __launch_bounds__(kWG) void k_spec_lam(Nll a) {
  constexpr int NS = 1 << D;
  const int g = blockIdx.y;
  const int64_t k = (int64_t)blockIdx.x * kWG + threadIdx.x;
  const int64_t n = (int64_t)1 << a.log2n;
  Hyp h;
  load_hyp_wave(a, g, h);
  if (k >= a.spec_K) return;
  const double* phib = a.basis + (int64_t)g * a.basis_stride;
  double phi[NS], dp[D];
#pragma unroll
  for (int s = 0; s < NS; ++s) phi[s] = phib[(int64_t)s * a.spec_KS + k];
  const double lam = h.scale * mlin<D>(phi, h.ls, dp);
  if constexpr (NET) {
    static_cast<double*>(a.grad_lam)[(int64_t)g * n + k] = lam;
  } else {
    double2* out = static_cast<double2*>(a.grad_lam) + (int64_t)g * n;
    out[k] = make_double2(lam, 0.0);
    if (k > 0 && k < n / 2) out[n - k] = make_double2(lam, 0.0);
  }
}

template <typename Fn>
static int with_spec_d(int d, Fn&& fn) {
  switch (d) {
    case 1: return fn(std::integral_constant<int, 1>{});
    case 2: return fn(std::integral_constant<int, 2>{});
    case 3: return fn(std::integral_constant<int, 3>{});
    case 4: return fn(std::integral_constant<int, 4>{});
    case 5: return fn(std::integral_constant<int, 5>{});
    case 6: return fn(std::integral_constant<int, 6>{});
    default: return set_error(kErrUnsupported, "spectral fit path: d = %d > %d", d, kSpecMaxD);
  }
}

// Geometry of the spectral iteration for n = 2^log2n, G problems.  Tile kernel (one shared set of spectra,
// PG <= 4, the chunk's tile <= 32 KB): workgroups of KW = max(CK, main / 512) frequencies, chunks of
// CK = 64 (4 / PGP).  Otherwise (k_spec_iter): nb k blocks of 64 kpl frequencies covering [0, main)
// (lattice main = n/2, plus k = n/2; net main = n), PPW problems per wave.
void spec_geometry(Nll& a) {
  const int64_t n = (int64_t)1 << a.log2n;
  const bool net = a.spec_net;
  a.spec_main = net ? n : n / 2;
  a.spec_K = net ? n : n / 2 + 1;
  a.spec_KS = spec_row_stride(net, a.log2n);
  a.spec_ppw = (a.G >= 2 && a.basis_stride == 0 && a.d <= 5) ? 2 : 1;
  a.spec_pg = (a.G + a.spec_ppw - 1) / a.spec_ppw;
  const int64_t lanes = std::max<int64_t>(1, a.spec_main / 64);
  a.nb = (int)std::min<int64_t>(kSpecBlocks, lanes);
  a.spec_kpl = (int)((a.spec_main + 64 * (int64_t)a.nb - 1) / (64 * (int64_t)a.nb));
  a.spec_tile = 0;
  a.spec_pgp = a.spec_ck = 0;
  a.spec_kw = 0;
  if (a.basis_stride == 0 && a.spec_pg <= 4 && a.d <= 5 && a.spec_main >= 256) {
    const int pgp = a.spec_pg <= 1 ? 1 : (a.spec_pg <= 2 ? 2 : 4);
    const int ck = 64 * (4 / pgp);   // frequencies per chunk (64 per block of the workgroup)
    if (((1 << a.d) + a.G) * ck <= 3072 && a.nb % (4 / pgp) == 0 && a.spec_main % (64 * (int64_t)a.nb) == 0) {
      a.spec_tile = 1;
      a.spec_pgp = pgp;
      a.spec_ck = ck;
      a.spec_kw = (int64_t)(4 / pgp) * 64 * a.spec_kpl;
    }
  }
}

int64_t spec_row_stride(bool net, int log2n) {
  const int64_t n = (int64_t)1 << log2n;
  return net ? n : n / 2 + 16;   // lattice: k = 0 .. n/2 and zero padding to a 128-byte row
}

int launch_spec_iter(const Nll& a, hipStream_t st, const FitFuse* fz) {
  if (a.spec_tile) {
    FitFuse none{};
    none.counters = nullptr;
    const FitFuse& f = fz ? *fz : none;
    const size_t shm = sizeof(double) * 2 * (size_t)(((1 << a.d) + a.G) * a.spec_ck);
    const unsigned grid = (unsigned)(a.nb / (4 / a.spec_pgp));
    return with_spec_d(a.d, [&](auto dc) {
      constexpr int D = decltype(dc)::value;
      if constexpr (D <= 5) {
        if (a.spec_net) {
          if (a.spec_ppw == 2) k_spec_tile<D, 2, true><<<grid, kWG, shm, st>>>(a, f);
          else k_spec_tile<D, 1, true><<<grid, kWG, shm, st>>>(a, f);
        } else {
          if (a.spec_ppw == 2) k_spec_tile<D, 2, false><<<grid, kWG, shm, st>>>(a, f);
          else k_spec_tile<D, 1, false><<<grid, kWG, shm, st>>>(a, f);
        }
        return check_launch("k_spec_tile");
      } else {
        return set_error(kErrInvalid, "spectral tile kernel: d > 5");
      }
    });
  }
  if (fz) return set_error(kErrInvalid, "spectral iteration: no fused step without the tile kernel");
  const int64_t tasks = (int64_t)a.nb * a.spec_pg;
  const unsigned grid = (unsigned)((tasks + kWG / 64 - 1) / (kWG / 64));
  return with_spec_d(a.d, [&](auto dc) {
    constexpr int D = decltype(dc)::value;
    if (a.spec_net) {
      if (a.spec_ppw == 2) k_spec_iter<D, 2, true><<<grid, kWG, 0, st>>>(a);
      else k_spec_iter<D, 1, true><<<grid, kWG, 0, st>>>(a);
    } else {
      if (a.spec_ppw == 2) k_spec_iter<D, 2, false><<<grid, kWG, 0, st>>>(a);
      else k_spec_iter<D, 1, false><<<grid, kWG, 0, st>>>(a);
    }
    return check_launch("k_spec_iter");
  });
}

int launch_spec_reduce_step(const Nll& a, const Fit& f, int iter, int do_update, hipStream_t st) {
  k_spec_reduce_step<<<(unsigned)((a.G + kWG / 64 - 1) / (kWG / 64)), kWG, 0, st>>>(a, f, iter, do_update);
  return check_launch("k_spec_reduce_step");
}

int launch_spec_lam(const Nll& a, hipStream_t st) {
  if (!a.grad_lam) return set_error(kErrInvalid, "fgp_nll_lam: null grad_lam (the output)");
  const dim3 grid((unsigned)((a.spec_K + kWG - 1) / kWG), (unsigned)a.G);
  return with_spec_d(a.d, [&](auto dc) {
    constexpr int D = decltype(dc)::value;
    if (a.spec_net) k_spec_lam<D, true><<<grid, kWG, 0, st>>>(a);
    else k_spec_lam<D, false><<<grid, kWG, 0, st>>>(a);
    return check_launch("k_spec_lam");
  });
}

// ---------------------------------------------------------------- building the spectra
// b_S[i] = prod_{j in S} parts[j][i] (ascending j; b_{} = 1) for the cnt subsets S = s0 .. s0 + cnt - 1.
template <int D>
__global__ __launch_bounds__(kWG) void k_spec_products(const double* __restrict__ parts, int64_t n, int s0, int cnt,
                                                       double* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * kWG + threadIdx.x;
  if (i >= n) return;
  double x[D];
#pragma unroll
  for (int j = 0; j < D; ++j) x[j] = parts[(int64_t)j * n + i];
  for (int c = 0; c < cnt; ++c) {
    const int S = s0 + c;
    double r = 1.0;
#pragma unroll
    for (int j = 0; j < D; ++j)
      if ((S >> j) & 1) r *= x[j];
    out[(int64_t)c * n + i] = r;
  }
}

// basis[s][k] = Re spec[s][k], k < K (the even spectrum's independent half), zeros to the row stride KS
__global__ __launch_bounds__(kWG) void k_spec_extract(const double2* __restrict__ spec, int64_t n, int64_t K,
                                                      int64_t KS, double* __restrict__ basis) {
  const int64_t k = (int64_t)blockIdx.x * kWG + threadIdx.x;
  const int s = blockIdx.y;
  if (k < KS) basis[(int64_t)s * KS + k] = k < K ? spec[(int64_t)s * n + k].x : 0.0;
}

static int64_t spec_subset_bytes(int family, int log2n) {
  const int64_t n = (int64_t)1 << log2n;
  if (family == FGP_FAMILY_NET) return 8 * n;                 // products, transformed into the basis
  return 8 * n + 16 * n + (log2n >= 17 ? 16 * n : 0);          // products + spectrum (+ fgp_fftbr_real scratch)
}

}  // namespace fgp

using namespace fgp;

extern "C" {

int fgp_spec_basis_work(int family, int log2n, int d, int64_t* bytes) {
  if (!bytes) return set_error(kErrInvalid, "fgp_spec_basis_work: null bytes");
  if ((family != FGP_FAMILY_LATTICE && family != FGP_FAMILY_NET) || log2n < 0 || log2n > kMaxLog2N || d < 1 ||
      d > kSpecMaxD)
    return set_error(kErrInvalid, "fgp_spec_basis_work: bad family / log2n / d");
  *bytes = spec_subset_bytes(family, log2n) << d;
  return kOk;
}

int fgp_spec_basis(int family, const double* parts, int64_t parts_stride, int64_t P, int log2n, int d, double* basis,
                   void* work, int64_t work_bytes, void* stream) {
  if ((family != FGP_FAMILY_LATTICE && family != FGP_FAMILY_NET) || log2n < 0 || log2n > kMaxLog2N)
    return set_error(kErrInvalid, "fgp_spec_basis: bad family / log2n");
  if (d < 1 || d > kSpecMaxD) return set_error(kErrUnsupported, "fgp_spec_basis: d = %d outside [1, %d]", d, kSpecMaxD);
  if (P < 1) return set_error(kErrInvalid, "fgp_spec_basis: P < 1");
  if (!parts || !basis || !work) return set_error(kErrInvalid, "fgp_spec_basis: null pointer");
  const int64_t n = (int64_t)1 << log2n;
  if (P > 1 && parts_stride < d * n) return set_error(kErrInvalid, "fgp_spec_basis: parts_stride below d n");
  const bool net = family == FGP_FAMILY_NET;
  const int64_t K = net ? n : n / 2 + 1, KS = spec_row_stride(net, log2n);
  const int NS = 1 << d;
  const int64_t per = spec_subset_bytes(family, log2n);
  const int chunk = (int)std::min<int64_t>(NS, work_bytes / per);
  if (chunk < 1) return set_error(kErrInvalid, "fgp_spec_basis: work below one subset (%lld bytes)", (long long)per);
  hipStream_t st = (hipStream_t)stream;
  char* wb = static_cast<char*>(work);
  double* prod = reinterpret_cast<double*>(wb);
  double2* spec = reinterpret_cast<double2*>(wb + 8 * n * (int64_t)chunk);
  void* scratch = wb + 24 * n * (int64_t)chunk;
  const unsigned gi = (unsigned)((n + kWG - 1) / kWG);
  for (int64_t p = 0; p < P; ++p) {
    const double* pp = parts + p * parts_stride;
    double* bp = basis + p * (int64_t)NS * KS;
    for (int s0 = 0; s0 < NS; s0 += chunk) {
      const int cnt = std::min(chunk, NS - s0);
      int rc = with_spec_d(d, [&](auto dc) {
        k_spec_products<decltype(dc)::value><<<gi, kWG, 0, st>>>(pp, n, s0, cnt, prod);
        return check_launch("k_spec_products");
      });
      if (rc != kOk) return rc;
      if (net) {
        rc = fgp_fwht(prod, n, bp + (int64_t)s0 * KS, cnt, log2n, 1, stream);
      } else {
        rc = log2n >= 17 ? fgp_fftbr_real(prod, n, spec, scratch, cnt, log2n, stream)
                         : fgp_fftbr(prod, n, 1, spec, cnt, log2n, 1, stream);
        if (rc == kOk) {
          k_spec_extract<<<dim3((unsigned)((KS + kWG - 1) / kWG), (unsigned)cnt), kWG, 0, st>>>(
              spec, n, K, KS, bp + (int64_t)s0 * KS);
          rc = check_launch("k_spec_extract");
        }
      }
      if (rc != kOk) return rc;
    }
  }
  return kOk;
}

}  // extern "C"
