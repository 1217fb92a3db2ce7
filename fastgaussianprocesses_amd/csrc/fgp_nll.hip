// Fused fit path: kernel parts, MLL forward (k1 -> lambda -> eigenvalue terms), adjoint backward
// (gradient w.r.t. raw scale / lengthscales / noise) and the Rprop step, all on device.
//
// Reference path replaced (single task, beta=kappa=0, loss_metric="MLL"):
//   k1     = scale * prod_j(1 + l_j parts_j)                  fastgps/abstract_fast_gp.py:181-191
//   lam    = ft(k1)                                           fastgps/util.py:102-112
//   ev     = sqrt(n) lam + noise; logdet = sum log|ev|        fastgps/util.py:285,292-299
//   norm   = Re sum conj(yt) yt/ev                            fastgps/util.py:354-370
//   loss   = 1/2 (norm + w logdet + d_out n log 2 pi)         fastgps/abstract_gp.py:235,253-261
//   grads  = autograd of the above                            fastgps/abstract_gp.py:294
//   Rprop  = torch.optim.Rprop(lr=0.1)                        fastgps/abstract_fast_gp.py:53-57
//
// Analytic gradient (G_e = dL/dRe(ev) + i dL/dIm(ev), Y = sum_b |yt_b|^2, w = logdet weight):
//   G_e = 1/2 conj(w/ev - Y/ev^2);  dL/dlam = sqrt(n) G_e;  g = Re(ft^H(dL/dlam)) = dL/dk1
//   dL/draw_scale = sum_i g_i k1_i;  dL/draw_l_j = sum_i g_i scale l_j p_ij prod_{m!=j}(1 + l_m p_im)
//   dL/draw_noise = noise * sum_k Re(G_e,k)
// (digital nets: everything real, ft = ft^H = fwht.)
//
// Launch structure per iteration:
//   n <= 4096 : k_iter_single  (forward + eigen terms + adjoint + gradient in ONE kernel, in LDS)
//   n >  4096 : k_fwd_rows (k1 + row transform + twiddle -> work) -> k_fwd_cols (column transform,
//               eigen terms, adjoint column transform of dL/dlambda, in place in work) -> k_bwd_rows
//               (twiddle + adjoint row transform + gradient terms).  HBM traffic per iteration:
//               16n write + (16n + 8n) read + 16n write + 16n read; the parts are read twice (8nd
//               each) or, with the lattice generator (FGP_PARTS_LATTICE), regenerated in registers.
//   then k_fit_step (one workgroup: deterministic reduction of the per-block partials, loss
//   assembly, histories, Rprop update).
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "fgp_nll.h"

namespace fgp {

// ------------------------------------------------------------------------------------------------
// kernel parts
struct PartsSpec {
  int order[FGP_MAX_D];
  double coef[FGP_MAX_D];
};

__global__ __launch_bounds__(kWG) void k_lattice_parts(const double* __restrict__ x, int64_t xs,
                                                        const double* __restrict__ z, int64_t n, int d,
                                                        PartsSpec spec, double* __restrict__ parts) {
  const int64_t i = (int64_t)blockIdx.x * kWG + threadIdx.x;
  if (i >= n) return;
  for (int j = 0; j < d; ++j) {
    const double delta = mod1(x[i * xs + j] - z[j]);
    parts[(int64_t)j * n + i] = spec.coef[j] * bernoulli(spec.order[j], delta);
  }
}

struct NetOrders {
  int order[FGP_MAX_D];   // Walsh kernel order per dimension, 1..4
};

__global__ __launch_bounds__(kWG) void k_net_parts(const int64_t* __restrict__ xb, int64_t xs,
                                                    const int64_t* __restrict__ z, int64_t n, int d, int t,
                                                    NetOrders no, double* __restrict__ parts) {
  const int64_t i = (int64_t)blockIdx.x * kWG + threadIdx.x;
  if (i >= n) return;
  for (int j = 0; j < d; ++j) {
    const unsigned long long delta = (unsigned long long)(xb[i * xs + j] ^ z[j]);
    parts[(int64_t)j * n + i] = no.order[j] == 1 ? walsh1(delta, t) : walsh_omega(no.order[j], delta, t);
  }
}

// ------------------------------------------------------------------------------------------------
// fused MLL
// ---------------------------------------------------------------- n <= 4096: one kernel
template <int P, typename T, bool EMIT, int PG>
__global__ __launch_bounds__(kWG) void k_iter_single(Nll a, const double2* __restrict__ tw) {
  constexpr int L = 1 << P, TL = L / 16, TPW = kTile / L;
  __shared__ T lds[kTile + kTile / 16];
  __shared__ T red[kWG / 64];
  __shared__ double redd[kWG / 64];
  const int tid = threadIdx.x;
  const int tr = tid / TL, tt = tid % TL;
  const int gq = blockIdx.x * TPW + tr;
  const bool live = gq < a.G;
  const int g = live ? gq : a.G - 1;
  Hyp h;
  load_hyp(a, g, h);
  fold_gen_coef<PG>(a, h);
  PSrc src;
  psrc_init(a, g, src);
  T* s = lds + tr * (L + L / 16);
  // k1 into LDS (each thread its own 16 strided elements of its transform)
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int i = tt + j * TL;
    double p[FGP_MAX_D];
    parts_one<PG, 0>(a, src, L, i, p);
    s[padi(i)] = real_to_T<T>(k1_from<0>(h, p));
  }
  __syncthreads();
  center_transform<P, false>(s, tt, 1, red, tw);
  const double rootn = sqrt((double)L), inv_rootn = 1.0 / rootn;
  if constexpr (EMIT) {
    if (live) {
      T* gl = static_cast<T*>(a.grad_lam) + (int64_t)g * L;
#pragma unroll
      for (int j = 0; j < 16; ++j) gl[tt + j * TL] = s[padi(tt + j * TL)] * inv_rootn;
    }
    return;
  }
  const double* yg = a.ysq + (int64_t)g * a.ysq_stride;
  double norm = 0.0, dnoise = 0.0;
  LogAcc la;
#pragma unroll 4
  for (int j = 0; j < 16; ++j) {
    const int k = tt + j * TL;
    const T lam = s[padi(k)] * inv_rootn;
    s[padi(k)] = eig_terms(lam, rootn, h.noise, yg[k], a.logdet_weight, norm, la, dnoise);
  }
  norm = group_sum<TL>(norm, redd);
  double logdet = group_sum<TL>(la.log_sum(LogHalf<T>::value), redd);
  dnoise = group_sum<TL>(dnoise, redd);
  __syncthreads();
  center_transform<P, true>(s, tt, 1, red, tw);
  double acc[1 + FGP_MAX_D];
#pragma unroll
  for (int q = 0; q < 1 + FGP_MAX_D; ++q) acc[q] = 0.0;
#pragma unroll 4
  for (int j = 0; j < 16; ++j) {
    const int i = tt + j * TL;
    double p[FGP_MAX_D];
    parts_one<PG, 0>(a, src, L, i, p);
    grad_terms_p<0>(h, p, re(s[padi(i)]) * inv_rootn, acc);
  }
#pragma unroll
  for (int q = 0; q < 1 + FGP_MAX_D; ++q)
    if (q <= a.d) acc[q] = group_sum<TL>(acc[q], redd) * grad_factor(h, q);
  if (live && tt == 0) {
    *part_ptr(a, g, 0, 0) = norm;
    *part_ptr(a, g, 1, 0) = logdet;
    *part_ptr(a, g, 2, 0) = dnoise;
#pragma unroll
    for (int q = 0; q < 1 + FGP_MAX_D; ++q)
      if (q <= a.d) *part_ptr(a, g, 3 + q, 0) = acc[q];
  }
}


// ---------------------------------------------------------------- n > 4096: forward row pass
template <int P2, typename T, int PG, int D>
__global__ __launch_bounds__(kWG) void k_fwd_rows(Nll a, const double2* __restrict__ tw, const double2* __restrict__ twm) {
  constexpr int N2 = 1 << P2, TL = N2 / 16, RPW = kTile / N2;
  // one row per workgroup (register-resident passes): a real 8-byte hand-over image (34.8 KB, complex
  // elements in two halves) leaves room for 4 workgroups per CU; several rows: the T-typed LDS tile
  __shared__ T lds[RPW == 1 ? 1 : kTile + kTile / 16];
  __shared__ double ldsd[RPW == 1 ? kTile + kTile / 16 : 1];
  __shared__ T red[kWG / 64];
  const int m = a.log2n, m1 = m - P2;
  const int64_t n = (int64_t)1 << m;
  const int64_t tiles = n >> kTileLog;
  const int g = (int)(blockIdx.x / tiles);
  const int row0 = (int)(blockIdx.x % tiles) * RPW;
  const int tid = threadIdx.x;
  stamp_begin(a);
  Hyp h;
  load_hyp_wave(a, g, h);
  fold_gen_coef<PG>(a, h);
  PSrc src;
  psrc_init(a, g, src);
  const int64_t base = (int64_t)row0 * N2;
  T* out = static_cast<T*>(a.work) + (int64_t)g * n;
  if constexpr (RPW == 1) {
    // register-resident row transform: k1 at the thread's 16 consecutive elements 16 tid + t (the first
    // radix-16 pass's inputs), centred by the row mean, 3 passes with 2 LDS hand-overs, output at
    // elements tid + 256 t (coalesced stores) with the inter-pass twiddle
    T v[16];
    double sum = 0.0;
    k1_run16<PG, D>(a, h, src, n, base + 16 * tid, v, sum);
    const double mean = block_sum(sum, (double*)red) * (1.0 / N2);
#pragma unroll
    for (int t = 0; t < 16; ++t) v[t] -= real_to_T<T>(mean);
    fwd_reg_passes<P2, 0, true>(v, ldsd, tid, tw);
    if (tid == 0) v[0] += real_to_T<T>(mean) * (double)N2;
    if constexpr (sizeof(T) == 16) {
      const RowTwiddle rt((unsigned)row0, tid, P2, m1, tw, twm);
#pragma unroll
      for (int k = 0; k < 16; ++k) out[work_pos(row0, tid + k * kWG, m1)] = tw_mul<T>(v[k], rt.at(k, P2, m1, tw, twm), false);
    } else {
#pragma unroll
      for (int k = 0; k < 16; ++k) out[work_pos(row0, tid + k * kWG, m1)] = v[k];
    }
    stamp_end(a);
    return;
  } else {
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      const int e = 2 * tid + 512 * kk;
      const double2 kv = k1_pair<PG, D>(a, h, src, n, base + e);
      lds[padi(e)] = real_to_T<T>(kv.x);
      lds[padi(e + 1)] = real_to_T<T>(kv.y);
    }
    __syncthreads();
    T* s = lds + (tid / TL) * (N2 + N2 / 16);
    center_transform<P2, false>(s, tid % TL, 1, red, tw);
  }
  {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int e = tid + k * kWG;
      T v = lds[padi(e)];
      if constexpr (sizeof(T) == 16) {
        const unsigned ex = brev_bits((unsigned)(row0 + (e >> P2)), m1) * (unsigned)(e & (N2 - 1));
        v = tw_mul<T>(v, inter_tw(ex, P2, m1, tw, twm), false);
      }
      out[work_pos(row0 + (e >> P2), e & (N2 - 1), m1)] = v;
    }
  }
  stamp_end(a);
}

// ---------------------------------------------------------------- n > 4096: forward column pass + eigen terms
// Column pass of the forward transform.  EMIT (fgp_nll_lam): write lambda.  Otherwise (the fit):
// eigen terms -> dL/dlambda -> the adjoint column transform of it, written back in place over the
// column tile of `work` this workgroup read (k_bwd_rows finishes the adjoint).  Per iteration the
// forward column output therefore never leaves the workgroup.
// Register-resident: thread (column c = tid mod C, tt = tid / C) keeps its 16 elements in registers
// through every radix-16 pass; LDS only hands them over between passes (reg_exchange).  The last
// forward pass and the first adjoint pass own the same elements (frequencies), so the eigen terms
// are evaluated in registers in between.
template <int P1, typename T, bool EMIT>
__global__ __launch_bounds__(kWG) void k_fwd_cols(Nll a, const double2* __restrict__ tw) {
  constexpr int N1 = 1 << P1, C = kTile / N1, CS = N1 + 1;
  constexpr int RL0 = PassRL<P1, 0>::value, R0 = 1 << RL0;
  constexpr int SL = LastPass<P1>::S, RLL = PassRL<P1, SL>::value, RLAST = 1 << RLL;
  __shared__ T lds[C * CS];
  __shared__ T part[ColPart<C>::size];
  __shared__ double redd[kWG / 64];
  const int m = a.log2n;
  const int64_t n = (int64_t)1 << m, N2 = n >> P1;
  const int64_t tiles = n >> kTileLog;
  const int g = (int)(blockIdx.x / tiles);
  const int blk = (int)(blockIdx.x % tiles);
  const int64_t c0 = (int64_t)blk * C;
  const int tid = threadIdx.x;
  const int c = tid % C, tt = tid / C;
  stamp_begin(a);
  T* wk = static_cast<T*>(a.work) + (int64_t)g * n + (int64_t)blk * kTile + c;   // contiguous tile (work_pos)
  T* col = lds + c * CS;
  T v[16];
#pragma unroll
  for (int j = 0; j < 16 / R0; ++j)
#pragma unroll
    for (int t = 0; t < R0; ++t) v[j * R0 + t] = wk[pass_pos<P1, 0, RL0>(tt, j, t) * C];
  double y[16];
  if constexpr (!EMIT) {   // Y at the frequencies this thread ends the forward transform on: in flight early
    const double* yg = a.ysq + (int64_t)g * a.ysq_stride + c0 + c;
#pragma unroll
    for (int j = 0; j < 16 / RLAST; ++j)
#pragma unroll
      for (int t = 0; t < RLAST; ++t) y[j * RLAST + t] = yg[(int64_t)pass_pos<P1, SL, RLL>(tt, j, t) * N2];
  }
  T sum = zero_v<T>();
#pragma unroll
  for (int k = 0; k < 16; ++k) sum += v[k];
  column_partials<C>(sum, part);
  T mean = column_total<C>(c, part) * (1.0 / N1);
#pragma unroll
  for (int k = 0; k < 16; ++k) v[k] -= mean;
  fwd_reg_passes<P1, 0, false>(v, col, tt, tw);
  if (tt == 0) v[0] += mean * (double)N1;          // frequency 0 (AbstractFastGP.ft's mean)
  const double rootn = sqrt((double)n), inv_rootn = 1.0 / rootn;
  if constexpr (EMIT) {   // lambda = ft(k1) (fgp_nll_lam)
    T* gl = static_cast<T*>(a.grad_lam) + (int64_t)g * n + c0 + c;
#pragma unroll
    for (int j = 0; j < 16 / RLAST; ++j)
#pragma unroll
      for (int t = 0; t < RLAST; ++t)
        gl[(int64_t)pass_pos<P1, SL, RLL>(tt, j, t) * N2] = v[j * RLAST + t] * inv_rootn;
    stamp_end(a);
    return;
  }
  Hyp h;
  load_hyp_wave(a, g, h);
  double norm = 0.0, dnoise = 0.0;
  LogAcc la;
  sum = zero_v<T>();
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    v[k] = eig_terms(v[k] * inv_rootn, rootn, h.noise, y[k], a.logdet_weight, norm, la, dnoise);
    sum += v[k];
  }
  double logdet = la.log_sum(LogHalf<T>::value);
  column_partials<C>(sum, part);
  mean = column_total<C>(c, part) * (1.0 / N1);
#pragma unroll
  for (int k = 0; k < 16; ++k) v[k] -= mean;
  adj_reg_passes<P1, SL, false>(v, col, tt, tw);   // adjoint (WHT: self-adjoint, w = 1)
  if (tt == 0) v[0] += mean * (double)N1;
#pragma unroll
  for (int j = 0; j < 16 / R0; ++j)
#pragma unroll
    for (int t = 0; t < R0; ++t) wk[pass_pos<P1, 0, RL0>(tt, j, t) * C] = v[j * R0 + t];
  norm = block_sum(norm, redd);
  logdet = block_sum(logdet, redd);
  dnoise = block_sum(dnoise, redd);
  if (tid == 0) {
    *part_ptr(a, g, 0, blk) = norm;
    *part_ptr(a, g, 1, blk) = logdet;
    *part_ptr(a, g, 2, blk) = dnoise;
  }
  stamp_end(a);
}

// ---------------------------------------------------------------- n > 4096: adjoint row pass + gradient terms
template <int P2, typename T, int PG, int D>
__global__ __launch_bounds__(kWG) void k_bwd_rows(Nll a, const double2* __restrict__ tw, const double2* __restrict__ twm) {
  constexpr int N2 = 1 << P2, TL = N2 / 16, RPW = kTile / N2;
  constexpr bool FFT = sizeof(T) == 16;   // FFT: adjoint network + conj twiddle; WHT: self-adjoint
  __shared__ T lds[RPW == 1 ? 1 : kTile + kTile / 16];           // (as k_fwd_rows)
  __shared__ double ldsd[RPW == 1 ? kTile + kTile / 16 : 1];
  __shared__ T red[kWG / 64];
  __shared__ double redd[kWG / 64];
  const int m = a.log2n, m1 = m - P2;
  const int64_t n = (int64_t)1 << m;
  const int64_t tiles = n >> kTileLog;
  const int g = (int)(blockIdx.x / tiles);
  const int blk = (int)(blockIdx.x % tiles);
  const int row0 = blk * RPW;
  const int64_t base = (int64_t)blk * kTile;
  const int tid = threadIdx.x;
  stamp_begin(a);
  const T* in = static_cast<const T*>(a.work) + (int64_t)g * n;   // column-tile layout (work_pos)
  if constexpr (RPW == 1) {
    T v[16];
    T sum = zero_v<T>();
    if constexpr (FFT) {
      const RowTwiddle rt((unsigned)row0, tid, P2, m1, tw, twm);
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        v[k] = tw_mul<T>(in[work_pos(row0, tid + k * kWG, m1)], rt.at(k, P2, m1, tw, twm), true);
        sum += v[k];
      }
    } else {
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        v[k] = in[work_pos(row0, tid + k * kWG, m1)];
        sum += v[k];
      }
    }
    const T mean = block_sum_t(sum, red) * (1.0 / N2);
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] -= mean;
    // register-resident adjoint row transform: the loaded elements tid + 256 k are the first DIF
    // pass's; 3 passes with 2 LDS hand-overs end on the elements 16 tid + t (WHT: self-adjoint)
    adj_reg_passes<P2, LastPass<P2>::S, true>(v, ldsd, tid, tw);
    if (tid == 0) v[0] += mean * (double)N2;
    Hyp h;
    load_hyp_wave(a, g, h);
    fold_gen_coef<PG>(a, h);
    PSrc src;
    psrc_init(a, g, src);
    constexpr int ND = Dims<D>::N;
    double acc[1 + ND];
#pragma unroll
    for (int q = 0; q < 1 + ND; ++q) acc[q] = 0.0;
    double* gl = ldsd + 17 * tid;                             // the thread's private slots
    __syncthreads();                                          // last hand-over's readers are done
#pragma unroll
    for (int t = 0; t < 16; ++t) gl[t] = re(v[t]);
    grad_run16<PG, D>(a, h, src, n, base + 16 * tid, gl, 1.0 / sqrt((double)n), acc);
#pragma unroll
    for (int q = 0; q < 1 + ND; ++q) {
      if (q <= a.d) {
        const double r = block_sum(acc[q], redd) * grad_factor(h, q);
        if (tid == 0) *part_ptr(a, g, 3 + q, blk) = r;
      }
    }
    stamp_end(a);
    return;
  } else {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int e = tid + k * kWG;
      T v = in[work_pos(row0 + (e >> P2), e & (N2 - 1), m1)];
      if constexpr (FFT) {
        const unsigned ex = brev_bits((unsigned)(row0 + (e >> P2)), m1) * (unsigned)(e & (N2 - 1));
        v = tw_mul<T>(v, inter_tw(ex, P2, m1, tw, twm), true);
      }
      lds[padi(e)] = v;
    }
    __syncthreads();
    T* s = lds + (tid / TL) * (N2 + N2 / 16);
    center_transform<P2, FFT>(s, tid % TL, 1, red, tw);
  }
  Hyp h;
  load_hyp_wave(a, g, h);
  fold_gen_coef<PG>(a, h);
  PSrc src;
  psrc_init(a, g, src);
  const double inv_rootn = 1.0 / sqrt((double)n);
  constexpr int ND = Dims<D>::N;
  double acc[1 + ND];
#pragma unroll
  for (int q = 0; q < 1 + ND; ++q) acc[q] = 0.0;
#pragma unroll 2
  for (int kk = 0; kk < 8; ++kk) {
    const int e = 2 * tid + 512 * kk;
    double p0[ND], p1[ND];
    parts_pair<PG, D>(a, src, n, base + e, p0, p1);
    grad_terms_p<D>(h, p0, re(lds[padi(e)]) * inv_rootn, acc);
    grad_terms_p<D>(h, p1, re(lds[padi(e + 1)]) * inv_rootn, acc);
  }
#pragma unroll
  for (int q = 0; q < 1 + ND; ++q) {
    if (q <= a.d) {
      const double v = block_sum(acc[q], redd) * grad_factor(h, q);
      if (tid == 0) *part_ptr(a, g, 3 + q, blk) = v;
    }
  }
  stamp_end(a);
}

// ---------------------------------------------------------------- half-length (R2C) lattice fit, n >= 2^17
// k1 is real, so the length-n bit-reversed-input FFT is done at half length (Stockham-free packing):
// with a = x[brev_m], a[2j] = x[brev_{m-1}(j)] and a[2j+1] = x[n/2 + brev_{m-1}(j)], hence
//   fftbr_n(x)[k], [k + n/2] = 1/2 (Z_k + conj Z_{n/2-k}) -/+ 1/2 i w_n^k (Z_k - conj Z_{n/2-k}),
//   Z = fftbr_{n/2}(x[:n/2] + i x[n/2:]),
// the existing engine at m - 1.  lambda, Y and dL/dlambda are Hermitian, so the adjoint needs no mirror:
// with E_k = G_k + G_{k+n/2}, O_k = (G_k - G_{k+n/2}) conj(w_n^k), the adjoint half-length transform of
// V = E + i O is grad_lo + i grad_hi (both real).  The mirror k <-> n/2 - k of the forward is column
// c <-> N2 - c with rows reversed: the intermediate is stored in paired column tiles (work_pos_pair),
// so both partners sit in one column workgroup and meet through one LDS exchange.
//
// Paired tile layout of the N1 x N2 half-length intermediate (C = kTile / N1 slots per tile, HC = C/2
// pair-columns): tile b holds the pair-columns q < HC, i.e. columns c = b HC + q in slots q and their
// mirrors N2 - c in slots HC + q -- except tile 0's pair-column 0, which holds the self-mirrored
// columns 0 (slot 0) and N2/2 (slot HC).  A row's consecutive columns c < N2/2 are therefore
// consecutive slots (runs of HC elements = 256 B at C = 32), and so are its columns > N2/2 (in
// descending order): the row kernels' 16-B-per-lane accesses are contiguous.
__device__ __forceinline__ int64_t work_pos_pair(int64_t u, int64_t k, int P1, int64_t N2) {
  const int CL = kTileLog - P1;
  const int64_t h = N2 >> 1;
  int64_t tile, slot;
  if (k == h) {
    tile = 0;
    slot = (int64_t)1 << (CL - 1);
  } else {
    const int64_t c = k < h ? k : N2 - k;     // (k = 0: c = 0, tile 0, slot 0)
    tile = c >> (CL - 1);
    slot = (c & ((1 << (CL - 1)) - 1)) + (k > h ? ((int64_t)1 << (CL - 1)) : 0);
  }
  return (tile << kTileLog) + (u << CL) + slot;
}

// A row of N2 = 16 kWG reals staged in the row kernels' ldsd (kTile + kTile/16 doubles): element p at
// run_pad(p), each thread's run of 16 padded to 17 (thread t's run starts at kRunPad t).
constexpr int kRunPad = 17;
__device__ __forceinline__ int run_pad(int p) { return p + (p >> 4); }

template <int PG, int D>
__global__ __launch_bounds__(kWG) void k_fwd_rows_r2c(Nll a, const double2* __restrict__ tw, const double2* __restrict__ twm) {
  constexpr int P2 = 12, N2 = 1 << P2;
  __shared__ double ldsd[kTile + kTile / 16];
  __shared__ double2 red[kWG / 64];
  const int mt = a.log2n - 1, m1 = mt - P2;
  const int64_t n = (int64_t)1 << a.log2n, nt = n >> 1;
  const int64_t tiles = nt >> kTileLog;
  const int g = (int)(blockIdx.x / tiles);
  const int row0 = (int)(blockIdx.x % tiles);
  const int tid = threadIdx.x;
  stamp_begin(a);
  Hyp h;
  load_hyp_wave(a, g, h);
  fold_gen_coef<PG>(a, h);
  PSrc src;
  psrc_init(a, g, src);
  const int64_t base = (int64_t)row0 * N2;
  double2* out = static_cast<double2*>(a.work) + (int64_t)g * n;
  double lo[16], hi[16];
  double slo = 0.0, shi = 0.0;
  k1_run16<PG, D>(a, h, src, n, base + 16 * tid, lo, slo);        // x[:n/2] -> real parts
  k1_run16<PG, D>(a, h, src, n, nt + base + 16 * tid, hi, shi);   // x[n/2:] -> imaginary parts
  double2 v[16];
#pragma unroll
  for (int t = 0; t < 16; ++t) v[t] = make_double2(lo[t], hi[t]);
  const double2 mean = block_sum_t(make_double2(slo, shi), red) * (1.0 / N2);
#pragma unroll
  for (int t = 0; t < 16; ++t) v[t] -= mean;
  fwd_reg_passes<P2, 0, true>(v, ldsd, tid, tw);
  if (tid == 0) v[0] += mean * (double)N2;
  const RowTwiddle rt((unsigned)row0, tid, P2, m1, tw, twm);
#pragma unroll
  for (int k = 0; k < 16; ++k)
    out[work_pos_pair(row0, tid + k * kWG, m1, N2)] = tw_mul<double2>(v[k], rt.at(k, P2, m1, tw, twm), false);
  stamp_end(a);
}

// The same row pass on a REAL input array (fgp_fftbr_real): x[:n/2] + i x[n/2:] of problem g read as
// 16-byte pairs instead of generated k1 (T = float: fp32 rows widened exactly on load, fgp_fftbr_real_half_f32).
template <typename T>
__global__ __launch_bounds__(kWG) void k_fwd_rows_r2c_in(const T* __restrict__ in, int64_t in_stride, int log2n,
                                                         double2* __restrict__ work, const double2* __restrict__ tw,
                                                         const double2* __restrict__ twm) {
  constexpr int P2 = 12, N2 = 1 << P2;
  __shared__ double ldsd[kTile + kTile / 16];
  __shared__ double2 red[kWG / 64];
  const int mt = log2n - 1, m1 = mt - P2;
  const int64_t n = (int64_t)1 << log2n, nt = n >> 1;
  const int64_t tiles = nt >> kTileLog;
  const int64_t g = blockIdx.x / tiles;
  const int row0 = (int)(blockIdx.x % tiles);
  const int tid = threadIdx.x;
  const T* x = in + g * in_stride + (int64_t)row0 * N2;
  double2 v[16];
  double2 sum = make_double2(0.0, 0.0);
  // thread t takes elements 16 t .. 16 t + 15 of x[:n/2] (Re) and x[n/2:] (Im); both halves are loaded
  // lane-consecutive (16 B per lane) and handed over through LDS (loading a thread's run directly puts the
  // lanes 128 B apart)
  constexpr int VW = 16 / sizeof(T), NL = 16 / VW;   // elements per 16-B load, loads per half
  using VT = typename std::conditional<sizeof(T) == 8, double2, float4>::type;
  VT lo[NL], hi[NL];
#pragma unroll
  for (int u = 0; u < NL; ++u) {
    lo[u] = *reinterpret_cast<const VT*>(x + VW * (tid + kWG * u));
    hi[u] = *reinterpret_cast<const VT*>(x + nt + VW * (tid + kWG * u));
  }
#pragma unroll
  for (int half = 0; half < 2; ++half) {
#pragma unroll
    for (int u = 0; u < NL; ++u) {
      const int a = run_pad(VW * (tid + kWG * u));
      const VT w = half ? hi[u] : lo[u];
      if constexpr (sizeof(T) == 8) {
        ldsd[a] = w.x;
        ldsd[a + 1] = w.y;
      } else {
        ldsd[a] = (double)w.x;
        ldsd[a + 1] = (double)w.y;
        ldsd[a + 2] = (double)w.z;
        ldsd[a + 3] = (double)w.w;
      }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      if (half) v[k].y = ldsd[kRunPad * tid + k];
      else v[k].x = ldsd[kRunPad * tid + k];
    }
    __syncthreads();
  }
#pragma unroll
  for (int t = 0; t < 16; ++t) sum += v[t];
  const double2 mean = block_sum_t(sum, red) * (1.0 / N2);
#pragma unroll
  for (int t = 0; t < 16; ++t) v[t] -= mean;
  fwd_reg_passes<P2, 0, true>(v, ldsd, tid, tw);
  if (tid == 0) v[0] += mean * (double)N2;
  const RowTwiddle rt((unsigned)row0, tid, P2, m1, tw, twm);
  double2* out = work + g * n;
#pragma unroll
  for (int k = 0; k < 16; ++k)
    out[work_pos_pair(row0, tid + k * kWG, m1, N2)] = tw_mul<double2>(v[k], rt.at(k, P2, m1, tw, twm), false);
}

// The same row pass on the products of a subset of the kernel parts (the spectral basis, fgp_spec_basis):
// workgroup (row, c) forms b_S = prod_{j in S} parts_j (S = s0 + c, ascending j from 1.0 -- the products
// of k_spec_products bit for bit) for its row in registers, instead of a products array written and read
// back.  Subsets fastest in the grid: a row's parts are read from L2 by every subset's workgroup.
template <int D>
__global__ __launch_bounds__(kWG) void k_fwd_rows_r2c_prod(const double* __restrict__ parts, int log2n, int s0,
                                                           int cnt, double2* __restrict__ work,
                                                           const double2* __restrict__ tw,
                                                           const double2* __restrict__ twm) {
  constexpr int P2 = 12, N2 = 1 << P2;
  __shared__ double ldsd[kTile + kTile / 16];
  __shared__ double2 red[kWG / 64];
  const int mt = log2n - 1, m1 = mt - P2;
  const int64_t n = (int64_t)1 << log2n, nt = n >> 1;
  // XCD-aware order (speed only): workgroups b and b + 8 share an XCD, so with (rows of the grid) % 8 == 0 the
  // cnt subsets of a row go to ONE XCD, consecutively -- its parts cross the fabric into that XCD's L2 once
  // instead of once per XCD
  const unsigned rows = gridDim.x / (unsigned)cnt;
  int c, row0;
  if (rows % 8u == 0u) {
    const unsigned xcd = blockIdx.x & 7u, local = blockIdx.x >> 3;
    c = (int)(local % (unsigned)cnt);
    row0 = (int)((local / (unsigned)cnt) * 8u + xcd);
  } else {
    c = (int)(blockIdx.x % (unsigned)cnt);
    row0 = (int)(blockIdx.x / (unsigned)cnt);
  }
  const int S = s0 + c;
  const int tid = threadIdx.x;
  const double* x = parts + (int64_t)row0 * N2 + 16 * tid;
  double2 v[16];
#pragma unroll
  for (int t = 0; t < 16; ++t) v[t] = make_double2(1.0, 1.0);
#pragma unroll
  for (int j = 0; j < D; ++j) {
    if ((S >> j) & 1) {                      // uniform over the workgroup
      const double* xj = x + (int64_t)j * n;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const double2 lo = *reinterpret_cast<const double2*>(xj + 2 * u);
        const double2 hi = *reinterpret_cast<const double2*>(xj + nt + 2 * u);
        v[2 * u].x *= lo.x;
        v[2 * u + 1].x *= lo.y;
        v[2 * u].y *= hi.x;
        v[2 * u + 1].y *= hi.y;
      }
    }
  }
  double2 sum = make_double2(0.0, 0.0);
#pragma unroll
  for (int t = 0; t < 16; ++t) sum += v[t];
  const double2 mean = block_sum_t(sum, red) * (1.0 / N2);
#pragma unroll
  for (int t = 0; t < 16; ++t) v[t] -= mean;
  fwd_reg_passes<P2, 0, true>(v, ldsd, tid, tw);
  if (tid == 0) v[0] += mean * (double)N2;
  const RowTwiddle rt((unsigned)row0, tid, P2, m1, tw, twm);
  double2* out = work + (int64_t)c * n;
#pragma unroll
  for (int k = 0; k < 16; ++k)
    out[work_pos_pair(row0, tid + k * kWG, m1, N2)] = tw_mul<double2>(v[k], rt.at(k, P2, m1, tw, twm), false);
}

// Mirror-pair evaluation of the R2C column kernel.  The pair (k, nt - k) of the half-length spectrum Z
// (primary Z_k = zk, partner Z_{nt-k} = zm, W = w_n^k) gives the length-n spectrum at k and k + n/2:
//   A0, A1 = (S -/+ i W D) / 2,  S = Z_k + conj Z_{nt-k},  D = Z_k - conj Z_{nt-k}
// (lambda = A / sqrt(n)); the partner's frequencies nt - k, n - k are their mirrors (lambda Hermitian).
// Returns dL/dlambda at k and k + n/2 (g0, g1) and accumulates that pair's loss terms.
struct EigAcc {
  double norm = 0.0, dnoise = 0.0;
  LogAcc la;
};

__device__ __forceinline__ void pair_eval(double2 zk, double2 zm, double2 W, double y0, double y1, double rootn,
                                          double inv_rootn, double noise, double wlog, EigAcc& acc, double2& g0,
                                          double2& g1, double2& A0, double2& A1) {
  const double2 S = make_double2(zk.x + zm.x, zk.y - zm.y);      // Z_k + conj Z_{nt-k}
  const double2 Dd = make_double2(zk.x - zm.x, zk.y + zm.y);     // Z_k - conj Z_{nt-k}
  const double2 wd = cmul(W, Dd);
  A0 = make_double2(0.5 * (S.x + wd.y), 0.5 * (S.y - wd.x));     // (S - i W D) / 2
  A1 = make_double2(0.5 * (S.x - wd.y), 0.5 * (S.y + wd.x));     // (S + i W D) / 2
  g0 = eig_terms(A0 * inv_rootn, rootn, noise, y0, wlog, acc.norm, acc.la, acc.dnoise);
  g1 = eig_terms(A1 * inv_rootn, rootn, noise, y1, wlog, acc.norm, acc.la, acc.dnoise);
}

// Column pass at half length + mirror exchange + split into the length-n spectrum + eigen terms + the
// adjoint packing V = E + i O + adjoint column pass, in place (k_fwd_cols for the R2C layout).
//
// Exact Hermitian symmetry, each mirror pair evaluated ONCE: after the forward passes the tile's
// spectrum goes to the LDS image; thread (q, rr) then takes the pairs of pair-column q (slots q,
// HC + q = columns c and N2 - c) at rows rr, rr + RSTEP, ...: from (Z_k, Z_{nt-k}, w_n^k, Y_k,
// Y_{k+n/2}) it evaluates the eigen terms of k and k + n/2 once and writes both elements' V back into
// the image: the primary's V = E + i O, E = G_k + G_{k+n/2}, O = (G_k - G_{k+n/2}) conj(w_n^k), and the
// partner's, whose G are the conjugates of the primary's (swapped) and whose twiddle is -conj(w_n^k):
// V' = (E.x + O.y, O.x - E.y), bit for bit the conjugate arithmetic.  So dL/dlambda is exactly
// Hermitian and the half-length adjoint of V has no leak of a rounding-level anti-Hermitian part
// (amplified by 1/ev^2 near the nugget) into the gradient.  A regular pair's loss terms count twice
// (its mirror frequencies); the self-mirrored frequencies 0, n/2 (column 0, row 0) and n/4, 3n/4
// (column 0, row N1/2) once.  Tile 0's pair-column 0 holds the self-mirrored columns 0 (rows r <->
// N1 - r) and N2/2 (rows r <-> N1 - 1 - r): its job rr < N1/2 is a column-0 pair (rr = 0: the two
// self pairs), rr >= N1/2 a column-N2/2 pair.
// Lanes run over q (consecutive columns: coalesced Y reads; the image reads of consecutive lanes fall
// on distinct bank quads).  Y for the thread's jobs is loaded before the forward passes.
template <int P1, int OUT>
__global__ __launch_bounds__(kWG, 2) void k_fwd_cols_r2c(Nll a, const double2* __restrict__ tw,
                                                          const double2* __restrict__ twmf) {
  constexpr int N1 = 1 << P1, C = kTile / N1, CS = N1 + 1, HC = C / 2;
  constexpr int RL0 = PassRL<P1, 0>::value, R0 = 1 << RL0;
  constexpr int SL = LastPass<P1>::S, RLL = PassRL<P1, SL>::value, RLAST = 1 << RLL;
  constexpr int JOBS = kTile / 2 / kWG, RSTEP = kWG / HC;     // JOBS * RSTEP = N1
  static_assert(JOBS * RSTEP == N1, "pair jobs cover the tile");
  __shared__ double2 lds[C * CS];
  __shared__ double2 part[ColPart<C>::size];
  __shared__ double redd[kWG / 64];
  const int m = a.log2n;
  const int64_t n = (int64_t)1 << m, nt = n >> 1, N2 = nt >> P1;
  const int64_t tiles = nt >> kTileLog;
  const int g = (int)(blockIdx.x / tiles);
  const int blk = (int)(blockIdx.x % tiles);
  const int tid = threadIdx.x;
  const int sl = tid % C, tt = tid / C;
  stamp_begin(a);
  double2* wk = static_cast<double2*>(a.work) + (int64_t)g * n + (int64_t)blk * kTile + sl;
  double2* col = lds + sl * CS;
  // pair jobs of this thread: pair-column q, rows rr0 + RSTEP j
  const int q = tid % HC, rr0 = tid / HC;
  const bool col0 = blk == 0 && q == 0;                      // tile 0's self-mirrored columns
  const int64_t cp_gen = (int64_t)blk * HC + q;              // primary column (q >= 1 or blk >= 1)
  const double* yg = a.ysq + (int64_t)g * a.ysq_stride;
  // primary (slot, row, column) of job j
  auto job_primary = [&](int j, int& sp, int& rp, int64_t& cp) {
    const int rr = rr0 + RSTEP * j;
    if (!col0) {
      sp = q; rp = rr; cp = cp_gen;
    } else if (rr < N1 / 2) {
      sp = 0; rp = rr; cp = 0;
    } else {
      sp = HC; rp = rr - N1 / 2; cp = N2 >> 1;
    }
  };
  double y0[JOBS], y1[JOBS];
  if constexpr (OUT == 0) {
#pragma unroll
    for (int j = 0; j < JOBS; ++j) {
      int sp, rp;
      int64_t cp;
      job_primary(j, sp, rp, cp);
      const double* yk = yg + cp + (int64_t)rp * N2;
      y0[j] = yk[0];
      y1[j] = yk[nt];
    }
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
  double2 mean = column_total<C>(sl, part) * (1.0 / N1);
#pragma unroll
  for (int k = 0; k < 16; ++k) v[k] -= mean;
  fwd_reg_passes<P1, 0, false>(v, col, tt, tw);
  if (tt == 0) v[0] += mean * (double)N1;
  // the tile's half-length spectrum into the image
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 16 / RLAST; ++j)
#pragma unroll
    for (int t = 0; t < RLAST; ++t) col[pass_pos<P1, SL, RLL>(tt, j, t)] = v[j * RLAST + t];
  __syncthreads();
  const double rootn = sqrt((double)n), inv_rootn = 1.0 / rootn;
  Hyp h;
  if constexpr (OUT == 0) load_hyp_wave(a, g, h);
  EigAcc acc2, acc1;          // regular pairs (weight 2), self-mirrored frequencies (weight 1)
  double2* gl = OUT == 1 ? static_cast<double2*>(a.grad_lam) + (int64_t)g * n : nullptr;
  double* gb = OUT == 2 ? static_cast<double*>(a.grad_lam) + (int64_t)g * 64 : nullptr;   // basis + (s0 + g) 64
  double2* gh = OUT == 3 ? static_cast<double2*>(a.grad_lam) + (int64_t)g * a.out_stride : nullptr;   // k <= n/2
  const int ns = 1 << a.d;
  const double2 wcp = twmf[col0 ? 0 : cp_gen];
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
    const bool self = col0 && sp == 0 && rp == 0;   // frequencies 0, n/2 and (second pair) n/4, 3n/4
    const double2 wc = col0 ? twmf[cp] : wcp;
    const double2 W = cmul(wc, tw[rp << (24 - m)]);                 // w_n^k, k = cp + N2 rp
    double2* ip = lds + sp * CS + rp;
    double2* is = lds + ss * CS + rs;
    const double2 zk = *ip, zm = *is;
    double2 g0, g1, A0, A1;
    double ya = 0.0, yb = 0.0;
    if constexpr (OUT == 0) {
      ya = y0[j];
      yb = y1[j];
    }
    EigAcc& ac = self ? acc1 : acc2;
    pair_eval(zk, zm, W, ya, yb, rootn, inv_rootn, h.noise, a.logdet_weight, ac, g0, g1, A0, A1);
    if constexpr (OUT == 1) {   // lambda at k, k + n/2 and (conjugates, swapped) at the partner's nt - k, n - k
      const int64_t kp = cp + (int64_t)rp * N2;
      gl[kp] = A0 * inv_rootn;
      gl[kp + nt] = A1 * inv_rootn;
      if (!self) {
        const int64_t ks = (col0 ? cp : N2 - cp) + (int64_t)rs * N2;
        gl[ks] = make_double2(A1.x, -A1.y) * inv_rootn;
        gl[ks + nt] = make_double2(A0.x, -A0.y) * inv_rootn;
      }
    } else if constexpr (OUT == 2) {   // the real parts at k <= n/2 only, into the chunked spectra
      const int64_t kp = cp + (int64_t)rp * N2;
      gb[spec_pos(kp, ns)] = A0.x * inv_rootn;
      if (kp == 0) gb[spec_pos(nt, ns)] = A1.x * inv_rootn;                 // the Nyquist frequency n/2
      if (!self) gb[spec_pos((col0 ? cp : N2 - cp) + (int64_t)rs * N2, ns)] = A1.x * inv_rootn;
    } else if constexpr (OUT == 3) {   // OUT == 1's values at k <= n/2 only (the Hermitian half of ft(real))
      const int64_t kp = cp + (int64_t)rp * N2;
      gh[kp] = A0 * inv_rootn;
      if (kp == 0) gh[nt] = A1 * inv_rootn;
      if (!self) gh[(col0 ? cp : N2 - cp) + (int64_t)rs * N2] = make_double2(A1.x, -A1.y) * inv_rootn;
    } else {
      const double2 E = g0 + g1;
      const double2 O = cmulc(g0 - g1, W);
      *ip = make_double2(E.x - O.y, E.y + O.x);                     // V = E + i O
      if (!self) *is = make_double2(E.x + O.y, O.x - E.y);          // the partner's (conjugate arithmetic)
    }
    if (self) {   // the second self-mirrored element of column 0: row N1/2 (frequencies n/4, 3n/4)
      constexpr int rh = N1 / 2;
      double2* ih = lds + rh;
      const double2 zh = *ih;
      const double2 Wh = tw[rh << (24 - m)];
      double yc = 0.0, yd = 0.0;
      if constexpr (OUT == 0) {
        yc = yg[(int64_t)rh * N2];
        yd = yg[(int64_t)rh * N2 + nt];
      }
      pair_eval(zh, zh, Wh, yc, yd, rootn, inv_rootn, h.noise, a.logdet_weight, acc1, g0, g1, A0, A1);
      if constexpr (OUT == 1) {
        gl[(int64_t)rh * N2] = A0 * inv_rootn;
        gl[(int64_t)rh * N2 + nt] = A1 * inv_rootn;
      } else if constexpr (OUT == 2) {
        gb[spec_pos((int64_t)rh * N2, ns)] = A0.x * inv_rootn;              // n/4 (3n/4 is past n/2)
      } else if constexpr (OUT == 3) {
        gh[(int64_t)rh * N2] = A0 * inv_rootn;
      } else {
        const double2 E = g0 + g1;
        const double2 O = cmulc(g0 - g1, Wh);
        *ih = make_double2(E.x - O.y, E.y + O.x);
      }
    }
  }
  if constexpr (OUT != 0) {
    stamp_end(a);
    return;
  }
  double norm = 2.0 * acc2.norm + acc1.norm;
  double dnoise = 2.0 * acc2.dnoise + acc1.dnoise;
  double logdet = 2.0 * acc2.la.log_sum(0.5) + acc1.la.log_sum(0.5);
  __syncthreads();
  sum = zero_v<double2>();
#pragma unroll
  for (int j = 0; j < 16 / RLAST; ++j)
#pragma unroll
    for (int t = 0; t < RLAST; ++t) {
      v[j * RLAST + t] = col[pass_pos<P1, SL, RLL>(tt, j, t)];
      sum += v[j * RLAST + t];
    }
  column_partials<C>(sum, part);
  mean = column_total<C>(sl, part) * (1.0 / N1);
#pragma unroll
  for (int k = 0; k < 16; ++k) v[k] -= mean;
  adj_reg_passes<P1, SL, false>(v, col, tt, tw);
  if (tt == 0) v[0] += mean * (double)N1;
#pragma unroll
  for (int j = 0; j < 16 / R0; ++j)
#pragma unroll
    for (int t = 0; t < R0; ++t) wk[pass_pos<P1, 0, RL0>(tt, j, t) * C] = v[j * R0 + t];
  norm = block_sum(norm, redd);
  logdet = block_sum(logdet, redd);
  dnoise = block_sum(dnoise, redd);
  if (tid == 0) {
    *part_ptr(a, g, 0, blk) = norm;
    *part_ptr(a, g, 1, blk) = logdet;
    *part_ptr(a, g, 2, blk) = dnoise;
  }
  stamp_end(a);
}

// ---------------------------------------------------------------- half-length real-output inverse
// x = Re ifftbr_n(X) (orthonormal) for a spectrum X [n] (fgp_ifftbr_real): the adjoint of the packed
// forward above.  With X~ the Hermitian part of X (X~_k = (X_k + conj X_{n-k}) / 2: Re ifftbr(X) =
// ifftbr(X~) exactly), V_k = E + i O, E = X~_k + X~_{k+n/2}, O = (X~_k - X~_{k+n/2}) conj(w_n^k), and
//   x[:n/2] + i x[n/2:] = DFT_{n/2}^H(V) / sqrt(n)
// (the fit kernels' V packing with X in place of dL/dlambda).  The column kernel takes each mirror pair
// (k, k + n/2; n/2 - k, n - k) once -- reading the four values, so X~ is the exact Hermitian part --
// writes V of both partners into the LDS image and runs the adjoint column pass; the row kernel runs the
// conjugate-twiddled adjoint row pass and writes the real rows.  f (optional): X = in * f, fused into the
// loads (the tilde-domain solve of gram_matrix_solve, util.py:341-343); FR: f holds real factor rows
// (float64: A = 1/ev of real eigenvalues, fgp_ifftbr_real_rf), else complex128.  HERM (with FR): X is
// Hermitian (ytilde = ft of real data times a real even factor), so X~ = X, X~_{k+n/2} = conj X_{n/2-k} and
// only k <= n/2 of `in` and `f` are read (half the input bytes).
template <int P1, bool FR, bool HERM>
__global__ __launch_bounds__(kWG, 2) void k_inv_cols_c2r(const double2* __restrict__ X, int64_t xs,
                                                         const void* __restrict__ f, int64_t fs,
                                                         double2* __restrict__ work, int log2n,
                                                         const double2* __restrict__ tw,
                                                         const double2* __restrict__ twmf) {
  constexpr int N1 = 1 << P1, C = kTile / N1, CS = N1 + 1, HC = C / 2;
  constexpr int RL0 = PassRL<P1, 0>::value, R0 = 1 << RL0;
  constexpr int SL = LastPass<P1>::S, RLL = PassRL<P1, SL>::value, RLAST = 1 << RLL;
  constexpr int JOBS = kTile / 2 / kWG, RSTEP = kWG / HC;     // JOBS * RSTEP = N1
  static_assert(JOBS * RSTEP == N1, "pair jobs cover the tile");
  __shared__ double2 lds[C * CS];
  __shared__ double2 part[ColPart<C>::size];
  const int m = log2n;
  const int64_t n = (int64_t)1 << m, nt = n >> 1, N2 = nt >> P1;
  const int64_t tiles = nt >> kTileLog;
  const int64_t g = blockIdx.x / tiles;
  const int blk = (int)(blockIdx.x % tiles);
  const int tid = threadIdx.x;
  const int sl = tid % C, tt = tid / C;
  double2* col = lds + sl * CS;
  const int q = tid % HC, rr0 = tid / HC;
  const bool col0 = blk == 0 && q == 0;                      // tile 0's self-mirrored columns
  const int64_t cp_gen = (int64_t)blk * HC + q;
  const double2* xg = X + g * xs;
  const double2* fg = (f && !FR) ? static_cast<const double2*>(f) + g * fs : nullptr;
  const double* fr = (f && FR) ? static_cast<const double*>(f) + g * fs : nullptr;
  auto xv = [&](int64_t k) {
    const double2 v = xg[k];
    if constexpr (FR) {
      return fr ? make_double2(v.x * fr[k], v.y * fr[k]) : v;
    } else {
      return fg ? cmul(v, fg[k]) : v;
    }
  };
  // Hermitian part at (k, k + n/2) given the partner pair (n/2 - k, n - k): X~_k, X~_{k+n/2}
  auto herm = [&](int64_t k, int64_t ks, double2& h0, double2& h1) {
    if constexpr (HERM) {
      h0 = xv(k);
      const double2 b0 = xv(ks);
      h1 = make_double2(b0.x, -b0.y);
    } else {
      const double2 a0 = xv(k), a1 = xv(k + nt), b0 = xv(ks), b1 = xv(ks + nt);   // X_k, X_{k+nt}, X_{nt-k}, X_{n-k}
      h0 = make_double2(0.5 * (a0.x + b1.x), 0.5 * (a0.y - b1.y));
      h1 = make_double2(0.5 * (a1.x + b0.x), 0.5 * (a1.y - b0.y));
    }
  };
  auto vpack = [](double2 h0, double2 h1, double2 W, double2& vp, double2& vs) {
    const double2 E = h0 + h1;
    const double2 O = cmulc(h0 - h1, W);
    vp = make_double2(E.x - O.y, E.y + O.x);                        // V = E + i O
    vs = make_double2(E.x + O.y, O.x - E.y);                        // the partner's (conjugate arithmetic)
  };
  const double2 wcp = twmf[col0 ? 0 : cp_gen];
#ifndef FGP_C2R_UNROLL
#define FGP_C2R_UNROLL 8   // measured: 1501 vs 1533 us at 512 x 2^18 (profiles/r02i_exp_half_length_transforms.jsonl)
#endif
  // pair job j: its (row, column) of the tile and of the mirrored partner (column 0 of tile 0 folds its
  // own mirror image: rows r and N1 - r of column 0, and column N2/2)
  auto job = [&](int j, int& sp, int& rp, int64_t& cp, int& ss, int& rs) {
    const int rr = rr0 + RSTEP * j;
    if (!col0) {
      sp = q; rp = rr; cp = cp_gen; ss = sp + HC; rs = N1 - 1 - rp;
    } else if (rr < N1 / 2) {
      sp = 0; rp = rr; cp = 0; ss = 0; rs = (N1 - rp) & (N1 - 1);
    } else {
      sp = HC; rp = rr - N1 / 2; cp = N2 >> 1; ss = HC; rs = N1 - 1 - rp;
    }
  };
  // HERM: every job's two input values (and factors) are loaded before any is used, so the JOBS x 2
  // loads of a thread are in flight together (the one-loop form waited for each job's loads in turn:
  // the column pass is bound by these loads)
  double2 av[HERM ? JOBS : 1], bv[HERM ? JOBS : 1], tv[HERM ? JOBS : 1], wv[HERM ? JOBS : 1];
  double fa[HERM ? JOBS : 1], fb[HERM ? JOBS : 1];
  if constexpr (HERM) {
#pragma unroll
    for (int j = 0; j < JOBS; ++j) {
      int sp, rp, ss, rs;
      int64_t cp;
      job(j, sp, rp, cp, ss, rs);
      const bool self = col0 && sp == 0 && rp == 0;
      const int64_t kp = cp + (int64_t)rp * N2, kb = self ? nt : nt - kp;
      tv[j] = tw[rp << (24 - m)];
      wv[j] = col0 ? twmf[cp] : wcp;
      av[j] = xg[kp];
      bv[j] = xg[kb];
      if (fr) {
        fa[j] = fr[kp];
        fb[j] = fr[kb];
      }
    }
  }
#pragma unroll FGP_C2R_UNROLL
  for (int j = 0; j < JOBS; ++j) {
    int sp, rp, ss, rs;
    int64_t cp;
    job(j, sp, rp, cp, ss, rs);
    const bool self = col0 && sp == 0 && rp == 0;   // frequencies 0, n/2 and (second element) n/4, 3n/4
    double2 W;                                                        // w_n^k, k = cp + N2 rp
    if constexpr (HERM) {
      W = cmul(wv[j], tv[j]);
    } else {
      W = cmul(col0 ? twmf[cp] : wcp, tw[rp << (24 - m)]);
    }
    const int64_t kp = cp + (int64_t)rp * N2;
    double2 h0, h1, vp, vs;
    if constexpr (HERM) {   // xv(kp), conj xv(nt - kp); self: the real parts of xv(0), xv(nt)
      const double2 a = fr ? make_double2(av[j].x * fa[j], av[j].y * fa[j]) : av[j];
      const double2 b = fr ? make_double2(bv[j].x * fb[j], bv[j].y * fb[j]) : bv[j];
      h0 = self ? make_double2(a.x, 0.0) : a;
      h1 = make_double2(b.x, self ? 0.0 : -b.y);
    } else {
      herm(kp, self ? 0 : nt - kp, h0, h1);
      if (self) {   // partners of 0 and n/2 are themselves: the real parts
        h0 = make_double2(xv(0).x, 0.0);
        h1 = make_double2(xv(nt).x, 0.0);
      }
    }
    vpack(h0, h1, W, vp, vs);
    lds[sp * CS + rp] = vp;
    if (!self) lds[ss * CS + rs] = vs;
    if (self) {   // column 0, row N1/2: frequencies n/4 and 3n/4, mirrors of each other
      constexpr int rh = N1 / 2;
      const int64_t kh = (int64_t)rh * N2;
      const double2 a0 = xv(kh), a1 = HERM ? make_double2(a0.x, -a0.y) : xv(kh + nt);
      const double2 hh0 = make_double2(0.5 * (a0.x + a1.x), 0.5 * (a0.y - a1.y));
      const double2 hh1 = make_double2(hh0.x, -hh0.y);
      double2 vh, unused;
      vpack(hh0, hh1, tw[rh << (24 - m)], vh, unused);
      lds[rh] = vh;
    }
  }
  __syncthreads();
  double2 v[16];
  double2 sum = zero_v<double2>();
#pragma unroll
  for (int j = 0; j < 16 / RLAST; ++j)
#pragma unroll
    for (int t = 0; t < RLAST; ++t) {
      v[j * RLAST + t] = col[pass_pos<P1, SL, RLL>(tt, j, t)];
      sum += v[j * RLAST + t];
    }
  column_partials<C>(sum, part);
  const double2 mean = column_total<C>(sl, part) * (1.0 / N1);
#pragma unroll
  for (int k = 0; k < 16; ++k) v[k] -= mean;
  adj_reg_passes<P1, SL, false>(v, col, tt, tw);
  if (tt == 0) v[0] += mean * (double)N1;
  const WtStore wo(work + g * n);
  const unsigned o0 = (unsigned)((int64_t)blk * kTile + sl);
#pragma unroll
  for (int j = 0; j < 16 / R0; ++j)
#pragma unroll
    for (int t = 0; t < R0; ++t) wo.put(o0 + (unsigned)(pass_pos<P1, 0, RL0>(tt, j, t) * C), v[j * R0 + t]);
}

__global__ __launch_bounds__(kWG) void k_inv_rows_c2r(const double2* __restrict__ work, int log2n, double* __restrict__ out,
                                                      int64_t out_stride, const double2* __restrict__ tw,
                                                      const double2* __restrict__ twm) {
  constexpr int P2 = 12, N2 = 1 << P2;
  __shared__ double ldsd[kTile + kTile / 16];
  __shared__ double2 red[kWG / 64];
  const int mt = log2n - 1, m1 = mt - P2;
  const int64_t n = (int64_t)1 << log2n, nt = n >> 1;
  const int64_t tiles = nt >> kTileLog;
  const int64_t g = blockIdx.x / tiles;
  const int row0 = (int)(blockIdx.x % tiles);
  const int tid = threadIdx.x;
  const double2* in = work + g * n;
  double2 v[16];
  double2 sum = zero_v<double2>();
  const RowTwiddle rt((unsigned)row0, tid, P2, m1, tw, twm);
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    v[k] = tw_mul<double2>(in[work_pos_pair(row0, tid + k * kWG, m1, N2)], rt.at(k, P2, m1, tw, twm), true);
    sum += v[k];
  }
  const double2 mean = block_sum_t(sum, red) * (1.0 / N2);
#pragma unroll
  for (int k = 0; k < 16; ++k) v[k] -= mean;
  adj_reg_passes<P2, LastPass<P2>::S, true>(v, ldsd, tid, tw);
  if (tid == 0) v[0] += mean * (double)N2;
  const double gs = 1.0 / sqrt((double)n);
  double* xo = out + g * out_stride + (int64_t)row0 * N2;
  // v[k] is element 16 tid + k of the row: the Re (then Im) parts go through LDS so that a store
  // instruction's lanes cover consecutive 16 B (direct stores put the lanes 128 B apart: 64 partial lines
  // per instruction)
  __syncthreads();
#pragma unroll
  for (int half = 0; half < 2; ++half) {
#pragma unroll
    for (int k = 0; k < 16; ++k) ldsd[kRunPad * tid + k] = (half ? v[k].y : v[k].x) * gs;
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int p = 2 * (tid + kWG * u), a = run_pad(p);
      *reinterpret_cast<double2*>(xo + half * nt + p) = make_double2(ldsd[a], ldsd[a + 1]);
    }
    if (half == 0) __syncthreads();
  }
}

// adjoint half-length row pass: Re -> gradient terms of x[:n/2], Im -> of x[n/2:]
template <int PG, int D>
__global__ __launch_bounds__(kWG) void k_bwd_rows_r2c(Nll a, const double2* __restrict__ tw, const double2* __restrict__ twm) {
  constexpr int P2 = 12, N2 = 1 << P2;
  __shared__ double ldsd[kTile + kTile / 16];
  __shared__ double2 red[kWG / 64];
  __shared__ double redd[kWG / 64];
  const int mt = a.log2n - 1, m1 = mt - P2;
  const int64_t n = (int64_t)1 << a.log2n, nt = n >> 1;
  const int64_t tiles = nt >> kTileLog;
  const int g = (int)(blockIdx.x / tiles);
  const int blk = (int)(blockIdx.x % tiles);
  const int row0 = blk;
  const int64_t base = (int64_t)blk * kTile;
  const int tid = threadIdx.x;
  stamp_begin(a);
  const double2* in = static_cast<const double2*>(a.work) + (int64_t)g * n;
  double2 v[16];
  double2 sum = zero_v<double2>();
  const RowTwiddle rt((unsigned)row0, tid, P2, m1, tw, twm);
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    v[k] = tw_mul<double2>(in[work_pos_pair(row0, tid + k * kWG, m1, N2)], rt.at(k, P2, m1, tw, twm), true);
    sum += v[k];
  }
  const double2 mean = block_sum_t(sum, red) * (1.0 / N2);
#pragma unroll
  for (int k = 0; k < 16; ++k) v[k] -= mean;
  adj_reg_passes<P2, LastPass<P2>::S, true>(v, ldsd, tid, tw);
  if (tid == 0) v[0] += mean * (double)N2;
  Hyp h;
  load_hyp_wave(a, g, h);
  fold_gen_coef<PG>(a, h);
  PSrc src;
  psrc_init(a, g, src);
  constexpr int ND = Dims<D>::N;
  double acc[1 + ND];
#pragma unroll
  for (int q = 0; q < 1 + ND; ++q) acc[q] = 0.0;
  double* gl = ldsd + 17 * tid;
  const double gs = 1.0 / sqrt((double)n);
  __syncthreads();
#pragma unroll
  for (int t = 0; t < 16; ++t) gl[t] = v[t].x;
  grad_run16<PG, D>(a, h, src, n, base + 16 * tid, gl, gs, acc);
#pragma unroll
  for (int t = 0; t < 16; ++t) gl[t] = v[t].y;
  grad_run16<PG, D>(a, h, src, n, nt + base + 16 * tid, gl, gs, acc);
#pragma unroll
  for (int q = 0; q < 1 + ND; ++q) {
    if (q <= a.d) {
      const double r = block_sum(acc[q], redd) * grad_factor(h, q);
      if (tid == 0) *part_ptr(a, g, 3 + q, blk) = r;
    }
  }
  stamp_end(a);
}

// ---------------------------------------------------------------- fit step (one workgroup)


__device__ __forceinline__ double* red_ptr(const Nll& a, int g, int q) {
  return a.partials + (int64_t)a.G * a.nq * a.nb + (int64_t)g * a.nq + q;
}

// one workgroup per problem: deterministic (fixed-order) reduction of its per-block partials
__global__ __launch_bounds__(kWG) void k_fit_reduce(Nll a) {
  __shared__ double redd[kWG / 64];
  const int g = blockIdx.x;
  for (int q = 0; q < a.nq; ++q) {
    double v = 0.0;
    for (int b = threadIdx.x; b < a.nb; b += kWG) v += *part_ptr(a, g, q, b);
    v = block_sum(v, redd);
    if (threadIdx.x == 0) *red_ptr(a, g, q) = v;
  }
}

// loss assembly, histories and the Rprop update (torch.optim.Rprop single-tensor semantics) of ONE loss
// over the G problems (per-output hyper-parameters of one GP): thread t takes problems t, t + kWG, ...
// (ascending): a per-problem parameter's gradient is written by the one thread owning that problem, the
// loss terms and the gradients of shared parameters are per-thread sums reduced in a fixed order
// (wave shuffles, then the waves in order) -- O(G / kWG) per thread instead of a serial pass over G.
__global__ __launch_bounds__(kWG) void k_fit_step(Nll a, Fit f, int iter, int do_update) {
  extern __shared__ double grad[];   // [n_params]
  constexpr int NV = 4 + FGP_MAX_D, NW = kWG / 64;
  __shared__ double red[NV * NW];
  const int tid = threadIdx.x;
  for (int p = tid; p < f.n_params; p += kWG) {
    grad[p] = 0.0;
    f.raw_hist[(int64_t)iter * f.n_params + p] = f.raw[p];
  }
  __syncthreads();
  double v[NV];   // term1, logdet, shared dnoise, shared dscale, shared dlengthscale[j]
#pragma unroll
  for (int q = 0; q < NV; ++q) v[q] = 0.0;
  for (int g = tid; g < a.G; g += kWG) {
    v[0] += *red_ptr(a, g, 0);
    v[1] += *red_ptr(a, g, 1);
    const int ni = a.noise_off + (a.noise_pp ? g : 0);
    const double dn = exp(a.raw[ni]) * *red_ptr(a, g, 2);
    if (a.noise_pp) grad[ni] += dn;
    else v[2] += dn;
    if (a.scale_pp) grad[a.scale_off + g] += *red_ptr(a, g, 3);
    else v[3] += *red_ptr(a, g, 3);
    const int lb = a.ls_off + (a.ls_pp ? g : 0) * (a.ls_pd ? a.d : 1);
    for (int j = 0; j < a.d; ++j) {
      const double r = *red_ptr(a, g, 4 + j);
      if (a.ls_pp) grad[lb + (a.ls_pd ? j : 0)] += r;
      else v[4 + (a.ls_pd ? j : 0)] += r;
    }
  }
#pragma unroll
  for (int q = 0; q < NV; ++q) {
    double x = v[q];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    if ((tid & 63) == 0) red[q * NW + (tid >> 6)] = x;
  }
  __syncthreads();
  if (tid == 0) {
    double tot[NV];
#pragma unroll
    for (int q = 0; q < NV; ++q) {
      tot[q] = 0.0;
#pragma unroll
      for (int w = 0; w < NW; ++w) tot[q] += red[q * NW + w];
    }
    if (!a.noise_pp) grad[a.noise_off] += tot[2];
    if (!a.scale_pp) grad[a.scale_off] += tot[3];
    if (!a.ls_pp) {
      for (int j = 0; j < (a.ls_pd ? a.d : 1); ++j) grad[a.ls_off + j] += tot[4 + j];
    }
    const double term2 = a.logdet_weight * tot[1];
    f.loss_hist[(int64_t)iter * 3 + 0] = 0.5 * (tot[0] + term2 + f.mll_const);
    f.loss_hist[(int64_t)iter * 3 + 1] = tot[0];
    f.loss_hist[(int64_t)iter * 3 + 2] = term2;
  }
  __syncthreads();
  const int scale_cnt = a.scale_pp ? a.G : 1;
  const int ls_cnt = (a.ls_pp ? a.G : 1) * (a.ls_pd ? a.d : 1);
  for (int p = tid; p < f.n_params; p += kWG) {
    const double gp = grad[p];
    f.grad_out[p] = gp;
    if (!do_update) continue;
    bool rg;
    if (p >= a.scale_off && p < a.scale_off + scale_cnt) rg = f.scale_rg;
    else if (p >= a.ls_off && p < a.ls_off + ls_cnt) rg = f.ls_rg;
    else rg = f.noise_rg;
    if (!rg) continue;
    rprop_update(f, p, gp);
  }
}

// Independent problems (per_problem): one workgroup per GP reduces its partials, records its loss
// and parameters and applies Rprop to the parameters it owns (reduce_step_wg, fgp_nll.h).
__global__ __launch_bounds__(kWG) void k_fit_reduce_step(Nll a, Fit f, int iter, int do_update) {
  __shared__ double red[(4 + FGP_MAX_D) * (kWG / 64)];
  __shared__ double vals[4 + FGP_MAX_D];
  reduce_step_wg<kWG, false>(a, f, blockIdx.x, iter, do_update, red, vals);
}

// ------------------------------------------------------------------------------------------------
// on-device lattice points and generated parts (the arithmetic of the FGP_PARTS_LATTICE fit path)
struct GenSpec {
  unsigned z[FGP_MAX_D];       // z_j mod 2^bits
  double coef[FGP_MAX_D];
  int order;
};

// x[i - n0, j] = ((brev_bits(i) z_j mod 2^bits) / 2^bits + shift_j) % 1,  i in [n0, n1)
__global__ __launch_bounds__(kWG) void k_lattice_points(GenSpec g, const double* __restrict__ shift, int64_t n0,
                                                        int64_t n1, int d, int bits, double* __restrict__ x) {
  const int64_t i = n0 + (int64_t)blockIdx.x * kWG + threadIdx.x;
  if (i >= n1) return;
  const unsigned br = brev_bits((unsigned)i, bits), mask = bits >= 32 ? 0xffffffffu : (1u << bits) - 1u;
  const double inv = ldexp(1.0, -bits);
  for (int j = 0; j < d; ++j) {
    double v = (double)((br * g.z[j]) & mask) * inv;
    v = v + shift[j];
    if (v >= 1.0) v -= 1.0;
    x[(i - n0) * d + j] = v;
  }
}

template <int ORD>
__global__ __launch_bounds__(kWG) void k_lattice_parts_gen(GenSpec g, const double* __restrict__ shift, int m, int d,
                                                           double* __restrict__ parts) {
  const int64_t n = (int64_t)1 << m;
  const int64_t i = (int64_t)blockIdx.x * kWG + threadIdx.x;
  if (i >= n) return;
  const unsigned br = brev_bits((unsigned)i, m), mask = (unsigned)(n - 1);
  const double inv_n = ldexp(1.0, -m);
  for (int j = 0; j < d; ++j) parts[(int64_t)j * n + i] = g.coef[j] * lattice_gen_part<ORD>(g.z[j], br, mask, inv_n);
}

// k_fwd_rows_r2c_prod with the lattice parts regenerated in the row (fgp_spec_basis_gen): part_j(i) =
// coef_j B_ORD((brev_m(i) z_j mod n) / n), k_lattice_parts_gen's values bit for bit, multiplied in ascending j
// from 1.0 as the parts-array kernel does -- so the spectra equal fgp_spec_basis(fgp_lattice_parts_gen(...))
// bit for bit, without the d n parts array written and re-read by every subset (the parts kernel's loads
// per subset dimension were the row kernel's bound: 152 us of C4's 32 subsets, profiles/r04c_*).
template <int D, int ORD>
__global__ __launch_bounds__(kWG) void k_fwd_rows_r2c_gen(GenSpec g, int log2n, int s0, int cnt,
                                                          double2* __restrict__ work, const double2* __restrict__ tw,
                                                          const double2* __restrict__ twm) {
  constexpr int P2 = 12, N2 = 1 << P2;
  __shared__ double ldsd[kTile + kTile / 16];
  __shared__ double2 red[kWG / 64];
  const int mt = log2n - 1, m1 = mt - P2;
  const int64_t n = (int64_t)1 << log2n;
  // XCD-aware order as k_fwd_rows_r2c_prod (speed only)
  const unsigned rows = gridDim.x / (unsigned)cnt;
  int c, row0;
  if (rows % 8u == 0u) {
    const unsigned xcd = blockIdx.x & 7u, local = blockIdx.x >> 3;
    c = (int)(local % (unsigned)cnt);
    row0 = (int)((local / (unsigned)cnt) * 8u + xcd);
  } else {
    c = (int)(blockIdx.x % (unsigned)cnt);
    row0 = (int)(blockIdx.x / (unsigned)cnt);
  }
  const int S = s0 + c;
  const int tid = threadIdx.x;
  const unsigned mask = (unsigned)(n - 1);
  const double inv_n = ldexp(1.0, -log2n);
  // element i0 + t of x[:n/2] (real parts) and its partner i0 + t + n/2 (imaginary parts): brev_m(i + n/2) =
  // brev_m(i) + 1 (i < n/2: bit 0 of brev_m(i) is clear)
  const unsigned br0 = brev_bits((unsigned)((int64_t)row0 * N2 + 16 * tid), log2n);
  double2 v[16];
#pragma unroll
  for (int t = 0; t < 16; ++t) v[t] = make_double2(1.0, 1.0);
#pragma unroll
  for (int j = 0; j < D; ++j) {
    if ((S >> j) & 1) {                      // uniform over the workgroup
      const unsigned zj = g.z[j];
      const double cj = g.coef[j];
      static_for<0, 16>([&](auto tc) {
        constexpr int t = decltype(tc)::value;
        const unsigned br = brev_run<t>(br0, log2n);
        v[t].x *= cj * lattice_gen_part<ORD>(zj, br, mask, inv_n);
        v[t].y *= cj * lattice_gen_part<ORD>(zj, br | 1u, mask, inv_n);
      });
    }
  }
  double2 sum = make_double2(0.0, 0.0);
#pragma unroll
  for (int t = 0; t < 16; ++t) sum += v[t];
  const double2 mean = block_sum_t(sum, red) * (1.0 / N2);
#pragma unroll
  for (int t = 0; t < 16; ++t) v[t] -= mean;
  fwd_reg_passes<P2, 0, true>(v, ldsd, tid, tw);
  if (tid == 0) v[0] += mean * (double)N2;
  const RowTwiddle rt((unsigned)row0, tid, P2, m1, tw, twm);
  double2* out = work + (int64_t)c * n;
#pragma unroll
  for (int k = 0; k < 16; ++k)
    out[work_pos_pair(row0, tid + k * kWG, m1, N2)] = tw_mul<double2>(v[k], rt.at(k, P2, m1, tw, twm), false);
}

// ------------------------------------------------------------------------------------------------
// host-side launch logic
static int to_nll(const fgp_nll_desc* d, Nll& a) {
  if (!d) return set_error(kErrInvalid, "null nll desc");
  if (d->family != FGP_FAMILY_LATTICE && d->family != FGP_FAMILY_NET) return set_error(kErrInvalid, "bad family");
  if (d->log2n < 4 || d->log2n > kMaxLog2N) return set_error(kErrUnsupported, "fused fit needs 4 <= log2n <= 24");
  if (d->d < 1 || d->d > FGP_MAX_D) return set_error(kErrUnsupported, "d=%d outside [1, %d]", d->d, FGP_MAX_D);
  if (d->G < 1) return set_error(kErrInvalid, "G < 1");
  const bool mt = d->mt_tasks != 0;
  if (!d->ysq || !d->raw || !d->partials || (d->log2n > 12 && !d->work && !d->basis && !mt))
    return set_error(kErrInvalid, "null pointer in nll desc");
  if (mt && (d->mt_tasks < 1 || d->mt_tasks > kMtMaxT || d->G != 1 || d->d > kSpecMaxD || d->basis))
    return set_error(kErrUnsupported, "multitask spectral fit: needs 1 <= T <= %d, G = 1, d <= %d, no basis",
                     kMtMaxT, kSpecMaxD);
  if (mt && (!d->mt_basis || !d->mt_ytilde || !d->mt_kt)) return set_error(kErrInvalid, "null pointer in nll desc (mt)");
  if (d->basis && d->d > kSpecMaxD)
    return set_error(kErrUnsupported, "spectral fit path: d = %d > %d", d->d, kSpecMaxD);
  if (d->basis && d->basis_stride < 0) return set_error(kErrInvalid, "negative basis_stride");
  if (d->parts_gen == FGP_PARTS_ARRAY) {
    if (!d->parts && !d->basis && !mt) return set_error(kErrInvalid, "null parts in nll desc");
  } else if (d->parts_gen == FGP_PARTS_LATTICE) {
    if (d->family != FGP_FAMILY_LATTICE) return set_error(kErrInvalid, "lattice parts generator needs the lattice family");
    if (!d->gen_shift) return set_error(kErrInvalid, "null gen_shift in nll desc");
    for (int j = 0; j < d->d; ++j) {
      const int o = d->gen_order[j];
      if (o < 2 || o > 8 || (o & 1)) return set_error(kErrUnsupported, "Bernoulli order %d unsupported", o);
      if (o != d->gen_order[0])
        return set_error(kErrUnsupported, "lattice parts generator needs one Bernoulli order for every dimension");
      if (d->gen_z[j] <= 0 || (d->log2n < 53 && d->gen_z[j] >= ((int64_t)1 << (53 - d->log2n))))
        return set_error(kErrUnsupported, "generating vector entry %lld outside (0, 2^(53-log2n))",
                         (long long)d->gen_z[j]);
    }
  } else {
    return set_error(kErrInvalid, "bad parts_gen %d", d->parts_gen);
  }
  a.log2n = d->log2n;
  a.d = d->d;
  a.G = d->G;
  // lattices with n >= 2^17: the real-even (RE) fit kernels when the parts are regenerated, else the
  // half-length (R2C) ones.  FGP_R2C=1 forces R2C, FGP_R2C=0 the full-length kernels.
  const char* r2c_env = getenv("FGP_R2C");
  const char mode = (r2c_env && r2c_env[0]) ? r2c_env[0] : '2';
  a.r2c = d->family == FGP_FAMILY_LATTICE && d->log2n >= 17 && mode != '0';
  const int re_p2 = re_row_log2(d->log2n);
  // the real-even kernels form each mirror pair's parts from one lattice index, which needs every
  // generating vector entry odd (M z_j = n/2 mod n); an even entry takes the R2C kernels
  bool z_odd = true;
  for (int j = 0; j < d->d && d->parts_gen == FGP_PARTS_LATTICE; ++j) z_odd = z_odd && (d->gen_z[j] & 1);
  // (the real-even kernels also take n = 2^16, where the R2C ones do not run: rows of 2^11, 16 rows)
  a.re = d->family == FGP_FAMILY_LATTICE && d->log2n >= 16 && mode != '0' && mode != '1' &&
         d->parts_gen == FGP_PARTS_LATTICE && re_p2 > 0 && z_odd;
  // per-block partials: one per row / row-pair workgroup (RE: N1/2 = n / 2^(P2 + 2) row pairs)
  a.nb = d->log2n > 12 ? 1 << (a.re ? d->log2n - 2 - re_p2 : d->log2n - 12 - (a.r2c ? 1 : 0)) : 1;
  a.nq = 4 + d->d;
  a.parts = d->parts;
  a.parts_stride = d->parts_stride;
  a.ysq = d->ysq;
  a.ysq_stride = d->ysq_stride;
  a.raw = d->raw;
  a.scale_off = d->scale_off;
  a.scale_pp = d->scale_pp;
  a.ls_off = d->ls_off;
  a.ls_pp = d->ls_pp;
  a.ls_pd = d->ls_pd;
  a.noise_off = d->noise_off;
  a.noise_pp = d->noise_pp;
  a.logdet_weight = d->logdet_weight;
  a.grad_lam = d->grad_lam;
  a.work = d->work;
  a.partials = d->partials;
  a.pgen = d->parts_gen == FGP_PARTS_LATTICE;
  a.pg = a.pgen ? d->gen_order[0] : 0;
  const uint64_t zmask = ((uint64_t)1 << d->log2n) - 1;
  for (int j = 0; j < FGP_MAX_D; ++j) {
    const bool on = a.pgen && j < d->d;
    a.gorder[j] = on ? d->gen_order[j] : 0;
    a.gcoef[j] = on ? d->gen_coef[j] : 0.0;
    a.gz[j] = on ? (unsigned)((uint64_t)d->gen_z[j] & zmask) : 0u;
  }
  a.gshift = d->gen_shift;
  a.gshift_stride = d->gen_shift_stride;
  a.stamps = reinterpret_cast<unsigned long long*>(d->stamps);
  // spectral path: the eigenvalues from the part-product spectra, one kernel per iteration
  a.basis = d->basis;
  a.basis_stride = d->basis_stride;
  a.ysq_chunked = d->ysq_chunked;
  if (a.ysq_chunked && !d->basis) return set_error(kErrInvalid, "ysq_chunked needs the spectral path (basis)");
  a.spec = d->basis != nullptr;
  a.spec_net = d->family == FGP_FAMILY_NET;
  a.spec_K = a.spec_KS = a.spec_main = a.spec_kw = 0;
  a.spec_kpl = a.spec_ppw = a.spec_pg = a.spec_tile = a.spec_pgp = a.spec_ck = a.spec_ps = 0;
  a.spec_nsl = 1;
  a.loss = d->loss_metric;
  a.cv_weight = d->cv_weight;
  if (a.loss != FGP_LOSS_MLL) {
    if (a.loss != FGP_LOSS_GCV && a.loss != FGP_LOSS_CV) return set_error(kErrInvalid, "bad loss_metric %d", a.loss);
    if (!d->basis && !mt) return set_error(kErrUnsupported, "GCV / CV fits need the spectral path (basis)");
  }
  if (a.spec) {
    a.re = a.r2c = 0;
    spec_geometry(a, a.loss == FGP_LOSS_MLL);
    if (a.loss != FGP_LOSS_MLL) {
      // the alternative losses' per-wave kernel: one problem per wave, 2 + 2 (2 + d) quantities per block
      a.spec_ppw = 1;
      a.spec_pg = a.G;
      a.nq = 6 + 2 * a.d;
    }
  }
  a.mt = 0;
  a.mt_F = a.mt_cpb = 0;
  a.mt_basis = d->mt_basis;
  a.mt_ytilde = d->mt_ytilde;
  a.mt_kt = d->mt_kt;
  a.mt_learn = a.mt_rank = a.mt_vexp = a.mt_f_off = a.mt_v_off = 0;
  if (d->mt_task_rg) {
    if (!mt || a.loss == FGP_LOSS_MLL || d->mt_task_rg < 0 || d->mt_task_rg > 3 || d->mt_rank < 0 ||
        d->mt_rank > d->mt_tasks || a.noise_pp || a.G != 1)
      return set_error(kErrUnsupported, "learned task kernel: multitask spectral GCV / CV, rank 0 .. T");
    a.mt_learn = d->mt_task_rg;
    a.mt_rank = d->mt_rank;
    a.mt_vexp = d->mt_vexp ? 1 : 0;
    a.mt_f_off = a.noise_off + 1;
    a.mt_v_off = a.mt_f_off + d->mt_tasks * d->mt_rank;
  }
  if (mt) {
    // one chunk of kMtF frequencies per step, up to kSpecBlocks blocks (the spectral reduction's limit)
    const int64_t n = (int64_t)1 << d->log2n;
    a.mt = d->mt_tasks;
    a.spec = 1;                      // the per-problem step is the spectral path's (k_spec_reduce_step)
    a.spec_net = d->family == FGP_FAMILY_NET;
    a.re = a.r2c = 0;
    a.mt_F = (int)std::min<int64_t>(kMtF, n);
    const int64_t chunks = n / a.mt_F;
    a.nb = (int)std::min<int64_t>(kSpecBlocks, chunks);
    a.mt_cpb = (int)(chunks / a.nb);
    if (a.loss != FGP_LOSS_MLL) a.nq = 6 + 2 * a.d;    // the single-task GCV / CV partial layout (k_spec_loss_step)
    // (a learned task kernel: + the two streams of dL/dK_task per task pair, k_mt_learn_step)
    if (a.mt_learn) a.nq += a.mt * (a.mt + 1);
  }
  return kOk;
}


template <typename T>
static int launch_iter_single(const Nll& a, const Tables* tb, hipStream_t st, bool emit = false) {
  const int P = a.log2n;
  const unsigned grid = (unsigned)((a.G + (kTile >> P) - 1) / (kTile >> P));
  return with_pg<T>(a, [&](auto pgc) {
    constexpr int PG = decltype(pgc)::value;
    switch (P) {
#define FGP_C(PP)                                                                     \
  case PP:                                                                            \
    if (emit) k_iter_single<PP, T, true, PG><<<grid, kWG, 0, st>>>(a, tb->tw4096);    \
    else k_iter_single<PP, T, false, PG><<<grid, kWG, 0, st>>>(a, tb->tw4096);        \
    break;
      FGP_C(4) FGP_C(5) FGP_C(6) FGP_C(7) FGP_C(8) FGP_C(9) FGP_C(10) FGP_C(11) FGP_C(12)
#undef FGP_C
      default: return set_error(kErrInvalid, "bad log2n");
    }
    return check_launch("k_iter_single");
  });
}

template <typename T>
static int launch_rows_fwd(const Nll& a, const Tables* tb, hipStream_t st) {
  const int m = a.log2n, m2 = split_m2(m);
  const unsigned grid = (unsigned)((int64_t)a.G << (m - kTileLog));
  return with_pg<T>(a, [&](auto pgc) {
    constexpr int PG = decltype(pgc)::value;
    switch (m2) {
#define FGP_C(PP) case PP: k_fwd_rows<PP, T, PG, 0><<<grid, kWG, 0, st>>>(a, tb->tw4096, tb->twm[m]); break;
      FGP_C(9) FGP_C(10) FGP_C(11)
#undef FGP_C
      case 12:   // n >= 2^16: the dimension count as a compile-time constant
        with_d(a.d, [&](auto dc) {
          k_fwd_rows<12, T, PG, decltype(dc)::value><<<grid, kWG, 0, st>>>(a, tb->tw4096, tb->twm[m]);
        });
        break;
      default: return set_error(kErrInvalid, "bad m2");
    }
    return check_launch("k_fwd_rows");
  });
}

template <typename T>
static int launch_cols_fwd(const Nll& a, const Tables* tb, hipStream_t st, bool emit) {
  const int m = a.log2n, m1 = m - split_m2(m);
  const unsigned grid = (unsigned)((int64_t)a.G << (m - kTileLog));
  switch (m1) {
#define FGP_C(PP)                                                           \
  case PP:                                                                  \
    if (emit) k_fwd_cols<PP, T, true><<<grid, kWG, 0, st>>>(a, tb->tw4096); \
    else k_fwd_cols<PP, T, false><<<grid, kWG, 0, st>>>(a, tb->tw4096);     \
    break;
    FGP_C(4) FGP_C(5) FGP_C(6) FGP_C(7) FGP_C(8) FGP_C(9) FGP_C(10) FGP_C(11) FGP_C(12)
#undef FGP_C
    default: return set_error(kErrInvalid, "bad m1");
  }
  return check_launch("k_fwd_cols");
}

template <typename T>
static int launch_rows_bwd(const Nll& a, const Tables* tb, hipStream_t st) {
  const int m = a.log2n, m2 = split_m2(m);
  const unsigned grid = (unsigned)((int64_t)a.G << (m - kTileLog));
  return with_pg<T>(a, [&](auto pgc) {
    constexpr int PG = decltype(pgc)::value;
    switch (m2) {
#define FGP_C(PP) case PP: k_bwd_rows<PP, T, PG, 0><<<grid, kWG, 0, st>>>(a, tb->tw4096, tb->twm[m]); break;
      FGP_C(9) FGP_C(10) FGP_C(11)
#undef FGP_C
      case 12:
        with_d(a.d, [&](auto dc) {
          k_bwd_rows<12, T, PG, decltype(dc)::value><<<grid, kWG, 0, st>>>(a, tb->tw4096, tb->twm[m]);
        });
        break;
      default: return set_error(kErrInvalid, "bad m2");
    }
    return check_launch("k_bwd_rows");
  });
}

// half-length (R2C) lattice kernels: transforms of length n/2 (rows of 4096, N1 = 2^(m - 13) rows)
static int launch_r2c(const Nll& a, int stage, const Tables* tb, hipStream_t st, bool emit) {
  const int m = a.log2n, mt = m - 1, p1 = mt - 12;
  const unsigned grid = (unsigned)((int64_t)a.G << (mt - kTileLog));
  if (stage == 0 || stage == 2) {
    return with_pg<double2>(a, [&](auto pgc) {
      constexpr int PG = decltype(pgc)::value;
      with_d(a.d, [&](auto dc) {
        constexpr int DD = decltype(dc)::value;
        if (stage == 0) k_fwd_rows_r2c<PG, DD><<<grid, kWG, 0, st>>>(a, tb->tw4096, tb->twm[mt]);
        else k_bwd_rows_r2c<PG, DD><<<grid, kWG, 0, st>>>(a, tb->tw4096, tb->twm[mt]);
      });
      return check_launch(stage == 0 ? "k_fwd_rows_r2c" : "k_bwd_rows_r2c");
    });
  }
  switch (p1) {
#define FGP_C(PP)                                                                              \
  case PP:                                                                                     \
    if (emit) k_fwd_cols_r2c<PP, 1><<<grid, kWG, 0, st>>>(a, tb->tw4096, tb->twm[m]);       \
    else k_fwd_cols_r2c<PP, 0><<<grid, kWG, 0, st>>>(a, tb->tw4096, tb->twm[m]);           \
    break;
    FGP_C(4) FGP_C(5) FGP_C(6) FGP_C(7) FGP_C(8) FGP_C(9) FGP_C(10) FGP_C(11)
#undef FGP_C
    default: return set_error(kErrInvalid, "bad r2c m1");
  }
  return check_launch("k_fwd_cols_r2c");
}

// one kernel of the pipeline: 0 = forward rows (n <= 4096: the single-kernel iteration), 1 = eigen
// terms + adjoint columns, 2 = adjoint rows + gradient terms
template <typename T>
static int nll_stage_t(const Nll& a, int stage, const Tables* tb, hipStream_t st) {
  if (a.log2n <= 12) return stage == 0 ? launch_iter_single<T>(a, tb, st) : kOk;
  if constexpr (sizeof(T) == 16) {
    if (a.r2c || a.re) {
      if (stage < 0 || stage > 2) return set_error(kErrInvalid, "bad stage %d", stage);
      return a.re ? launch_re(a, stage, tb, st) : launch_r2c(a, stage, tb, st, false);
    }
  }
  switch (stage) {
    case 0: return launch_rows_fwd<T>(a, tb, st);
    case 1: return launch_cols_fwd<T>(a, tb, st, false);
    case 2: return launch_rows_bwd<T>(a, tb, st);
    default: return set_error(kErrInvalid, "bad stage %d", stage);
  }
}

static int nll_stage(const Nll& a, int stage, hipStream_t st, bool lattice) {
  if (a.mt) {
    if (stage < 0 || stage > 2) return set_error(kErrInvalid, "bad stage %d", stage);
    return stage == 0 ? launch_mt_spec_iter(a, st) : kOk;
  }
  if (a.spec) {
    if (stage < 0 || stage > 2) return set_error(kErrInvalid, "bad stage %d", stage);
    return stage == 0 ? launch_spec_iter(a, st) : kOk;
  }
  const Tables* tb = get_tables(st);
  if (!tb) return set_error(kErrHip, "twiddle table initialisation failed");
  return lattice ? nll_stage_t<double2>(a, stage, tb, st) : nll_stage_t<double>(a, stage, tb, st);
}

static int nll_fwd(const Nll& a, hipStream_t st, bool lattice) {
  int rc = nll_stage(a, 0, st, lattice);
  return rc != kOk ? rc : nll_stage(a, 1, st, lattice);
}

static int nll_bwd(const Nll& a, hipStream_t st, bool lattice) { return nll_stage(a, 2, st, lattice); }

static int to_fit(const fgp_fit_desc* d, Fit& f) {
  if (!d || !d->raw || !d->rprop_prev || !d->rprop_step || !d->grad_out || !d->loss_hist || !d->raw_hist)
    return set_error(kErrInvalid, "null pointer in fit desc");
  if (d->n_params < 1 || d->n_params > 8192) return set_error(kErrInvalid, "bad n_params (1..8192)");
  f.n_params = d->n_params;
  f.raw = d->raw;
  f.prev = d->rprop_prev;
  f.step = d->rprop_step;
  f.grad_out = d->grad_out;
  f.loss_hist = d->loss_hist;
  f.raw_hist = d->raw_hist;
  f.scale_rg = d->scale_rg;
  f.ls_rg = d->ls_rg;
  f.noise_rg = d->noise_rg;
  f.mll_const = d->mll_const;
  f.eta_minus = d->eta_minus;
  f.eta_plus = d->eta_plus;
  f.step_min = d->step_min;
  f.step_max = d->step_max;
  f.per_problem = d->per_problem;
  f.hist_stride = d->hist_stride;
  f.hist_offset = d->hist_offset;
  if (f.hist_stride < 0 || f.hist_offset < 0) return set_error(kErrInvalid, "bad hist_stride / hist_offset");
  return kOk;
}

static int check_per_problem(const Nll& a, const Fit& f) {
  if (f.per_problem && a.G > 1 && !(a.scale_pp && a.ls_pp && a.noise_pp))
    return set_error(kErrInvalid, "per_problem fit needs per-problem scale, lengthscales and noise");
  return kOk;
}

static int fit_step(const Nll& a, const Fit& f, int iter, int do_update, hipStream_t st, bool counter_zero = false) {
  if (a.mt && a.mt_learn) return launch_mt_learn_step(a, f, iter, do_update, st);
  if (a.spec && a.loss != FGP_LOSS_MLL) return launch_spec_loss_step(a, f, iter, do_update, st);
  if (f.per_problem && a.spec) return launch_spec_reduce_step(a, f, iter, do_update, st);
  if (a.spec && a.nb <= kSpecBlocks && !getenv_off("FGP_SPEC_STEP_MANY")) {
    // one loss over many problems: the parallel step (k_spec_step_many); its counter is zeroed once per run
    if (!counter_zero && hipMemsetAsync(spec_step_many_counter(a), 0, sizeof(unsigned), st) != hipSuccess)
      return set_error(kErrHip, "fit step: counter reset failed");
    return launch_spec_step_many(a, f, iter, do_update, st);
  }
  if (f.per_problem) {
    k_fit_reduce_step<<<a.G, kWG, 0, st>>>(a, f, iter, do_update);
    return check_launch("k_fit_reduce_step");
  }
  k_fit_reduce<<<a.G, kWG, 0, st>>>(a);
  int rc = check_launch("k_fit_reduce");
  if (rc != kOk) return rc;
  k_fit_step<<<1, kWG, f.n_params * sizeof(double), st>>>(a, f, iter, do_update);
  return check_launch("k_fit_step");
}

}  // namespace fgp

using namespace fgp;

extern "C" {

int fgp_lattice_parts(const double* x, int64_t x_row_stride, const double* z, int64_t n, int d, const int* order,
                      const double* coef, double* parts, void* stream) {
  if (n < 0 || d < 1 || d > FGP_MAX_D) return set_error(kErrInvalid, "fgp_lattice_parts: bad n/d");
  if (n == 0) return kOk;
  if (!x || !z || !parts || !order || !coef) return set_error(kErrInvalid, "fgp_lattice_parts: null pointer");
  PartsSpec spec;
  for (int j = 0; j < FGP_MAX_D; ++j) {
    spec.order[j] = j < d ? order[j] : 0;
    spec.coef[j] = j < d ? coef[j] : 0.0;
    if (j < d && (order[j] < 2 || order[j] > 8 || (order[j] & 1)))
      return set_error(kErrUnsupported, "Bernoulli order %d unsupported", order[j]);
  }
  k_lattice_parts<<<(unsigned)((n + kWG - 1) / kWG), kWG, 0, (hipStream_t)stream>>>(x, x_row_stride, z, n, d, spec, parts);
  return check_launch("k_lattice_parts");
}

int fgp_net_parts(const int64_t* xb, int64_t xb_row_stride, const int64_t* z, int64_t n, int d, int t,
                  const int* order, double* parts, void* stream) {
  if (n < 0 || d < 1 || d > FGP_MAX_D || t < 1 || t > 63) return set_error(kErrInvalid, "fgp_net_parts: bad n/d/t");
  NetOrders no;
  for (int j = 0; j < FGP_MAX_D; ++j) {
    no.order[j] = (order && j < d) ? order[j] : 1;
    if (no.order[j] < 1 || no.order[j] > 4) return set_error(kErrUnsupported, "fgp_net_parts: Walsh order %d unsupported", no.order[j]);
  }
  if (n == 0) return kOk;
  if (!xb || !z || !parts) return set_error(kErrInvalid, "fgp_net_parts: null pointer");
  k_net_parts<<<(unsigned)((n + kWG - 1) / kWG), kWG, 0, (hipStream_t)stream>>>(xb, xb_row_stride, z, n, d, t, no, parts);
  return check_launch("k_net_parts");
}

int fgp_lattice_points(const int64_t* z, const double* shift, int64_t n_min, int64_t n_max, int d, double* x,
                       void* stream) {
  if (d < 1 || d > FGP_MAX_D || n_min < 0 || n_max < n_min || n_max > ((int64_t)1 << 30))
    return set_error(kErrInvalid, "fgp_lattice_points: bad n_min/n_max/d");
  if (n_max == n_min) return kOk;
  if (!z || !shift || !x) return set_error(kErrInvalid, "fgp_lattice_points: null pointer");
  int bits = 0;
  while (((int64_t)1 << bits) < n_max) ++bits;
  GenSpec g{};
  for (int j = 0; j < d; ++j) {
    if (z[j] <= 0 || (bits < 53 && z[j] >= ((int64_t)1 << (53 - bits))))
      return set_error(kErrUnsupported, "fgp_lattice_points: z[%d] outside (0, 2^(53-bits))", j);
    g.z[j] = (unsigned)((uint64_t)z[j] & (bits >= 32 ? 0xffffffffull : ((1ull << bits) - 1)));
  }
  const int64_t cnt = n_max - n_min;
  k_lattice_points<<<(unsigned)((cnt + kWG - 1) / kWG), kWG, 0, (hipStream_t)stream>>>(g, shift, n_min, n_max, d,
                                                                                       bits, x);
  return check_launch("k_lattice_points");
}

int fgp_lattice_parts_gen(const int64_t* z, const double* shift, int log2n, int d, int order, const double* coef,
                          double* parts, void* stream) {
  if (d < 1 || d > FGP_MAX_D || log2n < 0 || log2n > kMaxLog2N) return set_error(kErrInvalid, "fgp_lattice_parts_gen: bad d/log2n");
  if (!z || !shift || !coef || !parts) return set_error(kErrInvalid, "fgp_lattice_parts_gen: null pointer");
  GenSpec g{};
  const uint64_t zmask = ((uint64_t)1 << log2n) - 1;
  for (int j = 0; j < d; ++j) {
    if (z[j] <= 0 || (log2n < 53 && z[j] >= ((int64_t)1 << (53 - log2n))))
      return set_error(kErrUnsupported, "fgp_lattice_parts_gen: z[%d] outside (0, 2^(53-log2n))", j);
    g.z[j] = (unsigned)((uint64_t)z[j] & zmask);
    g.coef[j] = coef[j];
  }
  const int64_t n = (int64_t)1 << log2n;
  const dim3 grid((unsigned)((n + kWG - 1) / kWG));
  hipStream_t st = (hipStream_t)stream;
  switch (order) {
    case 2: k_lattice_parts_gen<2><<<grid, kWG, 0, st>>>(g, shift, log2n, d, parts); break;
    case 4: k_lattice_parts_gen<4><<<grid, kWG, 0, st>>>(g, shift, log2n, d, parts); break;
    case 6: k_lattice_parts_gen<6><<<grid, kWG, 0, st>>>(g, shift, log2n, d, parts); break;
    case 8: k_lattice_parts_gen<8><<<grid, kWG, 0, st>>>(g, shift, log2n, d, parts); break;
    default: return set_error(kErrUnsupported, "Bernoulli order %d unsupported", order);
  }
  return check_launch("k_lattice_parts_gen");
}

int fgp_spec_basis_gen(const int64_t* z, int log2n, int d, int order, const double* coef, double* basis, void* work,
                       int64_t work_bytes, void* stream) {
  if (d < 1 || d > kSpecMaxD || log2n < 17 || log2n > 24)
    return set_error(kErrUnsupported, "fgp_spec_basis_gen: needs 1 <= d <= %d, 17 <= log2n <= 24", kSpecMaxD);
  if (!z || !coef || !basis || !work) return set_error(kErrInvalid, "fgp_spec_basis_gen: null pointer");
  if (order != 2 && order != 4 && order != 6 && order != 8)
    return set_error(kErrUnsupported, "Bernoulli order %d unsupported", order);
  GenSpec g{};
  const uint64_t zmask = ((uint64_t)1 << log2n) - 1;
  for (int j = 0; j < d; ++j) {
    if (z[j] <= 0 || z[j] >= ((int64_t)1 << (53 - log2n)))
      return set_error(kErrUnsupported, "fgp_spec_basis_gen: z[%d] outside (0, 2^(53-log2n))", j);
    g.z[j] = (unsigned)((uint64_t)z[j] & zmask);
    g.coef[j] = coef[j];
  }
  g.order = order;
  const int64_t n = (int64_t)1 << log2n, per = 16 * n, NS = 1 << d;
  const int chunk = (int)std::min<int64_t>(NS, work_bytes / per);
  if (chunk < 1) return set_error(kErrInvalid, "fgp_spec_basis_gen: work below one subset (%lld bytes)", (long long)per);
  for (int s0 = 0; s0 < NS; s0 += chunk) {
    const int rc = spec_basis_r2c(nullptr, d, log2n, s0, (int)std::min<int64_t>(chunk, NS - s0), basis, work,
                                  (hipStream_t)stream, &g);
    if (rc != kOk) return rc;
  }
  return kOk;
}

int fgp_nll_fwd(const fgp_nll_desc* desc, void* stream) {
  Nll a;
  int rc = to_nll(desc, a);
  if (rc != kOk) return rc;
  return nll_fwd(a, (hipStream_t)stream, desc->family == FGP_FAMILY_LATTICE);
}

int fgp_spec_inv_eig(const fgp_nll_desc* desc, double* wa, void* stream) {
  Nll a;
  int rc = to_nll(desc, a);
  if (rc != kOk) return rc;
  if (!a.spec || a.mt) return set_error(kErrInvalid, "fgp_spec_inv_eig: needs the spectral desc (basis)");
  if (!wa) return set_error(kErrInvalid, "fgp_spec_inv_eig: null wa");
  return launch_spec_inv_eig(a, wa, (hipStream_t)stream);
}

int fgp_spec_post_var(const fgp_nll_desc* desc, const void* psi, int64_t N, const double* part0, double* out,
                      double* partial, void* stream) {
  Nll a;
  int rc = to_nll(desc, a);
  if (rc != kOk) return rc;
  if (!a.spec || a.mt || a.spec_net || a.basis_stride != 0 || a.d > 4)
    return set_error(kErrInvalid, "fgp_spec_post_var: needs the lattice spectral desc with shared spectra, d <= 4");
  if (N < 0 || N > 4096) return set_error(kErrInvalid, "fgp_spec_post_var: 0 <= N <= 4096");
  if (N == 0) return kOk;
  if (!psi || !part0 || !out || !partial) return set_error(kErrInvalid, "fgp_spec_post_var: null pointer");
  const int64_t half = ((int64_t)1 << a.log2n) / 2;
  const int nblk = (int)((half + 1 + 64 * kSpvKpl - 1) / (64 * kSpvKpl));
  return launch_spec_post_var(a, static_cast<const double2*>(psi), (int)N, part0, out, partial, nblk, kSpvKpl,
                              (hipStream_t)stream);
}

int fgp_nll_lam(const fgp_nll_desc* desc, void* stream) {
  Nll a;
  int rc = to_nll(desc, a);
  if (rc != kOk) return rc;
  if (!desc->grad_lam) return set_error(kErrInvalid, "fgp_nll_lam: null grad_lam (the output)");
  if (a.mt) return set_error(kErrUnsupported, "fgp_nll_lam: not available for the multitask spectral fit");
  if (a.spec) return launch_spec_lam(a, (hipStream_t)stream);
  if (a.re && !a.r2c) {   // n = 2^16: lambda by the full-length kernels (their block count)
    a.re = false;
    a.nb = 1 << (a.log2n - 12);
  }
  hipStream_t st = (hipStream_t)stream;
  const Tables* tb = get_tables(st);
  if (!tb) return set_error(kErrHip, "twiddle table initialisation failed");
  const bool lat = desc->family == FGP_FAMILY_LATTICE;
  if (a.log2n <= 12) return lat ? launch_iter_single<double2>(a, tb, st, true) : launch_iter_single<double>(a, tb, st, true);
  if (lat && a.r2c) {
    rc = launch_r2c(a, 0, tb, st, true);
    return rc != kOk ? rc : launch_r2c(a, 1, tb, st, true);
  }
  if (lat) {
    rc = launch_rows_fwd<double2>(a, tb, st);
    return rc != kOk ? rc : launch_cols_fwd<double2>(a, tb, st, true);
  }
  rc = launch_rows_fwd<double>(a, tb, st);
  return rc != kOk ? rc : launch_cols_fwd<double>(a, tb, st, true);
}

int fgp_nll_partials_len(const fgp_nll_desc* desc, int64_t* len) {
  if (!desc) return set_error(kErrInvalid, "null nll desc");
  fgp_nll_desc probe = *desc;   // the workspace is sized before it exists: placeholder pointers
  static const double dummy = 0.0;
  if (!probe.partials) probe.partials = const_cast<double*>(&dummy);
  if (!probe.ysq) probe.ysq = &dummy;
  if (!probe.raw) probe.raw = &dummy;
  Nll a;
  int rc = to_nll(&probe, a);
  if (rc != kOk) return rc;
  if (!len) return set_error(kErrInvalid, "fgp_nll_partials_len: null len");
  const int64_t nb_doc = std::max<int64_t>(1, ((int64_t)1 << a.log2n) >> 12);
  const int64_t gp = (a.mt > 0 && a.loss == FGP_LOSS_CV) ? a.mt : a.G;   // multitask CV: partials per task
  *len = gp * a.nq * (std::max<int64_t>(a.nb, nb_doc) + 1) + gp;
  if (a.spec) {   // level-1 + level-2 partials + counters of the fused spectral step (fgp_spectral.hip)
    int64_t off;
    int cnt;
    spec_counters_offset(a, &off, &cnt);
    *len = std::max<int64_t>(*len, off + cnt + 1);
    *len = std::max<int64_t>(*len, 3 * (int64_t)a.G * a.nq * a.nb);   // fgp_fit_persist's three partial buffers
  }
  return kOk;
}

int fgp_nll_stage(const fgp_nll_desc* desc, int stage, void* stream) {
  Nll a;
  int rc = to_nll(desc, a);
  if (rc != kOk) return rc;
  return nll_stage(a, stage, (hipStream_t)stream, desc->family == FGP_FAMILY_LATTICE);
}

int fgp_nll_bwd(const fgp_nll_desc* desc, void* stream) {
  Nll a;
  int rc = to_nll(desc, a);
  if (rc != kOk) return rc;
  return nll_bwd(a, (hipStream_t)stream, desc->family == FGP_FAMILY_LATTICE);
}

extern "C++" {
template <typename T>
static int fftbr_real_any(const T* in, int64_t in_batch_stride, void* out, int64_t out_stride, bool half,
                          void* work, int64_t batch, int log2n, void* stream);
}

int fgp_fftbr_real(const double* in, int64_t in_batch_stride, void* out, void* work, int64_t batch, int log2n,
                   void* stream) {
  return fftbr_real_any(in, in_batch_stride, out, (int64_t)1 << log2n, false, work, batch, log2n, stream);
}

int fgp_fftbr_real_half(const double* in, int64_t in_batch_stride, void* out, int64_t out_batch_stride, void* work,
                        int64_t batch, int log2n, void* stream) {
  if (log2n >= 1 && batch > 1 && out_batch_stride < ((int64_t)1 << (log2n - 1)) + 1)
    return set_error(kErrInvalid, "fgp_fftbr_real_half: out row stride below n/2 + 1");
  return fftbr_real_any(in, in_batch_stride, out, out_batch_stride, true, work, batch, log2n, stream);
}

int fgp_fftbr_real_half_f32(const float* in, int64_t in_batch_stride, void* out, int64_t out_batch_stride, void* work,
                            int64_t batch, int log2n, void* stream) {
  if (log2n >= 1 && batch > 1 && out_batch_stride < ((int64_t)1 << (log2n - 1)) + 1)
    return set_error(kErrInvalid, "fgp_fftbr_real_half_f32: out row stride below n/2 + 1");
  return fftbr_real_any(in, in_batch_stride, out, out_batch_stride, true, work, batch, log2n, stream);
}

extern "C++" {
template <typename T>
static int fftbr_real_any(const T* in, int64_t in_batch_stride, void* out, int64_t out_stride, bool half,
                          void* work, int64_t batch, int log2n, void* stream) {
  if (log2n < 17 || log2n > 24 || batch < 0) return set_error(kErrInvalid, "fgp_fftbr_real: needs 17 <= log2n <= 24");
  if (batch == 0) return kOk;
  if (!in || !out || !work) return set_error(kErrInvalid, "fgp_fftbr_real: null pointer");
  if (in_batch_stride < ((int64_t)1 << log2n) && batch > 1)
    return set_error(kErrInvalid, "fgp_fftbr_real: batch stride below n");
  if (((uintptr_t)in & 15) || (in_batch_stride & (16 / sizeof(T) - 1)))
    return set_error(kErrInvalid, "fgp_fftbr_real: in must be 16-byte aligned rows");
  const int64_t tiles = (int64_t)1 << (log2n - 1 - kTileLog);
  if (batch * tiles >= ((int64_t)1 << 31)) return set_error(kErrUnsupported, "fgp_fftbr_real: batch too large");
  hipStream_t st = (hipStream_t)stream;
  const Tables* tb = get_tables(st);
  if (!tb) return set_error(kErrHip, "twiddle table initialisation failed");
  const int mt = log2n - 1, p1 = mt - 12;
  const unsigned grid = (unsigned)(batch * tiles);
  k_fwd_rows_r2c_in<T><<<grid, kWG, 0, st>>>(in, in_batch_stride, log2n, static_cast<double2*>(work), tb->tw4096,
                                             tb->twm[mt]);
  int rc = check_launch("k_fwd_rows_r2c_in");
  if (rc != kOk) return rc;
  Nll a{};
  a.log2n = log2n;
  a.G = (int)batch;
  a.work = work;
  a.grad_lam = out;
  a.out_stride = out_stride;
  a.stamps = nullptr;
  switch (p1) {
#define FGP_C(PP)                                                                                   \
  case PP:                                                                                          \
    if (half) k_fwd_cols_r2c<PP, 3><<<grid, kWG, 0, st>>>(a, tb->tw4096, tb->twm[log2n]);           \
    else k_fwd_cols_r2c<PP, 1><<<grid, kWG, 0, st>>>(a, tb->tw4096, tb->twm[log2n]);                \
    break;
    FGP_C(4) FGP_C(5) FGP_C(6) FGP_C(7) FGP_C(8) FGP_C(9) FGP_C(10) FGP_C(11)
#undef FGP_C
    default: return set_error(kErrInvalid, "bad r2c m1");
  }
  return check_launch("k_fwd_cols_r2c");
}
}  // extern "C++"

static int ifftbr_real_any(const void* in, int64_t in_batch_stride, const void* f, bool freal, int64_t f_batch_stride,
                           double* out, int64_t out_batch_stride, void* work, int64_t batch, int log2n, void* stream) {
  if (log2n < 17 || log2n > 24 || batch < 0) return set_error(kErrInvalid, "fgp_ifftbr_real: needs 17 <= log2n <= 24");
  if (batch == 0) return kOk;
  if (!in || !out || !work) return set_error(kErrInvalid, "fgp_ifftbr_real: null pointer");
  const int64_t n = (int64_t)1 << log2n;
  // the Hermitian-input variant (fgp_ifftbr_real_rf) reads only k <= n/2: rows of n/2 + 1 (a half spectrum) do
  if (batch > 1 && (in_batch_stride < (freal ? n / 2 + 1 : n) || out_batch_stride < n))
    return set_error(kErrInvalid, "fgp_ifftbr_real: batch stride below n");
  if (((uintptr_t)out & 15) || (out_batch_stride & 1)) return set_error(kErrInvalid, "fgp_ifftbr_real: out must be 16-byte aligned rows");
  const int64_t tiles = (int64_t)1 << (log2n - 1 - kTileLog);
  if (batch * tiles >= ((int64_t)1 << 31)) return set_error(kErrUnsupported, "fgp_ifftbr_real: batch too large");
  hipStream_t st = (hipStream_t)stream;
  const Tables* tb = get_tables(st);
  if (!tb) return set_error(kErrHip, "twiddle table initialisation failed");
  const int mt = log2n - 1, p1 = mt - 12;
  const unsigned grid = (unsigned)(batch * tiles);
  const double2* X = static_cast<const double2*>(in);
  double2* wk = static_cast<double2*>(work);
  switch (p1) {
#define FGP_C(PP)                                                                                                \
  case PP:                                                                                                       \
    if (freal) k_inv_cols_c2r<PP, true, true><<<grid, kWG, 0, st>>>(X, in_batch_stride, f, f_batch_stride, wk,  \
                                                                    log2n, tb->tw4096, tb->twm[log2n]);          \
    else k_inv_cols_c2r<PP, false, false><<<grid, kWG, 0, st>>>(X, in_batch_stride, f, f_batch_stride, wk,      \
                                                                log2n, tb->tw4096, tb->twm[log2n]);              \
    break;
    FGP_C(4) FGP_C(5) FGP_C(6) FGP_C(7) FGP_C(8) FGP_C(9) FGP_C(10) FGP_C(11)
#undef FGP_C
    default: return set_error(kErrInvalid, "bad c2r m1");
  }
  int rc = check_launch("k_inv_cols_c2r");
  if (rc != kOk) return rc;
  k_inv_rows_c2r<<<grid, kWG, 0, st>>>(wk, log2n, out, out_batch_stride, tb->tw4096, tb->twm[mt]);
  return check_launch("k_inv_rows_c2r");
}

int fgp_ifftbr_real(const void* in, int64_t in_batch_stride, const void* f, int64_t f_batch_stride, double* out,
                    int64_t out_batch_stride, void* work, int64_t batch, int log2n, void* stream) {
  return ifftbr_real_any(in, in_batch_stride, f, false, f_batch_stride, out, out_batch_stride, work, batch, log2n,
                         stream);
}

int fgp_ifftbr_real_rf(const void* in, int64_t in_batch_stride, const double* f, int64_t f_batch_stride, double* out,
                       int64_t out_batch_stride, void* work, int64_t batch, int log2n, void* stream) {
  if (!f) return set_error(kErrInvalid, "fgp_ifftbr_real_rf: null factor rows");
  return ifftbr_real_any(in, in_batch_stride, f, true, f_batch_stride, out, out_batch_stride, work, batch, log2n,
                         stream);
}

}  // extern "C"

namespace fgp {

int spec_basis_r2c(const double* parts, int d, int log2n, int s0, int cnt, double* basis, void* work, hipStream_t st,
                   const GenSpec* gen) {
  if (log2n < 17 || log2n > 24 || d < 1 || d > kSpecMaxD || cnt < 1 || s0 < 0 || s0 + cnt > (1 << d))
    return set_error(kErrInvalid, "spec_basis_r2c: bad shape");
  const int64_t n = (int64_t)1 << log2n, nt = n >> 1;
  const int64_t tiles = nt >> kTileLog;
  const Tables* tb = get_tables(st);
  if (!tb) return set_error(kErrHip, "twiddle table initialisation failed");
  const int ns = 1 << d, mt = log2n - 1, p1 = mt - 12;
  // the last chunk holds n/2 and 63 zeros of padding: zero the subsets' runs before the kernel writes n/2
  if (hipMemsetAsync(basis + spec_pos(nt, ns) + 64 * (int64_t)s0, 0, sizeof(double) * 64 * (size_t)cnt, st) != hipSuccess)
    return set_error(kErrHip, "spec_basis_r2c: memset failed");
  const unsigned grid = (unsigned)(tiles * cnt);
  double2* wk = static_cast<double2*>(work);
  if (gen) {
    auto go = [&](auto oc) {
      constexpr int O = decltype(oc)::value;
      switch (d) {
#define FGP_R(DD) case DD: k_fwd_rows_r2c_gen<DD, O><<<grid, kWG, 0, st>>>(*gen, log2n, s0, cnt, wk, tb->tw4096, tb->twm[mt]); break;
        FGP_R(1) FGP_R(2) FGP_R(3) FGP_R(4) FGP_R(5) FGP_R(6)
#undef FGP_R
      }
    };
    switch (gen->order) {
      case 2: go(std::integral_constant<int, 2>{}); break;
      case 4: go(std::integral_constant<int, 4>{}); break;
      case 6: go(std::integral_constant<int, 6>{}); break;
      case 8: go(std::integral_constant<int, 8>{}); break;
      default: return set_error(kErrUnsupported, "Bernoulli order %d unsupported", gen->order);
    }
  } else {
    switch (d) {
#define FGP_R(DD) case DD: k_fwd_rows_r2c_prod<DD><<<grid, kWG, 0, st>>>(parts, log2n, s0, cnt, wk, tb->tw4096, tb->twm[mt]); break;
      FGP_R(1) FGP_R(2) FGP_R(3) FGP_R(4) FGP_R(5) FGP_R(6)
#undef FGP_R
    }
  }
  int rc = check_launch(gen ? "k_fwd_rows_r2c_gen" : "k_fwd_rows_r2c_prod");
  if (rc != kOk) return rc;
  Nll a{};
  a.log2n = log2n;
  a.G = cnt;
  a.d = d;
  a.work = work;
  a.grad_lam = basis + 64 * (int64_t)s0;
  a.stamps = nullptr;
  switch (p1) {
#define FGP_C(PP) case PP: k_fwd_cols_r2c<PP, 2><<<grid, kWG, 0, st>>>(a, tb->tw4096, tb->twm[log2n]); break;
    FGP_C(4) FGP_C(5) FGP_C(6) FGP_C(7) FGP_C(8) FGP_C(9) FGP_C(10) FGP_C(11)
#undef FGP_C
    default: return set_error(kErrInvalid, "bad r2c m1");
  }
  return check_launch("k_fwd_cols_r2c");
}

// fgp_handoff_check's device buffer while armed (kHandoffWords XOR words, checks, mismatches)
static unsigned long long* g_handoff_check = nullptr;

}  // namespace fgp

extern "C" {

int fgp_fit_step(const fgp_nll_desc* nll, const fgp_fit_desc* fit, int iter, int do_update, void* stream) {
  Nll a;
  Fit f;
  int rc = to_nll(nll, a);
  if (rc == kOk) rc = to_fit(fit, f);
  if (rc == kOk) rc = check_per_problem(a, f);
  if (rc != kOk) return rc;
  return fit_step(a, f, iter, do_update, (hipStream_t)stream);
}

int fgp_fit_persist_ok(const fgp_nll_desc* nll, int* ok) {
  if (!ok) return set_error(kErrInvalid, "fgp_fit_persist_ok: null ok");
  *ok = 0;
  fgp_nll_desc probe = *nll;
  static const double dummy = 0.0;
  if (!probe.partials) probe.partials = const_cast<double*>(&dummy);
  if (!probe.ysq) probe.ysq = &dummy;
  if (!probe.raw) probe.raw = &dummy;
  Nll a;
  int rc = to_nll(&probe, a);
  if (rc != kOk) return rc;
  int W, bpw;
  size_t shm;
  *ok = spec_persist_geometry(a, &W, &bpw, &shm) == kOk ? W : 0;
  return kOk;
}

int fgp_fit_persist(const fgp_nll_desc* nll, const fgp_fit_desc* fit, int iters, double logtol, int wait_max, void* ctrl,
                    void* stream) {
  Nll a;
  Fit f;
  int rc = to_nll(nll, a);
  if (rc == kOk) rc = to_fit(fit, f);
  if (rc != kOk) return rc;
  if (!ctrl) return set_error(kErrInvalid, "fgp_fit_persist: null ctrl");
  if (iters < 0 || wait_max < 1) return set_error(kErrInvalid, "fgp_fit_persist: iters / wait_max");
  unsigned* counter = static_cast<unsigned*>(ctrl);
  return launch_spec_persist(a, f, iters, logtol, wait_max, counter, reinterpret_cast<int*>(counter + 1),
                             (hipStream_t)stream);
}

int fgp_set_persist_poll_max(long long polls) {
  set_persist_poll_max(polls);
  return kOk;
}

int fgp_persist_giveups(unsigned long long* count, int reset) {
  if (!count) return set_error(kErrInvalid, "fgp_persist_giveups: null count");
  return persist_giveups(count, reset);
}

int fgp_handoff_check(int enable, unsigned long long* out) {
  const size_t bytes = sizeof(unsigned long long) * (kHandoffWords + 2);
  if (enable) {
    if (!g_handoff_check && hipMalloc(reinterpret_cast<void**>(&g_handoff_check), bytes) != hipSuccess) {
      g_handoff_check = nullptr;
      return set_error(kErrHip, "fgp_handoff_check: allocation failed");
    }
    if (hipMemset(g_handoff_check, 0, bytes) != hipSuccess) return set_error(kErrHip, "fgp_handoff_check: reset failed");
    return kOk;
  }
  if (!out) return set_error(kErrInvalid, "fgp_handoff_check: out is null");
  out[0] = out[1] = 0;
  if (!g_handoff_check) return kOk;
  if (hipDeviceSynchronize() != hipSuccess ||
      hipMemcpy(out, g_handoff_check + kHandoffWords, 2 * sizeof(unsigned long long), hipMemcpyDeviceToHost) != hipSuccess)
    return set_error(kErrHip, "fgp_handoff_check: read-back failed");
  (void)hipFree(g_handoff_check);
  g_handoff_check = nullptr;
  return kOk;
}

}  // extern "C"

static int fit_run_enqueue(const fgp_nll_desc* nll, const fgp_fit_desc* fit, int iter0, int iters, int final_no_update,
                           void* stream) {
  Nll a;
  Fit f;
  int rc = to_nll(nll, a);
  if (rc == kOk) rc = to_fit(fit, f);
  if (rc == kOk) rc = check_per_problem(a, f);
  if (rc != kOk) return rc;
  const bool lat = nll->family == FGP_FAMILY_LATTICE;
  hipStream_t st = (hipStream_t)stream;
  // real-even kernels, independent problems: the reduction + Rprop step runs in the backward kernel's
  // last workgroup per problem, with G counters in the documented partials workspace past the
  // G (4 + d) (nb + 1) doubles the kernels use (room while nb < n / 4096)
  const int64_t nb_doc = std::max<int64_t>(1, ((int64_t)1 << a.log2n) >> 12);
  // spectral tile kernel: the whole iteration (and the step, in its last workgroup) is one launch
  const bool fuse_spec = a.spec && a.spec_tile && f.per_problem && a.G <= 8 && iters > 0;
  const bool fuse = (a.re && f.per_problem && a.nb < nb_doc && iters > 0) || fuse_spec;
  FitFuse fz{};
  const Tables* tb = nullptr;
  if (fuse) {
    fz.f = f;
    int ncnt = a.G;
    if (fuse_spec) {
      int64_t off;
      spec_counters_offset(a, &off, &ncnt);
      fz.counters = reinterpret_cast<unsigned*>(a.partials + off);
    } else {
      fz.counters = reinterpret_cast<unsigned*>(a.partials + (int64_t)a.G * a.nq * (a.nb + 1));
      tb = get_tables(st);
      if (!tb) return set_error(kErrHip, "twiddle table initialisation failed");
    }
    if (hipMemsetAsync(fz.counters, 0, sizeof(unsigned) * (size_t)ncnt, st) != hipSuccess)
      return set_error(kErrHip, "fgp_fit_run: counter reset failed");
    if (fuse_spec) fz.check = g_handoff_check;
  }
  const char* pe = getenv("FGP_SPEC_PERSIST");   // (opt-in until measured on the device: FGP_SPEC_PERSIST=1)
  if (fuse_spec && pe && pe[0] == '1' && spec_nparams(a) <= kSpecStateMax) {
    // every iteration and the last step in ONE persistent k_spec_tile launch (falls through to the launch
    // per iteration when the grid cannot be co-resident)
    fz.iter = iter0;
    fz.par = iter0 & 1;
    fz.pending = 0;
    fz.piters = iters;
    fz.sin = fz.sout = RpState{f.raw, f.prev, f.step};
    fz.do_update = !final_no_update;
    rc = launch_spec_iter(a, st, &fz);
    if (rc != kErrUnsupported) return rc;
    fz.piters = 0;
  }
  if (fuse_spec) {
    // one k_spec_tile launch per iteration; the step of iteration i runs in launch i + 1's prologue (its
    // state read from the fit's vectors for the first step, else from the scratch copy of parity i,
    // written to parity i + 1) and the last one in k_spec_finish_step, back into the fit's vectors
    const RpState own{f.raw, f.prev, f.step};
    for (int it = 0; it <= iters; ++it) {
      const int i = iter0 + it;
      fz.iter = i;
      fz.par = i & 1;
      fz.pending = it > 0;
      fz.sin = it <= 1 ? own : spec_scratch_state(a, (i - 1) & 1);
      fz.sout = it == iters ? own : spec_scratch_state(a, i & 1);
      if (it == iters) {
        fz.do_update = !final_no_update;
        return launch_spec_finish_step(a, fz, st);
      }
      if ((rc = launch_spec_iter(a, st, &fz)) != kOk) return rc;
    }
    return kOk;
  }
  const bool many = a.spec && !f.per_problem && a.nb <= kSpecBlocks && !getenv_off("FGP_SPEC_STEP_MANY");
  if (many && iters > 0 && hipMemsetAsync(spec_step_many_counter(a), 0, sizeof(unsigned), st) != hipSuccess)
    return set_error(kErrHip, "fgp_fit_run: counter reset failed");
  for (int it = 0; it < iters; ++it) {
    const int upd = !(final_no_update && it == iters - 1);
    if ((rc = nll_fwd(a, st, lat)) != kOk) return rc;
    if (fuse) {
      fz.iter = iter0 + it;
      fz.do_update = upd;
      if ((rc = launch_re_bwd_fused(a, fz, tb, st)) != kOk) return rc;
      continue;
    }
    if ((rc = nll_bwd(a, st, lat)) != kOk) return rc;
    if ((rc = fit_step(a, f, iter0 + it, upd, st, many)) != kOk) return rc;
  }
  return kOk;
}

// ---------------------------------------------------------------- fgp_fit_run_graph (ABI 17)
// An eager launch costs the device ~3 us more than the same launch replayed from a graph (the eager dispatch's
// system-scope release: DESIGN.md section 8), i.e. ~150 us per C4 fit of 51 launches.  fgp_fit_run_graph captures the
// launch sequence of fgp_fit_run (thread-local mode, on a library side stream: torch's default stream cannot capture)
// into a hipGraph and replays it on the caller's stream.  Executable graphs are cached per caller token (one fit
// engine: its buffers never move) and the call's exact arguments (the descriptors' bytes, the iteration range, the
// device, the hand-off check hook, the library's A/B environment switches); a repeated call replays at once.  (Keyed
// by the arguments alone, a replay for ANOTHER engine whose buffers happened to sit at the same addresses returned
// garbage in the GPU suite -- not understood, so graphs are never shared between engines.)  Results are
// bit-identical to the eager sequence: the same kernels with the same arguments.  A stream that is itself capturing
// (bench.py's whole-step graph), a non-spectral desc or a capture error take the eager sequence.
namespace {
struct FitGraph {
  long long token;
  std::vector<unsigned char> key;
  int dev;
  hipGraph_t graph;
  hipGraphExec_t exec;
  hipEvent_t done;           // recorded after each launch: an evicted graph is destroyed only once it has finished
  unsigned long long used;
};
std::mutex g_fg_mu;
std::vector<FitGraph> g_fit_graphs;
unsigned long long g_fg_clock = 0;
hipStream_t g_fg_side[64] = {};
long long g_fg_stats[3] = {0, 0, 0};         // replays of a cached graph, captures, eager calls
constexpr size_t kFitGraphCache = 16;
}  // namespace

static void key_put(std::vector<unsigned char>& k, const void* p, size_t n) {
  const unsigned char* b = static_cast<const unsigned char*>(p);
  k.insert(k.end(), b, b + n);
}

static int fit_graph_wanted(const fgp_nll_desc* nll, hipStream_t st) {
  if (!nll || !nll->basis || nll->mt_tasks > 0) return 0;      // the spectral single-task fits
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return cs == hipStreamCaptureStatusNone;
}

static void fit_graph_free(FitGraph& e) {
  if (e.done) (void)hipEventSynchronize(e.done);
  if (e.exec) (void)hipGraphExecDestroy(e.exec);
  if (e.graph) (void)hipGraphDestroy(e.graph);
  if (e.done) (void)hipEventDestroy(e.done);
  e.exec = nullptr;
  e.graph = nullptr;
  e.done = nullptr;
}

static int fit_graph_launch(FitGraph& e, hipStream_t st) {
  e.used = ++g_fg_clock;
  if (hipGraphLaunch(e.exec, st) != hipSuccess || hipEventRecord(e.done, st) != hipSuccess)
    return set_error(kErrHip, "fgp_fit_run_graph: hipGraphLaunch failed");
  return kOk;
}

extern "C" {

int fgp_fit_run(const fgp_nll_desc* nll, const fgp_fit_desc* fit, int iter0, int iters, int final_no_update,
                void* stream) {
  return fit_run_enqueue(nll, fit, iter0, iters, final_no_update, stream);
}

int fgp_fit_run_graph(const fgp_nll_desc* nll, const fgp_fit_desc* fit, int iter0, int iters, int final_no_update,
                      long long token, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (!nll || !fit || !fit_graph_wanted(nll, st)) {
    std::lock_guard<std::mutex> lock(g_fg_mu);
    ++g_fg_stats[2];
    return fit_run_enqueue(nll, fit, iter0, iters, final_no_update, stream);
  }
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64)
    return set_error(kErrHip, "fgp_fit_run_graph: hipGetDevice");
  std::vector<unsigned char> key;
  key.reserve(sizeof(*nll) + sizeof(*fit) + 128);
  key_put(key, nll, sizeof(*nll));
  key_put(key, fit, sizeof(*fit));
  const int ints[4] = {iter0, iters, final_no_update, dev};
  key_put(key, ints, sizeof(ints));
  const void* hook = g_handoff_check;
  key_put(key, &hook, sizeof(hook));
  // the library's A/B switches that choose kernels / workspace layouts for a desc are inputs of the sequence too
  for (const char* nm : {"FGP_SPEC_TILE", "FGP_SPEC_SLICE_NB", "FGP_SPEC_PERSIST", "FGP_SPEC_STEP_MANY", "FGP_R2C"}) {
    const char* v = getenv(nm);
    key_put(key, nm, strlen(nm));
    if (v) key_put(key, v, strlen(v) + 1);
    else key.push_back(0xff);
  }
  std::lock_guard<std::mutex> lock(g_fg_mu);
  for (auto& e : g_fit_graphs)
    if (e.token == token && e.dev == dev && e.key == key) {
      ++g_fg_stats[0];
      return fit_graph_launch(e, st);
    }
  if (!g_fg_side[dev] && hipStreamCreateWithFlags(&g_fg_side[dev], hipStreamNonBlocking) != hipSuccess) {
    g_fg_side[dev] = nullptr;
    return set_error(kErrHip, "fgp_fit_run_graph: side stream");
  }
  hipStream_t cap = g_fg_side[dev];
  if (hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal) != hipSuccess) {
    (void)hipGetLastError();
    ++g_fg_stats[2];
    return fit_run_enqueue(nll, fit, iter0, iters, final_no_update, stream);
  }
  const int rc = fit_run_enqueue(nll, fit, iter0, iters, final_no_update, cap);
  hipGraph_t g = nullptr;
  const hipError_t ec = hipStreamEndCapture(cap, &g);
  hipGraphExec_t exec = nullptr;
  hipEvent_t done = nullptr;
  if (rc != kOk || ec != hipSuccess || !g || hipGraphInstantiate(&exec, g, nullptr, nullptr, 0) != hipSuccess ||
      hipEventCreateWithFlags(&done, hipEventDisableTiming) != hipSuccess) {
    if (exec) (void)hipGraphExecDestroy(exec);
    if (g) (void)hipGraphDestroy(g);
    (void)hipGetLastError();
    if (rc != kOk) return rc;                       // an argument error: reported as the eager call would
    ++g_fg_stats[2];
    return fit_run_enqueue(nll, fit, iter0, iters, final_no_update, stream);
  }
  ++g_fg_stats[1];
  FitGraph* slot = nullptr;
  if (g_fit_graphs.size() >= kFitGraphCache) {       // evict a released engine's graph, else the least recently used
    slot = &g_fit_graphs[0];
    for (auto& e : g_fit_graphs)
      if ((e.token < 0) > (slot->token < 0) || ((e.token < 0) == (slot->token < 0) && e.used < slot->used)) slot = &e;
    fit_graph_free(*slot);
  } else {
    g_fit_graphs.push_back(FitGraph{});
    slot = &g_fit_graphs.back();
  }
  slot->token = token;
  slot->key = std::move(key);
  slot->dev = dev;
  slot->graph = g;
  slot->exec = exec;
  slot->done = done;
  return fit_graph_launch(*slot, st);
}

int fgp_fit_graph_release(long long token) {
  std::lock_guard<std::mutex> lock(g_fg_mu);
  for (auto& e : g_fit_graphs)
    if (e.token == token) e.token = -1;             // never launched again; freed when evicted
  return kOk;
}

int fgp_fit_graph_stats(long long* out) {
  if (!out) return set_error(kErrInvalid, "fgp_fit_graph_stats: null out");
  std::lock_guard<std::mutex> lock(g_fg_mu);
  for (int i = 0; i < 3; ++i) out[i] = g_fg_stats[i];
  return kOk;
}

}  // extern "C"
