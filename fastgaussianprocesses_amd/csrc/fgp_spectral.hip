// Part-product spectra: the spectral fit path (ABI 11; multitask ABI 12).  See DESIGN.md section 3 "Spectral fit".
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
#include <cstdlib>

#include "fgp_nll.h"

// The last-arriver hand-offs of this file (k_spec_tile, k_spec_step_many) publish sc1 partial stores with a
// relaxed agent-scope add after `s_waitcnt vmcnt(0)`: on gfx9 (CDNA) vmcnt also counts the stores, so the
// add cannot overtake them (MI355X_MICROARCH.md hand-off row 1).  gfx10+ counts stores separately (vscnt):
// building for such a target needs a release fence before the add.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__GFX9__)
#error "fgp_spectral.hip: the relaxed sc1 hand-offs assume gfx9 (CDNA) store counting -- build for gfx950"
#endif

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

// Layout of the spectra (fgp_spec_basis): chunks of 64 frequencies, each holding the 2^d spectra of its
// frequencies contiguously -- [chunk][S][64], frequency k of spectrum S at (k / 64) 2^d 64 + 64 S + k mod 64
// (the lattice's k = n/2 in chunk n/128, zero padding after it).  A wave's 64 frequencies of every S, and
// an LDS tile chunk, are then one contiguous 2^d x 512-byte run instead of 2^d rows n/2 apart.
template <int NS>
__device__ __forceinline__ int64_t spec_at(int64_t k, int s) {
  return ((k >> 6) * NS + s) * 64 + (k & 63);
}

// Y of problem g at frequency k: rows [G][ysq_stride], or (ysq_chunked, the spectral path's copy) the
// chunked layout [k / 64][G][64] -- a chunk's Y of every problem then follows as one contiguous run
__device__ __forceinline__ int64_t ysq_at(const Nll& a, int g, int64_t k) {
  return a.ysq_chunked ? ((k >> 6) * a.G + g) * 64 + (k & 63) : (int64_t)g * a.ysq_stride + k;
}

// Per-problem accumulators of one lane (its frequencies of one block): UNWEIGHTED sums over them --
// the lattice's fold weights (2 for 0 < k < n/2, 1 at k = 0 and n/2) are applied once per block
// (spec_block_partials), not per frequency.
template <int D>
struct SpecAcc {
  double norm = 0.0, ge = 0.0, gs = 0.0, mant = 1.0;
  double gl[D];
  int ex = 0;
  __device__ __forceinline__ SpecAcc() {
#pragma unroll
    for (int j = 0; j < D; ++j) gl[j] = 0.0;
  }
};

// 1 / e: v_rcp_f64 and two Newton steps (within an ulp of the quotient; 5 VALU instead of the ~11 of
// the IEEE division sequence)
__device__ __forceinline__ double rcp_nr(double e) {
  double r = __builtin_amdgcn_rcp(e);
  r = __builtin_fma(__builtin_fma(-e, r, 1.0), r, r);
  return __builtin_fma(__builtin_fma(-e, r, 1.0), r, r);
}

// One frequency of one problem: ev = sqrt(n) scale P + noise and the loss terms of eig_terms (fgp_nll.h)
// with weight 1: norm += Y / ev, log|ev| (frexp mantissa product + exponent sum), and g = wl / ev - Y / ev^2
// (= 2 dL/dev) into dL/dnoise, the scale term g P and the lengthscale terms g dP/dl_j.
template <int D>
__device__ __forceinline__ void spec_terms(const double* phi, const Hyp& h, double rootn, double wl, double Y,
                                           SpecAcc<D>& acc) {
  double dp[D];
  const double P = mlin<D>(phi, h.ls, dp);
  const double e = __builtin_fma(rootn, h.scale * P, h.noise);
  const double r = rcp_nr(e);
  acc.norm = __builtin_fma(Y, r, acc.norm);
  int ex;
  const double m = frexp(fabs(e), &ex);
  acc.mant *= m;
  acc.ex += ex;
  const double g = r * __builtin_fma(-Y, r, wl);
  acc.ge += g;
  acc.gs = __builtin_fma(g, P, acc.gs);
#pragma unroll
  for (int j = 0; j < D; ++j) acc.gl[j] = __builtin_fma(g, dp[j], acc.gl[j]);
}

// spec_terms split in two (k_spec_persist): the per-frequency values of a chunk, then their accumulation -- two chunks'
// values computed side by side (independent chains a single wave per SIMD can overlap) and accumulated in chunk
// order, so the sums are spec_terms' bit for bit.
template <int D>
struct SpecTerm {
  double Y, r, m, g, P;
  double dp[D];
  int ex;
};

template <int D>
__device__ __forceinline__ void spec_term_values(const double* phi, const Hyp& h, double rootn, double wl, double Y,
                                                 SpecTerm<D>& t) {
  t.P = mlin<D>(phi, h.ls, t.dp);
  const double e = __builtin_fma(rootn, h.scale * t.P, h.noise);
  t.r = rcp_nr(e);
  t.Y = Y;
  t.m = frexp(fabs(e), &t.ex);
  t.g = t.r * __builtin_fma(-Y, t.r, wl);
}

template <int D>
__device__ __forceinline__ void spec_term_add(const SpecTerm<D>& t, SpecAcc<D>& acc) {
  acc.norm = __builtin_fma(t.Y, t.r, acc.norm);
  acc.mant *= t.m;
  acc.ex += t.ex;
  acc.ge += t.g;
  acc.gs = __builtin_fma(t.g, t.P, acc.gs);
#pragma unroll
  for (int j = 0; j < D; ++j) acc.gl[j] = __builtin_fma(t.g, t.dp[j], acc.gl[j]);
}

// One lane of a double through a DPP pattern (two 32-bit moves; every source lane valid for the patterns used)
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}

// The sum over the 64 lanes of a wave in a fixed order (valid in every lane 0..63 of each 16-lane row, the total
// from the four row sums): DPP quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror, row_mirror (VALU-latency moves
// instead of six LDS-crossbar ds_bpermute rounds of a butterfly), then ((r0 + r16) + (r32 + r48)) by v_readlane.
// Deterministic; the spectral kernels' per-block partials all use it, so they agree bit for bit.
__device__ __forceinline__ double wave_sum_dpp(double v) {
  v += dpp_f64<0xB1>(v);    // quad_perm [1,0,3,2]: pairs
  v += dpp_f64<0x4E>(v);    // quad_perm [2,3,0,1]: quads
  v += dpp_f64<0x141>(v);   // row_half_mirror (lane i <-> 7 - i): 8 lanes
  v += dpp_f64<0x140>(v);   // row_mirror (lane i <-> 15 - i): the 16-lane row
  return (read_lane(v, 0) + read_lane(v, 16)) + (read_lane(v, 32) + read_lane(v, 48));
}

// Two doubles exchange halves of the wave (gfx950 v_permlane32_swap: lanes 32-63 of x <-> lanes 0-31 of y) or
// rows (v_permlane16_swap: the odd 16-lane rows of x <-> the even rows of y), one 32-bit word at a time
template <bool R32>
__device__ __forceinline__ void swap_f64(double& x, double& y) {
  const unsigned xl = (unsigned)__double2loint(x), yl = (unsigned)__double2loint(y);
  const unsigned xh = (unsigned)__double2hiint(x), yh = (unsigned)__double2hiint(y);
  if constexpr (R32) {
    const auto lo = __builtin_amdgcn_permlane32_swap(xl, yl, false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap(xh, yh, false, false);
    x = __hiloint2double((int)hi[0], (int)lo[0]);
    y = __hiloint2double((int)hi[1], (int)lo[1]);
  } else {
    const auto lo = __builtin_amdgcn_permlane16_swap(xl, yl, false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap(xh, yh, false, false);
    x = __hiloint2double((int)hi[0], (int)lo[0]);
    y = __hiloint2double((int)hi[1], (int)lo[1]);
  }
}

// The wave sums of eight values at once, a transposed butterfly: each stage halves the values a lane still
// carries instead of reducing every value through all six stages.  lane ^ 32 (permlane32 swap of v[j], v[j + 4]:
// lanes 0-31 then sum v[j], 32-63 v[j + 4]), lane ^ 16 (permlane16 swap of those: row r of b[j] sums v[j + 2 r]),
// lane ^ 8 (DPP row_ror 8 of the value the lane's half-row does not keep), then the 8-lane group by DPP
// quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror.  Every lane of the group lane >> 3 = q holds the sum of v[q].
// Fixed order, deterministic; ~35 VALU for the eight values against ~23 per value one at a time (wave_sum_dpp).
__device__ __forceinline__ double wave_sum8(const double* v, int lane) {
  double a[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    double x = v[j], y = v[j + 4];
    swap_f64<true>(x, y);
    a[j] = x + y;
  }
  double b[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    double x = a[j], y = a[j + 2];
    swap_f64<false>(x, y);
    b[j] = x + y;
  }
  const bool odd = (lane & 8) != 0;
  double c = (odd ? b[1] : b[0]) + dpp_f64<0x128>(odd ? b[0] : b[1]);   // row_ror:8 = lane ^ 8 in the row
  c += dpp_f64<0xB1>(c);
  c += dpp_f64<0x4E>(c);
  c += dpp_f64<0x141>(c);
  return c;
}

// v[0..3+D] of one accumulator set: norm, log|ev| sum, g sum, g P sum, g dP/dl_j sums
template <int D>
__device__ __forceinline__ void spec_values(const SpecAcc<D>& acc, double* v) {
  v[0] = acc.norm;
  v[1] = log(acc.mant) + (double)acc.ex * 0.69314718055994530942;
  v[2] = acc.ge;
  v[3] = acc.gs;
#pragma unroll
  for (int j = 0; j < D; ++j) v[4 + j] = acc.gl[j];
}

// The block's partials of problem g from the lanes' unweighted sums: weights (lattice: 2 per frequency,
// then k = 0 taken back to weight 1 in lane 0 of block 0 and k = n/2 added with weight 1 in lane 0 of the
// last block; nets: 1), dL/dev = g / 2, wave sums (fixed shuffle order), the gradient factors
// (dL/dlambda = sqrt(n) dL/dev; dlambda/draw_scale = lambda, dlambda/draw_l_j = scale l_j dP/dl_j) and
// one store per quantity by lane 0 (sc1 when handed to a last-workgroup reduction).  The single-frequency
// corrections reload their spectra and Y from global memory, so every kernel computes the same values.
// The lattice's single-frequency corrections (k = 0 and k = n/2) of a wave's first / last block, loaded at the
// start of a launch (their latency then hides under the chunk stream instead of sitting in the block's
// epilogue, the critical path of the group hand-off / grid barrier): one double per lane -- phi0[s] / phi1[s]
// the spectra at k = 0 / n/2 (lane s), y[p] / y[32 + p] Y of the wave's problem g0 + p at k = 0 / n/2 --
// read back by v_readlane.  on = false: spec_block_partials loads them itself.
struct SpecCorr {
  double phi0, phi1, y;
  int g0;
  bool on;
};

// load the wave's corrections (wave-uniform condition: the wave holds block 0 or the last block)
template <int NS>
__device__ __forceinline__ SpecCorr spec_corr_load(const Nll& a, int blk, int g0, int cnt) {
  SpecCorr c{0.0, 0.0, 0.0, g0, false};
  if (a.spec_net || !(blk == 0 || blk == a.nb - 1)) return c;
  const int lane = tid_fresh() & 63;
  const double* phib = a.basis + (int64_t)g0 * a.basis_stride;
  if (lane < NS) {
    c.phi0 = phib[spec_at<NS>(0, lane)];
    c.phi1 = phib[spec_at<NS>(a.spec_main, lane)];
  }
  const int p = lane & 31;
  if (p < cnt) c.y = a.ysq[ysq_at(a, g0 + p, lane < 32 ? 0 : a.spec_main)];
  c.on = true;
  return c;
}

// global (address space 1) views of the partial buffers: the agent-scope accesses of the cross-workgroup hand-offs
// become global_load / global_store ... sc1 (MI355X_MICROARCH.md: sc1 loads to registers, never flat_)
typedef __attribute__((address_space(1))) double gdouble;
__device__ __forceinline__ gdouble* gptr(const double* p) { return (gdouble*)(const_cast<double*>(p)); }
__device__ __forceinline__ void st_part_sc1(double* p, double v) {
  __hip_atomic_store(gptr(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int D, bool NET>
__device__ __forceinline__ void spec_block_partials(const Nll& a, const Hyp& h, int g, int blk, double rootn, double wl,
                                                    const SpecAcc<D>& acc, bool sc1, double* pbase,
                                                    const SpecCorr& corr = SpecCorr{0.0, 0.0, 0.0, 0, false}) {
  constexpr int NS = 1 << D, NV = 4 + D;
  const int lane = tid_fresh() & 63;
  double v[NV];
  spec_values<D>(acc, v);
  const double wlin = NET ? 1.0 : 2.0;
  v[0] *= wlin;
  v[1] *= wlin;
#pragma unroll
  for (int q = 2; q < NV; ++q) v[q] *= 0.5 * wlin;
  if (!NET && lane == 0 && (blk == 0 || blk == a.nb - 1)) {
    const double* phib = a.basis + (int64_t)g * a.basis_stride;
#pragma unroll
    for (int side = 0; side < 2; ++side) {
      const bool here = side == 0 ? blk == 0 : blk == a.nb - 1;
      if (!here) continue;
      const int64_t k = side == 0 ? 0 : a.spec_main;
      double phi[NS];
      // (v_readlane of the preloaded values: exec-independent, inside the lane-0 branch)
#pragma unroll
      for (int s = 0; s < NS; ++s)
        phi[s] = corr.on ? read_lane(side == 0 ? corr.phi0 : corr.phi1, s) : phib[spec_at<NS>(k, s)];
      const double yk = corr.on ? read_lane(corr.y, (side == 0 ? 0 : 32) + g - corr.g0) : a.ysq[ysq_at(a, g, k)];
      SpecAcc<D> t;
      spec_terms<D>(phi, h, rootn, wl, yk, t);
      double tv[NV];
      spec_values<D>(t, tv);
      const double sg = side == 0 ? -1.0 : 1.0;   // k = 0: weight 2 -> 1; k = n/2: weight 1
      v[0] = __builtin_fma(sg, tv[0], v[0]);
      v[1] = __builtin_fma(sg, tv[1], v[1]);
#pragma unroll
      for (int q = 2; q < NV; ++q) v[q] = __builtin_fma(0.5 * sg, tv[q], v[q]);
    }
  }
  // quantities 0..7 by the transposed butterfly (zeros past NV), the rest (D >= 5) one at a time
  double t8[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) t8[q] = q < NV ? v[q] : 0.0;
  const double s8 = wave_sum8(t8, lane);
#pragma unroll
  for (int q = 8; q < NV; ++q) v[q] = wave_sum_dpp(v[q]);
  const double gsc = rootn * h.scale;
  const int q8 = lane >> 3;
  // one store per quantity: lane 8 q for q < 8, lane 0 for the rest (part_ptr's layout from this base)
  if ((lane & 7) == 0 && q8 < NV) {
    double f = 1.0;
    if (q8 == 3) f = gsc;
#pragma unroll
    for (int j = 0; j < (D < 4 ? D : 4); ++j)
      if (q8 == 4 + j) f = gsc * h.ls[j];
    double* dst = pbase + ((int64_t)g * a.nq + q8) * a.nb + blk;
    const double val = q8 < 3 ? s8 : s8 * f;
    if (sc1) st_part_sc1(dst, val);
    else *dst = val;
  }
  if (lane == 0) {
#pragma unroll
    for (int q = 8; q < NV; ++q) {
      double* dst = pbase + ((int64_t)g * a.nq + q) * a.nb + blk;
      const double val = v[q] * (gsc * h.ls[q - 4]);
      if (sc1) st_part_sc1(dst, val);
      else *dst = val;
    }
  }
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
  // the wave index through readfirstlane: wave-uniform to the compiler (scalar branches on the problem flags)
  const int task = (int)blockIdx.x * (kWG / 64) + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
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
    const int64_t main = a.spec_main;
    const double rootn = sqrt((double)((int64_t)1 << a.log2n)), wl = a.logdet_weight;
    const double* phib = a.basis + (int64_t)g0 * a.basis_stride;   // PPW = 2: shared spectra (stride 0)
    SpecAcc<D> acc[PPW];
    const int64_t kbase = (int64_t)kb * 64 * a.spec_kpl;
    // software-pipelined: the next frequency's spectra and Y are in flight while this one is evaluated
    double phn[NS], Yn[PPW];
    auto fetch = [&](int64_t k) {
#pragma unroll
      for (int s = 0; s < NS; ++s) phn[s] = phib[spec_at<NS>(k, s)];
#pragma unroll
      for (int p = 0; p < PPW; ++p) Yn[p] = a.ysq[ysq_at(a, on[p] ? g0 + p : g0, k)];
    };
    if (kbase + lane < main) fetch(kbase + lane);
    for (int i = 0; i < a.spec_kpl; ++i) {
      const int64_t k = kbase + lane + 64 * i;
      if (k >= main) break;
      double phi[NS], Y[PPW];
#pragma unroll
      for (int s = 0; s < NS; ++s) phi[s] = phn[s];
#pragma unroll
      for (int p = 0; p < PPW; ++p) Y[p] = Yn[p];
      if (i + 1 < a.spec_kpl && k + 64 < main) fetch(k + 64);
#pragma unroll
      for (int p = 0; p < PPW; ++p)
        if (on[p]) spec_terms<D>(phi, h[p], rootn, wl, Y[p], acc[p]);
    }
#pragma unroll
    for (int p = 0; p < PPW; ++p)
      if (on[p]) spec_block_partials<D, NET>(a, h[p], g0 + p, kb, rootn, wl, acc[p], false, a.partials);
  }
  stamp_end(a);
}

// ---------------------------------------------------------------- reduction + Rprop of the spectral path
// The nb per-block partials of each (problem, quantity) are summed in two levels, in ONE order used by
// both the stage launches (k_spec_reduce_step) and the fused step at the end of k_spec_tile, so the two
// are bit-identical: level 1 sums the blocks of each group of kSpecGroup consecutive blocks (ascending),
// level 2 sums the ng = ceil(nb / kSpecGroup) group sums (ascending).  One thread per (problem,
// quantity): a group's block loads are issued together (one round trip, not a dependent chain).
#ifndef FGP_SPEC_GROUP
#define FGP_SPEC_GROUP 32
#endif
constexpr int kSpecGroup = FGP_SPEC_GROUP;

__device__ __forceinline__ int spec_groups(const Nll& a) { return (a.nb + kSpecGroup - 1) / kSpecGroup; }

// The fused run's workspace after the level-1 partials [G][nq][nb]: level-2 inputs (the group sums) of two
// iterations [2][G][nq][ng] (parity of the iteration: a launch writes its own while it reads the previous
// one's), two Rprop state copies [2][3][np], then the group counters (ng)
__host__ __device__ __forceinline__ int64_t spec_part2_off(const Nll& a, int par) {
  return (int64_t)a.G * a.nq * a.nb + (int64_t)par * a.G * a.nq * ((a.nb + kSpecGroup - 1) / kSpecGroup);
}
__device__ __forceinline__ double* part2_ptr(const Nll& a, int par, int g, int q, int grp) {
  return a.partials + spec_part2_off(a, par) + ((int64_t)g * a.nq + q) * spec_groups(a) + grp;
}
__host__ __device__ __forceinline__ RpState spec_state(const Nll& a, int par) {
  const int np = spec_nparams(a);
  double* b = a.partials + spec_part2_off(a, 2) + (int64_t)par * 3 * np;
  return RpState{b, b + np, b + 2 * np};
}

template <bool SC1>
__device__ __forceinline__ double ld_part(const double* p) {
  return SC1 ? __hip_atomic_load(gptr(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : *p;
}

// level 1: sum of problem g's quantity q over the blocks of group grp
template <bool SC1>
__device__ __forceinline__ double spec_group_sum(const Nll& a, int g, int q, int grp) {
  const int b0 = grp * kSpecGroup, nbg = min(kSpecGroup, a.nb - b0);
  const double* pp = part_ptr(a, g, q, b0);
  double t[kSpecGroup];
#pragma unroll
  for (int b = 0; b < kSpecGroup; ++b) t[b] = ld_part<SC1>(pp + (b < nbg ? b : 0));
  double s = 0.0;
#pragma unroll
  for (int b = 0; b < kSpecGroup; ++b) s += b < nbg ? t[b] : 0.0;
  return s;
}

// level 2 of the fused run: tot[g nq + q] = the ascending sum over the groups of the level-1 sums of parity
// par (k_spec_reduce_step's order); every group's sum in flight at once (a serial chain of loads costs ~1 us
// each).  Threads t < G nq; plain loads when the sums were stored by an earlier launch, sc1 loads (SC1) when
// by this one (the persistent k_spec_tile: hand-off row 1).
template <int D, bool SC1 = false>
__device__ __forceinline__ void spec_level2(const Nll& a, int par, double* tot) {
  constexpr int MAXG = kSpecBlocks / kSpecGroup;
  const int t = tid_fresh(), ng = spec_groups(a);
  if (t < a.G * a.nq) {
    const int g = t / a.nq, q = t % a.nq;
    double v[MAXG];
#pragma unroll
    for (int gr = 0; gr < MAXG; ++gr) v[gr] = ld_part<SC1>(part2_ptr(a, par, g, q, gr < ng ? gr : 0));
    double s = 0.0;
#pragma unroll
    for (int gr = 0; gr < MAXG; ++gr)
      if (gr < ng) s += v[gr];
    tot[t] = s;
  }
}

// Loss history + Rprop of the problems g0 .. g0 + cnt - 1 (cnt <= kWG / 16) from their reduced totals
// tot[(g - g0) * nq + q] (LDS): thread 16 i + k owns parameter slot k (0 scale, 1 .. dl lengthscales,
// dl + 1 noise) of problem g0 + i -- the reduce_step_wg semantics (fgp_nll.h: torch.optim.Rprop
// single-tensor, loss = 1/2 (norm + w logdet + const), histories).  The state is read from `in`; with
// `write` the histories, the gradient and the new state (to `out`, which may be `in`) are stored; the new
// raw parameters also go to newraw[p] when given (the deferred step of k_spec_tile, in every workgroup).
// parameter slot k (0 scale, 1 .. dl lengthscales, dl + 1 noise) of problem g: its index in the raw vector
__device__ __forceinline__ int spec_slot_param(const Nll& a, int g, int k, int dl) {
  if (k == 0) return a.scale_off + (a.scale_pp ? g : 0);
  if (k <= dl) return a.ls_off + (a.ls_pp ? g : 0) * dl + (k - 1);
  return a.noise_off + (a.noise_pp ? g : 0);
}

template <int D>
__device__ __forceinline__ void spec_finish(const Nll& a, const Fit& f, const double* tot, int g0, int cnt, int iter,
                                            int do_update, const RpState& in, const RpState& out, bool write,
                                            double* newraw, int state_write = -1, const double* pf = nullptr,
                                            double* best = nullptr) {
  const bool wstate = state_write < 0 ? write : state_write != 0;   // the new state to `out` (default: with write)
  const int tf = tid_fresh(), i = tf >> 4, k = tf & 15;
  if (i >= cnt) return;
  const int g = g0 + i;
  const double* v = tot + i * a.nq;
  const int dl = a.ls_pd ? a.d : 1;
  if (k == 0 && write) {
    const double term2 = a.logdet_weight * v[1];
    double* lh = f.loss_hist + ((int64_t)iter * (f.hist_stride ? f.hist_stride : a.G) + f.hist_offset + g) * 3;
    lh[0] = 0.5 * (v[0] + term2 + f.mll_const);
    lh[1] = v[0];
    lh[2] = term2;
  }
  if (k >= 2 + dl) return;
  const int p = spec_slot_param(a, g, k, dl);
  int rg;
  double gp;
  if (k == 0) {
    rg = f.scale_rg;
    gp = v[3];
  } else if (k <= dl) {
    rg = f.ls_rg;
    gp = 0.0;
    if (a.ls_pd) {
#pragma unroll
      for (int j = 0; j < D; ++j) gp = (j == k - 1) ? v[4 + j] : gp;
    } else {
#pragma unroll
      for (int j = 0; j < D; ++j) gp += v[4 + j];
    }
  } else {
    rg = f.noise_rg;
    gp = 0.0;
  }
  // (pf: this thread's state, prefetched by the caller beside its other loads)
  const double raw_p = pf ? pf[0] : in.raw[p], prev_p = pf ? pf[1] : in.prev[p], step_p = pf ? pf[2] : in.step[p];
  if (k == dl + 1) gp = exp(raw_p) * v[2];
  if (best) best[p] = raw_p;                     // (k_spec_persist: this iteration's parameters are the best iterate)
  if (write) {
    f.raw_hist[(int64_t)iter * f.n_params + p] = raw_p;
    f.grad_out[p] = gp;
  }
  double nraw = raw_p, nstep = step_p, nprev = prev_p;
  if (do_update && rg) {
    const double prod = gp * prev_p;
    const double sgn = prod > 0.0 ? f.eta_plus : (prod < 0.0 ? f.eta_minus : 1.0);
    nstep = fmin(fmax(step_p * sgn, f.step_min), f.step_max);
    nprev = (sgn == f.eta_minus) ? 0.0 : gp;
    const double gs = nprev > 0.0 ? 1.0 : (nprev < 0.0 ? -1.0 : 0.0);
    nraw = raw_p + (-1.0) * (gs * nstep);
  }
  if (wstate) {
    out.raw[p] = nraw;
    out.step[p] = nstep;
    out.prev[p] = nprev;
  }
  if (newraw) newraw[p] = nraw;
}

// The per-problem step of the spectral path as its own launch (fgp_fit_step, stage-by-stage fits):
// workgroup b takes problems 16 b .. 16 b + 15, both levels per (problem, quantity) thread.
template <int D>
__global__ __launch_bounds__(kWG) void k_spec_reduce_step(Nll a, Fit f, int iter, int do_update) {
  constexpr int NQ = 4 + D, MAXG = kSpecBlocks / kSpecGroup;
  __shared__ double gs[16 * NQ * MAXG];   // level-1 sums [pair][group]
  __shared__ double tot[16 * NQ];
  const int g0 = (int)blockIdx.x * 16, cnt = min(16, a.G - g0), ng = spec_groups(a);
  // level 1: every (problem, quantity, group) triple by its own thread (the groups' loads in parallel)
  for (int t = threadIdx.x; t < cnt * NQ * ng; t += kWG) {
    const int pair = t / ng, grp = t % ng;
    gs[pair * MAXG + grp] = spec_group_sum<false>(a, g0 + pair / NQ, pair % NQ, grp);
  }
  __syncthreads();
  // level 2: ascending over the groups, as the fused step
  if ((int)threadIdx.x < cnt * NQ) {
    double s = 0.0;
    for (int grp = 0; grp < ng; ++grp) s += gs[threadIdx.x * MAXG + grp];
    tot[threadIdx.x] = s;
  }
  __syncthreads();
  const RpState st{f.raw, f.prev, f.step};
  spec_finish<D>(a, f, tot, g0, cnt, iter, do_update, st, st, true, nullptr);
}

// The step of ONE loss over many problems (per-output hyper-parameters of one GP, e.g. C5 per-output: 512
// eigen-problems, a summed MLL; not per_problem) -- k_fit_reduce + the one-workgroup k_fit_step of the
// transform path, spread over ceil(G / 16) workgroups.  Workgroup b: both levels of the partials of problems
// 16 b .. 16 b + 15 (k_spec_reduce_step's order) -> their totals red(g, q) (k_fit_reduce's output) and the
// Rprop step of the parameters only they own (per-problem scale / lengthscales / noise: thread 16 i + slot,
// k_fit_step's gradient of that parameter from red(g, .)); the workgroup whose arrival on `counter` comes
// last (sc1 totals, an agent-scope add: MI355X_MICROARCH.md hand-off row 1) then runs k_fit_step's loss and
// shared-parameter part -- the same per-thread (g = t, t + kWG, ...), wave and workgroup order, so the loss
// and shared gradients equal k_fit_step's given the totals -- and resets the counter for the next launch.
template <int D>
__global__ __launch_bounds__(kWG) void k_spec_step_many(Nll a, Fit f, int iter, int do_update, unsigned* counter) {
  constexpr int NQ = 4 + D, MAXG = kSpecBlocks / kSpecGroup, NV = 4 + FGP_MAX_D, NW = kWG / 64;
  __shared__ double gs[16 * NQ * MAXG];
  __shared__ double tot[16 * NQ];
  __shared__ double red[NV * NW];
  __shared__ int last;
  const int tid = threadIdx.x;
  const int g0 = (int)blockIdx.x * 16, cnt = min(16, a.G - g0), ng = spec_groups(a);
  for (int t = tid; t < cnt * NQ * ng; t += kWG) {
    const int pair = t / ng, grp = t % ng;
    gs[pair * MAXG + grp] = spec_group_sum<false>(a, g0 + pair / NQ, pair % NQ, grp);
  }
  __syncthreads();
  if (tid < cnt * NQ) {
    double s = 0.0;
    for (int grp = 0; grp < ng; ++grp) s += gs[tid * MAXG + grp];
    tot[tid] = s;
    __hip_atomic_store(a.partials + (int64_t)a.G * a.nq * a.nb + (int64_t)(g0 + tid / NQ) * a.nq + tid % NQ, s,
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  // the parameters problem g0 + i owns: slot 0 scale, 1 .. dl lengthscales, dl + 1 noise
  const int dl = a.ls_pd ? a.d : 1, i = tid >> 4, k = tid & 15;
  if (i < cnt && k < 2 + dl) {
    const int g = g0 + i;
    const double* v = tot + i * NQ;
    int p = -1, rg = 0;
    double gp = 0.0;
    if (k == 0 && a.scale_pp) {
      p = a.scale_off + g;
      rg = f.scale_rg;
      gp = 0.0 + v[3];
    } else if (k >= 1 && k <= dl && a.ls_pp) {
      p = a.ls_off + g * dl + (k - 1);
      rg = f.ls_rg;
      gp = 0.0;
      if (a.ls_pd) {
        gp += v[4 + (k - 1)];
      } else {
        for (int j = 0; j < a.d; ++j) gp += v[4 + j];
      }
    } else if (k == dl + 1 && a.noise_pp) {
      p = a.noise_off + g;
      rg = f.noise_rg;
      gp = 0.0 + exp(a.raw[p]) * v[2];
    }
    if (p >= 0) {
      f.raw_hist[(int64_t)iter * f.n_params + p] = f.raw[p];
      f.grad_out[p] = gp;
      if (do_update && rg) rprop_update(f, p, gp);
    }
  }
  // arrival: every wave's sc1 totals retired, then one add
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0)
    last = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  __syncthreads();
  if (!last) return;
  // k_fit_step's loss and shared-parameter part over all G problems
  auto rd = [&](int g, int q) {
    return __hip_atomic_load(a.partials + (int64_t)a.G * a.nq * a.nb + (int64_t)g * a.nq + q, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
  };
  double v[NV];
#pragma unroll
  for (int q = 0; q < NV; ++q) v[q] = 0.0;
  const double en = a.noise_pp ? 0.0 : exp(a.raw[a.noise_off]);
  for (int g = tid; g < a.G; g += kWG) {
    v[0] += rd(g, 0);
    v[1] += rd(g, 1);
    if (!a.noise_pp) v[2] += en * rd(g, 2);
    if (!a.scale_pp) v[3] += rd(g, 3);
    if (!a.ls_pp)
      for (int j = 0; j < a.d; ++j) v[4 + (a.ls_pd ? j : 0)] += rd(g, 4 + j);
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
    double t[NV];
#pragma unroll
    for (int q = 0; q < NV; ++q) {
      t[q] = 0.0;
#pragma unroll
      for (int w = 0; w < NW; ++w) t[q] += red[q * NW + w];
    }
    const double term2 = a.logdet_weight * t[1];
    f.loss_hist[(int64_t)iter * 3 + 0] = 0.5 * (t[0] + term2 + f.mll_const);
    f.loss_hist[(int64_t)iter * 3 + 1] = t[0];
    f.loss_hist[(int64_t)iter * 3 + 2] = term2;
    auto shared_param = [&](int p, int rg, double gp) {
      f.raw_hist[(int64_t)iter * f.n_params + p] = f.raw[p];
      f.grad_out[p] = gp;
      if (do_update && rg) rprop_update(f, p, gp);
    };
    if (!a.noise_pp) shared_param(a.noise_off, f.noise_rg, 0.0 + t[2]);
    if (!a.scale_pp) shared_param(a.scale_off, f.scale_rg, 0.0 + t[3]);
    if (!a.ls_pp)
      for (int j = 0; j < dl; ++j) shared_param(a.ls_off + j, f.ls_rg, 0.0 + t[4 + j]);
    __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// The deferred step of a fused spectral run's LAST iteration (its own launch, one workgroup): the level-2 sum
// of that iteration's group sums (parity fz.par ^ 1 as k_spec_tile's prologue reads them) and the step from
// fz.sin to fz.sout (the fit's own state vectors)
template <int D>
__global__ __launch_bounds__(kWG) void k_spec_finish_step(Nll a, FitFuse fz) {
  __shared__ double tot[16 * (4 + D)];
  spec_level2<D>(a, fz.par ^ 1, tot);
  __syncthreads();
  spec_finish<D>(a, fz.f, tot, 0, a.G, fz.iter - 1, fz.do_update, fz.sin, fz.sout, true, nullptr);
}

// ---------------------------------------------------------------- the whole fit of ONE small problem in one launch
// (fgp_fit_persist, ABI 14).  A single GP whose spectra and Y fit the LDS of kPersistMaxW workgroups (C2 / C3 at
// n = 2^16, the probnum25 paper's n = 2^10): workgroup b loads the blocks [b bpw, (b + 1) bpw) of k_spec_iter's
// geometry into LDS once, then every Rprop iteration is
//   block partials (spec_terms / spec_block_partials: k_spec_iter's arithmetic) -> agent-scope stores into one of
//   three rotating buffers whose empty slots hold a sentinel -> every workgroup polls the slots it sums until
//   none is empty (the grid barrier and the partial read in one round trip; bounded polls) and sums them in the
//   two-level order of k_spec_reduce_step -> the same Rprop step on each workgroup's own LDS copy of the state
//   -> AbstractGP.fit's early-stopping rule (abstract_gp.py:276-284) evaluated on the same loss values
// so the trajectory is the multi-launch fit's bit for bit, without a launch per iteration.  Workgroup 0 writes
// the histories and the final state; out[0] = the last iteration, out[1] = 1 if a barrier poll gave up.
constexpr int kPersistMaxW = 256;
constexpr long long kSpecPollMax = 1ll << 22;     // bounded waits of the persistent k_spec_tile
constexpr int kPersistLdsMax = 96 * 1024;
constexpr long long kPersistPollMax = 1ll << 22;
// the wall-clock bound of one barrier wait of the single-launch fit (device clock ticks: 5e6 = 50 ms at the 100 MHz
// constant clock of fgp_wall_clock_khz) -- a give-up then costs milliseconds, not 2^22 polls of seconds
constexpr unsigned long long kPersistWaitTicks = 5000000ull;
// give-ups of k_spec_persist since load / the last reset (fgp_persist_giveups): never cleared by a launch, so a failure
// inside a hipGraph replay is still visible after it
__device__ unsigned long long g_persist_giveups = 0;
// the poll bound of those waits (fgp_set_persist_poll_max): read by the kernel from device memory, so the test hook
// also reaches launches replayed from a hipGraph captured before it was set
__device__ long long g_persist_poll_max_dev = kPersistPollMax;
// an empty partial slot of the single-launch fit (all ones: a NaN payload no arithmetic produces; the buffers are
// filled with it before the launch)
constexpr long long kPartEmpty = -1ll;

// workgroup barrier that lets global loads / stores stay in flight across it (__syncthreads() drains them with
// vmcnt(0)): LDS-DMA chunks, workgroup 0's history stores; the waves' LDS accesses retired (lgkmcnt), the raw
// barrier, a compiler memory fence
__device__ __forceinline__ void barrier_keep_vm() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int D, bool NET>
__global__ __launch_bounds__(kWG) void k_spec_persist(Nll a, Fit f, int iters, double logtol, int wait_max, int bpw,
                                                      unsigned* counter, int* out) {
  constexpr int NS = 1 << D, NQ = 4 + D, MAXG = kSpecBlocks / kSpecGroup;
  extern __shared__ double lds[];                  // [bpw][kpl][NS + 1][64] spectra + Y of this workgroup's blocks
  __shared__ double st_raw[kSpecScratch], st_prev[kSpecScratch], st_step[kSpecScratch];
  __shared__ double st_best[kSpecScratch];         // the best iterate's parameters (AbstractGP.fit's best_params)
  __shared__ double gsum[NQ * MAXG];
  __shared__ double tot[NQ];
  __shared__ double es[3];                         // early stopping: best, save, waited
  __shared__ int brk_s, fail_s, isb_s, bi_s;
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int W = gridDim.x, kpl = a.spec_kpl, np = spec_nparams(a), ng = spec_groups(a);
  const int64_t main = a.spec_main, B = 64 * (int64_t)kpl;
  const int blk0 = (int)blockIdx.x * bpw;
  const long long poll_max = g_persist_poll_max_dev;
  // the blocks' spectra and Y into LDS (chunked layouts: chunk q of the spectra at q NS 64, Y at q 64 for G = 1)
  const int per_blk = kpl * (NS + 1) * 64;
  for (int e = tid; e < bpw * per_blk; e += kWG) {
    const int t = e / per_blk, r = e - t * per_blk, c = r / ((NS + 1) * 64), rr = r - c * (NS + 1) * 64;
    const int row = rr >> 6, col = rr & 63;
    const int64_t q = ((int64_t)(blk0 + t) * kpl + c);           // chunk
    double v = 0.0;
    if (blk0 + t < a.nb && q * 64 + col < a.spec_KS)
      v = row < NS ? a.basis[(q * NS + row) * 64 + col] : a.ysq[q * 64 + col];
    lds[e] = v;
  }
  for (int p = tid; p < np; p += kWG) {
    st_raw[p] = f.raw[p];
    st_best[p] = st_raw[p];                        // (no finite loss at all: iteration 0's, the host rule's best_i = 0)
    st_prev[p] = f.prev[p];
    st_step[p] = f.step[p];
  }
  if (tid == 0) {
    es[0] = INFINITY;
    es[1] = INFINITY;
    es[2] = 0.0;
    brk_s = 0;
    fail_s = 0;
    bi_s = 0;
  }
  __syncthreads();
  const double rootn = sqrt((double)((int64_t)1 << a.log2n)), wl = a.logdet_weight;
  const RpState st{st_raw, st_prev, st_step};
  const int64_t psize = (int64_t)a.nq * a.nb;      // one parity's partials (G = 1)
  // the single-frequency corrections, loaded once for the whole fit by the wave holding block 0 / the last
  // block (the blocks t = w, w + 4, ... of this workgroup)
  SpecCorr corr{0.0, 0.0, 0.0, 0, false};
  for (int t = w; t < bpw; t += kWG / 64) {
    const int blk = blk0 + t;
    if (blk < a.nb && (blk == 0 || blk == a.nb - 1)) corr = spec_corr_load<NS>(a, blk, 0, 1);
  }
  // (a.stamps: workgroup 0's device clock per iteration -- start, partials stored, barrier passed, reduced,
  // stepped -- at stamps[5 it + phase]; the round-5 tools/exp_persist_stamps.py, in git history: profiles/r05j_persist_stamps_sentinel.jsonl)
  auto stamp = [&](int it, int ph) {
    if (a.stamps && blockIdx.x == 0 && tid == 0) a.stamps[5 * it + ph] = wall_clock64();
  };
  // one workgroup over at most one group of blocks (the paper's n = 2^10 fits): the block partials go through
  // LDS and no barrier is needed -- the same values summed in the same order as the global hand-off
  __shared__ double lpart[NQ * kSpecGroup];
  const bool single = W == 1 && a.nb <= kSpecGroup;
  for (int it = 0; it <= iters; ++it) {
    // three rotating partial buffers, empty slots holding kPartEmpty: iteration it writes buffer it % 3, and a slot
    // is emptied again by its writer once every workgroup has read it (see the reset below)
    double* pbase = single ? static_cast<double*>(lpart) : a.partials + (it % 3) * psize;
    stamp(it, 0);
    Hyp h;
    load_hyp_wave(a, 0, h, st_raw);
    // the previous iteration's slot resets (and workgroup 0's history stores) retired before this iteration's
    // partials can be seen
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (int t = w; t < bpw; t += kWG / 64) {
      const int blk = blk0 + t;
      if (blk >= a.nb) break;
      SpecAcc<D> acc;
      const double* lb = lds + (int64_t)t * per_blk;
      // two chunks per pass: both chunks' terms first, then their accumulation in chunk order (spec_term_*)
      for (int i = 0; i < kpl; i += 2) {
        const int64_t k = (int64_t)blk * B + lane + 64 * i;
        if (k >= main) break;
        const bool two = i + 1 < kpl && k + 64 < main;
        const double* cb0 = lb + i * (NS + 1) * 64 + lane;
        const double* cb1 = two ? cb0 + (NS + 1) * 64 : cb0;
        double phi0[NS], phi1[NS];
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          phi0[s] = cb0[64 * s];
          phi1[s] = cb1[64 * s];
        }
        SpecTerm<D> t0, t1;
        spec_term_values<D>(phi0, h, rootn, wl, cb0[64 * NS], t0);
        spec_term_values<D>(phi1, h, rootn, wl, cb1[64 * NS], t1);
        spec_term_add<D>(t0, acc);
        if (!two) break;
        spec_term_add<D>(t1, acc);
      }
      spec_block_partials<D, NET>(a, h, 0, blk, rootn, wl, acc, !single, pbase, corr);
    }
    stamp(it, 1);
    // level 1 (groups of kSpecGroup blocks, ascending) and level 2 (groups ascending): k_spec_reduce_step's order.
    // One workgroup, one group: the partials are in LDS and level 2 adds the single group sum to 0.0 (exact), so
    // thread q sums its row of lpart directly (typed LDS loads, one barrier) -- the same additions in the same order.
    if (single) {
      __syncthreads();
      stamp(it, 2);
      if (tid < NQ) {
        double sq = 0.0;
        for (int b = 0; b < a.nb; ++b) sq += lpart[tid * a.nb + b];
        tot[tid] = sq;
      }
    } else {
      // the grid barrier IS the read: each (quantity, group) thread polls its group's 32 slots (one round trip
      // per poll, the loads issued together) until none is empty -- no counter, no separate re-read
      for (int e = tid; e < NQ * ng; e += kWG) {
        const int q = e / ng, grp = e - q * ng;
        const int b0 = grp * kSpecGroup, nbg = min(kSpecGroup, a.nb - b0);
        const double* pp = pbase + (int64_t)q * a.nb + b0;
        double tv[kSpecGroup];
        long long polls = 0;
        const unsigned long long t_wait = wall_clock64();
        for (;;) {
#pragma unroll
          for (int b = 0; b < kSpecGroup; ++b) tv[b] = ld_part<true>(pp + (b < nbg ? b : 0));
          bool full = true;
#pragma unroll
          for (int b = 0; b < kSpecGroup; ++b) full = full && __double_as_longlong(tv[b]) != kPartEmpty;
          if (full) break;
          // give up on the poll bound (test hook) or the wall-clock bound
          // (a fail word polled beside the slots -- a late workgroup stopping at its first poll -- made hipGraph replays
          // give up: it read nonzero there, profiles/r06d_persist_failword_ab.jsonl; not kept)
          if (++polls > poll_max || wall_clock64() - t_wait > kPersistWaitTicks) {
            fail_s = 1;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
        double sgrp = 0.0;
#pragma unroll
        for (int b = 0; b < kSpecGroup; ++b) sgrp += b < nbg ? tv[b] : 0.0;
        gsum[q * MAXG + grp] = sgrp;
      }
      __syncthreads();
      stamp(it, 2);
      if (fail_s) {
        // a wait gave up (every workgroup's next wait then fails too, so no final state is written): the fit's
        // parameters and every parameter-history row become NaN -- whichever row the caller restores as the best
        // iterate, the failure shows downstream even when `out` is never read (a hipGraph replay).  Rprop's prev /
        // step are untouched: with the caller's copy of the entry raw parameters the fit can be re-run.
        if (tid == 0) {
          out[1] = 1;
          atomicAdd(&g_persist_giveups, 1ull);        // the library's sticky count (fgp_persist_giveups)
        }
        for (int p = tid; p < np; p += kWG) f.raw[p] = NAN;
        if (f.raw_hist)
          for (int64_t e = tid; e < (int64_t)(iters + 1) * f.n_params; e += kWG) f.raw_hist[e] = NAN;
        return;
      }
      // every workgroup has read iteration it - 1's buffer ((it + 2) % 3: each wrote its iteration-it partials after
      // its own reads of it - 1 returned), so this workgroup empties its slots there for iteration it + 2
      double* pnext = a.partials + ((it + 2) % 3) * psize;
      for (int e = tid; e < NQ * bpw; e += kWG) {
        const int q = e / bpw, blk = blk0 + (e - q * bpw);
        if (blk < a.nb) st_part_sc1(pnext + (int64_t)q * a.nb + blk, __longlong_as_double(kPartEmpty));
      }
      if (tid < NQ) {
        double sq = 0.0;
        for (int grp = 0; grp < ng; ++grp) sq += gsum[tid * MAXG + grp];
        tot[tid] = sq;
      }
    }
    __syncthreads();
    stamp(it, 3);
    if (tid == 0) {
      // AbstractGP.fit's bookkeeping on the loss of this iteration (the value spec_finish records)
      const double lv = 0.5 * (tot[0] + a.logdet_weight * tot[1] + f.mll_const);
      double best = es[0], save = es[1], waited = es[2];
      isb_s = lv < best ? 1 : 0;                   // (NaN never best: the host rule `lv < best`)
      if (lv < best) {
        best = lv;
        bi_s = it;
      }
      if ((save - lv) > logtol) {
        waited = 0.0;
        save = best;
      } else {
        waited += 1.0;
      }
      es[0] = best;
      es[1] = save;
      es[2] = waited;
      brk_s = (it == iters || waited == (double)wait_max) ? 1 : 0;
    }
    __syncthreads();
    const int brk = brk_s;
    spec_finish<D>(a, f, tot, 0, 1, it, brk ? 0 : 1, st, st, blockIdx.x == 0, nullptr, 1, nullptr,
                   isb_s ? st_best : nullptr);
    // (the new state is in LDS; workgroup 0's history stores stay in flight -- drained by the next iteration's
    // vmcnt(0) before its grid barrier, under its compute: a __syncthreads here cost ~1 us per iteration)
    barrier_keep_vm();
    stamp(it, 4);
    if (brk) {
      if (blockIdx.x == 0) {
        // raw <- the BEST iterate (what AbstractGP.fit restores; fgp_fit_persist, ABI 18), prev / step <- the final
        // Rprop state; out[0] the last iteration, out[2] the best one
        for (int p = tid; p < np; p += kWG) {
          f.raw[p] = st_best[p];
          f.prev[p] = st_prev[p];
          f.step[p] = st_step[p];
        }
        if (tid == 0) {
          out[0] = it;
          out[2] = bi_s;
        }
      }
      return;
    }
  }
}

// ---------------------------------------------------------------- GCV / CV fits (ABI 16)
// The alternative losses of AbstractGP.fit (abstract_gp.py:242-273) for one task: with ev_k = sqrt(n) scale P_k +
// noise, lambda'_k = sqrt(n) scale P_k (= ev_k - noise) and Y_k = sum_b |ytilde_bk|^2,
//   GCV (util.py:371-380):  N1 = sum_k Y_k / ev_k^2 (= sum |z~|^2, z~ = ytilde / ev),  T = sum_k 1 / ev_k (the trace of
//                           the inverse),  loss = N1 / (T / n)^2;
//   CV  (util.py:381-385):  inv_diag I = (1/n) sum_k 1 / lambda'_k, coeffs = ift(ytilde / ev).real with
//                           sum_i coeffs_i^2 = N1 (Parseval; ytilde / ev is Hermitian), loss = w N1 / I^2.
// Both gradients are  dL/dtheta = c1 S1_theta + c2 S2_theta  with per-frequency sums
//   S1_theta = sum_k (Y_k / ev_k^3) dev_k/dtheta,   S2_theta = sum_k w2_k dx_k/dtheta,
//   GCV: w2 = 1 / ev^2, x = ev;  CV: w2 = 1 / lambda'^2, x = lambda' (no noise term),
// and the global factors (GCV: c1 = -2 / D, c2 = 2 N1 T / (n^2 D^2), D = (T / n)^2; CV: c1 = -2 w / I^2,
// c2 = 2 w N1 / (n I^3)) applied once the sums are reduced (k_spec_loss_step), the same way the MLL's weights are.
// dev/draw_scale = sqrt(n) scale P, dev/draw_l_j = sqrt(n) scale l_j dP/dl_j, dev/draw_noise = noise.
template <int D>
struct LossAcc {
  double n1 = 0.0, t = 0.0, s1n = 0.0, s1s = 0.0, s2n = 0.0, s2s = 0.0;
  double s1l[D], s2l[D];
  __device__ __forceinline__ LossAcc() {
#pragma unroll
    for (int j = 0; j < D; ++j) s1l[j] = s2l[j] = 0.0;
  }
};

template <int D, bool CV>
__device__ __forceinline__ void loss_terms(const double* phi, const Hyp& h, double rootn, double Y, LossAcc<D>& acc) {
  double dp[D];
  const double P = mlin<D>(phi, h.ls, dp);
  const double lp = rootn * (h.scale * P);
  const double e = lp + h.noise;
  const double r = rcp_nr(e);
  const double yr2 = Y * (r * r);
  acc.n1 += yr2;
  const double w1 = yr2 * r;
  double w2;
  if constexpr (CV) {
    const double rl = rcp_nr(lp);
    acc.t += rl;
    w2 = rl * rl;
  } else {
    acc.t += r;
    w2 = r * r;
    acc.s2n += w2;
  }
  acc.s1n += w1;
  acc.s1s = __builtin_fma(w1, P, acc.s1s);
  acc.s2s = __builtin_fma(w2, P, acc.s2s);
#pragma unroll
  for (int j = 0; j < D; ++j) {
    acc.s1l[j] = __builtin_fma(w1, dp[j], acc.s1l[j]);
    acc.s2l[j] = __builtin_fma(w2, dp[j], acc.s2l[j]);
  }
}

template <int D>
__device__ __forceinline__ void loss_values(const LossAcc<D>& acc, double* v) {
  v[0] = acc.n1;
  v[1] = acc.t;
  v[2] = acc.s1n;
  v[3] = acc.s1s;
#pragma unroll
  for (int j = 0; j < D; ++j) v[4 + j] = acc.s1l[j];
  v[4 + D] = acc.s2n;
  v[5 + D] = acc.s2s;
#pragma unroll
  for (int j = 0; j < D; ++j) v[6 + D + j] = acc.s2l[j];
}

// Per-block partials of the alternative losses: wave task = (k block, problem), one problem per wave; lane l sums
// k = block base + l + 64 i (ascending i); the lattice's fold (weight 2 for 0 < k < n/2, 1 at k = 0 and n/2) as in
// spec_block_partials; the chain factors sqrt(n) scale (scale sums) and sqrt(n) scale l_j (lengthscale sums); fixed
// wave-sum order.  Partials [G][6 + 2 d][nb] (part_ptr).
template <int D, bool NET, bool CV>
__global__ __launch_bounds__(kWG) void k_spec_loss_iter(Nll a) {
  constexpr int NS = 1 << D, NV = 6 + 2 * D;
  const int lane = threadIdx.x & 63;
  const int task = (int)blockIdx.x * (kWG / 64) + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int kb = task / a.G, g = task - kb * a.G;
  if (kb >= a.nb) return;
  Hyp h;
  load_hyp_wave(a, g, h);
  const double rootn = sqrt((double)((int64_t)1 << a.log2n));
  const double* phib = a.basis + (int64_t)g * a.basis_stride;
  LossAcc<D> acc;
  const int64_t kbase = (int64_t)kb * 64 * a.spec_kpl;
  for (int i = 0; i < a.spec_kpl; ++i) {
    const int64_t k = kbase + lane + 64 * i;
    if (k >= a.spec_main) break;
    double phi[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) phi[s] = phib[spec_at<NS>(k, s)];
    loss_terms<D, CV>(phi, h, rootn, a.ysq[ysq_at(a, g, k)], acc);
  }
  double v[NV];
  loss_values<D>(acc, v);
  if (!NET) {
#pragma unroll
    for (int q = 0; q < NV; ++q) v[q] *= 2.0;
    if (lane == 0 && (kb == 0 || kb == a.nb - 1)) {
#pragma unroll
      for (int side = 0; side < 2; ++side) {
        if (side == 0 ? kb != 0 : kb != a.nb - 1) continue;
        const int64_t k = side == 0 ? 0 : a.spec_main;
        double phi[NS];
#pragma unroll
        for (int s = 0; s < NS; ++s) phi[s] = phib[spec_at<NS>(k, s)];
        LossAcc<D> t;
        loss_terms<D, CV>(phi, h, rootn, a.ysq[ysq_at(a, g, k)], t);
        double tv[NV];
        loss_values<D>(t, tv);
        const double sg = side == 0 ? -1.0 : 1.0;   // k = 0: weight 2 -> 1; k = n/2: weight 1
#pragma unroll
        for (int q = 0; q < NV; ++q) v[q] = __builtin_fma(sg, tv[q], v[q]);
      }
    }
  }
  const double gsc = rootn * h.scale;
#pragma unroll
  for (int q = 0; q < NV; ++q) {
    double f = 1.0;
    if (q == 3 || q == 5 + D) f = gsc;
#pragma unroll
    for (int j = 0; j < D; ++j)
      if (q == 4 + j || q == 6 + D + j) f = gsc * h.ls[j];
    const double sq = wave_sum_dpp(v[q]);
    if (lane == 0) part_ptr(a, g, q, kb)[0] = sq * f;
  }
}

// Reduction + loss + Rprop of the alternative losses: problems 16 b .. 16 b + 15 per workgroup (one workgroup when
// the problems share one loss), the two-level block order of k_spec_reduce_step, then per problem the loss (GCV:
// history [loss, numer, denom]; CV: [loss, nan, nan] -- abstract_gp.py:242-273's term1 / term2) and the gradient
// c1 S1 + c2 S2 of every parameter it touches (a parameter shared by several problems sums theirs), then
// torch.optim.Rprop (rprop_update).
template <int D>
__global__ __launch_bounds__(kWG) void k_spec_loss_step(Nll a, Fit f, int iter, int do_update) {
  constexpr int NQ = 6 + 2 * D, MAXG = kSpecBlocks / kSpecGroup;
  __shared__ double gs[16 * NQ * MAXG];
  __shared__ double tot[16 * NQ];
  __shared__ double lossg[16], c1s[16], c2s[16];
  const int g0 = (int)blockIdx.x * 16, cnt = min(16, a.G - g0), ng = spec_groups(a);
  for (int t = threadIdx.x; t < cnt * NQ * ng; t += kWG) {
    const int pair = t / ng, grp = t % ng;
    gs[pair * MAXG + grp] = spec_group_sum<false>(a, g0 + pair / NQ, pair % NQ, grp);
  }
  __syncthreads();
  // strided: cnt NQ reaches 16 (6 + 2 D) = 288 > kWG totals at D = 6
  for (int u = threadIdx.x; u < cnt * NQ; u += kWG) {
    double s = 0.0;
    for (int grp = 0; grp < ng; ++grp) s += gs[u * MAXG + grp];
    tot[u] = s;
  }
  __syncthreads();
  // (multitask GCV: the trace is normalised by the points of all T tasks, util.py:379 self.n.sum())
  // (multitask CV: I_t over the n points of task t)
  const bool cv = a.loss == FGP_LOSS_CV;
  const double n = (double)((int64_t)1 << a.log2n) * (a.mt > 0 && !cv ? a.mt : 1);
  if ((int)threadIdx.x < cnt) {
    const int i = threadIdx.x;
    const double N1 = tot[i * NQ + 0], T = tot[i * NQ + 1];
    double L, c1, c2, t1, t2;
    if (cv) {
      const double I = T / n, w = a.cv_weight;
      L = w * N1 / (I * I);
      c1 = -2.0 * w / (I * I);
      c2 = 2.0 * w * N1 / (n * I * I * I);
      t1 = t2 = NAN;
    } else {
      const double Dn = (T / n) * (T / n);
      L = N1 / Dn;
      c1 = -2.0 / Dn;
      c2 = 2.0 * N1 * T / (n * n * Dn * Dn);
      t1 = N1;
      t2 = Dn;
    }
    lossg[i] = L;
    c1s[i] = c1;
    c2s[i] = c2;
    if (f.per_problem) {
      double* lh = f.loss_hist + ((int64_t)iter * (f.hist_stride ? f.hist_stride : a.G) + f.hist_offset + g0 + i) * 3;
      lh[0] = L;
      lh[1] = t1;
      lh[2] = t2;
    }
  }
  __syncthreads();
  if (!f.per_problem && threadIdx.x == 0) {
    double L = 0.0;
    for (int i = 0; i < cnt; ++i) L += lossg[i];
    f.loss_hist[(int64_t)iter * 3 + 0] = L;
    f.loss_hist[(int64_t)iter * 3 + 1] = cnt == 1 && !cv ? tot[0] : NAN;
    f.loss_hist[(int64_t)iter * 3 + 2] = cnt == 1 && !cv ? (tot[1] / n) * (tot[1] / n) : NAN;
  }
  // every parameter slot of this workgroup's problems: thread t takes raw index t and sums the gradient of every
  // (problem, slot) mapped to it, problems ascending
  const int dl = a.ls_pd ? a.d : 1, np = spec_nparams(a);
  for (int p = threadIdx.x; p < np; p += kWG) {
    double gp = 0.0;
    int rg = -1;
    for (int i = 0; i < cnt; ++i) {
      const int g = g0 + i;
      const double* v = tot + i * NQ;
      for (int k = 0; k < 2 + dl; ++k) {
        if (spec_slot_param(a, g, k, dl) != p) continue;
        double s1, s2;
        if (k == 0) {
          s1 = v[3];
          s2 = v[5 + D];
          rg = f.scale_rg;
        } else if (k <= dl) {
          s1 = s2 = 0.0;
          for (int j = 0; j < D; ++j)
            if (a.ls_pd ? j == k - 1 : true) {
              s1 += v[4 + j];
              s2 += v[6 + D + j];
            }
          rg = f.ls_rg;
        } else {
          const double nz = exp(a.raw[p]);
          s1 = nz * v[2];
          s2 = nz * v[4 + D];
          rg = f.noise_rg;
        }
        gp += c1s[i] * s1 + c2s[i] * s2;
      }
    }
    if (rg < 0) continue;                  // not a parameter of these problems
    f.raw_hist[(int64_t)iter * f.n_params + p] = f.raw[p];
    f.grad_out[p] = gp;
    if (do_update && rg) rprop_update(f, p, gp);
  }
}

// Reduction + loss + Rprop of a multitask GCV / CV fit with a LEARNED task kernel (ABI 18; k_mt_spec_iter<.., LEARN>'s
// partials): one workgroup.  The totals of every (problem, quantity) -- problems: 1 (GCV) or the T tasks (CV) --
// in k_spec_loss_step's two-level order, the loss and the factors c1, c2 of each problem as there, the scale /
// lengthscale / noise gradients as there, and dL/dK_task of pair p = sum_i c1_i K1_ip + c2_i K2_ip, then the chain rule
// through K_task = F F^T + diag(v): dL/dF[t, r] = sum_p dK_p (F[l_p, r] [k_p == t] + F[k_p, r] [l_p == t]) (ascending p),
// dL/draw_v[t] = dK_(t, t) (v_t when exp); torch.optim.Rprop on every parameter (rprop_update).
template <int D>
__global__ __launch_bounds__(kWG) void k_mt_learn_step(Nll a, Fit f, int iter, int do_update) {
  constexpr int NQ0 = 6 + 2 * D, NPM = kMtMaxT * (kMtMaxT + 1) / 2;
  __shared__ double tot[kMtMaxT * (NQ0 + 2 * NPM)];
  __shared__ double lossg[kMtMaxT], c1s[kMtMaxT], c2s[kMtMaxT], dk[NPM];
  __shared__ int rgs[kSpecScratch];
  const bool cv = a.loss == FGP_LOSS_CV;
  const int T = a.mt, NP = T * (T + 1) / 2, P = cv ? T : 1, nq = a.nq, ng = spec_groups(a), R = a.mt_rank;
  for (int t = threadIdx.x; t < P * nq; t += kWG) {
    const int g = t / nq, q = t - g * nq;
    double sum = 0.0;
    for (int grp = 0; grp < ng; ++grp) sum += spec_group_sum<false>(a, g, q, grp);
    tot[t] = sum;
  }
  __syncthreads();
  // (GCV: the trace is normalised by the points of all T tasks, util.py:379; CV: I_t over the n points of task t)
  const double n = (double)((int64_t)1 << a.log2n) * (cv ? 1 : T);
  if ((int)threadIdx.x < P) {
    const int i = threadIdx.x;
    const double N1 = tot[i * nq + 0], Tr = tot[i * nq + 1];
    if (cv) {
      const double I = Tr / n, w = a.cv_weight;
      lossg[i] = w * N1 / (I * I);
      c1s[i] = -2.0 * w / (I * I);
      c2s[i] = 2.0 * w * N1 / (n * I * I * I);
    } else {
      const double Dn = (Tr / n) * (Tr / n);
      lossg[i] = N1 / Dn;
      c1s[i] = -2.0 / Dn;
      c2s[i] = 2.0 * N1 * Tr / (n * n * Dn * Dn);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double L = 0.0;
    for (int i = 0; i < P; ++i) L += lossg[i];
    f.loss_hist[(int64_t)iter * 3 + 0] = L;
    f.loss_hist[(int64_t)iter * 3 + 1] = cv ? NAN : tot[0];
    f.loss_hist[(int64_t)iter * 3 + 2] = cv ? NAN : (tot[1] / n) * (tot[1] / n);
  }
  for (int p = threadIdx.x; p < NP; p += kWG) {
    double s = 0.0;
    for (int i = 0; i < P; ++i) s += c1s[i] * tot[i * nq + NQ0 + p] + c2s[i] * tot[i * nq + NQ0 + NP + p];
    dk[p] = s;
  }
  __syncthreads();
  const int dl = a.ls_pd ? a.d : 1, np = spec_nparams(a);
  const double* Fm = f.raw + a.mt_f_off;
  for (int pi = threadIdx.x; pi < np; pi += kWG) {
    double gp = 0.0;
    int rg;
    if (pi >= a.mt_v_off) {                               // task noise v_t
      const int t = pi - a.mt_v_off;
      gp = dk[t * T - t * (t - 1) / 2];
      if (a.mt_vexp) gp *= exp(f.raw[pi]);
      rg = (a.mt_learn >> 1) & 1;
    } else if (pi >= a.mt_f_off) {                        // task factor F[t, r]
      const int t = (pi - a.mt_f_off) / R, r = (pi - a.mt_f_off) - t * R;
      for (int p = 0, k = 0; k < T; ++k)
        for (int l = k; l < T; ++l, ++p) {
          if (k == t) gp += dk[p] * Fm[l * R + r];
          if (l == t) gp += dk[p] * Fm[k * R + r];
        }
      rg = a.mt_learn & 1;
    } else {
      rg = -1;
      for (int i = 0; i < P; ++i) {
        const double* v = tot + i * nq;
        for (int k = 0; k < 2 + dl; ++k) {
          if (spec_slot_param(a, 0, k, dl) != pi) continue;
          double s1, s2;
          if (k == 0) {
            s1 = v[3];
            s2 = v[5 + D];
            rg = f.scale_rg;
          } else if (k <= dl) {
            s1 = s2 = 0.0;
            for (int j = 0; j < D; ++j)
              if (a.ls_pd ? j == k - 1 : true) {
                s1 += v[4 + j];
                s2 += v[6 + D + j];
              }
            rg = f.ls_rg;
          } else {
            const double nz = exp(f.raw[pi]);
            s1 = nz * v[2];
            s2 = nz * v[4 + D];
            rg = f.noise_rg;
          }
          gp += c1s[i] * s1 + c2s[i] * s2;
        }
      }
    }
    rgs[pi] = rg;
    if (rg < 0) continue;
    f.raw_hist[(int64_t)iter * f.n_params + pi] = f.raw[pi];
    f.grad_out[pi] = gp;
  }
  // (every gradient reads the factor before any update: the steps after a barrier)
  __syncthreads();
  for (int pi = threadIdx.x; pi < np; pi += kWG)
    if (do_update && rgs[pi] > 0) rprop_update(f, pi, f.grad_out[pi]);
}

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void glb_void;

// s_waitcnt vmcnt(n) for a runtime n <= 15 (the immediate must be a constant)
__device__ __forceinline__ void wait_vmcnt(int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
    case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
    case 11: asm volatile("s_waitcnt vmcnt(11)" ::: "memory"); break;
    case 12: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    case 13: asm volatile("s_waitcnt vmcnt(13)" ::: "memory"); break;
    case 14: asm volatile("s_waitcnt vmcnt(14)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(15)" ::: "memory"); break;
  }
}

// k_spec_tile's prologue (A/B builds, tools/build_exp.sh): chunks issued before the deferred step (at most the
// ring), and the Rprop state loaded beside the level-2 sums (1) or after them (0)
#ifndef FGP_SPEC_PRE
#define FGP_SPEC_PRE 2
#endif
#ifndef FGP_SPEC_PF
#define FGP_SPEC_PF 0     // (1: ~100 more VALU per wave, no measurable gain: profiles/r04ab2_basis_gen_prefetch.txt)
#endif

// fgp_handoff_check (a test hook, fz.check): lane 0 of each storing wave reads back the partials it stored
// (its own retired stores) and XORs their bits into the group's words [grp][g][q] with agent-scope atomics,
// before the workgroup's arrival -- ordered like the partials by the same vmcnt(0) wait ...
__device__ __forceinline__ void handoff_check_store(const Nll& a, const FitFuse& fz, int grp, int g0, int ppw, int GS,
                                                 int blk, bool active) {
  if (!active || (threadIdx.x & 63) != 0) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  for (int p = 0; p < ppw && g0 + p < GS; ++p)
    for (int q = 0; q < a.nq; ++q) {
      const double v = __hip_atomic_load(part_ptr(a, g0 + p, q, blk), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_xor(fz.check + ((int64_t)grp * a.G + g0 + p) * a.nq + q, (unsigned long long)__double_as_longlong(v),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// ... and the group's last arriver (thread (g, q)) recomputes the XOR from the partials it reads (sc1 loads, as
// spec_group_sum), counts a mismatch, and re-arms the word
__device__ __forceinline__ void handoff_check_verify(const Nll& a, const FitFuse& fz, int grp, int g, int q) {
  const int b0 = grp * kSpecGroup, nbg = min(kSpecGroup, a.nb - b0);
  unsigned long long x = 0;
  for (int b = 0; b < nbg; ++b)
    x ^= (unsigned long long)__double_as_longlong(
        __hip_atomic_load(part_ptr(a, g, q, b0 + b), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  unsigned long long* wd = fz.check + ((int64_t)grp * a.G + g) * a.nq + q;
  if (__hip_atomic_load(wd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != x)
    __hip_atomic_fetch_add(fz.check + kHandoffWords + 1, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(wd, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One fit iteration when every problem shares ONE set of spectra and the problem groups fit in the four
// waves of a workgroup (PG = ceil(G / PPW) <= 4; the C4 shifts, single GPs) -- or, for many problems, over
// problem slices of 4 PPW problems (spec_geometry) -- and the ring of kSpecRing chunks fits kSpecLdsMax
// (two workgroups per CU).  The k blocks are those of
// k_spec_iter (nb blocks of B = 64 kpl frequencies, one partial per problem and block, lane l summing
// k = block base + l + 64 i in ascending i): workgroup b owns NBW = 4 / PGP consecutive blocks (PGP = PG
// rounded up to 1, 2 or 4), wave w the block w / PGP for problem group w mod PGP -- so every problem's
// arithmetic, and its partials, are those of k_spec_iter whatever G is (a batch equals its GPs' own fits
// bit for bit).  The spectra and Y stream through the LDS ring in chunks of 64 frequencies per
// block: the chunk's (2^d + G) rows x NBW segments are read ONCE from HBM by all four waves (16-byte LDS-DMA
// loads, global_load_lds_dwordx4, no register staging; RING - 1 chunks in flight under each chunk's compute,
// counted vmcnt waits and raw barriers so they stay in flight: cdna_hip_programming.md section 5
// "Pipelining across barriers") instead of once per problem group, and each wave reads its segment from
// LDS (lane-consecutive 8-byte reads: conflict-free).  With fz.counters the LAST workgroup to finish (sc1 partials, an agent-scope arrival
// counter: MI355X_MICROARCH.md hand-off row 1, as the real-even backward kernel) runs every problem's
// reduction + Rprop, wave w taking problems w, w + 4, ...
// The persistent k_spec_tile re-reads its kernel arguments in each phase (iteration prologue, epilogue) from the
// kernarg segment behind an opaque asm: otherwise their scalar values are held from one iteration to the next,
// through the chunk loop, and spill (SGPRs into VGPR lanes, v_readlane in the loop).
struct TileArgs {
  Nll a;
  FitFuse fz;
};
template <bool FRESH>
__device__ __forceinline__ const TileArgs* tile_args() {
  typedef const __attribute__((address_space(4))) TileArgs* KargPtr;
  KargPtr p = (KargPtr)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(p));
  return (const TileArgs*)p;
}

template <int D, int PPW, bool NET, bool PERSIST = false>
__global__ __launch_bounds__(kWG, 2) void k_spec_tile(Nll a, FitFuse fz) {
  constexpr int NS = 1 << D;
  constexpr int RING = kSpecRing;                   // chunks in LDS; RING - 1 in flight under a compute
  extern __shared__ double lds[];                   // [RING][NBW][NS + PS][64] ring
  // w through readfirstlane: wave-uniform to the compiler, so the problem flags, the DMA counts and the vmcnt
  // switch are scalar (a VGPR w compiled them into exec-mask branch trees inside the chunk loop)
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int PGP = a.spec_pgp, NBW = 4 / PGP, G = a.G;
  // problem slices (many problems on one set of spectra, a.spec_nsl > 1): workgroup = (k block, slice),
  // the slices of one block consecutive (they share its spectra chunks in L2); slice s holds problems
  // [s PS, s PS + GS) in the tile's Y rows (rows past G re-read problem G - 1 and are not evaluated)
  const int nsl = a.spec_nsl, PS = a.spec_ps ? a.spec_ps : G;
  const int slice = nsl > 1 ? (int)blockIdx.x % nsl : 0, wgb = nsl > 1 ? (int)blockIdx.x / nsl : (int)blockIdx.x;
  const int goff = slice * PS, GS = min(PS, G - goff);
  const int rows = NS + PS, tile = rows * NBW * 64, npieces = tile / 2, segp = 32 * rows;
  const int ninst = npieces / 64;                   // 1-KiB LDS-DMA wave-instructions per chunk (whole)
  const int cnt_w = (ninst - w + 3) / 4;            // ... issued by this wave: j = w, w + 4, ...
  const int pg = w % PGP, bw = w / PGP;
  const int g0 = pg * PPW;
  const bool active = g0 < GS;
  const int64_t B = 64 * (int64_t)a.spec_kpl;       // frequencies per block
  const int blk = wgb * NBW + bw;
  stamp_begin(a);
  bool on[PPW];
#pragma unroll
  for (int p = 0; p < PPW; ++p) on[p] = g0 + p < GS;
  const double rootn = sqrt((double)((int64_t)1 << a.log2n)), wl = a.logdet_weight;
  const int64_t wg_base = (int64_t)wgb * NBW * B;
  // chunk c into buffer buf: piece i (16 bytes) = segment i / (32 rows) (the workgroup's block), row
  // (i mod 32 rows) / 32 (spectrum rows, then Y rows), column i mod 32, at LDS byte 16 i -- a wave's
  // spectra and Y of a chunk are then at compile-time offsets from one base.  Wave-instruction j moves
  // pieces [64 j, 64 j + 64); this wave's instructions j = w + 4 t (t < cnt_w <= kMaxDma): chunk-0 source
  // and per-chunk step per lane, formed once (a chunk further is NS 64 doubles on in the chunked spectra,
  // 64 in a Y row).
  constexpr int kMaxDma = kSpecMaxDma;              // tile <= 512 kMaxDma doubles: 1-KiB instructions, kMaxDma per wave
  static_assert(RING >= 2, "a chunk in flight under each chunk's compute");
  const double* src0[kMaxDma];
  int64_t step[kMaxDma];
#pragma unroll
  for (int t = 0; t < kMaxDma; ++t) {
    const int jj = w + 4 * t;
    const int i = (jj < ninst ? jj : 0) * 64 + lane;
    const int sg = i / segp, rem = i - sg * segp, r = rem >> 5, col = rem & 31;
    const int64_t k = wg_base + sg * B;             // the segment's first frequency in chunk 0
    const int gy = min(goff + r - NS, G - 1);
    src0[t] = (r < NS ? a.basis + spec_at<NS>(k, r) : a.ysq + ysq_at(a, gy, k)) + 2 * col;
    step[t] = r < NS ? NS * 64 : (a.ysq_chunked ? (int64_t)G * 64 : 64);
  }
  auto issue = [&](int c, double* buf) {
#pragma unroll
    for (int t = 0; t < kMaxDma; ++t) {
      if (t < cnt_w) {
        const double* src = src0[t] + step[t] * c;
        __builtin_amdgcn_global_load_lds((glb_void*)src, (lds_void*)(buf + 128 * (w + 4 * t)), 16, 0, 0);
      }
    }
  };
  const int nc = a.spec_kpl;
  const unsigned wofs = (unsigned)(bw * rows * 64 + lane);   // this lane's spectra in a buffer: wofs + 64 s
  const unsigned yofs = wofs + (unsigned)(NS + g0) * 64u;     // ... its problems' Y: yofs + 64 p
  __shared__ double scr[kSpecScratch];              // [G nq] level-2 totals, then [np] new raw parameters
  // Persistent mode (fz.piters > 0, fgp_fit_run): the launch runs iterations fz.iter .. fz.iter + piters - 1,
  // every workgroup holding the Rprop state in LDS (st_*, updated identically by all, as k_spec_persist); the
  // launch boundary between iterations becomes a wait on the count of published group sums (the group
  // finishers' agent-scope adds after their sc1 stores: hand-off row 1; a bounded poll by one lane).
  __shared__ double st_raw[kSpecStateMax], st_prev[kSpecStateMax], st_step[kSpecStateMax];
  __shared__ int wfail;
  constexpr bool persist = PERSIST;                 // (fz.piters > 0: the launcher picks this instance)
  const int nit = persist ? fz.piters : 1, ng = spec_groups(a);
  const RpState lst{st_raw, st_prev, st_step};
  unsigned* done_ctr = fz.counters ? fz.counters + ng : nullptr;
  if constexpr (PERSIST) {
    const int np = spec_nparams(a);
    for (int p = threadIdx.x; p < np; p += kWG) {
      st_raw[p] = fz.sin.raw[p];
      st_prev[p] = fz.sin.prev[p];
      st_step[p] = fz.sin.step[p];
    }
  }
  // thread 0: wait until `target` group sums are published; false (and the fail word set) if the bounded
  // poll gave up.  Uniform over the workgroup (LDS word + barrier).
  auto wait_published = [&](unsigned target) -> bool {
    if (threadIdx.x == 0) {
      int f = 0;
      long long polls = 0;
      while (__hip_atomic_load(done_ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(1);
        if (++polls > kSpecPollMax) {
          f = 1;
          __hip_atomic_store(done_ctr + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
      wfail = f;
    }
    __syncthreads();
    return wfail == 0;
  };
  for (int li = 0; li < nit; ++li) {
  const int iter = fz.iter + li, par = persist ? (iter & 1) : fz.par;
  SpecAcc<D> acc[PPW];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // only the chunk loads below are counted
  if (persist) __syncthreads();                     // the previous iteration's ring / flag reads done; st_* loaded
  // the single-frequency corrections of block 0 / the last block, loaded ahead of the chunk DMAs (older: a
  // chunk's counted wait covers them too; first used in the epilogue)
  // (k_spec_tile loads them in its epilogue: preloading them here, 6 VGPRs and their v_readlane broadcasts, cost
  // SGPR spills through the chunk loop and measured no shorter tail, profiles/r04e_spec_stamps.jsonl)
  const SpecCorr corr{0.0, 0.0, 0.0, 0, false};
  // every ring slot filled before the loop (the prologue below runs under them): chunks 0 .. pre - 1
  const int pre = min(min(FGP_SPEC_PRE, RING), nc);
#pragma unroll
  for (int c = 0; c < RING; ++c)
    if (c < pre) issue(c, lds + c * tile);
  int issued = pre;
  // The parameters of this iteration.  With fz.pending the previous iteration's step was deferred into
  // this launch: every workgroup sums its group sums (level 2, fixed order) and applies the Rprop step
  // (identical arithmetic, identical results), workgroup 0 alone storing histories and the new state,
  // while the first chunks are in flight; the parameters then come from LDS (scr).  The Rprop state is
  // loaded beside the level-2 sums (one round trip, not two).
  Hyp h[PPW];
  if (fz.counters && persist && li > 0) {
    // the previous iteration's group sums (all ng published), its step on the LDS state
    if (!wait_published((unsigned)(li * ng))) {
      // (as k_spec_persist: no workgroup writes the final state after a failed wait; the parameters become NaN)
      for (int p = threadIdx.x; p < spec_nparams(a); p += kWG) fz.sout.raw[p] = NAN;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      return;
    }
    const TileArgs* ka = tile_args<PERSIST>();
    spec_level2<D, true>(ka->a, par ^ 1, scr);
    __syncthreads();
    spec_finish<D>(ka->a, ka->fz.f, scr, 0, G, iter - 1, 1, lst, lst, blockIdx.x == 0, nullptr, 1);
    __syncthreads();
#pragma unroll
    for (int p = 0; p < PPW; ++p) load_hyp_wave(ka->a, on[p] ? g0 + p : 0, h[p], st_raw);
  } else if (persist) {
#pragma unroll
    for (int p = 0; p < PPW; ++p) load_hyp_wave(a, on[p] ? g0 + p : 0, h[p], st_raw);
  } else if (fz.counters && fz.pending) {
    double* tot = scr;
    double* nraw = tot + G * a.nq;
    const int tf = tid_fresh(), si = tf >> 4, sk = tf & 15, dl = a.ls_pd ? a.d : 1;
    double pf[3] = {0.0, 0.0, 0.0};
    if (FGP_SPEC_PF && si < G && sk < 2 + dl) {
      const int p = spec_slot_param(a, si, sk, dl);
      pf[0] = fz.sin.raw[p];
      pf[1] = fz.sin.prev[p];
      pf[2] = fz.sin.step[p];
    }
    spec_level2<D>(a, fz.par ^ 1, tot);
    __syncthreads();
    spec_finish<D>(a, fz.f, tot, 0, G, fz.iter - 1, 1, fz.sin, fz.sout, blockIdx.x == 0, nraw, -1, FGP_SPEC_PF ? pf : nullptr);
    // (nraw is LDS; workgroup 0's history / state stores stay in flight: the chunk waits below count only the
    // older DMA loads as landed -- loads retire in order, so extra stores only make them more conservative)
    barrier_keep_vm();
#pragma unroll
    for (int p = 0; p < PPW; ++p) load_hyp_wave(a, on[p] ? g0 + p : 0, h[p], nraw);
  } else {
#pragma unroll
    for (int p = 0; p < PPW; ++p) load_hyp_wave(a, on[p] ? goff + g0 + p : 0, h[p]);
  }
  for (int c = 0; c < nc; ++c) {
#ifdef FGP_SPEC_PRIO
    // (experiment: issue priority falling with progress -- the workgroup behind on its CU wins the SIMDs' arbitration)
    if (FGP_SPEC_PRIO == 4) {
      const int q = (4 * c) / nc;
      if (q == 0) __builtin_amdgcn_s_setprio(3);
      else if (q == 1) __builtin_amdgcn_s_setprio(2);
      else if (q == 2) __builtin_amdgcn_s_setprio(1);
      else __builtin_amdgcn_s_setprio(0);
    } else {
      if (2 * c < nc) __builtin_amdgcn_s_setprio(1);
      else __builtin_amdgcn_s_setprio(0);
    }
#endif
    // this wave's loads of chunk c have landed (chunks c + 1 .. issued - 1 may stay in flight)
    wait_vmcnt(cnt_w * (issued - 1 - c));
    barrier_keep_vm();                              // ... every wave's; every wave done with chunk c - 1
    if (issued < nc && issued <= c + RING - 1) {    // into the slot of chunk c - 1
      issue(issued, lds + (issued % RING) * tile);
      ++issued;
    }
    const double* buf = lds + (unsigned)(c % RING) * (unsigned)tile;
    if (active) {
      const double* wb = buf + wofs;
      double phi[NS];
#pragma unroll
      for (int s = 0; s < NS; ++s) phi[s] = wb[64u * s];
      const double* yb = buf + yofs;
#pragma unroll
      for (int p = 0; p < PPW; ++p)
        if (on[p]) spec_terms<D>(phi, h[p], rootn, wl, yb[64u * p], acc[p]);
    }
  }
  {
  const TileArgs* ka = PERSIST ? tile_args<PERSIST>() : nullptr;
  const Nll& a_ = PERSIST ? ka->a : a;
  const FitFuse& fz_ = PERSIST ? ka->fz : fz;
  {
  const Nll& a = a_;
  const FitFuse& fz = fz_;
  // the block's partials (k_spec_iter's values; sc1 when handed to the last workgroup)
#pragma unroll
  for (int p = 0; p < PPW; ++p)
    if (on[p] && active)
      spec_block_partials<D, NET>(a, h[p], goff + g0 + p, blk, rootn, wl, acc[p], fz.counters != nullptr, a.partials,
                                  corr);
  if (fz.check && fz.counters) handoff_check_store(a, fz, blk / kSpecGroup, g0, PPW, GS, blk, active);
  if (fz.counters) {
    // Level 1 of the fused reduction (MI355X_MICROARCH.md hand-off row 1: sc1 stores retired by every
    // storing wave, then ONE lane's agent-scope add; the waiter reads with sc1 loads after a barrier): the
    // last workgroup of each group of kSpecGroup blocks sums the group into the level-2 inputs of parity
    // fz.par.  Level 2 and the step follow in the next launch's prologue (or k_spec_finish_step).
    const int grp = wgb * NBW / kSpecGroup;
    const int wg_in_grp = (min(kSpecGroup, a.nb - grp * kSpecGroup) + NBW - 1) / NBW;
    unsigned* cnt_grp = fz.counters + grp;
    int* flag = reinterpret_cast<int*>(lds);        // the ring is free now
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // (relaxed add on purpose: the partials are agent-scope atomic stores retired by the vmcnt(0) wait above,
    // the asm's memory clobber keeps the compiler from moving them; an acq_rel add / release fence emits an
    // L2 write-back per workgroup: 40.9 -> 46.4 us per C4 iteration, profiles/r03ar_exp_acq_rel_handoff.jsonl)
    if (threadIdx.x == 0) flag[0] = __hip_atomic_fetch_add(cnt_grp, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                                    (unsigned)(wg_in_grp - 1);
    __syncthreads();
    if (flag[0]) {
      const int t = tid_fresh();
      if (t < G * a.nq) {
        const int g = t / a.nq, q = t % a.nq;
        __hip_atomic_store(part2_ptr(a, par, g, q, grp), spec_group_sum<true>(a, g, q, grp), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        if (fz.check) handoff_check_verify(a, fz, grp, g, q);
      }
      if (fz.check && threadIdx.x == 0)
        __hip_atomic_fetch_add(fz.check + kHandoffWords, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (threadIdx.x == 0) __hip_atomic_store(cnt_grp, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (persist) {
        // publish: every storing wave's group sums (and the counter reset) retired, then one add
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) __hip_atomic_fetch_add(done_ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  }
  }
  }   // iterations
  // persistent: the last iteration's step (k_spec_finish_step's work) by workgroup 0, into the fit's vectors
  if (persist && fz.counters && blockIdx.x == 0) {
    if (!wait_published((unsigned)(nit * ng))) {
      for (int p = threadIdx.x; p < spec_nparams(a); p += kWG) fz.sout.raw[p] = NAN;
      return;
    }
    spec_level2<D, true>(a, (fz.iter + nit - 1) & 1, scr);
    __syncthreads();
    spec_finish<D>(a, fz.f, scr, 0, G, fz.iter + nit - 1, fz.do_update, lst, fz.sout, true, nullptr, 1);
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
  for (int s = 0; s < NS; ++s) phi[s] = phib[spec_at<NS>(k, s)];
  const double lam = h.scale * mlin<D>(phi, h.ls, dp);
  if constexpr (NET) {
    static_cast<double*>(a.grad_lam)[(int64_t)g * n + k] = lam;
  } else {
    double2* out = static_cast<double2*>(a.grad_lam) + (int64_t)g * n;
    out[k] = make_double2(lam, 0.0);
    if (k > 0 && k < n / 2) out[n - k] = make_double2(lam, 0.0);
  }
}

// ---------------------------------------------------------------- multitask spectral fit (ABI 12)
// One multitask / derivative-informed GP of T tasks with equal n (include/fgp_hip.h mt_tasks): the reference
// inverts, per frequency j, the T x T Hermitian block Lambda_j of its lams (util.py:277-337) and forms
// norm = Re sum_j y_j^H Lambda_j^-1 y_j and logdet = sum_j log|det Lambda_j| (util.py:364-370), y_j = (ytilde_k[j])_k;
// autograd then differentiates through the block recursion and the transforms.  Here the pair eigenvalues
// come from the pair spectra (lambda_kl = scale sum_S l^S Phi^{kl}_S, the part-product spectra of the
// single-task path, per task pair), the block is factored LDL^H in LDS, and the gradient is the closed form
//   dL = 1/2 tr(W dLambda),  W = Lambda^-1 - z z^H,  z = Lambda^-1 y:
//   dL/draw_scale = sum_j sum_{k<=l} w_kl Re(W[l,k] dLambda[k,l]/draw_scale),  w = 1/2 (k = l) or 1,
//   dLambda[k,l]/draw_scale = Kt[k,l] sqrt(n) scale P_kl,
//   dLambda[k,l]/draw_l_m   = Kt[k,l] sqrt(n) scale sum_{S contains m} l^S Phi^{kl}_S   (l_m dP/dl_m),
//   dL/dnoise = 1/2 sum_k Re W[k,k] Kt[k,k]
// -- the quantities of the single-task partials (norm, logdet, dL/dnoise, dL/draw_scale, dL/draw_l), so
// k_spec_reduce_step reduces them and applies the Rprop step (G = 1).  Workgroup = block of mt_cpb chunks of
// F frequencies: (1) threads over (pair, frequency) evaluate the pair polynomials into the blocks (LDS),
// (2) one thread per frequency factors its block, solves, and forms W (LDS), (3) threads over (pair,
// frequency) contract W with the spectra; fixed per-thread orders and a fixed block reduction.
__device__ __forceinline__ double2 mt_phi(const Nll& a, int64_t idx) {
  if (a.spec_net) return make_double2(static_cast<const double*>(a.mt_basis)[idx], 0.0);
  return static_cast<const double2*>(a.mt_basis)[idx];
}

__device__ __forceinline__ void mt_pair_kl(int p, int T, int& k, int& l) {
  k = 0;
  while (p >= T - k) {
    p -= T - k;
    ++k;
  }
  l = k + p;
}

// GCV (ABI 17, util.py:371-380 with T tasks of equal n): numer N = sum_j |z_j|^2, Tr = sum_j tr Lambda_j^-1, loss
// N / (Tr / (T n))^2; with u = Lambda^-1 z, dN = -2 Re(u^H dLambda z) and dTr = -Re tr(Lambda^-2 dLambda), so the block
// partials are the single-task GCV layout (k_spec_loss_step): [N, Tr, S1 (noise, scale, l_m), S2 (noise, scale, l_m)]
// with S1 = 1/2 Re tr(W1 dLambda), W1 = z u^H + u z^H, and S2 = 1/2 Re tr(W2 dLambda), W2 = 2 Lambda^-2.
// CV (ABI 18, util.py:381-394 + abstract_gp.py:261-272 with T tasks of equal n): K^-1's diagonal is constant over the
// points of task t, I_t = (1/n) sum_j Lambda_j^-1[t, t] (K^-1's block (t, t) is ift diag(Lambda^-1[t, t]) ft), and
// sum_i coeffs_{t,i}^2 = N_t = sum_j |z_{j,t}|^2 (Parseval), so loss = w sum_t N_t / I_t^2 -- the single-task CV of each
// task.  Workgroup (block, t) = blockIdx (x, y): with v = Lambda^-1 e_t (column t of the inverse) and u = v z_t,
// dN_t = -2 Re(u^H dLambda z) and d(n I_t) = -v^H dLambda v: the GCV layout per task, W1 = z u^H + u z^H, W2 = 2 v v^H,
// partials [t][N_t, n I_t, S1, S2] read by k_spec_loss_step as T problems of one loss.
// LEARN (ABI 18, GCV / CV): K_task = F F^T + diag(v) from raw (k_mt_learn_step's parameters) and, per task pair p = (k, l),
// the two streams of dK = w_kl Re(W[l, k] dLambda[k, l] / dK_task[k, l]) = w_kl Re(W[l, k] (sqrt(n) scale P_kl +
// noise [k == l])) for W = W1, W2 -- partials q = NQ + p and NQ + NP + p.  Thread it of the phase-3 loop holds pair
// it / F in its slot it / kWG; a slot's F threads of a pair are summed in ascending f at the end (fixed order).
constexpr int kMtSlots = (kMtMaxT * (kMtMaxT + 1) / 2 * kMtF + kWG - 1) / kWG;
template <int D, bool GCV = false, bool CV = false, bool LEARN = false>
__global__ __launch_bounds__(kWG) void k_mt_spec_iter(Nll a) {
  static_assert(!CV || GCV, "CV uses the GCV machinery");
  static_assert(!LEARN || GCV, "a learned task kernel on the GCV / CV paths");
  constexpr int NS = 1 << D, NQ = GCV ? 6 + 2 * D : 4 + D;
  __shared__ double ls_pow[NS];                          // l^S
  __shared__ double kt[kMtMaxT * kMtMaxT];
  __shared__ double2 blk[kMtF][kMtMaxT * kMtMaxT];       // Lambda_j (full), factored in place (GCV: then W2 packed)
  __shared__ double2 wv[kMtF][kMtMaxT * (kMtMaxT + 1) / 2];   // W[l, k] of pair (k, l)  (GCV: W1)
  __shared__ double2 iv[GCV ? kMtF : 1][GCV ? kMtMaxT * (kMtMaxT + 1) / 2 : 1];   // GCV: Lambda^-1[l, k], l >= k
  __shared__ double red[kWG / 64];
  const int T = a.mt, NP = T * (T + 1) / 2, F = a.mt_F, tid = threadIdx.x;
  const int tcv = CV ? (int)blockIdx.y : -1;             // CV: this workgroup's task
  const int64_t n = (int64_t)1 << a.log2n;
  stamp_begin(a);
  Hyp h;
  load_hyp_wave(a, 0, h);
  if (tid < NS) {
    double pw = 1.0;
#pragma unroll
    for (int j = 0; j < D; ++j)
      if ((tid >> j) & 1) pw *= h.ls[j];
    ls_pow[tid] = pw;
  }
  if (tid < T * T) {
    if constexpr (LEARN) {
      // K_task[ka, kb] = sum_r F[ka, r] F[kb, r] + [ka == kb] v_ka (util.py:157-162, ascending r)
      const int ka = tid / T, kb = tid - ka * T, R = a.mt_rank;
      const double* Fm = a.raw + a.mt_f_off;
      double s = 0.0;
      for (int r = 0; r < R; ++r) s += Fm[ka * R + r] * Fm[kb * R + r];
      if (ka == kb) s += a.mt_vexp ? exp(a.raw[a.mt_v_off + ka]) : a.raw[a.mt_v_off + ka];
      kt[tid] = s;
    } else {
      kt[tid] = a.mt_kt[tid];
    }
  }
  const double rootn = sqrt((double)n), sn = rootn * h.scale;
  double acc_norm = 0.0, acc_ld = 0.0, acc_noise = 0.0, acc_sc = 0.0, acc_l[D];
  double acc_noise2 = 0.0, acc_sc2 = 0.0, acc_l2[D];     // (GCV: the S2 sums; acc_ld holds Tr)
  double kta[LEARN ? kMtSlots : 1], ktb[LEARN ? kMtSlots : 1];   // LEARN: the pairs' dK streams, per slot
#pragma unroll
  for (int s2 = 0; s2 < (LEARN ? kMtSlots : 1); ++s2) kta[s2] = ktb[s2] = 0.0;
#pragma unroll
  for (int m = 0; m < D; ++m) acc_l[m] = acc_l2[m] = 0.0;
  for (int c = 0; c < a.mt_cpb; ++c) {
    const int64_t j0 = ((int64_t)blockIdx.x * a.mt_cpb + c) * F;
    __syncthreads();                                     // ls_pow / kt ready; previous chunk's wv consumed
    // (1) Lambda[k, l] = Kt[k, l] (sqrt(n) scale P_kl + noise [k == l]) (the reference's order of operations)
    for (int it = tid; it < NP * F; it += kWG) {
      const int p = it / F, f = it - p * F;
      int k, l;
      mt_pair_kl(p, T, k, l);
      const int64_t base = (int64_t)p * NS * n + j0 + f;
      double2 P = make_double2(0.0, 0.0);
      // the subsets in groups of 8, the group loop rolled (a fully unrolled 2^6-term loop spilled), S ascending
      constexpr int U = NS < 8 ? NS : 8;
#pragma unroll 1
      for (int sh = 0; sh < NS; sh += U) {
#pragma unroll
        for (int t = 0; t < U; ++t) {
          const int S = sh + t;
          const double2 ph = mt_phi(a, base + (int64_t)S * n);
          P.x = __builtin_fma(ls_pow[S], ph.x, P.x);
          P.y = __builtin_fma(ls_pow[S], ph.y, P.y);
        }
      }
      const double q = kt[k * T + l];
      double2 v = make_double2(sn * P.x, sn * P.y);
      if (k == l) v.x += h.noise;
      v = make_double2(v.x * q, v.y * q);
      blk[f][k * T + l] = v;
      if (k != l) blk[f][l * T + k] = make_double2(v.x, -v.y);
    }
    __syncthreads();
    // (2) per frequency: LDL^H (L strictly below the diagonal of blk, pivots Dg), logdet, z = Lambda^-1 y,
    // norm, X = L^-1 (strictly lower, stored transposed in the upper triangle), W = Lambda^-1 - z z^H
    if (tid < F) {
      double2* A = blk[tid];
      const int64_t j = j0 + tid;
      double Dg[kMtMaxT];
      double2 y[kMtMaxT], z[kMtMaxT];
      for (int k = 0; k < T; ++k) {
        double dk = A[k * T + k].x;
        for (int m = 0; m < k; ++m) {
          const double2 L = A[k * T + m];
          dk -= (L.x * L.x + L.y * L.y) * Dg[m];
        }
        Dg[k] = dk;
        for (int i = k + 1; i < T; ++i) {
          double2 s = A[i * T + k];
          for (int m = 0; m < k; ++m) {
            const double2 t = cmulc(A[i * T + m], A[k * T + m]);   // L[i][m] conj(L[k][m])
            s.x -= t.x * Dg[m];
            s.y -= t.y * Dg[m];
          }
          A[i * T + k] = make_double2(s.x / dk, s.y / dk);
        }
        if constexpr (!GCV) acc_ld += log(fabs(dk));
      }
      for (int k = 0; k < T; ++k) {
        if (a.spec_net) y[k] = make_double2(static_cast<const double*>(a.mt_ytilde)[(int64_t)k * n + j], 0.0);
        else y[k] = static_cast<const double2*>(a.mt_ytilde)[(int64_t)k * n + j];
      }
      // forward: w = L^-1 y (in z), norm = sum |w_k|^2 / D_k, then u = w / D, backward L^H z = u
      for (int i = 0; i < T; ++i) {
        double2 s = y[i];
        for (int m = 0; m < i; ++m) {
          const double2 t = cmul(A[i * T + m], z[m]);
          s.x -= t.x;
          s.y -= t.y;
        }
        z[i] = s;
        if constexpr (!GCV) acc_norm += (s.x * s.x + s.y * s.y) / Dg[i];
      }
      for (int i = 0; i < T; ++i) z[i] = make_double2(z[i].x / Dg[i], z[i].y / Dg[i]);
      for (int i = T - 1; i >= 0; --i) {
        double2 s = z[i];
        for (int m = i + 1; m < T; ++m) {
          const double2 t = cmulc(z[m], A[m * T + i]);            // conj(L[m][i]) z[m]
          s.x -= t.x;
          s.y -= t.y;
        }
        z[i] = s;
      }
      // X = L^-1: X[i][jj] = -(L[i][jj] + sum_{jj < m < i} L[i][m] X[m][jj]), stored at A[jj T + i]
      for (int jj = 0; jj < T; ++jj)
        for (int i = jj + 1; i < T; ++i) {
          double2 s = A[i * T + jj];
          for (int m = jj + 1; m < i; ++m) {
            const double2 t = cmul(A[i * T + m], A[jj * T + m]);
            s.x += t.x;
            s.y += t.y;
          }
          A[jj * T + i] = make_double2(-s.x, -s.y);
        }
      // Lambda^-1[l][k] = sum_{m >= l} conj(X[m][l]) X[m][k] / D_m  (l >= k, X[m][m] = 1)
      for (int p = 0, k = 0; k < T; ++k)
        for (int l = k; l < T; ++l, ++p) {
          double2 s = make_double2(0.0, 0.0);
          for (int m = l; m < T; ++m) {
            const double2 xl = m == l ? make_double2(1.0, 0.0) : A[l * T + m];
            const double2 xk = m == k ? make_double2(1.0, 0.0) : A[k * T + m];
            const double2 t = cmulc(xk, xl);                      // conj(X[m][l]) X[m][k]
            s.x += t.x / Dg[m];
            s.y += t.y / Dg[m];
          }
          if constexpr (GCV) {
            iv[tid][p] = s;
            if (k == l && (!CV || k == tcv)) acc_ld += s.x;      // Tr (CV: n I_t)
            continue;
          }
          const double2 zz = cmulc(z[l], z[k]);                  // z_l conj(z_k)
          const double2 w = make_double2(s.x - zz.x, s.y - zz.y);
          wv[tid][p] = w;
          if (k == l) acc_noise += 0.5 * w.x * kt[k * T + k];
        }
      if constexpr (GCV) {
        // N, u = Lambda^-1 z (the factor: L w = z, w / D, L^H u = w), W1 = z u^H + u z^H, W2 = 2 Lambda^-2 (packed into
        // the factor's block, which is no longer read)
        double2 u[kMtMaxT];
        const double2* V = iv[tid];
        auto inv_at = [&](int r, int c) -> double2 {            // Lambda^-1[r][c] from the packed l >= k entries
          if (r >= c) return V[c * T - c * (c - 1) / 2 + (r - c)];
          const double2 t = V[r * T - r * (r - 1) / 2 + (c - r)];
          return make_double2(t.x, -t.y);
        };
        if constexpr (CV) {
          // N_t, v = Lambda^-1 e_t, u = v z_t, W1 = z u^H + u z^H, W2 = 2 v v^H
          acc_norm += z[tcv].x * z[tcv].x + z[tcv].y * z[tcv].y;
          double2 v[kMtMaxT];
          for (int i = 0; i < T; ++i) {
            v[i] = inv_at(i, tcv);
            u[i] = cmul(v[i], z[tcv]);
          }
          for (int p = 0, k = 0; k < T; ++k)
            for (int l = k; l < T; ++l, ++p) {
              const double2 a1 = cmulc(z[l], u[k]), a2 = cmulc(u[l], z[k]);
              const double2 w1 = make_double2(a1.x + a2.x, a1.y + a2.y);
              const double2 vv = cmulc(v[l], v[k]);                    // v_l conj(v_k)
              const double2 w2 = make_double2(2.0 * vv.x, 2.0 * vv.y);
              wv[tid][p] = w1;
              A[p] = w2;
              if (k == l) {
                acc_noise += 0.5 * w1.x * kt[k * T + k];
                acc_noise2 += 0.5 * w2.x * kt[k * T + k];
              }
            }
        }
        for (int i = 0; i < T && !CV; ++i) {
          acc_norm += z[i].x * z[i].x + z[i].y * z[i].y;
          double2 s = z[i];
          for (int m = 0; m < i; ++m) {
            const double2 t = cmul(A[i * T + m], u[m]);
            s.x -= t.x;
            s.y -= t.y;
          }
          u[i] = s;
        }
        for (int i = 0; i < T && !CV; ++i) u[i] = make_double2(u[i].x / Dg[i], u[i].y / Dg[i]);
        for (int i = T - 1; i >= 0 && !CV; --i) {
          double2 s = u[i];
          for (int m = i + 1; m < T; ++m) {
            const double2 t = cmulc(u[m], A[m * T + i]);          // conj(L[m][i]) u[m]
            s.x -= t.x;
            s.y -= t.y;
          }
          u[i] = s;
        }
        for (int p = 0, k = 0; k < T && !CV; ++k)
          for (int l = k; l < T; ++l, ++p) {
            const double2 a1 = cmulc(z[l], u[k]), a2 = cmulc(u[l], z[k]);   // z_l conj(u_k) + u_l conj(z_k)
            const double2 w1 = make_double2(a1.x + a2.x, a1.y + a2.y);
            double2 w2 = make_double2(0.0, 0.0);
            for (int m = 0; m < T; ++m) {
              const double2 t = cmul(inv_at(l, m), inv_at(m, k));
              w2.x += t.x;
              w2.y += t.y;
            }
            w2 = make_double2(2.0 * w2.x, 2.0 * w2.y);
            wv[tid][p] = w1;
            A[p] = w2;
            if (k == l) {
              acc_noise += 0.5 * w1.x * kt[k * T + k];
              acc_noise2 += 0.5 * w2.x * kt[k * T + k];
            }
          }
      }
    }
    __syncthreads();
    // (3) gradient: c = w_kl sqrt(n) scale Kt[k, l] W[l, k]; r_S = l^S Re(c Phi^{kl}_S)
    for (int it = tid, slot = 0; it < NP * F; it += kWG, ++slot) {
      const int p = it / F, f = it - p * F;
      int k, l;
      mt_pair_kl(p, T, k, l);
      const double wkl = (k == l ? 0.5 : 1.0);
      const double wgt = wkl * sn * kt[k * T + l];
      const double2 w = wv[f][p];
      const double cx = wgt * w.x, cy = wgt * w.y;
      double c2x = 0.0, c2y = 0.0;
      double2 w2v = make_double2(0.0, 0.0);
      if constexpr (GCV) {
        const double2 w2 = blk[f][p];
        w2v = w2;
        c2x = wgt * w2.x;
        c2y = wgt * w2.y;
      }
      // (LEARN: the same products without K_task -- d Lambda / d K_task)
      const double ex = wkl * sn * w.x, ey = wkl * sn * w.y, e2x = wkl * sn * w2v.x, e2y = wkl * sn * w2v.y;
      double rk1 = 0.0, rk2 = 0.0;
      const int64_t base = (int64_t)p * NS * n + j0 + f;
      constexpr int U = NS < 8 ? NS : 8;
#pragma unroll 1
      for (int sh = 0; sh < NS; sh += U) {
#pragma unroll
        for (int t = 0; t < U; ++t) {
          const int S = sh + t;
          const double2 ph = mt_phi(a, base + (int64_t)S * n);
          const double r = ls_pow[S] * (cx * ph.x - cy * ph.y);
          acc_sc += r;
#pragma unroll
          for (int m = 0; m < D; ++m)
            if (m < 3 ? ((t >> m) & 1) : ((sh >> m) & 1)) acc_l[m] += r;
          if constexpr (GCV) {
            const double r2 = ls_pow[S] * (c2x * ph.x - c2y * ph.y);
            acc_sc2 += r2;
#pragma unroll
            for (int m = 0; m < D; ++m)
              if (m < 3 ? ((t >> m) & 1) : ((sh >> m) & 1)) acc_l2[m] += r2;
          }
          if constexpr (LEARN) {
            rk1 = __builtin_fma(ls_pow[S], ex * ph.x - ey * ph.y, rk1);
            rk2 = __builtin_fma(ls_pow[S], e2x * ph.x - e2y * ph.y, rk2);
          }
        }
      }
      if constexpr (LEARN) {
        if (k == l) {
          rk1 += 0.5 * h.noise * w.x;
          rk2 += 0.5 * h.noise * w2v.x;
        }
#pragma unroll
        for (int s2 = 0; s2 < kMtSlots; ++s2)
          if (s2 == slot) {
            kta[s2] += rk1;
            ktb[s2] += rk2;
          }
      }
    }
  }
  if constexpr (LEARN) {
    // the pairs' sums: slot s2 holds pairs kWG s2 / F .. (kWG s2 + kWG) / F - 1, F consecutive threads each
    __shared__ double pr[kWG];
    const int pc = kWG / F;
    for (int s2 = 0; s2 < kMtSlots && (kWG * s2) / F < NP; ++s2)
      for (int stream = 0; stream < 2; ++stream) {
        __syncthreads();
        double mine = 0.0;
#pragma unroll
        for (int u = 0; u < kMtSlots; ++u)
          if (u == s2) mine = stream ? ktb[u] : kta[u];
        pr[tid] = mine;
        __syncthreads();
        const int p = (kWG * s2) / F + tid;
        if (tid < pc && p < NP) {
          double sum = 0.0;
          for (int f2 = 0; f2 < F; ++f2) sum += pr[tid * F + f2];
          *part_ptr(a, CV ? tcv : 0, NQ + stream * NP + p, blockIdx.x) = sum;
        }
      }
  }
  double v[NQ];
  v[0] = acc_norm;
  v[1] = acc_ld;
  v[2] = acc_noise;
  v[3] = acc_sc;
#pragma unroll
  for (int m = 0; m < D; ++m) v[4 + m] = acc_l[m];
  if constexpr (GCV) {
    v[4 + D] = acc_noise2;
    v[5 + D] = acc_sc2;
#pragma unroll
    for (int m = 0; m < D; ++m) v[6 + D + m] = acc_l2[m];
  }
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const double s = block_sum(v[q], red);
    if (tid == 0) *part_ptr(a, CV ? tcv : 0, q, blockIdx.x) = s;
  }
  stamp_end(a);
}

// A = 1 / ev, ev = sqrt(n) lambda + noise (util.py:285,292-300) of every problem from the spectra
// (fgp_spec_inv_eig): the real eigenvalues' inverse, wa [G][n] float64 -- the factor of the coefficient
// solve (fgp_ifftbr_real_rf) and the post_var weights -- without materialising lambda.  Thread = frequency
// k <= K - 1 (lattice: k and its mirror n - k from one evaluation), looping over the problems sharing the
// spectra (one read of the 2^d values per frequency).
template <int D, bool NET>
__global__ __launch_bounds__(kWG) void k_spec_inv_eig(Nll a, double* __restrict__ wa) {
  constexpr int NS = 1 << D;
  const int64_t k = (int64_t)blockIdx.x * kWG + threadIdx.x;
  const int64_t n = (int64_t)1 << a.log2n;
  const double rootn = sqrt((double)n);
  const bool shared = a.basis_stride == 0;
  double phi[NS], dp[D];
  if (k < a.spec_K && shared) {
#pragma unroll
    for (int s = 0; s < NS; ++s) phi[s] = a.basis[spec_at<NS>(k, s)];
  }
  for (int g = 0; g < a.G; ++g) {
    Hyp h;
    load_hyp_wave(a, g, h);
    if (k >= a.spec_K) continue;
    if (!shared) {
      const double* phib = a.basis + (int64_t)g * a.basis_stride;
#pragma unroll
      for (int s = 0; s < NS; ++s) phi[s] = phib[spec_at<NS>(k, s)];
    }
    const double lam = h.scale * mlin<D>(phi, h.ls, dp);
    const double A = 1.0 / (rootn * lam + h.noise);
    double* w = wa + (int64_t)g * n;
    w[k] = A;
    if (!NET && k > 0 && k < n / 2) w[n - k] = A;
  }
}

// ---------------------------------------------------------------- posterior variance over many problems
// (fgp_spec_post_var, ABI 13).  G eigen-problems on ONE point set (per-output hyper-parameters, e.g. C5
// per-output) and N test points: the reference forms, per problem g and test point t, the kernel row
// r_gt[i] = K_g(x_t, x_i) and the quadratic form r^T K_g^-1 r = sum_k Re(A_gk) |ft(r_gt)_k|^2 (abstract_gp.py:
// 407-413, util.py:338-353; k_qf_* evaluate it by one transform per (g, t)).  The row is multilinear in the
// lengthscales, r_gt = scale_g sum_S l_g^S rho_S(t) with rho_S(t)[i] = prod_{j in S} part_j(x_t, x_i), so by
// linearity of ft
//     ft(r_gt)_k = scale_g sum_S l_g^S Psi_S(t, k),   Psi_S(t) = ft(rho_S(t))    (2^d N transforms, ONCE),
// and A_gk = 1 / (sqrt(n) scale_g sum_S l_g^S Phi_S(k) + noise_g) from the fit's part-product spectra
// (k_spec_inv_eig's arithmetic; 1 / ev by rcp_nr, within an ulp).  Real rows: |ft(r)_k| = |ft(r)_{n-k}| and A_k = A_{n-k}, so k <= n/2 with
// weights 2 (1 at k = 0, n/2).  Wave = (block of 64 kpl frequencies, kSpvPS problems); the 4 waves of a
// workgroup take consecutive problem slices of the same block (the Psi / Phi loads hit L1 / L2 three times
// in four); per (t, g) a lane sum over its frequencies, the fixed wave reduction, one partial per block:
// partial[(g N + t) nblk + blk] (k_qf_finish sums them in order and forms K(x,x) - sum).
constexpr int kSpvPS = 8;
template <int D>
__global__ __launch_bounds__(kWG) void k_spec_post_var(Nll a, const double2* __restrict__ psi, int N, int kpl,
                                                       int nblk, double* __restrict__ partial) {
  constexpr int NS = 1 << D, HS = 2 + D;
  __shared__ double hl[kWG / 64][kSpvPS][HS];          // scale, noise, l_j of the wave's problems
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int blk = (int)blockIdx.x;
  const int g0 = ((int)blockIdx.y * (kWG / 64) + w) * kSpvPS;
  if (g0 >= a.G) return;                              // wave-uniform; no barriers below
  const int cnt = min(kSpvPS, a.G - g0);
  for (int p = 0; p < cnt; ++p) {
    Hyp h;
    load_hyp_wave(a, g0 + p, h);
    if (lane == 0) {
      hl[w][p][0] = h.scale;
      hl[w][p][1] = h.noise;
#pragma unroll
      for (int j = 0; j < D; ++j) hl[w][p][2 + j] = h.ls[j];
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the wave's own LDS stores, read back by every lane
  const int64_t n = (int64_t)1 << a.log2n, half = n / 2;
  const double rootn = sqrt((double)n);
  double dp[D];
  for (int t = 0; t < N; ++t) {
    double acc[kSpvPS];
#pragma unroll
    for (int p = 0; p < kSpvPS; ++p) acc[p] = 0.0;
    // software-pipelined: the next frequency's spectra are in flight while this one is evaluated
    double phn[NS], prn[NS], pin[NS];
    auto fetch = [&](int64_t k) {
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        phn[s] = a.basis[spec_at<NS>(k, s)];
        const double2 v = psi[((int64_t)t * NS + s) * n + k];
        prn[s] = v.x;
        pin[s] = v.y;
      }
    };
    const int64_t k0 = (int64_t)blk * kpl * 64 + lane;
    if (k0 <= half) fetch(k0);
    for (int i = 0; i < kpl; ++i) {
      const int64_t k = k0 + 64 * i;
      if (k > half) break;
      double phi[NS], pr[NS], pi[NS];
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        phi[s] = phn[s];
        pr[s] = prn[s];
        pi[s] = pin[s];
      }
      if (i + 1 < kpl && k + 64 <= half) fetch(k + 64);
      const double wk = (k == 0 || k == half) ? 1.0 : 2.0;
#pragma unroll
      for (int p = 0; p < kSpvPS; ++p) {
        if (p < cnt) {
          double l[D];
#pragma unroll
          for (int j = 0; j < D; ++j) l[j] = hl[w][p][2 + j];
          const double sc = hl[w][p][0];
          const double A = rcp_nr(rootn * (sc * mlin<D>(phi, l, dp)) + hl[w][p][1]);
          const double re = mlin<D>(pr, l, dp), im = mlin<D>(pi, l, dp);
          acc[p] = __builtin_fma(wk * A * (sc * sc), __builtin_fma(re, re, im * im), acc[p]);
        }
      }
    }
#pragma unroll
    for (int p = 0; p < kSpvPS; ++p) {
      double v = acc[p];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
      if (lane == 0 && p < cnt) partial[((int64_t)(g0 + p) * N + t) * nblk + blk] = v;
    }
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
void spec_geometry(Nll& a, bool allow_tile) {
  const int64_t n = (int64_t)1 << a.log2n;
  const bool net = a.spec_net;
  a.spec_main = net ? n : n / 2;
  a.spec_K = net ? n : n / 2 + 1;
  a.spec_KS = spec_chunks(net, a.log2n) * 64;
  // problems per wave sharing one read of the spectra: 2 (the tile kernel's, G <= 8), and for many
  // problems (k_spec_iter, e.g. per-output hyper-parameters) 4 -- the spectra are then re-read from L2
  // G / 4 times instead of G / 2 and each wave's loads serve 4 evaluations.  d <= 3 only: 156 VGPRs,
  // 3 waves / SIMD there; at d = 4, 5 the four accumulator sets spill (8 per wave spills at d = 3)
  const int64_t lanes = std::max<int64_t>(1, a.spec_main / 64);
  // at least 4 chunks per block where the frequencies allow (>= 4 blocks): a block's epilogue (wave reduction of
  // 4 + d partials, the corrections) costs ~1 us of latency, so small problems (C2 / C3, the paper's n = 2^10,
  // whose single-launch fit runs one block per wave) no longer pay it per 64 frequencies; n >= 2^18 unchanged
  // (fewer chunks per block where a 4-chunk block of 2^d + 1 rows would not fit the single-launch fit's LDS:
  // d = 6 takes 2)
  int64_t minc = 4;
  while (minc > 1 && ((((int64_t)1 << a.d) + 1) * minc * 512 > 96 * 1024)) minc /= 2;
  a.nb = (int)std::min<int64_t>(kSpecBlocks, std::max<int64_t>(std::min<int64_t>(lanes, 4), lanes / minc));
  a.spec_kpl = (int)((a.spec_main + 64 * (int64_t)a.nb - 1) / (64 * (int64_t)a.nb));
  a.spec_tile = 0;
  a.spec_pgp = a.spec_ck = 0;
  a.spec_kw = 0;
  a.spec_ps = 0;
  a.spec_nsl = 1;
  const char* te = getenv("FGP_SPEC_TILE");   // 0: the per-wave kernel only (A/B experiments)
  const bool tile_ok = allow_tile && !(te && te[0] == '0');
  // Tile kernel (one shared set of spectra, d <= 5): 2 problems per wave (1 for G = 1), problem groups
  // PG <= 4 in the 4 waves of a workgroup.  (4 problems per wave at G = 8 -- 233 VGPRs, 2 blocks per
  // workgroup, 1024 blocks -- measured slower: 51.7 vs 42.0 us per C4 iteration, profiles/r03x_*.)
  if (tile_ok && a.basis_stride == 0 && a.d <= 5 && a.spec_main >= 256) {
    const int ppw = a.G >= 2 ? 2 : 1;
    const int pg = (a.G + ppw - 1) / ppw;
    const int pgp = pg <= 1 ? 1 : (pg <= 2 ? 2 : 4);
    const int ck = 64 * (4 / pgp);   // frequencies per chunk (64 per block of the workgroup)
    // the ring <= kSpecLdsMax (two workgroups per CU), whole 1-KiB wave-instructions, <= kSpecMaxDma per wave
    const int rows = (1 << a.d) + a.G;
    if (pg <= 4 && rows * ck * 8 * kSpecRing <= kSpecLdsMax && rows * ck <= 512 * kSpecMaxDma &&
        (rows * ck) % 128 == 0 && rows * ck >= kSpecScratch && a.nb % (4 / pgp) == 0 &&
        a.spec_main % (64 * (int64_t)a.nb) == 0) {
      a.spec_tile = 1;
      a.spec_ppw = ppw;
      a.spec_pg = pg;
      a.spec_pgp = pgp;
      a.spec_ck = ck;
      a.spec_kw = (int64_t)(4 / pgp) * 64 * a.spec_kpl;
      return;
    }
    // many problems (G > 8, e.g. per-output hyper-parameters): slices of PS = 4 PPW problems (PPW = 4 at
    // d <= 3, else 2), one slot per wave, one k block per workgroup -- every slice streams its own Y rows
    // and re-reads the shared spectra (from L2: the slices of a block run on consecutive workgroups)
    const int sppw = a.d <= 3 ? 4 : 2, ps = 4 * sppw, srows = (1 << a.d) + ps;
    // k blocks: 64 chunks per workgroup (with 4, the per-wave kernel's 512 blocks at n = 2^18, the
    // workgroups spend their life in the prologue: 383 vs 153 us per C5 per-output iteration; a 4-deep ring
    // does not pay, profiles/r03sl_exp_slices.jsonl), more blocks while the grid has fewer than 512
    // workgroups; FGP_SPEC_SLICE_NB overrides (A/B experiments)
    const int nsl = (a.G + ps - 1) / ps;
    int64_t snb = std::max<int64_t>(1, a.spec_main / (64 * 64));
    while (snb * nsl < 512 && snb * 2 <= lanes) snb *= 2;
    snb = std::min<int64_t>(snb, a.nb);
    const char* se = getenv("FGP_SPEC_SLICE_NB");
    if (se) snb = std::max(1, std::min(a.nb, atoi(se)));
    if (pg > 4 && srows * 64 * 8 * kSpecRing <= kSpecLdsMax && srows * 64 <= 512 * kSpecMaxDma &&
        (srows * 64) % 128 == 0 && srows * 64 >= kSpecScratch && a.spec_main % (64 * snb) == 0) {
      a.nb = (int)snb;
      a.spec_kpl = (int)(a.spec_main / (64 * snb));
      a.spec_tile = 1;
      a.spec_ppw = sppw;
      a.spec_pg = 4;
      a.spec_pgp = 4;
      a.spec_ck = 64;
      a.spec_kw = 64 * a.spec_kpl;
      a.spec_ps = ps;
      a.spec_nsl = nsl;
      return;
    }
  }
  // per-wave kernel k_spec_iter: problems per wave sharing one read of the spectra, 2, and for many
  // problems (e.g. per-output hyper-parameters) 4 -- the spectra are then re-read from L2 G / 4 times
  // instead of G / 2 and each wave's loads serve 4 evaluations.  d <= 3 only: 156 VGPRs, 3 waves / SIMD
  // there; at d = 4, 5 the four accumulator sets spill (8 per wave spills at d = 3)
  a.spec_ppw = (a.G >= 2 && a.basis_stride == 0 && a.d <= 5) ? 2 : 1;
  if (a.spec_ppw == 2 && a.G > 8 && a.d <= 3) a.spec_ppw = 4;
  a.spec_pg = (a.G + a.spec_ppw - 1) / a.spec_ppw;
}

int launch_spec_loss_iter(const Nll& a, hipStream_t st) {
  const int64_t tasks = (int64_t)a.nb * a.G;
  const unsigned grid = (unsigned)((tasks + kWG / 64 - 1) / (kWG / 64));
  return with_spec_d(a.d, [&](auto dc) {
    constexpr int D = decltype(dc)::value;
    auto go = [&](auto net, auto cv) {
      k_spec_loss_iter<D, decltype(net)::value, decltype(cv)::value><<<grid, kWG, 0, st>>>(a);
    };
    if (a.spec_net) {
      if (a.loss == FGP_LOSS_CV) go(std::true_type{}, std::true_type{});
      else go(std::true_type{}, std::false_type{});
    } else {
      if (a.loss == FGP_LOSS_CV) go(std::false_type{}, std::true_type{});
      else go(std::false_type{}, std::false_type{});
    }
    return check_launch("k_spec_loss_iter");
  });
}

int launch_spec_loss_step(const Nll& a, const Fit& f, int iter, int do_update, hipStream_t st) {
  if (a.mt > 0 && a.loss == FGP_LOSS_CV) {
    // multitask CV: the T tasks' partials as T problems of ONE loss (k_mt_spec_iter<D, true, true>)
    Nll b = a;
    b.G = a.mt;
    Fit g = f;
    g.per_problem = 0;
    return with_spec_d(a.d, [&](auto dc) {
      k_spec_loss_step<decltype(dc)::value><<<1, kWG, 0, st>>>(b, g, iter, do_update);
      return check_launch("k_spec_loss_step");
    });
  }
  if (!f.per_problem && a.G > 16) return set_error(kErrUnsupported, "GCV / CV fits: one loss over at most 16 problems");
  if (a.nb > kSpecBlocks) return set_error(kErrInvalid, "k_spec_loss_step: nb > %d", kSpecBlocks);
  return with_spec_d(a.d, [&](auto dc) {
    k_spec_loss_step<decltype(dc)::value><<<(unsigned)((a.G + 15) / 16), kWG, 0, st>>>(a, f, iter, do_update);
    return check_launch("k_spec_loss_step");
  });
}

int launch_mt_learn_step(const Nll& a, const Fit& f, int iter, int do_update, hipStream_t st) {
  if (a.mt > kMtMaxT || a.nb > kSpecBlocks || spec_nparams(a) > kSpecScratch)
    return set_error(kErrInvalid, "k_mt_learn_step: shape");
  return with_spec_d(a.d, [&](auto dc) {
    k_mt_learn_step<decltype(dc)::value><<<1, kWG, 0, st>>>(a, f, iter, do_update);
    return check_launch("k_mt_learn_step");
  });
}

int64_t spec_chunks(bool net, int log2n) {
  const int64_t n = (int64_t)1 << log2n, K = net ? n : n / 2 + 1;
  return (K + 63) / 64;
}

int launch_spec_iter(const Nll& a, hipStream_t st, const FitFuse* fz) {
  if (a.loss != FGP_LOSS_MLL) {
    if (fz) return set_error(kErrUnsupported, "GCV / CV fits: no fused spectral step");
    return launch_spec_loss_iter(a, st);
  }
  if (a.spec_tile) {
    if (a.spec_ppw > 4) return set_error(kErrInvalid, "spectral tile kernel: %d problems per wave", a.spec_ppw);
    if (fz && a.spec_ps) return set_error(kErrInvalid, "spectral tile kernel: no fused step over problem slices");
    FitFuse none{};
    none.counters = nullptr;
    const FitFuse& f = fz ? *fz : none;
    bool persist_ok = false;
    const int trows = (1 << a.d) + (a.spec_ps ? a.spec_ps : a.G);
#ifdef FGP_SPEC_SHM_MIN
    // (experiment build: at least this much dynamic LDS per workgroup -- fewer co-resident workgroups per CU)
    const size_t shm = std::max(sizeof(double) * (size_t)kSpecRing * (size_t)(trows * a.spec_ck), (size_t)FGP_SPEC_SHM_MIN);
#else
    const size_t shm = sizeof(double) * (size_t)kSpecRing * (size_t)(trows * a.spec_ck);
#endif
    const unsigned grid = (unsigned)(a.nb / (4 / a.spec_pgp) * a.spec_nsl);
    return with_spec_d(a.d, [&](auto dc) {
      constexpr int D = decltype(dc)::value;
      if constexpr (D <= 5) {
        auto go = [&](auto kern) {
          // the ring may exceed the 64 KB default of dynamic LDS: raise each kernel's limit once (one
          // static for every kernel of this lambda's type: remember which ones)
          static const void* raised[64];
          static int nraised = 0;
          const void* kp = reinterpret_cast<const void*>(kern);
          bool done = false;
          for (int i = 0; i < nraised; ++i) done = done || raised[i] == kp;
          if (!done) {
            (void)hipFuncSetAttribute(kp, hipFuncAttributeMaxDynamicSharedMemorySize, kSpecLdsMax);
            if (nraised < 64) raised[nraised++] = kp;
          }
          if (f.piters > 0) {
            // persistent: every workgroup must be resident at once (they wait on each other).  The residency
            // (workgroups per CU x CUs) is queried once per kernel and LDS size and remembered, so a launch
            // inside a hipGraph capture makes no query.
            static const void* rk[64];
            static size_t rshm[64];
            static int64_t rres[64];
            static int nr = 0;
            int64_t resident = -1;
            for (int i = 0; i < nr; ++i)
              if (rk[i] == kp && rshm[i] == shm) resident = rres[i];
            if (resident < 0) {
              int per_cu = 0, dev = 0, cus = 0;
              resident = (hipGetDevice(&dev) == hipSuccess &&
                          hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
                          hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kp, kWG, shm) == hipSuccess)
                             ? (int64_t)per_cu * cus : 0;
              if (nr < 64) {
                rk[nr] = kp;
                rshm[nr] = shm;
                rres[nr++] = resident;
              }
            }
            if (resident < (int64_t)grid) return;    // (rc stays kErrUnsupported: the caller launches per iteration)
            persist_ok = true;
          }
          kern<<<grid, kWG, shm, st>>>(a, f);
        };
        auto net = [&](auto nc) {
          constexpr bool NET = decltype(nc)::value;
          if (f.piters > 0) {
            if (a.spec_ppw == 2) go(k_spec_tile<D, 2, NET, true>);
            else if (a.spec_ppw == 1) go(k_spec_tile<D, 1, NET, true>);
          } else if (a.spec_ppw == 4) go(k_spec_tile<D, 4, NET>);
          else if (a.spec_ppw == 2) go(k_spec_tile<D, 2, NET>);
          else go(k_spec_tile<D, 1, NET>);
        };
        if (a.spec_net) net(std::true_type{});
        else net(std::false_type{});
        if (f.piters > 0 && !persist_ok)
          return set_error(kErrUnsupported, "persistent k_spec_tile: the grid is not co-resident");
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
    auto go = [&](auto net) {
      constexpr bool NET = decltype(net)::value;
      switch (a.spec_ppw) {
        case 4: if constexpr (D <= 3) { k_spec_iter<D, 4, NET><<<grid, kWG, 0, st>>>(a); break; } [[fallthrough]];
        case 2: k_spec_iter<D, 2, NET><<<grid, kWG, 0, st>>>(a); break;
        default: k_spec_iter<D, 1, NET><<<grid, kWG, 0, st>>>(a); break;
      }
    };
    if (a.spec_net) go(std::true_type{});
    else go(std::false_type{});
    return check_launch("k_spec_iter");
  });
}

int launch_mt_spec_iter(const Nll& a, hipStream_t st) {
  return with_spec_d(a.d, [&](auto dc) {
    constexpr int DD = decltype(dc)::value;
    if (a.loss == FGP_LOSS_CV && a.mt_learn) k_mt_spec_iter<DD, true, true, true><<<dim3((unsigned)a.nb, (unsigned)a.mt), kWG, 0, st>>>(a);
    else if (a.loss == FGP_LOSS_CV) k_mt_spec_iter<DD, true, true><<<dim3((unsigned)a.nb, (unsigned)a.mt), kWG, 0, st>>>(a);
    else if (a.loss == FGP_LOSS_GCV && a.mt_learn) k_mt_spec_iter<DD, true, false, true><<<(unsigned)a.nb, kWG, 0, st>>>(a);
    else if (a.loss == FGP_LOSS_GCV) k_mt_spec_iter<DD, true><<<(unsigned)a.nb, kWG, 0, st>>>(a);
    else k_mt_spec_iter<decltype(dc)::value><<<(unsigned)a.nb, kWG, 0, st>>>(a);
    return check_launch("k_mt_spec_iter");
  });
}

int launch_spec_reduce_step(const Nll& a, const Fit& f, int iter, int do_update, hipStream_t st) {
  return with_spec_d(a.d, [&](auto dc) {
    k_spec_reduce_step<decltype(dc)::value><<<(unsigned)((a.G + 15) / 16), kWG, 0, st>>>(a, f, iter, do_update);
    return check_launch("k_spec_reduce_step");
  });
}

// The k_spec_persist instance of a desc (D, NET), for the residency query.
static const void* spec_persist_kernel(const Nll& a) {
  const void* kp = nullptr;
  (void)with_spec_d(a.d, [&](auto dc) {
    constexpr int D = decltype(dc)::value;
    kp = a.spec_net ? reinterpret_cast<const void*>(k_spec_persist<D, true>)
                    : reinterpret_cast<const void*>(k_spec_persist<D, false>);
    return kOk;
  });
  return kp;
}

// Workgroups of `kp` at `shm` bytes of dynamic LDS that can be resident at once on the current device
// (workgroups per CU x CUs), queried once per (kernel, LDS size) and remembered -- so a launch inside a hipGraph
// capture makes no query.  0 when the query fails.
static int64_t persist_resident(const void* kp, size_t shm) {
  // keyed by the device too: devices of one process may differ in CU count / partition mode
  static const void* rk[64];
  static size_t rshm[64];
  static int rdev[64];
  static int64_t rres[64];
  static int nr = 0;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  for (int i = 0; i < nr; ++i)
    if (rk[i] == kp && rshm[i] == shm && rdev[i] == dev) return rres[i];
  (void)hipFuncSetAttribute(kp, hipFuncAttributeMaxDynamicSharedMemorySize, kPersistLdsMax);
  int per_cu = 0, cus = 0;
  const int64_t resident = (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
                            hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kp, kWG, shm) == hipSuccess)
                               ? (int64_t)per_cu * cus : 0;
  if (nr < 64) {
    rk[nr] = kp;
    rshm[nr] = shm;
    rdev[nr] = dev;
    rres[nr++] = resident;
  }
  return resident;
}

// Test hook (fgp_set_persist_poll_max): the bound of k_spec_persist's barrier polls (default 2^22), in device memory.
void set_persist_poll_max(long long v) {
  const long long pm = v < 0 ? kPersistPollMax : v;
  (void)hipDeviceSynchronize();
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_persist_poll_max_dev), &pm, sizeof(pm), 0, hipMemcpyHostToDevice);
}

int spec_persist_geometry(const Nll& a, int* W, int* bpw, size_t* shm) {
  if (!a.spec || a.G != 1 || a.basis_stride != 0 || a.d > kSpecMaxD || !a.ysq_chunked || a.loss != FGP_LOSS_MLL)
    return set_error(kErrUnsupported, "fgp_fit_persist: one problem on the spectral path only");
  if (spec_nparams(a) > kSpecScratch) return set_error(kErrUnsupported, "fgp_fit_persist: parameters");
  const size_t per_blk = (size_t)a.spec_kpl * (((size_t)1 << a.d) + 1) * 64 * sizeof(double);
  // (the fewest workgroups whose LDS holds the spectra: more of them -- 64, 128, 256 at C2 / C3 -- did not shorten the
  // fit, profiles/r06f_persist_wg_sweep.jsonl: the iteration is bound by its barrier / reduce / step chain)
  for (int w = 1; w <= kPersistMaxW && w <= a.nb; w *= 2) {
    const int b = (a.nb + w - 1) / w;
    if ((size_t)b * per_blk <= (size_t)kPersistLdsMax) {
      // the workgroups wait on each other at the in-kernel grid barrier: all W must be resident at once
      // (a partitioned device, or CUs held by other work, would otherwise turn every barrier into a give-up)
      if (w > 1 && persist_resident(spec_persist_kernel(a), (size_t)b * per_blk) < (int64_t)w)
        return set_error(kErrUnsupported, "fgp_fit_persist: %d workgroups are not co-resident", w);
      *W = w;
      *bpw = b;
      *shm = (size_t)b * per_blk;
      return kOk;
    }
  }
  return set_error(kErrUnsupported, "fgp_fit_persist: the spectra do not fit %d workgroups' LDS", kPersistMaxW);
}

int persist_giveups(unsigned long long* count, int reset) {
  if (hipDeviceSynchronize() != hipSuccess ||
      hipMemcpyFromSymbol(count, HIP_SYMBOL(g_persist_giveups), sizeof(unsigned long long), 0,
                          hipMemcpyDeviceToHost) != hipSuccess)
    return set_error(kErrHip, "fgp_persist_giveups: read failed");
  if (reset) {
    const unsigned long long z = 0;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_persist_giveups), &z, sizeof(z), 0, hipMemcpyHostToDevice) != hipSuccess)
      return set_error(kErrHip, "fgp_persist_giveups: reset failed");
  }
  return kOk;
}

int launch_spec_persist(const Nll& a, const Fit& f, int iters, double logtol, int wait_max, unsigned* counter, int* out,
                        hipStream_t st) {
  int W, bpw;
  size_t shm;
  int rc = spec_persist_geometry(a, &W, &bpw, &shm);
  if (rc != kOk) return rc;
  // the three partial buffers empty (kPartEmpty: all bytes 0xff), the control words out[0..2] cleared
  (void)counter;
  if (hipMemsetAsync(a.partials, 0xff, 3 * sizeof(double) * (size_t)a.nq * (size_t)a.nb, st) != hipSuccess ||
      hipMemsetAsync(out, 0, 3 * sizeof(int), st) != hipSuccess)
    return set_error(kErrHip, "fgp_fit_persist: workspace reset failed");
  return with_spec_d(a.d, [&](auto dc) {
    constexpr int D = decltype(dc)::value;
    auto go = [&](auto kern) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                kPersistLdsMax);
      kern<<<(unsigned)W, kWG, shm, st>>>(a, f, iters, logtol, wait_max, bpw, counter, out);
    };
    if (a.spec_net) go(k_spec_persist<D, true>);
    else go(k_spec_persist<D, false>);
    return check_launch("k_spec_persist");
  });
}

unsigned* spec_step_many_counter(const Nll& a) {
  const int64_t nb_doc = std::max<int64_t>(1, ((int64_t)1 << a.log2n) >> 12);
  return reinterpret_cast<unsigned*>(a.partials + (int64_t)a.G * a.nq * (std::max<int64_t>(a.nb, nb_doc) + 1));
}

int launch_spec_step_many(const Nll& a, const Fit& f, int iter, int do_update, hipStream_t st) {
  if (a.nb > kSpecBlocks) return set_error(kErrInvalid, "k_spec_step_many: nb > %d", kSpecBlocks);
  unsigned* counter = spec_step_many_counter(a);
  return with_spec_d(a.d, [&](auto dc) {
    k_spec_step_many<decltype(dc)::value><<<(unsigned)((a.G + 15) / 16), kWG, 0, st>>>(a, f, iter, do_update, counter);
    return check_launch("k_spec_step_many");
  });
}

int spec_counters_offset(const Nll& a, int64_t* off, int* count) {
  const int ng = (a.nb + kSpecGroup - 1) / kSpecGroup;
  *off = spec_part2_off(a, 2) + 2 * 3 * (int64_t)spec_nparams(a);
  *count = ng + 2;                                  // group counters, published-sums count, persistent fail word
  return kOk;
}

RpState spec_scratch_state(const Nll& a, int par) { return spec_state(a, par); }

int launch_spec_finish_step(const Nll& a, const FitFuse& fz, hipStream_t st) {
  return with_spec_d(a.d, [&](auto dc) {
    k_spec_finish_step<decltype(dc)::value><<<1, kWG, 0, st>>>(a, fz);
    return check_launch("k_spec_finish_step");
  });
}

// out[g, t] = K_g(x_t, x_t) - sum_b partial[(g N + t) nblk + b] (ascending b), negatives set to 0
// (abstract_gp.py:407-413; K(x, x) = scale prod_j (1 + l_j part0_j), k_qf_finish's arithmetic)
struct Part0 {
  double v[FGP_MAX_D];
};
__global__ __launch_bounds__(kWG) void k_spec_post_var_finish(Nll a, const double* __restrict__ partial, int N, int nblk,
                                                              Part0 p0, double* __restrict__ out) {
  const int e = (int)blockIdx.x * kWG + threadIdx.x, g = e / max(N, 1);
  if (e >= a.G * N) return;
  Hyp h;
  load_hyp(a, g, h);
  double s = 0.0;
  for (int b = 0; b < nblk; ++b) s += partial[(int64_t)e * nblk + b];
  double pr = 1.0;
  for (int j = 0; j < a.d; ++j) pr *= 1.0 + h.ls[j] * p0.v[j];
  const double v = h.scale * pr - s;
  out[e] = v < 0.0 ? 0.0 : v;
}

int launch_spec_post_var(const Nll& a, const double2* psi, int N, const double* part0, double* out, double* partial,
                         int nblk, int kpl, hipStream_t st) {
  const dim3 grid((unsigned)nblk, (unsigned)((a.G + kSpvPS * (kWG / 64) - 1) / (kSpvPS * (kWG / 64))));
  return with_spec_d(a.d, [&](auto dc) {
    constexpr int D = decltype(dc)::value;
    if constexpr (D <= 4) {
      k_spec_post_var<D><<<grid, kWG, 0, st>>>(a, psi, N, kpl, nblk, partial);
      int rc = check_launch("k_spec_post_var");
      if (rc != kOk) return rc;
      Part0 p0{};
      for (int j = 0; j < a.d && j < FGP_MAX_D; ++j) p0.v[j] = part0[j];
      k_spec_post_var_finish<<<(unsigned)(((int64_t)a.G * N + kWG - 1) / kWG), kWG, 0, st>>>(a, partial, N, nblk, p0, out);
      return check_launch("k_spec_post_var_finish");
    } else {
      return set_error(kErrInvalid, "fgp_spec_post_var: d <= 4");
    }
  });
}

int launch_spec_inv_eig(const Nll& a, double* wa, hipStream_t st) {
  const unsigned grid = (unsigned)((a.spec_K + kWG - 1) / kWG);
  return with_spec_d(a.d, [&](auto dc) {
    constexpr int D = decltype(dc)::value;
    if (a.spec_net) k_spec_inv_eig<D, true><<<grid, kWG, 0, st>>>(a, wa);
    else k_spec_inv_eig<D, false><<<grid, kWG, 0, st>>>(a, wa);
    return check_launch("k_spec_inv_eig");
  });
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

// spectra of the subsets s0 .. s0 + cnt - 1 into the chunked layout (spec_at): Re of a complex [cnt][n]
// spectrum (lattice: the even spectrum's independent half, k < K), or a real [cnt][n] one (net); zeros
// past K.  Thread = (chunk, subset, frequency within the chunk): 512-byte runs on both sides.
template <bool CX>
__global__ __launch_bounds__(kWG) void k_spec_extract(const void* __restrict__ spec, int64_t n, int64_t K, int64_t qs,
                                                      int ns, int s0, int cnt, double* __restrict__ basis) {
  const int64_t t = (int64_t)blockIdx.x * kWG + threadIdx.x;
  const int64_t e = t & 63, rest = t >> 6;
  const int c = (int)(rest % cnt);
  const int64_t q = rest / cnt, k = q * 64 + e;
  if (q >= qs) return;
  double v = 0.0;
  if (k < K) v = CX ? static_cast<const double2*>(spec)[(int64_t)c * n + k].x : static_cast<const double*>(spec)[(int64_t)c * n + k];
  basis[(q * ns + s0 + c) * 64 + e] = v;
}

static int64_t spec_subset_bytes(int family, int log2n) {
  const int64_t n = (int64_t)1 << log2n;
  if (family == FGP_FAMILY_NET) return 8 * n + 8 * n;         // products + their fwht
  if (log2n >= 17) return 16 * n;                              // the fused R2C pair's intermediate (spec_basis_r2c)
  return 8 * n + 16 * n;                                       // products + spectrum
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
  const int64_t K = net ? n : n / 2 + 1, QS = spec_chunks(net, log2n);
  const int NS = 1 << d;
  const int64_t per = spec_subset_bytes(family, log2n);
  const int chunk = (int)std::min<int64_t>(NS, work_bytes / per);
  if (chunk < 1) return set_error(kErrInvalid, "fgp_spec_basis: work below one subset (%lld bytes)", (long long)per);
  hipStream_t st = (hipStream_t)stream;
  char* wb = static_cast<char*>(work);
  double* prod = reinterpret_cast<double*>(wb);
  double2* spec = reinterpret_cast<double2*>(wb + 8 * n * (int64_t)chunk);
  const unsigned gi = (unsigned)((n + kWG - 1) / kWG);
  for (int64_t p = 0; p < P; ++p) {
    const double* pp = parts + p * parts_stride;
    double* bp = basis + p * QS * NS * 64;
    for (int s0 = 0; s0 < NS; s0 += chunk) {
      const int cnt = std::min(chunk, NS - s0);
      if (!net && log2n >= 17) {   // products in the row kernel, real parts k <= n/2 from the column kernel
        const int rc = spec_basis_r2c(pp, d, log2n, s0, cnt, bp, work, st);
        if (rc != kOk) return rc;
        continue;
      }
      int rc = with_spec_d(d, [&](auto dc) {
        k_spec_products<decltype(dc)::value><<<gi, kWG, 0, st>>>(pp, n, s0, cnt, prod);
        return check_launch("k_spec_products");
      });
      if (rc != kOk) return rc;
      const unsigned ge = (unsigned)((QS * 64 * cnt + kWG - 1) / kWG);
      if (net) {
        double* wht = reinterpret_cast<double*>(spec);
        rc = fgp_fwht(prod, n, wht, cnt, log2n, 1, stream);
        if (rc == kOk) {
          k_spec_extract<false><<<ge, kWG, 0, st>>>(wht, n, K, QS, NS, s0, cnt, bp);
          rc = check_launch("k_spec_extract");
        }
      } else {
        rc = fgp_fftbr(prod, n, 1, spec, cnt, log2n, 1, stream);
        if (rc == kOk) {
          k_spec_extract<true><<<ge, kWG, 0, st>>>(spec, n, K, QS, NS, s0, cnt, bp);
          rc = check_launch("k_spec_extract");
        }
      }
      if (rc != kOk) return rc;
    }
  }
  return kOk;
}

}  // extern "C"
