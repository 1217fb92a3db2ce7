// Real-even (RE) lattice fit kernels, n >= 2^17 (the default fused-fit path for regenerated lattice
// parts): see the section comment below and DESIGN.md section 3.
#include <cstdlib>

#include "fgp_nll.h"

namespace fgp {

// ---------------------------------------------------------------- real-even (RE) lattice fit, n >= 2^17
// The lattice k1 (natural index nu, c_nu = scale prod_j (1 + l_j B(nu z_j mod n / n))) is real and EVEN,
// c_nu = c_{n - nu} (B_{2 alpha}(1 - x) = B_{2 alpha}(x)), so lambda = DFT_n(c) / sqrt(n) is real and
// even: only c_0 .. c_{n/2} and lambda_0 .. lambda_{n/2} carry information.  One decimation-in-frequency
// stage packs the length-n transform into a length-M = n/2 complex one whose output needs no split:
//   z_i = a_i + i b_i w_n^i,  a_i = c_i + c_{i+M},  b_i = c_i - c_{i+M}   (i < M; c_{i+M} = c_{M-i})
//   Z = DFT_M(z):  Z_k = C_{2k} + i C_{2k+1}     (C = DFT_n(c); both parts real)
// and z_{M-i} = a_i + i b_i conj(w_n^i): the elements i and M - i come from the same two values
// (c_i, c_{M-i}), so each is generated ONCE (half the kernel-part work of the R2C path).
// The two-pass split M = N1 x N2 (N2 = 1024, rows = natural classes r = i mod N1, as the engine's
// bit-reversed storage rows u = brev(r)) puts element i and its mirror M - i in rows r and N1 - r
// (positions 16q + e and 16(63 - q) + 15 - e).  A row is ONE wavefront (64 threads x 16 elements, its
// sums are shuffles); a 128-thread workgroup takes the row pair, wave 0 row r, wave 1 row N1 - r, and
// the rows 0 / N1/2 (self-mirrored classes) share workgroup 0.  Barriers therefore span two waves.
// Output symmetry: C_{2k} = C_{n-2k} and C_{2k+1} = C_{n-2k-1}, i.e. column k1 of Z mirrors column
// N2 - k1 (real parts) and N2 - 1 - k1 (imaginary parts).  Columns [0, N2/2) therefore hold every
// imaginary part (weight 2) and every real part except those of column N2/2 (weight 2; column 0's
// real parts mirror inside the column, weight 1).  Column N2/2 contributes real parts only, whose
// N1/2 distinct values (mirror k2 <-> N1 - 1 - k2) are direct sums over its N1 rows, four per column
// workgroup.  The loss is this folded sum; its gradient along real-even c (the only direction c moves)
// is the true one, so the adjoint runs over the same half: V = dL/dC_{2k} + i dL/dC_{2k+1} on columns
// [0, N2/2), zero elsewhere, the Nyquist column's V by direct sums in the row kernel.  Per iteration:
// rows write n/4 complex (4n B), columns read 4n + Y 4n and write 4n, rows read 4n: 20n bytes
// (R2C 40n), and half the eigenvalue terms and kernel parts.
constexpr int kP2reDefault = 11;             // row length 2^P2 of the n/2-point transform
// unroll factor of the column kernel's eigen-term loop
#ifndef FGP_RE_EIG_UNROLL
#define FGP_RE_EIG_UNROLL 2
#endif

// v * exp(-2 pi i J / 32), J < 32 compile-time
template <int J>
__device__ __forceinline__ double2 mul_root32(double2 v) {
  if constexpr ((J & 1) == 0) {
    return mul_root<16, J / 2, false>(v);
  } else {
    constexpr double c32[32] = {1.0, 0.98078528040323044913, 0.92387953251128673848, 0.83146961230254523708,
                                0.70710678118654752440, 0.55557023301960222474, 0.38268343236508978178,
                                0.19509032201612826785, 0.0, -0.19509032201612826785, -0.38268343236508978178,
                                -0.55557023301960222474, -0.70710678118654752440, -0.83146961230254523708,
                                -0.92387953251128673848, -0.98078528040323044913, -1.0, -0.98078528040323044913,
                                -0.92387953251128673848, -0.83146961230254523708, -0.70710678118654752440,
                                -0.55557023301960222474, -0.38268343236508978178, -0.19509032201612826785, 0.0,
                                0.19509032201612826785, 0.38268343236508978178, 0.55557023301960222474,
                                0.70710678118654752440, 0.83146961230254523708, 0.92387953251128673848,
                                0.98078528040323044913};
    constexpr double cr = c32[J & 31], ci = c32[(J + 8) & 31];   // exp(-i t) = (cos t, cos(t + pi/2))
    return make_double2(__builtin_fma(cr, v.x, -(ci * v.y)), __builtin_fma(cr, v.y, ci * v.x));
  }
}

// c at natural index t (t <= n/2): the generated lattice k1
template <int PG, int D>
__device__ __forceinline__ double k1_nat(const Nll& a, const Hyp& h, unsigned t, unsigned mask, double inv_n) {
  double r = 1.0;
#pragma unroll
  for (int j = 0; j < D; ++j) r *= __builtin_fma(h.ls[j], lattice_gen_part<PG>(a.gz[j], t, mask, inv_n), 1.0);
  return h.scale * r;
}

// Bernoulli polynomial B_ORD as a polynomial in u = x (x - 1) (the forms of fgp_common.h bernoulli())
template <int ORD>
__device__ __forceinline__ double bern_u(double u) {
  if constexpr (ORD == 2) return u + 1.0 / 6.0;
  else if constexpr (ORD == 4) return __builtin_fma(u, u, -1.0 / 30.0);
  else if constexpr (ORD == 6) return __builtin_fma(u * u, u - 0.5, 1.0 / 42.0);
  else return __builtin_fma(u * u, __builtin_fma(u, u - 4.0 / 3.0, 2.0 / 3.0), -1.0 / 30.0);
}

// The parts of the mirror pair (t, M - t) from ONE lattice index per dimension (every z_j odd: the
// real-even path is taken only then, see to_nll).  With k = t z_j mod n and y = k / n - 1/2 (exact):
//   u(t)     = (k/n)^2 - k/n            = y^2 - 1/4
//   u(M - t) = u(frac(1/2 - k/n))       = y^2 - |y|          (M z_j = n/2 mod n for odd z_j)
// one fma each (|y| is a free source modifier).  Each is the exact value rounded once, so they equal the
// forms x^2 - x / x^2 - 1/4 of x = min(k, n - k) / n bit for bit, at 3 VALU per dimension fewer.
template <int PG, int D>
__device__ __forceinline__ void parts_mirror_pair(const Nll& a, unsigned t, unsigned /*n*/, unsigned mask,
                                                  double inv_n, double* p, double* pm) {
#pragma unroll
  for (int j = 0; j < D; ++j) {
    const unsigned k = mul_u24(t, a.gz[j]) & mask;
    const double y = __builtin_fma((double)k, inv_n, -0.5);
    const double ay = fabs(y);
    p[j] = bern_u<PG>(__builtin_fma(y, y, -0.25));
    pm[j] = bern_u<PG>(__builtin_fma(ay, ay, -ay));
  }
}

template <int D>
__device__ __forceinline__ double k1_of_parts(const Hyp& h, const double* p) {
  double r = 1.0;
#pragma unroll
  for (int j = 0; j < D; ++j) r *= __builtin_fma(h.ls[j], p[j], 1.0);
  return h.scale * r;
}

// whole-workgroup sum over NW waves (result in every thread)
template <int NW>
__device__ __forceinline__ double wg_sum(double v, double* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double tot = 0.0;
#pragma unroll
  for (int i = 0; i < NW; ++i) tot += red[i];
  __syncthreads();
  return tot;
}

// K whole-workgroup sums at once over NW waves (one barrier; the totals are valid in thread 0 only)
template <int NW, int K>
__device__ __forceinline__ void wg_sums_t0(double* v, double* red /* [K][NW] */) {
#pragma unroll
  for (int k = 0; k < K; ++k) {
    double x = v[k];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    if ((threadIdx.x & 63) == 0) red[k * NW + (threadIdx.x >> 6)] = x;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < K; ++k) {
      double t = 0.0;
#pragma unroll
      for (int i = 0; i < NW; ++i) t += red[k * NW + i];
      v[k] = t;
    }
  }
}


// Row geometry of the length-n/2 transform for rows of N2 = 2^P2 (P2 = 10, 11, 12): TL = N2/16 threads
// per row (one, two or four wavefronts), a row-pair workgroup of 2 TL threads.
template <int P2>
struct ReGeo {
  static constexpr int N2 = 1 << P2, TL = N2 / 16, WG = 2 * TL, IMG = N2 + N2 / 16;
  // the row transform's last radix pass leaves register R j + t of thread q holding output
  // k1 = pass_pos(q, j, t) = q + TL' j + 256 t; k1 < N2/2 are t < R/2, the Nyquist column k1 = N2/2 is
  // thread 0's register R/2
  static constexpr int SL = LastPass<P2>::S, RLL = PassRL<P2, SL>::value, R = 1 << RLL;
  static constexpr int NQ = 4096 / N2;   // Nyquist frequencies per column workgroup
};

// Row-pair geometry of workgroup (g, jp): this half's class r (natural residue mod N1), storage row u.
template <int P2>
struct RePair {
  using Geo = ReGeo<P2>;
  int g, jp, hh, q, r, N1, m1;
  unsigned u;
  bool cls0;        // workgroup 0, half 0: class 0 (mirror s <-> N2 - s inside the row)
  int partner_h;    // half holding the partner thread (logical group TL - 1 - q)
  __device__ __forceinline__ RePair(int log2n) {
    m1 = log2n - 1 - P2;
    N1 = 1 << m1;
    const int pairs = N1 >> 1;
    g = (int)(blockIdx.x / pairs);
    jp = (int)(blockIdx.x % pairs);
    hh = threadIdx.x / Geo::TL;
    q = threadIdx.x % Geo::TL;
    r = hh == 0 ? jp : (jp == 0 ? N1 / 2 : N1 - jp);
    u = brev_bits((unsigned)r, m1);
    cls0 = jp == 0 && hh == 0;
    partner_h = jp == 0 ? 1 : 1 - hh;
  }
  // position 16q + e of row r: s = brev_P2(16q + e) = brev_4(e) N2/16 + brev(q), natural index r + N1 s
  __device__ __forceinline__ unsigned s_of(unsigned e_brev4) const {
    return (e_brev4 << (P2 - 4)) | brev_bits((unsigned)q, P2 - 4);
  }
  __device__ __forceinline__ unsigned nat(unsigned e_brev4) const { return (unsigned)r + (unsigned)N1 * s_of(e_brev4); }
  // w_n^r w_{2 N2}^{brev(q)}: the element twiddle base (w_n^{N1 s} = w_{2 N2}^s; the w_32^{brev4(e)} factor
  // is a compile-time root).  w_{2 N2}^x: tw (w_4096) for N2 <= 2048, twm[13] (w_8192) for N2 = 4096.
  __device__ __forceinline__ double2 wbase(const double2* __restrict__ twm_n, const double2* __restrict__ tw2) const {
    const unsigned x = brev_bits((unsigned)q, P2 - 4);
    return cmul(twm_n[r], tw2[P2 >= 12 ? x : x << (11 - P2)]);
  }
};

// Inter-pass twiddles w_M^{r k1} of the thread's outputs: a per-lane base times a uniform step
template <int P2>
struct RowTwRe {
  double2 base;
  unsigned j1;
  __device__ __forceinline__ RowTwRe(unsigned r, int q, int m1, const double2* __restrict__ tw,
                                     const double2* __restrict__ twm) {
    j1 = r;
    base = inter_tw(j1 * (unsigned)q, P2, m1, tw, twm);
  }
  // twiddle of output k1 = q + off (off uniform)
  __device__ __forceinline__ double2 at(unsigned off, int m1, const double2* __restrict__ tw,
                                        const double2* __restrict__ twm) const {
    return cmul(base, inter_tw(j1 * off, P2, m1, tw, twm));
  }
};

template <int P2, int PG, int D>
__global__ __launch_bounds__(ReGeo<P2>::WG, 4) void k_fwd_rows_re(Nll a, const double2* __restrict__ tw,
                                                              const double2* __restrict__ twm_t,
                                                              const double2* __restrict__ twm_n,
                                                              const double2* __restrict__ tw2) {
  using Geo = ReGeo<P2>;
  constexpr int N2 = Geo::N2, TL = Geo::TL, IMG = Geo::IMG, R = Geo::R;
  __shared__ double img[2 * IMG];
  __shared__ double2 red[Geo::WG / 64];
  const RePair<P2> rp(a.log2n);
  const unsigned n = 1u << a.log2n, M = n >> 1, mask = n - 1;
  const double inv_n = ldexp(1.0, -a.log2n);
  const int q = rp.q;
  stamp_begin(a);
  Hyp h;
  load_hyp_wave(a, rp.g, h);
  fold_gen_coef<PG>(a, h);
  // element twiddles w_n^{i_e} = w_n^r w_{2 N2}^{brev(q)} w_32^{brev4(e)}
  const double2 wq = rp.wbase(twm_n, tw2);
  double2 v[16];
  double x0[16];
  double cM = 0.0;
  double2* xw = reinterpret_cast<double2*>(img + rp.partner_h * IMG);   // [8][TL] of the partner's wave
  const double2* xr = reinterpret_cast<const double2*>(img + rp.hh * IMG);
  double* c0 = img;                                                       // class 0: c at its N2 elements
  if (!rp.cls0) {
    // pairs e < 8: own element (16q + e) and the mirror (partner's 15 - e) from (c_i, c_{M-i})
    static_for<0, 8>([&](auto ec) {
      constexpr int e = decltype(ec)::value;
      const unsigned i = rp.nat(Brev4<e>::value);
      double pi[D], pmi[D];
      parts_mirror_pair<PG, D>(a, i, n, mask, inv_n, pi, pmi);
      const double x = k1_of_parts<D>(h, pi);
      const double y = k1_of_parts<D>(h, pmi);
      const double2 w = mul_root32<Brev4<e>::value>(wq);
      const double s = x + y, b = x - y;
      v[e] = make_double2(__builtin_fma(-b, w.y, s), b * w.x);                          // a + i b w
      xw[e * TL + (TL - 1 - q)] = make_double2(__builtin_fma(b, w.y, s), b * w.x);     // a + i b conj(w)
    });
  } else {
    static_for<0, 16>([&](auto ec) {
      constexpr int e = decltype(ec)::value;
      x0[e] = k1_nat<PG, D>(a, h, rp.nat(Brev4<e>::value), mask, inv_n);
      c0[16 * q + e] = x0[e];
    });
    if (q == 0) cM = k1_nat<PG, D>(a, h, M, mask, inv_n);
  }
  __syncthreads();
  if (!rp.cls0) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[15 - e] = xr[e * TL + q];
  } else {
    static_for<0, 16>([&](auto ec) {
      constexpr int e = decltype(ec)::value;
      const unsigned s = rp.s_of(Brev4<e>::value);
      const double y = s == 0 ? cM : c0[brev_bits((N2 - s) & (N2 - 1), P2)];
      const double x = x0[e];
      const double2 w = mul_root32<Brev4<e>::value>(wq);
      const double sa = x + y, b = x - y;
      v[e] = make_double2(__builtin_fma(-b, w.y, sa), b * w.x);
    });
  }
  double2 sum = make_double2(0.0, 0.0);
#pragma unroll
  for (int t = 0; t < 16; ++t) sum += v[t];
  const double2 mean = group_sum<TL>(sum, red) * (1.0 / N2);   // per row (one wave: shuffles only)
#pragma unroll
  for (int t = 0; t < 16; ++t) v[t] -= mean;
  fwd_reg_passes<P2, 0, true>(v, img + rp.hh * IMG, q, tw);
  if (q == 0) v[0] += mean * (double)N2;
  const RowTwRe<P2> rt(rp.r, q, rp.m1, tw, twm_t);
  double2* out = static_cast<double2*>(a.work) + (int64_t)rp.g * n;
  const WtStore wo(out);   // write-through: the column kernel reads the intermediate from HBM / MALL
#pragma unroll
  for (int j = 0; j < 16 / R; ++j)
#pragma unroll
    for (int t = 0; t < R / 2; ++t) {
      const int k1 = pass_pos<P2, Geo::SL, Geo::RLL>(q, j, t);
      const double2 o = tw_mul<double2>(v[j * R + t], rt.at(k1 - q, rp.m1, tw, twm_t), false);
      wo.put((unsigned)work_pos(rp.u, k1, rp.m1), o);
    }
  if (q == 0) out[(n >> 2) + rp.u] = tw_mul<double2>(v[R / 2], rt.at(N2 / 2, rp.m1, tw, twm_t), false);   // column N2/2
  stamp_end(a);
}

// Column pass over columns [0, N2/2) (tile blk of C = 4096/N1 columns, all N1 rows), eigenvalue terms
// of C_{2k} = Re Z_k and C_{2k+1} = Im Z_k (Y read as the pairs (Y_2k, Y_2k+1)), the adjoint column pass
// in place, and four of the Nyquist column's N1/2 distinct frequencies (b = 4 blk + j) by direct sums.
// Partial sums go to slot 4 blk of the per-block partials (slots 4 blk + 1..3 zero: the row-pair
// kernel's N1/2 blocks set the count).
template <int P2, int P1>
__global__ __launch_bounds__(kWG) void k_fwd_cols_re(Nll a, const double2* __restrict__ tw) {
  constexpr int N1 = 1 << P1, C = kTile / N1, CS = N1 + 1;
  constexpr int RL0 = PassRL<P1, 0>::value, R0 = 1 << RL0;
  constexpr int SL = LastPass<P1>::S, RLL = PassRL<P1, SL>::value, RLAST = 1 << RLL;
  constexpr int64_t N2 = 1 << P2;
  constexpr int NQ = ReGeo<P2>::NQ;
  constexpr int tiles = (int)(N2 / 2 / C);
  static_assert(tiles * NQ == N1 / 2 && NQ <= kWG / 64, "Nyquist frequencies per column workgroup");
  __shared__ double2 lds[C * CS];
  __shared__ double2 part[ColPart<C>::size];
  __shared__ double red3[3 * (kWG / 64)];
  __shared__ double2 red2[kWG / 64];
  __shared__ double redn[kWG / 64];
  const int m = a.log2n;
  const int64_t n = (int64_t)1 << m;
  const int g = (int)(blockIdx.x / tiles);
  const int blk = (int)(blockIdx.x % tiles);
  const int tid = threadIdx.x;
  const int c = tid % C, tt = tid / C;
  const int k1 = blk * C + c;
  stamp_begin(a);
  double2* base = static_cast<double2*>(a.work) + (int64_t)g * n;
  double2* wk = base + (int64_t)blk * kTile + c;
  double2* col = lds + c * CS;
  double2 v[16];
#pragma unroll
  for (int j = 0; j < 16 / R0; ++j)
#pragma unroll
    for (int t = 0; t < R0; ++t) v[j * R0 + t] = wk[pass_pos<P1, 0, RL0>(tt, j, t) * C];
  const double* ysq = a.ysq + (int64_t)g * a.ysq_stride;
  const double2* y2 = reinterpret_cast<const double2*>(ysq);   // (Y_2k, Y_2k+1)
  Hyp h;
  load_hyp_wave(a, g, h);
  const double rootn = sqrt((double)n), inv_rootn = 1.0 / rootn;
  double2 sum = make_double2(0.0, 0.0);
#pragma unroll
  for (int k = 0; k < 16; ++k) sum += v[k];
  column_partials<C>(sum, part);
  double2 mean = column_total<C>(c, part) * (1.0 / N1);
#pragma unroll
  for (int k = 0; k < 16; ++k) v[k] -= mean;
  fwd_reg_passes<P1, 0, false>(v, col, tt, tw);
  if (tt == 0) v[0] += mean * (double)N1;
  const double wA = k1 == 0 ? 1.0 : 2.0;    // column 0's real parts mirror inside the column
  double nA = 0.0, nB = 0.0, dA = 0.0, dB = 0.0;
  LogAcc lA, lB;
  // eigenvalue terms in a rolled loop over the thread's own image slots (the unrolled form keeps every
  // element, its Y pair and the divisions live at once: > 300 VGPRs, one wave per SIMD)
#pragma unroll
  for (int j = 0; j < 16 / RLAST; ++j)
#pragma unroll
    for (int t = 0; t < RLAST; ++t) col[pass_pos<P1, SL, RLL>(tt, j, t)] = v[j * RLAST + t];
#pragma unroll FGP_RE_EIG_UNROLL
  for (int k = 0; k < 16; ++k) {
    const int pos = pass_pos<P1, SL, RLL>(tt, k / RLAST, k % RLAST);
    const double2 yk = y2[k1 + N2 * pos];
    const double2 vk = col[pos];
    const double gA = eig_terms(vk.x * inv_rootn, rootn, h.noise, yk.x, a.logdet_weight, nA, lA, dA);
    const double gB = eig_terms(vk.y * inv_rootn, rootn, h.noise, yk.y, a.logdet_weight, nB, lB, dB);
    col[pos] = make_double2(wA * gA, 2.0 * gB);
  }
  sum = make_double2(0.0, 0.0);
#pragma unroll
  for (int j = 0; j < 16 / RLAST; ++j)
#pragma unroll
    for (int t = 0; t < RLAST; ++t) {
      v[j * RLAST + t] = col[pass_pos<P1, SL, RLL>(tt, j, t)];
      sum += v[j * RLAST + t];
    }
  double norm = wA * nA + 2.0 * nB;
  double dnoise = wA * dA + 2.0 * dB;
  double logdet = wA * lA.log_sum(1.0) + 2.0 * lB.log_sum(1.0);
  column_partials<C>(sum, part);
  mean = column_total<C>(c, part) * (1.0 / N1);
#pragma unroll
  for (int k = 0; k < 16; ++k) v[k] -= mean;
  adj_reg_passes<P1, SL, false>(v, col, tt, tw);
  if (tt == 0) v[0] += mean * (double)N1;
  {
    const WtStore wo(base);   // write-through, as the row kernel's stores
    const unsigned o0 = (unsigned)(blk * kTile + c);
#pragma unroll
    for (int j = 0; j < 16 / R0; ++j)
#pragma unroll
      for (int t = 0; t < R0; ++t) wo.put(o0 + (unsigned)(pass_pos<P1, 0, RL0>(tt, j, t) * C), v[j * R0 + t]);
  }
  // Nyquist column (k1 = N2/2): Z_b = sum_u T_u w_N1^{brev(u) b} (mean-centred), real part, weight 2;
  // wave j < NQ of the workgroup takes b = NQ blk + j
  const double2* nyq = base + (n >> 2);
  double2 ts = make_double2(0.0, 0.0);
  for (int uu = tid; uu < N1; uu += kWG) ts += nyq[uu];
  const double2 mu = block_sum_t(ts, red2) * (1.0 / N1);
  const int wv = tid >> 6, ln = tid & 63;
  const unsigned b = (unsigned)(NQ * blk + (wv % NQ));
  double as = 0.0;
  for (int uu = ln; uu < N1 && wv < NQ; uu += 64) {
    const double2 d = nyq[uu] - mu;
    const double2 w = tw[((brev_bits((unsigned)uu, P1) * b) & (N1 - 1)) << (kTileLog - P1)];
    as += __builtin_fma(d.x, w.x, -(d.y * w.y));
  }
  as = group_sum<64>(as, redn);
  if (ln == 0 && wv < NQ) {
    if (b == 0) as += mu.x * (double)N1;
    const int64_t kq = N2 / 2 + N2 * (int64_t)b;   // Z index; frequency 2 kq
    double normN = 0.0, dnN = 0.0;
    LogAcc lN;
    const double gq = eig_terms(as * inv_rootn, rootn, h.noise, ysq[2 * kq], a.logdet_weight, normN, lN, dnN);
    reinterpret_cast<double*>(base + (n >> 2) + N1)[b] = 2.0 * gq;
    norm += 2.0 * normN;
    dnoise += 2.0 * dnN;
    logdet += 2.0 * lN.log_sum(1.0);
  }
  double tot[3] = {norm, logdet, dnoise};
  wg_sums_t0<kWG / 64, 3>(tot, red3);
  if (tid < NQ) {
#pragma unroll
    for (int k = 0; k < 3; ++k) *part_ptr(a, g, k, NQ * blk + tid) = tid == 0 ? tot[k] : 0.0;
  }
  stamp_end(a);
}

// Adjoint row pass of the row pair (inputs: columns [0, N2/2) from the column kernel, the Nyquist
// column by a direct sum over its V, zero elsewhere), then dL/dc at the pair's generated values:
//   dL/dc_i = P + Q, dL/dc_{M-i} = P - Q,  P = Re W_i + Re W_{M-i},
//   Q = (Im W_i + Im W_{M-i}) Re w - (Re W_i - Re W_{M-i}) Im w,  w = w_n^i
// (class 0: each element's own c_i with the mirror's W; element 0 also c_M), and the gradient terms.
template <int P2, int PG, int D>
__global__ __launch_bounds__(ReGeo<P2>::WG, 4) void k_bwd_rows_re(Nll a, const double2* __restrict__ tw,
                                                              const double2* __restrict__ twm_t,
                                                              const double2* __restrict__ twm_n,
                                                              const double2* __restrict__ tw2, FitFuse fz) {
  using Geo = ReGeo<P2>;
  constexpr int N2 = Geo::N2, TL = Geo::TL, IMG = Geo::IMG, R = Geo::R;
  __shared__ double img[2 * IMG];
  __shared__ int last_wg;
  __shared__ double2 red[Geo::WG / 64];
  __shared__ double redd[(1 + D) * (Geo::WG / 64)];
  const RePair<P2> rp(a.log2n);
  const unsigned n = 1u << a.log2n, M = n >> 1, mask = n - 1;
  const double inv_n = ldexp(1.0, -a.log2n);
  const int q = rp.q, N1 = rp.N1;
  stamp_begin(a);
  const double2* in = static_cast<const double2*>(a.work) + (int64_t)rp.g * n;
  const double* vny = reinterpret_cast<const double*>(in + (n >> 2) + N1);
  const RowTwRe<P2> rt(rp.r, q, rp.m1, tw, twm_t);
  double2 v[16];
  double2 sum = make_double2(0.0, 0.0);
#pragma unroll
  for (int j = 0; j < 16 / R; ++j)
#pragma unroll
    for (int t = 0; t < R; ++t) {
      if (t < R / 2) {
        const int k1 = pass_pos<P2, Geo::SL, Geo::RLL>(q, j, t);
        v[j * R + t] = tw_mul<double2>(in[work_pos(rp.u, k1, rp.m1)], rt.at(k1 - q, rp.m1, tw, twm_t), true);
        sum += v[j * R + t];
      } else {
        v[j * R + t] = make_double2(0.0, 0.0);
      }
    }
  // Nyquist input of row u: sum_b V_b conj(w_N1^{r b}) over the N1/2 distinct frequencies b
  double2 ny = make_double2(0.0, 0.0);
  for (int b = q; b < N1 / 2; b += TL) {
    const double2 w = tw[(((unsigned)rp.r * (unsigned)b) & (unsigned)(N1 - 1)) << (kTileLog - rp.m1)];
    const double vb = vny[b];
    ny += make_double2(vb * w.x, -(vb * w.y));
  }
  ny = group_sum<TL>(ny, red);
  if (q == 0) {
    v[R / 2] = tw_mul<double2>(ny, rt.at(N2 / 2, rp.m1, tw, twm_t), true);
    sum += v[R / 2];
  }
  const double2 mean = group_sum<TL>(sum, red) * (1.0 / N2);
#pragma unroll
  for (int k = 0; k < 16; ++k) v[k] -= mean;
  adj_reg_passes<P2, LastPass<P2>::S, true>(v, img + rp.hh * IMG, q, tw);
  if (q == 0) v[0] += mean * (double)N2;
  // W at the mirror elements -- from the partner thread (regular), or the class-0 image (Re, then Im)
  // -- combined into dL/dc as they arrive (gv: the thread's 16 generated points, in loop order)
  double2* xw = reinterpret_cast<double2*>(img + rp.partner_h * IMG);
  const double2* xr = reinterpret_cast<const double2*>(img + rp.hh * IMG);
  double* c0 = img;
  const double2 wq = rp.wbase(twm_n, tw2);
  double gv[16];
  double gM = 0.0;
  __syncthreads();
  if (!rp.cls0) {
#pragma unroll
    for (int e = 8; e < 16; ++e) xw[(e - 8) * TL + (TL - 1 - q)] = v[e];
  } else {
#pragma unroll
    for (int e = 0; e < 16; ++e) c0[16 * q + e] = v[e].x;
  }
  __syncthreads();
  if (!rp.cls0) {
    static_for<0, 8>([&](auto ec) {
      constexpr int e = decltype(ec)::value;
      const double2 w = mul_root32<Brev4<e>::value>(wq);
      const double2 wi = v[e], wr = xr[(7 - e) * TL + q];
      const double P = wi.x + wr.x;
      const double Q = __builtin_fma(wi.y + wr.y, w.x, -((wi.x - wr.x) * w.y));
      gv[2 * e] = P + Q;
      gv[2 * e + 1] = P - Q;
    });
  } else {
    // P + Q = W_i.x (1 - w.y) + W_m.x (1 + w.y) + (W_i.y + W_m.y) w.x; element s = 0 (q = 0, e = 0):
    // no mirror, dL/dc_0 = W.x + W.y, dL/dc_M = W.x - W.y
    static_for<0, 16>([&](auto ec) {
      constexpr int e = decltype(ec)::value;
      const double2 w = mul_root32<Brev4<e>::value>(wq);
      const unsigned s = rp.s_of(Brev4<e>::value);
      const double wmx = s == 0 ? 0.0 : c0[brev_bits((N2 - s) & (N2 - 1), P2)];
      gv[e] = __builtin_fma(v[e].y, w.x, __builtin_fma(wmx, 1.0 + w.y, v[e].x * (1.0 - w.y)));
    });
    gM = v[0].x - v[0].y;
  }
  __syncthreads();
  if (rp.cls0) {
#pragma unroll
    for (int e = 0; e < 16; ++e) c0[16 * q + e] = v[e].y;
  }
  __syncthreads();
  if (rp.cls0) {
    static_for<0, 16>([&](auto ec) {
      constexpr int e = decltype(ec)::value;
      const double2 w = mul_root32<Brev4<e>::value>(wq);
      const unsigned s = rp.s_of(Brev4<e>::value);
      const double wmy = s == 0 ? 0.0 : c0[brev_bits((N2 - s) & (N2 - 1), P2)];
      gv[e] = __builtin_fma(wmy, w.x, gv[e]);
    });
  }
  __syncthreads();
  // dL/dc values into private LDS slots (stride 17: conflict-free) for the rolled gradient loop
  double* gl = img + 17 * threadIdx.x;
#pragma unroll
  for (int t = 0; t < 16; ++t) gl[t] = gv[t];
  Hyp h;
  load_hyp_wave(a, rp.g, h);
  fold_gen_coef<PG>(a, h);
  double acc[1 + D];
#pragma unroll
  for (int k = 0; k < 1 + D; ++k) acc[k] = 0.0;
  const double gs = 1.0 / sqrt((double)n);
  const unsigned sq = brev_bits((unsigned)q, P2 - 4);
  if (rp.cls0) {
#pragma unroll 2
    for (int t = 0; t < 16; ++t) {
      const unsigned nat = (unsigned)N1 * (((__builtin_bitreverse32((unsigned)t) >> 28) << (P2 - 4)) | sq);
      double p[D];
#pragma unroll
      for (int j = 0; j < D; ++j) p[j] = lattice_gen_part<PG>(a.gz[j], nat, mask, inv_n);
      grad_terms_p<D>(h, p, gl[t] * gs, acc);
    }
  } else {
    // the mirror pairs (i, M - i): both points' parts from one lattice index per dimension
    for (int e = 0; e < 8; ++e) {
      const unsigned i = (unsigned)rp.r + (unsigned)N1 * (((__builtin_bitreverse32((unsigned)e) >> 28) << (P2 - 4)) | sq);
      double p[D], pm[D];
      parts_mirror_pair<PG, D>(a, i, n, mask, inv_n, p, pm);
      grad_terms_p<D>(h, p, gl[2 * e] * gs, acc);
      grad_terms_p<D>(h, pm, gl[2 * e + 1] * gs, acc);
    }
  }
  if (rp.cls0 && q == 0) {
    double p[D];
#pragma unroll
    for (int j = 0; j < D; ++j) p[j] = lattice_gen_part<PG>(a.gz[j], M, mask, inv_n);
    grad_terms_p<D>(h, p, gM * gs, acc);
  }
  wg_sums_t0<Geo::WG / 64, 1 + D>(acc, redd);
  if (!fz.counters) {
    if (threadIdx.x == 0) {
#pragma unroll
      for (int k = 0; k < 1 + D; ++k) *part_ptr(a, rp.g, 3 + k, rp.jp) = acc[k] * grad_factor(h, k);
    }
    stamp_end(a);
    return;
  }
  // Fused reduction + Rprop (fgp_fit_run, per-problem fits).  Hand-off (MI355X_MICROARCH.md row 1): the
  // one storing lane writes this workgroup's partials sc1, waits for them, then adds to the problem's
  // counter at agent scope; the workgroup whose add returns nb - 1 is the last of its problem and, behind
  // a barrier, reads every partial with sc1 loads and applies the step; it re-arms the counter.
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < 1 + D; ++k)
      __hip_atomic_store(part_ptr(a, rp.g, 3 + k, rp.jp), acc[k] * grad_factor(h, k), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned prev = __hip_atomic_fetch_add(fz.counters + rp.g, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last_wg = prev == (unsigned)(a.nb - 1);
  }
  __syncthreads();
  if (last_wg) {
    double* red = img;                        // (4 + FGP_MAX_D) WG/64 + 4 + FGP_MAX_D doubles << 2 IMG
    double* vals = img + (4 + FGP_MAX_D) * (Geo::WG / 64);
    reduce_step_wg<Geo::WG, true>(a, fz.f, rp.g, fz.iter, fz.do_update, red, vals);
    if (threadIdx.x == 0) __hip_atomic_store(fz.counters + rp.g, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  stamp_end(a);
}

// real-even lattice kernels: row pairs of the length-n/2 transform (G N1/2 workgroups of N2/8 threads),
// column tiles of its columns [0, N2/2) (G n/16384 workgroups of 256); N1 = n / (2 N2).
// Rows of 2^11 (measured best of 2^10 / 2^11 / 2^12: profiles/r02d_exp_re_rows_*).
int re_row_log2(int log2n) {
  const int p2 = kP2reDefault;
  return (p2 >= 10 && p2 <= 12 && log2n - 1 - p2 <= 12 && log2n - 1 - p2 >= 4) ? p2 : -1;
}

template <int P2>
static int launch_re_p2(const Nll& a, int stage, const Tables* tb, hipStream_t st, const FitFuse& fz) {
  using Geo = ReGeo<P2>;
  const int m = a.log2n, mt = m - 1, p1 = mt - P2;
  const double2* tw2 = P2 >= 12 ? tb->twm[13] : tb->tw4096;
  if (stage == 0 || stage == 2) {
    const unsigned grid = (unsigned)((int64_t)a.G << (p1 - 1));
    return with_pg<double2>(a, [&](auto pgc) {
      constexpr int PG = decltype(pgc)::value;
      if constexpr (PG == 0) {
        return set_error(kErrInvalid, "real-even fit kernels need the lattice parts generator");
      } else {
        with_d(a.d, [&](auto dc) {
          constexpr int DD = decltype(dc)::value;
          if (stage == 0)
            k_fwd_rows_re<P2, PG, DD><<<grid, Geo::WG, 0, st>>>(a, tb->tw4096, tb->twm[mt], tb->twm[m], tw2);
          else
            k_bwd_rows_re<P2, PG, DD><<<grid, Geo::WG, 0, st>>>(a, tb->tw4096, tb->twm[mt], tb->twm[m], tw2, fz);
        });
        return check_launch(stage == 0 ? "k_fwd_rows_re" : "k_bwd_rows_re");
      }
    });
  }
  if (stage != 1) return set_error(kErrInvalid, "bad stage %d", stage);
  const unsigned grid = (unsigned)((int64_t)a.G << (m - 14));
  switch (p1) {
#define FGP_C(PP) case PP: k_fwd_cols_re<P2, PP><<<grid, kWG, 0, st>>>(a, tb->tw4096); break;
    FGP_C(4) FGP_C(5) FGP_C(6) FGP_C(7) FGP_C(8) FGP_C(9) FGP_C(10) FGP_C(11) FGP_C(12)
#undef FGP_C
    default: return set_error(kErrInvalid, "bad re m1");
  }
  return check_launch("k_fwd_cols_re");
}

static int launch_re_any(const Nll& a, int stage, const Tables* tb, hipStream_t st, const FitFuse& fz) {
  switch (re_row_log2(a.log2n)) {
    case 11: return launch_re_p2<11>(a, stage, tb, st, fz);
    default: return set_error(kErrInvalid, "real-even fit kernels: no row split for log2n=%d", a.log2n);
  }
}

int launch_re(const Nll& a, int stage, const Tables* tb, hipStream_t st) {
  FitFuse none{};
  none.counters = nullptr;
  return launch_re_any(a, stage, tb, st, none);
}

int launch_re_bwd_fused(const Nll& a, const FitFuse& fz, const Tables* tb, hipStream_t st) {
  return launch_re_any(a, 2, tb, st, fz);
}

}  // namespace fgp
