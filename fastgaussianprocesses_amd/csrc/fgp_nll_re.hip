// Real-even (RE) lattice fit kernels, n >= 2^17 (the default fused-fit path for regenerated lattice
// parts): see the section comment below and DESIGN.md section 3.
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
// The two-pass split M = N1 x N2 (N2 = 4096, rows = natural classes r = i mod N1, as the engine's
// bit-reversed storage rows u = brev(r)) puts element i and its mirror M - i in rows r and N1 - r
// (positions 16q + e and 16(255 - q) + 15 - e): one 512-thread workgroup takes the row pair, half 0
// row r, half 1 row N1 - r, and the rows 0 / N1/2 (self-mirrored classes) share workgroup 0.
// Output symmetry: C_{2k} = C_{n-2k} and C_{2k+1} = C_{n-2k-1}, i.e. column k1 of Z mirrors column
// N2 - k1 (real parts) and N2 - 1 - k1 (imaginary parts).  Columns [0, N2/2) therefore hold every
// imaginary part (weight 2) and every real part except those of column N2/2 (weight 2; column 0's
// real parts mirror inside the column, weight 1).  Column N2/2 contributes real parts only, whose
// N1/2 distinct values (mirror k2 <-> N1 - 1 - k2) are direct sums over its N1 rows, one per column
// workgroup.  The loss is this folded sum; its gradient along real-even c (the only direction c moves)
// is the true one, so the adjoint runs over the same half: V = dL/dC_{2k} + i dL/dC_{2k+1} on columns
// [0, N2/2), zero elsewhere, the Nyquist column's V by direct sums in the row kernel.  Per iteration:
// rows write n/4 complex (4n B), columns read 4n + Y 4n and write 4n, rows read 4n: 20n bytes
// (R2C 40n), and half the eigenvalue terms and kernel parts.
constexpr int kWGre = 512;

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

// end stamps of a 512-thread launch: after a barrier, waves 0..3 record (the record has 1 + kWG/64 slots)
__device__ __forceinline__ void stamp_end_re(const Nll& a) {
  if (a.stamps) {
    __syncthreads();
    if (threadIdx.x < kWG) stamp_end(a);
  }
}

// Row-pair geometry of workgroup (g, jp): this half's class r (natural residue mod N1), storage row u.
struct RePair {
  int g, jp, hh, q, r, N1, m1;
  unsigned u;
  bool cls0;        // workgroup 0, half 0: class 0 (mirror s <-> N2 - s inside the row)
  int partner_h;    // half holding the partner thread (logical group 255 - q)
  __device__ __forceinline__ RePair(int log2n) {
    m1 = log2n - 1 - 12;
    N1 = 1 << m1;
    const int pairs = N1 >> 1;
    g = (int)(blockIdx.x / pairs);
    jp = (int)(blockIdx.x % pairs);
    hh = threadIdx.x >> 8;
    q = threadIdx.x & 255;
    r = hh == 0 ? jp : (jp == 0 ? N1 / 2 : N1 - jp);
    u = brev_bits((unsigned)r, m1);
    cls0 = jp == 0 && hh == 0;
    partner_h = jp == 0 ? 1 : 1 - hh;
  }
  // natural index of element e of the thread's group (position 16q + e of row r: s = brev_12(16q + e))
  __device__ __forceinline__ unsigned nat(unsigned e_brev4) const {
    return (unsigned)r + ((unsigned)N1 << 8) * e_brev4 + (unsigned)N1 * brev_bits((unsigned)q, 8);
  }
};

template <int PG, int D>
__global__ __launch_bounds__(kWGre, 4) void k_fwd_rows_re(Nll a, const double2* __restrict__ tw,
                                                       const double2* __restrict__ twm_t,
                                                       const double2* __restrict__ twm_n,
                                                       const double2* __restrict__ twm13) {
  constexpr int P2 = 12, N2 = 1 << P2, IMG = kTile + kTile / 16;
  __shared__ double img[2 * IMG];
  __shared__ double2 red[kWGre / 64];
  const RePair rp(a.log2n);
  const unsigned n = 1u << a.log2n, M = n >> 1, mask = n - 1;
  const double inv_n = ldexp(1.0, -a.log2n);
  const int q = rp.q;
  stamp_begin(a);
  Hyp h;
  load_hyp_wave(a, rp.g, h);
  fold_gen_coef<PG>(a, h);
  // element twiddles w_n^{i_e} = w_n^r w_8192^{brev8(q)} w_32^{brev4(e)}
  const double2 wq = cmul(twm_n[rp.r], twm13[brev_bits((unsigned)q, 8)]);
  double2 v[16];
  double x0[16];
  double cM = 0.0;
  double2* xw = reinterpret_cast<double2*>(img + rp.partner_h * IMG);   // [8][256] of the partner's half
  const double2* xr = reinterpret_cast<const double2*>(img + rp.hh * IMG);
  double* c0 = img;                                                       // class 0: c at its 4096 elements
  if (!rp.cls0) {
    // pairs e < 8: own element (16q + e) and the mirror (partner's 15 - e) from (c_i, c_{M-i})
    static_for<0, 8>([&](auto ec) {
      constexpr int e = decltype(ec)::value;
      const unsigned i = rp.nat(Brev4<e>::value);
      const double x = k1_nat<PG, D>(a, h, i, mask, inv_n);
      const double y = k1_nat<PG, D>(a, h, M - i, mask, inv_n);
      const double2 w = mul_root32<Brev4<e>::value>(wq);
      const double s = x + y, b = x - y;
      v[e] = make_double2(__builtin_fma(-b, w.y, s), b * w.x);           // a + i b w
      xw[e * 256 + (255 - q)] = make_double2(__builtin_fma(b, w.y, s), b * w.x);   // a + i b conj(w)
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
    for (int e = 0; e < 8; ++e) v[15 - e] = xr[e * 256 + q];
  } else {
    static_for<0, 16>([&](auto ec) {
      constexpr int e = decltype(ec)::value;
      const unsigned s = (Brev4<e>::value << 8) | brev_bits((unsigned)q, 8);
      const unsigned sm = (N2 - s) & (N2 - 1);
      const double y = s == 0 ? cM : c0[brev_bits(sm, 12)];
      const double x = x0[e];
      const double2 w = mul_root32<Brev4<e>::value>(wq);
      const double sa = x + y, b = x - y;
      v[e] = make_double2(__builtin_fma(-b, w.y, sa), b * w.x);
    });
  }
  double2 sum = make_double2(0.0, 0.0);
#pragma unroll
  for (int t = 0; t < 16; ++t) sum += v[t];
  const double2 mean = group_sum<256>(sum, red) * (1.0 / N2);
#pragma unroll
  for (int t = 0; t < 16; ++t) v[t] -= mean;
  fwd_reg_passes<P2, 0, true>(v, img + rp.hh * IMG, q, tw);
  if (q == 0) v[0] += mean * (double)N2;
  const RowTwiddle rt(rp.u, q, P2, rp.m1, tw, twm_t);
  double2* out = static_cast<double2*>(a.work) + (int64_t)rp.g * n;
#pragma unroll
  for (int k = 0; k < 8; ++k)
    out[work_pos(rp.u, q + k * 256, rp.m1)] = tw_mul<double2>(v[k], rt.at(k, P2, rp.m1, tw, twm_t), false);
  if (q == 0) out[(n >> 2) + rp.u] = tw_mul<double2>(v[8], rt.at(8, P2, rp.m1, tw, twm_t), false);   // column N2/2
  stamp_end_re(a);
}

// Column pass over columns [0, N2/2) (tile blk of C = 4096/N1 columns, all N1 rows), eigenvalue terms
// of C_{2k} = Re Z_k and C_{2k+1} = Im Z_k (Y read as the pairs (Y_2k, Y_2k+1)), the adjoint column pass
// in place, and the Nyquist column's distinct frequency b = blk by a direct sum.
template <int P1>
__global__ __launch_bounds__(kWG) void k_fwd_cols_re(Nll a, const double2* __restrict__ tw) {
  constexpr int N1 = 1 << P1, C = kTile / N1, CS = N1 + 1;
  constexpr int RL0 = PassRL<P1, 0>::value, R0 = 1 << RL0;
  constexpr int SL = LastPass<P1>::S, RLL = PassRL<P1, SL>::value, RLAST = 1 << RLL;
  constexpr int64_t N2 = 4096;
  __shared__ double2 lds[C * CS];
  __shared__ double2 part[ColPart<C>::size];
  __shared__ double redd[kWG / 64];
  __shared__ double2 red2[kWG / 64];
  const int m = a.log2n;
  const int64_t n = (int64_t)1 << m;
  constexpr int tiles = N1 / 2;
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
#pragma unroll 2
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
#pragma unroll
  for (int j = 0; j < 16 / R0; ++j)
#pragma unroll
    for (int t = 0; t < R0; ++t) wk[pass_pos<P1, 0, RL0>(tt, j, t) * C] = v[j * R0 + t];
  // Nyquist column (k1 = N2/2): Z_b = sum_u T_u w_N1^{brev(u) b} (mean-centred), real part, weight 2
  const double2* nyq = base + (n >> 2);
  double2 ts = make_double2(0.0, 0.0);
  for (int uu = tid; uu < N1; uu += kWG) ts += nyq[uu];
  const double2 mu = block_sum_t(ts, red2) * (1.0 / N1);
  double as = 0.0;
  for (int uu = tid; uu < N1; uu += kWG) {
    const double2 d = nyq[uu] - mu;
    const double2 w = tw[((brev_bits((unsigned)uu, P1) * (unsigned)blk) & (N1 - 1)) << (kTileLog - P1)];
    as += __builtin_fma(d.x, w.x, -(d.y * w.y));
  }
  double anyq = block_sum(as, redd);
  if (tid == 0) {
    if (blk == 0) anyq += mu.x * (double)N1;
    const int64_t kq = N2 / 2 + N2 * blk;   // Z index; frequency 2 kq
    double normN = 0.0, dnN = 0.0;
    LogAcc lN;
    const double gq = eig_terms(anyq * inv_rootn, rootn, h.noise, ysq[2 * kq], a.logdet_weight, normN, lN, dnN);
    reinterpret_cast<double*>(base + (n >> 2) + N1)[blk] = 2.0 * gq;
    norm += 2.0 * normN;
    dnoise += 2.0 * dnN;
    logdet += 2.0 * lN.log_sum(1.0);
  }
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

// Adjoint row pass of the row pair (inputs: columns [0, N2/2) from the column kernel, the Nyquist
// column by a direct sum over its V, zero elsewhere), then dL/dc at the pair's generated values:
//   dL/dc_i = P + Q, dL/dc_{M-i} = P - Q,  P = Re W_i + Re W_{M-i},
//   Q = (Im W_i + Im W_{M-i}) Re w - (Re W_i - Re W_{M-i}) Im w,  w = w_n^i
// (class 0: each element's own c_i with the mirror's W; element 0 also c_M), and the gradient terms.
template <int PG, int D>
__global__ __launch_bounds__(kWGre, 4) void k_bwd_rows_re(Nll a, const double2* __restrict__ tw,
                                                       const double2* __restrict__ twm_t,
                                                       const double2* __restrict__ twm_n,
                                                       const double2* __restrict__ twm13) {
  constexpr int P2 = 12, N2 = 1 << P2, IMG = kTile + kTile / 16;
  __shared__ double img[2 * IMG];
  __shared__ double2 red[kWGre / 64];
  __shared__ double redd[kWGre / 64];
  const RePair rp(a.log2n);
  const unsigned n = 1u << a.log2n, M = n >> 1, mask = n - 1;
  const double inv_n = ldexp(1.0, -a.log2n);
  const int q = rp.q, N1 = rp.N1;
  stamp_begin(a);
  const double2* in = static_cast<const double2*>(a.work) + (int64_t)rp.g * n;
  const double* vny = reinterpret_cast<const double*>(in + (n >> 2) + N1);
  const RowTwiddle rt(rp.u, q, P2, rp.m1, tw, twm_t);
  double2 v[16];
  double2 sum = make_double2(0.0, 0.0);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    v[k] = tw_mul<double2>(in[work_pos(rp.u, q + k * 256, rp.m1)], rt.at(k, P2, rp.m1, tw, twm_t), true);
    sum += v[k];
  }
#pragma unroll
  for (int k = 8; k < 16; ++k) v[k] = make_double2(0.0, 0.0);
  // Nyquist input of row u: sum_b V_b conj(w_N1^{r b}) over the N1/2 distinct frequencies b
  double2 ny = make_double2(0.0, 0.0);
  for (int b = q; b < N1 / 2; b += 256) {
    const double2 w = tw[(((unsigned)rp.r * (unsigned)b) & (unsigned)(N1 - 1)) << (kTileLog - rp.m1)];
    const double vb = vny[b];
    ny += make_double2(vb * w.x, -(vb * w.y));
  }
  ny = group_sum<256>(ny, red);
  if (q == 0) {
    v[8] = tw_mul<double2>(ny, rt.at(8, P2, rp.m1, tw, twm_t), true);
    sum += v[8];
  }
  const double2 mean = group_sum<256>(sum, red) * (1.0 / N2);
#pragma unroll
  for (int k = 0; k < 16; ++k) v[k] -= mean;
  adj_reg_passes<P2, LastPass<P2>::S, true>(v, img + rp.hh * IMG, q, tw);
  if (q == 0) v[0] += mean * (double)N2;
  // W at the mirror elements -- from the partner thread (regular), or the class-0 image (Re, then Im)
  // -- combined into dL/dc as they arrive (gv: the thread's 16 generated points, in loop order)
  double2* xw = reinterpret_cast<double2*>(img + rp.partner_h * IMG);
  const double2* xr = reinterpret_cast<const double2*>(img + rp.hh * IMG);
  double* c0 = img;
  const double2 wq = cmul(twm_n[rp.r], twm13[brev_bits((unsigned)q, 8)]);
  const unsigned sq = brev_bits((unsigned)q, 8);
  double gv[16];
  double gM = 0.0;
  __syncthreads();
  if (!rp.cls0) {
#pragma unroll
    for (int e = 8; e < 16; ++e) xw[(e - 8) * 256 + (255 - q)] = v[e];
  } else {
#pragma unroll
    for (int e = 0; e < 16; ++e) c0[16 * q + e] = v[e].x;
  }
  __syncthreads();
  if (!rp.cls0) {
    static_for<0, 8>([&](auto ec) {
      constexpr int e = decltype(ec)::value;
      const double2 w = mul_root32<Brev4<e>::value>(wq);
      const double2 wi = v[e], wr = xr[(7 - e) * 256 + q];
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
      const unsigned s = (Brev4<e>::value << 8) | sq;
      const double wmx = s == 0 ? 0.0 : c0[brev_bits((N2 - s) & (N2 - 1), 12)];
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
      const unsigned s = (Brev4<e>::value << 8) | sq;
      const double wmy = s == 0 ? 0.0 : c0[brev_bits((N2 - s) & (N2 - 1), 12)];
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
#pragma unroll 2
  for (int t = 0; t < 16; ++t) {
    unsigned nat;
    if (rp.cls0) {
      nat = (unsigned)N1 * (((__builtin_bitreverse32((unsigned)t) >> 28) << 8) | sq);
    } else {
      const unsigned i = (unsigned)rp.r + (unsigned)N1 * (((__builtin_bitreverse32((unsigned)(t >> 1)) >> 28) << 8) | sq);
      nat = (t & 1) ? M - i : i;
    }
    double p[D];
#pragma unroll
    for (int j = 0; j < D; ++j) p[j] = lattice_gen_part<PG>(a.gz[j], nat, mask, inv_n);
    grad_terms_p<D>(h, p, gl[t] * gs, acc);
  }
  if (rp.cls0 && q == 0) {
    double p[D];
#pragma unroll
    for (int j = 0; j < D; ++j) p[j] = lattice_gen_part<PG>(a.gz[j], M, mask, inv_n);
    grad_terms_p<D>(h, p, gM * gs, acc);
  }
#pragma unroll
  for (int k = 0; k < 1 + D; ++k) {
    const double r = wg_sum<kWGre / 64>(acc[k], redd) * grad_factor(h, k);
    if (threadIdx.x == 0) *part_ptr(a, rp.g, 3 + k, rp.jp) = r;
  }
  stamp_end_re(a);
}

// real-even lattice kernels: row pairs of the length-n/2 transform (G N1/2 workgroups of 512 threads),
// column tiles of its columns [0, N2/2) (G N1/2 workgroups of 256)
int launch_re(const Nll& a, int stage, const Tables* tb, hipStream_t st) {
  const int m = a.log2n, mt = m - 1, p1 = mt - 12;
  const unsigned grid = (unsigned)((int64_t)a.G << (p1 - 1));
  if (stage == 0 || stage == 2) {
    return with_pg<double2>(a, [&](auto pgc) {
      constexpr int PG = decltype(pgc)::value;
      if constexpr (PG == 0) {
        return set_error(kErrInvalid, "real-even fit kernels need the lattice parts generator");
      } else {
        with_d(a.d, [&](auto dc) {
          constexpr int DD = decltype(dc)::value;
          if (stage == 0)
            k_fwd_rows_re<PG, DD><<<grid, kWGre, 0, st>>>(a, tb->tw4096, tb->twm[mt], tb->twm[m], tb->twm[13]);
          else
            k_bwd_rows_re<PG, DD><<<grid, kWGre, 0, st>>>(a, tb->tw4096, tb->twm[mt], tb->twm[m], tb->twm[13]);
        });
        return check_launch(stage == 0 ? "k_fwd_rows_re" : "k_bwd_rows_re");
      }
    });
  }
  if (stage != 1) return set_error(kErrInvalid, "bad stage %d", stage);
  switch (p1) {
#define FGP_C(PP) case PP: k_fwd_cols_re<PP><<<grid, kWG, 0, st>>>(a, tb->tw4096); break;
    FGP_C(4) FGP_C(5) FGP_C(6) FGP_C(7) FGP_C(8) FGP_C(9) FGP_C(10) FGP_C(11)
#undef FGP_C
    default: return set_error(kErrInvalid, "bad re m1");
  }
  return check_launch("k_fwd_cols_re");
}

}  // namespace fgp
