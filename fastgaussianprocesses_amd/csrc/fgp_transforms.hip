// Batched orthonormal transforms of the fast-GP hot path (drop-in for qmcpy.fftbr_torch,
// qmcpy.ifftbr_torch, qmcpy.fwht_torch as injected at fast_gp_lattice.py:224-225 and
// fast_gp_digital_net_b2.py:226, wrapped by AbstractFastGP.ft/ift, abstract_fast_gp.py:197-228).
//
// Length n = 2^m, 0 <= m <= 24, transform along the last (contiguous) axis of a [batch, n] array.
//   m <= 3       : k_tiny   (one thread per transform, registers only)
//   4 <= m <= 12 : k_single (one LDS pass: 4096/n transforms per 256-thread workgroup)
//   13 <= m <= 24: two passes over an N1 x N2 view (N2 = 2^m2 contiguous rows, N1 = 2^(m-m2)):
//        fftbr  = rows(fftbr_N2) -> twiddle w_n^{brev(u) k2} -> columns(fftbr_N1)
//        ifftbr = columns(ifftbr_N1) -> conj twiddle -> rows(ifftbr_N2)      (exact adjoint)
//        fwht   = rows(fwht_N2) -> columns(fwht_N1)
//      The bit-reversal of fftbr's input is never materialised: for i = u*N2 + v,
//      brev_m(i) = brev(v)*N1 + brev(u), so the row pass is itself a bit-reversed-input transform
//      of each contiguous row and the column pass one of each column (natural-order output).
//
// "stable" reproduces AbstractFastGP.ft's mean-centring (abstract_fast_gp.py:209-211) inside the
// kernels: every row / column is centred by its own mean before its transform and the mean is
// added back to its frequency-0 bin afterwards (exact in exact arithmetic: the transform of a
// constant vector is supported on bin 0), keeping large DC components out of the butterflies.
#include "fgp_common.h"
#include "fgp_runtime.h"
#include "../../include/fgp_hip.h"

namespace fgp {

// Optional elementwise factor applied to the input of the inverse's first pass (fgp_ifftbr_mul):
// element i of row b is multiplied by f[b * bs + i] (bs = 0: one row shared by all) -- the
// tilde-domain solve A * y~ of gram_matrix_solve (util.py:341-343) fused into the load.
struct Pre {
  const void* f;
  int64_t bs;
};
template <typename T>
__device__ __forceinline__ T pre_mul(T v, const Pre& p, int64_t b, int64_t i) {
  if (!p.f) return v;
  const T w = static_cast<const T*>(p.f)[b * p.bs + i];
  if constexpr (Elem<T>::cx) return cmul(v, w);
  else return v * w;
}

// ------------------------------------------------------------------ m <= 3: registers only
template <int P, typename T, bool ADJ>
__global__ __launch_bounds__(kWG) void k_tiny(const void* in, int64_t in_bs, int in_real, void* out,
                                               int64_t out_bs, int out_real, int64_t batch, int stable,
                                               double scale, const double2* __restrict__ tw, Pre pre) {
  constexpr int L = 1 << P;
  const int64_t b = (int64_t)blockIdx.x * kWG + threadIdx.x;
  if (b >= batch) return;
  T v[L];
  T mean = zero_v<T>();
#pragma unroll
  for (int i = 0; i < L; ++i) {
    v[i] = pre_mul(load_in<T>(in, b * in_bs + i, in_real), pre, b, i);
    mean += v[i];
  }
  mean = mean * (1.0 / L);
  if (stable) {
#pragma unroll
    for (int i = 0; i < L; ++i) v[i] -= mean;
  }
  if constexpr (!ADJ) {
#pragma unroll
    for (int s = 0; s < P; ++s)
#pragma unroll
      for (int a = 0; a < L; ++a)
        if (!(a & (1 << s))) bfly_dit(v[a], v[a | (1 << s)], tw, (a & ((1 << s) - 1)) << (11 - s));
  } else {
#pragma unroll
    for (int s = P - 1; s >= 0; --s)
#pragma unroll
      for (int a = 0; a < L; ++a)
        if (!(a & (1 << s))) bfly_dif(v[a], v[a | (1 << s)], tw, (a & ((1 << s) - 1)) << (11 - s));
  }
  if (stable) v[0] += mean * (double)L;
#pragma unroll
  for (int i = 0; i < L; ++i) store_out(out, b * out_bs + i, scaled(v[i], scale), out_real);
}

// ------------------------------------------------------------------ 4 <= m <= 12: one LDS pass
template <int P, typename T, bool ADJ>
__global__ __launch_bounds__(kWG) void k_single(const void* in, int64_t in_bs, int in_real, void* out,
                                                 int64_t out_bs, int out_real, int64_t batch, int stable,
                                                 double scale, const double2* __restrict__ tw, Pre pre) {
  constexpr int L = 1 << P;
  constexpr int TL = L / 16;
  constexpr int TPW = kTile / L;
  __shared__ T lds[kTile + kTile / 16];
  __shared__ T red[kWG / 64];
  const int tid = threadIdx.x;
  const int64_t b0 = (int64_t)blockIdx.x * TPW;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int e = tid + k * kWG;
    const int64_t b = b0 + (e >> P);
    T v = zero_v<T>();
    if (b < batch) v = pre_mul(load_in<T>(in, b * in_bs + (e & (L - 1)), in_real), pre, b, e & (L - 1));
    lds[padi(e)] = v;
  }
  __syncthreads();
  const int tt = tid % TL;
  T* s = lds + (tid / TL) * (L + L / 16);
  center_transform<P, ADJ>(s, tt, stable, red, tw);
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int e = tid + k * kWG;
    const int64_t b = b0 + (e >> P);
    if (b < batch) store_out(out, b * out_bs + (e & (L - 1)), scaled(lds[padi(e)], scale), out_real);
  }
}

// ------------------------------------------------------------------ m > 12: row pass
// View of one batch item: N1 rows of N2 = 2^P2 contiguous elements.  4096/N2 rows per workgroup.
// Forward (!ADJ): row transform, then (twiddle) multiply position (u, k2) by w_n^{brev_m1(u) k2}.
// Adjoint  (ADJ): (twiddle) multiply the column pass' output by conj(w_n^{brev_m1(u) k2}) on load,
//                 then the row transform.
template <int P2, typename T, bool ADJ>
__global__ __launch_bounds__(kWG) void k_rows(const void* in, int64_t in_bs, int in_real, void* out,
                                               int64_t out_bs, int out_real, int m, int stable, double scale,
                                               int twiddle, const double2* __restrict__ tw,
                                               const double2* __restrict__ twm) {
  constexpr int N2 = 1 << P2;
  constexpr int TL = N2 / 16;
  constexpr int RPW = kTile / N2;
  constexpr bool FFT = Elem<T>::cx;
  __shared__ T lds[kTile + kTile / 16];
  __shared__ T red[kWG / 64];
  const int m1 = m - P2;
  const int64_t tiles = (int64_t)1 << (m - kTileLog);
  const int64_t b = blockIdx.x / tiles;
  const int row0 = (int)(blockIdx.x % tiles) * RPW;
  const int tid = threadIdx.x;
  const int64_t ibase = b * in_bs + (int64_t)row0 * N2;   // rows are contiguous: the tile is one slab
  const int64_t obase = b * out_bs + (int64_t)row0 * N2;
  if constexpr (RPW == 1) {
    // one row per workgroup: uniform twiddle row, mean folded into the staging store
    const RowTwiddle rt((unsigned)row0, tid, P2, m1, tw, twm);
    T v[16];
    T sum = zero_v<T>();
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      v[k] = load_in<T>(in, ibase + tid + k * kWG, in_real);
      if (ADJ && FFT && twiddle) v[k] = tw_mul<T>(v[k], rt.at(k, P2, m1, tw, twm), true);
      sum += v[k];
    }
    const T mean = stable ? block_sum_t(sum, red) * (1.0 / N2) : zero_v<T>();
#pragma unroll
    for (int k = 0; k < 16; ++k) lds[padi(tid + k * kWG)] = v[k] - mean;
    __syncthreads();
    transform_add_mean<P2, ADJ>(lds, tid, mean, tw);
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int e = tid + k * kWG;
      T r = lds[padi(e)];
      if (!ADJ && FFT && twiddle) r = tw_mul<T>(r, rt.at(k, P2, m1, tw, twm), false);
      store_out(out, obase + e, scaled(r, scale), out_real);
    }
    return;
  }
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int e = tid + k * kWG;
    T v = load_in<T>(in, ibase + e, in_real);
    if (ADJ && FFT && twiddle) {
      const unsigned ex = brev_bits((unsigned)(row0 + (e >> P2)), m1) * (unsigned)(e & (N2 - 1));
      v = tw_mul<T>(v, inter_tw(ex, P2, m1, tw, twm), true);
    }
    lds[padi(e)] = v;
  }
  __syncthreads();
  T* s = lds + (tid / TL) * (N2 + N2 / 16);
  center_transform<P2, ADJ>(s, tid % TL, stable, red, tw);
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int e = tid + k * kWG;
    T v = lds[padi(e)];
    if (!ADJ && FFT && twiddle) {
      const unsigned ex = brev_bits((unsigned)(row0 + (e >> P2)), m1) * (unsigned)(e & (N2 - 1));   // < 2^m
      v = tw_mul<T>(v, inter_tw(ex, P2, m1, tw, twm), false);
    }
    store_out(out, obase + e, scaled(v, scale), out_real);
  }
}

// ------------------------------------------------------------------ m > 12: column pass
// C = 4096/N1 adjacent columns (k2 in [c0, c0+C)) of length N1 = 2^P1 per workgroup, staged
// column-major in LDS with an odd column stride (conflict-free transposing ds_write_b128).
// Forward (!ADJ): column transform (natural-order output rows k1); adjoint (ADJ): its transpose-
// conjugate (output row u in bit-reversed position).  No twiddle here: both directions apply the
// inter-pass twiddle in the row pass, where a workgroup's row index is uniform.
// In-place safe (in == out): each workgroup reads its whole tile before writing it.
template <int P1>
struct ColLayout {
  static constexpr int N1 = 1 << P1;
  static constexpr int C = kTile / N1;
  static constexpr int PADLEN = N1 + N1 / 16;
  static constexpr int CS = (PADLEN % 2 == 0) ? PADLEN + 1 : PADLEN;
  static_assert(C * CS <= kLds, "column tile exceeds LDS budget");
};

template <int P1, typename T, bool ADJ>
__global__ __launch_bounds__(kWG) void k_cols(const void* in, int64_t in_bs, int in_real, void* out,
                                               int64_t out_bs, int out_real, int m, int stable, double scale,
                                               int twiddle, const double2* __restrict__ tw,
                                               const double2* __restrict__ twm, Pre pre) {
  using Lay = ColLayout<P1>;
  constexpr int N1 = Lay::N1, C = Lay::C, CS = Lay::CS, TL = N1 / 16;
  __shared__ T lds[kLds];
  __shared__ T part[ColPart<C>::size];
  (void)twiddle;
  (void)twm;
  const int P2 = m - P1;
  const int64_t N2 = (int64_t)1 << P2;
  const int64_t tiles = (int64_t)1 << (m - kTileLog);
  const int64_t b = blockIdx.x / tiles;
  const int64_t c0 = (blockIdx.x % tiles) * C;
  const int tid = threadIdx.x;
  const int64_t ibase = b * in_bs + c0;
  const int cl = tid % C;         // column this thread stages (e = tid + 256 k keeps e mod C fixed)
  T v[16];
  T sum = zero_v<T>();
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int e = tid + k * kWG;
    v[k] = pre_mul(load_in<T>(in, ibase + (int64_t)(e / C) * N2 + cl, in_real), pre, b, (int64_t)(e / C) * N2 + c0 + cl);
    sum += v[k];
  }
  T mean_l = zero_v<T>(), mean_t = zero_v<T>();
  const int col = tid / TL;       // column this thread transforms
  if (stable) {
    column_partials<C>(sum, part);
    mean_l = column_total<C>(cl, part) * (1.0 / N1);
    mean_t = column_total<C>(col, part) * (1.0 / N1);
  }
#pragma unroll
  for (int k = 0; k < 16; ++k) lds[cl * CS + padi((tid + k * kWG) / C)] = v[k] - mean_l;
  __syncthreads();
  transform_add_mean<P1, ADJ>(lds + col * CS, tid % TL, mean_t, tw);
  const int64_t obase = b * out_bs + c0;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int e = tid + k * kWG;
    const int r = e / C;
    store_out(out, obase + (int64_t)r * N2 + cl, scaled(lds[cl * CS + padi(r)], scale), out_real);
  }
}

// ------------------------------------------------------------------ launch helpers
template <typename T, bool ADJ>
static int launch_tiny(int m, const void* in, int64_t in_bs, int in_real, void* out, int out_real, int64_t batch,
                       int stable, double scale, const double2* tw, hipStream_t st, Pre pre = Pre{nullptr, 0}) {
  const dim3 g((unsigned)((batch + kWG - 1) / kWG));
  const int64_t n = (int64_t)1 << m;
  switch (m) {
    case 0: k_tiny<0, T, ADJ><<<g, kWG, 0, st>>>(in, in_bs, in_real, out, n, out_real, batch, stable, scale, tw, pre); break;
    case 1: k_tiny<1, T, ADJ><<<g, kWG, 0, st>>>(in, in_bs, in_real, out, n, out_real, batch, stable, scale, tw, pre); break;
    case 2: k_tiny<2, T, ADJ><<<g, kWG, 0, st>>>(in, in_bs, in_real, out, n, out_real, batch, stable, scale, tw, pre); break;
    case 3: k_tiny<3, T, ADJ><<<g, kWG, 0, st>>>(in, in_bs, in_real, out, n, out_real, batch, stable, scale, tw, pre); break;
    default: return set_error(kErrInvalid, "launch_tiny: bad m");
  }
  return check_launch("k_tiny");
}

#define FGP_SINGLE_CASE(P)                                                                                   \
  case P:                                                                                                    \
    k_single<P, T, ADJ><<<dim3((unsigned)((batch + (kTile >> P) - 1) / (kTile >> P))), kWG, 0, st>>>(      \
        in, in_bs, in_real, out, (int64_t)1 << P, out_real, batch, stable, scale, tw, pre);                  \
    break;

template <typename T, bool ADJ>
static int launch_single(int m, const void* in, int64_t in_bs, int in_real, void* out, int out_real,
                         int64_t batch, int stable, double scale, const double2* tw, hipStream_t st,
                         Pre pre = Pre{nullptr, 0}) {
  switch (m) {
    FGP_SINGLE_CASE(4) FGP_SINGLE_CASE(5) FGP_SINGLE_CASE(6) FGP_SINGLE_CASE(7) FGP_SINGLE_CASE(8)
    FGP_SINGLE_CASE(9) FGP_SINGLE_CASE(10) FGP_SINGLE_CASE(11) FGP_SINGLE_CASE(12)
    default: return set_error(kErrInvalid, "launch_single: bad m");
  }
  return check_launch("k_single");
}
#undef FGP_SINGLE_CASE

#define FGP_ROWS_CASE(P)                                                                                       \
  case P:                                                                                                      \
    k_rows<P, T, ADJ><<<g, kWG, 0, st>>>(in, in_bs, in_real, out, out_bs, out_real, m, stable, scale, twiddle, \
                                         tw, twm);                                                             \
    break;

template <typename T, bool ADJ>
static int launch_rows(int m, const void* in, int64_t in_bs, int in_real, void* out, int64_t out_bs, int out_real,
                       int64_t batch, int stable, double scale, int twiddle, const Tables* tb, hipStream_t st) {
  const int m2 = split_m2(m);
  const dim3 g((unsigned)(batch << (m - kTileLog)));
  const double2* tw = tb->tw4096;
  const double2* twm = tb->twm[m];
  switch (m2) {
    FGP_ROWS_CASE(9) FGP_ROWS_CASE(10) FGP_ROWS_CASE(11) FGP_ROWS_CASE(12)
    default: return set_error(kErrInvalid, "launch_rows: bad m2");
  }
  return check_launch("k_rows");
}
#undef FGP_ROWS_CASE

#define FGP_COLS_CASE(P)                                                                                       \
  case P:                                                                                                      \
    k_cols<P, T, ADJ><<<g, kWG, 0, st>>>(in, in_bs, in_real, out, out_bs, out_real, m, stable, scale, twiddle, \
                                         tw, twm, pre);                                                        \
    break;

template <typename T, bool ADJ>
static int launch_cols(int m, const void* in, int64_t in_bs, int in_real, void* out, int64_t out_bs, int out_real,
                       int64_t batch, int stable, double scale, int twiddle, const Tables* tb, hipStream_t st,
                       Pre pre = Pre{nullptr, 0}) {
  const int m1 = m - split_m2(m);
  const dim3 g((unsigned)(batch << (m - kTileLog)));
  const double2* tw = tb->tw4096;
  const double2* twm = tb->twm[m];
  switch (m1) {
    FGP_COLS_CASE(4) FGP_COLS_CASE(5) FGP_COLS_CASE(6) FGP_COLS_CASE(7) FGP_COLS_CASE(8)
    FGP_COLS_CASE(9) FGP_COLS_CASE(10) FGP_COLS_CASE(11) FGP_COLS_CASE(12)
    default: return set_error(kErrInvalid, "launch_cols: bad m1");
  }
  return check_launch("k_cols");
}
#undef FGP_COLS_CASE

static int validate(const void* in, const void* out, int64_t batch, int log2n, int64_t in_bs) {
  if (log2n < 0 || log2n > kMaxLog2N)
    return set_error(kErrUnsupported, "log2n=%d outside supported range [0, %d]", log2n, kMaxLog2N);
  if (batch < 0) return set_error(kErrInvalid, "negative batch");
  if (batch > 0 && (in == nullptr || out == nullptr)) return set_error(kErrInvalid, "null data pointer");
  if (batch > 1 && in_bs < ((int64_t)1 << log2n)) return set_error(kErrInvalid, "in_batch_stride < n");
  if ((batch << log2n) >= ((int64_t)1 << 31) * kTile) return set_error(kErrUnsupported, "batch*n too large");
  return kOk;
}

int cols_adjoint_launch(bool fft, int m, const void* in, void* out, int64_t batch, const Tables* tb,
                        hipStream_t st) {
  const int64_t n = (int64_t)1 << m;
  if (fft) return launch_cols<double2, true>(m, in, n, 0, out, n, 0, batch, 1, 1.0, 0, tb, st);
  return launch_cols<double, false>(m, in, n, 0, out, n, 0, batch, 1, 1.0, 0, tb, st);
}

// Y[g, k] = sum_{r < R} |x[r G + g, k]|^2 in fp64 (fastgaussianprocesses_amd.fast_gp._ysq: the data
// term of the MLL, Y = sum over the outputs sharing problem g of |y~|^2, util.py:364-370).  Thread per
// (g, k): loads coalesced along k, rows summed in fixed ascending order (deterministic).
template <typename T>
__global__ __launch_bounds__(kWG) void k_sum_sq(const T* __restrict__ x, int64_t xs, int64_t R, int64_t G, int64_t n,
                                                 double* __restrict__ out) {
  const int64_t e = (int64_t)blockIdx.x * kWG + threadIdx.x;
  if (e >= G * n) return;
  const int64_t g = e / n, k = e % n;
  const T* p = x + g * xs + k;
  double acc = 0.0;
#pragma unroll 8
  for (int64_t r = 0; r < R; ++r) {
    const T v = p[r * G * xs];
    if constexpr (Elem<T>::cx) acc += (double)v.x * (double)v.x + (double)v.y * (double)v.y;
    else acc += (double)v * (double)v;
  }
  out[e] = acc;
}

// Y from the Hermitian halves of ft(real rows): x [R G][H] complex128 rows holding k = 0 .. n/2 (H = n/2 + 1,
// row stride xs >= H); out[g][k] and out[g][n - k] = sum_r |x[r G + g][k]|^2 (ascending r: k_sum_sq's values on the
// full spectra bit for bit, |X_{n-k}| = |conj X_k|).
__global__ __launch_bounds__(kWG) void k_sum_sq_half(const double2* __restrict__ x, int64_t xs, int64_t R, int64_t G,
                                                      int64_t n, double* __restrict__ out) {
  const int64_t H = n / 2 + 1;
  const int64_t e = (int64_t)blockIdx.x * kWG + threadIdx.x;
  if (e >= G * H) return;
  const int64_t g = e / H, k = e % H;
  const double2* p = x + g * xs + k;
  double acc = 0.0;
#pragma unroll 8
  for (int64_t r = 0; r < R; ++r) {
    const double2 v = p[r * G * xs];
    acc += v.x * v.x + v.y * v.y;
  }
  out[g * n + k] = acc;
  if (k > 0 && k < n / 2) out[g * n + n - k] = acc;
}

// Entry-point bodies for the fp64 (T = double2 / double) and fp32 (T = float2 / float) variants.
template <typename T>
static int fftbr_impl(const void* in, int64_t in_bs, int in_real, void* out, int64_t batch, int log2n, int stable,
                      hipStream_t st) {
  int rc = validate(in, out, batch, log2n, in_bs);
  if (rc != kOk || batch == 0) return rc;
  const Tables* tb = get_tables(st);
  if (!tb) return set_error(kErrHip, "twiddle table initialisation failed");
  const int64_t n = (int64_t)1 << log2n;
  const double scale = 1.0 / sqrt((double)n);
  if (log2n <= 3) return launch_tiny<T, false>(log2n, in, in_bs, in_real, out, 0, batch, stable, scale, tb->tw4096, st);
  if (log2n <= 12) return launch_single<T, false>(log2n, in, in_bs, in_real, out, 0, batch, stable, scale, tb->tw4096, st);
  rc = launch_rows<T, false>(log2n, in, in_bs, in_real, out, n, 0, batch, stable, 1.0, 1, tb, st);
  if (rc != kOk) return rc;
  return launch_cols<T, false>(log2n, out, n, 0, out, n, 0, batch, stable, scale, 0, tb, st);
}

template <typename T>
static int ifftbr_impl(const void* in, int64_t in_bs, void* out, int out_real, void* work, int64_t batch, int log2n,
                       int stable, hipStream_t st, Pre pre = Pre{nullptr, 0}) {
  int rc = validate(in, out, batch, log2n, in_bs);
  if (rc != kOk || batch == 0) return rc;
  const Tables* tb = get_tables(st);
  if (!tb) return set_error(kErrHip, "twiddle table initialisation failed");
  const int64_t n = (int64_t)1 << log2n;
  const double scale = 1.0 / sqrt((double)n);
  if (log2n <= 3) return launch_tiny<T, true>(log2n, in, in_bs, 0, out, out_real, batch, stable, scale, tb->tw4096, st, pre);
  if (log2n <= 12)
    return launch_single<T, true>(log2n, in, in_bs, 0, out, out_real, batch, stable, scale, tb->tw4096, st, pre);
  void* mid = out_real ? work : out;
  if (mid == nullptr) return set_error(kErrInvalid, "ifftbr: out_real with n > 4096 needs a complex work buffer");
  rc = launch_cols<T, true>(log2n, in, in_bs, 0, mid, n, 0, batch, stable, 1.0, 0, tb, st, pre);
  if (rc != kOk) return rc;
  return launch_rows<T, true>(log2n, mid, n, 0, out, n, out_real, batch, stable, scale, 1, tb, st);
}

template <typename T>
static int fwht_impl(const void* in, int64_t in_bs, void* out, int64_t batch, int log2n, int stable, hipStream_t st,
                     Pre pre = Pre{nullptr, 0}) {
  int rc = validate(in, out, batch, log2n, in_bs);
  if (rc != kOk || batch == 0) return rc;
  const Tables* tb = get_tables(st);
  if (!tb) return set_error(kErrHip, "twiddle table initialisation failed");
  const int64_t n = (int64_t)1 << log2n;
  const double scale = 1.0 / sqrt((double)n);
  if (log2n <= 3) return launch_tiny<T, false>(log2n, in, in_bs, 0, out, 0, batch, stable, scale, tb->tw4096, st, pre);
  if (log2n <= 12)
    return launch_single<T, false>(log2n, in, in_bs, 0, out, 0, batch, stable, scale, tb->tw4096, st, pre);
  if (pre.f) {   // the WHT is separable in any order: columns first (they take the factor), then rows
    rc = launch_cols<T, false>(log2n, in, in_bs, 0, out, n, 0, batch, stable, 1.0, 0, tb, st, pre);
    if (rc != kOk) return rc;
    return launch_rows<T, false>(log2n, out, n, 0, out, n, 0, batch, stable, scale, 0, tb, st);
  }
  rc = launch_rows<T, false>(log2n, in, in_bs, 0, out, n, 0, batch, stable, 1.0, 0, tb, st);
  if (rc != kOk) return rc;
  return launch_cols<T, false>(log2n, out, n, 0, out, n, 0, batch, stable, scale, 0, tb, st);
}

// One DIT doubling stage (fastgps/util.py:113-132 _LamCaches, :173-178 _YtildeCache): from the
// transforms of the first n and the next n values to the transform of all 2n,
//   out[k] = (prev[k] + w^k nxt[k]) / sqrt(2),  out[k + n] = (prev[k] - w^k nxt[k]) / sqrt(2),
// w^k = exp(-pi i k / n) (get_omega, fast_gp_lattice.py:261-262) for lattices, 1 for nets
// (fast_gp_digital_net_b2.py:264-265).  One thread per k: 16 + 16 B read, 32 B written (lattice).
__global__ __launch_bounds__(kWG) void k_double_cx(const double2* __restrict__ prev, int64_t ps,
                                                   const double2* __restrict__ nxt, int64_t ns, int64_t B,
                                                   int64_t n, double2* __restrict__ out, int64_t os) {
  const int64_t e = (int64_t)blockIdx.x * kWG + threadIdx.x;
  if (e >= B * n) return;
  const int64_t b = e / n, k = e - b * n;
  double sn, cs;
  sincospi(-(double)k / (double)n, &sn, &cs);
  const double2 a = prev[b * ps + k], v = nxt[b * ns + k];
  const double2 wv = make_double2(cs * v.x - sn * v.y, cs * v.y + sn * v.x);
  const double r = 0.70710678118654752440;
  out[b * os + k] = make_double2((a.x + wv.x) * r, (a.y + wv.y) * r);
  out[b * os + k + n] = make_double2((a.x - wv.x) * r, (a.y - wv.y) * r);
}

__global__ __launch_bounds__(kWG) void k_double_re(const double* __restrict__ prev, int64_t ps,
                                                   const double* __restrict__ nxt, int64_t ns, int64_t B,
                                                   int64_t n, double* __restrict__ out, int64_t os) {
  const int64_t e = (int64_t)blockIdx.x * kWG + threadIdx.x;
  if (e >= B * n) return;
  const int64_t b = e / n, k = e - b * n;
  const double a = prev[b * ps + k], v = nxt[b * ns + k];
  const double r = 0.70710678118654752440;
  out[b * os + k] = (a + v) * r;
  out[b * os + k + n] = (a - v) * r;
}

}  // namespace fgp

using namespace fgp;

extern "C" {

int fgp_fftbr(const void* in, int64_t in_batch_stride, int in_is_real, void* out, int64_t batch, int log2n,
              int stable, void* stream) {
  return fftbr_impl<double2>(in, in_batch_stride, in_is_real, out, batch, log2n, stable, (hipStream_t)stream);
}

int fgp_ifftbr(const void* in, int64_t in_batch_stride, void* out, int out_real, void* work, int64_t batch,
               int log2n, int stable, void* stream) {
  return ifftbr_impl<double2>(in, in_batch_stride, out, out_real, work, batch, log2n, stable, (hipStream_t)stream);
}

int fgp_fwht(const double* in, int64_t in_batch_stride, double* out, int64_t batch, int log2n, int stable,
             void* stream) {
  return fwht_impl<double>(in, in_batch_stride, out, batch, log2n, stable, (hipStream_t)stream);
}

int fgp_fftbr_c64(const void* in, int64_t in_batch_stride, int in_is_real, void* out, int64_t batch, int log2n,
                  int stable, void* stream) {
  return fftbr_impl<float2>(in, in_batch_stride, in_is_real, out, batch, log2n, stable, (hipStream_t)stream);
}

int fgp_ifftbr_c64(const void* in, int64_t in_batch_stride, void* out, int out_real, void* work, int64_t batch,
                   int log2n, int stable, void* stream) {
  return ifftbr_impl<float2>(in, in_batch_stride, out, out_real, work, batch, log2n, stable, (hipStream_t)stream);
}

int fgp_fwht_f32(const float* in, int64_t in_batch_stride, float* out, int64_t batch, int log2n, int stable,
                 void* stream) {
  return fwht_impl<float>(in, in_batch_stride, out, batch, log2n, stable, (hipStream_t)stream);
}

int fgp_sum_sq_half(const void* x, int64_t x_row_stride, int64_t R, int64_t G, int64_t n, double* out, void* stream) {
  if (R < 1 || G < 1 || n < 2 || (n & (n - 1)) || x_row_stride < n / 2 + 1)
    return set_error(kErrInvalid, "fgp_sum_sq_half: bad sizes");
  if (!x || !out) return set_error(kErrInvalid, "fgp_sum_sq_half: null pointer");
  const int64_t cnt = G * (n / 2 + 1);
  k_sum_sq_half<<<(unsigned)((cnt + kWG - 1) / kWG), kWG, 0, (hipStream_t)stream>>>(static_cast<const double2*>(x),
                                                                                   x_row_stride, R, G, n, out);
  return check_launch("k_sum_sq_half");
}

int fgp_sum_sq(const void* x, int64_t x_row_stride, int kind, int64_t R, int64_t G, int64_t n, double* out,
               void* stream) {
  if (R < 1 || G < 1 || n < 1 || x_row_stride < n) return set_error(kErrInvalid, "fgp_sum_sq: bad sizes");
  if (!x || !out) return set_error(kErrInvalid, "fgp_sum_sq: null pointer");
  const unsigned grid = (unsigned)((G * n + kWG - 1) / kWG);
  hipStream_t st = (hipStream_t)stream;
  switch (kind) {
    case 0: k_sum_sq<double><<<grid, kWG, 0, st>>>(static_cast<const double*>(x), x_row_stride, R, G, n, out); break;
    case 1: k_sum_sq<double2><<<grid, kWG, 0, st>>>(static_cast<const double2*>(x), x_row_stride, R, G, n, out); break;
    case 2: k_sum_sq<float><<<grid, kWG, 0, st>>>(static_cast<const float*>(x), x_row_stride, R, G, n, out); break;
    case 3: k_sum_sq<float2><<<grid, kWG, 0, st>>>(static_cast<const float2*>(x), x_row_stride, R, G, n, out); break;
    default: return set_error(kErrInvalid, "fgp_sum_sq: bad kind %d", kind);
  }
  return check_launch("k_sum_sq");
}

int fgp_double_update(int family, const void* prev, int64_t prev_stride, const void* nxt, int64_t nxt_stride,
                      int64_t batch, int log2n, void* out, int64_t out_stride, void* stream) {
  if (log2n < 0 || log2n >= kMaxLog2N || batch < 0) return set_error(kErrInvalid, "fgp_double_update: bad sizes");
  const int64_t n = (int64_t)1 << log2n;
  if (batch == 0) return kOk;
  if (!prev || !nxt || !out) return set_error(kErrInvalid, "fgp_double_update: null pointer");
  if (prev_stride < n || nxt_stride < n || out_stride < 2 * n) return set_error(kErrInvalid, "fgp_double_update: strides");
  const unsigned grid = (unsigned)((batch * n + kWG - 1) / kWG);
  hipStream_t st = (hipStream_t)stream;
  if (family == FGP_FAMILY_LATTICE)
    k_double_cx<<<grid, kWG, 0, st>>>(static_cast<const double2*>(prev), prev_stride, static_cast<const double2*>(nxt),
                                      nxt_stride, batch, n, static_cast<double2*>(out), out_stride);
  else
    k_double_re<<<grid, kWG, 0, st>>>(static_cast<const double*>(prev), prev_stride, static_cast<const double*>(nxt),
                                      nxt_stride, batch, n, static_cast<double*>(out), out_stride);
  return check_launch("k_double_update");
}

/* Inverse transform of in * f (fgp_hip.h fgp_ifftbr_mul): lattice complex128 / complex64 via ifftbr,
 * net float64 / float32 via the (self-inverse) fwht. */
int fgp_ifftbr_mul(int family, int single, const void* in, int64_t in_batch_stride, const void* f, int64_t f_batch_stride,
                   void* out, int out_real, void* work, int64_t batch, int log2n, int stable, void* stream) {
  if (!f) return set_error(kErrInvalid, "fgp_ifftbr_mul: null factor");
  const Pre pre{f, f_batch_stride};
  hipStream_t st = (hipStream_t)stream;
  if (family == FGP_FAMILY_LATTICE)
    return single ? ifftbr_impl<float2>(in, in_batch_stride, out, out_real, work, batch, log2n, stable, st, pre)
                  : ifftbr_impl<double2>(in, in_batch_stride, out, out_real, work, batch, log2n, stable, st, pre);
  return single ? fwht_impl<float>(in, in_batch_stride, out, batch, log2n, stable, st, pre)
                : fwht_impl<double>(in, in_batch_stride, out, batch, log2n, stable, st, pre);
}

}  // extern "C"
