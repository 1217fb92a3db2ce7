// Shared device code for the fast-transform GP kernels (gfx950 / CDNA4).
//
// Transform engine: every in-LDS transform works on a 4096-element tile per 256-thread workgroup
// (16 elements per thread, 4 wave64s).  A length-L = 2^P transform (4 <= P <= 12) is run by
// TL = L/16 threads; a tile holds 4096/L such transforms (rows or columns of a larger transform).
//
//   forward  (fftbr, qmcpy.fftbr_torch):  bit-reversed-order input, natural-order output  = radix-2
//            DIT network  x[a], x[a+h] <- x[a] + w x[a+h], x[a] - w x[a+h],  w = exp(-2 pi i pos/2h)
//   adjoint  (ifftbr, qmcpy.ifftbr_torch): the exact transpose-conjugate of that network = DIF with
//            conj twiddles, natural input, bit-reversed output.
//   WHT      (fwht, qmcpy.fwht_torch): same network with w = 1 (self-adjoint, Sylvester order).
//
// Stages are executed as radix-16 register passes (4 radix-2 stages per LDS round trip).
// LDS index padding i + (i >> 4) keeps every pass's 16-byte (double2) / 8-byte (double) accesses
// bank-conflict free.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace fgp {

constexpr int kWG = 256;         // threads per workgroup
constexpr int kTileLog = 12;
constexpr int kTile = 1 << kTileLog;   // elements per workgroup tile
constexpr int kLds = 4608;       // >= every padded tile layout used below (max 4480)

__device__ __forceinline__ int padi(int i) { return i + (i >> 4); }

// ---------------------------------------------------------------- scalar / complex arithmetic
__device__ __forceinline__ double2 operator+(double2 a, double2 b) { return make_double2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ double2 operator-(double2 a, double2 b) { return make_double2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ double2 operator*(double2 a, double s) { return make_double2(a.x * s, a.y * s); }
__device__ __forceinline__ double2& operator+=(double2& a, double2 b) { a.x += b.x; a.y += b.y; return a; }
__device__ __forceinline__ double2& operator-=(double2& a, double2 b) { a.x -= b.x; a.y -= b.y; return a; }
// Complex products with explicit fma (the library is compiled with -ffp-contract=off, so rounding
// never depends on the compiler's contraction choices in a particular kernel).
__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
  return make_double2(__builtin_fma(a.x, b.x, -(a.y * b.y)), __builtin_fma(a.x, b.y, a.y * b.x));
}
__device__ __forceinline__ double2 cmulc(double2 a, double2 w) {  // a * conj(w)
  return make_double2(__builtin_fma(a.x, w.x, a.y * w.y), __builtin_fma(a.y, w.x, -(a.x * w.y)));
}

template <typename T> __device__ __forceinline__ T zero_v();
template <> __device__ __forceinline__ double zero_v<double>() { return 0.0; }
template <> __device__ __forceinline__ double2 zero_v<double2>() { return make_double2(0.0, 0.0); }

// ---------------------------------------------------------------- single precision (c64 / f32)
// The same engine instantiated on float2 / float (fgp_fftbr_c64, fgp_ifftbr_c64, fgp_fwht_f32):
// arithmetic in fp32 with explicit fmaf, twiddles read from the fp64 tables and rounded once.
__device__ __forceinline__ float2 operator+(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 operator-(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 operator*(float2 a, double s) {
  const float f = (float)s;
  return make_float2(a.x * f, a.y * f);
}
__device__ __forceinline__ float2& operator+=(float2& a, float2 b) { a.x += b.x; a.y += b.y; return a; }
__device__ __forceinline__ float2& operator-=(float2& a, float2 b) { a.x -= b.x; a.y -= b.y; return a; }
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(__builtin_fmaf(a.x, b.x, -(a.y * b.y)), __builtin_fmaf(a.x, b.y, a.y * b.x));
}
__device__ __forceinline__ float2 cmulc(float2 a, float2 w) {  // a * conj(w)
  return make_float2(__builtin_fmaf(a.x, w.x, a.y * w.y), __builtin_fmaf(a.y, w.x, -(a.x * w.y)));
}
__device__ __forceinline__ float2 to_f2(double2 w) { return make_float2((float)w.x, (float)w.y); }
template <> __device__ __forceinline__ float zero_v<float>() { return 0.0f; }
template <> __device__ __forceinline__ float2 zero_v<float2>() { return make_float2(0.0f, 0.0f); }

// Element traits: real scalar, complex type (twiddles / complex products), complex-ness.
template <typename T> struct Elem;
template <> struct Elem<double> { using R = double; using C = double2; static constexpr bool cx = false; };
template <> struct Elem<double2> { using R = double; using C = double2; static constexpr bool cx = true; };
template <> struct Elem<float> { using R = float; using C = float2; static constexpr bool cx = false; };
template <> struct Elem<float2> { using R = float; using C = float2; static constexpr bool cx = true; };
// a twiddle from the fp64 tables in the complex type C of the data
template <typename C> __device__ __forceinline__ C twid(double2 w);
template <> __device__ __forceinline__ double2 twid<double2>(double2 w) { return w; }
template <> __device__ __forceinline__ float2 twid<float2>(double2 w) { return to_f2(w); }

// ---------------------------------------------------------------- butterflies
// tw = exp(-2 pi i k / 4096), k < 4096 (full circle); a stage of span 2h = 2^(s+1) uses
// w = exp(-2 pi i pos / 2h) = tw[pos << (11 - s)].
__device__ __forceinline__ void bfly_dit(double2& a, double2& b, const double2* __restrict__ tw, int k) {
  const double2 bw = cmul(b, tw[k]);
  b = a - bw;
  a = a + bw;
}
__device__ __forceinline__ void bfly_dit(double& a, double& b, const double2* __restrict__, int) {
  const double t = a;
  a = t + b;
  b = t - b;
}
__device__ __forceinline__ void bfly_dif(double2& a, double2& b, const double2* __restrict__ tw, int k) {
  const double2 d = a - b;
  a = a + b;
  b = cmulc(d, tw[k]);
}
__device__ __forceinline__ void bfly_dif(double& a, double& b, const double2* __restrict__, int) {
  const double t = a;
  a = t + b;
  b = t - b;
}
__device__ __forceinline__ void bfly_dit(float2& a, float2& b, const double2* __restrict__ tw, int k) {
  const float2 bw = cmul(b, to_f2(tw[k]));
  b = a - bw;
  a = a + bw;
}
__device__ __forceinline__ void bfly_dit(float& a, float& b, const double2* __restrict__, int) {
  const float t = a;
  a = t + b;
  b = t - b;
}
__device__ __forceinline__ void bfly_dif(float2& a, float2& b, const double2* __restrict__ tw, int k) {
  const float2 d = a - b;
  a = a + b;
  b = cmulc(d, to_f2(tw[k]));
}
__device__ __forceinline__ void bfly_dif(float& a, float& b, const double2* __restrict__, int) {
  const float t = a;
  a = t + b;
  b = t - b;
}

// v * exp(-2 pi i J / K) for compile-time J, K (K | 16): +-1 and +-i are free, the eighth roots
// cost 2 multiplies, the rest a constant complex multiply.  CONJ multiplies by the conjugate root.
template <int K, int J, bool CONJ>
__device__ __forceinline__ double2 mul_root(double2 v) {
  constexpr int j = (J * (16 / K)) & 15;              // exponent in units of 2 pi / 16
  constexpr double c16[16] = {1.0, 0.92387953251128673848, 0.70710678118654752440, 0.38268343236508978178,
                              0.0, -0.38268343236508978178, -0.70710678118654752440, -0.92387953251128673848,
                              -1.0, -0.92387953251128673848, -0.70710678118654752440, -0.38268343236508978178,
                              0.0, 0.38268343236508978178, 0.70710678118654752440, 0.92387953251128673848};
  constexpr double cr = c16[j];
  constexpr double ci = CONJ ? -c16[(j + 4) & 15] : c16[(j + 4) & 15];   // exp(-i t) = (cos t, cos(t + pi/2))
  if constexpr (j == 0) {
    return v;
  } else if constexpr (j == 8) {
    return make_double2(-v.x, -v.y);
  } else if constexpr (j == 4) {
    return CONJ ? make_double2(-v.y, v.x) : make_double2(v.y, -v.x);
  } else if constexpr (j == 12) {
    return CONJ ? make_double2(v.y, -v.x) : make_double2(-v.y, v.x);
  } else {
    return make_double2(__builtin_fma(cr, v.x, -(ci * v.y)), __builtin_fma(cr, v.y, ci * v.x));
  }
}

template <int K, int J, bool CONJ>
__device__ __forceinline__ float2 mul_root(float2 v) {
  constexpr int j = (J * (16 / K)) & 15;
  constexpr float c16[16] = {1.0f, 0.92387953251128673848f, 0.70710678118654752440f, 0.38268343236508978178f,
                             0.0f, -0.38268343236508978178f, -0.70710678118654752440f, -0.92387953251128673848f,
                             -1.0f, -0.92387953251128673848f, -0.70710678118654752440f, -0.38268343236508978178f,
                             0.0f, 0.38268343236508978178f, 0.70710678118654752440f, 0.92387953251128673848f};
  constexpr float cr = c16[j];
  constexpr float ci = CONJ ? -c16[(j + 4) & 15] : c16[(j + 4) & 15];
  if constexpr (j == 0) {
    return v;
  } else if constexpr (j == 8) {
    return make_float2(-v.x, -v.y);
  } else if constexpr (j == 4) {
    return CONJ ? make_float2(-v.y, v.x) : make_float2(v.y, -v.x);
  } else if constexpr (j == 12) {
    return CONJ ? make_float2(v.y, -v.x) : make_float2(-v.y, v.x);
  } else {
    return make_float2(__builtin_fmaf(cr, v.x, -(ci * v.y)), __builtin_fmaf(cr, v.y, ci * v.x));
  }
}

// DIT / DIF butterflies at stage Q2 of a register group for element pair (t, t | 2^Q2), given the
// group's base twiddle wb = exp(-2 pi i blo / 2^(S+Q2+1)) (unused when S == 0): the full twiddle is
// wb * exp(-2 pi i (t mod 2^Q2) / 2^(Q2+1)).
template <int S, int Q2, int T0, bool ADJ, typename C>
__device__ __forceinline__ void group_bfly_cx(C& a, C& b, C wb) {
  constexpr int J = T0 & ((1 << Q2) - 1);
  if constexpr (!ADJ) {
    C bw = mul_root<(2 << Q2), J, false>(b);
    if constexpr (S > 0) bw = cmul(bw, wb);
    b = a - bw;
    a = a + bw;
  } else {
    C d = a - b;
    a = a + b;
    if constexpr (S > 0) d = cmulc(d, wb);
    b = mul_root<(2 << Q2), J, true>(d);
  }
}
template <int S, int Q2, int T0, bool ADJ>
__device__ __forceinline__ void group_bfly(double2& a, double2& b, double2 wb) { group_bfly_cx<S, Q2, T0, ADJ>(a, b, wb); }
template <int S, int Q2, int T0, bool ADJ>
__device__ __forceinline__ void group_bfly(float2& a, float2& b, float2 wb) { group_bfly_cx<S, Q2, T0, ADJ>(a, b, wb); }
template <int S, int Q2, int T0, bool ADJ>
__device__ __forceinline__ void group_bfly(double& a, double& b, double2) {
  const double t = a;
  a = t + b;
  b = t - b;
}
template <int S, int Q2, int T0, bool ADJ>
__device__ __forceinline__ void group_bfly(float& a, float& b, float2) {
  const float t = a;
  a = t + b;
  b = t - b;
}

template <int Q2, int T, int RL, int S, bool ADJ, typename E, typename W>
__device__ __forceinline__ void stage_pairs(E* v, W wb) {
  if constexpr (T < (1 << RL)) {
    if constexpr (!(T & (1 << Q2))) group_bfly<S, Q2, T, ADJ>(v[T], v[T | (1 << Q2)], wb);
    stage_pairs<Q2, T + 1, RL, S, ADJ>(v, wb);
  }
}

template <int Q2, int RL, int S, bool ADJ, typename E, typename W>
__device__ __forceinline__ void stages_dit(E* v, const W* wb) {
  if constexpr (Q2 < RL) {
    stage_pairs<Q2, 0, RL, S, ADJ>(v, wb[Q2]);
    stages_dit<Q2 + 1, RL, S, ADJ>(v, wb);
  }
}
template <int Q2, int RL, int S, bool ADJ, typename E, typename W>
__device__ __forceinline__ void stages_dif(E* v, const W* wb) {
  if constexpr (Q2 >= 0) {
    stage_pairs<Q2, 0, RL, S, ADJ>(v, wb[Q2]);
    stages_dif<Q2 - 1, RL, S, ADJ>(v, wb);
  }
}

// One radix-2^RL register pass over stages [S, S+RL) of a length-2^P transform held in LDS
// (padded layout, base pointer s), run by TL = 2^P/16 threads (tt = thread index in the group).
// Twiddles: exp(-2 pi i pos / 2h) with pos = blo + (t mod 2^q2) 2^S factors into a per-group base
// tw[blo << (11 - S - q2)] (one table load per stage, none when S = 0) times a compile-time root.
template <int P, int S, int RL, bool ADJ, typename T>
__device__ __forceinline__ void lds_pass(T* s, int tt, const double2* __restrict__ tw) {
  constexpr int R = 1 << RL;
  constexpr int GPT = 16 / R;      // register groups per thread
  constexpr int TL = (1 << P) / 16;
#pragma unroll
  for (int j = 0; j < GPT; ++j) {
    const int q = tt + j * TL;
    const int blo = q & ((1 << S) - 1);
    const int base = blo + ((q >> S) << (S + RL));
    using C = typename Elem<T>::C;
    C wb[RL];
#pragma unroll
    for (int q2 = 0; q2 < RL; ++q2) {
      if constexpr (S > 0 && Elem<T>::cx) wb[q2] = twid<C>(tw[blo << (11 - S - q2)]);
      else wb[q2] = twid<C>(make_double2(1.0, 0.0));
    }
    T v[R];
#pragma unroll
    for (int t = 0; t < R; ++t) v[t] = s[padi(base + (t << S))];
    if constexpr (!ADJ) stages_dit<0, RL, S, false>(v, wb);
    else stages_dif<RL - 1, RL, S, true>(v, wb);
#pragma unroll
    for (int t = 0; t < R; ++t) s[padi(base + (t << S))] = v[t];
  }
}

template <int P, int S, typename T>
__device__ __forceinline__ void lds_dit_all(T* s, int tt, const double2* __restrict__ tw) {
  if constexpr (S < P) {
    constexpr int RL = (P - S) < 4 ? (P - S) : 4;
    lds_pass<P, S, RL, false>(s, tt, tw);
    __syncthreads();
    lds_dit_all<P, S + 4>(s, tt, tw);
  }
}

template <int P, int S, typename T>
__device__ __forceinline__ void lds_dif_all(T* s, int tt, const double2* __restrict__ tw) {
  constexpr int RL = (P - S) < 4 ? (P - S) : 4;
  lds_pass<P, S, RL, true>(s, tt, tw);
  __syncthreads();
  if constexpr (S >= 4) lds_dif_all<P, S - 4>(s, tt, tw);
}

// Full in-LDS transform of length 2^P (4 <= P <= 12).  Caller syncs before; ends with a sync.
template <int P, bool ADJ, typename T>
__device__ __forceinline__ void lds_transform(T* s, int tt, const double2* __restrict__ tw) {
  static_assert(P >= 4 && P <= 12, "in-LDS transforms cover 2^4..2^12");
  if constexpr (ADJ) {
    lds_dif_all<P, ((P - 1) / 4) * 4>(s, tt, tw);
  } else {
    lds_dit_all<P, 0>(s, tt, tw);
  }
}

// f(std::integral_constant<int, I>{}) for I = B .. E-1 (compile-time loop index)
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

// ---------------------------------------------------------------- register-resident passes
// The radix-2^RL pass of lds_pass on a thread's 16 elements held in registers: group j of the thread
// (q = tt + j TL) owns the elements at pass_pos<P, S, RL>(tt, j, t), t < 2^RL, in v[j 2^RL + t].
// Same butterflies and twiddles as lds_pass, so the same results; the data only goes through LDS to
// change hands between passes (reg_exchange), not before / after every pass.
template <int P, int S> struct PassRL { static constexpr int value = (P - S) < 4 ? (P - S) : 4; };
template <int P> struct LastPass { static constexpr int S = ((P - 1) / 4) * 4; };

template <int P, int S, int RL>
__device__ __forceinline__ int pass_pos(int tt, int j, int t) {
  constexpr int TL = (1 << P) / 16;
  const int q = tt + j * TL;
  const int blo = q & ((1 << S) - 1);
  return blo + ((q >> S) << (S + RL)) + (t << S);
}

template <int P, int S, int RL, bool ADJ, typename T>
__device__ __forceinline__ void reg_pass(T* v, int tt, const double2* __restrict__ tw) {
  constexpr int R = 1 << RL;
  constexpr int GPT = 16 / R;
  constexpr int TL = (1 << P) / 16;
#pragma unroll
  for (int j = 0; j < GPT; ++j) {
    const int q = tt + j * TL;
    const int blo = q & ((1 << S) - 1);
    using C = typename Elem<T>::C;
    C wb[RL];
#pragma unroll
    for (int q2 = 0; q2 < RL; ++q2) {
      if constexpr (S > 0 && Elem<T>::cx) wb[q2] = twid<C>(tw[blo << (11 - S - q2)]);
      else wb[q2] = twid<C>(make_double2(1.0, 0.0));
    }
    if constexpr (!ADJ) stages_dit<0, RL, S, false>(v + j * R, wb);
    else stages_dif<RL - 1, RL, S, true>(v + j * R, wb);
  }
}

// Hand the 16 elements over from pass (SA, RLA) to pass (SB, RLB) through the thread's transform image
// `col` in LDS.  PAD = false: positions as they are (column images of stride = 1 mod 16 with
// consecutive lanes on consecutive columns are conflict-free); PAD = true: padi(position) (one
// transform per workgroup, lanes along the transform).  Leading barrier: readers of the previous
// exchange are done.
template <bool PAD>
__device__ __forceinline__ int img_pos(int pos) { return PAD ? padi(pos) : pos; }

template <int P, int SA, int RLA, int SB, int RLB, bool PAD, typename T>
__device__ __forceinline__ void reg_exchange(T* v, T* col, int tt) {
  constexpr int RA = 1 << RLA, RB = 1 << RLB;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 16 / RA; ++j)
#pragma unroll
    for (int t = 0; t < RA; ++t) col[img_pos<PAD>(pass_pos<P, SA, RLA>(tt, j, t))] = v[j * RA + t];
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 16 / RB; ++j)
#pragma unroll
    for (int t = 0; t < RB; ++t) v[j * RB + t] = col[img_pos<PAD>(pass_pos<P, SB, RLB>(tt, j, t))];
}

// The same hand-over for complex elements through a real (8-byte) image of half the size: real parts,
// then imaginary parts.  Halves the LDS a workgroup holds (more workgroups per CU) for two more barriers.
template <int P, int SA, int RLA, int SB, int RLB, bool PAD>
__device__ __forceinline__ void reg_exchange_split(double2* v, double* img, int tt) {
  constexpr int RA = 1 << RLA, RB = 1 << RLB;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 16 / RA; ++j)
#pragma unroll
    for (int t = 0; t < RA; ++t) img[img_pos<PAD>(pass_pos<P, SA, RLA>(tt, j, t))] = v[j * RA + t].x;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 16 / RB; ++j)
#pragma unroll
    for (int t = 0; t < RB; ++t) v[j * RB + t].x = img[img_pos<PAD>(pass_pos<P, SB, RLB>(tt, j, t))];
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 16 / RA; ++j)
#pragma unroll
    for (int t = 0; t < RA; ++t) img[img_pos<PAD>(pass_pos<P, SA, RLA>(tt, j, t))] = v[j * RA + t].y;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 16 / RB; ++j)
#pragma unroll
    for (int t = 0; t < RB; ++t) v[j * RB + t].y = img[img_pos<PAD>(pass_pos<P, SB, RLB>(tt, j, t))];
}

// hand-over through an image of element type I: T itself, or (I = double, T = double2) split halves
template <int P, int SA, int RLA, int SB, int RLB, bool PAD, typename T, typename I>
__device__ __forceinline__ void reg_handover(T* v, I* img, int tt) {
  if constexpr (std::is_same<T, I>::value) reg_exchange<P, SA, RLA, SB, RLB, PAD>(v, img, tt);
  else reg_exchange_split<P, SA, RLA, SB, RLB, PAD>(v, img, tt);
}

// forward (DIT) passes S, S + 4, ... < P
template <int P, int S, bool PAD, typename T, typename I>
__device__ __forceinline__ void fwd_reg_passes(T* v, I* col, int tt, const double2* __restrict__ tw) {
  constexpr int RL = PassRL<P, S>::value;
  if constexpr (S > 0) reg_handover<P, S - 4, 4, S, RL, PAD>(v, col, tt);
  reg_pass<P, S, RL, false>(v, tt, tw);
  if constexpr (S + 4 < P) fwd_reg_passes<P, S + 4, PAD>(v, col, tt, tw);
}

// adjoint (DIF) passes S, S - 4, ..., 0 (start at LastPass<P>::S: the elements the forward passes end on)
template <int P, int S, bool PAD, typename T, typename I>
__device__ __forceinline__ void adj_reg_passes(T* v, I* col, int tt, const double2* __restrict__ tw) {
  constexpr int RL = PassRL<P, S>::value;
  reg_pass<P, S, RL, true>(v, tt, tw);
  if constexpr (S >= 4) {
    reg_handover<P, S, RL, S - 4, 4, PAD>(v, col, tt);
    adj_reg_passes<P, S - 4, PAD>(v, col, tt, tw);
  }
}

// 4-bit bit reversal as a compile-time constant
template <int T4> struct Brev4 {
  static constexpr unsigned value = ((T4 & 1) << 3) | ((T4 & 2) << 1) | ((T4 & 4) >> 1) | ((T4 & 8) >> 3);
};

// ---------------------------------------------------------------- reductions
__device__ __forceinline__ double shfl_xor_d(double v, int o) { return __shfl_xor(v, o, 64); }
__device__ __forceinline__ double2 shfl_xor_d(double2 v, int o) {
  return make_double2(__shfl_xor(v.x, o, 64), __shfl_xor(v.y, o, 64));
}
__device__ __forceinline__ float shfl_xor_d(float v, int o) { return __shfl_xor(v, o, 64); }
__device__ __forceinline__ float2 shfl_xor_d(float2 v, int o) {
  return make_float2(__shfl_xor(v.x, o, 64), __shfl_xor(v.y, o, 64));
}

// Sum over a group of TL consecutive threads (TL a power of two, groups aligned to TL).
// Every thread of the group receives the total.  `red` is LDS scratch of >= kWG/64 entries.
// Must be called by all threads of the workgroup (contains barriers when TL > 64).
template <int TL, typename T>
__device__ __forceinline__ T group_sum(T v, T* red) {
  if constexpr (TL <= 64) {
#pragma unroll
    for (int o = TL / 2; o > 0; o >>= 1) v += shfl_xor_d(v, o);
    return v;
  } else {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += shfl_xor_d(v, o);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    constexpr int NW = TL / 64;
    const int g0 = (w / NW) * NW;
    T tot = red[g0];
#pragma unroll
    for (int i = 1; i < NW; ++i) tot += red[g0 + i];
    __syncthreads();
    return tot;
  }
}

// Whole-workgroup sum of a double (result valid in every thread).
__device__ __forceinline__ double block_sum(double v, double* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  double tot = 0.0;
#pragma unroll
  for (int i = 0; i < kWG / 64; ++i) tot += red[i];
  __syncthreads();
  return tot;
}

__device__ __forceinline__ unsigned brev_bits(unsigned u, int bits) {
  return bits == 0 ? 0u : (__builtin_bitreverse32(u) >> (32 - bits));
}

// low 32 bits of a 24 x 24-bit product (full-rate v_mul_u32_u24; v_mul_lo_u32 is quarter rate):
// brev_m(i) and z_j mod n are < 2^24, and only the low m <= 24 bits of the product are used
__device__ __forceinline__ unsigned mul_u24(unsigned a, unsigned b) {
  unsigned r;
  asm("v_mul_u32_u24 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// 16-byte write-through stores (cache policy sc1) into a buffer whose base is wave-uniform: the line
// leaves the XCD's L2 with the store, so the kernel's end has no dirty bytes to write back before a
// dependent launch can start (MI355X_MICROARCH.md price list, "boundary": + B / 6 TB/s for B dirty
// bytes; "publish-large": write-through wins for tens of KB per workgroup).  Element offsets are
// 32-bit byte offsets from the base (a buffer of < 2^28 double2 per base).
struct WtStore {
  __amdgpu_buffer_rsrc_t r;
  __device__ __forceinline__ explicit WtStore(const void* base)
      : r(__builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, -1, 0x00020000)) {}
  __device__ __forceinline__ void put(unsigned idx, double2 v) const {
    typedef int v4i __attribute__((ext_vector_type(4)));
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i, v), r, (int)(idx << 4), 0, 16 /* sc1 */);
  }
};

// Natural-order rank-1 lattice coordinate of point i (brev = brev_m(i), zm = z_j mod n):
//   x = ((brev z_j mod n) / n + shift_j) % 1   -- the host generator's value (seqs.Lattice), bit for bit
__device__ __forceinline__ double lattice_coord(unsigned brev, unsigned zm, unsigned mask, double inv_n, double sh) {
  return __builtin_amdgcn_fract(__builtin_fma((double)(mul_u24(brev, zm) & mask), inv_n, sh));
}

// Inter-pass twiddle of a length-2^m transform split as N1 = 2^m1 rows of N2 = 2^P2:
//   w_n^e, e < n, from the two-level table  twm[e mod N2] * tw[(e >> P2) << (12 - m1)]
__device__ __forceinline__ double2 inter_tw(unsigned e, int P2, int m1, const double2* __restrict__ tw,
                                            const double2* __restrict__ twm) {
  return cmul(twm[e & ((1u << P2) - 1)], tw[(e >> P2) << (kTileLog - m1)]);
}

// Twiddles w_n^{j1 e_k} of the 16 elements e_k = tid + 256 k of a thread whose workgroup holds ONE row
// (row index u, j1 = brev_m1(u) uniform): base = w^{j1 tid} (one per-lane table pair) times the
// uniform step w^{j1 256 k} (broadcast table loads); exponents add exactly.
struct RowTwiddle {
  double2 base;
  unsigned j1;
  __device__ __forceinline__ RowTwiddle(unsigned u, int tid, int P2, int m1, const double2* __restrict__ tw,
                                        const double2* __restrict__ twm) {
    j1 = brev_bits(u, m1);
    base = inter_tw(j1 * (unsigned)tid, P2, m1, tw, twm);
  }
  __device__ __forceinline__ double2 at(int k, int P2, int m1, const double2* __restrict__ tw,
                                        const double2* __restrict__ twm) const {
    return cmul(base, inter_tw(j1 * 256u * (unsigned)k, P2, m1, tw, twm));
  }
};

// ---------------------------------------------------------------- generic element I/O
template <typename T> __device__ __forceinline__ T load_in(const void* p, int64_t i, int in_real);
template <> __device__ __forceinline__ double2 load_in<double2>(const void* p, int64_t i, int in_real) {
  if (in_real) return make_double2(static_cast<const double*>(p)[i], 0.0);
  return static_cast<const double2*>(p)[i];
}
template <> __device__ __forceinline__ double load_in<double>(const void* p, int64_t i, int) {
  return static_cast<const double*>(p)[i];
}

__device__ __forceinline__ void store_out(void* p, int64_t i, double2 v, int out_real) {
  if (out_real) static_cast<double*>(p)[i] = v.x;
  else static_cast<double2*>(p)[i] = v;
}
__device__ __forceinline__ void store_out(void* p, int64_t i, double v, int) { static_cast<double*>(p)[i] = v; }

template <> __device__ __forceinline__ float2 load_in<float2>(const void* p, int64_t i, int in_real) {
  if (in_real) return make_float2(static_cast<const float*>(p)[i], 0.0f);
  return static_cast<const float2*>(p)[i];
}
template <> __device__ __forceinline__ float load_in<float>(const void* p, int64_t i, int) {
  return static_cast<const float*>(p)[i];
}
__device__ __forceinline__ void store_out(void* p, int64_t i, float2 v, int out_real) {
  if (out_real) static_cast<float*>(p)[i] = v.x;
  else static_cast<float2*>(p)[i] = v;
}
__device__ __forceinline__ void store_out(void* p, int64_t i, float v, int) { static_cast<float*>(p)[i] = v; }

// v * s in the element's own precision
__device__ __forceinline__ double scaled(double v, double s) { return v * s; }
__device__ __forceinline__ double2 scaled(double2 v, double s) { return v * s; }
__device__ __forceinline__ float scaled(float v, double s) { return v * (float)s; }
__device__ __forceinline__ float2 scaled(float2 v, double s) { return v * s; }

template <typename T> __device__ __forceinline__ T tw_mul(T v, double2 w, bool conj);
template <> __device__ __forceinline__ double2 tw_mul<double2>(double2 v, double2 w, bool conj) {
  return conj ? cmulc(v, w) : cmul(v, w);
}
template <> __device__ __forceinline__ double tw_mul<double>(double v, double2, bool) { return v; }
template <> __device__ __forceinline__ float2 tw_mul<float2>(float2 v, double2 w, bool conj) {
  return conj ? cmulc(v, to_f2(w)) : cmul(v, to_f2(w));
}
template <> __device__ __forceinline__ float tw_mul<float>(float v, double2, bool) { return v; }


// Centre (optional) -> in-LDS transform -> add the mean back to bin 0, for one length-2^P
// transform at LDS base s run by TL = 2^P/16 threads.  Caller syncs before; ends synced.
// The mean-centring mirrors AbstractFastGP.ft/ift (abstract_fast_gp.py:209-211, 225-227).
template <int P, bool ADJ, typename T>
__device__ __forceinline__ void center_transform(T* s, int tt, int stable, T* red, const double2* __restrict__ tw) {
  constexpr int L = 1 << P;
  constexpr int TL = L / 16;
  T mean = zero_v<T>();
  if (stable) {
    T acc = zero_v<T>();
#pragma unroll
    for (int j = 0; j < 16; ++j) acc += s[padi(tt + j * TL)];
    mean = group_sum<TL>(acc, red) * (1.0 / L);
#pragma unroll
    for (int j = 0; j < 16; ++j) s[padi(tt + j * TL)] -= mean;
    __syncthreads();
  }
  lds_transform<P, ADJ>(s, tt, tw);
  if (stable && tt == 0) s[0] += mean * (double)L;
  __syncthreads();
}

// ---------------------------------------------------------------- centring folded into the load
// Whole-workgroup sum of a T (result in every thread).
template <typename T>
__device__ __forceinline__ T block_sum_t(T v, T* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += shfl_xor_d(v, o);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  T tot = red[0];
#pragma unroll
  for (int i = 1; i < kWG / 64; ++i) tot += red[i];
  __syncthreads();
  return tot;
}

// Column sums of a column tile (C columns of a 4096-element tile; the thread with index tid staged
// elements of column tid mod C).  column_partials() stores per-wave partials in `part` ((C < 64 ?
// 4 C : kWG) entries) and synchronises; column_total(c) then returns the sum of column c.
template <int C, typename T>
__device__ __forceinline__ void column_partials(T v, T* part) {
  if constexpr (C < 64) {
#pragma unroll
    for (int o = C; o < 64; o <<= 1) v += shfl_xor_d(v, o);
    if ((threadIdx.x & 63) < C) part[(threadIdx.x >> 6) * C + (threadIdx.x & 63)] = v;
  } else {
    part[threadIdx.x] = v;
  }
  __syncthreads();
}
template <int C, typename T>
__device__ __forceinline__ T column_total(int c, const T* part) {
  constexpr int K = C < 64 ? kWG / 64 : kWG / C;
  constexpr int STRIDE = C;
  T tot = part[c];
#pragma unroll
  for (int i = 1; i < K; ++i) tot += part[c + i * STRIDE];
  return tot;
}
template <int C> struct ColPart { static constexpr int size = C < 64 ? 4 * C : kWG; };

// Transform of data staged in LDS with its mean already removed; adds mean * L back to bin 0.
template <int P, bool ADJ, typename T>
__device__ __forceinline__ void transform_add_mean(T* s, int tt, T mean, const double2* __restrict__ tw) {
  lds_transform<P, ADJ>(s, tt, tw);
  if (tt == 0) s[0] += mean * (double)(1 << P);
  __syncthreads();
}

// ---------------------------------------------------------------- Walsh kernels of order 2..4
// Per-dimension part of FastGPDigitalNetB2 of order a = alpha - beta - kappa in 2..4
// (fast_gp_digital_net_b2.py:295-301: qmcpy.kernel_methods.weighted_walsh_funcs(a, delta, t) - 1):
//   omega_a(x) = sum_{k >= 1} 2^(-mu_a(k)) wal_k(x),   x = delta / 2^t,
// mu_a(k) = sum_{i <= min(a, v)} (a_i + 1) for k = 2^a_1 + ... + 2^a_v, a_1 > ... > a_v (Dick's weight).
// With beta = -floor(log2 x) and t1 = 2^-beta the series sums to
//   omega_2 = -beta x + 5/2 (1 - t1) - 1
//   omega_3 =  beta x^2 - 5 (1 - t1) x + 43/18 (1 - t1^2) - 1
// and omega_4 by the digit recursion (y_a = s_a 2^-(a+1), s_a = (-1)^(bit a+1 of x), e_r = elementary
// symmetric sums of the y above the current digit, seeded with the all-zero tail a >= t):
//   omega_a = sum_{r < a} e_r(all) + sum_{b < beta} s_b e_{a-1}(y_{>b}) / 2.
// omega_a(0) = 3/2, 25/18, 407/294.  (tests/test_oracle_golden.py checks the closed forms and the
// recursion against the truncated series itself.)
__device__ __forceinline__ double walsh_omega(int ord, unsigned long long delta, int t) {
  if (delta == 0ull) return ord == 2 ? 1.5 : (ord == 3 ? 25.0 / 18.0 : 407.0 / 294.0);
  const int beta = t - (63 - __clzll((long long)delta));
  const double x = ldexp((double)delta, -t);
  const double t1 = ldexp(1.0, -beta), b = (double)beta;
  if (ord == 2) return __builtin_fma(-b, x, 2.5 * (1.0 - t1)) - 1.0;
  if (ord == 3)
    return __builtin_fma(b * x, x, __builtin_fma(-5.0 * (1.0 - t1), x, (43.0 / 18.0) * __builtin_fma(-t1, t1, 1.0))) - 1.0;
  const double c = ldexp(1.0, -(t + 1));
  double e1 = 2.0 * c, e2 = (4.0 / 3.0) * c * c, e3 = (8.0 / 21.0) * c * c * c, E = 0.0;
  for (int a = t - 1; a >= 0; --a) {
    const double s = ((delta >> (t - 1 - a)) & 1ull) ? -1.0 : 1.0;
    if (a < beta) E = __builtin_fma(0.5 * s, e3, E);
    const double y = ldexp(s, -(a + 1));
    e3 = __builtin_fma(y, e2, e3);
    e2 = __builtin_fma(y, e1, e2);
    e1 += y;
  }
  return e1 + e2 + e3 + E;
}

// ---------------------------------------------------------------- kernel parts (shared by the fit,
// parts and multitask kernels)
// torch.remainder(v, 1.0) for floating point (fmod, then shift negative results by the divisor)
__device__ __forceinline__ double mod1(double v) {
  double r = fmod(v, 1.0);
  if (r != 0.0 && r < 0.0) r += 1.0;
  return r;
}

// Even Bernoulli polynomial B_order(x) as a polynomial in u = x (x - 1) (the even B_2a are symmetric
// about 1/2):  B2 = u + 1/6,  B4 = u^2 - 1/30,  B6 = u^2 (u - 1/2) + 1/42,
// B8 = u^2 (u (u - 4/3) + 2/3) - 1/30  -- 2 / 4 / 5 operations instead of Horner's 2 / 4 / 6 / 8 in x
// (the fit row kernels are FP64-VALU bound and evaluate one per element and dimension).  Every
// multiply-add is an explicit fma, so the value does not depend on the compiler's contraction choices
// in the inlining context: the parts array (k_lattice_parts) and the parts regenerated inside the fit
// kernels are bit-identical.
__device__ __forceinline__ double bernoulli(int order, double x) {
  const double u = __builtin_fma(x, x, -x);
  switch (order) {
    case 2: return u + 1.0 / 6.0;
    case 4: return __builtin_fma(u, u, -1.0 / 30.0);
    case 6: return __builtin_fma(u * u, u - 0.5, 1.0 / 42.0);
    case 8: return __builtin_fma(u * u, __builtin_fma(u, u - 4.0 / 3.0, 2.0 / 3.0), -1.0 / 30.0);
    default: return __builtin_nan("");
  }
}

// Order-1 Walsh part for an XOR distance (fast_gp_digital_net_b2.py:297-298).
__device__ __forceinline__ double walsh1(unsigned long long delta, int t) {
  if (delta == 0ull) return 6.0 * (1.0 / 6.0 - 0.0);
  const int fl = 63 - __clzll((long long)delta);   // floor(log2(delta)), exact
  return 6.0 * (1.0 / 6.0 - ldexp(1.0, fl - t - 1));
}

}  // namespace fgp
