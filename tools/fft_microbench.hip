// Microbenchmark of the transform pass structure (tuning aid, not product code).
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -I fastgaussianprocesses_amd/csrc tools/fft_microbench.hip -o /tmp/fmb
// Times, on G x 2^20 complex128 data: a 16-B copy, the row pass (load/store only, + LDS transform,
// + inter-pass twiddle by table lookup, + twiddle by per-thread recurrence) and the column pass.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "fgp_common.h"

using namespace fgp;

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e = (x);                                                           \
    if (e != hipSuccess) {                                                        \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

__global__ void k_init(double2* tw, int logn, int cnt) {
  int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= cnt) return;
  double s, c;
  sincospi(ldexp((double)(2 * k), -logn), &s, &c);
  tw[k] = make_double2(c, -s);
}

__global__ __launch_bounds__(256) void k_copy(const double2* __restrict__ in, double2* __restrict__ out, int64_t cnt) {
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  for (; i < cnt; i += (int64_t)gridDim.x * 256) out[i] = in[i];
}

// MODE 0: load/store through LDS only; 1: + transform; 2: + table twiddle; 3: + recurrence twiddle
template <int MODE>
__global__ __launch_bounds__(256) void k_rows_v(const double2* __restrict__ in, double2* __restrict__ out, int m,
                                                const double2* __restrict__ tw, const double2* __restrict__ twm) {
  constexpr int P2 = 12, N2 = 4096;
  __shared__ double2 lds[kTile + kTile / 16];
  __shared__ double2 red[4];
  const int m1 = m - P2;
  const int64_t n = (int64_t)1 << m;
  const int64_t tiles = n >> 12;
  const int64_t b = blockIdx.x / tiles;
  const int row0 = (int)(blockIdx.x % tiles);
  const int tid = threadIdx.x;
  const double2* src = in + b * n + (int64_t)row0 * N2;
#pragma unroll
  for (int k = 0; k < 16; ++k) lds[padi(tid + k * 256)] = src[tid + k * 256];
  __syncthreads();
  if (MODE >= 1) center_transform<P2, false>(lds, tid, 1, red, tw);
  double2* dst = out + b * n + (int64_t)row0 * N2;
  const unsigned j1 = brev_bits((unsigned)row0, m1);
  double2 w = make_double2(1.0, 0.0), step = make_double2(1.0, 0.0);
  if (MODE == 3) {
    const unsigned e0 = j1 * (unsigned)tid, es = j1 * 256u;
    w = cmul(twm[e0 & (N2 - 1)], tw[(e0 >> P2) << (kTileLog - m1)]);
    step = cmul(twm[es & (N2 - 1)], tw[(es >> P2) << (kTileLog - m1)]);
  }
  double2 base = make_double2(1.0, 0.0);
  if (MODE == 4) {
    const unsigned e0 = j1 * (unsigned)tid;
    base = cmul(twm[e0 & (N2 - 1)], tw[(e0 >> P2) << (kTileLog - m1)]);
  }
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int e = tid + k * 256;
    double2 v = lds[padi(e)];
    if (MODE == 2) {
      const unsigned ex = j1 * (unsigned)e;
      v = cmul(v, cmul(twm[ex & (N2 - 1)], tw[(ex >> P2) << (kTileLog - m1)]));
    } else if (MODE == 3) {
      v = cmul(v, w);
      w = cmul(w, step);
    } else if (MODE == 4) {   // base (per lane) x uniform step^k (broadcast table loads)
      const unsigned es = (j1 * 256u * (unsigned)k) & ((1u << m) - 1);
      v = cmul(v, cmul(base, cmul(twm[es & (N2 - 1)], tw[(es >> P2) << (kTileLog - m1)])));
    }
    dst[e] = v;
  }
}

// column pass, N1 = 256 (m = 20), C = 16 columns per workgroup
template <int MODE>
__global__ __launch_bounds__(256) void k_cols_v(const double2* __restrict__ in, double2* __restrict__ out, int m,
                                                const double2* __restrict__ tw) {
  constexpr int P1 = 8, N1 = 256, C = 16, CS = 273, TL = 16;
  __shared__ double2 lds[kLds];
  __shared__ double2 red[4];
  const int64_t n = (int64_t)1 << m, N2 = n >> P1;
  const int64_t tiles = n >> 12;
  const int64_t b = blockIdx.x / tiles;
  const int64_t c0 = (blockIdx.x % tiles) * C;
  const int tid = threadIdx.x;
  const double2* src = in + b * n + c0;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int e = tid + k * 256;
    lds[(e % C) * CS + padi(e / C)] = src[(int64_t)(e / C) * N2 + e % C];
  }
  __syncthreads();
  if (MODE >= 1) center_transform<P1, false>(lds + (tid / TL) * CS, tid % TL, 1, red, tw);
  double2* dst = out + b * n + c0;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int e = tid + k * 256;
    dst[(int64_t)(e / C) * N2 + e % C] = lds[(e % C) * CS + padi(e / C)];
  }
}

int main() {
  const int m = 20, G = 8;
  const int64_t n = (int64_t)1 << m, tot = n * G;
  double2 *a, *bb, *tw, *twm;
  CK(hipMalloc(&a, tot * 16));
  CK(hipMalloc(&bb, tot * 16));
  CK(hipMalloc(&tw, 4096 * 16));
  CK(hipMalloc(&twm, 4096 * 16));
  CK(hipMemset(a, 0, tot * 16));
  k_init<<<16, 256>>>(tw, 12, 4096);
  k_init<<<16, 256>>>(twm, m, 4096);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const unsigned grid = (unsigned)(G * (n >> 12));
  auto timeit = [&](const char* name, auto launch) {
    for (int i = 0; i < 3; ++i) launch();
    CK(hipDeviceSynchronize());
    const int reps = 20;
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / reps;
    printf("%-40s %9.1f us  %7.0f GB/s (2 x %.0f MB)\n", name, us, 2.0 * tot * 16 / (us * 1e3), tot * 16 / 1e6);
    return 0;
  };
  timeit("copy 16B grid-stride (2048 WG)", [&] { k_copy<<<2048, 256>>>(a, bb, tot); });
  timeit("copy 16B one elem/thread", [&] { k_copy<<<(unsigned)(tot / 256), 256>>>(a, bb, tot); });
  timeit("rows: load/store via LDS", [&] { k_rows_v<0><<<grid, 256>>>(a, bb, m, tw, twm); });
  timeit("rows: + transform", [&] { k_rows_v<1><<<grid, 256>>>(a, bb, m, tw, twm); });
  timeit("rows: + transform + table twiddle", [&] { k_rows_v<2><<<grid, 256>>>(a, bb, m, tw, twm); });
  timeit("rows: + transform + recurrence twiddle", [&] { k_rows_v<3><<<grid, 256>>>(a, bb, m, tw, twm); });
  timeit("rows: + transform + base*step twiddle", [&] { k_rows_v<4><<<grid, 256>>>(a, bb, m, tw, twm); });
  timeit("cols: load/store via LDS", [&] { k_cols_v<0><<<grid, 256>>>(a, bb, m, tw); });
  timeit("cols: + transform", [&] { k_cols_v<1><<<grid, 256>>>(a, bb, m, tw); });
  return 0;
}
