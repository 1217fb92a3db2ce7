// Read bandwidth of a re-read working set the size of the spectral fit iteration's (spectra + Y of C4:
// 168 MB), to price k_spec_tile against what the chip streams for this footprint.  Variants:
//   reg<U>:  global_load_dwordx4 into registers, U independent 16-B loads in flight per lane, grid-stride;
//   lds<R>:  LDS-DMA (global_load_lds_dwordx4) ring of R 16-KiB slots per 256-thread workgroup, the
//            k_spec_tile pattern (counted vmcnt waits, raw barriers), two workgroups per CU.
// Each launch reads the whole buffer once; launches run back to back (the buffer stays in the 256 MiB
// Infinity Cache between them if it can).  Prints one JSON line per variant.
//
//   hipcc -O3 --offload-arch=gfx950 tools/stream_microbench.hip -o tools/stream_microbench && ./tools/stream_microbench [MB]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                \
  do {                                                                       \
    hipError_t e = (x);                                                      \
    if (e != hipSuccess) {                                                   \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                 \
      exit(1);                                                               \
    }                                                                        \
  } while (0)

template <int U>
__global__ __launch_bounds__(256) void k_reg(const double4* __restrict__ p, long n4, double* out) {
  double s = 0.0;
  const long stride = (long)gridDim.x * 256;
  long i = (long)blockIdx.x * 256 + threadIdx.x;
  for (; i + (U - 1) * stride < n4; i += U * stride) {
    double4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = p[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) s += v[u].x + v[u].y + v[u].z + v[u].w;
  }
  for (; i < n4; i += stride) s += p[i].x;
  if (s == 123.456) out[blockIdx.x] = s;   // keep the loads
}

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void glb_void;

// R-slot ring of 16 KiB per workgroup: each wave issues 4 x 1 KiB per slot; chunk c of workgroup b is the
// 16 KiB at ((c * gridDim.x) + b) * 16 KiB (consecutive workgroups read consecutive chunks)
template <int R>
__global__ __launch_bounds__(256, 2) void k_lds(const char* __restrict__ p, long chunks, double* out) {
  extern __shared__ double lds[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long per = chunks / gridDim.x;
  double s = 0.0;
  auto issue = [&](long c, int slot) {
    const char* src = p + ((c * gridDim.x) + blockIdx.x) * 16384 + (w * 4) * 1024 + lane * 16;
#pragma unroll
    for (int t = 0; t < 4; ++t)
      __builtin_amdgcn_global_load_lds((glb_void*)(src + t * 1024), (lds_void*)(lds + slot * 2048 + (w * 4 + t) * 128),
                                       16, 0, 0);
  };
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  for (int c = 0; c < R - 1; ++c)
    if (c < per) issue(c, c);
  for (long c = 0; c < per; ++c) {
    if (R == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if (R == 3) { if (c + 1 < per) asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); else asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
    else { if (c + 2 < per) asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); else asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (c + R - 1 < per) issue(c + R - 1, (int)((c + R - 1) % R));
    const double* b = lds + (c % R) * 2048;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += b[threadIdx.x + 256 * k];
  }
  if (s == 123.456) out[blockIdx.x] = s;
}

template <typename F>
static double time_us(F launch, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) launch();
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) launch();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return 1e3 * ms / reps;
}

int main(int argc, char** argv) {
  const double mb = argc > 1 ? atof(argv[1]) : 168.0;
  const long chunks = (long)(mb * 1e6 / 16384) / 1024 * 1024;   // whole 16 KiB chunks, a multiple of 1024
  const long bytes = chunks * 16384;
  char* p;
  double* out;
  CK(hipMalloc(&p, bytes));
  CK(hipMalloc(&out, 1 << 20));
  CK(hipMemset(p, 1, bytes));
  auto rep = [&](const char* name, int grid, double us) {
    printf("{\"variant\": \"%s\", \"grid\": %d, \"MB\": %.1f, \"us\": %.2f, \"GBps\": %.0f}\n", name, grid, bytes / 1e6, us,
           bytes / us / 1e3);
    fflush(stdout);
  };
  const long n4 = bytes / 32;
  for (int grid : {512, 1024, 2048, 4096}) {
    rep("reg<2>", grid, time_us([&] { k_reg<2><<<grid, 256>>>((const double4*)p, n4, out); }, 20));
    rep("reg<4>", grid, time_us([&] { k_reg<4><<<grid, 256>>>((const double4*)p, n4, out); }, 20));
    rep("reg<8>", grid, time_us([&] { k_reg<8><<<grid, 256>>>((const double4*)p, n4, out); }, 20));
  }
  for (int grid : {512, 1024}) {
    hipFuncSetAttribute((const void*)k_lds<4>, hipFuncAttributeMaxDynamicSharedMemorySize, 4 * 16384);
    rep("lds<2>", grid, time_us([&] { k_lds<2><<<grid, 256, 2 * 16384>>>(p, chunks, out); }, 20));
    rep("lds<3>", grid, time_us([&] { k_lds<3><<<grid, 256, 3 * 16384>>>(p, chunks, out); }, 20));
    rep("lds<4>", grid, time_us([&] { k_lds<4><<<grid, 256, 4 * 16384>>>(p, chunks, out); }, 20));
  }
  CK(hipFree(p));
  CK(hipFree(out));
  return 0;
}
