// Laboratory for the spectral fit iteration of C4 (k_spec_tile<5, 2>): n = 2^20 lattice, d = 5, G = 8
// problems sharing one set of 2^d spectra.  Standalone (synthetic spectra / Y of the real layout, the real
// per-frequency arithmetic of fgp_spectral.hip's spec_terms), per-block partials only (no reduction / Rprop
// hand-off), so kernel structures can be compared on the device clock of back-to-back launches.
//
//   hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 tools/spec_lab.hip -o tools/spec_lab
//   ./tools/spec_lab            one JSON line per variant
//
// Variants (template parameters of k_lab):
//   RING     LDS ring slots (chunks); RING - 1 chunks in flight under a chunk's compute
//   DYN      blocks handed out by an atomic counter (per-block partials at the block's index: the same
//            arithmetic whichever workgroup runs a block) vs a fixed block per workgroup
//   SADDR    DMA source = wave-uniform base + lane offset (one VGPR) vs per-lane pointer arrays
//   MODE     0 full, 1 stream only (no arithmetic), 2 arithmetic only (no loads)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                \
  do {                                                                       \
    hipError_t e_ = (x);                                                     \
    if (e_ != hipSuccess) {                                                  \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                \
      exit(1);                                                               \
    }                                                                        \
  } while (0)

constexpr int D = 5, NS = 1 << D, G = 8, ROWS = NS + G, TILE = ROWS * 64;   // doubles per chunk tile
constexpr int NQ = 4 + D;
constexpr int LOG2N = 20;
constexpr long K = 1L << (LOG2N - 1);      // frequencies (lattice half; k = n/2 ignored here)
constexpr long Q = K / 64;                  // chunks

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void glb_void;

template <int DD>
__device__ __forceinline__ double mlin(const double* phi, const double* l, double* dp) {
  if constexpr (DD == 0) {
    return phi[0];
  } else {
    constexpr int H = 1 << (DD - 1);
    double d0[DD > 1 ? DD - 1 : 1], d1[DD > 1 ? DD - 1 : 1];
    const double p0 = mlin<DD - 1>(phi, l, d0);
    const double p1 = mlin<DD - 1>(phi + H, l, d1);
#pragma unroll
    for (int j = 0; j < DD - 1; ++j) dp[j] = __builtin_fma(l[DD - 1], d1[j], d0[j]);
    dp[DD - 1] = p1;
    return __builtin_fma(l[DD - 1], p1, p0);
  }
}

struct Acc {
  double norm = 0.0, ge = 0.0, gs = 0.0, mant = 1.0;
  double gl[D];
  int ex = 0;
  __device__ __forceinline__ Acc() {
#pragma unroll
    for (int j = 0; j < D; ++j) gl[j] = 0.0;
  }
};

__device__ __forceinline__ double rcp_nr(double e) {
  double r = __builtin_amdgcn_rcp(e);
  r = __builtin_fma(__builtin_fma(-e, r, 1.0), r, r);
  return __builtin_fma(__builtin_fma(-e, r, 1.0), r, r);
}

struct HypS {
  double scale, noise, ls[D];
};

__device__ __forceinline__ void terms(const double* phi, const HypS& h, double rootn, double wl, double Y, Acc& acc) {
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

__device__ __forceinline__ void wave_partials(const Acc& acc, double* out /* [NQ] at stride */, long stride) {
  double v[NQ];
  v[0] = acc.norm;
  v[1] = log(acc.mant) + (double)acc.ex * 0.69314718055994530942;
  v[2] = acc.ge;
  v[3] = acc.gs;
#pragma unroll
  for (int j = 0; j < D; ++j) v[4 + j] = acc.gl[j];
#pragma unroll
  for (int q = 0; q < NQ; ++q)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v[q] += __shfl_xor(v[q], o, 64);
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int q = 0; q < NQ; ++q) out[q * stride] = v[q];
}

template <int RING>
__device__ __forceinline__ void wait_ring(int inflight_instr) {
  if constexpr (RING == 2) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    switch (inflight_instr) {
      case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
      case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
      case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
      default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
  }
}

__device__ __forceinline__ void barrier_keep_vm() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

struct Args {
  const double* basis;   // [Q][NS][64]
  const double* ysq;     // [Q][G][64]
  const double* hyp;     // [G][2 + D] scale, noise, ls
  double* partials;      // [G][NQ][nblk]
  int nblk, cpb;         // blocks, chunks per block
  unsigned* counters;    // [0] head, [1] done (DYN)
  unsigned long long* stamps;   // [grid][2] start / end (optional)
  int* xcc;                     // [grid] XCC id of the workgroup (with stamps)
};

// 20 wave-instructions of 1 KiB per chunk: j < 16 spectra (chunk q at basis + q NS 64), j >= 16 Y; wave w
// issues j = w, w + 4, ...  (5 each).  DYN: the workgroup's blocks come from an atomic counter, dequeued two
// ahead into an LDS ring seq[4] (thread 0 issues the add behind a chunk's DMA; its value is stored to LDS at
// the next iteration, before that iteration's barrier); requires cpb >= RING - 1.
template <int RING, bool DYN, bool SADDR, int MODE, int WPC, int PPW = 2>
__global__ __launch_bounds__(64 * G / PPW, WPC) void k_lab(Args a) {
  constexpr int W = G / PPW, TPW = (20 + W - 1) / W;   // waves; DMA wave-instructions per wave (at most)
  extern __shared__ double lds[];
  __shared__ int seq[4];
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  if (a.stamps && threadIdx.x == 0) a.stamps[blockIdx.x * 2] = wall_clock64();
  HypS h[PPW];
#pragma unroll
  for (int p = 0; p < PPW; ++p) {
    const double* hp = a.hyp + (PPW * w + p) * (2 + D);
    h[p].scale = hp[0];
    h[p].noise = hp[1];
#pragma unroll
    for (int j = 0; j < D; ++j) h[p].ls[j] = hp[2 + j];
  }
  const double rootn = 1024.0, wl = 1.0;
  const double* src0[TPW];
  long step[TPW];
  if (!SADDR) {
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
      const int j = w + W * t;
      src0[t] = j < 16 ? a.basis + j * 128 + lane * 2 : a.ysq + (j - 16) * 128 + lane * 2;
      step[t] = j < 16 ? NS * 64 : G * 64;
    }
  }
  auto issue = [&](long q, double* buf) {
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
      const int j = w + W * t;
      if (j >= 20) break;
      const double* src;
      if (SADDR) {
        const double* base = j < 16 ? a.basis + q * (NS * 64) + j * 128 : a.ysq + q * (G * 64) + (j - 16) * 128;
        src = base + lane * 2;
      } else {
        src = src0[t] + step[t] * q;
      }
      __builtin_amdgcn_global_load_lds((glb_void*)src, (lds_void*)(buf + 128 * j), 16, 0, 0);
    }
  };
  const int cpb = a.cpb, nblk = a.nblk;
  int kd = 0;   // blocks dequeued (DYN)
  if (DYN) {
    // RING blocks ahead: the issue position runs up to RING - 1 chunks (<= one block at cpb >= RING - 1) past
    // the compute position, and the block after it must be known by then
    static_assert(RING <= 3, "seq[4] holds the compute block and at most 3 ahead");
    if (threadIdx.x == 0)
      for (int i = 0; i < RING; ++i) seq[i] = (int)atomicAdd(a.counters, 1u);
    kd = RING;
    __syncthreads();
  }
  auto block_of = [&](int k) -> int { return DYN ? seq[k & 3] : (k == 0 ? (int)blockIdx.x : nblk); };
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  int ki = 0, ii = 0;            // issue position: block sequence index, chunk in block
  int ib = block_of(0);
  int issued = 0;
  auto issue_next = [&](int slot) {
    if ((unsigned)ib >= (unsigned)nblk) return;
    if (MODE != 2) issue((long)ib * cpb + ii, lds + slot * TILE);
    ++issued;
    if (++ii == cpb) {
      ii = 0;
      ++ki;
      ib = block_of(ki);
    }
  };
#pragma unroll
  for (int c = 0; c < RING - 1; ++c) issue_next(c);
  Acc acc[PPW];
  int c = 0, kp = 0, pi = 0;
  int pb = block_of(0);
  unsigned pend = 0;      // thread 0: a dequeue in flight (its value goes to seq[pend_slot] next iteration)
  int pend_slot = -1;
  while ((unsigned)pb < (unsigned)nblk) {
    const int behind = issued - c - 1;
    wait_ring<RING>(MODE == 2 ? 0 : TPW * std::min(behind, RING - 2));
    if (DYN && pend_slot >= 0) {
      if (threadIdx.x == 0) seq[pend_slot] = (int)pend;
      pend_slot = -1;
    }
    barrier_keep_vm();
    issue_next((c + RING - 1) % RING);
    const double* buf = lds + (c % RING) * TILE;
    if (MODE != 1) {
      double phi[NS];
#pragma unroll
      for (int s = 0; s < NS; ++s) phi[s] = buf[64 * s + lane];
#pragma unroll
      for (int p = 0; p < PPW; ++p) terms(phi, h[p], rootn, wl, buf[64 * (NS + PPW * w + p) + lane], acc[p]);
    } else {
      acc[0].norm += buf[lane] + buf[64 * (NS + PPW * w) + lane];
    }
    ++c;
    if (++pi == cpb) {
#pragma unroll
      for (int p = 0; p < PPW; ++p) {
        wave_partials(acc[p], a.partials + (long)(PPW * w + p) * NQ * nblk + pb, nblk);
        acc[p] = Acc();
      }
      pi = 0;
      ++kp;
      if (DYN) {
        // dequeue the block after the last one known (sequence index kd), stored next iteration
        if (threadIdx.x == 0) pend = atomicAdd(a.counters, 1u);
        pend_slot = kd & 3;
        ++kd;
      }
      pb = block_of(kp);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (DYN) {
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned done = atomicAdd(a.counters + 1, 1u);
      if (done == gridDim.x - 1) {
        atomicExch(a.counters, 0u);
        atomicExch(a.counters + 1, 0u);
      }
    }
  }
  if (a.stamps && threadIdx.x == 0) {
    a.stamps[blockIdx.x * 2 + 1] = wall_clock64();
    a.xcc[blockIdx.x] = __builtin_amdgcn_s_getreg((3 << 11) | 20);   // HW_REG_XCC_ID[3:0]
  }
}


template <int N>
__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// Second family (fixed block per workgroup, 2-slot ring, 2 problems per wave, wave-uniform DMA bases):
//   CK     64-frequency sub-chunks per ring slot (fewer barriers per byte; CK = 2: 80 KB of LDS per workgroup)
//   AUX    cache-policy bits of the LDS-DMA loads (2 = nt)
//   PROUS  a synthetic prologue of PROUS us before the loop (the fused kernel's deferred step: level-2 sums +
//          Rprop), with PRE = 1 or 2 chunks issued in front of it
template <int CK, int AUX, int PROUS, int PRE, int MODE>
__global__ __launch_bounds__(256, 2) void k_lab2(Args a) {
  constexpr int W = 4, NI = 20 * CK, TPW = NI / W, T2 = TILE * CK, SPX = CK * NS * 64;
  static_assert(NI % W == 0, "whole DMA rounds");
  extern __shared__ double lds[];
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  if (a.stamps && threadIdx.x == 0) a.stamps[blockIdx.x * 2] = wall_clock64();
  HypS h[2];
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const double* hp = a.hyp + (2 * w + p) * (2 + D);
    h[p].scale = hp[0];
    h[p].noise = hp[1];
#pragma unroll
    for (int j = 0; j < D; ++j) h[p].ls[j] = hp[2 + j];
  }
  const double rootn = 1024.0, wl = 1.0;
  const int nc = a.cpb;
  const long q0 = (long)blockIdx.x * nc;
  auto issue = [&](int c, double* buf) {
    const long q = q0 + c;
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
      const int j = w + W * t;
      const double* base = j < 16 * CK ? a.basis + q * (CK * NS * 64) + j * 128 : a.ysq + q * (CK * G * 64) + (j - 16 * CK) * 128;
      __builtin_amdgcn_global_load_lds((glb_void*)(base + lane * 2), (lds_void*)(buf + 128 * j), 16, 0, AUX);
    }
  };
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (MODE != 2) {
    issue(0, lds);
    if (PRE == 2 && nc > 1) issue(1, lds + T2);
  }
  if (PROUS > 0) {
    const unsigned long long t0 = wall_clock64();
    while (wall_clock64() - t0 < (unsigned long long)(PROUS * 100)) __builtin_amdgcn_s_sleep(2);
  }
  Acc acc[2];
  for (int c = 0; c < nc; ++c) {
    if (PRE == 2 && c == 0 && nc > 1 && MODE != 2) wait_vm<TPW>();
    else wait_vm<0>();
    barrier_keep_vm();
    if (MODE != 2 && c + 1 < nc && c + 1 >= PRE) issue(c + 1, lds + ((c + 1) & 1) * T2);
    const double* buf = lds + (c & 1) * T2;
    if (MODE != 1) {
#pragma unroll
      for (int sc = 0; sc < CK; ++sc) {
        double phi[NS];
#pragma unroll
        for (int s = 0; s < NS; ++s) phi[s] = buf[(sc * NS + s) * 64 + lane];
#pragma unroll
        for (int p = 0; p < 2; ++p) terms(phi, h[p], rootn, wl, buf[SPX + (sc * G + 2 * w + p) * 64 + lane], acc[p]);
      }
    } else {
      acc[0].norm += buf[lane] + buf[SPX + 2 * w * 64 + lane];
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int p = 0; p < 2; ++p) wave_partials(acc[p], a.partials + (long)(2 * w + p) * NQ * a.nblk + blockIdx.x, a.nblk);
  if (a.stamps && threadIdx.x == 0) {
    a.stamps[blockIdx.x * 2 + 1] = wall_clock64();
    a.xcc[blockIdx.x] = __builtin_amdgcn_s_getreg((3 << 11) | 20);
  }
}

// Third family (round 6): a dedicated DMA producer wave per workgroup.  Waves 0-3 compute (2
// problems each, as the fused kernel), wave 4 only issues the LDS-DMA loads: it keeps up to RING - 1 chunks in flight,
// and for the oldest one waits for its own loads (counted vmcnt) and publishes it by an LDS flag (full[slot] = chunk + 1);
// a compute wave spins on that flag, computes, and counts itself done in done[slot] (ds_add), which the producer waits
// for before it refills the slot.  No workgroup barrier in the chunk loop.
template <int RING, int MODE>
__global__ __launch_bounds__(320, 2) void k_lab3(Args a) {
  extern __shared__ double lds[];
  __shared__ int full[RING], done[RING];
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  if (a.stamps && threadIdx.x == 0) a.stamps[blockIdx.x * 2] = wall_clock64();
  if (threadIdx.x < RING) {
    full[threadIdx.x] = 0;
    done[threadIdx.x] = 0;
  }
  __syncthreads();
  const int nc = a.cpb;
  const long q0 = (long)blockIdx.x * nc;
  volatile int* vfull = full;
  volatile int* vdone = done;
  if (w == 4) {
    // producer
    int issued = 0, flagged = 0;
    while (flagged < nc) {
      while (issued < nc && issued < flagged + RING - 1) {
        const int slot = issued % RING;
        const int need = 4 * (issued / RING);          // consumers done with chunk issued - RING in this slot
        for (int spin = 0; vdone[slot] < need && spin < (1 << 24); ++spin) __builtin_amdgcn_s_sleep(1);   // (bounded)
        double* buf = lds + slot * TILE;
        if (MODE != 2) {
          const long q = q0 + issued;
#pragma unroll
          for (int j = 0; j < 20; ++j) {
            const double* base = j < 16 ? a.basis + q * (NS * 64) + j * 128 : a.ysq + q * (G * 64) + (j - 16) * 128;
            __builtin_amdgcn_global_load_lds((glb_void*)(base + lane * 2), (lds_void*)(buf + 128 * j), 16, 0, 0);
          }
        }
        ++issued;
      }
      // the oldest chunk in flight: its 20 loads are the oldest of the wave's outstanding ones
      const int newer = issued - 1 - flagged;
      if (newer >= 2) asm volatile("s_waitcnt vmcnt(40)" ::: "memory");
      else if (newer == 1) asm volatile("s_waitcnt vmcnt(20)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) vfull[flagged % RING] = flagged + 1;
      ++flagged;
    }
  } else {
    HypS h[2];
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const double* hp = a.hyp + (2 * w + p) * (2 + D);
      h[p].scale = hp[0];
      h[p].noise = hp[1];
#pragma unroll
      for (int j = 0; j < D; ++j) h[p].ls[j] = hp[2 + j];
    }
    const double rootn = 1024.0, wl = 1.0;
    Acc acc[2];
    for (int c = 0; c < nc; ++c) {
      const int slot = c % RING;
      for (int spin = 0; __builtin_amdgcn_readfirstlane(vfull[slot]) != c + 1 && spin < (1 << 24); ++spin)
        __builtin_amdgcn_s_sleep(1);                   // (bounded: a broken hand-off ends, with wrong partials)
      const double* buf = lds + slot * TILE;
      if (MODE != 1) {
        double phi[NS];
#pragma unroll
        for (int s = 0; s < NS; ++s) phi[s] = buf[64 * s + lane];
#pragma unroll
        for (int p = 0; p < 2; ++p) terms(phi, h[p], rootn, wl, buf[64 * (NS + 2 * w + p) + lane], acc[p]);
      } else {
        acc[0].norm += buf[lane] + buf[64 * (NS + 2 * w) + lane];
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (lane == 0) atomicAdd(&done[slot], 1);
    }
#pragma unroll
    for (int p = 0; p < 2; ++p) wave_partials(acc[p], a.partials + (long)(2 * w + p) * NQ * a.nblk + blockIdx.x, a.nblk);
  }
  if (a.stamps && threadIdx.x == 0) {
    a.stamps[blockIdx.x * 2 + 1] = wall_clock64();
    a.xcc[blockIdx.x] = __builtin_amdgcn_s_getreg((3 << 11) | 20);
  }
}

template <typename F>
static double time_us(F launch, int reps) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 5; ++i) launch();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i) launch();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return 1e3 * ms / reps;
}

int main(int argc, char** argv) {
  const size_t nb = (size_t)Q * NS * 64, ny = (size_t)Q * G * 64;
  std::vector<double> hb(nb), hy(ny), hh(G * (2 + D));
  srand(7);
  for (size_t i = 0; i < nb; ++i) hb[i] = (i % (NS * 64)) < 64 ? 1.0 + (rand() % 1000) * 1e-3 : (rand() % 1000) * 1e-6;
  for (size_t i = 0; i < ny; ++i) hy[i] = (rand() % 1000) * 1e-3;
  for (int g = 0; g < G; ++g) {
    hh[g * (2 + D)] = 1.0 + 0.01 * g;
    hh[g * (2 + D) + 1] = 1e-8;
    for (int j = 0; j < D; ++j) hh[g * (2 + D) + 2 + j] = 0.5 + 0.1 * j;
  }
  Args a{};
  double *db, *dy, *dh, *dp;
  unsigned* dc;
  unsigned long long* ds;
  CK(hipMalloc(&db, nb * 8));
  CK(hipMalloc(&dy, ny * 8));
  CK(hipMalloc(&dh, hh.size() * 8));
  CK(hipMalloc(&dp, (size_t)G * NQ * 8192 * 8));
  CK(hipMalloc(&dc, 64));
  CK(hipMalloc(&ds, 8192 * 2 * 8));
  int* dx;
  CK(hipMalloc(&dx, 8192 * 4));
  a.xcc = dx;
  CK(hipMemset(dc, 0, 64));
  CK(hipMemcpy(db, hb.data(), nb * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dy, hy.data(), ny * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dh, hh.data(), hh.size() * 8, hipMemcpyHostToDevice));
  a.basis = db;
  a.ysq = dy;
  a.hyp = dh;
  a.partials = dp;
  a.counters = dc;
  std::vector<double> ref;
  auto run = [&](const char* name, auto kern, int ring, int grid, int cpb, bool check, int threads = 256, int ck = 1) {
    a.cpb = cpb;
    a.nblk = (int)(Q / ((long)cpb * ck));
    a.stamps = nullptr;
    const size_t shm = (size_t)ring * TILE * 8 * ck;
    CK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
    CK(hipMemset(dp, 0, (size_t)G * NQ * 8192 * 8));
    const double us = time_us([&] { kern<<<grid, threads, shm>>>(a); }, 50);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    // checksum of the partials against the first full variant (same blocks => same values)
    std::vector<double> hp((size_t)G * NQ * a.nblk);
    CK(hipMemcpy(hp.data(), dp, hp.size() * 8, hipMemcpyDeviceToHost));
    double tot[NQ] = {0};
    for (int g = 0; g < G; ++g)
      for (int q = 0; q < NQ; ++q)
        for (int b = 0; b < a.nblk; ++b) tot[q] += hp[((size_t)g * NQ + q) * a.nblk + b];
    double err = 0.0;
    if (check) {
      if (ref.empty()) ref.assign(tot, tot + NQ);
      for (int q = 0; q < NQ; ++q) err = std::max(err, fabs(tot[q] - ref[q]) / (fabs(ref[q]) + 1e-300));
    }
    // stamps pass
    a.stamps = ds;
    kern<<<grid, threads, shm>>>(a);
    CK(hipDeviceSynchronize());
    std::vector<unsigned long long> st((size_t)grid * 2);
    std::vector<int> xc(grid);
    CK(hipMemcpy(st.data(), ds, st.size() * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(xc.data(), dx, grid * 4, hipMemcpyDeviceToHost));
    unsigned long long t0 = ~0ull, t1 = 0;
    std::vector<double> dur(grid), endt(grid);
    std::vector<std::vector<double>> per(8);
    for (int b = 0; b < grid; ++b) t0 = std::min(t0, st[2 * b]);
    for (int b = 0; b < grid; ++b) {
      t1 = std::max(t1, st[2 * b + 1]);
      dur[b] = (st[2 * b + 1] - st[2 * b]) / 100.0;
      endt[b] = (st[2 * b + 1] - t0) / 100.0;
      per[xc[b] & 7].push_back(endt[b]);
    }
    std::sort(dur.begin(), dur.end());
    std::sort(endt.begin(), endt.end());
    char xs[256];
    int o = 0;
    for (int x = 0; x < 8; ++x) {
      std::sort(per[x].begin(), per[x].end());
      o += snprintf(xs + o, sizeof xs - o, "%s%.1f", x ? "," : "", per[x].empty() ? 0.0 : per[x].back());
    }
    printf("{\"variant\": \"%s\", \"ring\": %d, \"grid\": %d, \"cpb\": %d, \"us\": %.2f, \"GBps\": %.0f, "
           "\"span_us\": %.2f, \"dur_p10\": %.2f, \"dur_p50\": %.2f, \"dur_p90\": %.2f, \"end_p50\": %.2f, "
           "\"end_p90\": %.2f, \"xcc_last_end\": [%s], \"check_rel\": %.3g}\n",
           name, ring, grid, cpb, us, (nb + ny) * 8.0 / us / 1e3, (t1 - t0) / 100.0, dur[grid / 10], dur[grid / 2],
           dur[grid * 9 / 10], endt[grid / 2], endt[grid * 9 / 10], xs, err);
    fflush(stdout);
  };
  const bool all = argc > 1;   // the slower families measured in r04a / r04b (profiles/r04_lab.jsonl)
  // the current structure: fixed block per workgroup, 512 x 16 chunks, pointer arrays, 2-slot ring
  run("fixed ptr r2", k_lab<2, false, false, 0, 2>, 2, 512, 16, true);
  run("fixed ptr r2 stream", k_lab<2, false, false, 1, 2>, 2, 512, 16, false);
  run("fixed ptr r2 compute", k_lab<2, false, false, 2, 2>, 2, 512, 16, false);
  run("fixed saddr r2", k_lab<2, false, true, 0, 2>, 2, 512, 16, true);
  run("fixed saddr r3", k_lab<3, false, true, 0, 2>, 3, 512, 16, true);
  run("fixed saddr r2 1024x8", k_lab<2, false, true, 0, 2>, 2, 1024, 8, true);
  if (all) run("fixed saddr r2 1024x8 wpc3", k_lab<2, false, true, 0, 3>, 2, 1024, 8, true);
  if (all) run("fixed saddr r2 2048x4 wpc3", k_lab<2, false, true, 0, 3>, 2, 2048, 4, true);
  for (int cpb : {2, 4, 8}) {
    if (!all) break;
    for (int res : {2, 3}) {
      char nm[64];
      snprintf(nm, sizeof nm, "dyn saddr r2 res%d", res);
      if (res == 2) run(nm, k_lab<2, true, true, 0, 2>, 2, 256 * res, cpb, true);
      else run(nm, k_lab<2, true, true, 0, 3>, 2, 256 * res, cpb, true);
      snprintf(nm, sizeof nm, "dyn saddr r3 res%d", res);
      if (res == 2) run(nm, k_lab<3, true, true, 0, 2>, 3, 256 * res, cpb, true);
    }
  }
  if (all) run("fixed saddr r2 1024x8 wpc4", k_lab<2, false, true, 0, 4>, 2, 1024, 8, true);
  if (all) run("dyn saddr r2 res4 cpb4", k_lab<2, true, true, 0, 4>, 2, 1024, 4, true);
  if (all) run("dyn saddr r2 res4 cpb8", k_lab<2, true, true, 0, 4>, 2, 1024, 8, true);
  if (all) run("dyn saddr r2 res3 stream", k_lab<2, true, true, 1, 3>, 2, 768, 4, false);
  if (all) run("dyn saddr r2 res3 compute", k_lab<2, true, true, 2, 3>, 2, 768, 4, false);
  // one problem per wave, 8 waves per workgroup (one acc set, fewer VGPRs, 4 waves per SIMD)
  run("fixed saddr r2 ppw1 wpc4", k_lab<2, false, true, 0, 4, 1>, 2, 512, 16, true, 512);
  run("fixed saddr r2 ppw1 wpc4 stream", k_lab<2, false, true, 1, 4, 1>, 2, 512, 16, false, 512);
  run("fixed saddr r2 ppw1 wpc4 compute", k_lab<2, false, true, 2, 4, 1>, 2, 512, 16, false, 512);
  run("fixed saddr r2 ppw1 1024x8 wpc4", k_lab<2, false, true, 0, 4, 1>, 2, 1024, 8, true, 512);
  if (all) run("dyn saddr r2 ppw1 res2 cpb4", k_lab<2, true, true, 0, 4, 1>, 2, 512, 4, true, 512);
  if (all) run("dyn saddr r2 ppw1 res2 cpb8", k_lab<2, true, true, 0, 4, 1>, 2, 512, 8, true, 512);
  // third family (round 6): a DMA producer wave + 4 compute waves, LDS flags instead of barriers
  run("lab3 producer r3", k_lab3<3, 0>, 3, 512, 16, true, 320);
  run("lab3 producer r3 stream", k_lab3<3, 1>, 3, 512, 16, false, 320);
  run("lab3 producer r3 compute", k_lab3<3, 2>, 3, 512, 16, false, 320);
  run("lab3 producer r2", k_lab3<2, 0>, 2, 512, 16, true, 320);
  // second family: sub-chunks per slot, nt, prologue overlap
  run("lab2 ck1", k_lab2<1, 0, 0, 1, 0>, 2, 512, 16, true, 256, 1);
  run("lab2 ck2", k_lab2<2, 0, 0, 1, 0>, 2, 512, 8, true, 256, 2);
  run("lab2 ck2 compute", k_lab2<2, 0, 0, 1, 2>, 2, 512, 8, false, 256, 2);
  run("lab2 ck2 stream", k_lab2<2, 0, 0, 1, 1>, 2, 512, 8, false, 256, 2);
  run("lab2 ck1 nt", k_lab2<1, 2, 0, 1, 0>, 2, 512, 16, true, 256, 1);
  run("lab2 ck1 nt stream", k_lab2<1, 2, 0, 1, 1>, 2, 512, 16, false, 256, 1);
  run("lab2 ck2 nt", k_lab2<2, 2, 0, 1, 0>, 2, 512, 8, true, 256, 2);
  run("lab2 ck1 pro2 pre1", k_lab2<1, 0, 2, 1, 0>, 2, 512, 16, true, 256, 1);
  run("lab2 ck1 pro2 pre2", k_lab2<1, 0, 2, 2, 0>, 2, 512, 16, true, 256, 1);
  run("lab2 ck2 pro2 pre2", k_lab2<2, 0, 2, 2, 0>, 2, 512, 8, true, 256, 2);
  return 0;
}
