// Error reporting + per-device twiddle tables for the fgp C-ABI.
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <mutex>

#include "fgp_common.h"
#include "fgp_runtime.h"
#include "../../include/fgp_hip.h"

namespace fgp {

static thread_local char g_err[512] = "";

int set_error(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(kErrHip, "%s: %s", what, hipGetErrorString(e));
  return kOk;
}

// exp(-2 pi i k / 2^logn) for k < count, via sincospi (argument 2k/2^logn is exact).
__global__ void k_init_twiddles(double2* out, int logn, int count) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= count) return;
  const double x = ldexp((double)(2 * k), -logn);
  double s, c;
  sincospi(x, &s, &c);
  out[k] = make_double2(c, -s);
}

static std::mutex g_mu;
static Tables g_tables[64];
static bool g_ready[64] = {};

const Tables* get_tables(hipStream_t stream) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  std::lock_guard<std::mutex> lock(g_mu);
  if (g_ready[dev]) return &g_tables[dev];
  Tables& t = g_tables[dev];
  size_t total = 4096;
  for (int m = 13; m <= kMaxLog2N; ++m) total += (size_t)1 << split_m2(m);
  double2* buf = nullptr;
  if (hipMalloc(&buf, total * sizeof(double2)) != hipSuccess) return nullptr;
  t.tw4096 = buf;
  k_init_twiddles<<<16, 256, 0, stream>>>(buf, 12, 4096);
  size_t off = 4096;
  for (int m = 13; m <= kMaxLog2N; ++m) {
    const int cnt = 1 << split_m2(m);
    t.twm[m] = buf + off;
    k_init_twiddles<<<(cnt + 255) / 256, 256, 0, stream>>>(buf + off, m, cnt);
    off += cnt;
  }
  if (hipGetLastError() != hipSuccess || hipStreamSynchronize(stream) != hipSuccess) return nullptr;
  g_ready[dev] = true;
  return &t;
}

}  // namespace fgp

namespace fgp {
__global__ void k_clock_stamp(unsigned long long* dst) { *dst = (unsigned long long)wall_clock64(); }
}  // namespace fgp

extern "C" {

const char* fgp_last_error(void) { return fgp::g_err; }

int fgp_abi_version(void) { return FGP_ABI_VERSION; }

int fgp_wall_clock_khz(int device, int* khz) {
  if (!khz) return fgp::set_error(fgp::kErrInvalid, "fgp_wall_clock_khz: null output");
  if (hipDeviceGetAttribute(khz, hipDeviceAttributeWallClockRate, device) != hipSuccess)
    return fgp::set_error(fgp::kErrHip, "fgp_wall_clock_khz: hipDeviceGetAttribute failed");
  return fgp::kOk;
}

int fgp_clock_stamp(unsigned long long* dst, void* stream) {
  if (!dst) return fgp::set_error(fgp::kErrInvalid, "fgp_clock_stamp: null destination");
  fgp::k_clock_stamp<<<1, 1, 0, (hipStream_t)stream>>>(dst);
  return fgp::check_launch("k_clock_stamp");
}

int fgp_init(void* stream) {
  return fgp::get_tables((hipStream_t)stream) ? fgp::kOk
                                              : fgp::set_error(fgp::kErrHip, "fgp_init: table allocation failed");
}

}  // extern "C"
