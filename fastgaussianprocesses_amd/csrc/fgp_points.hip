// Natural-order base-2 digital net points on the device (the generator of FastGPDigitalNetB2's sequences:
// qmcpy.DigitalNetB2 order="NATURAL", randomize in {"FALSE", "DS"}, used at fast_gp_digital_net_b2.py:
// 266-269 through _XXbSeq, util.py:17-38):
//   xb_i[j] = XOR_{k : bit k of i} C[j][k]  XOR  shift[j]       (t-bit integers, exact)
//   x_i[j]  = xb_i[j] * 2^-t                                     (_convert_from_b, :272-273; exact in fp64
//                                                                 for t <= 53, the product's only rounding
//                                                                 otherwise -- the host's too)
// One thread per point; the generating-matrix columns C[j][k] (t-bit ints) and the shift are read
// from a small device table (uniform, cached).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/fgp_hip.h"
#include "fgp_common.h"
#include "fgp_runtime.h"

namespace fgp {

__global__ __launch_bounds__(kWG) void k_net_points(const uint64_t* __restrict__ C, int mcols,
                                                    const uint64_t* __restrict__ shift, int64_t n0, int64_t n1, int d,
                                                    int t, int64_t* __restrict__ xb, double* __restrict__ x) {
  const int64_t e = (int64_t)blockIdx.x * kWG + threadIdx.x;
  if (e >= n1 - n0) return;
  const uint64_t i = (uint64_t)(n0 + e);
  const double sc = ldexp(1.0, -t);
  for (int j = 0; j < d; ++j) {
    uint64_t v = shift[j];
    uint64_t bits = i;
    while (bits) {
      const int k = __builtin_ctzll(bits);
      v ^= C[(int64_t)j * mcols + k];
      bits &= bits - 1;
    }
    if (xb) xb[e * d + j] = (int64_t)v;
    if (x) x[e * d + j] = (double)v * sc;
  }
}

}  // namespace fgp

using namespace fgp;

extern "C" {

int fgp_net_points(const uint64_t* C, int mcols, const uint64_t* shift, int64_t n_min, int64_t n_max, int d, int t,
                   int64_t* xb, double* x, void* stream) {
  if (d < 1 || d > 64 || t < 1 || t > 63 || mcols < 1 || mcols > 64 || n_min < 0 || n_max < n_min)
    return set_error(kErrInvalid, "fgp_net_points: bad d/t/mcols/n range");
  if (n_max == n_min) return kOk;
  if (n_max > ((int64_t)1 << (mcols < 63 ? mcols : 62)))
    return set_error(kErrUnsupported, "fgp_net_points: n_max %lld needs more than %d generating-matrix columns",
                     (long long)n_max, mcols);
  if (!C || !shift || (!xb && !x)) return set_error(kErrInvalid, "fgp_net_points: null pointer");
  const int64_t cnt = n_max - n_min;
  k_net_points<<<(unsigned)((cnt + kWG - 1) / kWG), kWG, 0, (hipStream_t)stream>>>(C, mcols, shift, n_min, n_max, d,
                                                                                     t, xb, x);
  return check_launch("k_net_points");
}

}  // extern "C"
