// Host-side runtime shared by the fgp C-ABI entry points: error reporting and per-device
// twiddle tables.  Internal header (not part of the public C-ABI in include/fgp_hip.h).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fgp {

constexpr int kMaxLog2N = 24;   // largest supported transform length 2^24

// Split of a length-2^m transform (m > 12) into N1 x N2 with N2 = 2^m2 rows-length, N1 = 2^m1.
inline int split_m2(int m) { return m - 4 < 12 ? m - 4 : 12; }

struct Tables {
  double2* tw4096 = nullptr;             // exp(-2 pi i k / 4096), k < 4096
  double2* twm[kMaxLog2N + 1] = {};      // for m > 12: exp(-2 pi i k / 2^m), k < 2^split_m2(m)
};

// Returns the (lazily initialised, stream-synchronised) tables of the current device.
const Tables* get_tables(hipStream_t stream);

int set_error(int code, const char* fmt, ...);

// Adjoint column pass of a [batch, 2^m] transform (m > 12), stable, unscaled: FFT (conj twiddle)
// when fft, else WHT columns.  Defined in fgp_transforms.hip; used by the fused backward.
int cols_adjoint_launch(bool fft, int m, const void* in, void* out, int64_t batch, const Tables* tb,
                        hipStream_t st);
int check_launch(const char* what);

enum Status : int {
  kOk = 0,
  kErrInvalid = -1,
  kErrUnsupported = -2,
  kErrHip = -3,
};

}  // namespace fgp
