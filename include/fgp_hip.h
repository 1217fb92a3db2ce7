/* fgp_hip.h — C-ABI of the MI355X-native fast-transform GP hot path (libfgp_hip.so).
 *
 * Plain pointers, sizes and an opaque hipStream_t (passed as void*): no torch types cross this
 * boundary.  Every entry point is stream-ordered (no host synchronisation except the one-time
 * table initialisation), returns 0 on success or a negative FGP_ERR_* code, and records a
 * message retrievable with fgp_last_error().  All device pointers are HIP device memory.
 *
 * Layout conventions: a "[batch, n]" array is batch rows of n contiguous elements, row i starting
 * at element i*batch_stride.  complex128 = interleaved (re, im) doubles (torch.complex128).
 *
 * Reference interfaces replaced (alegresor/FastGaussianProcesses @ /root/reference):
 *   fgp_fftbr   <- qmcpy.fftbr_torch injected as ft   (fastgps/fast_gp_lattice.py:224,231) and its
 *                  stabilising wrapper AbstractFastGP.ft (fastgps/abstract_fast_gp.py:197-212)
 *   fgp_ifftbr  <- qmcpy.ifftbr_torch injected as ift (fastgps/fast_gp_lattice.py:225,231) and
 *                  AbstractFastGP.ift (fastgps/abstract_fast_gp.py:213-228); `out_real` fuses the
 *                  `.real` taken by gram_matrix_solve (fastgps/util.py:343)
 *   fgp_fwht    <- qmcpy.fwht_torch injected as ft = ift (fastgps/fast_gp_digital_net_b2.py:226,231)
 */
#ifndef FGP_HIP_H_
#define FGP_HIP_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FGP_ABI_VERSION 18

#define FGP_OK 0
#define FGP_ERR_INVALID (-1)     /* bad argument (shape, stride, null pointer) */
#define FGP_ERR_UNSUPPORTED (-2) /* size outside the supported range (n > 2^24, ...) */
#define FGP_ERR_HIP (-3)         /* HIP runtime / launch failure */

/* Library identification and error reporting. */
int fgp_abi_version(void);
const char* fgp_last_error(void);
/* Optional eager initialisation of the per-device twiddle tables on `stream` (otherwise done on
 * first use; call before hipGraph capture). */
int fgp_init(void* stream);
/* Frequency (kHz) of the device wall clock that fgp_nll_desc.stamps records (hipDeviceAttributeWallClockRate). */
int fgp_wall_clock_khz(int device, int* khz);
/* ABI 16 -- measurement hook (no reference counterpart): one single-lane kernel on `stream` that stores the device
 * wall clock (fgp_wall_clock_khz ticks) into *dst when it runs; placed between the launches of a hipGraph capture,
 * the differences of such stamps are the replayed phases' device time. */
int fgp_clock_stamp(unsigned long long* dst, void* stream);

/* Orthonormal DFT of bit-reversed-order input along the last axis:
 *   out[b, k] = n^-1/2 * sum_i in[b, brev_m(i)] exp(-2 pi i k i / n),  n = 2^log2n, 0 <= log2n <= 24.
 * in: [batch, n] float64 (in_is_real=1) or complex128, row stride in_batch_stride (elements).
 * out: [batch, n] complex128, contiguous, must not alias `in` unless in is complex and contiguous.
 * stable=1 applies AbstractFastGP.ft's mean-centring (mathematically the identity). */
int fgp_fftbr(const void* in, int64_t in_batch_stride, int in_is_real, void* out, int64_t batch, int log2n,
              int stable, void* stream);

/* Adjoint of fgp_fftbr (= ifft(x, norm="ortho")[..., brev_m]):
 *   out[b, i] = n^-1/2 * sum_k in[b, k] exp(+2 pi i k brev_m(i) / n).
 * in: [batch, n] complex128 (row stride in_batch_stride).  out: [batch, n] contiguous, complex128,
 * or float64 holding only the real part when out_real=1 (then, for n > 4096, `work` must be a
 * complex128 [batch, n] scratch buffer; otherwise work may be NULL). */
int fgp_ifftbr(const void* in, int64_t in_batch_stride, void* out, int out_real, void* work, int64_t batch,
               int log2n, int stable, void* stream);

/* Orthonormal Walsh-Hadamard transform in Sylvester (natural) order, self-inverse:
 *   out[b, k] = n^-1/2 * sum_i in[b, i] (-1)^popcount(i & k).   float64 in/out, in-place allowed
 * when in_batch_stride == n. */
int fgp_fwht(const double* in, int64_t in_batch_stride, double* out, int64_t batch, int log2n, int stable,
             void* stream);

/* fftbr of REAL float64 input at half length (ABI 10), 17 <= log2n <= 24: the packed
 * z = x[:n/2] + i x[n/2:] through an n/2-point transform and the split
 *   out[k], out[k + n/2] = 1/2 (Z_k + conj Z_{n/2-k}) -/+ 1/2 i w_n^k (Z_k - conj Z_{n/2-k})
 * in the column pass (the fit's R2C kernels, emitting the spectrum): 40n bytes moved per row instead of
 * the full-length transform's 56n.  out: [batch][n] complex128 (the whole spectrum); work: device
 * scratch of batch * n complex128.  Same values as fgp_fftbr(in_is_real = 1) up to rounding (the
 * engine centres every row / column internally, so `stable` needs no separate pass). */
int fgp_fftbr_real(const double* in, int64_t in_batch_stride, void* out, void* work, int64_t batch, int log2n,
                   void* stream);

/* Real part of the orthonormal ifftbr of complex128 rows at half length (ABI 10), 17 <= log2n <= 24:
 *   out[b] = Re ifftbr(in[b] * f[b])      (f NULL: no product; f_batch_stride 0: one shared row)
 * (gram_matrix_solve's ift(A * y~).real, util.py:341-343) through the adjoint of fgp_fftbr_real: the
 * Hermitian part of each mirror pair packed into V = E + i O, an n/2-point adjoint transform, real rows
 * out.  out: [batch][n] float64 (16-byte aligned rows); work: device scratch of batch * n complex128. */
int fgp_ifftbr_real(const void* in, int64_t in_batch_stride, const void* f, int64_t f_batch_stride, double* out,
                    int64_t out_batch_stride, void* work, int64_t batch, int log2n, void* stream);
/* The same with REAL factor rows f (float64 [batch or 1][n], f_batch_stride 0: one shared row): out[b] =
 * Re ifftbr(in[b] * f[b]) for the real A = 1/ev of the spectral path (ABI 12).  ABI 13: in[b] must be
 * Hermitian (in_{n-k} = conj in_k: ft of real data, as ytilde) and f[b] even (f_{n-k} = f_k, as A): only
 * k <= n/2 of both are read. */
int fgp_ifftbr_real_rf(const void* in, int64_t in_batch_stride, const double* f, int64_t f_batch_stride, double* out,
                       int64_t out_batch_stride, void* work, int64_t batch, int log2n, void* stream);

/* Single-precision variants (complex64 / float32; SURVEY §8(b) fgp_fftbr_c64 / fgp_ifftbr_c64 /
 * fgp_fwht_f32): the same transforms, arguments and layouts with float / complex64 in place of
 * double / complex128 (fgp_fftbr_c64: in float32 when in_is_real, else complex64; out complex64;
 * fgp_ifftbr_c64: out complex64, or float32 real parts when out_real, work complex64).  fp32
 * arithmetic (explicit fmaf) with twiddles rounded once from the fp64 tables.  The reference forbids
 * fp32 (fastgps/abstract_gp.py:46); these serve the mixed-precision data path of BASELINE config C5
 * (float32 observations, fp64 eigenvalues), tolerance stated where used. */
int fgp_fftbr_c64(const void* in, int64_t in_batch_stride, int in_is_real, void* out, int64_t batch, int log2n,
                  int stable, void* stream);
int fgp_ifftbr_c64(const void* in, int64_t in_batch_stride, void* out, int out_real, void* work, int64_t batch,
                   int log2n, int stable, void* stream);
int fgp_fwht_f32(const float* in, int64_t in_batch_stride, float* out, int64_t batch, int log2n, int stable,
                 void* stream);

/* The tilde-domain solve + inverse transform of gram_matrix_solve (fastgps/util.py:341-343,
 * ift(A * y~).real) in one call: out[b] = inverse(in[b] * f[b]) with f row b at f + b * f_batch_stride
 * (0: one row shared by every b, e.g. A = 1/ev of outputs sharing their hyper-parameters), applied in
 * the load of the inverse's first pass.  family LATTICE: ifftbr (complex128, or complex64 when single;
 * out_real / work as fgp_ifftbr); family NET: fwht (float64 / float32, out_real ignored). */
int fgp_ifftbr_mul(int family, int single, const void* in, int64_t in_batch_stride, const void* f, int64_t f_batch_stride,
                   void* out, int out_real, void* work, int64_t batch, int log2n, int stable, void* stream);

/* Y[g, k] = sum_{r < R} |x[r G + g, k]|^2 in float64, x rows of n elements (row stride x_row_stride) of
 * kind 0 float64, 1 complex128, 2 float32, 3 complex64: the MLL's data term over the outputs sharing
 * eigen-problem g (fastgps/util.py:364-370), summed in ascending r. */
int fgp_sum_sq(const void* x, int64_t x_row_stride, int kind, int64_t R, int64_t G, int64_t n, double* out,
               void* stream);


/* ---------------------------------------------------------------------------------------------
 * Kernel parts and the fused negative-log-likelihood / gradient / Rprop fit step.
 *
 * Replaces, for the single-task beta=kappa=0 MLL fit driven by AbstractGP.fit
 * (fastgps/abstract_gp.py:152-306, default Rprop optimizer fastgps/abstract_fast_gp.py:53-57):
 *   _K1PartsSeq / _kernel_parts            (fastgps/util.py:50-62, abstract_fast_gp.py:173-180)
 *   _kernel_from_parts                     (fastgps/abstract_fast_gp.py:181-191)
 *   _LamCaches lam = ft(k1)                (fastgps/util.py:95-112)
 *   _FastInverseLogDetCache.__call__       (fastgps/util.py:275-300, single-task branch)
 *   get_norm_term_logdet_term              (fastgps/util.py:354-370)
 *   MLL assembly + loss.backward()         (fastgps/abstract_gp.py:235,253-261,294)
 *   torch.optim.Rprop(lr).step()           (fastgps/abstract_fast_gp.py:53-57)
 * ------------------------------------------------------------------------------------------- */

#define FGP_FAMILY_LATTICE 0 /* shift-invariant kernel on lattice points: bit-reversed FFT */
#define FGP_FAMILY_NET 1     /* digitally-shift-invariant kernel on digital nets: FWHT */
#define FGP_MAX_D 8

/* Lattice first-column kernel parts (fastgps/fast_gp_lattice.py:263-273, beta=kappa=0):
 *   parts[j, i] = coef[j] * B_{order[j]}((x[i, j] - x[0, j]) % 1),   i < n, j < d.
 * x: [n, d] float64 with row stride x_row_stride; order[j] = 2*alpha_j in {2,4,6,8};
 * coef[j] = (-1)^(alpha_j+1) (2 pi)^(2 alpha_j) / (2 alpha_j)!  (host arrays of length d).
 * parts: [d, n] float64 (dimension-major).  z: [d] float64 reference point (x[0] for the first column). */
int fgp_lattice_parts(const double* x, int64_t x_row_stride, const double* z, int64_t n, int d, const int* order,
                      const double* coef, double* parts, void* stream);

/* Digital-net first-column kernel parts (fastgps/fast_gp_digital_net_b2.py:274-301), Walsh order
 * order[j] in 1..4 per dimension (order = NULL: all 1):
 *   delta = xb[i, j] XOR z[j];
 *   order 1:    parts[j, i] = 6*(1/6 - 2^(floor(log2 delta) - t - 1))  (1 when delta = 0)  (:297-298)
 *   order 2..4: parts[j, i] = omega_a(delta / 2^t) = sum_{k>=1} 2^(-mu_a(k)) wal_k  -- the reference's
 *               qmcpy.kernel_methods.weighted_walsh_funcs(a, delta, t) - 1 (:300), restated from its
 *               series definition (qmcpy itself is absent offline: parity unpinned at that boundary).
 * xb: [n, d] int64 t-bit integers (row stride xb_row_stride), z: [d] int64 (device).  ABI 6: `order`. */
int fgp_net_parts(const int64_t* xb, int64_t xb_row_stride, const int64_t* z, int64_t n, int d, int t,
                  const int* order, double* parts, void* stream);

/* On-device natural-order rank-1 lattice points (seqs.Lattice / qmcpy Lattice, the point generation
 * of AbstractGP.get_x_next, fastgps/abstract_gp.py:307-309 -> util.py:17-48), bit-identical to the host
 * generator: with bits = ceil(log2(n_max)),
 *   x[i - n_min, j] = ((brev_bits(i) z[j] mod 2^bits) / 2^bits + shift[j]) % 1,   n_min <= i < n_max.
 * z: host [d] int64 with 0 < z[j] < 2^(53 - bits); shift: device [d] float64 in [0, 1);
 * x: device [n_max - n_min, d] float64 row-major. */
int fgp_lattice_points(const int64_t* z, const double* shift, int64_t n_min, int64_t n_max, int d, double* x,
                       void* stream);

/* The lattice parts as the FGP_PARTS_LATTICE fit kernels regenerate them (equal to fgp_lattice_parts
 * on the fgp_lattice_points points of size n = 2^log2n with x_0 = shift):
 *   parts[j, i] = coef[j] * B_order(((brev_m(i) z_j mod n) / n + shift_j) % 1 - shift_j) % 1).
 * z, coef: host [d]; shift: device [d]; order in {2, 4, 6, 8}; parts: device [d][n]. */
int fgp_lattice_parts_gen(const int64_t* z, const double* shift, int log2n, int d, int order, const double* coef,
                          double* parts, void* stream);

/* One fused MLL problem batch: G independent eigen-problems of size n = 2^log2n (log2n >= 4). */
typedef struct fgp_nll_desc {
  int family;                 /* FGP_FAMILY_LATTICE / FGP_FAMILY_NET */
  int log2n;                  /* 4 .. 24 */
  int d;                      /* 1 .. FGP_MAX_D */
  int G;                      /* number of eigen-problems */
  const double* parts;        /* [G][d][n] kernel parts; parts_stride elements between problems (0 = shared) */
  int64_t parts_stride;
  const double* ysq;          /* [G][n] sum over the outputs of problem g of |ytilde|^2 */
  int64_t ysq_stride;
  const double* raw;          /* raw (log) hyper-parameters, device; indexed as below */
  int scale_off, scale_pp;    /* log scale of g    = raw[scale_off + (scale_pp ? g : 0)] */
  int ls_off, ls_pp, ls_pd;   /* log lengthscale_j = raw[ls_off + (ls_pp ? g : 0) * (ls_pd ? d : 1) + (ls_pd ? j : 0)] */
  int noise_off, noise_pp;    /* log noise of g    = raw[noise_off + (noise_pp ? g : 0)] */
  double logdet_weight;       /* d_out / numel(logdet)  (fastgps/abstract_gp.py:256) */
  void* grad_lam;             /* output [G][n] of fgp_nll_lam (lambda; complex128 lattice, float64 net);
                                 unused (may be NULL) by fgp_nll_fwd / fgp_nll_bwd */
  void* work;                 /* workspace [G][n] complex128 (lattice) / float64 (net), n > 4096 */
  double* partials;           /* workspace [G][4 + d][max(1, n / 4096) + 1] */
  /* Parts source.  parts_gen = FGP_PARTS_ARRAY: `parts` above.  parts_gen = FGP_PARTS_LATTICE: the
   * lattice parts are regenerated inside the kernels (no parts array is read) from the natural-order
   * rank-1 lattice x[i, j] = ((brev_m(i) z_j mod n) / n + shift_j) % 1, i < n, with exactly the
   * floating-point operations of fgp_lattice_parts applied to those points and x[0] = shift, so the
   * result is bit-identical to the FGP_PARTS_ARRAY path on the same points.  Requires
   * 0 < gen_z[j] < 2^(53 - log2n) (the host point generator is then exact) and 0 <= shift < 1. */
  int parts_gen;
  int gen_order[FGP_MAX_D];   /* 2 alpha_j in {2, 4, 6, 8} */
  double gen_coef[FGP_MAX_D]; /* (-1)^(alpha_j+1) (2 pi)^(2 alpha_j) / (2 alpha_j)! */
  int64_t gen_z[FGP_MAX_D];   /* generating vector */
  const double* gen_shift;    /* device [G][d] (row stride gen_shift_stride; 0 = shared): x[0] = shift */
  int64_t gen_shift_stride;
  /* Optional device-clock kernel timing (ABI 7; NULL = off): a fit kernel launched with this desc
   * stores the wall clock (fgp_wall_clock_khz ticks) into stamps[b * 5] when workgroup b starts and
   * into stamps[b * 5 + 1 + w] when its wave w ends (b < grid size of the launch, 256-thread
   * workgroups); max(ends) - min(starts) is the kernel's duration as rocprofv3 --kernel-trace sees it,
   * measured in-process without the dependent-launch gap that HIP events include. */
  uint64_t* stamps;
  /* ABI 11 -- spectral fit path.  basis non-NULL: the part-product spectra of fgp_spec_basis
   * ([G or 1][Q][2^d][64], problem g's at basis + g * basis_stride; stride 0 = one set shared by all G
   * problems).  Every kernel of this desc then evaluates
   *   lambda_g = scale_g sum_S (prod_{j in S} l_gj) Phi_S
   * instead of transforming k1 (parts / parts_gen / work are not read; d <= 6): fgp_nll_fwd / fgp_fit_run
   * run ONE kernel per iteration (stage 0: loss and gradient partials; stages 1, 2 are no-ops), fgp_nll_lam
   * writes lambda (lattice: the even spectrum mirrored, imaginary parts 0).  The partials workspace must
   * hold fgp_nll_partials_len doubles. */
  const double* basis;
  int64_t basis_stride;
  /* 1: ysq is laid out in chunks of 64 frequencies, [Q][G][64] (Y of problem g at frequency k at
   * ((k / 64) G + g) 64 + k mod 64; ysq_stride unused) -- every problem's Y of a chunk contiguous, read
   * beside the chunk's spectra.  Spectral path only (basis non-NULL). */
  int ysq_chunked;
  /* ABI 12 -- multitask spectral fit.  mt_tasks = T > 0 (with G = 1): ONE multitask / derivative-informed GP
   * of T tasks, every task with the same n = 2^log2n points, the task kernel Kt = gram_matrix_tasks fixed
   * (not learned), the MLL of util.py:364-370 / abstract_gp.py:252-261.  With the pair spectra (k <= l)
   *   Phi^{kl}_S = ft( sum_{b0 in beta_k, b1 in beta_l: S holds every j with b0_j + b1_j > 0}
   *                    c0 c1 prod_{j in S} parts^{b0 b1}_j )
   * (ft = fftbr, complex128 (lattice) / fwht, float64 (net); the parts and coefficients of _kernel_parts /
   * _kernel_from_parts, abstract_fast_gp.py:173-191), each iteration forms per frequency the T x T Hermitian
   * block of the reference's lams (util.py:277-298)
   *   Lambda[k, l] = Kt[k, l] (sqrt(n) scale sum_S l^S Phi^{kl}_S + noise [k == l])
   * factors it (LDL^H, real pivots), and writes the norm / logdet / gradient partials that fgp_fit_step /
   * fgp_fit_run reduce and step (per_problem fit desc).  parts, basis and ysq are not read (ysq: any non-NULL
   * pointer); fgp_nll_lam is not available.  1 <= T <= 8, d <= 6. */
  int mt_tasks;
  const void* mt_basis;       /* [T (T + 1) / 2][2^d][n] pair spectra, pairs (k, l), k <= l, row-major */
  const void* mt_ytilde;      /* [T][n] ytilde of every task (complex128 lattice / float64 net) */
  const double* mt_kt;        /* device [T][T] task kernel */
  /* ABI 16 -- the alternative fit losses of AbstractGP.fit (abstract_gp.py:242-273) on the spectral path:
   * loss_metric FGP_LOSS_MLL (0, the default: everything above), FGP_LOSS_GCV (1) or FGP_LOSS_CV (2).  With
   * ev_k = sqrt(n) lambda_k + noise (lambda from the spectra, basis non-NULL, mt_tasks = 0) and Y = ysq:
   *   GCV (util.py:371-380):  numer = sum_k Y_k / ev_k^2,  denom = (sum_k 1 / ev_k / n)^2,  loss = numer / denom;
   *   CV  (util.py:381-385, abstract_gp.py:262-273, one task): inv_diag = mean_k 1 / (sqrt(n) lambda_k) and, by
   *       Parseval, sum_i coeffs_i^2 = numer, so loss = cv_weight numer / inv_diag^2 (a scalar cv_weights),
   * summed over the problems (or per problem with a per_problem fit desc), gradients in closed form.  Every
   * iteration is the per-wave partials kernel (2 + 2 (2 + d) quantities per problem and k block) plus the
   * reduction / step kernel; the tile, single-launch and persistent kernels are MLL-only.  A desc that is not
   * per_problem holds at most 16 problems.
   * ABI 17 -- GCV of a multitask spectral fit (mt_tasks = T, equal n, fixed task kernel): numer = sum_j |z_j|^2 with
   * z_j = Lambda_j^-1 y_j, denom = (sum_j tr Lambda_j^-1 / (T n))^2 (util.py:371-380), the gradient from u = Lambda^-1 z
   * and Lambda^-2 per frequency block.
   * ABI 18 -- CV of a multitask spectral fit (mt_tasks = T >= 2, equal n, fixed task kernel; util.py:381-394,
   * abstract_gp.py:261-272): K^-1's diagonal over the points of task t is I_t = (1/n) sum_j Lambda_j^-1[t, t] and
   * sum_i coeffs_{t,i}^2 = N_t = sum_j |z_{j,t}|^2, so loss = cv_weight sum_t N_t / I_t^2 (history [loss, nan, nan]);
   * one partials workgroup per (frequency block, task). */
  int loss_metric;
  double cv_weight;
  /* ABI 18 -- a LEARNED task kernel on the multitask spectral path (GCV / CV, mt_tasks = T, equal n; the reference's
   * default for num_tasks > 1, abstract_gp.py:116-139): mt_task_rg != 0 (bit 0: the factor, bit 1: the task noise
   * require grad) makes K_task = F F^T + diag(v) from raw itself -- raw = [scale, lengthscales, noise, F [T][mt_rank],
   * task noise [T]], v = exp (mt_vexp = 1) or the identity of the raw task noise; mt_kt is then not read -- and adds
   * the task parameters' closed-form gradients (dL/dK_task per task pair, the chain rule through F F^T + diag(v)) and
   * their Rprop steps (fgp_fit_desc.n_params covers them). */
  int mt_task_rg;
  int mt_rank;
  int mt_vexp;
} fgp_nll_desc;

#define FGP_LOSS_MLL 0
#define FGP_LOSS_GCV 1
#define FGP_LOSS_CV 2

/* A = 1/ev, ev = sqrt(n) lambda + exp(raw_noise), of the G problems of a spectral desc (basis non-NULL;
 * util.py:285,292-300 with lambda = scale sum_S l^S Phi_S, real): wa [G][n] float64 (lattice: the even
 * spectrum mirrored) -- fgp_inv_eig's wa without materialising lambda (ABI 12).  ysq / partials unused. */
int fgp_spec_inv_eig(const fgp_nll_desc* desc, double* wa, void* stream);

/* Posterior variance of the G problems of a lattice spectral desc with SHARED spectra (per-output
 * hyper-parameters on one point set; d <= 4) at N test points (ABI 13): abstract_gp.py:407-413's
 * K(x,x) - r^T K^-1 r with r^T K^-1 r = sum_k Re(A_k) |ft(r)_k|^2 (util.py:338-353), where ft of the kernel
 * row is formed from the hyper-parameter-free row spectra by linearity, ft(r_gt) = scale_g sum_S l_g^S
 * Psi_S(t), and A from the fit's part-product spectra -- one pass over Psi for every problem instead of
 * one transform per (problem, test point).
 *   psi      device complex128 [N][2^d][n]: fftbr (stable) of rho_S(t)[i] = prod_{j in S} part_j(x_t, x_i),
 *            the points in the GP's order (S = 0: the all-ones row)
 *   part0    host [d]: the parts at zero distance (K(x, x) = scale prod_j (1 + l_j part0_j))
 *   out      device float64 [G][N], clamped at 0
 *   partial  device scratch of G N ceil((n/2 + 1) / 1024) doubles
 * ysq / partials of the desc unused. */
int fgp_spec_post_var(const fgp_nll_desc* desc, const void* psi, int64_t N, const double* part0, double* out,
                      double* partial, void* stream);

/* Doubles the `partials` workspace of this desc needs (per-block partials + the fused fit's counters):
 * G (4 + d) (max(nb, n / 4096) + 1) + G, nb the kernels' block count (spectral path: up to 512). */
int fgp_nll_partials_len(const fgp_nll_desc* desc, int64_t* len);

/* Part-product spectra (ABI 11) for the spectral fit path.  With b_S[i] = prod_{j in S} parts[j, i]
 * (ascending j; b_{} = 1) for every subset S of the d dimensions (bit j of S = dimension j):
 *   Phi_S[k] = ft(b_S)[k],  k < K:
 *   lattice: Re fftbr(b_S) (stable; the lattice b_S is even in the natural index, so the spectrum is real
 *            and even and k = 0 .. n/2 carry it: K = n/2 + 1);  net: fwht(b_S) (stable), K = n.
 * Then for every (scale, l) the eigenvalues are lambda = scale sum_S l^S Phi_S -- ft(k1) of the
 * reference's _LamCaches (fastgps/util.py:95-112), k1 = scale prod_j (1 + l_j parts_j) of
 * abstract_fast_gp.py:181-191, by linearity of ft.
 * parts: [P][d][n] float64 (fgp_lattice_parts / fgp_lattice_parts_gen / fgp_net_parts layout; problem
 * stride parts_stride elements); 1 <= d <= 6.
 * basis: [P][Q][2^d][64] float64, Q = ceil(K / 64) chunks of 64 frequencies: Phi_S[k] at
 *   basis[p][k / 64][S][k mod 64]  (zeros past K)
 * -- the 2^d spectra of 64 consecutive frequencies are one contiguous 2^d x 512-byte run, the unit the fit
 * kernels stream (a row-per-spectrum layout puts them n/2 apart).
 * work: device scratch of work_bytes >= fgp_spec_basis_work bytes for ONE subset (the subsets are then
 * transformed in chunks; the bytes for all 2^d at once make it one chunk). */
int fgp_spec_basis(int family, const double* parts, int64_t parts_stride, int64_t P, int log2n, int d, double* basis,
                   void* work, int64_t work_bytes, void* stream);
/* Bytes of `work` for all 2^d subsets at once (divide by 2^d for the one-subset minimum). */
int fgp_spec_basis_work(int family, int log2n, int d, int64_t* bytes);
/* ABI 15 -- fgp_spec_basis of a LATTICE from its generating vector: the parts of fgp_lattice_parts_gen
 * (coef_j B_order((brev_m(i) z_j mod n) / n), z: [d] int64, coef: [d] host) regenerated inside the transform's
 * row pass instead of read from a d n parts array -- the same basis bit for bit.  17 <= log2n <= 24 (the
 * half-length transform path); work as fgp_spec_basis (family lattice). */
int fgp_spec_basis_gen(const int64_t* z, int log2n, int d, int order, const double* coef, double* basis, void* work,
                       int64_t work_bytes, void* stream);

#define FGP_PARTS_ARRAY 0
#define FGP_PARTS_LATTICE 1

/* Forward: k1 from the parts, lambda = ft(k1), ev = sqrt(n) lambda + noise; per-problem partial sums
 * of the norm term sum|ytilde|^2 Re(1/ev), logdet sum log|ev| and dL/dnoise.  The eigen-terms kernel
 * also runs the first (column) pass of the adjoint transform of dL/dlambda in place, so for
 * n > 4096 `work` holds that intermediate afterwards (consumed by fgp_nll_bwd). */
int fgp_nll_fwd(const fgp_nll_desc* desc, void* stream);
/* Eigenvalues only: lambda = ft(k1) (stable) written to desc->grad_lam ([G][n], complex128 lattice /
 * float64 net); ysq and partials are not used (replaces _LamCaches, fastgps/util.py:95-112). */
int fgp_nll_lam(const fgp_nll_desc* desc, void* stream);
/* Backward (after fgp_nll_fwd): g = Re(ft^H(dL/dlambda)), partial sums of dL/draw_scale and
 * dL/draw_lengthscales. */
int fgp_nll_bwd(const fgp_nll_desc* desc, void* stream);
/* One kernel of the fwd/bwd pipeline, for per-kernel timing (bench.py): stage 0 = forward row pass
 * (n <= 4096: the whole single-kernel iteration), 1 = column pass (eigen terms + adjoint columns),
 * 2 = adjoint row pass + gradient terms.  Stages 1-2 are no-ops for n <= 4096. */
int fgp_nll_stage(const fgp_nll_desc* desc, int stage, void* stream);

/* Rprop state and histories for the device-side fit loop. */
typedef struct fgp_fit_desc {
  int n_params;               /* length of raw (== total hyper-parameters of the desc) */
  double* raw;                /* [n_params] updated in place (the desc's raw) */
  double* rprop_prev;         /* [n_params] previous gradient (init 0) */
  double* rprop_step;         /* [n_params] step sizes (init lr) */
  double* grad_out;           /* [n_params] gradient of the last step (diagnostics) */
  double* loss_hist;          /* [max_iters][3] (or [max_iters][G][3] when per_problem): loss, term1 (norm),
                                 term2 (weighted logdet) */
  double* raw_hist;           /* [max_iters][n_params]: raw parameters at which the loss was evaluated */
  int scale_rg, ls_rg, noise_rg; /* requires_grad of each block */
  double mll_const;           /* d_out * n * log(2 pi) (fastgps/abstract_gp.py:235) */
  double eta_minus, eta_plus, step_min, step_max; /* torch.optim.Rprop defaults 0.5, 1.2, 1e-6, 50 */
  int per_problem;            /* 1: the G problems are independent GPs (each owns its parameters, loss, Rprop
                                 state; every *_pp flag must be set when G > 1), one fused reduce+step kernel */
  int hist_stride;            /* per_problem: problems per loss_hist row (0: G) -- a desc over problems
                                 [hist_offset, hist_offset + G) of a larger batch writes its slice of the rows */
  int hist_offset;
} fgp_fit_desc;

/* Reduce the partials of fgp_nll_fwd/bwd, assemble loss = 1/2 (term1 + term2 + mll_const), record
 * loss_hist[iter] and raw_hist[iter], and (if do_update) apply one Rprop step to raw. */
int fgp_fit_step(const fgp_nll_desc* nll, const fgp_fit_desc* fit, int iter, int do_update, void* stream);

/* Run `iters` complete fit iterations starting at history index iter0 (fwd, bwd, step per iteration;
 * the last one without update when final_no_update=1). Stream-ordered, no host synchronisation.
 */
int fgp_fit_run(const fgp_nll_desc* nll, const fgp_fit_desc* fit, int iter0, int iters, int final_no_update,
                void* stream);

/* ABI 17 -- fgp_fit_run through a hipGraph (AbstractGP.fit's loop at the replayed per-launch rate,
 * abstract_gp.py:241-296): on the spectral path (basis set, single task) and a stream that is not capturing, the
 * launch sequence is captured once per (token, arguments) and replayed; `token` names the caller's fit engine (its
 * buffers must not move while the token is live; fgp_fit_graph_release(token) when they are freed).  Bit-identical
 * to fgp_fit_run; other descs / a capturing stream run fgp_fit_run's eager sequence.  fgp_fit_graph_stats: out[0]
 * replays of a cached graph, out[1] captures, out[2] eager calls (since load). */
int fgp_fit_run_graph(const fgp_nll_desc* nll, const fgp_fit_desc* fit, int iter0, int iters, int final_no_update,
                      long long token, void* stream);
int fgp_fit_graph_release(long long token);
int fgp_fit_graph_stats(long long* out);

/* ---------------------------------------------------------------------------------------------
 * Prediction.
 * ------------------------------------------------------------------------------------------- */

/* Matrix-free posterior mean (replaces the kmat build + einsum of AbstractGP.post_mean,
 * fastgps/abstract_gp.py:352-380, with the fast-GP kernel of abstract_fast_gp.py:192-196):
 *   out[b, t] = sum_i K_g(xt[t], z[:, i]) coeffs[b, i],  g = b mod Gk,
 *   K_g(x, z) = hyp[g, 0] * prod_j (1 + hyp[g, 1 + j] part_j(x, z))   (hyp holds scale, lengthscales)
 * lattice: part_j = coef[j] B_{order[j]}((x_j - z_j) % 1), z float64 [d][n];
 * net:     part_j = walsh part of order order[j] (1..4, as fgp_net_parts; order = NULL: 1) of
 *          floor((x_j % 1) 2^tbits) XOR z_j, z int64 [d][n] (coef unused).
 * xt: [N, d] float64 contiguous; coeffs: [B][n] with row stride coeff_stride; 1 <= B <= 4, or (ABI 16) any B
 * when Gk == B (every output its own hyper-parameters: the blocks of 4 outputs run as one launch; out_stride
 * must then be N); out: [B][N] row stride out_stride; work: float64 scratch of ceil(n/chunk) * B * N entries. */
int fgp_post_mean(int family, const double* xt, int64_t N, const void* z, int64_t n, int d, int tbits, const int* order,
                  const double* coef, const double* hyp, int Gk, const double* coeffs, int64_t coeff_stride, int B,
                  double* out, int64_t out_stride, double* work, int64_t chunk, void* stream);

/* Posterior-variance quadratic form by Parseval, 13 <= log2n <= 24:
 *   out[t] = sum_i r_t[i] (K^-1 r_t)[i] = sum_k wa[k] |ft(r_t)[k]|^2,  r_t[i] = K(xt[t], z[:, i])
 * with wa = Re(1 / ev) (fastgps/abstract_gp.py:408-412 + util.py:338-353 for real kernel rows).
 * hyp: device [1 + d] (scale, lengthscales).  work: device scratch [N][n] (complex128 lattice,
 * float64 net); partial: device [N][n / 4096]; out: device [N]. */
int fgp_post_var_qf(int family, const double* xt, int64_t N, const void* z, int log2n, int d, int tbits,
                    const int* order, const double* coef, const double* hyp, const double* wa, void* work,
                    double* partial, double* out, void* stream);

/* Batched prediction over P independent GPs of one family / n / d (e.g. the randomly shifted
 * replicas of BASELINE config C4; each replaces one GP's AbstractGP.post_mean / post_var,
 * fastgps/abstract_gp.py:352-416).  Problem p owns training points z + p*z_stride ([d][n], float64
 * lattice / int64 net), hyper-parameter row hyp + p*hyp_stride ([1 + d]: scale, lengthscales),
 * coefficients coeffs + p*coeff_stride ([n], K^-1 y) and eigenvalue weights wa + p*wa_stride ([n],
 * Re(1/ev), post_var only).  order/coef as fgp_post_mean (lattice); tbits (net). */
typedef struct fgp_pred_desc {
  int family;
  int d;
  int tbits;
  int P;
  int64_t n;
  int order[FGP_MAX_D];
  double coef[FGP_MAX_D];
  const void* z;
  int64_t z_stride;
  const double* hyp;
  int64_t hyp_stride;
  const double* coeffs;
  int64_t coeff_stride;
  const double* wa;
  int64_t wa_stride;
  /* Training points source for fgp_post_var_batched: FGP_PARTS_ARRAY reads z; FGP_PARTS_LATTICE
   * regenerates the natural-order rank-1 lattice points x_ij = ((brev_m(i) z_j mod n) / n + shift_j) % 1
   * (bit-identical to fgp_lattice_points) from gen_z (host, 0 < gen_z[j] < 2^(53 - log2 n)) and the
   * device shift rows gen_shift + p * gen_shift_stride; z may then be NULL. */
  int points_gen;
  int64_t gen_z[FGP_MAX_D];
  const double* gen_shift;
  int64_t gen_shift_stride;
} fgp_pred_desc;

/* out[p, t] = sum_i K_p(xt_p[t], z_p[:, i]) coeffs_p[i]; xt_p = xt + p*xt_stride ([N, d]; stride 0 =
 * shared test points); out [P][N]; work: float64 scratch of fgp_post_mean_batched_work entries (ABI 16: the
 * training points per workgroup are chosen so that the launch fills its rounds of resident workgroups). */
int fgp_post_mean_batched(const fgp_pred_desc* desc, const double* xt, int64_t xt_stride, int64_t N, double* out,
                          double* work, void* stream);
int fgp_post_mean_batched_work(const fgp_pred_desc* desc, int64_t N, int64_t* work);

/* Posterior variance, 13 <= log2(n) <= 24 (AbstractGP.post_var, abstract_gp.py:381-416, n = the GP's n):
 *   out[p, t] = max(K_p(x, x) - sum_k wa_p[k] |ft(K_p(x_t, z_p))_k|^2, 0)  (negatives set to 0, :413)
 * with K_p(x, x) = scale_p prod_j (1 + l_pj part0[j]), part0 = the zero-distance kernel parts (host [d]).
 * work: device scratch [P][N][n] (complex128 lattice / float64 net); partial: [P][N][n / 4096]. */
int fgp_post_var_batched(const fgp_pred_desc* desc, const double* xt, int64_t xt_stride, int64_t N, const double* part0,
                         double* out, void* work, double* partial, void* stream);

/* A = 1/ev, ev = sqrt(n) lam + exp(raw_noise) (fastgps/util.py:285,292-300), for P problems:
 *   ya[p, k] = ytilde[p, k] * A[p, k]  (the tilde-domain solve of util.py:341-342), wa[p, k] = Re(A[p, k])
 * lam, ya: [P][n] contiguous (complex128 lattice / float64 net); ytilde row stride yt_stride; raw_noise
 * device, problem p at raw_noise[p * noise_stride]; wa may be NULL. */
int fgp_inv_eig(int family, const void* lam, const void* ytilde, int64_t yt_stride, const double* raw_noise,
                int64_t noise_stride, int64_t P, int log2n, void* ya, double* wa, void* stream);

/* Cross-kernel rows rows[g, t, i] = K_g(xt[t], z[:, i]) (same kernel as fgp_post_mean), [Gk][N][n],
 * N <= 65535: the kmat of AbstractGP.post_var / post_cov (fastgps/abstract_gp.py:407-411,452-457). */
int fgp_kernel_rows(int family, const double* xt, int64_t N, const void* z, int64_t n, int d, int tbits,
                    const int* order, const double* coef, const double* hyp, int Gk, double* rows, void* stream);




/* Natural-order digital net points (FastGPDigitalNetB2's sequences, fast_gp_digital_net_b2.py:266-273):
 * xb[i - n_min][j] = XOR_{k: bit k of i} C[j][k] XOR shift[j] (t-bit ints), x = xb 2^-t; C [d][mcols] and
 * shift [d] are DEVICE uint64 arrays; xb [n][d] int64 and / or x [n][d] float64 (either may be NULL). */
int fgp_net_points(const uint64_t* C, int mcols, const uint64_t* shift, int64_t n_min, int64_t n_max, int d, int t,
                   int64_t* xb, double* x, void* stream);

/* One DIT doubling stage (_LamCaches / _YtildeCache, fastgps/util.py:113-132,173-178): from ft of the first
 * n = 2^log2n values (prev) and of the next n (nxt) to ft of all 2n (out [batch][2n]):
 *   out[k] = (prev[k] + w^k nxt[k]) / sqrt(2), out[k + n] = (prev[k] - w^k nxt[k]) / sqrt(2),
 * w = exp(-pi i / n) for lattices (complex128, get_omega, fast_gp_lattice.py:261-262), w = 1 for nets
 * (float64, fast_gp_digital_net_b2.py:264-265).  Row strides in elements. */
int fgp_double_update(int family, const void* prev, int64_t prev_stride, const void* nxt, int64_t nxt_stride,
                      int64_t batch, int log2n, void* out, int64_t out_stride, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Multitask / derivative-informed fast GPs (num_tasks > 1 or derivative multi-indices).
 * Reference: fastgps/util.py:275-363 (_FastInverseLogDetCache with num_tasks > 1),
 * abstract_fast_gp.py:29-31,155-191 (task-pair lam caches, kernel parts with beta / kappa),
 * fast_gp_lattice.py:267-273 and fast_gp_digital_net_b2.py:289-301 (derivative parts).
 *
 * Block layout: the T ACTIVE tasks (n > 0) sorted by n descending (util.py:273), n[k] powers of two,
 * nmin = n[T-1], R = sum_k n[k] / nmin block rows.  The packed "lams" array of one problem holds, for
 * every pair k <= l (row-major over k, then l), the n[k] values lams[k, l] (the reference's
 * sqrt(n_l) lam_{k,l} * K_task[k, l] with the nugget on the diagonal pairs, util.py:284-298):
 * offset(k, l) = sum of n[k'] over the pairs before (k, l); L = sum_{k <= l} n[k] per problem.
 * Value q nmin + j of pair (k, l) is the coupling of block row (k, q) with (l, q mod (n[l]/nmin)) in
 * frequency class j.  All multitask arrays are complex128, [problem][L], problem stride L. */
#define FGP_MT_MAX_TASKS 16
#define FGP_MT_MAX_ROWS (1 << 24)

typedef struct fgp_mt_layout {
  int T;                              /* active tasks, 1 .. FGP_MT_MAX_TASKS */
  int64_t n[FGP_MT_MAX_TASKS];        /* their n, descending */
} fgp_mt_layout;

/* Kernel parts with derivative orders (_kernel_parts, abstract_fast_gp.py:173-180):
 *   parts[i][k][p][j], i < N (points x, row stride x_row_stride), k < M (points z), p < P (beta, kappa)
 *   pairs, j < d:  lattice (family 0, float64 points): coef[p d + j] * B_order((x_ij - z_kj) mod 1),
 *   order 1..8 (fast_gp_lattice.py:269-273);  net (family 1, int64 t-bit points):
 *   coef[p d + j] * (add[p d + j] + omega_order(xb_ij ^ zb_kj)), order 1..4 (fast_gp_digital_net_b2.py:
 *   291-301).  order / coef / add are DEVICE arrays [P][d].  zip = 1 (N == M): only the pairs (x_i, z_i),
 *   parts[i][p][j] (the kernel of x with itself in post_var, abstract_gp.py:407). */
int fgp_mt_parts(int family, const void* x, int64_t x_row_stride, int64_t N, const void* z, int64_t z_row_stride,
                 int64_t M, int zip, int d, int P, const int* order, const double* coef, const double* add, int tbits,
                 double* parts, void* stream);

/* Factor the transform-domain Gram blocks of G problems (replaces _FastInverseLogDetCache.__call__,
 * util.py:275-337): structured LDL^H per frequency class in the packed layout (factor [G][L]),
 * logdet [G][nmin] per class (sum over the classes = the reference's logdet, sum log|pivot| as its
 * recursion's log|S|, util.py:299,310), *info set to 1 (device int, zeroed by the caller) if a pivot is not
 * positive (a numerically indefinite block). */
int fgp_mt_factor(const fgp_mt_layout* layout, const void* lams, int64_t G, void* factor, double* logdet, int* info,
                  void* stream);

/* out[b] = Lambda_{b mod G}^-1 v[b] for B vectors v [B][R nmin] (row stride v_row_stride >= R nmin):
 * the tilde-domain solve of _gram_matrix_solve_tilde_to_tilde (util.py:354-363); out [B][R nmin]. */
int fgp_mt_solve(const fgp_mt_layout* layout, const void* factor, int64_t G, const void* v, int64_t v_row_stride,
                 int64_t B, void* out, void* stream);

/* Entries of A = Lambda^-1 on the packed coupling pattern (zinv [G][L]): the entries of the reference's
 * dense inverse `inv` (util.py:336) that the MLL gradient and post_cubature_var / cov
 * (abstract_fast_gp.py:82-154, inv[mvec, mvec, 0]) read. */
int fgp_mt_selinv(const fgp_mt_layout* layout, const void* factor, int64_t G, void* zinv, void* stream);

/* d(loss)/d(packed lams) for loss = f(norm_b, logdet_g), norm_b = Re(y_b^H A y_b), logdet_g = log det:
 * z = A y [B][R nmin] (fgp_mt_solve), grad_norm [B], grad_logdet [G], B a multiple of G (output b uses
 * problem b mod G); grad_lams [G][L] in torch's complex-gradient convention (dL/dRe + i dL/dIm). */
int fgp_mt_mll_grad(const fgp_mt_layout* layout, const void* zinv, const void* z, const double* grad_norm,
                    const double* grad_logdet, int64_t B, int64_t G, void* grad_lams, void* stream);

/* ABI 14 -- the Hermitian half of ft(real): fgp_fftbr_real's values at k = 0 .. n/2 only, rows of
 * out_batch_stride >= n/2 + 1 complex128 (ytilde of real observations: the coefficient solve
 * fgp_ifftbr_real_rf and Y read no more, and the other half is the conjugate mirror -- half the bytes
 * written).  fgp_sum_sq_half: Y [G][n] from such halves (x [R G] rows, Y mirrored to k > n/2), fgp_sum_sq's
 * values bit for bit. */
int fgp_fftbr_real_half(const double* in, int64_t in_batch_stride, void* out, int64_t out_batch_stride, void* work,
                        int64_t batch, int log2n, void* stream);
/* ABI 16 -- the same of float32 rows (16-byte aligned, stride a multiple of 4), widened to float64 exactly on load:
 * fgp_fftbr_real_half of the widened rows bit for bit (data_dtype=float32 observations, BASELINE config C5). */
int fgp_fftbr_real_half_f32(const float* in, int64_t in_batch_stride, void* out, int64_t out_batch_stride, void* work,
                            int64_t batch, int log2n, void* stream);
int fgp_sum_sq_half(const void* x, int64_t x_row_stride, int64_t R, int64_t G, int64_t n, double* out, void* stream);

/* ABI 14 -- the WHOLE fit of one small problem on the spectral path in ONE launch (G = 1, the part-product
 * spectra and Y within the LDS of 64 workgroups: e.g. n = 2^16, d = 3, or the probnum25 paper's n = 2^10):
 * iterations 0 .. iters of AbstractGP.fit (abstract_gp.py:241-296) -- loss history, gradient, Rprop and the
 * early-stopping rule (:276-284, logtol = log(1 + stop_crit_improvement_threshold), wait_max =
 * stop_crit_wait_iterations) -- with the multi-launch fgp_fit_run's arithmetic (bit-identical histories).
 * The last evaluated iteration applies no update.  ctrl: device scratch of >= 16 bytes; afterwards
 * ((int*)ctrl)[1] = the last iteration, ((int*)ctrl)[2] = 1 if an in-kernel barrier gave up (an error).
 * ABI 18: ((int*)ctrl)[3] = the best iteration (the first minimum of the loss history, NaN never best) and the fit
 * desc's raw holds ITS parameters (AbstractGP.fit's restored best_params, :285-296) -- rprop_prev / rprop_step the
 * final Rprop state -- so a caller restores the best iterate without reading anything back.
 * fgp_fit_persist_ok: *ok = the workgroup count it would use, 0 when the desc is outside its domain. */
int fgp_fit_persist_ok(const fgp_nll_desc* nll, int* ok);
int fgp_fit_persist(const fgp_nll_desc* nll, const fgp_fit_desc* fit, int iters, double logtol, int wait_max, void* ctrl,
                    void* stream);

/* ABI 14 -- device-resident MLL fit of a GENERAL multitask / derivative-informed GP: any n per task (the
 * structured blocks above), the task kernel K_task = F F^T + diag(v) learned or fixed, a data batch of B
 * vectors sharing the hyper-parameters.  Replaces AbstractGP.fit's MLL loop (abstract_gp.py:152-306) with
 * _FastInverseLogDetCache's lams / block inverse (util.py:275-370), its autograd gradient (:294, including
 * raw_factor_task_kernel / raw_noise_task_kernel, abstract_gp.py:116-139) and torch.optim.Rprop
 * (abstract_fast_gp.py:53-57).  Per iteration, with no host work:
 *   lams[k, l] = K_task[a_k, a_l] (sqrt(n_l) lam_kl + noise [k == l]),  lam_kl = scale sum_S l^S Phi^{kl}_S
 *   (the pair spectra: Phi^{kl}_S = fftbr / fwht of the part products of get_lam(a_k, a_l, n_k), conjugated
 *   when a_k > a_l -- util.py:280-284), the structured factor / solve / selected inverse / gradient of each
 *   frequency class, the contraction of dL/dlams with the spectra into the parameter gradients, and one
 *   reduction + Rprop step.
 * raw = [raw_scale, raw_lengthscales (dl), raw_noise, raw_factor_task_kernel (T_all x rank, row-major),
 *        raw_noise_task_kernel (T_all)]: scale / lengthscales / noise exp-transformed, the factor identity,
 *        the task noise exp (vtask_exp = 1) or identity (0).
 * loss_hist [iters][3] (loss, term1 = sum_b norm_b, term2 = logdet_weight logdet), raw_hist [iters][n_params]
 * (the parameters at which the row's loss was evaluated), grad_out [n_params] of the last iteration. */
typedef struct fgp_mt_fit_desc {
  int family, d, B;                   /* B data vectors (the reference's shape_batch, parameters unbatched) */
  fgp_mt_layout layout;               /* active tasks sorted by n descending */
  int task[FGP_MT_MAX_TASKS];         /* task index of active (sorted) task k */
  int T_all, rank, dl;                /* num_tasks, columns of the task factor, lengthscale count (1 or d) */
  const void* spectra;                /* complex128 pair spectra: sorted pair p = (k, l), k <= l row-major over
                                         (k, l), at spec_off[p]: [2^d][n_k] */
  int64_t spec_off[FGP_MT_MAX_TASKS * (FGP_MT_MAX_TASKS + 1) / 2];
  const void* y;                      /* complex128 [B][R nmin]: ytilde of the sorted tasks, rows concatenated */
  double* raw;
  int vtask_exp;
  int rg_scale, rg_ls, rg_noise, rg_factor, rg_vtask;   /* requires_grad of each parameter tensor */
  double* rprop_prev;                 /* [n_params] Rprop state (torch.optim.Rprop: prev, step_size) */
  double* rprop_step;
  double* grad_out;
  double* loss_hist;
  double* raw_hist;
  double grad_norm, grad_logdet;      /* dL/dnorm_b (1/2), dL/dlogdet (1/2 d_out / numel(logdet)) */
  double logdet_weight, mll_const, eta_minus, eta_plus, step_min, step_max;
  void* work;                         /* fgp_mt_fit_work bytes */
  /* ABI 16 -- PARAMETER batches (docs/examples/batch_multitask/fgp_lattice.ipynb: scale / lengthscales / noise / task
   * factor / task noise with batch dimensions broadcast to shape_batch, abstract_gp.py:73-139).  G >= 1 problems
   * (0 = 1), each with its own B data vectors at y + g B R nmin; problem g's parameters are row prow of each
   * parameter block, rows[q * G + g] (q = scale, lengthscales, noise, task factor, task noise; device int array;
   * NULL: every problem row 0) of nrows[q] rows (0 = 1).  raw = [scale rows, lengthscale rows (dl each), noise rows,
   * task-factor rows (T_all x rank each), task-noise rows (T_all each)].  The loss is the sum over the problems'
   * MLLs with logdet_weight; a parameter row shared by several problems gets the sum of their gradients. */
  int G;
  const int* rows;
  int nrows[5];
  /* ABI 16 -- the ADAPTIVE nugget (adaptive_nugget=True, util.py:286-290): sorted task k's diagonal block gets
   * noise |tr_kk / tr_ref| instead of noise, tr_kk = sum_i sqrt(n_k) lam_kk[i] = scale sqrt(n_k) sum_S l^S c_kS with
   * nugget_coef[k][S] = sum_i Phi^{kk}_S[i] (complex128 [T][2^d], the pair spectra's sums; NULL: the plain nugget)
   * and ref = the sorted position of task 0 (nugget_ref) -- its gradient w.r.t. the noise and the lengthscales
   * included. */
  const void* nugget_coef;
  int nugget_ref;
} fgp_mt_fit_desc;

int fgp_mt_fit_nparams(const fgp_mt_fit_desc* desc, int* n_params);
int fgp_mt_fit_work(const fgp_mt_fit_desc* desc, int64_t* bytes);
/* iterations iter0 .. iter0 + iters - 1 (history rows); with final_no_update the last one evaluates only */
int fgp_mt_fit_run(const fgp_mt_fit_desc* desc, int iter0, int iters, int final_no_update, void* stream);

/* ABI 15 -- consistency check of the fused spectral fit's last-arriver hand-off (a test hook, no reference
 * counterpart).  enable != 0 arms it for the following fgp_fit_run calls: every wave of the one-launch
 * iteration kernel XORs the bits of the partials it stored into a per-group word (agent-scope atomics, before
 * its arrival), and each group's last arriver recomputes that XOR from the partials it reads and counts a
 * mismatch.  enable == 0 synchronises the device, disarms it and returns out[0] = group hand-offs checked,
 * out[1] = mismatches (0 when every arriver saw every stored partial). */
int fgp_handoff_check(int enable, unsigned long long* out);

/* ABI 16 -- test hook (no reference counterpart): the bound of fgp_fit_persist's in-kernel barrier polls (a
 * negative value restores the default 2^22).  0 makes every barrier wait that does not find the grid complete
 * give up at once, so the failure path (fit parameters and parameter history set to NaN, ((int*)ctrl)[2] = 1)
 * and the host's fallback to the launch per iteration can be tested.  fgp_fit_persist_ok / fgp_fit_persist
 * also report unsupported (0 / an error) when the workgroups would not all be co-resident. */
int fgp_set_persist_poll_max(long long polls);

/* ABI 17 -- the library's sticky count of fgp_fit_persist barrier give-ups (a give-up counts once per workgroup that
 * gave up; never cleared by a launch): read after hipGraph replays of captured fits, whose control words cannot be read
 * during the capture (AbstractGP.fit's result would otherwise be NaN parameters nobody reported, abstract_gp.py:297-298).
 * Synchronises the device; reset != 0 zeroes the count after reading it. */
int fgp_persist_giveups(unsigned long long* count, int reset);

/* ABI 16 -- test hook (no reference counterpart): the per-class kernel of fgp_mt_fit_run: 0 automatic (a wave per
 * frequency class while problems x classes <= 8192 and a class fits 60 KB of LDS, else a thread per class), 1 a
 * thread per class, 2 a wave per class where it fits.  Both give the same results bit for bit. */
int fgp_set_mt_class_kernel(int mode);

#ifdef __cplusplus
}
#endif

#endif /* FGP_HIP_H_ */
