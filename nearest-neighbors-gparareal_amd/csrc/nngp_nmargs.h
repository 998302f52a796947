// nngp_nmargs.h -- the argument block of the Nelder-Mead fit kernels (nngp_gp.hip: the packed,
// speculative and mean kernels; nngp_nmlane.hip: the throughput kernel), and the launch entry of
// the throughput kernel.
#pragma once

#include "common.h"
#include "nngp_nm.h"

namespace nngp {

static constexpr int MAX_JIT = 16;

struct NMArgs {
    int m, d, n_fits;
    const double *D2;      // [m][m]
    const double *kd2;     // [m] (FUSED)
    const double *Y;       // y of fit f, row r: Y[coord*ys_c + r*ys_r]
    int ys_c, ys_r;
    const int32_t *coord;        // unfused: per-fit coordinate
    const int32_t *jitter_idx;   // unfused: per-fit jitter index
    const double *theta0;        // [n_fits][2]
    double fatol, xatol;
    int maxfev;
    int nj, R, cpw;              // FUSED: jitters, restarts, coordinates per workgroup
    double jit_pow[MAX_JIT];     // 10**jitter_exp (host pow)
    double *theta_out;           // [n_fits][2] or null
    double *fval_out;            // [n_fits] or null
    int32_t *nfev_out;           // [n_fits] or null
    double *fits_out;            // [n_fits][4] or null
    double *preds;               // FUSED [d]
    const double *bias;          // FUSED [d] or null
    double *out;                 // FUSED [d] (preds + bias) or null
    // speculative sweep
    const int32_t *skip;         // fits kernels: if *skip the launch does nothing (speculation hit)
    const double *fits_alt;      // gp_mean_kernel: arg-min over fits_alt instead if *skip == 1,
    const double *fits_alt2;     //   over fits_alt2 if *skip == 2
    // batched predictions (unfused fits kernel, blockIdx.y = prediction): per-prediction strides
    int64_t qs_D2, qs_Y, qs_th, qs_fits;
    // unfused fits kernel: per-prediction work queues ([gridDim.y] counters, zeroed) -- a row whose
    // fit is done takes the next unassigned fit, or NULL (one fit per row)
    int32_t *queue;
    // tail hand-off (single prediction): the packed kernel parks a fit whose evaluation count
    // reaches park_cap (its Nelder-Mead state, pending request included, in park[f], f appended to
    // park_list); the speculative kernels then resume the parked fits (resume != 0).  park_count[0]
    // finite fits sit at the front of park_list, park_count[1] all-+inf ones at its back.  The
    // two-level resume (nm_spec2_kernel<M, 0>) gives a finite fit 4 waves while their count is
    // <= resume_w4, 2 while <= resume_w2, else 1; an all-+inf fit one
    int park_cap, resume, resume_w4, resume_w2;
    // unfused fits in product order (coord null): rows take fits jitter-major (slot s -> fit
    // (s % d) * nfc + s / d), so a wave's rows share a jitter (and, for R = 1, differ in the
    // coordinate only); the kernel matrix K depends on (theta, jitter), not on the coordinate
    int jmajor;
    NM *park;
    int32_t *park_list, *park_count;
    // overlapped speculative batch: the fits kernel counts each prediction's finished fits
    // (done[blockIdx.y], after a device-scope fence); the sweep's mean kernel, on a hit served by
    // that batch, waits until wait_done reaches wait_n -- for at most wait_ticks of the 100 MHz
    // wall clock (NNGP_SPEC_WAIT_US, default 2 s; 0 = give up at once, even if the fits are done);
    // past that, or once an earlier slice has given up (*err != 0), it sets *err and writes nothing
    int32_t *done;
    const int32_t *wait_done;
    int wait_n;
    int32_t *err;
    uint64_t wait_ticks;
};

// apply the blockIdx.y prediction offsets of a batched launch (all zero otherwise)
__device__ __forceinline__ void nm_batch_offsets(NMArgs &a) {
    const int64_t y = blockIdx.y;
    a.D2 += y * a.qs_D2;
    a.Y += y * a.qs_Y;
    a.theta0 += y * a.qs_th;
    if (a.fits_out) a.fits_out += y * a.qs_fits;
}

// static-index lookup (a runtime index into a by-value kernel-argument array would go to scratch)
__device__ __forceinline__ double jit_lookup(const NMArgs &a, int j) {
    double v = 1.0;
#pragma unroll
    for (int i = 0; i < MAX_JIT; i++)
        if (i == j) v = a.jit_pow[i];
    return v;
}


// the throughput-shaped fits kernel (nngp_nmlane.hip): LPF lanes per fit, exact m (no padding);
// for the unfused batched mode (work queues per prediction, no tail hand-off).  Returns
// NNGP_E_UNSUPPORTED -- and launches nothing -- when m has no instantiation.
bool nm_lanes_supported(int m);
int run_nm_lanes(NMArgs &a, hipStream_t st, int nq, int qslot);

}  // namespace nngp
