// common.h -- shared host/device helpers of libnngp_hip.so (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdio>
#include <cstdlib>
#include <string>

#include "../../include/nngp.h"

namespace nngp {

// integer tuning/test knob from the environment (read on every call: tests toggle them in-process)
inline int env_int(const char *name, int dflt) {
    const char *e = getenv(name);
    return e ? atoi(e) : dflt;
}

// attributes of the CURRENT device (hipGetDevice), cached per device: compute units, and the
// rate of the 100 MHz wall clock the kernels read (wall_clock64) in kHz
int device_cus();
double device_wallclock_khz();

// thread-local last error, returned by nngp_last_error()
void set_error(const char *fmt, ...);

#define NNGP_HIP_CHECK(expr)                                                                 \
    do {                                                                                     \
        hipError_t _e = (expr);                                                              \
        if (_e != hipSuccess) {                                                              \
            ::nngp::set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e),         \
                              __FILE__, __LINE__);                                           \
            return NNGP_E_HIP;                                                               \
        }                                                                                    \
    } while (0)

#define NNGP_REQUIRE(cond, ...)                                                              \
    do {                                                                                     \
        if (!(cond)) {                                                                       \
            ::nngp::set_error(__VA_ARGS__);                                                  \
            return NNGP_E_ARG;                                                               \
        }                                                                                    \
    } while (0)

// launch-error check right after a <<<>>> launch
#define NNGP_LAUNCH_CHECK()                                                                  \
    do {                                                                                     \
        hipError_t _e = hipGetLastError();                                                   \
        if (_e != hipSuccess) {                                                              \
            ::nngp::set_error("kernel launch failed: %s (%s:%d)", hipGetErrorString(_e),     \
                              __FILE__, __LINE__);                                           \
            return NNGP_E_HIP;                                                               \
        }                                                                                    \
    } while (0)

// Grow-only device scratch owned by the library (per device and slot), so that steady-state
// calls never allocate.  Slot 0: per-call scratch (nngp_knn / nngp_predict / ...); slot 1: the
// speculative sweep's batch buffers, which must outlive the per-slice calls.  Growing a slot
// frees the old buffer after hipFree's implicit device synchronisation.  Not thread-safe across
// host threads sharing a device.
constexpr int N_WS_SLOTS = 10;   // slot 2: the sweep's speculation buffers; 3: full-GP factors; 4: fit queues; 5: parked fits;
                                // 6: the re-speculation window's batch (slot 1 may still be read by an overlapped batch);
                                // 7 / 8: the fit queues of the overlapped batch / of the re-speculation window;
                                // 9: the sharded sweep's zeros (nngp_comm.hip)
void *workspace(size_t bytes, int *err, int slot = 0);

// A prepared coordinate of gp_pre_kernel: alpha rows 0..maxm-1 | c | psy | ok
__host__ __device__ constexpr int HM_STRIDE(int maxm) { return maxm + 3; }

// The sweep's split prediction (nngp_sweep.hip): a select whose ordered list hits a speculative
// prediction that gp_pre_kernel has already prepared (done[0] == target) finishes the slice's
// posterior mean itself -- from the prepared coordinates and the query's kd2, gp_mean_finish --
// and reports hit + 2 to the host, which then launches no mean kernel for the slice.
struct HitMean {
    const double *AP1, *AP2;          // the slice's prepared coordinates for hit 1 / hit 2 (or null)
    const int32_t *done1, *done2;     // their gp_pre workgroup counters (the slice's entry)
    int target;                       // gp_pre workgroups per prediction
    int maxm;                         // the padded fit size the coordinates were prepared at
    const double *bias;               // UG1[i+1]
    double *out, *preds;              // U1[i+1] = mean + bias, preds = mean
    // profiling (NNGP_SEL_PROF=1, any select of predict_impl): wall-clock sums, relative to each
    // launch's start, at the select's marks (rounds | merges | gathers | D2) and its end, + launches
    uint64_t *marks;
};
// the select-profile buffer (uint64_t[6]) when NNGP_SEL_PROF=1, else null; sel_prof_report prints
// and clears it (the correction sweep, at its end)
uint64_t *sel_prof_marks();
void sel_prof_report(const char *what);

// predict_impl's launches in parts (the speculative sweep issues the select, reads its hit flag on
// the host, and then launches the fits only on a miss): all | kNN + select | fits + mean | mean only
enum { PREDICT_ALL = 0, PREDICT_SELECT = 1, PREDICT_FITS_MEAN = 2, PREDICT_MEAN = 3, PREDICT_SELECT_ONLY = 4 };
// the slice head G(U1[i]) + the query's distances as one launch (gdist_kernel): PREDICT_SELECT_ONLY
// then launches the select alone.  gdist_supported: systems with an in-kernel G (NNGP_GDIST=0: off)
bool gdist_supported(const nngp_system *sys, int g_step_mode);
bool g_side_supported(const nngp_system *sys, int g_step_mode);
int gdist(const nngp_system *sys, int g_tableau, int g_step_mode, int64_t g_steps, const double *t, int i,
          const double *X, int64_t rows, int d, int m, int n_jitter, int n_restarts, const double *ui,
          double *ug_next, hipStream_t st);
int predict_impl(const double *X, const double *Y, int64_t rows, int d, const double *new_x, int m,
                 int n_jitter, const double *jitter_exp_host, int n_restarts, const double *theta0,
                 double fatol, double xatol, int maxfev, double *preds_out, const double *bias,
                 double *out, double *fits_out, const int32_t *spec_idx, const double *spec_fits,
                 int32_t *hit_flag, const int32_t *spec2_idx, const double *spec2_fits, int32_t *host_flag,
                 hipStream_t st, int c0 = 0, int c1 = -1, const int32_t *wait_done = nullptr,
                 int32_t *wait_err = nullptr, int phase = PREDICT_ALL, const HitMean *hm = nullptr,
                 hipEvent_t bias_ready = nullptr);
int gpfull_mean(const double *X, int64_t rows, int d, const double *q, const double *coef, const double *alpha,
                const double *bias, double *out, hipStream_t st);
int spec_batch(const double *X, const double *Y, int64_t rows, int d, const double *Q, int nq, int m,
               int n_jitter, const double *jitter_exp_host, int n_restarts, const double *theta0,
               double fatol, double xatol, int maxfev, int32_t *idx_out, double *fits_out, bool latency,
               hipStream_t st, int slot = 1, int32_t *done = nullptr, hipEvent_t ev_select = nullptr,
               double *pre_AP = nullptr, int32_t *pre_done = nullptr);
// gp_pre_kernel's workgroups per prediction (the HitMean target) for d coordinates at fit size m
int pre_target(int d, int m);
int pre_maxm(int m);   // the padded fit size of m
// the fused correction chain (nngp_gp.hip): one persistent kernel per run of hit slices
void chain_release();   // nngp_shutdown's parts (nngp_gp.hip / nngp_sweep.hip / nngp_comm.hip)
void sweep_release();
void comm_release();
// grow-only pool of timing events (nngp_sweep.hip): *out = n events
int timing_events(size_t n, hipEvent_t **out);
bool chain_supported(const nngp_system *sys, int g_step_mode, int m);
bool guess_chain_supported(const nngp_system *sys, int g_step_mode);
int guess_chain(const nngp_system *sys, int g_tableau, int g_step_mode, int64_t g_steps, const double *t, int I,
                int nq, const double *UF, const double *UG, double *Q, double *gtmp, hipStream_t st);
int chain_sweep(const nngp_system *sys, int g_tableau, int g_step_mode, int64_t g_steps, const double *t, int I,
                int N, int i0, double *U1, double *UG1, const double *X, const double *Y, int64_t rows, int m,
                int n_jitter, const double *jitter_exp_host, int n_restarts, int32_t *flags,
                const int32_t *spec_idx, const double *spec_fits, const int32_t *spec2_idx,
                const double *spec2_fits, double *preds, int *stop_out, float *g_ms_out, hipStream_t st);
int chain_miss_fits(int64_t rows, int d, int m, int n_jitter, const double *jitter_exp_host, int n_restarts,
                    const double *theta0, double fatol, double xatol, int maxfev, double *preds,
                    const double *bias, double *out, hipStream_t st);

}  // namespace nngp
