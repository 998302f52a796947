/*
 * nngp.h -- C-ABI of libnngp_hip.so, the MI355X (gfx950) hot path of nnGParareal.
 *
 * The reference (Python + jax, /root/reference) has no native code: its hot path is three
 * duck-typed Python plugin calls that a process pool fans out:
 *
 *   1. propagator  SolverAbstr.run_F/run_G(t0, t1, u0) -> u1      solver.py:29-69, 86-107
 *                  (Parareal fans run_F over slices: parareal.py:310-315)
 *   2. model       NNGP_p.predict(new_x, ...) -> preds[d]          models.py:171-226
 *                  (kNN :177-179, n*9*R Nelder-Mead fits of the -LML :185-202, 228-260,
 *                   argmin :207-215, posterior mean :162-168, 217)
 *   3. executor    pool.map(fn, *iterables)                        parareal.py:16-24, 58-64
 *
 * Each entry point below replaces one of those call sites with ONE stream-ordered launch
 * sequence on the GPU.  Python binds them through ctypes (INTEGRATION.md shows the binding).
 *
 * Conventions
 *   - All array arguments are DEVICE pointers (hipMalloc / torch.cuda memory) unless the
 *     parameter name ends in `_host`.  Layouts are row-major: states are [n_slices][d], which
 *     is exactly the reference's u[i, :, k] slice for consecutive i.
 *   - Every call is asynchronous on `stream` (a hipStream_t; NULL = default stream) and
 *     returns 0 on success, a negative NNGP_E_* code otherwise; nngp_last_error() gives a
 *     thread-local message.  Nothing here allocates per call except the library's own
 *     grow-only device workspace (nngp_predict), so steady-state calls never hit hipMalloc.
 *   - Arithmetic is IEEE fp64 throughout (the reference runs jax with x64 enabled,
 *     e.g. models.py:8, RK.py:13).  Kernels are built with -ffp-contract=off so that every
 *     add/mul rounds exactly where the reference's does.
 */
#ifndef NNGP_H_
#define NNGP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NNGP_ABI_VERSION 1

/* error codes */
#define NNGP_OK 0
#define NNGP_E_ARG (-1)       /* invalid argument (shape, enum, null pointer)            */
#define NNGP_E_HIP (-2)       /* a HIP runtime call failed                               */
#define NNGP_E_UNSUPPORTED (-3) /* valid in the reference but not (yet) on this path     */

/* Vector fields.  Reference: systems.py (modern) and new_lib.Systems (legacy twin). */
enum nngp_system_kind {
    NNGP_SYS_LORENZ = 0,            /* systems.py:225-247                                  */
    NNGP_SYS_HOPF = 1,              /* systems.py:140-172 (non-autonomous Hopf), param[0]=maxtime */
    NNGP_SYS_THOMAS_LABYRINTH = 2,  /* systems.py:250-288                                  */
    NNGP_SYS_FHN_ODE = 3,           /* systems.py:80-106                                   */
    NNGP_SYS_ROSSLER = 4,           /* systems.py:109-137                                  */
    NNGP_SYS_BRUSSELATOR = 5,       /* systems.py:202-222                                  */
    NNGP_SYS_DBL_PEND = 6,          /* systems.py:175-199                                  */
    NNGP_SYS_BURGERS = 7,           /* systems.py:402-459, nx = d, param[0] = nu           */
    NNGP_SYS_FHN_PDE = 8            /* systems.py:291-398, nx = d_x, d = 2*d_x*d_x         */
};

/* Explicit Runge-Kutta tableaux, RK.py:30-48 (value = order). */
enum nngp_tableau { NNGP_RK1 = 1, NNGP_RK2 = 2, NNGP_RK4 = 4, NNGP_RK8 = 8 };

/* Step-size convention.
 *   FIXED:    h = (t1 - t0)/steps for every step          RK.run_get_last, RK.py:101-109
 *   LINSPACE: h_n = t[n+1] - t[n], t = np.linspace(t0, t1, steps+1)
 *             RK.run / legacy new_lib.RK (RK.py:91-99, new_lib.py:87-137) -- the convention
 *             of every published scalability run.
 * NNGP_STEP_CONTRACT (a flag OR-ed onto either mode; opt-in, not a reference behaviour): run the
 *   propagator's second code object, compiled with a*b+c contracted to fma.  Fewer fp64
 *   instructions per step (the fine sweep is instruction-issue-bound), results no longer bitwise
 *   the reference's rounding order: per-slice end states agree to <= 1e-12 relative on the
 *   test schedules (tests/test_gpu_contract.py).  Every other entry point ignores it.        */
enum nngp_step_mode { NNGP_STEP_FIXED = 0, NNGP_STEP_LINSPACE = 1, NNGP_STEP_CONTRACT = 16 };

/* One ODE/PDE right-hand side, optionally wrapped by the '-11' normalisation of
 * ODE.get_vector_field (systems.py:32-44, utils.py:14-33):
 *     f_n(u) = f((u+1)/2*(mx-mn) + mn) * (2/(mx-mn))                                       */
typedef struct nngp_system {
    int32_t kind;        /* enum nngp_system_kind                                         */
    int32_t d;           /* state dimension                                               */
    int32_t nx;          /* grid points per axis (Burgers: d; FHN_PDE: d_x); else 0        */
    int32_t normalized;  /* 0: identity, 1: '-11' wrapper                                 */
    double param[4];     /* HOPF: [0]=maxtime (tspan[1]); BURGERS: [0]=nu; else unused     */
    const double *norm;  /* DEVICE [3*d] = mn | (mx-mn) | 2/(mx-mn), or NULL if identity   */
} nngp_system;

/* ---- library ---------------------------------------------------------------------------- */
int nngp_abi_version(void);
const char *nngp_last_error(void);
/* Number of visible HIP devices (0 when no GPU); never fails. */
int nngp_device_count(void);

/* ---- 1. fine / coarse propagator --------------------------------------------------------
 * Replaces: SolverRK.run_F / run_G for every slice of one Parareal iteration
 *           (solver.py:86-107 via RK.run_get_last RK.py:101-109 / _RK_jax_last RK.py:146-174),
 *           as fanned out by pool.map(solver.run_F_timed, ...) at parareal.py:310-315, and the
 *           legacy RK_last (new_lib.py:57-69, 939-945).
 * Integrates n_slices independent initial values u0[i] from t0[i] to t1[i] with `steps`
 * steps of tableau `tableau`; writes the end states to uF[i].  The paging quirk of
 * solver.py:86-99 is a host-side loop over pages calling this once per page.
 * t0, t1: DEVICE [n_slices]; u0, uF: DEVICE [n_slices][sys->d]; uF may alias u0.          */
int nngp_rk_batch(const nngp_system *sys, int tableau, int step_mode, int n_slices,
                  const double *t0, const double *t1, int64_t steps, const double *u0,
                  double *uF, void *stream);

/* Legacy global-grid variant (the legacy driver's initial coarse sweep, new_lib.py:902-906,
 * integrates ONE np.linspace(g0, g1, gsteps+1) grid and sub-samples it at slice boundaries).
 * Slice i performs grid steps j0[i] .. j0[i]+steps-1 of the grid (g0[i], g1[i], gsteps):
 * t[j] = j*((g1-g0)/gsteps) + g0, t[gsteps] = g1, h = t[j+1]-t[j].  j0: DEVICE int64 [n].  */
int nngp_rk_batch_grid(const nngp_system *sys, int tableau, int n_slices, const double *g0,
                       const double *g1, int64_t gsteps, const int64_t *j0, int64_t steps,
                       const double *u0, double *uF, void *stream);

/* Vector field evaluation f_n(u) for n states (what ODE.get_vector_field() returns as a
 * callable, systems.py:32-44).  u, out: DEVICE [n][sys->d].                                 */
int nngp_rhs_batch(const nngp_system *sys, int n, const double *u, double *out, void *stream);

/* Elementwise  out = (a - b) + c   (c may be NULL: out = a - b), n doubles, DEVICE.
 *   Parareal update with the classic model: u = (uF_prev - uG_prev) + uG_new
 *   (models.py:82-83 + parareal.py:382); training targets D = uF - uG (parareal.py:337).     */
int nngp_parareal_update(int64_t n, const double *a, const double *b, const double *c,
                         double *out, void *stream);

/* ---- 2. nnGP correction -----------------------------------------------------------------
 * kNN (models.py:177-179): indices of the m rows of X[rows][d] nearest to q[d] in squared
 * euclidean distance, ascending, ties broken by row index.  idx_out: DEVICE int32 [m];
 * dist_out: DEVICE [m] or NULL.  Requires 1 <= m <= rows.                                   */
int nngp_knn(const double *X, int64_t rows, int d, const double *q, int m, int32_t *idx_out,
             double *dist_out, void *stream);

/* Batched hyper-parameter fits, replacing pool.map(NNGP_p._get_opt_par, ...) at
 * models.py:197-202 -> opt_theta (models.py:254-260) -> scipy Nelder-Mead on log_lik
 * (models.py:240-252).  Fit f minimises -LML(theta | xm, ym[:, coord[f]], 10**jitter) with
 * jitter = jitter_exp_host[jitter_idx[f]], starting from theta0[f], by the rules of scipy's
 * _minimize_neldermead (rho=1, chi=2, psi=0.5, sigma=0.5, 5% initial simplex, xatol/fatol stop,
 * maxiter = maxfev).  A NaN -LML (failed Cholesky) counts as +inf (models.py:250-251).
 *   xm, ym: DEVICE [m][d]; coord, jitter_idx: DEVICE int32 [n_fits]; theta0: DEVICE [n_fits][2];
 *   jitter_exp_host: HOST [n_jitter] exponents (e.g. -20..-12, models.py:186);
 *   theta_out: DEVICE [n_fits][2]; fval_out: DEVICE [n_fits]; nfev_out: DEVICE int32 or NULL.
 * Requires 1 <= m <= 64 (fits padded to 8/16/20/24/32/48/64 rows; m > 32 runs 3-4 kernel rows
 * per lane, one wave per workgroup).                                                        */
int nngp_nm_fit_batch(int m, int d, const double *xm, const double *ym, int n_fits,
                      const int32_t *coord, const int32_t *jitter_idx, int n_jitter,
                      const double *jitter_exp_host, const double *theta0, double fatol,
                      double xatol, int maxfev, double *theta_out, double *fval_out,
                      int32_t *nfev_out, void *stream);

/* Posterior mean K(xm, new_x)^T alpha per coordinate c with hyper-parameters theta[c] and
 * jitter 10**jitter_exp_host[jitter_idx[c]] (models.py:162-168, 217).  NaN if the Cholesky
 * fails (jax semantics).  theta: DEVICE [d][2]; jitter_idx: DEVICE int32 [d]; out: DEVICE [d]. */
int nngp_gp_mean(int m, int d, const double *xm, const double *ym, const double *new_x,
                 const double *theta, const int32_t *jitter_idx, int n_jitter,
                 const double *jitter_exp_host, double *out, void *stream);

/* One full correction for one slice = NNGP_p.predict (models.py:171-226) fused:
 * kNN over the training set X/Y[rows][d] at new_x[d], d*n_jitter*n_restarts fits in the
 * reference's product(coord, jitter, restart) order (models.py:186-192) starting from
 * theta0[d*n_jitter*n_restarts][2] (the host replays rng.integers(-8, 0, 2) in that order),
 * per-coordinate first-argmin of fval (models.py:207-215) and the posterior mean.
 *   preds_out = mean;  if bias != NULL also out = preds + bias (parareal.py:382).
 *   fits_out: DEVICE [n_fits][4] = (theta_x, theta_y, fval, nfev) or NULL.
 *   jitter_exp_host: HOST [n_jitter]. All other arrays DEVICE.  Requires 1 <= m <= 64.   */
int nngp_predict(const double *X, const double *Y, int64_t rows, int d, const double *new_x,
                 int m, int n_jitter, const double *jitter_exp_host, int n_restarts,
                 const double *theta0, double fatol, double xatol, int maxfev,
                 double *preds_out, const double *bias, double *out, double *fits_out,
                 void *stream);

/* nngp_predict_range: the coordinates [c0, c1) of nngp_predict (their fits, in the same
 * product order with their own rows of theta0 = the FULL [d*n_jitter*n_restarts][2] draws, and
 * their means) into preds_out [c1-c0]: a rank's share of one prediction when the multi-GPU
 * sweep shards the d*9*R fits by coordinate (parareal.correction_sweep_sharded).
 * Concatenating the ranges gives nngp_predict's preds bit for bit. */
int nngp_predict_range(const double *X, const double *Y, int64_t rows, int d, const double *new_x,
                       int m, int n_jitter, const double *jitter_exp_host, int n_restarts,
                       const double *theta0, int c0, int c1, double fatol, double xatol, int maxfev,
                       double *preds_out, void *stream);

/* ---- 3. the sequential correction sweep of one Parareal iteration ------------------------
 * Replaces the loop parareal.py:359-382 (legacy new_lib.py:990-1012): for i = I .. N-1
 *     UG1[i+1] = G(t[i], t[i+1], U1[i])                     run_G_timed, parareal.py:361
 *     U1[i+1]  = correction(U1[i]) + UG1[i+1]                  parareal.py:367-368, 382
 * with correction = (UF[i+1] - UG[i+1]) for NNGP_MODEL_PARAREAL (models.py:82-83) or the
 * nnGP prediction for NNGP_MODEL_NNGP (= nngp_predict on X/Y[rows][d] with m neighbours,
 * theta0 = the (N-I) predictions' initial thetas back to back, [(N-I)][d*n_jitter*n_restarts][2]).
 * All slice launches are queued on `stream` without host synchronisation.
 *   t: DEVICE [N+1]; U1, UG1: DEVICE [N+1][d] (rows I.. read, rows I+1.. written);
 *   UF, UG: DEVICE [N+1][d] (parareal model; for nngp they enable speculation);
 *   preds_scratch: DEVICE [d] (nngp only);
 *   speculate (nngp): -1 auto, 0 off, 1 on.  Every slice's query is guessed by the classic
 *     Parareal update along the coarse chain and all their fits run as ONE batched launch; a
 *     slice whose actual ordered kNN list equals its guess reuses those fits (bitwise identical:
 *     a fit depends only on the ordered neighbours, coordinate, jitter and theta0), the others
 *     are recomputed in the sweep.  Auto speculates while (N-I)*d*n_jitter*n_restarts <= 262144.
 *     The batch's fits overlap the sweep on a side stream (a hit waits for its own prediction's
 *     fits; NNGP_SPEC_OVERLAP=0 serialises them); the call returns after both have drained.
 *   spec_hits_out: HOST, number of slices served by the speculative batch, or NULL;
 *   g_ms_out: HOST, total device time of the G launches (ms), or NULL (no timing events).
 * With NNGP_CHAIN=1, speculation on, an ODE or Burgers (d = 64k <= 256) system, exact G and m <= 24, the runs
 * of hit slices go through ONE persistent cooperative kernel (G, kNN, hit check, arg-min, mean
 * and update per slice, grid barriers between the phases; the host takes over at each miss):
 * bitwise the launch chain.  Opt-in (NNGP_CHAIN=1): measured not faster than the launch chain
 * on MI355X, so the launch chain stays the default.                        */
#define NNGP_MODEL_PARAREAL 0
#define NNGP_MODEL_NNGP 1
/* NNGP_MODEL_GPFULL: the full-data GP posterior mean (GPjax_p.predict, models.py:456-462) with
 * Y = alpha DEVICE [d][rows] and theta0 = coefficients DEVICE [d][2] = (-0.5/sigma_x^2, sigma_y^2)
 * from nngp_gpfull_fit/nngp_gpfull_lml; m, n_jitter, jitter_exp_host, n_restarts, fatol, xatol,
 * maxfev, preds_scratch and speculate are unused. */
#define NNGP_MODEL_GPFULL 2
int nngp_correction_sweep(const nngp_system *sys, int g_tableau, int g_step_mode, int64_t g_steps,
                          const double *t, int I, int N, double *U1, double *UG1, const double *UF,
                          const double *UG, int model, const double *X, const double *Y, int64_t rows,
                          int m, int n_jitter, const double *jitter_exp_host, int n_restarts,
                          const double *theta0, double fatol, double xatol, int maxfev,
                          double *preds_scratch, int speculate, int32_t *spec_hits_out, float *g_ms_out,
                          void *stream);

/* Counters of the fused correction chain since the library was loaded (this process): kernel
 * launches, and slices it completed (G through the update) -- the rest of the sweep's slices were
 * misses finished by the host's fits.  Returns launches; *slices_out (HOST, optional). */
int64_t nngp_chain_stats(int64_t *slices_out);

/* Sweeps (this process) that were run a second time with the speculative batch serialised
 * because a hit slice's wait for the overlapped batch timed out (NNGP_SPEC_WAIT_US, default 2 s;
 * the first pass wrote nothing for that slice, and the rerun gives the same bits).            */
int64_t nngp_sweep_late_reruns(void);

/* Drains the device and releases every resource the library holds (workspaces, side streams,
 * events, host-mapped flags); the next call re-creates what it needs.  Registered with atexit
 * by the Python package, so none of them is left to the HIP runtime's process-exit teardown.
 * (No reference counterpart: the reference holds no device resources.)  Returns 0.
 * Threading: the library serves one host thread per process (the reference's host loop is
 * single-threaded, parareal.py); nngp_shutdown must not run while another thread is inside a
 * library call. */
int nngp_shutdown(void);

/* ---- 4. full-data GParareal (models.GPjax_p, models.py:273-473) ------------------------------
 * The training set X, Y: DEVICE [rows][d], 1 <= rows <= 46 000 (32-bit offsets inside a matrix;
 * the scratch is rows^2 doubles for D^2 plus (rows+1)^2 per point factored together, in slabs of
 * <= NNGP_GPF_SLAB_MB, default 32 GB, but at least one point; up to 7 936 rows the alpha solve
 * keeps its vector in LDS, past that in its output row).  The factor is a left-looking Cholesky
 * on 64-column panels.  K = sigma_y^2 exp(-0.5/sigma_x^2 D^2) + 10^jitter I over
 * ALL rows (kernel_np / _fit_gp_np, models.py:300-312), theta = (sigma_x, sigma_y) in linear
 * units.  Points and fits are batched: one blocked Cholesky per point.
 *
 * nngp_gpfull_lml: -LML of n_pts points (GPjax_p.log_lik, models.py:321-327; +inf when the
 * Cholesky fails).  coord, jitter_exp, theta [n_pts][2], fval_out: HOST.  alpha_out: DEVICE
 * [n_pts][rows] = L^-T L^-1 y (the posterior weights _predict uses, models.py:446-451) or NULL. */
int nngp_gpfull_lml(const double *X, int64_t rows, int d, const double *Y, int n_pts,
                    const int32_t *coord, const double *jitter_exp, const double *theta,
                    double *fval_out, double *alpha_out, void *stream);

/* nngp_gpfull_fit: n_fit Nelder-Mead fits (GPjax_p.opt_theta, models.py:329-335: scipy NM,
 * fatol/xatol, maxiter = maxfev) of -LML for (coord[f], jitter_exp[f]) from theta0[f], all fits
 * advancing together, one batched evaluation per round; replaces pool.map(_get_opt_par, ...)
 * in GPjax_p._train (models.py:376-407) and _train_coord_rnd (:352-374).  All arrays HOST
 * except X, Y.  theta_out [n_fit][2], fval_out [n_fit], nfev_out [n_fit] or NULL, rounds_out
 * (number of evaluation rounds) or NULL. */
int nngp_gpfull_fit(const double *X, int64_t rows, int d, const double *Y, int n_fit,
                    const int32_t *coord, const double *jitter_exp, const double *theta0,
                    double fatol, double xatol, int maxfev, double *theta_out, double *fval_out,
                    int32_t *nfev_out, int32_t *rounds_out, void *stream);

/* nngp_gpfull_mean: posterior means of all d coordinates at q (GPjax_p.predict -> _predict,
 * models.py:441-462): out[j] = sum_i sigma_y^2 exp(c cdist(x_i, q)) alpha[j][i] (+ bias[j]).
 * coef DEVICE [d][2] = (-0.5/sigma_x^2, sigma_y^2), alpha DEVICE [d][rows]; bias may be NULL. */
int nngp_gpfull_mean(const double *X, int64_t rows, int d, const double *q, const double *coef,
                     const double *alpha, const double *bias, double *out, void *stream);

/* ---- 5. multi-GPU: one RCCL communicator per process (one process per GPU) -------------------
 * Replaces the reference's task farm across MPI ranks (parareal.py:310-315, F over slices;
 * models.py:197-202, fits over the pool; launched as `srun ... mpi4py.futures`, Hopf.py:43-46) with
 * the two exchanges of SURVEY.md §8e.  RCCL is resolved at run time (the process's loaded
 * librccl.so.1 -- torch's -- else the system's), so the library loads without it; every call
 * below returns NNGP_E_UNSUPPORTED when it is absent.
 * nngp_comm_unique_id: rank 0 creates the id (NNGP_COMM_UID_BYTES bytes, HOST), the caller
 *   broadcasts it (e.g. torch.distributed.broadcast_object_list); nngp_comm_init: every rank, on
 *   its device (collective); nngp_comm_size: (ranks, rank) of the live communicator, (0, -1) if
 *   none, and NNGP_E_HIP once the watchdog has aborted it; nngp_comm_destroy: releases it
 *   (nngp_shutdown does too); nngp_comm_available: resolves RCCL only (NNGP_OK or
 *   NNGP_E_UNSUPPORTED) -- the every-rank check before rank 0 alone creates the id.
 * Deadline (NNGP_COMM_TIMEOUT_S, default 600 s): nngp_comm_init is RCCL's non-blocking init polled
 *   to the deadline -- a rank whose peers never arrive aborts (ncclCommAbort) and returns
 *   NNGP_E_HIP; every collective is bracketed by two events that a watchdog thread checks, and one
 *   that has not finished the deadline after its stream reached it aborts the communicator (RCCL's
 *   kernels return, the stream drains, later calls return NNGP_E_HIP).                          */
#define NNGP_COMM_UID_BYTES 128
int nngp_comm_available(void);
int nngp_comm_unique_id(void *uid_out);
int nngp_comm_init(int nranks, int rank, const void *uid);
int nngp_comm_size(int *nranks_out, int *rank_out);
int nngp_comm_destroy(void);

/* All-gather of equal [per_rank_elems] fp64 blocks in rank order, recv = [nranks][per_rank_elems]
 * (DEVICE; send may be recv + rank*per_rank_elems, in place): the ONE collective of a Parareal
 * iteration -- the fine end states of every rank's contiguous slice block (parareal.py:310-315's
 * gather), stream-ordered on `stream`.                                                          */
int nngp_allgather_states(const double *send, double *recv, size_t per_rank_elems, void *stream);

/* nngp_correction_sweep for NNGP_MODEL_NNGP with every prediction's d*n_jitter*n_restarts fits
 * sharded by coordinate over the communicator's ranks (rank r fits coordinates
 * [r*chunk, min((r+1)*chunk, d)), chunk = ceil(d/nranks)): per slice G (replicated), this rank's
 * coordinates (nngp_predict_range), one in-place all-gather of the predictions, and
 * U1[i+1] = preds + UG1[i+1] -- all on `stream`, no host synchronisation.  Bitwise the unsharded
 * sweep on every rank (same inputs, same theta0 draws).  gather: DEVICE [nranks*chunk] scratch.
 * No speculation (every rank would need the whole batch).                                       */
int nngp_correction_sweep_sharded(const nngp_system *sys, int g_tableau, int g_step_mode, int64_t g_steps,
                                  const double *t, int I, int N, double *U1, double *UG1, const double *X,
                                  const double *Y, int64_t rows, int m, int n_jitter,
                                  const double *jitter_exp_host, int n_restarts, const double *theta0,
                                  double fatol, double xatol, int maxfev, double *gather, float *g_ms_out,
                                  void *stream);

/* Test entry (one GPU): nngp_correction_sweep_sharded on a ONE-rank communicator with this process
 * playing the emulate_ranks >= 1 ranks of the coordinate split in turn (each rank's coordinates into
 * its gather block, no collective).  gather_elems: the length of gather, checked against
 * emulate_ranks * ceil(d / emulate_ranks) before any launch.                                      */
int nngp_correction_sweep_sharded_emulated(const nngp_system *sys, int g_tableau, int g_step_mode,
                                           int64_t g_steps, const double *t, int I, int N, double *U1,
                                           double *UG1, const double *X, const double *Y, int64_t rows, int m,
                                           int n_jitter, const double *jitter_exp_host, int n_restarts,
                                           const double *theta0, double fatol, double xatol, int maxfev,
                                           double *gather, size_t gather_elems, int emulate_ranks,
                                           float *g_ms_out, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* NNGP_H_ */
