// nngp_sweep.hip -- the sequential correction sweep of one Parareal iteration, driven natively.
//
// Reference: parareal.py:359-382 (modern) / new_lib.py:990-1012 (legacy).  For i = I .. N-1:
//     uG[i+1, :, k+1] = run_G(t[i], t[i+1], u[i, :, k+1])                 (:361-363)
//     preds           = model.predict(u[i, :, k+1], uF[i+1, :, k], uG[i+1, :, k])   (:367-368)
//     u[i+1, :, k+1]  = preds + uG[i+1, :, k+1]                            (:382)
// Slice i+1 depends on slice i, so the sweep is a chain of small launches (G: one RK launch;
// nnGP: kNN distance, kNN select, fused fits + arg-min + mean + update).  Driving that chain from
// Python costs tens of microseconds of interpreter/ctypes work per launch; here the loop issues the
// launches back to back on one stream, so the GPU never waits for the host.
#include <algorithm>
#include <atomic>
#include <mutex>
#include <vector>

#include "common.h"

namespace nngp {
// grow-only pool of timing events (G time per slice without host synchronisation in the loop)
static std::vector<hipEvent_t> g_events;
static std::mutex g_events_mu;

int timing_events(size_t n, hipEvent_t **out) {
    std::lock_guard<std::mutex> lk(g_events_mu);
    while (g_events.size() < n) {
        hipEvent_t e;
        NNGP_HIP_CHECK(hipEventCreate(&e));
        g_events.push_back(e);
    }
    *out = g_events.data();
    return NNGP_OK;
}

// nngp_shutdown: the sweep's timing events (re-created on next use)
static void events_release() {
    std::lock_guard<std::mutex> lk(g_events_mu);
    for (hipEvent_t e : g_events) (void)hipEventDestroy(e);
    g_events.clear();
}

// re-speculation resources (per process; one device per process): a side stream, the events
// that order it against the sweep's stream, and host-mapped hit flags the select kernel writes
struct Respec {
    int dev = -1;
    hipStream_t st2 = nullptr;
    hipEvent_t ev_g = nullptr, ev_r = nullptr;
    hipStream_t st3 = nullptr;      // the overlapped speculative batch
    hipEvent_t ev_pre = nullptr, ev_sel = nullptr, ev_b = nullptr;
    int32_t *herr = nullptr;        // host-mapped: a mean kernel's wait timed out
    int32_t *hflags = nullptr;   // host-mapped, fine-grained
    size_t nflags = 0;
};
static Respec g_respec;
static std::mutex g_respec_mu;

static int respec_resources(size_t nflags, Respec **out) {
    std::lock_guard<std::mutex> lk(g_respec_mu);
    Respec &r = g_respec;
    int dev = 0;
    NNGP_HIP_CHECK(hipGetDevice(&dev));
    if (r.dev != dev) {   // first use (or another device): fresh stream / events / flags
        if (r.st2) (void)hipStreamDestroy(r.st2);
        if (r.ev_g) (void)hipEventDestroy(r.ev_g);
        if (r.ev_r) (void)hipEventDestroy(r.ev_r);
        if (r.st3) (void)hipStreamDestroy(r.st3);
        for (hipEvent_t e : {r.ev_pre, r.ev_sel, r.ev_b})
            if (e) (void)hipEventDestroy(e);
        if (r.herr) (void)hipHostFree(r.herr);
        if (r.hflags) (void)hipHostFree(r.hflags);
        r = Respec{};
        NNGP_HIP_CHECK(hipStreamCreateWithFlags(&r.st2, hipStreamNonBlocking));
        NNGP_HIP_CHECK(hipEventCreateWithFlags(&r.ev_g, hipEventDisableTiming));
        NNGP_HIP_CHECK(hipEventCreateWithFlags(&r.ev_r, hipEventDisableTiming));
        NNGP_HIP_CHECK(hipStreamCreateWithFlags(&r.st3, hipStreamNonBlocking));
        NNGP_HIP_CHECK(hipEventCreateWithFlags(&r.ev_pre, hipEventDisableTiming));
        NNGP_HIP_CHECK(hipEventCreateWithFlags(&r.ev_sel, hipEventDisableTiming));
        NNGP_HIP_CHECK(hipEventCreateWithFlags(&r.ev_b, hipEventDisableTiming));
        NNGP_HIP_CHECK(hipHostMalloc((void **)&r.herr, 64, hipHostMallocMapped | hipHostMallocCoherent));
        r.dev = dev;
    }
    if (r.nflags < nflags) {
        if (r.hflags) (void)hipHostFree(r.hflags);
        r.hflags = nullptr;
        r.nflags = 0;
        NNGP_HIP_CHECK(hipHostMalloc((void **)&r.hflags, sizeof(int32_t) * nflags,
                                     hipHostMallocMapped | hipHostMallocCoherent));
        r.nflags = nflags;
    }
    *out = &r;
    return NNGP_OK;
}

// G beside the prediction (g_side_supported): a side stream and its two ordering events
struct GSide {
    int dev = -1;
    hipStream_t st = nullptr;
    hipEvent_t ev_u = nullptr, ev_g = nullptr;   // U1[i] ready (sweep stream) / G(U1[i]) done (side)
};
static GSide g_gside;

static int gside_resources(GSide **out) {
    std::lock_guard<std::mutex> lk(g_respec_mu);
    int dev = 0;
    NNGP_HIP_CHECK(hipGetDevice(&dev));
    if (g_gside.dev != dev) {
        if (g_gside.st) (void)hipStreamDestroy(g_gside.st);
        for (hipEvent_t e : {g_gside.ev_u, g_gside.ev_g})
            if (e) (void)hipEventDestroy(e);
        g_gside = GSide{};
        NNGP_HIP_CHECK(hipStreamCreateWithFlags(&g_gside.st, hipStreamNonBlocking));
        NNGP_HIP_CHECK(hipEventCreateWithFlags(&g_gside.ev_u, hipEventDisableTiming));
        NNGP_HIP_CHECK(hipEventCreateWithFlags(&g_gside.ev_g, hipEventDisableTiming));
        g_gside.dev = dev;
    }
    *out = &g_gside;
    return NNGP_OK;
}

// nngp_shutdown: the side streams, events and host-mapped flags (re-created on next use)
void sweep_release() {
    events_release();
    std::lock_guard<std::mutex> lk(g_respec_mu);
    Respec &r = g_respec;
    if (r.st2) (void)hipStreamDestroy(r.st2);
    if (r.st3) (void)hipStreamDestroy(r.st3);
    for (hipEvent_t e : {r.ev_g, r.ev_r, r.ev_pre, r.ev_sel, r.ev_b})
        if (e) (void)hipEventDestroy(e);
    if (r.herr) (void)hipHostFree(r.herr);
    if (r.hflags) (void)hipHostFree(r.hflags);
    r = Respec{};
    if (g_gside.st) (void)hipStreamDestroy(g_gside.st);
    for (hipEvent_t e : {g_gside.ev_u, g_gside.ev_g})
        if (e) (void)hipEventDestroy(e);
    g_gside = GSide{};
}

// wait for the select kernel's host-mapped hit flag (-1 = not yet written); a stream that has
// drained (or failed) without writing it is an error, never a hang
static int wait_flag(const int32_t *flag, hipStream_t st, int32_t *out) {
    for (uint64_t spin = 1;; spin++) {
        const int32_t v = __atomic_load_n(flag, __ATOMIC_ACQUIRE);
        if (v >= 0) {
            *out = v;
            return NNGP_OK;
        }
        if ((spin & 1023) == 0) {
            const hipError_t q = hipStreamQuery(st);
            if (q == hipSuccess && __atomic_load_n(flag, __ATOMIC_ACQUIRE) < 0) {
                set_error("correction sweep: speculation flag was not written");
                return NNGP_E_HIP;
            }
            if (q != hipSuccess && q != hipErrorNotReady) {
                set_error("correction sweep: %s", hipGetErrorString(q));
                return NNGP_E_HIP;
            }
        }
    }
}

// slices re-speculated after a miss (NNGP_RESPEC_W; 0 disables)
static int respec_window() {
    return std::max(0, env_int("NNGP_RESPEC_W", 4));
}

}  // namespace nngp

// Speculation policy: worth it while the batch of every slice's fits is a throughput-shaped
// launch much cheaper than the latency-bound sweep it shortens (Burgers N=128: 146k fits; not
// FHN-PDE d=800 N=512: 3.7M).  NNGP_SPEC_MAX_FITS overrides the bound (0 disables).
// sweeps rerun with the batch serialised because a hit's wait timed out (nngp_sweep_late_reruns)
static std::atomic<int64_t> g_late_reruns{0};

static bool speculate_ok(int speculate, int64_t nq, int64_t n_fits) {
    if (speculate == 0 || nq < 2) return false;
    if (speculate > 0) return true;
    const char *e = getenv("NNGP_SPEC_MAX_FITS");
    const int64_t bound = e ? atoll(e) : 262144;
    return nq * n_fits <= bound;
}

static int correction_sweep(const nngp_system *sys, int g_tableau, int g_step_mode, int64_t g_steps,
                            const double *t, int I, int N, double *U1, double *UG1, const double *UF,
                            const double *UG, int model, const double *X, const double *Y, int64_t rows, int m,
                            int n_jitter, const double *jitter_exp_host, int n_restarts, const double *theta0,
                            double fatol, double xatol, int maxfev, double *preds_scratch, int speculate,
                            int32_t *spec_hits_out, float *g_ms_out, void *stream, bool allow_overlap,
                            bool allow_chain, int *late) {
    using namespace nngp;
    *late = 0;
    NNGP_REQUIRE(sys != nullptr && t && U1 && UG1, "null argument");
    NNGP_REQUIRE(0 <= I && I <= N, "need 0 <= I <= N (I=%d N=%d)", I, N);
    NNGP_REQUIRE(model == NNGP_MODEL_PARAREAL || model == NNGP_MODEL_NNGP || model == NNGP_MODEL_GPFULL,
                 "unknown model %d", model);
    const int d = sys->d;
    hipStream_t st = (hipStream_t)stream;
    if (model == NNGP_MODEL_PARAREAL) NNGP_REQUIRE(UF && UG, "parareal model needs UF and UG");
    if (model == NNGP_MODEL_NNGP)
        NNGP_REQUIRE(X && Y && theta0 && preds_scratch && rows >= m && m >= 1, "nngp model arguments");
    if (model == NNGP_MODEL_GPFULL)
        NNGP_REQUIRE(X && Y && theta0 && rows >= 1, "full-GP model arguments (X, alpha, coefficients)");
    const int64_t n_fits = (int64_t)d * n_jitter * n_restarts;
    // G time (g_ms_out): event pairs around the G launch of every g_every-th slice, scaled to all of
    // them (NNGP_G_TIME_EVERY, default 8; 1 = every slice).  Each event record costs the host ~3 us
    // on a chain whose hit slices are host-bound (profiles/r05/sweep/).
    const int g_every = std::max(1, env_int("NNGP_G_TIME_EVERY", 8));
    const bool gdist_ok = gdist_supported(sys, g_step_mode);
    GSide *gs = nullptr;
    if (model == NNGP_MODEL_NNGP && g_side_supported(sys, g_step_mode)) {
        const int rc0 = gside_resources(&gs);
        if (rc0) return rc0;
    }
    int64_t hit_codes[5] = {0, 0, 0, 0, 0};   // host-flag codes seen (NNGP_SWEEP_STATS=1 prints them)
    const bool ahead_on = env_int("NNGP_SWEEP_AHEAD", 1) != 0;
    hipEvent_t *ev = nullptr;
    if (g_ms_out) {
        *g_ms_out = 0.f;
        if (N > I) {
            const int rc0 = timing_events(2 * (size_t)(N - I), &ev);
            if (rc0) return rc0;
        }
    }
    int rc = NNGP_OK;
    // ---- speculation (nnGP): guess every slice's query by the classic Parareal update along the
    // coarse chain, g[I] = U1[I], g[i+1] = G(g[i]) + (UF[i+1] - UG[i+1]) (models.py:82-83), and
    // run all of their fits as one batch; the sweep below then only recomputes the slices whose
    // actual ordered neighbour list differs from the guessed one.
    const int64_t nq = N - I;
    int32_t *spec_idx = nullptr, *flags = nullptr, *spec2_idx = nullptr;
    double *spec_fits = nullptr, *spec2_fits = nullptr, *Qr = nullptr, *gtmp = nullptr;
    const bool spec = model == NNGP_MODEL_NNGP && UF && UG && speculate_ok(speculate, nq, n_fits);
    // ---- re-speculation: the chain guesses drift; when slice i misses, the next W slices are
    // guessed again by the same update along the coarse chain, restarted from the actual U1[i]
    // (its G(U1[i]) is the sweep's own UG1[i+1]), and their fits run as one launch on a side
    // stream while slice i's own fits run.  Their lists/fits form a second candidate set (hit = 2).
    const int W = spec ? (int)std::min<int64_t>(respec_window(), nq - 1) : 0;
    Respec *rs = nullptr;
    if (spec) {
        const int rc0 = respec_resources((size_t)nq, &rs);
        if (rc0) return rc0;
    }
    // overlapped batch (NNGP_SPEC_OVERLAP, default 1; launch chain only): the batch's fits run on a
    // side stream while the sweep starts as soon as the batch's neighbour lists exist; a hit slice's
    // mean waits for that slice's fits only (per-prediction completion counters)
    const bool chained = spec && allow_chain && chain_supported(sys, g_step_mode, m);
    const bool overlap = spec && !chained && allow_overlap && env_int("NNGP_SPEC_OVERLAP", 1) != 0;
    int32_t *done = nullptr;
    // hit means finished in the select (NNGP_HIT_MEAN, default 1; launch chain with host flags only):
    // every prediction of the batch (AP1) and of each re-speculation window (AP2) prepared by
    // gp_pre_kernel after its fits, pre1 / pre2 counting the prepared workgroups per slice
    const bool hitmean = spec && !chained && W > 0 && env_int("NNGP_HIT_MEAN", 1) != 0;
    const size_t hst = hitmean ? (size_t)d * HM_STRIDE(pre_maxm(m)) : 0;   // doubles per slice
    double *AP1 = nullptr, *AP2 = nullptr;
    int32_t *pre1 = nullptr, *pre2 = nullptr;
    if (spec) {
        int err = 0;
        const size_t bytes = sizeof(double) * ((size_t)nq * d + d + (size_t)nq * n_fits * 4) +
                             sizeof(int32_t) * ((size_t)nq * m + nq + nq) +
                             (W > 0 ? sizeof(double) * ((size_t)W * d + d + (size_t)nq * n_fits * 4) +
                                          sizeof(int32_t) * (size_t)nq * m
                                    : 0) +
                             (hitmean ? sizeof(double) * (2 * (size_t)nq * hst + 1) + sizeof(int32_t) * 2 * (size_t)nq
                                      : 0);
        char *ws = (char *)workspace(bytes, &err, 2);
        if (err) return err;
        double *Qg = (double *)ws;
        gtmp = Qg + (size_t)nq * d;
        spec_fits = gtmp + d;
        double *tail = spec_fits + (size_t)nq * n_fits * 4;
        if (W > 0) {
            Qr = tail;
            spec2_fits = Qr + (size_t)W * d + d;   // Qr[W][d] | gtmp2[d] | fits
            tail = spec2_fits + (size_t)nq * n_fits * 4;
        }
        spec_idx = (int32_t *)tail;
        flags = spec_idx + (size_t)nq * m;
        done = flags + nq;   // [nq] (then spec2_idx)
        if (W > 0) {
            spec2_idx = done + nq;
            NNGP_HIP_CHECK(hipMemsetAsync(spec2_idx, 0xFF, sizeof(int32_t) * (size_t)nq * m, st));   // -1: none
            for (int64_t j = 0; j < nq; j++) rs->hflags[j] = -1;
        }
        if (hitmean) {   // after the int32 arrays, 8-byte aligned
            const size_t off = ((size_t)((char *)(done + nq + (size_t)nq * m) - ws) + 7) & ~(size_t)7;
            AP1 = (double *)(ws + off);
            AP2 = AP1 + (size_t)nq * hst;
            pre1 = (int32_t *)(AP2 + (size_t)nq * hst);
            pre2 = pre1 + nq;
            NNGP_HIP_CHECK(hipMemsetAsync(pre1, 0, sizeof(int32_t) * 2 * (size_t)nq, st));
        }
        NNGP_HIP_CHECK(hipMemcpyAsync(Qg, U1 + (size_t)I * d, sizeof(double) * d, hipMemcpyDeviceToDevice, st));
        if (guess_chain_supported(sys, g_step_mode))   // one launch for the whole chain (bitwise)
            rc = guess_chain(sys, g_tableau, g_step_mode, g_steps, t, I, (int)nq, UF, UG, Qg, gtmp, st);
        else
        for (int64_t j = 0; j + 1 < nq && rc == NNGP_OK; j++) {
            const int i = I + (int)j;
            rc = nngp_rk_batch(sys, g_tableau, g_step_mode, 1, t + i, t + i + 1, g_steps, Qg + j * d, gtmp, stream);
            if (rc == NNGP_OK)
                rc = nngp_parareal_update(d, UF + (size_t)(i + 1) * d, UG + (size_t)(i + 1) * d, gtmp,
                                          Qg + (j + 1) * d, stream);
        }
        if (rc == NNGP_OK && overlap) {
            *rs->herr = 0;
            NNGP_HIP_CHECK(hipEventRecord(rs->ev_pre, st));             // the guesses Qg
            NNGP_HIP_CHECK(hipStreamWaitEvent(rs->st3, rs->ev_pre, 0));
            rc = spec_batch(X, Y, rows, d, Qg, (int)nq, m, n_jitter, jitter_exp_host, n_restarts, theta0, fatol,
                            xatol, maxfev, spec_idx, spec_fits, false, rs->st3, 1, done, rs->ev_sel, AP1, pre1);
            if (rc == NNGP_OK) {
                NNGP_HIP_CHECK(hipEventRecord(rs->ev_b, rs->st3));
                NNGP_HIP_CHECK(hipStreamWaitEvent(st, rs->ev_sel, 0));   // lists ready; fits may run on
            }
        } else if (rc == NNGP_OK) {
            rc = spec_batch(X, Y, rows, d, Qg, (int)nq, m, n_jitter, jitter_exp_host, n_restarts, theta0, fatol,
                            xatol, maxfev, spec_idx, spec_fits, false, st, 1, nullptr, nullptr, AP1, pre1);
        }
        if (rc) return rc;
    }
    bool respec_pending = false;
    // ---- the fused chain (nngp_gp.hip chain_kernel): runs of hit slices as one persistent kernel;
    // the host takes over at each miss (that slice's fits, the re-speculation), then resumes it
    if (chained) {
        float g_ms = 0.f;
        int i = I;
        while (i < N && rc == NNGP_OK) {
            if (respec_pending) NNGP_HIP_CHECK(hipStreamWaitEvent(st, rs->ev_r, 0));   // lists/fits ready
            respec_pending = false;
            int s = N;
            rc = chain_sweep(sys, g_tableau, g_step_mode, g_steps, t, I, N, i, U1, UG1, X, Y, rows, m, n_jitter,
                             jitter_exp_host, n_restarts, flags, spec_idx, spec_fits, W > 0 ? spec2_idx : nullptr,
                             W > 0 ? spec2_fits : nullptr, preds_scratch, &s, &g_ms, st);
            if (rc && s == -2) *late = 1;   // a grid barrier timed out: rerun on the launch chain
            if (rc || s >= N) break;
            // miss at slice s: G(U1[s]) and its select are done (the chain kernel has drained)
            const size_t j = (size_t)(s - I);
            double *ug_next = UG1 + (size_t)(s + 1) * d;
            rc = chain_miss_fits(rows, d, m, n_jitter, jitter_exp_host, n_restarts, theta0 + j * n_fits * 2, fatol,
                                 xatol, maxfev, preds_scratch, ug_next, U1 + (size_t)(s + 1) * d, st);
            if (rc == NNGP_OK && W > 0 && s + 1 < N) {   // re-guess slices s+1 .. s+w from U1[s]
                const int w = (int)std::min<int64_t>(W, N - 1 - s);
                hipStream_t s2 = rs->st2;
                double *g2 = Qr + (size_t)W * d;
                rc = nngp_parareal_update(d, UF + (size_t)(s + 1) * d, UG + (size_t)(s + 1) * d, ug_next, Qr, s2);
                for (int q = 1; q < w && rc == NNGP_OK; q++) {
                    const int sq = s + q;
                    rc = nngp_rk_batch(sys, g_tableau, g_step_mode, 1, t + sq, t + sq + 1, g_steps,
                                       Qr + (size_t)(q - 1) * d, g2, s2);
                    if (rc == NNGP_OK)
                        rc = nngp_parareal_update(d, UF + (size_t)(sq + 1) * d, UG + (size_t)(sq + 1) * d, g2,
                                                  Qr + (size_t)q * d, s2);
                }
                if (rc == NNGP_OK)
                    rc = spec_batch(X, Y, rows, d, Qr, w, m, n_jitter, jitter_exp_host, n_restarts,
                                    theta0 + (j + 1) * n_fits * 2, fatol, xatol, maxfev, spec2_idx + (j + 1) * m,
                                    spec2_fits + (j + 1) * n_fits * 4, true, s2, 6);
                if (rc == NNGP_OK) {
                    NNGP_HIP_CHECK(hipEventRecord(rs->ev_r, s2));
                    respec_pending = true;
                }
            }
            i = s + 1;
        }
        if (g_ms_out && rc == NNGP_OK) *g_ms_out = g_ms;
        ev = nullptr;   // G time comes from the chain's clock
    }
    // ---- the launch chain
    auto split_at = [&](int i) { return spec && W > 0 && i + 1 < N; };
    // with a host flag (W > 0, not the last slice) the prediction is issued in two parts: the kNN +
    // select, then -- once the host has read the select's hit code -- the mean alone on a hit (the
    // fits are the batch's) or the fits and the mean on a miss.  The fits launch a hit would have
    // skipped on the device is never issued: its waves (191 VGPRs) could only be dispatched once the
    // overlapped batch's waves drained a SIMD.  With HitMean the select finishes a hit's mean itself
    // once the prediction is prepared (host code 3 / 4), and no mean launch follows.
    auto predict_at = [&](int i, int phase, bool host_flag, hipEvent_t bias_ready = nullptr) {
        const size_t j = (size_t)(i - I);
        HitMean hm{};
        if (hitmean && host_flag && split_at(i))
            hm = HitMean{AP1 + j * hst, AP2 + j * hst, pre1 + j, pre2 + j, pre_target(d, m), pre_maxm(m),
                         UG1 + (size_t)(i + 1) * d, U1 + (size_t)(i + 1) * d, preds_scratch};
        return predict_impl(X, Y, rows, d, U1 + (size_t)i * d, m, n_jitter, jitter_exp_host, n_restarts,
                            theta0 + j * n_fits * 2, fatol, xatol, maxfev, preds_scratch, UG1 + (size_t)(i + 1) * d,
                            U1 + (size_t)(i + 1) * d, nullptr, spec ? spec_idx + j * m : nullptr,
                            spec ? spec_fits + j * n_fits * 4 : nullptr, spec ? flags + j : nullptr,
                            W > 0 ? spec2_idx + j * m : nullptr, W > 0 ? spec2_fits + j * n_fits * 4 : nullptr,
                            (host_flag && split_at(i)) ? rs->hflags + j : nullptr, st, 0, -1,   // every written
                            overlap ? done + j : nullptr, overlap ? rs->herr : nullptr, phase,  // flag is awaited
                            hm.out ? &hm : nullptr, bias_ready);
    };
    // slice i's head: G(U1[i]) (with the kNN distances as one launch, gdist, on the untimed split
    // slices), the re-speculation window's lists, and the select (or the whole prediction)
    auto head = [&](int i) -> int {
        const size_t j = (size_t)(i - I);
        const double *ui = U1 + (size_t)i * d;
        double *ug_next = UG1 + (size_t)(i + 1) * d;
        double *u_next = U1 + (size_t)(i + 1) * d;
        const bool timed = ev && j % (size_t)g_every == 0;
        const bool fused = model == NNGP_MODEL_NNGP && split_at(i) && gdist_ok && !timed;
        // an unsplit prediction's G on the side stream: only the mean needs G(U1[i]) (its bias)
        const bool side = model == NNGP_MODEL_NNGP && !split_at(i) && gs && !timed;
        if (fused) {
            const int r = gdist(sys, g_tableau, g_step_mode, g_steps, t, i, X, rows, d, m, n_jitter, n_restarts, ui,
                                ug_next, st);
            if (r) return r;
        } else if (side) {
            NNGP_HIP_CHECK(hipEventRecord(gs->ev_u, st));   // U1[i] (the previous slice's mean)
            NNGP_HIP_CHECK(hipStreamWaitEvent(gs->st, gs->ev_u, 0));
            const int r = nngp_rk_batch(sys, g_tableau, g_step_mode, 1, t + i, t + i + 1, g_steps, ui, ug_next, gs->st);
            if (r) return r;
            NNGP_HIP_CHECK(hipEventRecord(gs->ev_g, gs->st));
        } else {
            if (timed) NNGP_HIP_CHECK(hipEventRecord(ev[2 * j], st));
            const int r = nngp_rk_batch(sys, g_tableau, g_step_mode, 1, t + i, t + i + 1, g_steps, ui, ug_next, stream);
            if (r) return r;
            if (timed) NNGP_HIP_CHECK(hipEventRecord(ev[2 * j + 1], st));
        }
        if (model == NNGP_MODEL_PARAREAL)   // (uF - uG_prev) + uG_new, models.py:82-83
            return nngp_parareal_update(d, UF + (size_t)(i + 1) * d, UG + (size_t)(i + 1) * d, ug_next, u_next, stream);
        if (model == NNGP_MODEL_GPFULL)     // GPjax_p.predict + uG (models.py:456-462)
            return gpfull_mean(X, rows, d, ui, theta0, Y, ug_next, u_next, st);
        if (W > 0) {
            if (respec_pending) NNGP_HIP_CHECK(hipStreamWaitEvent(st, rs->ev_r, 0));   // lists/fits ready
            respec_pending = false;
        }
        return predict_at(i, split_at(i) ? (fused ? PREDICT_SELECT_ONLY : PREDICT_SELECT) : PREDICT_ALL, true,
                          side ? gs->ev_g : nullptr);
    };
    // Look-ahead (HitMean only): once the batch's predictions are all prepared, a hit finishes in its
    // select, so slice i+1's head is queued behind slice i's select before the host reads slice i's
    // code.  On a miss or a hit that still needs the mean kernel, the early head read a U1[i+1] that
    // was not written yet: the host waits for its select's host flag, resets it, redoes slice i's
    // distances and select (the workspace the fits / mean read), and slice i+1's head follows later --
    // every value the early launches wrote is written again.  (Before the batch is prepared, queueing
    // slice i's mean kernel first and the head behind it measured no gain: those slices wait on the
    // batch's fits, profiles/r05/sweep/host_path_ab.txt.)
    bool pre_ready = !overlap;   // serialised batch: prepared before the sweep
    bool issued = false;         // slice i's head was queued by slice i-1's look-ahead
    for (int i = chained ? N : I; i < N && rc == NNGP_OK; i++) {
        const size_t j = (size_t)(i - I);
        if (!issued) rc = head(i);
        issued = false;
        if (rc) break;
        if (model != NNGP_MODEL_NNGP || !split_at(i)) continue;
        if (hitmean && !pre_ready) pre_ready = hipEventQuery(rs->ev_b) == hipSuccess;
        const bool ahead = ahead_on && hitmean && pre_ready && split_at(i + 1);
        if (ahead && (rc = head(i + 1)) != NNGP_OK) break;
        int32_t hit = 0;
        rc = wait_flag(rs->hflags + j, st, &hit);
        // a mean that gave up waiting for the overlapped batch: stop issuing, the caller reruns
        if (rc == NNGP_OK && overlap && __atomic_load_n(rs->herr, __ATOMIC_ACQUIRE) != 0) break;
        if (rc) break;
        // a miss's re-speculation window starts from G(U1[i]): the event is recorded only on a miss,
        // behind the select the host has just seen finish (so behind G), before the slice's fits
        if (hit == 0) NNGP_HIP_CHECK(hipEventRecord(rs->ev_g, st));
        hit_codes[std::min(hit, 4)]++;
        if (hit >= 3) {   // the select finished the mean (HitMean)
            issued = ahead;
            continue;
        }
        if (ahead) {   // undo the look-ahead (above)
            int32_t early = 0;
            if ((rc = wait_flag(rs->hflags + j + 1, st, &early)) != NNGP_OK) break;
            __atomic_store_n(rs->hflags + j + 1, -1, __ATOMIC_RELEASE);
            if ((rc = predict_at(i, PREDICT_SELECT, false)) != NNGP_OK) break;
        }
        rc = predict_at(i, hit != 0 ? PREDICT_MEAN : PREDICT_FITS_MEAN, true);
        if (rc || hit != 0) continue;
        // miss: re-guess slices i+1 .. i+w from the actual U1[i] on the side stream
        double *ug_next = UG1 + (size_t)(i + 1) * d;
        const int w = (int)std::min<int64_t>(W, N - 1 - i);
        hipStream_t s2 = rs->st2;
        double *g2 = Qr + (size_t)W * d;
        NNGP_HIP_CHECK(hipStreamWaitEvent(s2, rs->ev_g, 0));
        rc = nngp_parareal_update(d, UF + (size_t)(i + 1) * d, UG + (size_t)(i + 1) * d, ug_next, Qr, s2);
        for (int q = 1; q < w && rc == NNGP_OK; q++) {
            const int s = i + q;
            rc = nngp_rk_batch(sys, g_tableau, g_step_mode, 1, t + s, t + s + 1, g_steps, Qr + (size_t)(q - 1) * d, g2,
                               s2);
            if (rc == NNGP_OK)
                rc = nngp_parareal_update(d, UF + (size_t)(s + 1) * d, UG + (size_t)(s + 1) * d, g2,
                                          Qr + (size_t)q * d, s2);
        }
        if (rc == NNGP_OK)   // a wave per fit: the sweep waits on this window's fits
            rc = spec_batch(X, Y, rows, d, Qr, w, m, n_jitter, jitter_exp_host, n_restarts,
                            theta0 + (j + 1) * n_fits * 2, fatol, xatol, maxfev, spec2_idx + (j + 1) * m,
                            spec2_fits + (j + 1) * n_fits * 4, true, s2, 6, nullptr, nullptr,
                            hitmean ? AP2 + (j + 1) * hst : nullptr, hitmean ? pre2 + j + 1 : nullptr);
        if (rc == NNGP_OK) {
            NNGP_HIP_CHECK(hipEventRecord(rs->ev_r, s2));
            respec_pending = true;
        }
    }
    // the side streams never outlive the sweep (also on an error path: their buffers are reused)
    if (respec_pending) NNGP_HIP_CHECK(hipStreamWaitEvent(st, rs->ev_r, 0));
    if (overlap) {
        NNGP_HIP_CHECK(hipStreamWaitEvent(st, rs->ev_b, 0));
        NNGP_HIP_CHECK(hipStreamSynchronize(st));
        if (rc == NNGP_OK && __atomic_load_n(rs->herr, __ATOMIC_ACQUIRE) != 0) {
            // a hit slice's mean gave up waiting for the batch's fits (bounded spin; e.g. a GPU
            // shared by several ranks) and wrote nothing: the caller redoes the sweep serially
            set_error("correction sweep: a speculative fit count was not reached in time");
            *late = 1;
            rc = NNGP_E_HIP;
        }
    }
    if (spec_hits_out && rc == NNGP_OK) {   // speculation hits (0 when not speculating)
        *spec_hits_out = 0;
        if (spec) {
            std::vector<int32_t> h((size_t)nq);
            NNGP_HIP_CHECK(hipMemcpyAsync(h.data(), flags, sizeof(int32_t) * nq, hipMemcpyDeviceToHost, st));
            NNGP_HIP_CHECK(hipStreamSynchronize(st));
            for (int32_t v : h) *spec_hits_out += v != 0;
        }
    }
    sel_prof_report("sweep");
    if (env_int("NNGP_SWEEP_STATS", 0))
        fprintf(stderr, "sweep I=%d N=%d: miss %lld, hit (mean kernel) %lld / %lld, hit (mean in select) %lld / %lld\n",
                I, N, (long long)hit_codes[0], (long long)hit_codes[1], (long long)hit_codes[2],
                (long long)hit_codes[3], (long long)hit_codes[4]);
    if (ev && rc == NNGP_OK) {   // the G launches' time once the sweep has drained
        const int ns = (N - I - 1) / g_every + 1;   // timed slices j = 0, g_every, 2 g_every, ...
        NNGP_HIP_CHECK(hipEventSynchronize(ev[2 * (size_t)(ns - 1) * g_every + 1]));
        float total = 0.f;
        for (int k = 0; k < ns; k++) {
            const size_t j = (size_t)k * g_every;
            float ms = 0.f;
            NNGP_HIP_CHECK(hipEventElapsedTime(&ms, ev[2 * j], ev[2 * j + 1]));
            total += ms;
        }
        *g_ms_out = total * (float)(N - I) / (float)ns;   // every G launch of a sweep is the same work
    }
    return rc;
}

extern "C" int nngp_correction_sweep(const nngp_system *sys, int g_tableau, int g_step_mode,
                                     int64_t g_steps, const double *t, int I, int N, double *U1,
                                     double *UG1, const double *UF, const double *UG, int model,
                                     const double *X, const double *Y, int64_t rows, int m,
                                     int n_jitter, const double *jitter_exp_host, int n_restarts,
                                     const double *theta0, double fatol, double xatol, int maxfev,
                                     double *preds_scratch, int speculate, int32_t *spec_hits_out,
                                     float *g_ms_out, void *stream) {
    // The sweep writes UG1[i+1] and U1[i+1] for i >= I only and reads none of them before writing,
    // so a sweep whose overlapped batch fell behind, or whose fused chain's grid barrier timed out
    // (see correction_sweep), is simply run again with the batch serialised on the launch chain:
    // the same bits, later.
    int late = 0;
    int rc = correction_sweep(sys, g_tableau, g_step_mode, g_steps, t, I, N, U1, UG1, UF, UG, model, X, Y, rows, m,
                              n_jitter, jitter_exp_host, n_restarts, theta0, fatol, xatol, maxfev, preds_scratch,
                              speculate, spec_hits_out, g_ms_out, stream, true, true, &late);
    if (rc != NNGP_OK && late) {
        g_late_reruns.fetch_add(1);
        rc = correction_sweep(sys, g_tableau, g_step_mode, g_steps, t, I, N, U1, UG1, UF, UG, model, X, Y, rows, m,
                              n_jitter, jitter_exp_host, n_restarts, theta0, fatol, xatol, maxfev, preds_scratch,
                              speculate, spec_hits_out, g_ms_out, stream, false, false, &late);
    }
    return rc;
}

extern "C" int64_t nngp_sweep_late_reruns(void) { return g_late_reruns.load(); }
