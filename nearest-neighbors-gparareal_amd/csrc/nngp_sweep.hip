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
#include <mutex>
#include <vector>

#include "common.h"

namespace nngp {
// grow-only pool of timing events (G time per slice without host synchronisation in the loop)
static std::vector<hipEvent_t> g_events;
static std::mutex g_events_mu;

static int timing_events(size_t n, hipEvent_t **out) {
    std::lock_guard<std::mutex> lk(g_events_mu);
    while (g_events.size() < n) {
        hipEvent_t e;
        NNGP_HIP_CHECK(hipEventCreate(&e));
        g_events.push_back(e);
    }
    *out = g_events.data();
    return NNGP_OK;
}
}  // namespace nngp

// Speculation policy: worth it while the batch of every slice's fits is a throughput-shaped
// launch much cheaper than the latency-bound sweep it shortens (Burgers N=128: 146k fits; not
// FHN-PDE d=800 N=512: 3.7M).  NNGP_SPEC_MAX_FITS overrides the bound (0 disables).
static bool speculate_ok(int speculate, int64_t nq, int64_t n_fits) {
    if (speculate == 0 || nq < 2) return false;
    if (speculate > 0) return true;
    static int64_t bound = -1;
    if (bound < 0) {
        const char *e = getenv("NNGP_SPEC_MAX_FITS");
        bound = e ? atoll(e) : 262144;
    }
    return nq * n_fits <= bound;
}

extern "C" int nngp_correction_sweep(const nngp_system *sys, int g_tableau, int g_step_mode,
                                     int64_t g_steps, const double *t, int I, int N, double *U1,
                                     double *UG1, const double *UF, const double *UG, int model,
                                     const double *X, const double *Y, int64_t rows, int m,
                                     int n_jitter, const double *jitter_exp_host, int n_restarts,
                                     const double *theta0, double fatol, double xatol, int maxfev,
                                     double *preds_scratch, int speculate, int32_t *spec_hits_out,
                                     float *g_ms_out, void *stream) {
    using namespace nngp;
    NNGP_REQUIRE(sys != nullptr && t && U1 && UG1, "null argument");
    NNGP_REQUIRE(0 <= I && I <= N, "need 0 <= I <= N (I=%d N=%d)", I, N);
    NNGP_REQUIRE(model == NNGP_MODEL_PARAREAL || model == NNGP_MODEL_NNGP, "unknown model %d", model);
    const int d = sys->d;
    hipStream_t st = (hipStream_t)stream;
    if (model == NNGP_MODEL_PARAREAL) NNGP_REQUIRE(UF && UG, "parareal model needs UF and UG");
    if (model == NNGP_MODEL_NNGP)
        NNGP_REQUIRE(X && Y && theta0 && preds_scratch && rows >= m && m >= 1, "nngp model arguments");
    const int64_t n_fits = (int64_t)d * n_jitter * n_restarts;
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
    int32_t *spec_idx = nullptr, *flags = nullptr;
    double *spec_fits = nullptr;
    const bool spec = model == NNGP_MODEL_NNGP && UF && UG && speculate_ok(speculate, nq, n_fits);
    if (spec) {
        int err = 0;
        const size_t bytes = sizeof(double) * ((size_t)nq * d + d + (size_t)nq * n_fits * 4) +
                             sizeof(int32_t) * ((size_t)nq * m + nq);
        char *ws = (char *)workspace(bytes, &err, 2);
        if (err) return err;
        double *Qg = (double *)ws;
        double *gtmp = Qg + (size_t)nq * d;
        spec_fits = gtmp + d;
        spec_idx = (int32_t *)(spec_fits + (size_t)nq * n_fits * 4);
        flags = spec_idx + (size_t)nq * m;
        NNGP_HIP_CHECK(hipMemcpyAsync(Qg, U1 + (size_t)I * d, sizeof(double) * d, hipMemcpyDeviceToDevice, st));
        for (int64_t j = 0; j + 1 < nq && rc == NNGP_OK; j++) {
            const int i = I + (int)j;
            rc = nngp_rk_batch(sys, g_tableau, g_step_mode, 1, t + i, t + i + 1, g_steps, Qg + j * d, gtmp, stream);
            if (rc == NNGP_OK)
                rc = nngp_parareal_update(d, UF + (size_t)(i + 1) * d, UG + (size_t)(i + 1) * d, gtmp,
                                          Qg + (j + 1) * d, stream);
        }
        if (rc == NNGP_OK)
            rc = spec_batch(X, Y, rows, d, Qg, (int)nq, m, n_jitter, jitter_exp_host, n_restarts, theta0, fatol,
                            xatol, maxfev, spec_idx, spec_fits, st);
        if (rc) return rc;
    }
    for (int i = I; i < N && rc == NNGP_OK; i++) {
        const double *ui = U1 + (size_t)i * d;
        double *ug_next = UG1 + (size_t)(i + 1) * d;
        double *u_next = U1 + (size_t)(i + 1) * d;
        if (ev) NNGP_HIP_CHECK(hipEventRecord(ev[2 * (i - I)], st));
        rc = nngp_rk_batch(sys, g_tableau, g_step_mode, 1, t + i, t + i + 1, g_steps, ui, ug_next, stream);
        if (rc) break;
        if (ev) NNGP_HIP_CHECK(hipEventRecord(ev[2 * (i - I) + 1], st));
        if (model == NNGP_MODEL_PARAREAL) {   // (uF - uG_prev) + uG_new, models.py:82-83
            rc = nngp_parareal_update(d, UF + (size_t)(i + 1) * d, UG + (size_t)(i + 1) * d, ug_next,
                                      u_next, stream);
        } else {
            const size_t j = (size_t)(i - I);
            rc = predict_impl(X, Y, rows, d, ui, m, n_jitter, jitter_exp_host, n_restarts,
                              theta0 + j * n_fits * 2, fatol, xatol, maxfev, preds_scratch, ug_next, u_next,
                              nullptr, spec ? spec_idx + j * m : nullptr, spec ? spec_fits + j * n_fits * 4 : nullptr,
                              spec ? flags + j : nullptr, st);
        }
    }
    if (spec_hits_out && rc == NNGP_OK) {   // speculation hits (0 when not speculating)
        *spec_hits_out = 0;
        if (spec) {
            std::vector<int32_t> h((size_t)nq);
            NNGP_HIP_CHECK(hipMemcpyAsync(h.data(), flags, sizeof(int32_t) * nq, hipMemcpyDeviceToHost, st));
            NNGP_HIP_CHECK(hipStreamSynchronize(st));
            for (int32_t v : h) *spec_hits_out += v;
        }
    }
    if (ev && rc == NNGP_OK) {   // sum the G launches once the sweep has drained
        NNGP_HIP_CHECK(hipEventSynchronize(ev[2 * (N - I) - 1]));
        float total = 0.f;
        for (int j = 0; j < N - I; j++) {
            float ms = 0.f;
            NNGP_HIP_CHECK(hipEventElapsedTime(&ms, ev[2 * j], ev[2 * j + 1]));
            total += ms;
        }
        *g_ms_out = total;
    }
    return rc;
}
