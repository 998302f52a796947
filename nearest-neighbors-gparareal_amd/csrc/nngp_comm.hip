// nngp_comm.hip -- the multi-GPU exchange behind the C-ABI: one RCCL communicator per process (one
// process per GPU), the fine sweep's all-gather of end states, and the coordinate-sharded
// correction sweep issued natively.
//
// Reference: the task farm of parareal.py:310-315 (F fanned over MPI ranks, results gathered by
// pool.map) and models.py:185-226 (the d*9*R fits of one prediction fanned over the pool).  Here
// (SURVEY.md §8e): every rank integrates a contiguous block of the unconverged slices and ONE
// all-gather per iteration assembles U_F; a prediction with many fits (FHN-PDE d = 800: 7 200) is
// sharded by coordinate, each rank fitting its block, and one all-gather of the d predictions per
// slice assembles u = preds + uG.  The sequential sweep is replicated: G, the kNN and the RNG
// draws are identical on every rank, so ranks stay bit-identical without a broadcast.
//
// RCCL is resolved at run time: the process's own copy when one is loaded (torch's bundled
// librccl.so.1, soname-matched, so torch.distributed and this library share one RCCL), else the
// system's.  The library therefore does not link RCCL and loads without it.
#include <dlfcn.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

#include <rccl/rccl.h>

#include "common.h"

namespace nngp {

struct RcclApi {
    void *handle = nullptr;
    ncclResult_t (*get_unique_id)(ncclUniqueId *) = nullptr;
    ncclResult_t (*comm_init_rank_config)(ncclComm_t *, int, ncclUniqueId, int, ncclConfig_t *) = nullptr;
    ncclResult_t (*all_gather)(const void *, void *, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*comm_abort)(ncclComm_t) = nullptr;
    ncclResult_t (*get_async_error)(ncclComm_t, ncclResult_t *) = nullptr;
    const char *(*error_string)(ncclResult_t) = nullptr;
};

static RcclApi g_rccl;
static ncclComm_t g_comm = nullptr;
static int g_comm_ranks = 0, g_comm_rank = -1, g_comm_dev = -1;
static bool g_comm_aborted = false;   // the watchdog aborted the communicator (a collective timed out)
static std::mutex g_comm_mu;

static int rccl_api(RcclApi **out) {
    if (!g_rccl.handle) {
        void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);   // already in the process (torch)
        if (!h) h = dlopen("librccl.so.1", RTLD_NOW);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW);
        if (!h) {
            set_error("RCCL not found (librccl.so.1): %s", dlerror());
            return NNGP_E_UNSUPPORTED;
        }
        RcclApi a;
        a.handle = h;
        a.get_unique_id = (decltype(a.get_unique_id))dlsym(h, "ncclGetUniqueId");
        a.comm_init_rank_config = (decltype(a.comm_init_rank_config))dlsym(h, "ncclCommInitRankConfig");
        a.all_gather = (decltype(a.all_gather))dlsym(h, "ncclAllGather");
        a.comm_destroy = (decltype(a.comm_destroy))dlsym(h, "ncclCommDestroy");
        a.comm_abort = (decltype(a.comm_abort))dlsym(h, "ncclCommAbort");
        a.get_async_error = (decltype(a.get_async_error))dlsym(h, "ncclCommGetAsyncError");
        a.error_string = (decltype(a.error_string))dlsym(h, "ncclGetErrorString");
        if (!a.get_unique_id || !a.comm_init_rank_config || !a.all_gather || !a.comm_destroy || !a.comm_abort ||
            !a.get_async_error || !a.error_string) {
            set_error("RCCL library lacks an entry point (the communicator needs ncclCommInitRankConfig, "
                      "ncclCommGetAsyncError and ncclCommAbort for its deadline)");
            return NNGP_E_UNSUPPORTED;
        }
        g_rccl = a;
    }
    *out = &g_rccl;
    return NNGP_OK;
}

#define NNGP_RCCL_CHECK(api, expr)                                                               \
    do {                                                                                         \
        ncclResult_t _r = (expr);                                                                \
        if (_r != ncclSuccess) {                                                                 \
            ::nngp::set_error("%s failed: %s (%s:%d)", #expr, (api)->error_string(_r), __FILE__, \
                              __LINE__);                                                         \
            return NNGP_E_HIP;                                                                   \
        }                                                                                        \
    } while (0)

// The communicator's deadline (NNGP_COMM_TIMEOUT_S, default 600 s): how long nngp_comm_init waits
// for the other ranks, and how long one collective may run once the stream has reached it.  A
// missing or failed peer then ends in ncclCommAbort and NNGP_E_HIP instead of a hang.
static double comm_timeout_s() {
    const char *e = getenv("NNGP_COMM_TIMEOUT_S");
    const double v = e ? atof(e) : 600.0;
    return v > 0 ? v : 600.0;
}

static double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// A non-blocking communicator's pending host-side operation (init, or an enqueue that returned
// ncclInProgress): poll ncclCommGetAsyncError until it leaves ncclInProgress or the deadline passes
// (returns ncclInProgress then).
static ncclResult_t comm_poll(RcclApi *api, ncclComm_t c, double timeout) {
    const double t0 = now_s();
    for (;;) {
        ncclResult_t st = ncclSuccess;
        const ncclResult_t r = api->get_async_error(c, &st);
        if (r != ncclSuccess) return r;
        if (st != ncclInProgress) return st;
        if (now_s() - t0 > timeout) return ncclInProgress;
        std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
}

// ---- collective watchdog -------------------------------------------------------------------------
// Every collective is bracketed by two events on its stream.  A watchdog thread polls the oldest
// pending pair: once the stream has reached the collective (the first event done), the collective
// must finish (the second event) within the deadline, else the thread aborts the communicator --
// RCCL's kernels see the abort flag and return, the stream drains, and every later nngp_comm_* /
// collective call reports NNGP_E_HIP ("aborted").  Host-side waits (the caller's synchronise) are
// therefore bounded too.
struct Watch {
    hipEvent_t a, b;
    double reached;   // wall time the watchdog first saw `a` complete (0: not yet)
};
static std::mutex g_wd_mu;
static std::condition_variable g_wd_cv;
static std::deque<Watch> g_wd_pending;
static std::vector<hipEvent_t> g_wd_free;
static std::thread g_wd_thread;
static bool g_wd_stop = false;
static std::atomic<long> g_wd_aborts{0};

static void watchdog_loop(int dev) {
    (void)hipSetDevice(dev);
    std::unique_lock<std::mutex> lk(g_wd_mu);
    while (!g_wd_stop) {
        if (g_wd_pending.empty()) {
            g_wd_cv.wait_for(lk, std::chrono::milliseconds(50));
            continue;
        }
        Watch &w = g_wd_pending.front();
        if (hipEventQuery(w.b) == hipSuccess) {
            g_wd_free.push_back(w.a);
            g_wd_free.push_back(w.b);
            g_wd_pending.pop_front();
            continue;
        }
        if (w.reached == 0.0 && hipEventQuery(w.a) == hipSuccess) w.reached = now_s();
        if (w.reached > 0.0 && now_s() - w.reached > comm_timeout_s()) {
            // abort (outside g_wd_mu: the abort drains RCCL's kernels, and callers may hold g_comm_mu)
            lk.unlock();
            {
                std::lock_guard<std::mutex> ck(g_comm_mu);
                if (g_comm && g_rccl.comm_abort) (void)g_rccl.comm_abort(g_comm);
                g_comm = nullptr;
                g_comm_aborted = true;
            }
            g_wd_aborts++;
            lk.lock();
            for (Watch &x : g_wd_pending) {
                g_wd_free.push_back(x.a);
                g_wd_free.push_back(x.b);
            }
            g_wd_pending.clear();
            continue;
        }
        g_wd_cv.wait_for(lk, std::chrono::milliseconds(2));
    }
}

// record the bracketing events of one collective: `before` ahead of it, `after` behind it
static int watch_begin(hipStream_t st, hipEvent_t *a) {
    std::lock_guard<std::mutex> lk(g_wd_mu);
    if (!g_wd_thread.joinable()) {
        g_wd_stop = false;
        g_wd_thread = std::thread(watchdog_loop, g_comm_dev);
    }
    for (int k = 0; k < 2 && g_wd_free.size() < 2; k++) {
        hipEvent_t e;
        NNGP_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        g_wd_free.push_back(e);
    }
    *a = g_wd_free.back();
    g_wd_free.pop_back();
    NNGP_HIP_CHECK(hipEventRecord(*a, st));
    return NNGP_OK;
}

static int watch_end(hipStream_t st, hipEvent_t a) {
    std::lock_guard<std::mutex> lk(g_wd_mu);
    hipEvent_t b = g_wd_free.back();
    g_wd_free.pop_back();
    NNGP_HIP_CHECK(hipEventRecord(b, st));
    g_wd_pending.push_back({a, b, 0.0});
    g_wd_cv.notify_one();
    return NNGP_OK;
}

static void watchdog_release() {
    {
        std::lock_guard<std::mutex> lk(g_wd_mu);
        g_wd_stop = true;
        g_wd_cv.notify_one();
    }
    if (g_wd_thread.joinable()) g_wd_thread.join();
    std::lock_guard<std::mutex> lk(g_wd_mu);
    for (Watch &x : g_wd_pending) {
        g_wd_free.push_back(x.a);
        g_wd_free.push_back(x.b);
    }
    g_wd_pending.clear();
    for (hipEvent_t e : g_wd_free) (void)hipEventDestroy(e);
    g_wd_free.clear();
}

// nngp_shutdown: the communicator (re-created by the next nngp_comm_init)
void comm_release() {
    watchdog_release();
    std::lock_guard<std::mutex> lk(g_comm_mu);
    if (g_comm && g_rccl.comm_destroy) (void)g_rccl.comm_destroy(g_comm);
    g_comm = nullptr;
    g_comm_aborted = false;
    g_comm_ranks = 0;
    g_comm_rank = -1;
    g_comm_dev = -1;
}

}  // namespace nngp

extern "C" int nngp_comm_unique_id(void *uid_out) {
    using namespace nngp;
    NNGP_REQUIRE(uid_out, "null argument");
    RcclApi *api = nullptr;
    const int rc = rccl_api(&api);
    if (rc) return rc;
    ncclUniqueId id;
    NNGP_RCCL_CHECK(api, api->get_unique_id(&id));
    static_assert(sizeof(ncclUniqueId) == NNGP_COMM_UID_BYTES, "ncclUniqueId size");
    memcpy(uid_out, &id, sizeof(id));
    return NNGP_OK;
}

extern "C" int nngp_comm_available(void) {
    using namespace nngp;
    RcclApi *api = nullptr;
    return rccl_api(&api);
}

extern "C" int nngp_comm_init(int nranks, int rank, const void *uid) {
    using namespace nngp;
    NNGP_REQUIRE(uid && nranks >= 1 && 0 <= rank && rank < nranks, "bad communicator arguments");
    RcclApi *api = nullptr;
    int rc = rccl_api(&api);
    if (rc) return rc;
    int dev = 0;
    NNGP_HIP_CHECK(hipGetDevice(&dev));
    watchdog_release();   // a previous communicator's watchdog (it is restarted on the next collective)
    std::lock_guard<std::mutex> lk(g_comm_mu);
    if (g_comm) {
        (void)api->comm_destroy(g_comm);
        g_comm = nullptr;
    }
    g_comm_aborted = false;
    ncclUniqueId id;
    memcpy(&id, uid, sizeof(id));
    // non-blocking init (collective over the ranks), bounded by the deadline: a rank whose peers
    // never arrive aborts its half-built communicator and returns NNGP_E_HIP
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    ncclComm_t c = nullptr;
    const double timeout = comm_timeout_s();
    ncclResult_t r = api->comm_init_rank_config(&c, nranks, id, rank, &cfg);
    if (r == ncclInProgress || (r == ncclSuccess && c)) r = comm_poll(api, c, timeout);
    if (r != ncclSuccess) {
        if (c) (void)api->comm_abort(c);
        if (r == ncclInProgress)
            set_error("nngp_comm_init: rank %d of %d still waiting for its peers after %.0f s "
                      "(NNGP_COMM_TIMEOUT_S); communicator aborted", rank, nranks, timeout);
        else
            set_error("ncclCommInitRankConfig failed: %s", api->error_string(r));
        return NNGP_E_HIP;
    }
    g_comm = c;
    g_comm_ranks = nranks;
    g_comm_rank = rank;
    g_comm_dev = dev;
    return NNGP_OK;
}

extern "C" int nngp_comm_size(int *nranks_out, int *rank_out) {
    using namespace nngp;
    std::lock_guard<std::mutex> lk(g_comm_mu);
    if (nranks_out) *nranks_out = g_comm ? g_comm_ranks : 0;
    if (rank_out) *rank_out = g_comm ? g_comm_rank : -1;
    if (g_comm_aborted) {
        set_error("the communicator was aborted: a collective ran past NNGP_COMM_TIMEOUT_S");
        return NNGP_E_HIP;
    }
    return NNGP_OK;
}

extern "C" int nngp_comm_destroy(void) {
    nngp::comm_release();
    return NNGP_OK;
}

namespace nngp {

static int comm_allgather(const double *send, double *recv, size_t per_rank, hipStream_t st) {
    RcclApi *api = nullptr;
    const int rc = rccl_api(&api);
    if (rc) return rc;
    int dev = 0;
    NNGP_HIP_CHECK(hipGetDevice(&dev));
    // held across the enqueue: the watchdog's abort waits for it (never the other way round)
    std::lock_guard<std::mutex> lk(g_comm_mu);
    if (g_comm_aborted) {
        set_error("the communicator was aborted: a collective ran past NNGP_COMM_TIMEOUT_S");
        return NNGP_E_HIP;
    }
    NNGP_REQUIRE(g_comm, "no communicator: call nngp_comm_init first");
    NNGP_REQUIRE(dev == g_comm_dev, "the communicator belongs to device %d, the current one is %d", g_comm_dev, dev);
    hipEvent_t a = nullptr;
    int w = watch_begin(st, &a);
    if (w) return w;
    ncclResult_t r = api->all_gather(send, recv, per_rank, ncclDouble, g_comm, st);
    if (r == ncclInProgress) r = comm_poll(api, g_comm, comm_timeout_s());   // non-blocking enqueue
    w = watch_end(st, a);
    if (r != ncclSuccess) {
        (void)api->comm_abort(g_comm);
        g_comm = nullptr;
        g_comm_aborted = true;
        set_error("ncclAllGather: %s; communicator aborted",
                  r == ncclInProgress ? "enqueue still in progress past NNGP_COMM_TIMEOUT_S" : api->error_string(r));
        return NNGP_E_HIP;
    }
    return w;
}

}  // namespace nngp

extern "C" int nngp_allgather_states(const double *send, double *recv, size_t per_rank_elems, void *stream) {
    using namespace nngp;
    NNGP_REQUIRE(send && recv, "null argument");
    if (per_rank_elems == 0) return NNGP_OK;
    return comm_allgather(send, recv, per_rank_elems, (hipStream_t)stream);
}

// The coordinate-sharded correction sweep (parareal.py:359-382 with each prediction's fits split
// by coordinate): for i = I .. N-1, on `stream`, with no host synchronisation --
//   UG1[i+1] = G(U1[i])                                      (replicated)
//   gather[rank*chunk .. +c1-c0] = preds[c0:c1](U1[i])       (this rank's coordinates)
//   all-gather of the [chunk] blocks (in place)              (RCCL)
//   U1[i+1] = (gather[0:d] - 0) + UG1[i+1]                   (bitwise mean + uG, as the fused kernel)
// The caller's Python loop (parareal.correction_sweep_sharded) issued the same launches one by one.
namespace nngp {

// emulate_ranks = 0: the communicator's ranks.  emulate_ranks = W >= 1 (one-rank communicator only):
// this process plays all W ranks of the coordinate split in turn -- each rank's [c0, c1) into its
// own gather block, no collective -- so the split, the partial last block and the block placement
// are checked on one GPU against the unsharded sweep (tests/test_gpu_distributed.py).
// gather_elems: the caller's gather length, checked against ranks * chunk before any launch.
static int sweep_sharded(const nngp_system *sys, int g_tableau, int g_step_mode, int64_t g_steps, const double *t,
                         int I, int N, double *U1, double *UG1, const double *X, const double *Y, int64_t rows,
                         int m, int n_jitter, const double *jitter_exp_host, int n_restarts, const double *theta0,
                         double fatol, double xatol, int maxfev, double *gather, size_t gather_elems,
                         int emulate_ranks, float *g_ms_out, void *stream) {
    NNGP_REQUIRE(sys && t && U1 && UG1 && X && Y && theta0 && gather, "null argument");
    NNGP_REQUIRE(0 <= I && I <= N, "need 0 <= I <= N (I=%d N=%d)", I, N);
    int nranks = 0, rank = -1;
    {
        std::lock_guard<std::mutex> lk(g_comm_mu);
        if (g_comm_aborted) {
            set_error("the communicator was aborted: a collective ran past NNGP_COMM_TIMEOUT_S");
            return NNGP_E_HIP;
        }
        nranks = g_comm ? g_comm_ranks : 0;
        rank = g_comm_rank;
    }
    NNGP_REQUIRE(nranks >= 1, "no communicator: call nngp_comm_init first");
    NNGP_REQUIRE(emulate_ranks == 0 || (nranks == 1 && emulate_ranks >= 1),
                 "rank emulation needs a one-rank communicator (have %d ranks)", nranks);
    const int d = sys->d;
    const int vranks = emulate_ranks > 0 ? emulate_ranks : nranks;
    const int chunk = (d + vranks - 1) / vranks;   // parareal.shard_bounds(0, d, vranks, rank)
    NNGP_REQUIRE(gather_elems >= (size_t)vranks * chunk, "gather holds %zu doubles, the split needs %d x %d",
                 gather_elems, vranks, chunk);
    const int r_lo = emulate_ranks > 0 ? 0 : rank, r_hi = emulate_ranks > 0 ? vranks : rank + 1;
    const int64_t n_fits = (int64_t)d * n_jitter * n_restarts;
    hipStream_t st = (hipStream_t)stream;
    int err = 0;
    // zeros[d] for the update's (a - b) + c form
    double *zeros = (double *)workspace(sizeof(double) * (size_t)d, &err, 9);
    if (err) return err;
    NNGP_HIP_CHECK(hipMemsetAsync(zeros, 0, sizeof(double) * (size_t)d, st));
    hipEvent_t *ev = nullptr;   // G launch timing from the sweep's event pool (summed at the end)
    if (g_ms_out) {
        *g_ms_out = 0.f;
        if (N > I) {
            const int rc0 = timing_events(2 * (size_t)(N - I), &ev);
            if (rc0) return rc0;
        }
    }
    int rc = NNGP_OK;
    for (int i = I; i < N && rc == NNGP_OK; i++) {
        const size_t j = (size_t)(i - I);
        const double *ui = U1 + (size_t)i * d;
        double *ug_next = UG1 + (size_t)(i + 1) * d;
        if (ev) NNGP_HIP_CHECK(hipEventRecord(ev[2 * j], st));
        rc = nngp_rk_batch(sys, g_tableau, g_step_mode, 1, t + i, t + i + 1, g_steps, ui, ug_next, stream);
        if (rc) break;
        if (ev) NNGP_HIP_CHECK(hipEventRecord(ev[2 * j + 1], st));
        for (int r = r_lo; r < r_hi && rc == NNGP_OK; r++) {
            const int c0 = std::min(r * chunk, d), c1 = std::min((r + 1) * chunk, d);
            if (c1 > c0)
                rc = predict_impl(X, Y, rows, d, ui, m, n_jitter, jitter_exp_host, n_restarts,
                                  theta0 + j * n_fits * 2, fatol, xatol, maxfev, gather + (size_t)r * chunk, nullptr,
                                  nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, st, c0, c1,
                                  nullptr, nullptr);
        }
        if (rc) break;
        if (nranks > 1) {   // in place: this rank's block sits at rank * chunk of the gather buffer
            rc = comm_allgather(gather + (size_t)rank * chunk, gather, (size_t)chunk, st);
            if (rc) break;
        }
        rc = nngp_parareal_update(d, gather, zeros, ug_next, U1 + (size_t)(i + 1) * d, stream);
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

}  // namespace nngp

extern "C" int nngp_correction_sweep_sharded(const nngp_system *sys, int g_tableau, int g_step_mode,
                                             int64_t g_steps, const double *t, int I, int N, double *U1,
                                             double *UG1, const double *X, const double *Y, int64_t rows, int m,
                                             int n_jitter, const double *jitter_exp_host, int n_restarts,
                                             const double *theta0, double fatol, double xatol, int maxfev,
                                             double *gather, float *g_ms_out, void *stream) {
    int nranks = 0;
    {
        std::lock_guard<std::mutex> lk(nngp::g_comm_mu);
        nranks = nngp::g_comm ? nngp::g_comm_ranks : 0;
    }
    const size_t need = nranks >= 1 && sys ? (size_t)nranks * ((sys->d + nranks - 1) / nranks) : 0;
    return nngp::sweep_sharded(sys, g_tableau, g_step_mode, g_steps, t, I, N, U1, UG1, X, Y, rows, m, n_jitter,
                               jitter_exp_host, n_restarts, theta0, fatol, xatol, maxfev, gather, need, 0, g_ms_out,
                               stream);
}

extern "C" int nngp_correction_sweep_sharded_emulated(const nngp_system *sys, int g_tableau, int g_step_mode,
                                                      int64_t g_steps, const double *t, int I, int N, double *U1,
                                                      double *UG1, const double *X, const double *Y, int64_t rows,
                                                      int m, int n_jitter, const double *jitter_exp_host,
                                                      int n_restarts, const double *theta0, double fatol,
                                                      double xatol, int maxfev, double *gather, size_t gather_elems,
                                                      int emulate_ranks, float *g_ms_out, void *stream) {
    if (emulate_ranks < 1) {
        nngp::set_error("emulate_ranks must be >= 1");
        return NNGP_E_ARG;
    }
    return nngp::sweep_sharded(sys, g_tableau, g_step_mode, g_steps, t, I, N, U1, UG1, X, Y, rows, m, n_jitter,
                               jitter_exp_host, n_restarts, theta0, fatol, xatol, maxfev, gather, gather_elems,
                               emulate_ranks, g_ms_out, stream);
}
