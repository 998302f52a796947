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
#include <cstring>
#include <mutex>

#include <rccl/rccl.h>

#include "common.h"

namespace nngp {

struct RcclApi {
    void *handle = nullptr;
    ncclResult_t (*get_unique_id)(ncclUniqueId *) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*all_gather)(const void *, void *, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    const char *(*error_string)(ncclResult_t) = nullptr;
};

static RcclApi g_rccl;
static ncclComm_t g_comm = nullptr;
static int g_comm_ranks = 0, g_comm_rank = -1, g_comm_dev = -1;
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
        a.comm_init_rank = (decltype(a.comm_init_rank))dlsym(h, "ncclCommInitRank");
        a.all_gather = (decltype(a.all_gather))dlsym(h, "ncclAllGather");
        a.comm_destroy = (decltype(a.comm_destroy))dlsym(h, "ncclCommDestroy");
        a.error_string = (decltype(a.error_string))dlsym(h, "ncclGetErrorString");
        if (!a.get_unique_id || !a.comm_init_rank || !a.all_gather || !a.comm_destroy || !a.error_string) {
            set_error("RCCL library lacks an entry point");
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

// nngp_shutdown: the communicator (re-created by the next nngp_comm_init)
void comm_release() {
    std::lock_guard<std::mutex> lk(g_comm_mu);
    if (g_comm && g_rccl.comm_destroy) (void)g_rccl.comm_destroy(g_comm);
    g_comm = nullptr;
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

extern "C" int nngp_comm_init(int nranks, int rank, const void *uid) {
    using namespace nngp;
    NNGP_REQUIRE(uid && nranks >= 1 && 0 <= rank && rank < nranks, "bad communicator arguments");
    RcclApi *api = nullptr;
    int rc = rccl_api(&api);
    if (rc) return rc;
    int dev = 0;
    NNGP_HIP_CHECK(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lk(g_comm_mu);
    if (g_comm) {
        (void)api->comm_destroy(g_comm);
        g_comm = nullptr;
    }
    ncclUniqueId id;
    memcpy(&id, uid, sizeof(id));
    NNGP_RCCL_CHECK(api, api->comm_init_rank(&g_comm, nranks, id, rank));   // collective over the ranks
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
    NNGP_REQUIRE(g_comm, "no communicator: call nngp_comm_init first");
    int dev = 0;
    NNGP_HIP_CHECK(hipGetDevice(&dev));
    NNGP_REQUIRE(dev == g_comm_dev, "the communicator belongs to device %d, the current one is %d", g_comm_dev, dev);
    NNGP_RCCL_CHECK(api, api->all_gather(send, recv, per_rank, ncclDouble, g_comm, st));
    return NNGP_OK;
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
extern "C" int nngp_correction_sweep_sharded(const nngp_system *sys, int g_tableau, int g_step_mode,
                                             int64_t g_steps, const double *t, int I, int N, double *U1,
                                             double *UG1, const double *X, const double *Y, int64_t rows, int m,
                                             int n_jitter, const double *jitter_exp_host, int n_restarts,
                                             const double *theta0, double fatol, double xatol, int maxfev,
                                             double *gather, float *g_ms_out, void *stream) {
    using namespace nngp;
    NNGP_REQUIRE(sys && t && U1 && UG1 && X && Y && theta0 && gather, "null argument");
    NNGP_REQUIRE(0 <= I && I <= N, "need 0 <= I <= N (I=%d N=%d)", I, N);
    int nranks = 0, rank = -1;
    {
        std::lock_guard<std::mutex> lk(g_comm_mu);
        nranks = g_comm ? g_comm_ranks : 0;
        rank = g_comm_rank;
    }
    NNGP_REQUIRE(nranks >= 1, "no communicator: call nngp_comm_init first");
    const int d = sys->d;
    // NNGP_SHARD_EMULATE_RANKS=W on a one-rank communicator: this process plays all W ranks of the
    // coordinate split in turn -- each rank's [c0, c1) into its own gather block, no collective --
    // so the split, the partial last block and the block placement are checked on one GPU against
    // the unsharded sweep (tests/test_gpu_distributed.py).  The caller sizes gather to W * chunk.
    const int vranks = nranks == 1 ? std::max(1, env_int("NNGP_SHARD_EMULATE_RANKS", 1)) : nranks;
    const int chunk = (d + vranks - 1) / vranks;   // parareal.shard_bounds(0, d, vranks, rank)
    const int r_lo = nranks == 1 ? 0 : rank, r_hi = nranks == 1 ? vranks : rank + 1;
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
