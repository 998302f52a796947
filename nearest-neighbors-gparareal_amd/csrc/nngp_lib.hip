// nngp_lib.hip -- library-level entry points: version, errors, device count, workspace.
#include <stdarg.h>

#include <mutex>
#include <vector>

#include "common.h"

namespace nngp {

static thread_local char g_err[1024] = "";

void set_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

struct Ws {
    void *ptr = nullptr;
    size_t bytes = 0;
};
static std::vector<Ws> g_ws;   // [device * N_WS_SLOTS + slot]
static std::mutex g_ws_mu;

void *workspace(size_t bytes, int *err, int slot) {
    int dev = 0;
    *err = 0;
    if (hipGetDevice(&dev) != hipSuccess) {
        set_error("hipGetDevice failed");
        *err = NNGP_E_HIP;
        return nullptr;
    }
    std::lock_guard<std::mutex> lk(g_ws_mu);
    const int key = dev * N_WS_SLOTS + slot;
    if ((int)g_ws.size() <= key) g_ws.resize(key + 1);
    Ws &w = g_ws[key];
    if (w.bytes < bytes) {
        // grow (x1.5) -- the stream-ordered users are synchronised by hipFree's implicit sync
        if (w.ptr) (void)hipFree(w.ptr);
        size_t nb = bytes + bytes / 2 + 4096;
        hipError_t e = hipMalloc(&w.ptr, nb);
        if (e != hipSuccess) {
            w.ptr = nullptr;
            w.bytes = 0;
            set_error("hipMalloc(%zu) for workspace failed: %s", nb, hipGetErrorString(e));
            *err = NNGP_E_HIP;
            return nullptr;
        }
        w.bytes = nb;
    }
    return w.ptr;
}

static std::mutex g_attr_mu;
static std::vector<int> g_cus;
static std::vector<double> g_khz;

static void device_attrs(int *cus, double *khz) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    std::lock_guard<std::mutex> lk(g_attr_mu);
    if ((int)g_cus.size() <= dev) {
        g_cus.resize(dev + 1, 0);
        g_khz.resize(dev + 1, 0.0);
    }
    if (g_cus[dev] <= 0) {
        int n = 0, k = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
        if (hipDeviceGetAttribute(&k, hipDeviceAttributeWallClockRate, dev) != hipSuccess || k <= 0) k = 100000;
        g_cus[dev] = n;
        g_khz[dev] = k;
    }
    if (cus) *cus = g_cus[dev];
    if (khz) *khz = g_khz[dev];
}

int device_cus() {
    int n;
    device_attrs(&n, nullptr);
    return n;
}

double device_wallclock_khz() {
    double k;
    device_attrs(nullptr, &k);
    return k;
}

// nngp_shutdown: free every workspace slot (re-allocated on next use)
static void ws_release() {
    std::lock_guard<std::mutex> lk(g_ws_mu);
    for (Ws &w : g_ws)
        if (w.ptr) (void)hipFree(w.ptr);
    g_ws.clear();
}

}  // namespace nngp

// Release every device / host-mapped resource the library holds (workspaces, side streams,
// events, the fused chain's flags) after draining the device, so that nothing of ours is left
// for the HIP runtime's own process-exit teardown.  The Python package registers it with atexit;
// later calls simply re-create what they need.
extern "C" int nngp_shutdown(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return NNGP_OK;
    (void)hipDeviceSynchronize();
    nngp::chain_release();
    nngp::sweep_release();
    nngp::comm_release();
    nngp::ws_release();
    return NNGP_OK;
}

extern "C" int nngp_abi_version(void) { return NNGP_ABI_VERSION; }

extern "C" const char *nngp_last_error(void) { return nngp::g_err; }

extern "C" int nngp_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}
