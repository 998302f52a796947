// ubench_halo.hip -- what one RK stage of a slice split over two workgroups would pay to exchange
// its halo (the 64-slices-per-GPU FHN-PDE sweep).  Two workgroups on the same XCD
// (workgroups w and w+8 of the grid: dispatch is round-robin over the 8 XCDs) ping-pong a 20-double
// halo row per "stage": each writes its row, publishes a stage counter (agent-scope release), waits
// for the partner's counter (agent-scope acquire, s_sleep between polls) and reads the partner's
// row.  A pair on different XCDs (w and w+1) is timed too.  Reports microseconds per exchange,
// against the 0.36 us a stage of the one-workgroup slice takes now (4.0 us per 11-stage RK8 step).
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/ubench_halo.hip -o scratch_bin/ubench_halo
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int HALO = 20;   // one grid row of a 20 x 20 FHN-PDE field

__global__ void __launch_bounds__(256) pingpong(double *buf, unsigned *flag, int stages, int a, int b,
                                                 double *sink, long long *cyc) {
    const int w = blockIdx.x;
    if (w != a && w != b) return;
    const int me = w == a ? 0 : 1, other = 1 - me;
    double *mine = buf + me * HALO, *theirs = buf + other * HALO;
    double acc = 0.0;
    const long long t0 = wall_clock64();
    for (int s = 1; s <= stages; s++) {
        if (threadIdx.x < HALO) mine[threadIdx.x] = acc + s;   // this stage's halo row
        __syncthreads();
        if (threadIdx.x == 0) {
            __hip_atomic_store(flag + me, (unsigned)s, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            unsigned spin = 0;   // bounded: never a hang
            while (__hip_atomic_load(flag + other, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)s &&
                   ++spin < (1u << 22))
                __builtin_amdgcn_s_sleep(1);
        }
        __syncthreads();
        if (threadIdx.x < HALO) acc += __hip_atomic_load(theirs + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
    }
    const long long t1 = wall_clock64();
    if (threadIdx.x < HALO) sink[me * HALO + threadIdx.x] = acc;
    if (threadIdx.x == 0 && me == 0) cyc[0] = t1 - t0;
}

int main() {
    double *buf, *sink;
    unsigned *flag;
    long long *cyc, h = 0;
    (void)hipMalloc(&buf, sizeof(double) * 2 * HALO);
    (void)hipMalloc(&sink, sizeof(double) * 2 * HALO);
    (void)hipMalloc(&flag, sizeof(unsigned) * 2);
    (void)hipMalloc(&cyc, sizeof(long long));
    int khz = 100000;
    (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0);
    const int stages = 20000;
    for (int pair = 0; pair < 2; pair++) {
        const int a = 0, b = pair == 0 ? 8 : 1;
        for (int rep = 0; rep < 2; rep++) {
            (void)hipMemset(flag, 0, sizeof(unsigned) * 2);
            (void)hipMemset(buf, 0, sizeof(double) * 2 * HALO);
            pingpong<<<16, 256>>>(buf, flag, stages, a, b, sink, cyc);
            if (hipDeviceSynchronize() != hipSuccess) return 1;
            (void)hipMemcpy(&h, cyc, sizeof h, hipMemcpyDeviceToHost);
            printf("%s pair (wg %d, %d): %.3f us per stage exchange (%d stages)\n",
                   pair == 0 ? "same-XCD" : "cross-XCD", a, b, (double)h / (khz * 1e-3) / stages, stages);
        }
    }
    return 0;
}
