// ubench_fp64.hip -- FP64 VALU dependent-chain latency and issue cost on one wave (gfx950).
// Informs the lane-kernel design ("latency roofline"): a fine RK slice is one
// dependent chain, so the per-step floor is (critical-path ops) x (dependent fp64 latency).
// Build: hipcc -O3 --offload-arch=gfx950 tools/ubench_fp64.hip -o tools/_ubench_fp64
#include <hip/hip_runtime.h>

#include <cstdio>

#define REP 4096

template <int CHAINS, int OP>
__global__ void chain(double *out, long long *cyc, double a, double b) {
    double x[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; c++) x[c] = threadIdx.x * 1e-3 + c;
    __syncthreads();
    long long t0 = clock64();
    for (int r = 0; r < REP; r += 8) {
#pragma unroll
        for (int u = 0; u < 8; u++)
#pragma unroll
            for (int c = 0; c < CHAINS; c++) {
                if (OP == 0) x[c] = __builtin_fma(x[c], a, b);
                if (OP == 1) x[c] = x[c] * a;
                if (OP == 2) x[c] = x[c] + b;
            }
    }
    long long t1 = clock64();
    double s = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; c++) s += x[c];
    out[threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void clk(long long *c) {
    c[0] = clock64();
    c[1] = wall_clock64();
    long long t = clock64();
    while (clock64() - t < 100000000LL) {
    }
    c[2] = clock64();
    c[3] = wall_clock64();
}

template <int CHAINS, int OP>
static void run(const char *name, int lanes) {
    double *o;
    long long *c, h = 0;
    hipMalloc(&o, 64 * 8);
    hipMalloc(&c, 8);
    chain<CHAINS, OP><<<1, lanes>>>(o, c, 1.0000001, 1e-9);
    chain<CHAINS, OP><<<1, lanes>>>(o, c, 1.0000001, 1e-9);
    hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
    printf("%-6s chains=%d lanes=%2d : %.2f cycles per op-instruction (per chain step %.2f)\n", name, CHAINS,
           lanes, (double)h / (REP * CHAINS), (double)h / REP);
    hipFree(o);
    hipFree(c);
}

int main() {
    long long *c, h[4];
    hipMalloc(&c, 32);
    clk<<<1, 1>>>(c);
    hipMemcpy(h, c, 32, hipMemcpyDeviceToHost);
    int wclk = 0;
    hipDeviceGetAttribute(&wclk, hipDeviceAttributeWallClockRate, 0);
    printf("shader clock ~ %.0f MHz (wall clock %d kHz)\n",
           (double)(h[2] - h[0]) / (double)(h[3] - h[1]) * wclk / 1e3, wclk);
    run<1, 0>("fma", 64);
    run<1, 0>("fma", 1);
    run<8, 0>("fma", 1);
    run<8, 0>("fma", 16);
    run<8, 0>("fma", 32);
    run<8, 0>("fma", 48);
    run<2, 0>("fma", 64);
    run<4, 0>("fma", 64);
    run<8, 0>("fma", 64);
    run<1, 1>("mul", 64);
    run<4, 1>("mul", 64);
    run<1, 2>("add", 64);
    run<4, 2>("add", 64);
    return 0;
}
