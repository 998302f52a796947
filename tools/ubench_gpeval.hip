// ubench_gpeval.hip -- registers and cycles of ONE likelihood evaluation (nngp_gpeval.h) per
// padded size, 4 fits per wave, outside any Nelder-Mead kernel.  Compiles in seconds, so layouts
// of the evaluation core can be compared quickly.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off -DUB_MAXM=20 \
//        -Rpass-analysis=kernel-resource-usage tools/ubench_gpeval.hip -o tools/_ubench_gpeval
#ifdef UB_HEADER   // another copy of the evaluation core, for old/new comparisons
#include UB_HEADER
#else
#include "../nearest-neighbors-gparareal_amd/csrc/nngp_gpeval.h"
#endif

#include <cstdio>
#include <cstring>
#include <vector>

#ifndef UB_MAXM
#define UB_MAXM 20
#endif

using namespace nngp;

template <int MAXM>
__global__ void __launch_bounds__(256) eval_loop(int m, const double *D2, const double *Y, int reps, double *out,
                                                 long long *cyc) {
    constexpr int RPL = GP<MAXM>::RPL, IMG = GP<MAXM>::IMG;
    __shared__ double sD2[MAXM * MAXM];
    extern __shared__ double sK[];
    const int tid = threadIdx.x, g = tid / 16, l = tid % 16;
    for (int i = tid; i < m * m; i += blockDim.x) sD2[i] = D2[i];
    __syncthreads();
    double y[RPL];
    for (int s = 0; s < RPL; s++) y[s] = (l + 16 * s < m) ? Y[l + 16 * s] : 0.0;
    GPLane<MAXM> P;
    gp_lane_init<MAXM>(P, m, l);
    double *Kimg = sK + g * IMG;
    gp_image_init<MAXM>(Kimg, m, l);
    double acc = 0.0, sx = -1.0 - 0.1 * (g % 4), sy = -2.0;
    long long t0 = clock64();
    for (int r = 0; r < reps; r++) {
        const double v = gp_nlml<MAXM>(m, l, P, sD2, sx, sy, 1e-12, y, Kimg);
        acc += v;
        sx += 1e-3 * (v > 0 ? 1 : -1);   // data dependence between evaluations
    }
    long long t1 = clock64();
    out[blockIdx.x * blockDim.x + tid] = acc;
    if (tid == 0 && blockIdx.x == 0) cyc[0] = t1 - t0;
}

int main() {
    constexpr int M = UB_MAXM;
    const int m = M;
    std::vector<double> X(m * 3), D2(m * m), Y(m);
    for (int i = 0; i < m * 3; i++) X[i] = 0.01 * ((i * 37) % 101) - 0.5;
    for (int r = 0; r < m; r++) {
        Y[r] = 0.01 * sin(3.0 * X[r * 3]);
        for (int j = 0; j < m; j++) {
            double s = 0;
            for (int c = 0; c < 3; c++) s += (X[r * 3 + c] - X[j * 3 + c]) * (X[r * 3 + c] - X[j * 3 + c]);
            D2[r * m + j] = s;
        }
    }
    double *dD2, *dY, *dout;
    long long *dc, h = 0;
    (void)hipMalloc(&dD2, 8 * m * m);
    (void)hipMalloc(&dY, 8 * m);
    (void)hipMalloc(&dout, 8 * 256 * 1024);
    (void)hipMalloc(&dc, 8);
    (void)hipMemcpy(dD2, D2.data(), 8 * m * m, hipMemcpyHostToDevice);
    (void)hipMemcpy(dY, Y.data(), 8 * m, hipMemcpyHostToDevice);
    const int reps = 200;
    for (int blocks : {1, 256, 512, 1024}) {
        hipEvent_t a, b;
        (void)hipEventCreate(&a);
        (void)hipEventCreate(&b);
        eval_loop<M><<<blocks, 256, 16 * GP<M>::IMG * 8>>>(m, dD2, dY, reps, dout, dc);
        (void)hipEventRecord(a);
        eval_loop<M><<<blocks, 256, 16 * GP<M>::IMG * 8>>>(m, dD2, dY, reps, dout, dc);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        (void)hipMemcpy(&h, dc, 8, hipMemcpyDeviceToHost);
        const double evals = (double)blocks * 16 * reps;
        std::vector<double> o(256);
        (void)hipMemcpy(o.data(), dout, 8 * 256, hipMemcpyDeviceToHost);
        unsigned long long hsh = 1469598103934665603ull;
        for (double v : o) { unsigned long long b; memcpy(&b, &v, 8); hsh = (hsh ^ b) * 1099511628211ull; }
        printf("MAXM=%d blocks=%d: %.0f cycles/eval (one wave), %.3f ms, %.2f M evals/s, out hash %016llx\n", M, blocks,
               (double)h / reps, ms, evals / (ms * 1e-3) / 1e6, hsh);
    }
    return 0;
}
