// ubench_gpf.hip -- where the full-GP factorisation round spends its time:
// clock64 cycles of the 32x32 diagonal-block factor (one wave) and of one thread's 32-column row
// solve, and HIP-event times of panel 0's diag + rows launches and one whole batched -LML evaluation.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off -w tools/ubench_gpf.hip \
//        -o scratch_bin/ubench_gpf
#include "../nearest-neighbors-gparareal_amd/csrc/nngp_gpfull.hip"
#include "../nearest-neighbors-gparareal_amd/csrc/nngp_lib.hip"

#include <cstdio>
#include <vector>

namespace nngp {   // nngp_shutdown's parts in the translation units this bench does not link
void chain_release() {}
void sweep_release() {}
void comm_release() {}
}  // namespace nngp

using namespace nngp;

__global__ void __launch_bounds__(64) diag_loop(const double *A, int reps, double *out, long long *cyc) {
    __shared__ double col[2 * GPB];
    const int i = threadIdx.x;
    double a[GPB], rv[GPB];
    for (int k = 0; k < GPB; k++) a[k] = (k <= (i & 31)) ? A[(i & 31) * GPB + k] : 0.0;
    double acc = 0.0;
    long long t0 = clock64();
    for (int r = 0; r < reps; r++) {
        double b[GPB];
        for (int k = 0; k < GPB; k++) b[k] = a[k] + acc * 1e-300;
        bool bad;
        diag_factor(b, rv, i & 31, i >> 5, GPB, col, bad);
        acc += b[GPB - 1] + rv[3];
    }
    long long t1 = clock64();
    out[i] = acc;
    if (i == 0) cyc[0] = t1 - t0;
}

__global__ void __launch_bounds__(256) rowsolve_loop(const double *L0, int reps, double *out, long long *cyc) {
    __shared__ double L[GPB][GPB + 1];
    __shared__ double Rv[GPB];
    const int tid = threadIdx.x;
    for (int t = tid; t < GPB * GPB; t += blockDim.x) L[t / GPB][t % GPB] = L0[t];
    if (tid < GPB) Rv[tid] = 1.0 / L0[tid * GPB + tid];
    __syncthreads();
    double x[GPB];
    for (int k = 0; k < GPB; k++) x[k] = 1.0 + 0.01 * (k + tid);
    long long t0 = clock64();
    for (int r = 0; r < reps; r++) {
#pragma unroll
        for (int j = 0; j < GPB; j++) {
            x[j] = x[j] * Rv[j];
#pragma unroll
            for (int k = j + 1; k < GPB; k++) x[k] = x[k] - x[j] * L[k][j];
        }
    }
    long long t1 = clock64();
    double s = 0.0;
    for (int k = 0; k < GPB; k++) s += x[k];
    out[tid] = s;
    if (tid == 0) cyc[0] = t1 - t0;
}

int main() {
    // a well-conditioned 32x32 SPD block
    std::vector<double> A(GPB * GPB);
    for (int i = 0; i < GPB; i++)
        for (int j = 0; j < GPB; j++) A[i * GPB + j] = (i == j ? GPB + 1.0 : 0.0) + 1.0 / (1 + i + j);
    std::vector<double> Lh(GPB * GPB, 0.0);   // its Cholesky factor (host) for the row-solve bench
    for (int j = 0; j < GPB; j++) {
        double s = A[j * GPB + j];
        for (int k = 0; k < j; k++) s -= Lh[j * GPB + k] * Lh[j * GPB + k];
        Lh[j * GPB + j] = sqrt(s);
        for (int i = j + 1; i < GPB; i++) {
            double t = A[i * GPB + j];
            for (int k = 0; k < j; k++) t -= Lh[i * GPB + k] * Lh[j * GPB + k];
            Lh[i * GPB + j] = t / Lh[j * GPB + j];
        }
    }
    double *dA, *dL, *dout;
    long long *dc;
    hipMalloc(&dA, sizeof(double) * GPB * GPB);
    hipMalloc(&dL, sizeof(double) * GPB * GPB);
    hipMalloc(&dout, sizeof(double) * 256);
    hipMalloc(&dc, sizeof(long long));
    hipMemcpy(dA, A.data(), sizeof(double) * GPB * GPB, hipMemcpyHostToDevice);
    hipMemcpy(dL, Lh.data(), sizeof(double) * GPB * GPB, hipMemcpyHostToDevice);
    long long cyc = 0;
    const int reps = 50;
    hipLaunchKernelGGL(diag_loop, dim3(1), dim3(64), 0, 0, dA, reps, dout, dc);
    hipMemcpy(&cyc, dc, sizeof(cyc), hipMemcpyDeviceToHost);
    printf("diag_factor 2 x 32x32 (one wave): %.0f cycles\n", (double)cyc / reps);
    hipLaunchKernelGGL(rowsolve_loop, dim3(1), dim3(256), 0, 0, dL, reps, dout, dc);
    hipMemcpy(&cyc, dc, sizeof(cyc), hipMemcpyDeviceToHost);
    printf("row solve 32 columns (256 threads): %.0f cycles\n", (double)cyc / reps);

    // one batched evaluation: nb points, n rows, d = 3
    for (int n : {128, 377, 700}) {
        const int d = 3, nb = 27;
        std::vector<double> X((size_t)n * d), Y((size_t)n * d);
        for (int i = 0; i < n * d; i++) {
            X[i] = sin(0.37 * i) + 0.01 * i / n;
            Y[i] = cos(0.11 * i);
        }
        double *dX, *dY;
        hipMalloc(&dX, sizeof(double) * n * d);
        hipMalloc(&dY, sizeof(double) * n * d);
        hipMemcpy(dX, X.data(), sizeof(double) * n * d, hipMemcpyHostToDevice);
        hipMemcpy(dY, Y.data(), sizeof(double) * n * d, hipMemcpyHostToDevice);
        GPFWork w;
        gpf_workspace(n, nb, w);
        hipLaunchKernelGGL(gpf_d2_kernel, dim3((n + 15) / 16, (n + 15) / 16), dim3(16, 16), 0, 0, dX, n, d, w.D2);
        std::vector<GPPoint> hp(nb);
        for (int b = 0; b < nb; b++) hp[b] = gp_point(0.5 + 0.01 * b, 1.0, -12.0, b % d);
        hipMemcpy(w.pts, hp.data(), sizeof(GPPoint) * nb, hipMemcpyHostToDevice);
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        gpf_eval(w.D2, n, dY, d, w.pts, nb, w.A, w.fail, w.fval, nullptr, w.Lpan, 0);
        hipEventRecord(e0, 0);
        for (int r = 0; r < 10; r++) gpf_eval(w.D2, n, dY, d, w.pts, nb, w.A, w.fail, w.fval, nullptr, w.Lpan, 0);
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        // panel 0 alone (diagonal factor + row solve)
        hipEventRecord(e0, 0);
        for (int r = 0; r < 10; r++) {
            const int below = n + 1 - GPB;
            hipLaunchKernelGGL(gpf_diag_kernel, dim3((nb + 1) / 2), dim3(64), 0, 0, w.A, n, 0, GPB, nb, w.fail, w.Lpan);
            hipLaunchKernelGGL(gpf_rows_kernel<true>, dim3((below + 63) / 64, nb), dim3(64), 0, 0, w.A, n, 0, GPB,
                               w.fail, w.Lpan);
        }
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float mp = 0;
        hipEventElapsedTime(&mp, e0, e1);
        printf("n=%d nb=%d: eval %.1f us (%d panels), panel0 %.1f us\n", n, nb, 1e3 * ms / 10, (n + GPB - 1) / GPB,
               1e3 * mp / 10);
        hipFree(dX);
        hipFree(dY);
    }
    return 0;
}
