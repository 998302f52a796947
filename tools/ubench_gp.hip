// ubench_gp.hip -- cycles per GP likelihood evaluation (one 16-lane DPP row per fit) on gfx950,
// with and without the Nelder-Mead state machine around it.  Informs DESIGN.md §3.3.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off tools/ubench_gp.hip \
//        -o tools/_ubench_gp
#include "../nearest-neighbors-gparareal_amd/csrc/nngp_gp.hip"
#include "../nearest-neighbors-gparareal_amd/csrc/nngp_lib.hip"

#include <cstdio>
#include <vector>

using namespace nngp;

template <int MAXM>
__global__ void __launch_bounds__(64) eval_loop(int m, const double *D2, const double *Y, int reps, double *out, long long *cyc) {
    constexpr int RPL = GP<MAXM>::RPL, IMG = GP<MAXM>::IMG;
    __shared__ double sD2[32 * 32];
    __shared__ double sK[4 * GP<32>::IMG];
    const int tid = threadIdx.x, g = tid / 16, l = tid % 16;
    for (int i = tid; i < m * m; i += blockDim.x) sD2[i] = D2[i];
    __syncthreads();
    double y[RPL];
    for (int s = 0; s < RPL; s++) y[s] = (l + 16 * s < m) ? Y[l + 16 * s] : 0.0;
    GPLane<MAXM> P;
    gp_lane_init<MAXM>(P, m, l);
    double *Kimg = sK + g * IMG;
    gp_image_init<MAXM>(Kimg, m, l);
    double acc = 0.0, sx = -1.0 - 0.1 * g, sy = -2.0;
    long long t0 = clock64();
    for (int r = 0; r < reps; r++) {
        const double v = gp_nlml<MAXM>(m, l, P, sD2, sx, sy, 1e-12, y, Kimg);
        acc += v;
        sx += 1e-3 * (v > 0 ? 1 : -1);   // data dependence between evaluations
    }
    long long t1 = clock64();
    out[tid] = acc;
    if (tid == 0) cyc[0] = t1 - t0;
}

template <int MAXM>
static void run(int m) {
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
    (void)hipMalloc(&dout, 8 * 64);
    (void)hipMalloc(&dc, 8);
    (void)hipMemcpy(dD2, D2.data(), 8 * m * m, hipMemcpyHostToDevice);
    (void)hipMemcpy(dY, Y.data(), 8 * m, hipMemcpyHostToDevice);
    const int reps = 200;
    eval_loop<MAXM><<<1, 64>>>(m, dD2, dY, reps, dout, dc);
    eval_loop<MAXM><<<1, 64>>>(m, dD2, dY, reps, dout, dc);
    (void)hipMemcpy(&h, dc, 8, hipMemcpyDeviceToHost);
    printf("MAXM=%2d m=%2d: %8.0f cycles per evaluation (%.2f us at 2.4 GHz)\n", MAXM, m, (double)h / reps,
           (double)h / reps / 2400.0);
    (void)hipFree(dD2); (void)hipFree(dY); (void)hipFree(dout); (void)hipFree(dc);
}

int main() {
    run<8>(8);
    run<16>(10);
    run<16>(15);
    run<24>(20);
    run<32>(30);
    return 0;
}
