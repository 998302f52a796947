// nngp_gpfull.hip -- full-data GParareal correction (models.GPjax_p, models.py:273-473) on gfx950.
//
// The reference fits, per coordinate j and jitter in arange(-20, -11), the squared-exponential GP
// of ALL training rows (rows ~ N*K, hundreds to thousands) by Nelder-Mead on theta = (sigma_x,
// sigma_y) warm-started at the previous iteration's optimum (models.py:376-407 -> opt_theta
// :329-335 -> log_lik :321-327 -> _log_lik_np :314-319 -> _fit_gp_np :306-312):
//     K     = sigma_y^2 * exp(-0.5 * (1/sigma_x^2) * cdist(x, x, 'sqeuclidean')) + 10^jitter I
//     L     = cholesky(K)                 (LinAlgError -> +inf)
//     alpha = L^-T (L^-1 y)
//     -LML  = -(-0.5 y.alpha - sum(log diag L) - (rows/2) log 2 pi)
// Every Nelder-Mead round evaluates one point per unfinished fit; all of them form ONE batch of
// factorisations of the (n+1) x (n+1) matrix [K; y^T] (row n rides along as a "row below", so the
// factor's last row is z = L^-1 y and y.alpha = z.z):
//   gpf_build_kernel   K of every point of the batch (lower triangle) from the hoisted D^2, + y^T
//   gpf_panel_kernel   blocked right-looking Cholesky, panel j: a wave factors the 32x32 diagonal
//                      block in registers (dpotf2 order), each thread solves one row below it
//   gpf_syrk_kernel    trailing update A22 -= L21 L21^T, 32x32 lower tiles, LDS-staged panels
//   gpf_lml_kernel     -LML = 0.5 z.z + sum log L_ii + (n/2) log 2pi
//   gpf_alpha_kernel   alpha = L^-T z for the posterior weights (once per fit() per coordinate)
// FP64 VALU is the MI355X's FP64 peak (the FP64 MFMA rate is the same), so the tiles use plain
// VALU FMAs.  The arithmetic order of LAPACK's blocked potrf is not reproduced (it is
// third-party and build-dependent); parity is to tolerance (tests/test_gpu_gpfull.py).
// The Nelder-Mead state machines (nngp_nm.h, scipy's semantics) run on the host, one per fit.
#include <cmath>
#include <vector>

#include "common.h"
#include "nngp_nm.h"

namespace nngp {
#ifndef GPF_PANEL
#define GPF_PANEL 32
#endif

static constexpr int GPB = GPF_PANEL;                // panel width
static constexpr double GPF_LOG_2PI = 1.8378770664093453;   // np.log(2*np.pi)
static constexpr int GPF_LDS_ROWS = 7936;            // alpha_kernel keeps the vector in LDS (<= 62 KB) up to here,
                                                     // beyond it in its own output row (no row limit)

__device__ __forceinline__ void wave_sync_lds() {   // order one wave's LDS writes before its reads
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

struct GPPoint {      // one evaluation: kernel coefficients and the training column
    double c;         // -0.5 * (1 / sigma_x^2)
    double psy;       // sigma_y^2
    double jp;        // 10^jitter
    int coord;        // column of Y
    int pad;
};

// D2 = cdist(x, x, 'sqeuclidean'): sequential sum over the d components (scipy's loop)
__global__ void gpf_d2_kernel(const double *__restrict__ X, int n, int d, double *__restrict__ D2) {
    const int j = blockIdx.x * 16 + threadIdx.x, i = blockIdx.y * 16 + threadIdx.y;
    if (i >= n || j >= n) return;
    double acc = 0.0;
    for (int c = 0; c < d; c++) {
        const double t = X[(size_t)i * d + c] - X[(size_t)j * d + c];
        acc = acc + t * t;
    }
    D2[(size_t)i * n + j] = acc;
}

// Matrix b of the batch is stored (n+1) x (n+1) (ld = n+1): K in the leading n x n block and y^T
// in row n.  Factoring it with pivots 0..n-1 turns row n into z^T = (L^-1 y)^T -- the forward
// solve of _fit_gp_np rides along the Cholesky as one more "row below" -- so that
// y.alpha = y^T K^-1 y = z.z without a separate substitution.

// lower triangle (incl. diagonal) of K for point b: sigma_y^2 * exp(c * D2) (+ 10^jitter on the
// diagonal), kernel_np's order (models.py:302-304) and K + eye*10**jitter (:308); row n = y^T
__global__ void gpf_build_kernel(const double *__restrict__ D2, int n, const double *__restrict__ Y, int d,
                                 const GPPoint *__restrict__ pts, double *__restrict__ A,
                                 const int32_t *__restrict__ fail) {
    const int b = blockIdx.y;
    if (fail[b]) return;
    const GPPoint p = pts[b];
    const int ld = n + 1;
    double *Ab = A + (size_t)b * ld * ld;
    const size_t nn = (size_t)n * n;
    for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < nn + n; t += (size_t)gridDim.x * blockDim.x) {
        if (t >= nn) {   // row n: the training column
            const int j = (int)(t - nn);
            Ab[(size_t)n * ld + j] = Y[(size_t)j * d + p.coord];
            continue;
        }
        const int i = (int)(t / n), j = (int)(t - (size_t)i * n);
        if (j > i) continue;
        double v = p.psy * exp(p.c * D2[t]);
        if (i == j) v = v + p.jp;
        Ab[(size_t)i * ld + j] = v;
    }
}

__device__ __forceinline__ double lane_double(double v, int lane) {   // v of lane `lane` (uniform)
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
    return __hiloint2double(hi, lo);
}

// Right-looking Cholesky of the pb x pb diagonal block held by one wave: lane i < pb owns row i
// in a[0..GPB) (lower part meaningful).  Column j (dpotf2's order): L_jj = sqrt(a_jj), L_ij =
// a_ij * (1/L_jj), then a_ik -= L_ij L_kj for j < k <= i.  The column goes through LDS (col[]:
// one write per lane, then every lane reads the whole column -- broadcast reads issued together)
// and the updates are selects, not branches.  rinv[j] = 1/L_jj.  False (uniformly) on a pivot
// that is not > 0 or NaN (LAPACK's info > 0).
__device__ __forceinline__ bool diag_factor(double (&a)[GPB], double (&rinv)[GPB], int i, int pb, double *col) {
#pragma unroll
    for (int j = 0; j < GPB; j++) {
        rinv[j] = 1.0;
        if (j < pb) {
            const double djj = lane_double(a[j], j);
            if (!(djj > 0.0)) return false;
            const double ljj = sqrt(djj);
            const double rj = 1.0 / ljj;
            rinv[j] = rj;
            const double lij = a[j] * rj;
            a[j] = (i == j) ? ljj : ((i > j) ? lij : a[j]);
            if (i < GPB) col[i] = a[j];
            wave_sync_lds();
            double lk[GPB];
#pragma unroll
            for (int k = j + 1; k < GPB; k++) lk[k] = col[k];
#pragma unroll
            for (int k = j + 1; k < GPB; k++) {
                const double upd = a[k] - a[j] * lk[k];
                a[k] = (i >= k && k < pb) ? upd : a[k];
            }
            wave_sync_lds();
        }
    }
    return true;
}

// Panel p0 (width pb).  Every workgroup of the matrix factors the diagonal block (wave 0, in
// registers) and solves its 256 rows below it (rows p0+pb .. n, row n = y^T),
// L21[r,:] = A21[r,:] L11^-T, right-looking with 1/L_jj (dtrsm's order); workgroup 0 leaves L11
// in Lpan (the SYRK launch copies it into A, so no workgroup of this launch can read a
// half-written diagonal block).
__global__ void __launch_bounds__(256) gpf_panel_kernel(double *__restrict__ A, int n, int p0, int pb,
                                                         int32_t *__restrict__ fail, double *__restrict__ Lpan) {
    const int b = blockIdx.y;
    if (fail[b]) return;
    const int ld = n + 1;
    double *Ab = A + (size_t)b * ld * ld;
    __shared__ double L[GPB][GPB + 1];
    __shared__ double Rv[GPB];
    __shared__ double col[GPB];
    __shared__ int bad;
    const int tid = threadIdx.x;
    if (tid < 64) {
        const int i = tid;
        double a[GPB], rv[GPB];
#pragma unroll
        for (int k = 0; k < GPB; k++) a[k] = (i < pb && k <= i) ? Ab[(size_t)(p0 + i) * ld + p0 + k] : 0.0;
        const bool ok = diag_factor(a, rv, i, pb, col);
        if (i == 0) bad = ok ? 0 : 1;
        if (ok && i < GPB) {
#pragma unroll
            for (int k = 0; k < GPB; k++) L[i][k] = (i < pb && k <= i) ? a[k] : 0.0;
            if (i == 0) {
#pragma unroll
                for (int k = 0; k < GPB; k++) Rv[k] = rv[k];
            }
        }
    }
    __syncthreads();
    if (bad) {
        if (tid == 0) fail[b] = 1;
        return;
    }
    if (blockIdx.x == 0)
        for (int t = tid; t < GPB * GPB; t += 256) Lpan[(size_t)b * GPB * GPB + t] = L[t / GPB][t % GPB];
    const int r = p0 + pb + blockIdx.x * 256 + tid;
    if (r > n) return;
    double x[GPB];
    double *row = Ab + (size_t)r * ld + p0;
#pragma unroll
    for (int k = 0; k < GPB; k++) x[k] = k < pb ? row[k] : 0.0;
#pragma unroll
    for (int j = 0; j < GPB; j++) {
        if (j < pb) {
            x[j] = x[j] * Rv[j];
#pragma unroll
            for (int k = j + 1; k < GPB; k++)
                if (k < pb) x[k] = x[k] - x[j] * L[k][j];
        }
    }
#pragma unroll
    for (int k = 0; k < GPB; k++)
        if (k < pb) row[k] = x[k];
}

// trailing update below panel p0: A[i][j] -= sum_k L[i][p0+k] L[j][p0+k] for q0 <= j <= i <= n
// (row n: the forward solve's update of y); workgroup = one 32x32 tile (ti >= tj), thread = 2x2
// outputs.  The extra block ntiles copies the panel's L11 into A.
__global__ void __launch_bounds__(256) gpf_syrk_kernel(double *__restrict__ A, int n, int p0, int pb,
                                                        const int32_t *__restrict__ fail,
                                                        const double *__restrict__ Lpan, int ntiles) {
    const int b = blockIdx.y;
    if (fail[b]) return;
    const int ld = n + 1;
    double *Ab = A + (size_t)b * ld * ld;
    if ((int)blockIdx.x == ntiles) {
        for (int t = threadIdx.x; t < pb * pb; t += 256) {
            const int i = t / pb, j = t % pb;
            if (j <= i) Ab[(size_t)(p0 + i) * ld + p0 + j] = Lpan[(size_t)b * GPB * GPB + i * GPB + j];
        }
        return;
    }
    const int q0 = p0 + pb;
    int ti = (int)((sqrt(8.0 * blockIdx.x + 1.0) - 1.0) / 2.0);
    while ((ti + 1) * (ti + 2) / 2 <= (int)blockIdx.x) ti++;
    while (ti * (ti + 1) / 2 > (int)blockIdx.x) ti--;
    const int tj = blockIdx.x - ti * (ti + 1) / 2;
    const int i0 = q0 + ti * 32, j0 = q0 + tj * 32;
    __shared__ double Li[32][GPB + 1], Lj[32][GPB + 1];
    const int tid = threadIdx.x;
    for (int t = tid; t < 32 * GPB; t += 256) {
        const int rr = t / GPB, k = t % GPB;
        Li[rr][k] = (i0 + rr <= n && k < pb) ? Ab[(size_t)(i0 + rr) * ld + p0 + k] : 0.0;
        Lj[rr][k] = (j0 + rr < n && k < pb) ? Ab[(size_t)(j0 + rr) * ld + p0 + k] : 0.0;
    }
    __syncthreads();
    const int ri = (tid / 16) * 2, rj = (tid % 16) * 2;
    double acc[2][2] = {{0.0, 0.0}, {0.0, 0.0}};
    for (int k = 0; k < pb; k++) {
        const double a0 = Li[ri][k], a1 = Li[ri + 1][k], b0 = Lj[rj][k], b1 = Lj[rj + 1][k];
        acc[0][0] = acc[0][0] + a0 * b0;
        acc[0][1] = acc[0][1] + a0 * b1;
        acc[1][0] = acc[1][0] + a1 * b0;
        acc[1][1] = acc[1][1] + a1 * b1;
    }
#pragma unroll
    for (int u = 0; u < 2; u++)
#pragma unroll
        for (int v = 0; v < 2; v++) {
            const int i = i0 + ri + u, j = j0 + rj + v;
            if (i <= n && j < n && j <= i) Ab[(size_t)i * ld + j] = Ab[(size_t)i * ld + j] - acc[u][v];
        }
}

__device__ __forceinline__ double block_sum(double v, double *red) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) red[wid] = v;
    __syncthreads();
    double s = 0.0;
    for (int w = 0; w < (int)(blockDim.x >> 6); w++) s = s + red[w];
    __syncthreads();
    return s;
}

// -LML = -(-0.5 * y.alpha - sum(log diag L) - (n/2) log 2pi) (models.py:318) with
// y.alpha = z.z (z = row n of the factor); +inf on a failed factorisation or NaN
__global__ void __launch_bounds__(256) gpf_lml_kernel(const double *__restrict__ A, int n,
                                                       const int32_t *__restrict__ fail, double *__restrict__ fval) {
    __shared__ double red[4];
    const int b = blockIdx.x;
    if (fail[b]) {
        if (threadIdx.x == 0) fval[b] = INFINITY;
        return;
    }
    const int ld = n + 1;
    const double *Ab = A + (size_t)b * ld * ld;
    double zz = 0.0, lg = 0.0;
    for (int i = threadIdx.x; i < n; i += 256) {
        const double z = Ab[(size_t)n * ld + i];
        zz = zz + z * z;
        lg = lg + log(Ab[(size_t)i * ld + i]);
    }
    const double ydot = block_sum(zz, red);
    const double slog = block_sum(lg, red);
    if (threadIdx.x == 0) {
        const double res = -(((-0.5 * ydot) - slog) - ((double)n / 2) * GPF_LOG_2PI);
        fval[b] = (res != res) ? INFINITY : res;
    }
}

// alpha = L^-T z (the second solve_triangular of _fit_gp_np / _predict's weights), 32-row blocks
// bottom-up: the block's L staged in LDS, wave 0 solves it in registers (alpha_j read from lane
// j), the workgroup updates the rows above.  The working vector lives in LDS up to GPF_LDS_ROWS
// rows and in the point's alpha_out row beyond (the same arithmetic; the rows grow by N+1-I per
// Parareal iteration, so long GParareal runs pass the LDS size -- the reference has no limit)
__global__ void __launch_bounds__(256) gpf_alpha_kernel(const double *__restrict__ A, int n,
                                                         const int32_t *__restrict__ fail,
                                                         double *__restrict__ alpha_out) {
    const int b = blockIdx.x;
    if (fail[b]) return;
    const int ld = n + 1;
    const double *Ab = A + (size_t)b * ld * ld;
    const int tid = threadIdx.x, lane = tid & 63;
    extern __shared__ double r_lds[];   // [n] when n <= GPF_LDS_ROWS
    double *r = (n <= GPF_LDS_ROWS) ? r_lds : alpha_out + (size_t)b * n;
    __shared__ double Lb[GPB][GPB + 1];
    for (int i = tid; i < n; i += 256) r[i] = Ab[(size_t)n * ld + i];
    __syncthreads();
    const int nblk = (n + GPB - 1) / GPB;
    for (int bk = nblk - 1; bk >= 0; bk--) {
        const int p0 = bk * GPB, pb = min(GPB, n - p0);
        for (int t = tid; t < GPB * GPB; t += 256) {
            const int i = t / GPB, j = t % GPB;
            Lb[i][j] = (i < pb && j <= i) ? Ab[(size_t)(p0 + i) * ld + p0 + j] : 0.0;
        }
        __syncthreads();
        if (tid < 64) {
            double v = lane < pb ? r[p0 + lane] : 0.0;
#pragma unroll
            for (int j = GPB - 1; j >= 0; j--) {
                if (j < pb) {
                    const double aj = lane_double(v, j) / Lb[j][j];
                    if (lane == j) v = aj;
                    if (lane < j) v = v - Lb[j][lane] * aj;
                }
            }
            if (lane < pb) r[p0 + lane] = v;
        }
        __syncthreads();
        for (int i = tid; i < p0; i += 256) {   // rows above: r_i -= sum_k L[p0+k][i] alpha_k
            double s = r[i];
            for (int k = 0; k < pb; k++) s = s - Ab[(size_t)(p0 + k) * ld + i] * r[p0 + k];
            r[i] = s;
        }
        __syncthreads();
    }
    if (n <= GPF_LDS_ROWS)
        for (int i = tid; i < n; i += 256) alpha_out[(size_t)b * n + i] = r[i];
}

// posterior mean of every coordinate j at one query q (models.py:456-462 -> _predict :441-453):
// K_star = sigma_y^2 exp(c * cdist(x, q)); mean = K_star . alpha_j; out[j] = mean + bias[j]
__global__ void __launch_bounds__(256) gpf_mean_kernel(const double *__restrict__ X, int n, int d,
                                                        const double *__restrict__ q,
                                                        const double *__restrict__ coef,
                                                        const double *__restrict__ alpha,
                                                        const double *__restrict__ bias, double *__restrict__ out) {
    __shared__ double red[4];
    const int j = blockIdx.x;
    const double c = coef[2 * j], psy = coef[2 * j + 1];
    double acc = 0.0;
    for (int i = threadIdx.x; i < n; i += 256) {
        double dist = 0.0;
        for (int k = 0; k < d; k++) {
            const double t = X[(size_t)i * d + k] - q[k];
            dist = dist + t * t;
        }
        acc = acc + (psy * exp(c * dist)) * alpha[(size_t)j * n + i];
    }
    const double mean = block_sum(acc, red);
    if (threadIdx.x == 0) out[j] = bias ? mean + bias[j] : mean;
}

int gpfull_mean(const double *X, int64_t rows, int d, const double *q, const double *coef, const double *alpha,
                const double *bias, double *out, hipStream_t st) {
    hipLaunchKernelGGL(gpf_mean_kernel, dim3(d), dim3(256), 0, st, X, (int)rows, d, q, coef, alpha, bias, out);
    NNGP_LAUNCH_CHECK();
    return NNGP_OK;
}

// The batched -LML pipeline for nb points (device pts), D2 [n][n] given; A: nb*(n+1)^2 scratch.
static int gpf_eval(const double *D2, int n, const double *Y, int d, const GPPoint *pts, int nb, double *A,
                    int32_t *fail, double *fval, double *alpha_out, double *Lpan, hipStream_t st) {
    NNGP_HIP_CHECK(hipMemsetAsync(fail, 0, sizeof(int32_t) * nb, st));
    const size_t cnt = (size_t)n * n + n;
    const unsigned bx = (unsigned)std::min<size_t>((cnt + 255) / 256, 1024);
    hipLaunchKernelGGL(gpf_build_kernel, dim3(bx, nb), dim3(256), 0, st, D2, n, Y, d, pts, A, fail);
    NNGP_LAUNCH_CHECK();
    for (int p0 = 0; p0 < n; p0 += GPB) {
        const int pb = std::min(GPB, n - p0);
        const int below = n + 1 - p0 - pb;   // includes row n (y)
        const unsigned chunks = (unsigned)std::max(1, (below + 255) / 256);
        hipLaunchKernelGGL(gpf_panel_kernel, dim3(chunks, nb), dim3(256), 0, st, A, n, p0, pb, fail, Lpan);
        NNGP_LAUNCH_CHECK();
        const int nt = (below + 31) / 32, ntiles = nt * (nt + 1) / 2;
        hipLaunchKernelGGL(gpf_syrk_kernel, dim3((unsigned)(ntiles + 1), nb), dim3(256), 0, st, A, n, p0, pb, fail,
                           Lpan, ntiles);
        NNGP_LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(gpf_lml_kernel, dim3(nb), dim3(256), 0, st, A, n, fail, fval);
    NNGP_LAUNCH_CHECK();
    if (alpha_out) {
        hipLaunchKernelGGL(gpf_alpha_kernel, dim3(nb), dim3(256), n <= GPF_LDS_ROWS ? sizeof(double) * n : 0, st, A,
                           n, fail, alpha_out);
        NNGP_LAUNCH_CHECK();
    }
    return NNGP_OK;
}

static GPPoint gp_point(double sx, double sy, double jexp, int coord) {
    GPPoint p;
    p.c = -0.5 * (1 / (sx * sx));   // -0.5 * (1/(sigma_x**2))
    p.psy = sy * sy;                // sigma_y**2
    p.jp = pow(10.0, jexp);         // 10**jitter
    p.coord = coord;
    p.pad = 0;
    return p;
}

struct GPFWork {   // device buffers of one call
    double *D2, *A, *fval, *Lpan;
    GPPoint *pts;
    int32_t *fail;
};

static int gpf_workspace(int n, int nb, GPFWork &w) {
    int err = 0;
    const size_t nn = (size_t)n * n, mm = (size_t)(n + 1) * (n + 1);
    const size_t bytes = sizeof(double) * (nn + (size_t)nb * mm + nb + (size_t)nb * GPB * GPB) + sizeof(GPPoint) * nb +
                         sizeof(int32_t) * nb + 64;
    char *p = (char *)workspace(bytes, &err, 3);
    if (err) return err;
    w.D2 = (double *)p;
    w.A = w.D2 + nn;
    w.fval = w.A + (size_t)nb * mm;
    w.Lpan = w.fval + nb;
    w.pts = (GPPoint *)(w.Lpan + (size_t)nb * GPB * GPB);
    w.fail = (int32_t *)(w.pts + nb);
    return NNGP_OK;
}

static int gpf_check(int64_t rows, int d, int n_fit) {
    NNGP_REQUIRE(rows >= 1 && rows <= (int64_t)1 << 30, "full GP needs 1 <= rows (got %lld)", (long long)rows);
    NNGP_REQUIRE(d >= 1 && n_fit >= 1, "bad d / fit count");
    return NNGP_OK;
}

// points per batch: all fits, capped so the factor scratch stays under ~8 GB
static int gpf_batch_cap(int n, int n_fit) {
    const size_t per = sizeof(double) * (size_t)(n + 1) * (n + 1);
    const size_t cap = std::max<size_t>(1, ((size_t)8 << 30) / per);
    return (int)std::min<size_t>(cap, (size_t)n_fit);
}

}  // namespace nngp

using namespace nngp;

extern "C" int nngp_gpfull_lml(const double *X, int64_t rows, int d, const double *Y, int n_pts,
                               const int32_t *coord, const double *jitter_exp, const double *theta,
                               double *fval_out, double *alpha_out, void *stream) {
    NNGP_REQUIRE(X && Y && coord && jitter_exp && theta && fval_out, "null argument");
    int rc = gpf_check(rows, d, n_pts);
    if (rc) return rc;
    hipStream_t st = (hipStream_t)stream;
    const int n = (int)rows, nbc = gpf_batch_cap(n, n_pts);
    GPFWork w;
    rc = gpf_workspace(n, nbc, w);
    if (rc) return rc;
    hipLaunchKernelGGL(gpf_d2_kernel, dim3((n + 15) / 16, (n + 15) / 16), dim3(16, 16), 0, st, X, n, d, w.D2);
    NNGP_LAUNCH_CHECK();
    std::vector<GPPoint> hp((size_t)n_pts);
    for (int i = 0; i < n_pts; i++) {
        NNGP_REQUIRE(coord[i] >= 0 && coord[i] < d, "coordinate %d out of range", coord[i]);
        hp[i] = gp_point(theta[2 * i], theta[2 * i + 1], jitter_exp[i], coord[i]);
    }
    std::vector<double> hf((size_t)n_pts);
    for (int s = 0; s < n_pts; s += nbc) {
        const int nb = std::min(nbc, n_pts - s);
        NNGP_HIP_CHECK(hipMemcpyAsync(w.pts, hp.data() + s, sizeof(GPPoint) * nb, hipMemcpyHostToDevice, st));
        rc = gpf_eval(w.D2, n, Y, d, w.pts, nb, w.A, w.fail, w.fval, alpha_out ? alpha_out + (size_t)s * n : nullptr,
                      w.Lpan, st);
        if (rc) return rc;
        NNGP_HIP_CHECK(hipMemcpyAsync(hf.data() + s, w.fval, sizeof(double) * nb, hipMemcpyDeviceToHost, st));
    }
    NNGP_HIP_CHECK(hipStreamSynchronize(st));
    for (int i = 0; i < n_pts; i++) fval_out[i] = hf[i];
    return NNGP_OK;
}

extern "C" int nngp_gpfull_fit(const double *X, int64_t rows, int d, const double *Y, int n_fit,
                               const int32_t *coord, const double *jitter_exp, const double *theta0,
                               double fatol, double xatol, int maxfev, double *theta_out, double *fval_out,
                               int32_t *nfev_out, int32_t *rounds_out, void *stream) {
    NNGP_REQUIRE(X && Y && coord && jitter_exp && theta0 && theta_out && fval_out, "null argument");
    int rc = gpf_check(rows, d, n_fit);
    if (rc) return rc;
    NNGP_REQUIRE(maxfev >= 1, "maxfev must be >= 1");
    hipStream_t st = (hipStream_t)stream;
    const int n = (int)rows, nbc = gpf_batch_cap(n, n_fit);
    GPFWork w;
    rc = gpf_workspace(n, nbc, w);
    if (rc) return rc;
    hipLaunchKernelGGL(gpf_d2_kernel, dim3((n + 15) / 16, (n + 15) / 16), dim3(16, 16), 0, st, X, n, d, w.D2);
    NNGP_LAUNCH_CHECK();
    const NMCfg cfg{fatol, xatol, maxfev, maxfev};   // maxiter = maxfev = 200*N (scipy defaults)
    std::vector<NM> S((size_t)n_fit);
    for (int f = 0; f < n_fit; f++) {
        NNGP_REQUIRE(coord[f] >= 0 && coord[f] < d, "coordinate %d out of range", coord[f]);
        S[f].f0 = S[f].f1 = S[f].f2 = INFINITY;
        S[f].xbx = S[f].xby = S[f].xrx = S[f].xry = S[f].fxr = 0.0;
        nm_start(S[f], cfg, theta0[2 * f], theta0[2 * f + 1]);
    }
    std::vector<GPPoint> hp;
    std::vector<int> who;
    std::vector<double> hf;
    int rounds = 0;
    for (;;) {
        hp.clear();
        who.clear();
        for (int f = 0; f < n_fit; f++)
            if (S[f].st != ST_DONE) {
                hp.push_back(gp_point(S[f].px, S[f].py, jitter_exp[f], coord[f]));
                who.push_back(f);
            }
        if (hp.empty()) break;
        rounds++;
        const int np = (int)hp.size();
        hf.resize((size_t)np);
        for (int s = 0; s < np; s += nbc) {
            const int nb = std::min(nbc, np - s);
            NNGP_HIP_CHECK(hipMemcpyAsync(w.pts, hp.data() + s, sizeof(GPPoint) * nb, hipMemcpyHostToDevice, st));
            rc = gpf_eval(w.D2, n, Y, d, w.pts, nb, w.A, w.fail, w.fval, nullptr, w.Lpan, st);
            if (rc) return rc;
            NNGP_HIP_CHECK(hipMemcpyAsync(hf.data() + s, w.fval, sizeof(double) * nb, hipMemcpyDeviceToHost, st));
        }
        NNGP_HIP_CHECK(hipStreamSynchronize(st));
        for (int q = 0; q < np; q++) nm_consume(S[who[q]], cfg, hf[q]);
    }
    for (int f = 0; f < n_fit; f++) {
        theta_out[2 * f] = S[f].s0x;
        theta_out[2 * f + 1] = S[f].s0y;
        fval_out[f] = S[f].f0;
        if (nfev_out) nfev_out[f] = S[f].fcalls;
    }
    if (rounds_out) *rounds_out = rounds;
    return NNGP_OK;
}

extern "C" int nngp_gpfull_mean(const double *X, int64_t rows, int d, const double *q, const double *coef,
                                const double *alpha, const double *bias, double *out, void *stream) {
    NNGP_REQUIRE(X && q && coef && alpha && out, "null argument");
    NNGP_REQUIRE(rows >= 1 && d >= 1, "bad rows / d");
    return gpfull_mean(X, rows, d, q, coef, alpha, bias, out, (hipStream_t)stream);
}
