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
//   gpf_diag_kernel    blocked right-looking Cholesky, panel j: one wave per two matrices factors
//                      their 32x32 diagonal blocks in registers (dpotf2 order)
//   gpf_rows_kernel    each thread solves one row below the diagonal block
//   gpf_update_kernel  trailing update A22 -= L21 L21^T, 64x64 lower tiles, LDS-staged panels, on
//                      the FP64 matrix cores (v_mfma_f64_16x16x4_f64)
//   gpf_lml_kernel     -LML = 0.5 z.z + sum log L_ii + (n/2) log 2pi
//   gpf_alpha_kernel   alpha = L^-T z for the posterior weights (once per fit() per coordinate)
// The trailing update runs on the FP64 MFMA (same peak rate as the VALU, but operands come from
// registers: two LDS reads per 1 024 multiply-adds instead of one per FMA).  The arithmetic order
// of LAPACK's blocked potrf is not reproduced (it is third-party and build-dependent); parity is
// to tolerance (tests/test_gpu_gpfull.py).
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
// gpf_diag_kernel (two 32x32 blocks per wave, col[32*h+i]), the FULL staging (tid>>5, tid&31) and
// gpf_update_tile (kq/SU) are written for 32-column panels
static_assert(GPB == 32, "the full-GP kernels assume 32-column panels");
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
// Workgroup = GPF_BROWS consecutive rows of one matrix (blockIdx.y), its threads over each row's
// lower-triangle columns j <= i only (a grid-stride loop over all n^2 entries left half of its
// threads on the upper triangle and divided by n per entry); the block past the last row writes y.
static constexpr int GPF_BROWS = 8;
__global__ void __launch_bounds__(256) gpf_build_kernel(const double *__restrict__ D2, int n,
                                                        const double *__restrict__ Y, int d,
                                                        const GPPoint *__restrict__ pts, double *__restrict__ A,
                                                        const int32_t *__restrict__ fail) {
    const int b = blockIdx.y;
    if (fail[b]) return;
    const GPPoint p = pts[b];
    const int ld = n + 1;
    double *Ab = A + (size_t)b * ld * ld;
    const int r0 = blockIdx.x * GPF_BROWS;
    if (r0 >= n) {   // row n: the training column
        for (int j = threadIdx.x; j < n; j += 256) Ab[(size_t)n * ld + j] = Y[(size_t)j * d + p.coord];
        return;
    }
    for (int i = r0; i < min(r0 + GPF_BROWS, n); i++) {
        const double *drow = D2 + (size_t)i * n;
        double *arow = Ab + (size_t)i * ld;
        for (int j = threadIdx.x; j <= i; j += 256) {
            double v = p.psy * exp(p.c * drow[j]);
            if (i == j) v = v + p.jp;
            arow[j] = v;
        }
    }
}

__device__ __forceinline__ double lane_double(double v, int lane) {   // v of lane `lane` (uniform)
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
    return __hiloint2double(hi, lo);
}

// Right-looking Cholesky of the pb x pb diagonal blocks of TWO matrices held by one wave: lane
// 32h + i owns row i of matrix h in a[0..GPB) (lower part meaningful).  Column j (dpotf2's
// order): L_jj = sqrt(a_jj), L_ij = a_ij * (1/L_jj), then a_ik -= L_ij L_kj for j < k <= i.  The
// column goes through LDS (col[32h + i]: one write per lane, then every lane reads its half's
// column -- broadcast reads issued together) and the updates are selects, not branches.
// rinv[j] = 1/L_jj.  bad: this half met a pivot that is not > 0 or NaN (LAPACK's info > 0); its
// later columns then compute garbage that nobody reads.  (One matrix per wave left lanes 32-63
// idle and put 1 152 matrices on 1 024 SIMDs, two waves on some: the launch took two waves' time.)
__device__ __forceinline__ void diag_factor(double (&a)[GPB], double (&rinv)[GPB], int i, int h, int pb,
                                            double *col, bool &bad) {
    bad = false;
#pragma unroll
    for (int j = 0; j < GPB; j++) {
        rinv[j] = 1.0;
        if (j < pb) {
            const double d0 = lane_double(a[j], j), d1 = lane_double(a[j], 32 + j);
            const double djj = h ? d1 : d0;
            bad = bad || !(djj > 0.0);
            const double ljj = sqrt(djj);
            const double rj = 1.0 / ljj;
            rinv[j] = rj;
            const double lij = a[j] * rj;
            a[j] = (i == j) ? ljj : ((i > j) ? lij : a[j]);
            col[32 * h + i] = a[j];
            wave_sync_lds();
            double lk[GPB];
#pragma unroll
            for (int k = j + 1; k < GPB; k++) lk[k] = col[32 * h + k];
#pragma unroll
            for (int k = j + 1; k < GPB; k++) {
                const double upd = a[k] - a[j] * lk[k];
                a[k] = (i >= k && k < pb) ? upd : a[k];
            }
            wave_sync_lds();
        }
    }
}

// Panel p0 (width pb), in two launches.
// gpf_diag_kernel: one wave per TWO matrices factors their diagonal blocks in registers (diag_factor) and
// leaves L11 and 1/L_jj in Lpan[b] = [L11 (GPB x GPB, lower) | rinv (GPB)]; fail[b] on a failed
// pivot.  (Round 3 factored it in every row-solve workgroup of the matrix, and the factor's ~190
// VGPRs held the whole row-solve launch at two waves per SIMD: 118 us per panel at n = 753 with
// 1 152 matrices, profiles/r04/gparareal_burgers_kernel_stats.csv.)
// gpf_rows_kernel: every workgroup (one wave) stages its 64 rows below the block (rows p0+pb .. n,
// row n = y^T) through LDS -- coalesced, a row's 32 doubles by consecutive lanes (one thread per
// row reading its own row touched 64 cache lines per load instruction: 107 us per panel) -- and
// solves L21[r,:] = A21[r,:] L11^-T, right-looking with 1/L_jj (dtrsm's order), L11 broadcast
// from LDS (as wave-uniform scalar loads its 528 values spilled 920 SGPRs).  The update launch copies L11 into A, so no workgroup reads a half-written diagonal
// block.
static constexpr int LPS = GPB * GPB + GPB;   // Lpan doubles per matrix

__global__ void __launch_bounds__(64) gpf_diag_kernel(const double *__restrict__ A, int n, int p0, int pb, int nmat,
                                                       int32_t *__restrict__ fail, double *__restrict__ Lpan) {
    const int h = threadIdx.x >> 5, i = threadIdx.x & 31;
    const int b = 2 * blockIdx.x + h;
    const bool act = b < nmat && !fail[b];   // half-uniform; an idle half runs along on zeros
    const int ld = n + 1;
    const double *Ab = A + (size_t)(act ? b : 0) * ld * ld;
    __shared__ double col[2 * GPB];
    double a[GPB], rv[GPB];
#pragma unroll
    for (int k = 0; k < GPB; k++) a[k] = (act && i < pb && k <= i) ? Ab[(size_t)(p0 + i) * ld + p0 + k] : 0.0;
    bool bad;
    diag_factor(a, rv, i, h, pb, col, bad);
    if (!act) return;
    if (bad) {
        if (i == 0) fail[b] = 1;
        return;
    }
    double *Lb = Lpan + (size_t)b * LPS;
#pragma unroll
    for (int k = 0; k < GPB; k++) Lb[i * GPB + k] = (i < pb && k <= i) ? a[k] : 0.0;
    if (i == 0) {
#pragma unroll
        for (int k = 0; k < GPB; k++) Lb[GPB * GPB + k] = rv[k];
    }
}

template <bool FULL>   // FULL: pb == GPB (every panel but a short last one) -- no per-column tests
__global__ void __launch_bounds__(64) gpf_rows_kernel(double *__restrict__ A, int n, int p0, int pb,
                                                       const int32_t *__restrict__ fail,
                                                       const double *__restrict__ Lpan) {
    const int b = blockIdx.y;
    if (fail[b]) return;
    const int ld = n + 1;
    double *Ab = A + (size_t)b * ld * ld;
    __shared__ double L[GPB * GPB + GPB];   // L11 | 1/L_jj (Lpan's layout)
    __shared__ double X[64][GPB + 1];       // this wave's 64 rows of the panel, staged coalesced
    const int tid = threadIdx.x;
    const double *Lsrc = Lpan + (size_t)b * LPS;
    const int r0 = p0 + pb + blockIdx.x * 64;
    {   // every load issued before the first LDS write (rolled, one HBM round trip per 64 doubles)
        constexpr int LU = (LPS + 63) / 64;
        double lv[LU], xv[GPB];
#pragma unroll
        for (int u = 0; u < LU; u++) lv[u] = (tid + 64 * u < LPS) ? Lsrc[tid + 64 * u] : 0.0;
#pragma unroll
        for (int u = 0; u < GPB; u++) {   // consecutive lanes read consecutive columns of a row
            const int t = tid + 64 * u, rr = t / GPB, k = t % GPB;
            xv[u] = (r0 + rr <= n && (FULL || k < pb)) ? Ab[(size_t)(r0 + rr) * ld + p0 + k] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < LU; u++)
            if (tid + 64 * u < LPS) L[tid + 64 * u] = lv[u];
#pragma unroll
        for (int u = 0; u < GPB; u++) {
            const int t = tid + 64 * u;
            X[t / GPB][t % GPB] = xv[u];
        }
    }
    const double *Lb = L;
    __syncthreads();
    double x[GPB];
#pragma unroll
    for (int k = 0; k < GPB; k++) x[k] = X[tid][k];
#pragma unroll
    for (int j = 0; j < GPB; j++) {
        if (FULL || j < pb) {
            x[j] = x[j] * Lb[GPB * GPB + j];
#pragma unroll
            for (int k = j + 1; k < GPB; k++)
                if (FULL || k < pb) x[k] = x[k] - x[j] * Lb[k * GPB + j];
        }
    }
#pragma unroll
    for (int k = 0; k < GPB; k++) X[tid][k] = x[k];
    __syncthreads();
#pragma unroll
    for (int u = 0; u < GPB; u++) {
        const int t = tid + 64 * u, rr = t / GPB, k = t % GPB;
        if (r0 + rr <= n && (FULL || k < pb)) Ab[(size_t)(r0 + rr) * ld + p0 + k] = X[rr][k];
    }
}

// Trailing update A[i][j] -= sum_{k < pb} L[i][p0+k] L[j][p0+k] (the factored panel's L columns)
// over rows q0 <= i <= n (row n: the forward solve's update of y), columns q0 <= j < n, j <= i.
// Workgroup = one 64x64 tile of the region's lower triangle (4 waves); the extra block `ntiles`
// copies the L11 that Lpan holds into A.  The lane's 16 elements of A are loaded first, so their
// HBM latency overlaps the rest; the tile's 64 + 64 panel rows are staged through LDS (row stride
// GPB + 2 doubles: the 16 rows x 4 k of one MFMA operand read fall on distinct banks in each
// 32-lane half), every load issued before the first LDS write; wave w multiplies its 16 rows by
// the tile's 4 column blocks on the FP64 matrix cores (v_mfma_f64_16x16x4_f64: A[l&15][k + (l>>4)]
// / B[k + (l>>4)][l&15] per lane; D col = l&15, row = (l>>4) + 4 reg).  Blocks j > i of a diagonal
// tile are skipped.  Workgroups go round-robin over the 8 XCDs by linear id; the k-th workgroup of
// XCD x takes matrix x + 8 (k / T), tile k % T (T = ntiles + 1, grid y padded to a multiple of 8),
// so every tile of a matrix shares one L2.
// Measured at Burgers N = 128 (profiles/r04/gparareal_burgers_r4*.txt): a rolled staging loop
// (one HBM round trip per 256 elements) cost 25 %; two-panel look-ahead updates (64 L columns per
// pass, half the trailing matrix's read-modify-write stream) were 5-30 % slower in every register
// budget tried (the extra staging registers cost a wave per SIMD or spilled), so one panel per pass.
// The accumulation order inside an MFMA k-step is the hardware's; GParareal's parity is to
// tolerance and K (tests/test_gpu_gpfull.py), as LAPACK's blocked order is not reproduced anyway.
typedef double f64x4 __attribute__((ext_vector_type(4)));
static constexpr int GPF_TM = 64;              // update tile
static constexpr int GPF_US = GPB + 2;         // LDS row stride of the staged panel rows

template <bool FULL>
__device__ __forceinline__ void gpf_update_tile(double *__restrict__ Ab, int ld, int n, int p0, int pb, int i0,
                                                int j0, bool diag, double *Li, double *Lj) {
    const int tid = threadIdx.x;
    const int w = tid >> 6, lane = tid & 63;
    const int kq = lane >> 4, ra = 16 * w + (lane & 15);
    const int ncb = FULL ? 4 : (diag ? w + 1 : 4);   // column blocks at or left of the diagonal
    // this lane's 16 elements of A: rows i0 + 16w + kq + 4r, columns j0 + 16cb + (lane & 15)
    double *arow = Ab + (size_t)(i0 + 16 * w + kq) * ld + j0 + (lane & 15);
    double old[4][4];
#pragma unroll
    for (int r = 0; r < 4; r++) {
#pragma unroll
        for (int cb = 0; cb < 4; cb++) {
            if constexpr (FULL) {
                old[cb][r] = arow[(size_t)(4 * r) * ld + 16 * cb];
            } else {
                const int i = i0 + 16 * w + kq + 4 * r, j = j0 + 16 * cb + (lane & 15);
                old[cb][r] = (cb < ncb && i <= n && j < n && j <= i) ? Ab[(size_t)i * ld + j] : 0.0;
            }
        }
    }
    constexpr int SU = GPF_TM * GPB / 256;   // consecutive lanes: consecutive k of a row
    double vi[SU], vj[SU];
    if constexpr (FULL) {   // thread: rows tid/32 + 8u, column tid%32 of the panel
        const double *pi = Ab + (size_t)(i0 + (tid >> 5)) * ld + p0 + (tid & 31);
        const double *pj = Ab + (size_t)(j0 + (tid >> 5)) * ld + p0 + (tid & 31);
#pragma unroll
        for (int u = 0; u < SU; u++) {
            vi[u] = pi[(size_t)(8 * u) * ld];
            vj[u] = pj[(size_t)(8 * u) * ld];
        }
    } else {
#pragma unroll
        for (int u = 0; u < SU; u++) {
            const int t = tid + 256 * u, rr = t / GPB, k = t % GPB;
            vi[u] = (i0 + rr <= n && k < pb) ? Ab[(size_t)(i0 + rr) * ld + p0 + k] : 0.0;
            vj[u] = (j0 + rr < n && k < pb) ? Ab[(size_t)(j0 + rr) * ld + p0 + k] : 0.0;
        }
    }
#pragma unroll
    for (int u = 0; u < SU; u++) {
        const int t = tid + 256 * u, rr = t / GPB, k = t % GPB;
        Li[rr * GPF_US + k] = vi[u];
        Lj[rr * GPF_US + k] = vj[u];
    }
    __syncthreads();
    const int kend = FULL ? GPB : (pb + 3) & ~3;   // the zero padding past pb adds exact zeros
    f64x4 acc[4];
#pragma unroll
    for (int cb = 0; cb < 4; cb++) acc[cb] = f64x4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int k = 0; k < GPB; k += 4) {
        if (k >= kend) break;
        const double av = Li[ra * GPF_US + k + kq];
#pragma unroll
        for (int cb = 0; cb < 4; cb++)
            if (cb < ncb)
                acc[cb] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, Lj[(16 * cb + (lane & 15)) * GPF_US + k + kq],
                                                               acc[cb], 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 4; r++) {
#pragma unroll
        for (int cb = 0; cb < 4; cb++) {
            if constexpr (FULL) {
                arow[(size_t)(4 * r) * ld + 16 * cb] = old[cb][r] - acc[cb][r];
            } else {
                if (cb >= ncb) continue;
                const int i = i0 + 16 * w + kq + 4 * r, j = j0 + 16 * cb + (lane & 15);
                if (i <= n && j < n && j <= i) Ab[(size_t)i * ld + j] = old[cb][r] - acc[cb][r];
            }
        }
    }
}

__global__ void __launch_bounds__(256, 3) gpf_update_kernel(double *__restrict__ A, int n, int p0, int pb,
                                                             const int32_t *__restrict__ fail,
                                                             const double *__restrict__ Lpan, int ntiles, int nmat) {
    const int T = ntiles + 1;
    const int lin = blockIdx.x + blockIdx.y * T;
    const int kx = lin >> 3;
    const int b = (lin & 7) + 8 * (kx / T);
    const int tile = kx % T;
    if (b >= nmat || fail[b]) return;
    const int ld = n + 1;
    double *Ab = A + (size_t)b * ld * ld;
    if (tile == ntiles) {
        for (int t = threadIdx.x; t < pb * pb; t += 256) {
            const int i = t / pb, j = t % pb;
            if (j <= i) Ab[(size_t)(p0 + i) * ld + p0 + j] = Lpan[(size_t)b * LPS + i * GPB + j];
        }
        return;
    }
    int ti = (int)((sqrt(8.0 * tile + 1.0) - 1.0) / 2.0);
    while ((ti + 1) * (ti + 2) / 2 <= tile) ti++;
    while (ti * (ti + 1) / 2 > tile) ti--;
    const int tj = tile - ti * (ti + 1) / 2;
    const int q0 = p0 + pb;
    const int i0 = q0 + ti * GPF_TM, j0 = q0 + tj * GPF_TM;
    // an off-diagonal tile inside the matrix with a full panel (most of them): no guards, and
    // row pointers with the column blocks as immediate offsets (the guarded form spent ~1 000
    // VALU per wave on index arithmetic, issue-stalling 39 % of its cycles beside 27 % active,
    // profiles/r04/pmc_gpf_update_r4af.txt)
    __shared__ double Li[GPF_TM * GPF_US], Lj[GPF_TM * GPF_US];
    if (ti != tj && i0 + GPF_TM - 1 <= n && j0 + GPF_TM <= n && pb == GPB)
        gpf_update_tile<true>(Ab, ld, n, p0, pb, i0, j0, false, Li, Lj);
    else
        gpf_update_tile<false>(Ab, ld, n, p0, pb, i0, j0, ti == tj, Li, Lj);
}

// ---------------------------------------------------------------------------------------------
// Left-looking order on 64-column panels (round 6, the default; NNGP_GPF_ORDER=1 keeps the
// right-looking 32-column order above).  Per panel c0 (width pb = min(64, n - c0)):
//   gpf_ll_gemm_kernel  A[c0..n][c0..c0+pb) -= L[c0..n][0..c0) L[c0..c0+pb)[0..c0)^T: one 64-row
//                       tile per workgroup, the whole k = 0..c0 sum accumulated on the FP64 matrix
//                       cores and subtracted once (OpenBLAS's potrf also subtracts a K-block's
//                       register-accumulated product at once).  Row n = y^T rides along: its
//                       update is the forward solve's z_j -= sum_k z_k L_jk.
//   gpf_ll_diag_kernel  one wave factors the 64x64 diagonal block (lane i = row i), L11 and 1/L_jj
//                       into Lpan (column-major, so the lanes' stores coalesce)
//   gpf_ll_rows_kernel  the rows below: x L11^T = a by substitution, one lane per row, 256 rows per
//                       workgroup sharing one LDS copy of L11; its first workgroup also writes L11
//                       into A
// Why: the right-looking 32-column update re-reads and re-writes the whole trailing matrix per
// panel (4 flop/B, HBM-bound at ~52 % of HBM); the left-looking panel GEMM reads
// each L row once per panel and writes only the panel (nb/4 = 16 flop/B), and the chain per
// Nelder-Mead round has 3 launches per 64 columns instead of per 32.
static constexpr int LB = 64;                // panel width
static constexpr int LPS64 = LB * LB + LB;   // Lpan doubles per matrix: L11 column-major | 1/L_jj
static constexpr int LKC = 32;               // k chunk of the panel GEMM (c0 is a multiple: no tail; 64 measured slower: 68 KB of LDS and 237 VGPRs left 2 workgroups per CU instead of 3)
static constexpr int LKS = LKC + 2;          // its LDS row stride (the gpf_update_tile operand pattern)

// (matrix, tile) of linear workgroup `lin`: workgroups go round-robin over the 8 XCDs, the k-th of
// XCD x takes matrix x + 8 (k / T), tile k % T -- a matrix's tiles share one L2 (grid y padded to 8)
__device__ __forceinline__ void gpf_xcd_map(int lin, int T, int &b, int &t) {
    const int kx = lin >> 3;
    b = (lin & 7) + 8 * (kx / T);
    t = kx % T;
}

// The point's original matrix entry, computed where the left-looking order first reads it (each
// column block exactly once: the panel GEMM's epilogue, or panel 0's factor and row solve) instead
// of built in HBM beforehand: gpf_build_kernel's expression (kernel_np, models.py:302-304, + 10^jitter
// on the diagonal), row n = y.  At Burgers N = 128 sizes the build kernel wrote 2.6 GB per round and
// the factor read it back.  r, c must be inside the matrix (callers clamp).
__device__ __forceinline__ double gpf_entry(const double *__restrict__ D2, int n, const double *__restrict__ Y, int d,
                                            const GPPoint &p, int r, int c) {
    const double dv = D2[(unsigned)(min(r, n - 1) * n + c)];   // both loads unconditional (no branch per entry)
    const double yv = Y[(unsigned)(c * d + p.coord)];
    double v = p.psy * exp(p.c * dv);
    v = (r == c) ? v + p.jp : v;
    return (r == n) ? yv : v;
}

// Every guarded access below loads from a clamped (valid) address and selects zero afterwards:
// a load under a lane condition compiles to a branch with its own wait, and a row solve whose 65
// loads were serialised that way took ~90 us per workgroup (profiles/r06/gparareal).
// FULL: the tile's 64 rows exist and pb == LB -- no guards.  DIAG: tile 0 (its B rows are its own A
// rows; only j <= i is stored).  Both compile-time, and every MFMA block and original entry is
// computed for every tile (the diagonal tile's upper blocks are wasted work): a branch around the
// MFMAs or the loads made the compiler wait for the next chunk's prefetch before the MFMAs.
template <bool FULL, bool DIAG>
__device__ __forceinline__ void gpf_ll_gemm_tile(double *__restrict__ Ab, int ld, int n, int c0, int pb, int r0,
                                                 double *Sa, double *Sb, double *Xd,
                                                 const double *__restrict__ D2, const double *__restrict__ Y, int d,
                                                 const GPPoint &pt) {
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const int kq = lane >> 4, cl = lane & 15;
    constexpr int SU = LB * LKC / 256;        // staged doubles per thread and operand
    const int sr = tid / LKC, sk = tid % LKC; // staging: rows sr + (256 / LKC) u, column sk of the chunk
    constexpr int RS = 256 / LKC;
    double *SB = DIAG ? Sa : Sb;              // the diagonal tile's B rows are its own A rows
    double va[SU], vb[SU];
#define GPF_LL_LOAD(kk)                                                                                  \
    _Pragma("unroll") for (int u = 0; u < SU; u++) {                                                   \
        const int rr = sr + RS * u;                                                                    \
        const int ra = FULL ? r0 + rr : min(r0 + rr, n), rb = FULL ? rr : min(rr, pb - 1);             \
        const double x = Ab[(unsigned)(ra * ld + (kk) + sk)];                                          \
        const double y = DIAG ? 0.0 : Ab[(unsigned)((c0 + rb) * ld + (kk) + sk)];                      \
        va[u] = (FULL || r0 + rr <= n) ? x : 0.0;                                                      \
        vb[u] = (FULL || rr < pb) ? y : 0.0;                                                           \
    }
    f64x4 acc[4];
#pragma unroll
    for (int cb = 0; cb < 4; cb++) acc[cb] = f64x4{0.0, 0.0, 0.0, 0.0};
    GPF_LL_LOAD(0)
    for (int kk = 0; kk < c0; kk += LKC) {
        __syncthreads();                      // the previous chunk's operand reads are done
#pragma unroll
        for (int u = 0; u < SU; u++) {
            Sa[(sr + RS * u) * LKS + sk] = va[u];
            if constexpr (!DIAG) Sb[(sr + RS * u) * LKS + sk] = vb[u];
        }
        __syncthreads();
        if (kk + LKC < c0) {                  // the next chunk's loads fly under this chunk's MFMAs
            GPF_LL_LOAD(kk + LKC)
        }
#pragma unroll
        for (int k = 0; k < LKC; k += 4) {
            const double av = Sa[(16 * w + cl) * LKS + k + kq];
#pragma unroll
            for (int cb = 0; cb < 4; cb++)
                acc[cb] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, SB[(16 * cb + cl) * LKS + k + kq], acc[cb], 0, 0, 0);
        }
    }
    if (Xd) __syncthreads();                  // the last chunk's operand reads are done: Xd reuses their LDS
    // the original entries of this tile's panel columns (computed, not read), one row group at a time
    // (a group's four entries are loaded and computed before its stores; all sixteen at once held 32
    // more VGPRs through the epilogue)
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const int i = 16 * w + kq + 4 * r;
        double ov[4];
#pragma unroll
        for (int cb = 0; cb < 4; cb++) {
            const int j = 16 * cb + cl;
            ov[cb] = gpf_entry(D2, n, Y, d, pt, FULL ? r0 + i : min(r0 + i, n), c0 + (FULL ? j : min(j, pb - 1)));
        }
#pragma unroll
        for (int cb = 0; cb < 4; cb++) {
            const int j = 16 * cb + cl;
            if ((FULL || (r0 + i <= n && j < pb)) && (!DIAG || j <= i)) {
                const double v = ov[cb] - acc[cb][r];
                // the fused diagonal factor's input stays in LDS; the rows below it in tile 0 (the
                // last, short panel: row n) go to A for the row solve
                if (Xd && i < pb) Xd[i * (LB + 1) + j] = v;
                else Ab[(unsigned)((r0 + i) * ld + c0 + j)] = v;
            }
        }
    }
#undef GPF_LL_LOAD
}

template <bool FMA>
__device__ __forceinline__ double gpf_msub(double x, double a, double b) {   // x - a*b
    if constexpr (FMA) return fma(-a, b, x);
    else return x - a * b;
}

// The 64x64 diagonal block of one matrix on one wave (lane i = row i, right-looking by columns:
// L_jj = sqrt(a_jj), L_ij = a_ij * (1/L_jj), a_ik -= L_ij L_kj for k > j), the column broadcast
// through LDS.  Lanes i < k carry garbage in a[k] (the upper triangle), never stored.  Leaves L11
// (column-major) and 1/L_jj in Lpan[b], or sets fail[b].
template <bool FMA>
__device__ __forceinline__ void gpf_ll_factor(double (&a)[LB], int i, int pb, double *col, int b,
                                              int32_t *__restrict__ fail, double *__restrict__ Lpan) {
    bool bad = false;
    double myr = 1.0;
#pragma unroll
    for (int j = 0; j < LB; j++) {
        if (j < pb) {
            const double djj = lane_double(a[j], j);
            bad = bad || !(djj > 0.0);
            const double ljj = sqrt(djj);
            const double rj = 1.0 / ljj;
            const double lij = a[j] * rj;
            a[j] = (i == j) ? ljj : lij;
            myr = (i == j) ? rj : myr;
            col[i] = a[j];
            wave_sync_lds();
#pragma unroll
            for (int k = j + 1; k < LB; k++) a[k] = gpf_msub<FMA>(a[k], a[j], col[k]);
            wave_sync_lds();
        }
    }
    if (bad) {
        if (i == 0) fail[b] = 1;
        return;
    }
    double *Lb = Lpan + (size_t)b * LPS64;
#pragma unroll
    for (int k = 0; k < LB; k++) Lb[k * LB + i] = (i < pb && k <= i) ? a[k] : 0.0;
    Lb[LB * LB + i] = myr;
}

// FLY: panel 0, the block's original entries computed (gpf_entry); else read from A (the panel
// GEMM left them there, NNGP_GPF_FUSE=0)
template <bool FMA>
__global__ void __launch_bounds__(64) gpf_ll_diag_kernel(const double *__restrict__ A, int n, int c0, int pb,
                                                          int32_t *__restrict__ fail, double *__restrict__ Lpan,
                                                          int nmat, const double *__restrict__ D2,
                                                          const double *__restrict__ Y, int d,
                                                          const GPPoint *__restrict__ pts) {
    const int b = blockIdx.x;
    if (b >= nmat || fail[b]) return;
    const int i = threadIdx.x, ld = n + 1;
    const double *Ab = A + (size_t)b * ld * ld;
    __shared__ __attribute__((aligned(16))) double col[LB];
    const bool fly = (c0 == 0);
    const GPPoint pt = pts[b];
    const int ic = min(i, pb - 1);
    double a[LB];
    if (fly) {
#pragma unroll
        for (int k = 0; k < LB; k++) a[k] = gpf_entry(D2, n, Y, d, pt, c0 + ic, c0 + min(k, ic));
    } else {
#pragma unroll
        for (int k = 0; k < LB; k++) a[k] = Ab[(size_t)(c0 + ic) * ld + c0 + min(k, ic)];
    }
#pragma unroll
    for (int k = 0; k < LB; k++) a[k] = (i < pb && k <= i) ? a[k] : 0.0;
    gpf_ll_factor<FMA>(a, i, pb, col, b, fail, Lpan);
}

// FUSED: the diagonal tile's workgroup (dispatched before the matrix's other tiles: gpf_xcd_map
// gives tile 0 the matrix's lowest linear id) leaves its updated block in LDS and factors it on
// wave 0 -- gpf_ll_diag_kernel's arithmetic on the same values, one launch fewer per panel.  (The
// factor on all four waves, a barrier per column, and the row solve reading L11 by scalar loads
// were both measured slower at Burgers sizes and removed: DESIGN.md §8.)
template <bool FUSED, bool FMA>
__global__ void __launch_bounds__(256, FUSED ? 2 : 4) gpf_ll_gemm_kernel(double *__restrict__ A, int n, int c0, int pb,
                                                              int32_t *__restrict__ fail, double *__restrict__ Lpan,
                                                              int T, int nmat, const double *__restrict__ D2,
                                                              const double *__restrict__ Y, int d,
                                                              const GPPoint *__restrict__ pts) {
    int b, t;
    gpf_xcd_map(blockIdx.x + blockIdx.y * T, T, b, t);
    if (b >= nmat || fail[b]) return;
    const int ld = n + 1;
    double *Ab = A + (size_t)b * ld * ld;
    const int r0 = c0 + LB * t;
    const GPPoint pt = pts[b];
    __shared__ __attribute__((aligned(16))) double S[2 * LB * LKS];   // Sa | Sb; then the fused factor's block
    static_assert(2 * LB * LKS >= LB * (LB + 1), "the fused factor's block reuses the operand LDS");
    double *Xd = (FUSED && t == 0) ? S : nullptr;
    const bool full = r0 + LB - 1 <= n && pb == LB;
    if (t == 0) {
        if (full) gpf_ll_gemm_tile<true, true>(Ab, ld, n, c0, pb, r0, S, S + LB * LKS, Xd, D2, Y, d, pt);
        else gpf_ll_gemm_tile<false, true>(Ab, ld, n, c0, pb, r0, S, S + LB * LKS, Xd, D2, Y, d, pt);
    } else {
        if (full) gpf_ll_gemm_tile<true, false>(Ab, ld, n, c0, pb, r0, S, S + LB * LKS, nullptr, D2, Y, d, pt);
        else gpf_ll_gemm_tile<false, false>(Ab, ld, n, c0, pb, r0, S, S + LB * LKS, nullptr, D2, Y, d, pt);
    }
    if constexpr (FUSED) {
        if (t != 0) return;
        __syncthreads();
        if (threadIdx.x >= 64) return;
        __shared__ __attribute__((aligned(16))) double col[LB];
        const int i = threadIdx.x;
        double a[LB];
#pragma unroll
        for (int k = 0; k < LB; k++) a[k] = (i < pb && k <= i) ? Xd[i * (LB + 1) + k] : 0.0;
        gpf_ll_factor<FMA>(a, i, pb, col, b, fail, Lpan);
    }
}

// The rows below the diagonal block: x L11^T = a by substitution (dtrsm's right-looking order with
// 1/L_jj), one lane per row, staged through LDS 16 columns at a time (coalesced).  Panel 0 (FLY)
// computes the rows' original entries instead of reading them.
template <bool FMA>
__global__ void __launch_bounds__(256) gpf_ll_rows_kernel(double *__restrict__ A, int n, int c0, int pb,
                                                           const int32_t *__restrict__ fail,
                                                           const double *__restrict__ Lpan, int T, int nmat,
                                                           const double *__restrict__ D2,
                                                           const double *__restrict__ Y, int d,
                                                           const GPPoint *__restrict__ pts) {
    int b, t;
    gpf_xcd_map(blockIdx.x + blockIdx.y * T, T, b, t);
    if (b >= nmat || fail[b]) return;
    const int ld = n + 1;
    double *Ab = A + (size_t)b * ld * ld;
    __shared__ __attribute__((aligned(16))) double L[LPS64];   // column-major L11 | 1/L_jj
    __shared__ double X[4][LB * 17];                           // per wave: 64 rows x 16 columns
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const double *Lsrc = Lpan + (size_t)b * LPS64;
    const int rw = c0 + pb + 256 * t + 64 * w;   // this wave's first row
    const bool fly = (c0 == 0), act = rw <= n;
    const GPPoint pt = pts[b];
    double *Xw = X[w];
    // 16 columns of the wave's 64 rows per round, coalesced; round q + 1's loads are issued before
    // round q goes through LDS, and round 0's before the L11 copy (software-pipelined: each round
    // used to wait out a full memory latency)
    double sv[16], sn[16];
#define GPF_ROWS_STAGE(dst, q)                                                                          \
    if (fly) {                                                                                        \
        _Pragma("unroll") for (int v = 0; v < 16; v++) {                                               \
            const int e = lane + 64 * v, rr = e >> 4, k = 16 * (q) + (e & 15);                         \
            dst[v] = gpf_entry(D2, n, Y, d, pt, min(rw + rr, n), min(k, pb - 1));                      \
        }                                                                                             \
    } else {                                                                                          \
        _Pragma("unroll") for (int v = 0; v < 16; v++) {                                               \
            const int e = lane + 64 * v, rr = e >> 4, k = 16 * (q) + (e & 15);                         \
            dst[v] = Ab[(size_t)min(rw + rr, n) * ld + c0 + min(k, pb - 1)];                           \
        }                                                                                             \
    }
    if (act) {
        GPF_ROWS_STAGE(sv, 0)
    }
    {   // all 17 loads issued before the first LDS store
        constexpr int NL = (LPS64 + 255) / 256;
        double lv[NL];
#pragma unroll
        for (int u = 0; u < NL; u++) lv[u] = Lsrc[min(tid + 256 * u, LPS64 - 1)];
#pragma unroll
        for (int u = 0; u < NL; u++)
            if (tid + 256 * u < LPS64) L[tid + 256 * u] = lv[u];
        __syncthreads();
    }
    const double *Lr = L;
    if (t == 0)   // L11 into A's diagonal block, coalesced along the rows
        for (int e = tid; e < LB * LB; e += 256) {
            const int ii = e >> 6, k = e & 63;
            if (k <= ii && ii < pb) Ab[(size_t)(c0 + ii) * ld + c0 + k] = Lr[k * LB + ii];
        }
    if (!act) return;                            // (no barrier follows)
    double x[LB];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        if (q < 3) {
            GPF_ROWS_STAGE(sn, q + 1)
        }
#pragma unroll
        for (int v = 0; v < 16; v++) {
            const int e = lane + 64 * v, rr = e >> 4, k = 16 * q + (e & 15);
            Xw[rr * 17 + (e & 15)] = (rw + rr <= n && k < pb) ? sv[v] : 0.0;
        }
        wave_sync_lds();
#pragma unroll
        for (int c = 0; c < 16; c++) x[16 * q + c] = Xw[lane * 17 + c];
        wave_sync_lds();
#pragma unroll
        for (int v = 0; v < 16; v++) sv[v] = sn[v];
    }
#undef GPF_ROWS_STAGE
#pragma unroll
    for (int j = 0; j < LB; j++) {
        if (j < pb) {
            x[j] = x[j] * Lr[LB * LB + j];
            // L11's row j in chunks of 16, each chunk's LDS reads issued together ahead of its
            // updates (a scheduling barrier keeps them grouped): left to itself the compiler
            // interleaved read and update and waited on ~1 100 of the ~1 200 reads, 450 of them
            // full drains; grouped, 134 full drains and the rest with 2-5 reads still in flight
#pragma unroll
            for (int k0 = j + 1; k0 < LB; k0 += 16) {
                double lv[16];
#pragma unroll
                for (int k = k0; k < k0 + 16 && k < LB; k++) lv[k - k0] = Lr[j * LB + k];
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int k = k0; k < k0 + 16 && k < LB; k++) x[k] = gpf_msub<FMA>(x[k], x[j], lv[k - k0]);
            }
        }
    }
#pragma unroll
    for (int q = 0; q < 4; q++) {
#pragma unroll
        for (int c = 0; c < 16; c++) Xw[lane * 17 + c] = x[16 * q + c];
        wave_sync_lds();
#pragma unroll
        for (int v = 0; v < 16; v++) {
            const int e = lane + 64 * v, rr = e >> 4, k = 16 * q + (e & 15);
            if (rw + rr <= n && k < pb) Ab[(size_t)(rw + rr) * ld + c0 + k] = Xw[rr * 17 + (e & 15)];
        }
        wave_sync_lds();
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
// Factor order: NNGP_GPF_ORDER=0 (default) the left-looking 64-column panels, 1 the right-looking
// 32-column order (rounds 3-5); NNGP_GPF_FMA=1 fuses the diagonal factor's and the row solve's
// updates a - l*l' into one FMA (left-looking order only; ~5 % faster, but the FHN-ODE GParareal
// iterates then part from the reference's by 1.9e-5, against 1e-6 unfused: not the default); NNGP_GPF_FUSE=0 factors the diagonal block in its own launch
// instead of in the panel GEMM's tile-0 workgroups (bitwise the same).
static int gpf_eval(const double *D2, int n, const double *Y, int d, const GPPoint *pts, int nb, double *A,
                    int32_t *fail, double *fval, double *alpha_out, double *Lpan, hipStream_t st) {
    NNGP_HIP_CHECK(hipMemsetAsync(fail, 0, sizeof(int32_t) * nb, st));
    const bool ll = env_int("NNGP_GPF_ORDER", 0) == 0;
    if (!ll) {   // the left-looking order computes each entry where it first reads it (gpf_entry)
        const unsigned bx = (unsigned)((n + GPF_BROWS - 1) / GPF_BROWS + 1);   // + the y row's block
        hipLaunchKernelGGL(gpf_build_kernel, dim3(bx, nb), dim3(256), 0, st, D2, n, Y, d, pts, A, fail);
        NNGP_LAUNCH_CHECK();
    }
    const unsigned ny8 = (unsigned)((nb + 7) / 8 * 8);   // grid y padded: XCD order
    if (ll) {
        const bool fma = env_int("NNGP_GPF_FMA", 0) != 0, fused = env_int("NNGP_GPF_FUSE", 1) != 0;
        for (int c0 = 0; c0 < n; c0 += LB) {
            const int pb = std::min(LB, n - c0);
            const int T = (n + 1 - c0 + LB - 1) / LB;
            const dim3 gg((unsigned)T, ny8);
            if (c0 > 0 && fused) {   // panel GEMM with the diagonal factor in its tile-0 workgroups
                if (fma)
                    hipLaunchKernelGGL((gpf_ll_gemm_kernel<true, true>), gg, dim3(256), 0, st, A, n, c0, pb, fail, Lpan,
                                       T, nb, D2, Y, d, pts);
                else
                    hipLaunchKernelGGL((gpf_ll_gemm_kernel<true, false>), gg, dim3(256), 0, st, A, n, c0, pb, fail,
                                       Lpan, T, nb, D2, Y, d, pts);
            } else {
                if (c0 > 0)
                    hipLaunchKernelGGL((gpf_ll_gemm_kernel<false, false>), gg, dim3(256), 0, st, A, n, c0, pb, fail,
                                       Lpan, T, nb, D2, Y, d, pts);
                if (fma)
                    hipLaunchKernelGGL(gpf_ll_diag_kernel<true>, dim3(nb), dim3(64), 0, st, A, n, c0, pb, fail, Lpan,
                                       nb, D2, Y, d, pts);
                else
                    hipLaunchKernelGGL(gpf_ll_diag_kernel<false>, dim3(nb), dim3(64), 0, st, A, n, c0, pb, fail, Lpan,
                                       nb, D2, Y, d, pts);
            }
            const int TR = (n + 1 - c0 - pb + 255) / 256;   // >= 1: row n is always below
            const dim3 gr((unsigned)TR, ny8);
            if (fma)
                hipLaunchKernelGGL(gpf_ll_rows_kernel<true>, gr, dim3(256), 0, st, A, n, c0, pb, fail, Lpan, TR, nb, D2, Y,
                                   d, pts);
            else
                hipLaunchKernelGGL(gpf_ll_rows_kernel<false>, gr, dim3(256), 0, st, A, n, c0, pb, fail, Lpan, TR, nb, D2,
                                   Y, d, pts);
        }
    } else {
        for (int p0 = 0; p0 < n; p0 += GPB) {
            const int pb = std::min(GPB, n - p0);
            const int below = n + 1 - p0 - pb;   // includes row n (y)
            const unsigned chunks = (unsigned)std::max(1, (below + 63) / 64);
            hipLaunchKernelGGL(gpf_diag_kernel, dim3((nb + 1) / 2), dim3(64), 0, st, A, n, p0, pb, nb, fail, Lpan);
            if (pb == GPB)
                hipLaunchKernelGGL(gpf_rows_kernel<true>, dim3(chunks, nb), dim3(64), 0, st, A, n, p0, pb, fail, Lpan);
            else
                hipLaunchKernelGGL(gpf_rows_kernel<false>, dim3(chunks, nb), dim3(64), 0, st, A, n, p0, pb, fail, Lpan);
            const int nt = (below + GPF_TM - 1) / GPF_TM;
            const int ntiles = nt * (nt + 1) / 2;
            const dim3 grid((unsigned)(ntiles + 1), ny8);
            hipLaunchKernelGGL(gpf_update_kernel, grid, dim3(256), 0, st, A, n, p0, pb, fail, Lpan, ntiles, nb);
        }
    }
    NNGP_LAUNCH_CHECK();
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
    const size_t bytes = sizeof(double) * (nn + (size_t)nb * mm + nb + (size_t)nb * LPS64) + sizeof(GPPoint) * nb +
                         sizeof(int32_t) * nb + 64;
    char *p = (char *)workspace(bytes, &err, 3);
    if (err) return err;
    w.D2 = (double *)p;
    w.A = w.D2 + nn;
    w.fval = w.A + (size_t)nb * mm;
    w.Lpan = w.fval + nb;
    w.pts = (GPPoint *)(w.Lpan + (size_t)nb * LPS64);
    w.fail = (int32_t *)(w.pts + nb);
    return NNGP_OK;
}

static int gpf_check(int64_t rows, int d, int n_fit) {
    // (rows+1)^2 and rows*d index in 32 bits inside the left-looking kernels (32-bit offsets from a
    // uniform base let the loads use scalar bases: fewer VGPRs, 4 workgroups per CU)
    NNGP_REQUIRE(rows >= 1 && rows <= 46000, "full GP needs 1 <= rows <= 46000 (got %lld)", (long long)rows);
    NNGP_REQUIRE((int64_t)rows * d < ((int64_t)1 << 31), "full GP: rows x d too large");
    NNGP_REQUIRE(d >= 1 && n_fit >= 1, "bad d / fit count");
    return NNGP_OK;
}

// points per batch: all fits, capped so the factor slab stays under NNGP_GPF_SLAB_MB (default 32 GB
// of the 288 GB HBM: FHN-PDE d_x = 10 at N = 512 factors 1 800 matrices of ~4 100 rows per round,
// 240 GB in one slab, so its rounds run in chunks of ~230 matrices, each chunk filling the chip)
static int gpf_batch_cap(int n, int n_fit) {
    const size_t per = sizeof(double) * (size_t)(n + 1) * (n + 1);
    const size_t slab = (size_t)std::max(1, env_int("NNGP_GPF_SLAB_MB", 32768)) << 20;
    const size_t cap = std::max<size_t>(1, slab / per);
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
