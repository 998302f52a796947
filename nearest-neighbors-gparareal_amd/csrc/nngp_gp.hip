// nngp_gp.hip -- the nearest-neighbour GP correction on gfx950 (MI355X).
//
// Replaces NNGP_p.predict (models.py:171-226): kNN (177-179), the n*9*R hyper-parameter fits
// fanned out by pool.map(_get_opt_par) (185-202, 228-237), each a scipy Nelder-Mead on the
// negative log marginal likelihood (254-260 -> 240-252 -> _fit_gp_jit 86-92), the per-coordinate
// argmin (207-215) and the posterior mean (162-168, 217).
//
// Kernels
//   knn_dist_kernel    squared distance of every training row to the query, sequential sum
//                      (scipy cdist 'sqeuclidean' order); rows tiled through LDS so the global
//                      loads stay coalesced while each lane keeps its row's sequential order.
//   knn_select_kernel  one workgroup: m rounds of (dist, index) arg-min -> idx; gathers
//                      y[:, c] columns and builds D2 = pairwise |xm_r - xm_j|^2 (numpy pairwise
//                      order) and kd2 = |xm_r - new_x|^2, all theta-independent (hoisted out of
//                      the ~10^2 likelihood evaluations each fit makes).
//   nm_fit_kernel<G>   one GROUP of G = 16 or 32 lanes per fit (m <= G), lane r owns row r of the
//                      m x m kernel matrix in VGPRs.  Each evaluation builds the row
//                      (10^sy exp(c D2) + jitter I), runs a left-looking Cholesky whose row
//                      broadcasts are wave shuffles, forward/back triangular solves, and the
//                      -LML with xor-butterfly reductions.  Nelder-Mead itself is an in-register
//                      state machine (scipy's rules) so every group of a wave always performs
//                      exactly one evaluation per loop trip -- no divergent evaluation code.
//                      FUSED: a workgroup holds whole coordinates, so after a __syncthreads the
//                      first group of each coordinate does the arg-min and the posterior mean and
//                      writes preds (+ uG bias = the Parareal update, parareal.py:382).
// Numerics: -ffp-contract=off; orders documented in oracle/nngp_oracle.c, which restates the
// same arithmetic on the CPU so GPU-vs-oracle parity is (near) bitwise.

#include <math.h>

#include <algorithm>

#include "common.h"
#include "nngp_math.h"

namespace nngp {

static constexpr double LOG_2PI = 1.8378770664093453;   // np.log(2*np.pi)
static constexpr int MAX_JIT = 16;

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// (value, index) order of numpy argsort with NaN last; strict
__device__ __forceinline__ bool key_less(double av, int64_t ai, double bv, int64_t bi) {
    const bool an = av != av, bn = bv != bv;
    if (an != bn) return bn;
    if (!an && av != bv) return av < bv;
    return ai < bi;
}

// numpy pairwise_sum of (a[i]-b[i])^2, i < n (numpy/_core/src/umath/loops_utils.h.src)
__device__ double pw_leaf(const double *__restrict__ a, const double *__restrict__ b, int n) {
    if (n < 8) {
        double res = 0.;
        for (int i = 0; i < n; i++) {
            const double t = a[i] - b[i];
            res += t * t;
        }
        return res;
    }
    double r[8];
#pragma unroll
    for (int j = 0; j < 8; j++) {
        const double t = a[j] - b[j];
        r[j] = t * t;
    }
    int i;
    for (i = 8; i < n - (n % 8); i += 8) {
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const double t = a[i + j] - b[i + j];
            r[j] += t * t;
        }
    }
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; i++) {
        const double t = a[i] - b[i];
        res += t * t;
    }
    return res;
}

__device__ double pw_sqdiff(const double *__restrict__ a, const double *__restrict__ b, int n) {
    if (n <= 128) return pw_leaf(a, b, n);
    // post-order walk of numpy's recursion: split at n2 = n/2 - (n/2)%8 until n <= 128
    int off[32], len[32], stage[32];
    double left[32];
    int sp = 1;
    off[0] = 0; len[0] = n; stage[0] = 0;
    double ret = 0.0;
    bool have = false;
    while (sp > 0) {
        const int t = sp - 1;
        if (have) {
            if (stage[t] == 1) {
                left[t] = ret;
                stage[t] = 2;
                have = false;
                int n2 = len[t] / 2;
                n2 -= n2 % 8;
                off[sp] = off[t] + n2; len[sp] = len[t] - n2; stage[sp] = 0; sp++;
            } else {   // stage 2: combine
                ret = left[t] + ret;
                sp--;
            }
            continue;
        }
        if (len[t] <= 128) {
            ret = pw_leaf(a + off[t], b + off[t], len[t]);
            have = true;
            sp--;
            continue;
        }
        int n2 = len[t] / 2;
        n2 -= n2 % 8;
        stage[t] = 1;
        off[sp] = off[t]; len[sp] = n2; stage[sp] = 0; sp++;
    }
    return ret;
}

// ---------------------------------------------------------------------------------------------
// kNN
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(64) knn_dist_kernel(const double *__restrict__ X, int64_t rows,
                                                      int d, const double *__restrict__ q,
                                                      double *__restrict__ dist) {
    __shared__ double tile[64][65];   // +1 pad: lane l reads row l -> distinct banks
    __shared__ double qs[64];
    const int lane = threadIdx.x;
    const int64_t r0 = (int64_t)blockIdx.x * 64;
    double acc = 0.0;
    if (d <= 8) {   // tiny rows: direct
        const int64_t r = r0 + lane;
        if (r < rows)
            for (int c = 0; c < d; c++) {
                const double t = q[c] - X[r * d + c];
                acc = acc + t * t;
            }
    } else {
        for (int c0 = 0; c0 < d; c0 += 64) {
            const int nc = min(64, d - c0);
            for (int rr = 0; rr < 64; rr++) {
                const int64_t r = r0 + rr;
                tile[rr][lane] = (r < rows && lane < nc) ? X[r * d + c0 + lane] : 0.0;
            }
            qs[lane] = lane < nc ? q[c0 + lane] : 0.0;
            __syncthreads();
            for (int c = 0; c < nc; c++) {
                const double t = qs[c] - tile[lane][c];
                acc = acc + t * t;
            }
            __syncthreads();
        }
    }
    if (r0 + lane < rows) dist[r0 + lane] = acc;
}

// one workgroup of 256 threads
__global__ void __launch_bounds__(256) knn_select_kernel(
    const double *__restrict__ dist, int64_t rows, int m, const double *__restrict__ X,
    const double *__restrict__ Y, int d, const double *__restrict__ q, int32_t *__restrict__ idx_out,
    double *__restrict__ dist_out, double *__restrict__ ymT, double *__restrict__ D2,
    double *__restrict__ kd2) {
    __shared__ double wv[4];
    __shared__ int64_t wi[4];
    __shared__ int32_t sel[64];
    __shared__ double seld[64];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    double pv = -INFINITY;
    int64_t pi = -1;
    for (int k = 0; k < m; k++) {
        double bv = 0.0;
        int64_t bi = -1;
        for (int64_t r = tid; r < rows; r += 256) {
            const double v = dist[r];
            if (!key_less(pv, pi, v, r)) continue;   // must come strictly after previous pick
            if (bi < 0 || key_less(v, r, bv, bi)) {
                bv = v;
                bi = r;
            }
        }
        // wave reduce (xor butterfly on (value, index); no candidate = index -1)
        for (int s = 1; s < 64; s <<= 1) {
            const double ov = __shfl_xor(bv, s, 64);
            const int64_t oi = __shfl_xor(bi, s, 64);
            if (oi >= 0 && (bi < 0 || key_less(ov, oi, bv, bi))) {
                bv = ov;
                bi = oi;
            }
        }
        if (lane == 0) {
            wv[wid] = bv;
            wi[wid] = bi;
        }
        __syncthreads();
        if (tid == 0) {
            double b = wv[0];
            int64_t bidx = wi[0];
            for (int w = 1; w < 4; w++)
                if (wi[w] >= 0 && (bidx < 0 || key_less(wv[w], wi[w], b, bidx))) {
                    b = wv[w];
                    bidx = wi[w];
                }
            sel[k] = (int32_t)bidx;
            seld[k] = b;
        }
        __syncthreads();
        pv = seld[k];
        pi = sel[k];
    }
    for (int k = tid; k < m; k += 256) {
        idx_out[k] = sel[k];
        if (dist_out) dist_out[k] = seld[k];
    }
    if (ymT) {
        for (int t = tid; t < m * d; t += 256) {
            const int r = t % m, c = t / m;
            ymT[c * m + r] = Y[(int64_t)sel[r] * d + c];
        }
    }
    if (D2) {
        // lower triangle incl. diagonal, mirrored ((a-b)^2 == (b-a)^2 bitwise)
        const int npairs = m * (m + 1) / 2;
        for (int t = tid; t < npairs; t += 256) {
            int r = 0;
            while ((r + 1) * (r + 2) / 2 <= t) r++;
            const int j = t - r * (r + 1) / 2;
            const double v = pw_sqdiff(X + (int64_t)sel[r] * d, X + (int64_t)sel[j] * d, d);
            D2[r * m + j] = v;
            D2[j * m + r] = v;
        }
        for (int r = tid; r < m; r += 256) kd2[r] = pw_sqdiff(X + (int64_t)sel[r] * d, q, d);
    }
}

// D2 / kd2 from an explicit xm (unfused entry points)
__global__ void __launch_bounds__(256) d2_kernel(const double *__restrict__ xm, int m, int d,
                                                 const double *__restrict__ q,
                                                 double *__restrict__ D2, double *__restrict__ kd2) {
    const int npairs = m * (m + 1) / 2;
    for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < npairs + m; t += gridDim.x * blockDim.x) {
        if (t < npairs) {
            int r = 0;
            while ((r + 1) * (r + 2) / 2 <= t) r++;
            const int j = t - r * (r + 1) / 2;
            const double v = pw_sqdiff(xm + (int64_t)r * d, xm + (int64_t)j * d, d);
            D2[r * m + j] = v;
            D2[j * m + r] = v;
        } else if (q && kd2) {
            const int r = t - npairs;
            kd2[r] = pw_sqdiff(xm + (int64_t)r * d, q, d);
        }
    }
}

// ---------------------------------------------------------------------------------------------
// group-level GP factorisation: K = psy*exp(c*D2) + jit*I, Cholesky, L z = y, L^T alpha = z
// lane r (0 <= r < G) of the group owns row r; lanes r >= m carry zeros.
// ---------------------------------------------------------------------------------------------
template <int G>
__device__ __forceinline__ bool group_factor(int m, int lr, int gbase,
                                             const double *__restrict__ sD2, double c, double psy,
                                             double jit, double y_r, double *Limg, double &alpha_r,
                                             double &diag_r) {
    double a[G];
    const bool rowv = lr < m;
    const double *drow = sD2 + (rowv ? lr : 0) * m;
#pragma unroll
    for (int j = 0; j < G; j++) {
        double v = 0.0;
        if (j < m) {   // wave-uniform
            const double e = psy * nn_exp(c * drow[j]);     // k_gauss, models.py:146-148
            v = (rowv && j <= lr) ? e : 0.0;
            v = (rowv && j == lr) ? v + jit : v;             // + eye*10**jitter, models.py:88
        }
        a[j] = v;
    }
    // left-looking Cholesky; jax returns NaN on failure (models.py:89).  Row j of L reaches the
    // other lanes by shuffles; sum_k L_rk L_jk is a balanced tree over k (zero padded to a power
    // of two) -- the same tree as the oracle -- so the dependent chain is log2(j) adds, not j.
    bool fail = false;
    diag_r = 1.0;
    double rinv_r = 1.0;
#pragma unroll
    for (int j = 0; j < G; j++) {
        if (j < m) {   // m is wave-uniform: a scalar branch, the loop stays fully unrolled
            double t = a[j];
            if (j > 0) {
                double pr[G];
#pragma unroll
                for (int k = 0; k < G; k++) pr[k] = (k < j) ? a[k] * __shfl(a[k], gbase + j, 64) : 0.0;
                int P = 1;
                while (P < j) P <<= 1;   // compile-time after unrolling
#pragma unroll
                for (int sft = 1; sft < G; sft <<= 1)
                    if (sft < P) {
#pragma unroll
                        for (int k = 0; k + sft < G; k += 2 * sft)
                            if (k < P) pr[k] = pr[k] + pr[k + sft];
                    }
                t = t - pr[0];
            }
            const double piv = __shfl(t, gbase + j, 64);
            fail = fail || !(piv > 0.0);
            const double ljj = sqrt(piv);
            const double rinv = 1.0 / ljj;
            if (lr > j) {
                a[j] = t * rinv;
            } else if (lr == j) {
                a[j] = ljj;
                diag_r = ljj;
                rinv_r = rinv;
            }
        }
    }
    // division by L_ii as x*r corrected by one fma (Markstein; r = RN(1/L_ii) -> RN(x/L_ii))
    auto divd = [&](double x) {
        const double q = x * rinv_r;
        return fma(fma(-q, diag_r, x), rinv_r, q);
    };
    // forward solve L z = y (models.py:90, inner solve_triangular)
    double acc = rowv ? y_r : 0.0, z = 0.0;
#pragma unroll
    for (int i = 0; i < G; i++) {
        if (i < m) {
            const double zi = __shfl(divd(acc), gbase + i, 64);
            if (lr > i) acc = acc - a[i] * zi;
            if (lr == i) z = zi;
        }
    }
    // rows of L to the group's LDS image for the transposed (back) solve
#pragma unroll
    for (int k = 0; k < G; k++)
        if (k < m && rowv && k <= lr) Limg[lr * G + k] = a[k];
    wave_lds_sync();
    double acc2 = z, alpha = 0.0;
#pragma unroll
    for (int i = G - 1; i >= 0; i--) {
        if (i < m) {
            const double ai = __shfl(divd(acc2), gbase + i, 64);
            if (lr < i) acc2 = acc2 - Limg[i * G + lr] * ai;
            if (lr == i) alpha = ai;
        }
    }
    wave_lds_sync();
    alpha_r = alpha;
    return !fail;
}

template <int G>
__device__ __forceinline__ double group_sum(double v) {
#pragma unroll
    for (int s = 1; s < G; s <<= 1) v = v + __shfl_xor(v, s, 64);
    return v;
}

// -LML (models.py:240-252): NaN (incl. failed Cholesky) -> +inf
template <int G>
__device__ __forceinline__ double group_nlml(int m, int lr, int gbase, const double *sD2,
                                             double sx, double sy, double jit, double y_r,
                                             double *Limg) {
    const double c = -0.5 * (1 / nn_pow10(sx));
    const double psy = nn_pow10(sy);
    double alpha, diag;
    const bool ok = group_factor<G>(m, lr, gbase, sD2, c, psy, jit, y_r, Limg, alpha, diag);
    const bool rowv = lr < m;
    const double ydot = group_sum<G>(rowv ? y_r * alpha : 0.0);
    const double slog = group_sum<G>(rowv ? nn_log(diag) : 0.0);
    const double res = -(((-0.5 * ydot) - slog) - ((double)m / 2) * LOG_2PI);
    return (!ok || res != res) ? INFINITY : res;
}

// posterior mean K(xm, new_x)^T alpha (models.py:162-168); NaN on Cholesky failure
template <int G>
__device__ __forceinline__ double group_mean(int m, int lr, int gbase, const double *sD2,
                                             const double *skd2, double sx, double sy, double jit,
                                             double y_r, double *Limg) {
    const double c = -0.5 * (1 / nn_pow10(sx));
    const double psy = nn_pow10(sy);
    double alpha, diag;
    const bool ok = group_factor<G>(m, lr, gbase, sD2, c, psy, jit, y_r, Limg, alpha, diag);
    const bool rowv = lr < m;
    const double ks = rowv ? psy * nn_exp(c * skd2[lr]) : 0.0;
    const double mean = group_sum<G>(rowv ? ks * alpha : 0.0);
    return ok ? mean : NAN;
}

// ---------------------------------------------------------------------------------------------
// Nelder-Mead state machine (scipy.optimize._optimize._minimize_neldermead, N = 2)
// ---------------------------------------------------------------------------------------------
enum { ST_INIT0, ST_INIT1, ST_INIT2, ST_REFLECT, ST_EXPAND, ST_CONTRACT, ST_ICONTRACT, ST_SHRINK1,
       ST_SHRINK2, ST_DONE };

struct NM {
    double s0x, s0y, s1x, s1y, s2x, s2y;   // simplex (sorted by f after each iteration)
    double f0, f1, f2;
    double xbx, xby, xrx, xry, fxr;        // centroid, reflection
    double px, py;                         // point being evaluated
    int st, fcalls, iters;
};

__device__ __forceinline__ bool nm_less(double a, double b) { return a < b || (b != b && a == a); }

__device__ __forceinline__ void nm_sort(NM &S) {   // stable insertion sort of 3 (numpy argsort)
    if (nm_less(S.f1, S.f0)) {
        double t;
        t = S.f0; S.f0 = S.f1; S.f1 = t;
        t = S.s0x; S.s0x = S.s1x; S.s1x = t;
        t = S.s0y; S.s0y = S.s1y; S.s1y = t;
    }
    if (nm_less(S.f2, S.f1)) {
        double f = S.f2, x = S.s2x, y = S.s2y;
        S.f2 = S.f1; S.s2x = S.s1x; S.s2y = S.s1y;
        if (nm_less(f, S.f0)) {
            S.f1 = S.f0; S.s1x = S.s0x; S.s1y = S.s0y;
            S.f0 = f; S.s0x = x; S.s0y = y;
        } else {
            S.f1 = f; S.s1x = x; S.s1y = y;
        }
    }
}

struct NMCfg {
    double fatol, xatol;
    int maxfun, maxiter;
};

// request an evaluation at (x, y); false = _MaxFuncCallError
__device__ __forceinline__ bool nm_req(NM &S, const NMCfg &c, double x, double y, int st) {
    if (S.fcalls >= c.maxfun) return false;
    S.fcalls++;
    S.px = x;
    S.py = y;
    S.st = st;
    return true;
}

// loop head of the while in _minimize_neldermead
__device__ __forceinline__ void nm_check(NM &S, const NMCfg &c) {
    if (!(S.fcalls < c.maxfun && S.iters < c.maxiter)) {
        S.st = ST_DONE;
        return;
    }
    const bool xok = fabs(S.s1x - S.s0x) <= c.xatol && fabs(S.s1y - S.s0y) <= c.xatol &&
                     fabs(S.s2x - S.s0x) <= c.xatol && fabs(S.s2y - S.s0y) <= c.xatol;
    const bool fok = fabs(S.f0 - S.f1) <= c.fatol && fabs(S.f0 - S.f2) <= c.fatol;
    if (xok && fok) {
        S.st = ST_DONE;
        return;
    }
    S.xbx = (S.s0x + S.s1x) / 2;   // np.add.reduce(sim[:-1], 0) / N
    S.xby = (S.s0y + S.s1y) / 2;
    S.xrx = 2 * S.xbx - 1 * S.s2x;  // (1+rho)*xbar - rho*sim[-1]
    S.xry = 2 * S.xby - 1 * S.s2y;
    if (!nm_req(S, c, S.xrx, S.xry, ST_REFLECT)) {   // aborted: finally-sort, loop exits
        nm_sort(S);
        S.st = ST_DONE;
    }
}

__device__ __forceinline__ void nm_abort(NM &S, const NMCfg &c) {
    nm_sort(S);
    nm_check(S, c);   // fcalls >= maxfun -> DONE
}

__device__ __forceinline__ void nm_end_iter(NM &S, const NMCfg &c) {
    S.iters += 1;
    nm_sort(S);
    nm_check(S, c);
}

__device__ __forceinline__ void nm_shrink_start(NM &S, const NMCfg &c) {
    S.s1x = S.s0x + 0.5 * (S.s1x - S.s0x);   // sim[j] = sim[0] + sigma*(sim[j]-sim[0])
    S.s1y = S.s0y + 0.5 * (S.s1y - S.s0y);
    if (!nm_req(S, c, S.s1x, S.s1y, ST_SHRINK1)) nm_abort(S, c);
}

__device__ void nm_consume(NM &S, const NMCfg &c, double f) {
    switch (S.st) {
    case ST_INIT0:
        S.f0 = f;
        if (!nm_req(S, c, S.s1x, S.s1y, ST_INIT1)) { nm_sort(S); S.st = ST_DONE; }
        break;
    case ST_INIT1:
        S.f1 = f;
        if (!nm_req(S, c, S.s2x, S.s2y, ST_INIT2)) { nm_sort(S); S.st = ST_DONE; }
        break;
    case ST_INIT2:
        S.f2 = f;
        nm_sort(S);
        S.iters = 1;
        nm_check(S, c);
        break;
    case ST_REFLECT:
        S.fxr = f;
        if (f < S.f0) {
            const double xe = 3 * S.xbx - 2 * S.s2x, ye = 3 * S.xby - 2 * S.s2y;
            if (!nm_req(S, c, xe, ye, ST_EXPAND)) nm_abort(S, c);
        } else if (f < S.f1) {
            S.s2x = S.xrx; S.s2y = S.xry; S.f2 = f;
            nm_end_iter(S, c);
        } else if (f < S.f2) {
            const double xc = 1.5 * S.xbx - 0.5 * S.s2x, yc = 1.5 * S.xby - 0.5 * S.s2y;
            if (!nm_req(S, c, xc, yc, ST_CONTRACT)) nm_abort(S, c);
        } else {
            const double xcc = 0.5 * S.xbx + 0.5 * S.s2x, ycc = 0.5 * S.xby + 0.5 * S.s2y;
            if (!nm_req(S, c, xcc, ycc, ST_ICONTRACT)) nm_abort(S, c);
        }
        break;
    case ST_EXPAND:
        if (f < S.fxr) { S.s2x = S.px; S.s2y = S.py; S.f2 = f; }
        else { S.s2x = S.xrx; S.s2y = S.xry; S.f2 = S.fxr; }
        nm_end_iter(S, c);
        break;
    case ST_CONTRACT:
        if (f <= S.fxr) { S.s2x = S.px; S.s2y = S.py; S.f2 = f; nm_end_iter(S, c); }
        else nm_shrink_start(S, c);
        break;
    case ST_ICONTRACT:
        if (f < S.f2) { S.s2x = S.px; S.s2y = S.py; S.f2 = f; nm_end_iter(S, c); }
        else nm_shrink_start(S, c);
        break;
    case ST_SHRINK1:
        S.f1 = f;
        S.s2x = S.s0x + 0.5 * (S.s2x - S.s0x);
        S.s2y = S.s0y + 0.5 * (S.s2y - S.s0y);
        if (!nm_req(S, c, S.s2x, S.s2y, ST_SHRINK2)) nm_abort(S, c);
        break;
    case ST_SHRINK2:
        S.f2 = f;
        nm_end_iter(S, c);
        break;
    default:
        break;
    }
}

struct NMArgs {
    int m, d, n_fits;
    const double *D2;      // [m][m]
    const double *kd2;     // [m] (FUSED)
    const double *Y;       // y of fit f, row r: Y[coord*ys_c + r*ys_r]
    int ys_c, ys_r;
    const int32_t *coord;        // unfused: per-fit coordinate
    const int32_t *jitter_idx;   // unfused: per-fit jitter index
    const double *theta0;        // [n_fits][2]
    double fatol, xatol;
    int maxfev;
    int nj, R, cpw;              // FUSED: jitters, restarts, coordinates per workgroup
    double jit_pow[MAX_JIT];     // 10**jitter_exp (host pow)
    double *theta_out;           // [n_fits][2] or null
    double *fval_out;            // [n_fits] or null
    int32_t *nfev_out;           // [n_fits] or null
    double *fits_out;            // [n_fits][4] or null
    double *preds;               // FUSED [d]
    const double *bias;          // FUSED [d] or null
    double *out;                 // FUSED [d] (preds + bias) or null
};

// static-index lookup (a runtime index into a by-value kernel-argument array would go to scratch)
__device__ __forceinline__ double jit_lookup(const NMArgs &a, int j) {
    double v = 1.0;
#pragma unroll
    for (int i = 0; i < MAX_JIT; i++)
        if (i == j) v = a.jit_pow[i];
    return v;
}

// register budget: G=16 needs ~162 VGPRs (3 waves/SIMD -> <= 768 threads), G=32 ~245
// (2 waves/SIMD -> <= 512 threads); tighter bounds make the compiler spill to scratch
template <int G> struct NMBound { static constexpr int T = (G == 16) ? 768 : 512; };

template <int G, bool FUSED>
__global__ void __launch_bounds__(NMBound<G>::T) nm_fit_kernel(NMArgs a) {
    extern __shared__ __attribute__((aligned(16))) double sm[];
    const int m = a.m;
    const int nfc = a.nj * a.R;                         // fits per coordinate
    const int ngroups = FUSED ? a.cpw * nfc : (int)(blockDim.x / G);
    const int galloc = blockDim.x / G;                  // groups incl. padding lanes
    double *sD2 = sm;
    double *skd2 = sD2 + m * m;
    double *sRes = skd2 + m;                            // [galloc][4]
    double *sL = sRes + galloc * 4;                     // [galloc][G*G]
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int g = tid / G;                              // group in block
    const int lr = tid % G;
    const int gbase = (lane / G) * G;

    for (int i = tid; i < m * m; i += blockDim.x) sD2[i] = a.D2[i];
    if (FUSED)
        for (int i = tid; i < m; i += blockDim.x) skd2[i] = a.kd2[i];
    __syncthreads();

    int f = -1, coord = 0, jidx = 0, q = 0;
    bool valid = g < ngroups;
    if (valid) {
        if (FUSED) {
            coord = blockIdx.x * a.cpw + g / nfc;
            q = g % nfc;
            f = coord * nfc + q;
            jidx = q / a.R;
            valid = coord < a.d;
        } else {
            f = blockIdx.x * ngroups + g;
            valid = f < a.n_fits;
            if (valid) {
                coord = a.coord[f];
                jidx = a.jitter_idx[f];
            }
        }
    }
    const double y_r = (valid && lr < m) ? a.Y[(int64_t)coord * a.ys_c + (int64_t)lr * a.ys_r] : 0.0;
    const double jit = valid ? jit_lookup(a, jidx) : 1.0;
    double *Limg = sL + (size_t)g * G * G;

    NMCfg cfg{a.fatol, a.xatol, a.maxfev, a.maxfev};
    NM S;
    S.fcalls = 0;
    S.iters = 0;
    S.f0 = S.f1 = S.f2 = INFINITY;
    S.xbx = S.xby = S.xrx = S.xry = S.fxr = 0.0;
    if (valid) {
        const double t0x = a.theta0[2 * f], t0y = a.theta0[2 * f + 1];
        S.s0x = t0x; S.s0y = t0y;
        S.s1x = (t0x != 0) ? (1 + 0.05) * t0x : 0.00025; S.s1y = t0y;   // nonzdelt / zdelt
        S.s2x = t0x; S.s2y = (t0y != 0) ? (1 + 0.05) * t0y : 0.00025;
        S.st = ST_INIT0;
        if (!nm_req(S, cfg, S.s0x, S.s0y, ST_INIT0)) S.st = ST_DONE;
    } else {
        S.s0x = S.s0y = S.s1x = S.s1y = S.s2x = S.s2y = 0.0;
        S.px = S.py = 0.0;
        S.st = ST_DONE;
    }
    while (true) {
        const bool need = S.st != ST_DONE;
        if (!__any(need)) break;
        const double fv = group_nlml<G>(m, lr, gbase, sD2, S.px, S.py, jit, y_r, Limg);
        if (need) nm_consume(S, cfg, fv);
    }
    const double fval = (S.f1 != S.f1 || S.f2 != S.f2) ? NAN : S.f0;
    if (valid && lr == 0) {
        if (a.theta_out) { a.theta_out[2 * f] = S.s0x; a.theta_out[2 * f + 1] = S.s0y; }
        if (a.fval_out) a.fval_out[f] = fval;
        if (a.nfev_out) a.nfev_out[f] = S.fcalls;
        if (a.fits_out) {
            a.fits_out[4 * f + 0] = S.s0x;
            a.fits_out[4 * f + 1] = S.s0y;
            a.fits_out[4 * f + 2] = fval;
            a.fits_out[4 * f + 3] = (double)S.fcalls;
        }
        if (FUSED) {
            sRes[4 * g + 0] = S.s0x;
            sRes[4 * g + 1] = S.s0y;
            sRes[4 * g + 2] = fval;
        }
    }
    if (!FUSED) return;
    __syncthreads();
    // first group of each coordinate: first arg-min over its nfc fits (models.py:207-215 reduces
    // to a first-occurrence arg-min), then the posterior mean with that (theta, jitter)
    if (valid && q == 0) {
        int best = 0;
        double bv = sRes[4 * g + 2];
        for (int t = 1; t < nfc; t++) {
            const double v = sRes[4 * (g + t) + 2];
            if (v < bv) {
                bv = v;
                best = t;
            }
        }
        const double sx = sRes[4 * (g + best)], sy = sRes[4 * (g + best) + 1];
        const double jb = jit_lookup(a, best / a.R);
        const double mean = group_mean<G>(m, lr, gbase, sD2, skd2, sx, sy, jb, y_r, Limg);
        if (lr == 0) {
            a.preds[coord] = mean;
            if (a.out) a.out[coord] = a.bias ? mean + a.bias[coord] : mean;
        }
    }
}

// posterior mean for given (theta, jitter) per coordinate; one group per coordinate
template <int G>
__global__ void __launch_bounds__(256) gp_mean_kernel(int m, int d, const double *__restrict__ D2,
                                                      const double *__restrict__ kd2,
                                                      const double *__restrict__ ym,
                                                      const double *__restrict__ theta,
                                                      const int32_t *__restrict__ jitter_idx,
                                                      NMArgs jt, double *__restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) double sm[];
    double *sD2 = sm, *skd2 = sm + m * m, *sL = skd2 + m;
    const int tid = threadIdx.x, lane = tid & 63, g = tid / G, lr = tid % G, gbase = (lane / G) * G;
    for (int i = tid; i < m * m; i += blockDim.x) sD2[i] = D2[i];
    for (int i = tid; i < m; i += blockDim.x) skd2[i] = kd2[i];
    __syncthreads();
    const int c = blockIdx.x * (blockDim.x / G) + g;
    const bool valid = c < d;
    const int cc = valid ? c : 0;
    const double y_r = (valid && lr < m) ? ym[(int64_t)lr * d + cc] : 0.0;
    const double mean = group_mean<G>(m, lr, gbase, sD2, skd2, theta[2 * cc], theta[2 * cc + 1],
                                      jit_lookup(jt, jitter_idx[cc]), y_r, sL + (size_t)g * G * G);
    if (valid && lr == 0) out[c] = mean;
}

// ---------------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------------
static int fill_jitters(NMArgs &a, int n_jitter, const double *jexp) {
    NNGP_REQUIRE(n_jitter >= 1 && n_jitter <= MAX_JIT, "n_jitter must be in [1, %d]", MAX_JIT);
    NNGP_REQUIRE(jexp != nullptr, "jitter_exp_host is NULL");
    for (int i = 0; i < n_jitter; i++) a.jit_pow[i] = pow(10.0, jexp[i]);   // 10**jitter
    a.nj = n_jitter;
    return NNGP_OK;
}

static int group_size_for(int m) { return m <= 16 ? 16 : 32; }

template <int G>
static int launch_nm(NMArgs &a, bool fused, int nblocks, int threads, size_t lds, hipStream_t st) {
    if (fused)
        hipLaunchKernelGGL((nm_fit_kernel<G, true>), dim3(nblocks), dim3(threads), lds, st, a);
    else
        hipLaunchKernelGGL((nm_fit_kernel<G, false>), dim3(nblocks), dim3(threads), lds, st, a);
    NNGP_LAUNCH_CHECK();
    return NNGP_OK;
}

static int run_nm(NMArgs &a, bool fused, hipStream_t st) {
    const int G = group_size_for(a.m);
    int threads, nblocks, ngroups;
    if (fused) {
        const int nfc = a.nj * a.R;
        // whole coordinates per workgroup; keep <= 1024 threads and the LDS under ~150 KB
        // few coordinates per workgroup so the fits spread over every CU (latency-bound NM
        // chains: one workgroup per CU beats packing), capped by LDS / thread budgets below
        static int ncu = 0;
        if (!ncu && hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0) != hipSuccess) ncu = 256;
        if (ncu <= 0) ncu = 256;
        int cpw = (a.d + ncu - 1) / ncu;
        const int cpw_max = std::max(1, (G == 16) ? (36 / nfc) : (18 / nfc));
        cpw = std::max(1, std::min(cpw, std::min(cpw_max, a.d)));
        auto lds_of = [&](int c) {
            const int ng = ((c * nfc * G + 63) / 64) * 64 / G;   // groups incl. padding
            return sizeof(double) * ((size_t)a.m * a.m + a.m + 4 * (size_t)ng + (size_t)ng * G * G);
        };
        const int tmax = (G == 16) ? NMBound<16>::T : NMBound<32>::T;
        auto thr = [&](int c) { return ((c * nfc * G + 63) / 64) * 64; };
        while (cpw > 1 && (lds_of(cpw) > 150 * 1024 || thr(cpw) > tmax)) cpw--;
        if (lds_of(cpw) > 150 * 1024 || thr(cpw) > tmax) {
            set_error("m=%d with %d fits per coordinate exceeds the fused kernel's LDS/threads", a.m, nfc);
            return NNGP_E_UNSUPPORTED;
        }
        a.cpw = cpw;
        ngroups = cpw * nfc;
        (void)ngroups;
        threads = ((ngroups * G + 63) / 64) * 64;
        nblocks = (a.d + cpw - 1) / cpw;
    } else {
        threads = 256;
        ngroups = threads / G;
        (void)ngroups;
        nblocks = (a.n_fits + ngroups - 1) / ngroups;
        a.cpw = 1;
    }
    const int galloc = threads / G;
    const size_t lds = sizeof(double) * ((size_t)a.m * a.m + a.m + 4 * (size_t)galloc + (size_t)galloc * G * G);
    if (G == 16) return launch_nm<16>(a, fused, nblocks, threads, lds, st);
    return launch_nm<32>(a, fused, nblocks, threads, lds, st);
}

}  // namespace nngp

using namespace nngp;

extern "C" int nngp_knn(const double *X, int64_t rows, int d, const double *q, int m,
                        int32_t *idx_out, double *dist_out, void *stream) {
    NNGP_REQUIRE(X && q && idx_out, "null array argument");
    NNGP_REQUIRE(d >= 1, "d must be >= 1");
    NNGP_REQUIRE(m >= 1 && m <= 64 && m <= rows, "need 1 <= m <= min(64, rows) (m=%d rows=%lld)", m,
                 (long long)rows);
    hipStream_t st = (hipStream_t)stream;
    int err = 0;
    double *dist = (double *)workspace(sizeof(double) * rows, &err);
    if (err) return err;
    hipLaunchKernelGGL(knn_dist_kernel, dim3((unsigned)((rows + 63) / 64)), dim3(64), 0, st, X, rows,
                       d, q, dist);
    NNGP_LAUNCH_CHECK();
    hipLaunchKernelGGL(knn_select_kernel, dim3(1), dim3(256), 0, st, dist, rows, m, X, (const double *)nullptr,
                       d, q, idx_out, dist_out, (double *)nullptr, (double *)nullptr, (double *)nullptr);
    NNGP_LAUNCH_CHECK();
    return NNGP_OK;
}

extern "C" int nngp_nm_fit_batch(int m, int d, const double *xm, const double *ym, int n_fits,
                                 const int32_t *coord, const int32_t *jitter_idx, int n_jitter,
                                 const double *jitter_exp_host, const double *theta0, double fatol,
                                 double xatol, int maxfev, double *theta_out, double *fval_out,
                                 int32_t *nfev_out, void *stream) {
    NNGP_REQUIRE(m >= 1 && m <= 32, "need 1 <= m <= 32 (got %d)", m);
    NNGP_REQUIRE(d >= 1 && n_fits >= 0, "bad d / n_fits");
    if (n_fits == 0) return NNGP_OK;
    NNGP_REQUIRE(xm && ym && coord && jitter_idx && theta0, "null array argument");
    NNGP_REQUIRE(maxfev >= 1, "maxfev must be >= 1");
    hipStream_t st = (hipStream_t)stream;
    NMArgs a{};
    int rc = fill_jitters(a, n_jitter, jitter_exp_host);
    if (rc) return rc;
    int err = 0;
    double *D2 = (double *)workspace(sizeof(double) * m * m, &err);
    if (err) return err;
    hipLaunchKernelGGL(d2_kernel, dim3(1), dim3(256), 0, st, xm, m, d, (const double *)nullptr, D2,
                       (double *)nullptr);
    NNGP_LAUNCH_CHECK();
    a.m = m; a.d = d; a.n_fits = n_fits; a.D2 = D2; a.kd2 = nullptr;
    a.Y = ym; a.ys_c = 1; a.ys_r = d;
    a.coord = coord; a.jitter_idx = jitter_idx; a.theta0 = theta0;
    a.fatol = fatol; a.xatol = xatol; a.maxfev = maxfev; a.R = 1;
    a.theta_out = theta_out; a.fval_out = fval_out; a.nfev_out = nfev_out;
    return run_nm(a, false, st);
}

extern "C" int nngp_gp_mean(int m, int d, const double *xm, const double *ym, const double *new_x,
                            const double *theta, const int32_t *jitter_idx, int n_jitter,
                            const double *jitter_exp_host, double *out, void *stream) {
    NNGP_REQUIRE(m >= 1 && m <= 32, "need 1 <= m <= 32 (got %d)", m);
    NNGP_REQUIRE(xm && ym && new_x && theta && jitter_idx && out, "null array argument");
    hipStream_t st = (hipStream_t)stream;
    NMArgs jt{};
    int rc = fill_jitters(jt, n_jitter, jitter_exp_host);
    if (rc) return rc;
    int err = 0;
    double *D2 = (double *)workspace(sizeof(double) * (m * m + m), &err);
    if (err) return err;
    double *kd2 = D2 + m * m;
    hipLaunchKernelGGL(d2_kernel, dim3(1), dim3(256), 0, st, xm, m, d, new_x, D2, kd2);
    NNGP_LAUNCH_CHECK();
    const int G = group_size_for(m);
    const int threads = 256, per = threads / G;
    const size_t lds = sizeof(double) * ((size_t)m * m + m + (size_t)per * G * G);
    if (G == 16)
        hipLaunchKernelGGL(gp_mean_kernel<16>, dim3((d + per - 1) / per), dim3(threads), lds, st, m, d, D2,
                           kd2, ym, theta, jitter_idx, jt, out);
    else
        hipLaunchKernelGGL(gp_mean_kernel<32>, dim3((d + per - 1) / per), dim3(threads), lds, st, m, d, D2,
                           kd2, ym, theta, jitter_idx, jt, out);
    NNGP_LAUNCH_CHECK();
    return NNGP_OK;
}

extern "C" int nngp_predict(const double *X, const double *Y, int64_t rows, int d, const double *new_x,
                            int m, int n_jitter, const double *jitter_exp_host, int n_restarts,
                            const double *theta0, double fatol, double xatol, int maxfev,
                            double *preds_out, const double *bias, double *out, double *fits_out,
                            void *stream) {
    NNGP_REQUIRE(X && Y && new_x && theta0 && preds_out, "null array argument");
    NNGP_REQUIRE(m >= 1 && m <= 32, "need 1 <= m <= 32 (got %d)", m);
    NNGP_REQUIRE(m <= rows, "m=%d exceeds training rows=%lld", m, (long long)rows);
    NNGP_REQUIRE(d >= 1 && n_restarts >= 1 && maxfev >= 1, "bad d / n_restarts / maxfev");
    hipStream_t st = (hipStream_t)stream;
    NMArgs a{};
    int rc = fill_jitters(a, n_jitter, jitter_exp_host);
    if (rc) return rc;
    // workspace: dist[rows] | D2[m*m] | kd2[m] | ymT[d*m] | idx[m] (int32)
    const size_t nd = (size_t)rows + (size_t)m * m + m + (size_t)d * m;
    int err = 0;
    char *ws = (char *)workspace(sizeof(double) * nd + sizeof(int32_t) * 64, &err);
    if (err) return err;
    double *dist = (double *)ws;
    double *D2 = dist + rows;
    double *kd2 = D2 + (size_t)m * m;
    double *ymT = kd2 + m;
    int32_t *idx = (int32_t *)(ymT + (size_t)d * m);
    hipLaunchKernelGGL(knn_dist_kernel, dim3((unsigned)((rows + 63) / 64)), dim3(64), 0, st, X, rows,
                       d, new_x, dist);
    NNGP_LAUNCH_CHECK();
    hipLaunchKernelGGL(knn_select_kernel, dim3(1), dim3(256), 0, st, dist, rows, m, X, Y, d, new_x,
                       idx, (double *)nullptr, ymT, D2, kd2);
    NNGP_LAUNCH_CHECK();
    a.m = m; a.d = d; a.n_fits = d * n_jitter * n_restarts;
    a.D2 = D2; a.kd2 = kd2; a.Y = ymT; a.ys_c = m; a.ys_r = 1;
    a.theta0 = theta0; a.fatol = fatol; a.xatol = xatol; a.maxfev = maxfev; a.R = n_restarts;
    a.fits_out = fits_out; a.preds = preds_out; a.bias = bias; a.out = out;
    return run_nm(a, true, st);
}
