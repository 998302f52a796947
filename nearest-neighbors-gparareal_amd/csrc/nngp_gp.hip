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
//   nm_spec_kernel<MAXM>  one WAVE per fit; its four 16-lane DPP rows evaluate the reflection,
//                      expansion and both contractions of a Nelder-Mead iteration (or the initial
//                      simplex / the shrink points) in one round, consumed in scipy's order by the
//                      unchanged state machine -- identical fits in ~1.5x fewer sequential rounds.
//   nm_fit_kernel<MAXM, FUSED>  four fits per wave (one DPP row each), one evaluation per trip;
//                      FUSED: a workgroup holds whole coordinates and its first row per
//                      coordinate does the arg-min, the posterior mean and u = mean + uG
//                      (parareal.py:382).  Used when the fits would oversubscribe the SIMDs.
//   gp_mean_kernel<MAXM>  arg-min (from a fits array) or given (theta, jitter), posterior mean.
// A likelihood evaluation (gp_factor/gp_nlml): lane l of a fit's row holds rows l (and l+16) of
// the m x m kernel matrix, padded to MAXM in {8,16,24,32} with exact identity rows; the triangle's
// exps are spread over the 16 lanes through an LDS image; the Cholesky / solve broadcasts are
// `v_mov_b64_dpp row_newbcast` (no LDS round trip); the -LML sums are DPP butterflies.
// Numerics: -ffp-contract=off; orders documented in oracle/nngp_oracle.c, which restates the
// same arithmetic on the CPU so GPU-vs-oracle parity is (near) bitwise.

#include <math.h>

#include <algorithm>
#include <mutex>

#include "common.h"
#include "nngp_math.h"
#include "nngp_gpeval.h"
#include "nngp_nm.h"
#include "nngp_nmargs.h"
#include "tableau.h"

namespace nngp {



// (value, index) order of numpy argsort with NaN last, on the squared distances the kNN selects
// from (always >= +0 or NaN): the IEEE bit pattern of a non-negative double orders like its value,
// and every NaN maps to one key above +inf, so a (u64 key, index) pair compares with integer ops.
__device__ __forceinline__ uint64_t dist_key(double v) {
    return (v != v) ? 0x7FF8000000000000ull : (uint64_t)__double_as_longlong(v);
}

__device__ __forceinline__ bool key_less(uint64_t a, int ai, uint64_t b, int bi) {
    return (a < b) | ((a == b) & (ai < bi));
}

// take (k, r) as the running minimum when it is a candidate (r >= 0) ahead of the current one
__device__ __forceinline__ void key_take(uint64_t &bk, int &bi, uint64_t k, int r) {
    const bool t = (r >= 0) & ((bi < 0) | key_less(k, r, bk, bi));
    bk = t ? k : bk;
    bi = t ? r : bi;
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

// numpy's pairwise recursion over n terms (split at n2 = n/2 - (n/2)%8 until n <= 128) as a
// post-order walk: leaf(off, len) gives a leaf's value, the walk combines them as the recursion does
template <typename Leaf>
__device__ __forceinline__ double pw_walk(int n, Leaf &&leaf) {
    if (n <= 128) return leaf(0, n);
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
            ret = leaf(off[t], len[t]);
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

__device__ double pw_sqdiff(const double *__restrict__ a, const double *__restrict__ b, int n) {
    return pw_walk(n, [&](int o, int l) { return pw_leaf(a + o, b + o, l); });
}

// ---------------------------------------------------------------------------------------------
// kNN
// ---------------------------------------------------------------------------------------------
// blockIdx.y = query (batched: query y is q + y*d, its distances dist + y*rows).
// One lane per training row: the row is read with 16-byte vector loads that are all in flight at
// once (no LDS staging, no barriers), then summed sequentially in column order (scipy cdist).
// squared distance of training row r to q (the kernel's and the correction chain's row body)
__device__ __forceinline__ double knn_dist_row(const double *__restrict__ X, int d, const double *__restrict__ q,
                                               int64_t r) {
    const double *xr = X + r * d;
    double acc = 0.0;
    int c = 0;
    if ((((uintptr_t)xr | (uintptr_t)q) & 15) == 0) {   // 16-byte aligned rows: double2 loads
        // 16 double2 loads in flight per lane: 74 VGPRs, so a sweep's kNN launch fits beside the
        // overlapped batch's fit waves (2 per SIMD at 192 VGPRs); at 32 in flight (139 VGPRs) it
        // waited ~3 ms for a SIMD to drain at the start of each Burgers iteration
        constexpr int B = 16;
        for (; c + 2 * B <= d; c += 2 * B) {
            double2 v[B];
#pragma unroll
            for (int j = 0; j < B; j++) v[j] = *(const double2 *)(xr + c + 2 * j);
#pragma unroll
            for (int j = 0; j < B; j++) {
                const double t0 = q[c + 2 * j] - v[j].x;
                acc = acc + t0 * t0;
                const double t1 = q[c + 2 * j + 1] - v[j].y;
                acc = acc + t1 * t1;
            }
        }
    }
    for (; c < d; c++) {
        const double t = q[c] - xr[c];
        acc = acc + t * t;
    }
    return acc;
}

__global__ void __launch_bounds__(64) knn_dist_kernel(const double *__restrict__ X, int64_t rows,
                                                      int d, const double *__restrict__ q,
                                                      double *__restrict__ dist) {
    q += (size_t)blockIdx.y * d;
    dist += (size_t)blockIdx.y * rows;
    const int64_t r = (int64_t)blockIdx.x * 64 + threadIdx.x;
    if (r >= rows) return;
    dist[r] = knn_dist_row(X, d, q, r);
}

__device__ __forceinline__ double wave_lane_double(double v, int lane) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
    return __hiloint2double(hi, lo);
}

// Wave-wide minimum of the (key, index) pair (index -1 = no candidate) with DPP moves inside each
// 16-lane row (quad_perm 1,0,3,2 / 2,3,0,1, row_half_mirror, row_mirror: after each level every
// lane of the aligned block holds the block's minimum, so a mirror reaches the partner block) and
// v_readlane across the four rows.  The order is total, so every lane ends with the same pair.
template <int CTRL>
__device__ __forceinline__ void key_min_dpp(uint64_t &bk, int &bi) {
    const uint32_t lo = __builtin_amdgcn_mov_dpp((int)(uint32_t)bk, CTRL, 0xF, 0xF, false);
    const uint32_t hi = __builtin_amdgcn_mov_dpp((int)(uint32_t)(bk >> 32), CTRL, 0xF, 0xF, false);
    const int oi = __builtin_amdgcn_mov_dpp(bi, CTRL, 0xF, 0xF, false);
    key_take(bk, bi, ((uint64_t)hi << 32) | lo, oi);
}

__device__ __forceinline__ void wave_key_min(uint64_t &bk, int &bi) {
    key_min_dpp<0xB1>(bk, bi);    // quad_perm [1,0,3,2]
    key_min_dpp<0x4E>(bk, bi);    // quad_perm [2,3,0,1]
    key_min_dpp<0x141>(bk, bi);   // row_half_mirror
    key_min_dpp<0x140>(bk, bi);   // row_mirror
    uint64_t rk = 0;
    int ri = -1;
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)bk, 16 * r);
        const uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(bk >> 32), 16 * r);
        key_take(rk, ri, ((uint64_t)hi << 32) | lo, __builtin_amdgcn_readlane(bi, 16 * r));
    }
    bk = rk;
    bi = ri;
}

// total order of doubles as u64 keys (NaN above everything, -0.0 == +0.0) for arg-min reductions
__device__ __forceinline__ uint64_t fval_key(double v) {
    if (v != v) return ~0ull;
    if (v == 0.0) return 0x8000000000000000ull;
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

// minimum over each 16-lane row only (the 4 DPP levels of wave_key_min)
__device__ __forceinline__ void row_key_min(uint64_t &bk, int &bi) {
    key_min_dpp<0xB1>(bk, bi);
    key_min_dpp<0x4E>(bk, bi);
    key_min_dpp<0x141>(bk, bi);
    key_min_dpp<0x140>(bk, bi);
}

// Merge 4 ascending lists of m (key, index) pairs (lists k[0..3][*], index -1 = empty slot) into
// the m smallest in order: a wave's lane t < 4m ranks its pair against all 4m, and a valid pair
// of rank < m lands at that position (ok[]/oi[], or as index + value into oi32/od when ok null).
template <typename KI>
__device__ __forceinline__ void rank_merge(const uint64_t (*k)[64], const int (*ki)[64], int m, int lane, KI *ok,
                                           int *oi, double *od = nullptr) {
    const int n = 4 * m;
    for (int t = lane; t < n; t += 64) {
        const int tl = t / m, tq = t - tl * m;
        const uint64_t ck = k[tl][tq];
        const int ci = ki[tl][tq];
        if (ci < 0) continue;
        int rank = 0;
#pragma unroll
        for (int L = 0; L < 4; L++)
            for (int q = 0; q < m; q++) {
                const int ui = ki[L][q];
                rank += (ui >= 0) & key_less(k[L][q], ui, ck, ci);
            }
        if (rank < m) {
            if (ok) ok[rank] = ck;
            oi[rank] = ci;
            if (od) od[rank] = __longlong_as_double((long long)ck);
        }
    }
}

// LDS staging of the m selected rows for the pair distances (at most 48 KB; larger m*d reads X)
static inline int knn_xs_doubles(int m, int64_t d) { return (int64_t)m * (d + 1) <= 6144 ? (int)(m * (d + 1)) : 0; }
static inline size_t knn_xs_bytes(int m, int64_t d) { return (size_t)knn_xs_doubles(m, d) * sizeof(double); }
// D2/kd2 by d2_wave_kernel (a wave per pair) where the select's own pass would leave one lane per
// pair walking d terms from global memory: d > 128 or rows not staged.  NNGP_D2_WAVES=0: never.
static inline bool d2_by_waves(int m, int d) {
    return env_int("NNGP_D2_WAVES", 1) != 0 && (d > 128 || knn_xs_doubles(m, d) == 0);
}
// D2 / kd2 by d2_pairs_kernel (one thread per pair): the cases neither the select kernel (rows
// staged, d <= 128) nor the wave-per-pair kernel (NNGP_D2_WAVES=0) takes
static inline bool d2_by_pairs(int m, int d) {
    return !d2_by_waves(m, d) && (d > 128 || knn_xs_doubles(m, d) == 0);
}

// LDS of one select (the caller's: a kernel-level __shared__ object, one per kernel)
static constexpr int SEL_CAND = 256;   // candidates the threshold select ranks exactly
struct SelShm {
    int32_t sel[64];
    double seld[64];
    uint32_t hist[256];
    uint64_t ck[SEL_CAND];
    int ci[SEL_CAND];
    int nc, digit, need;
    uint64_t rk[16][64];   // m <= 64
    int ri[16][64];
    uint64_t wk[4][64];
    int wi[4][64];
};

template <int K> __global__ void knn_select_kernel(const double *, int64_t, int, const double *, const double *, int,
                                                  const double *, int32_t *, double *, double *, double *,
                                                  double *, const int32_t *, int32_t *, int, const int32_t *,
                                                  int32_t *, HitMean, int);

// K = 0 (rows > 4 096): up to this many rows the keys are staged once in the dynamic LDS (which
// the launcher sizes for them; the y_m / D2 staging reuses it afterwards) instead of being re-read
// from L2 on each of the radix passes (TomLab N = 256: ~20 of a select's ~24 us at 5 000 rows)
static constexpr int64_t KEY_LDS_ROWS = 14336;

// register-resident keys when rows <= 256*K (K = 2..16), else the streaming form (K = 0)
template <typename... A>
static void launch_knn_select(dim3 grid, size_t shmem, hipStream_t st, const double *dist, int64_t rows,
                              A... args) {
    const int64_t per = (rows + 255) / 256;
    const int kl = (per > 16 && rows <= KEY_LDS_ROWS && env_int("NNGP_KEY_LDS", 1) != 0) ? 1 : 0;
    if (kl) shmem = std::max(shmem, (size_t)rows * sizeof(uint64_t));
    if (per <= 2)
        hipLaunchKernelGGL(knn_select_kernel<2>, grid, dim3(256), shmem, st, dist, rows, args..., kl);
    else if (per <= 4)
        hipLaunchKernelGGL(knn_select_kernel<4>, grid, dim3(256), shmem, st, dist, rows, args..., kl);
    else if (per <= 8)
        hipLaunchKernelGGL(knn_select_kernel<8>, grid, dim3(256), shmem, st, dist, rows, args..., kl);
    else if (per <= 16)
        hipLaunchKernelGGL(knn_select_kernel<16>, grid, dim3(256), shmem, st, dist, rows, args..., kl);
    else
        hipLaunchKernelGGL(knn_select_kernel<0>, grid, dim3(256), shmem, st, dist, rows, args..., kl);
}

// pw_leaf (8 <= n <= 128) on the 8 lanes of an aligned octet, lane j = lane & 7: lane j sums the
// elements i = j (mod 8) below n - n%8 in ascending order (pw_leaf's r[j]); the octet combines
// ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) with DPP moves (lane^1, lane^2, then the mirrored 4-block;
// a+b == b+a, so every lane holds the same bits); the n%8 tail follows in ascending order.
// Bitwise pw_leaf, with 8 lanes on one pair instead of one.  All 8 lanes must be active.
__device__ __forceinline__ double pw_leaf_octet(const double *__restrict__ a, const double *__restrict__ b, int n,
                                                int j) {
    const int nb = n - (n % 8);
    double av[16], bv[16];   // all loads in flight before the sum (n <= 128: <= 16 per lane)
#pragma unroll
    for (int u = 0; u < 16; u++) {
        const int i = j + 8 * u;
        av[u] = i < nb ? a[i] : 0.0;
        bv[u] = i < nb ? b[i] : 0.0;
    }
    double t = av[0] - bv[0];
    double r = t * t;
#pragma unroll
    for (int u = 1; u < 16; u++) {
        if (8 * u < nb) {   // nb is a multiple of 8: the same trip count on every lane
            t = av[u] - bv[u];
            r += t * t;
        }
    }
    r = r + __builtin_amdgcn_mov_dpp(r, 0xB1, 0xF, 0xF, false);    // quad_perm [1,0,3,2]
    r = r + __builtin_amdgcn_mov_dpp(r, 0x4E, 0xF, 0xF, false);    // quad_perm [2,3,0,1]
    r = r + __builtin_amdgcn_mov_dpp(r, 0x141, 0xF, 0xF, false);   // row_half_mirror
    for (int i = nb; i < n; i++) {
        t = a[i] - b[i];
        r += t * t;
    }
    return r;
}

// one workgroup of 256 threads per query (blockIdx.y; batched outputs at query-strided offsets).
// spec_idx / hit_flag (single query): hit_flag = 1 iff the selected ordered neighbour list equals
// spec_idx, else 2 iff it equals spec2_idx (when given), else 0 -- the speculative sweep then
// reuses the fits it computed for that list.  host_flag (host-mapped, optional) gets the same value.
template <int K, bool GENERIC_D2 = true>
__device__ __forceinline__ void knn_select_dev(
    SelShm &sh, const double *__restrict__ dist, int64_t rows, int m, const double *__restrict__ X,
    const double *__restrict__ Y, int d, const double *__restrict__ q, int32_t *__restrict__ idx_out,
    double *__restrict__ dist_out, double *__restrict__ ymT, double *__restrict__ D2,
    double *__restrict__ kd2, const int32_t *__restrict__ spec_idx, int32_t *__restrict__ hit_flag,
    int xs_doubles, const int32_t *__restrict__ spec2_idx, int32_t *host_flag, uint64_t *marks = nullptr,
    const HitMean *hm = nullptr, bool key_lds = false) {
    // marks (profiling, thread 0's clock): after the rounds | the merges | the gathers | D2
#define SEL_MARK(k) \
    if (marks && tid == 0) marks[k] += wall_clock64();
    int32_t *sel = sh.sel;
    double *seld = sh.seld;
    uint64_t(*rk)[64] = sh.rk;
    int(*ri)[64] = sh.ri;
    uint64_t(*wk)[64] = sh.wk;
    int(*wi)[64] = sh.wi;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    // K > 0: the thread's K keys (rows tid + 256*j) stay in registers
    uint64_t kv[K > 0 ? K : 1];
    int kr[K > 0 ? K : 1];
    if constexpr (K > 0) {
#pragma unroll
        for (int j = 0; j < K; j++) {
            const int r = tid + 256 * j;
            kr[j] = r < rows ? r : -1;
            kv[j] = r < rows ? dist_key(dist[r]) : 0;
        }
    }
    // 0) threshold select: the m-th smallest high word T of the keys by a 4-pass radix select
    //    (8-bit digits, LDS histograms), then every row with high word <= T -- a superset of the
    //    m nearest, usually m plus a few -- is ranked exactly by (key, row) against the others.
    //    Bitwise the rounds below (the ordered m smallest pairs are unique); they remain the path
    //    when more than SEL_CAND rows tie at or below T (duplicated training rows).  K > 0: the
    //    thread's keys from registers; K = 0 (rows > 4 096): re-read from dist (L2-resident) on
    //    each of the 5 passes -- against the rounds' m passes over all rows (TomLab N = 256 late
    //    in its run: ~25 000 rows, m = 18, 172 us per select with the rounds alone).
    bool done = false;
    // K = 0 with key_lds: the keys staged once in the dynamic LDS (KEY_LDS_ROWS)
    extern __shared__ __attribute__((aligned(16))) double sel_dyn[];
    uint64_t *kc = reinterpret_cast<uint64_t *>(sel_dyn);
    if constexpr (K == 0) {
        if (key_lds) {
#pragma unroll 8
            for (int r = tid; r < rows; r += 256) kc[r] = dist_key(dist[r]);
            __syncthreads();
        }
    }
    auto for_keys = [&](auto &&f) {
        if constexpr (K > 0) {
#pragma unroll
            for (int j = 0; j < K; j++)
                if (kr[j] >= 0) f(kv[j], kr[j]);
        } else if (key_lds) {
#pragma unroll 8
            for (int r = tid; r < rows; r += 256) f(kc[r], r);
        } else {
#pragma unroll 8
            for (int r = tid; r < rows; r += 256) f(dist_key(dist[r]), r);
        }
    };
    {
        uint32_t prefix = 0;
        int need = m;
        for (int pass = 0; pass < 4; pass++) {
            const int shift = 24 - 8 * pass;
            sh.hist[tid] = 0;   // 256 threads = 256 bins
            __syncthreads();
            for_keys([&](uint64_t key, int) {
                const uint32_t hk = (uint32_t)(key >> 32);
                const bool in = pass == 0 || (hk >> (shift + 8)) == (prefix >> (shift + 8));
                if (in) atomicAdd(&sh.hist[(hk >> shift) & 255], 1u);
            });
            __syncthreads();
            if (wid == 0) {   // the digit whose bin holds the need-th smallest: lane l scans bins 4l..4l+3
                const uint32_t h0 = sh.hist[4 * lane], h1 = sh.hist[4 * lane + 1], h2 = sh.hist[4 * lane + 2],
                               h3 = sh.hist[4 * lane + 3];
                const int own = (int)(h0 + h1 + h2 + h3);
                int incl = own;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const int v = __shfl_up(incl, o, 64);
                    if (lane >= o) incl += v;
                }
                const int excl = incl - own;
                if (excl < need && need <= incl) {
                    int c = excl, b = 0;
                    const int hb[4] = {(int)h0, (int)h1, (int)h2, (int)h3};
#pragma unroll
                    for (int u = 0; u < 3; u++)
                        if (b == u && c + hb[u] < need) {
                            c += hb[u];
                            b = u + 1;
                        }
                    sh.digit = 4 * lane + b;
                    sh.need = need - c;
                }
            }
            __syncthreads();
            prefix |= (uint32_t)sh.digit << shift;
            need = sh.need;
        }
        if (tid == 0) sh.nc = 0;
        __syncthreads();
        for_keys([&](uint64_t key, int row) {
            if ((uint32_t)(key >> 32) <= prefix) {
                const int p = atomicAdd(&sh.nc, 1);
                if (p < SEL_CAND) {
                    sh.ck[p] = key;
                    sh.ci[p] = row;
                }
            }
        });
        __syncthreads();
        const int L = sh.nc;
        if (L <= SEL_CAND) {   // uniform
            for (int t = tid; t < L; t += 256) {
                const uint64_t k0 = sh.ck[t];
                const int i0 = sh.ci[t];
                int rank = 0;
#pragma unroll 8
                for (int u = 0; u < L; u++) rank += key_less(sh.ck[u], sh.ci[u], k0, i0);
                if (rank < m) {
                    sel[rank] = i0;
                    seld[rank] = __longlong_as_double((long long)k0);
                }
            }
            done = true;
        }
    }
    // 1) each 16-lane row of the workgroup: its m best (key, index) pairs among its lanes' rows
    //    (row r of the training set belongs to thread r % 256), in ascending order, by m rounds of
    //    "smallest pair strictly after the previous pick" with a 4-level DPP row minimum
    if (!done) {
        const int grp = tid >> 4;
        if constexpr (K > 0) {
            // sort the thread's K pairs once (odd-even transposition; an empty slot, row -1, sorts
            // last), then every round only the lanes' heads compete: the 16-lane minimum is the
            // row's next pick and its owner pops its head (~3x fewer instructions per round than
            // rescanning all K keys against the previous pick)
#pragma unroll
            for (int p = 0; p < K; p++) {
#pragma unroll
                for (int j = p & 1; j + 1 < K; j += 2) {
                    const bool sw = (kr[j + 1] >= 0) & ((kr[j] < 0) | key_less(kv[j + 1], kr[j + 1], kv[j], kr[j]));
                    const uint64_t tk = kv[j];
                    const int ti = kr[j];
                    kv[j] = sw ? kv[j + 1] : kv[j];
                    kr[j] = sw ? kr[j + 1] : kr[j];
                    kv[j + 1] = sw ? tk : kv[j + 1];
                    kr[j + 1] = sw ? ti : kr[j + 1];
                }
            }
            for (int k = 0; k < m; k++) {
                uint64_t bk = kv[0];
                int bi = kr[0];
                row_key_min(bk, bi);
                if ((tid & 15) == 0) {
                    rk[grp][k] = bk;
                    ri[grp][k] = bi;
                }
                const bool pop = (bi >= 0) & (kr[0] == bi);   // rows are distinct: one owner
#pragma unroll
                for (int j = 0; j + 1 < K; j++) {
                    kv[j] = pop ? kv[j + 1] : kv[j];
                    kr[j] = pop ? kr[j + 1] : kr[j];
                }
                kv[K - 1] = pop ? 0 : kv[K - 1];
                kr[K - 1] = pop ? -1 : kr[K - 1];
            }
        } else {
            uint64_t pk = 0;   // (0, -1) precedes every (key, row >= 0)
            int pi = -1;
            for (int k = 0; k < m; k++) {
                uint64_t bk = 0;
                int bi = -1;
                for (int r = tid; r < rows; r += 256) {
                    const uint64_t v = dist_key(dist[r]);
                    key_take(bk, bi, v, key_less(pk, pi, v, r) ? r : -1);
                }
                row_key_min(bk, bi);
                if ((tid & 15) == 0) {
                    rk[grp][k] = bk;
                    ri[grp][k] = bi;
                }
                if (bi >= 0) {   // an exhausted row keeps its last pick (no re-picking from the start)
                    pk = bk;
                    pi = bi;
                }
            }
        }
    }
    __syncthreads();
    SEL_MARK(0);
    // 2) each wave merges its 4 row lists by rank (a pair's rank = how many valid pairs precede
    //    it; pairs are distinct, so ranks are too), 3) wave 0 merges the 4 wave lists the same way
    if (!done) {   // uniform
        for (int t = lane; t < m; t += 64) wi[wid][t] = -1;
        rank_merge(&rk[4 * wid], &ri[4 * wid], m, lane, wk[wid], wi[wid]);
        __syncthreads();
        if (wid == 0) rank_merge(wk, wi, m, lane, (uint64_t *)nullptr, sel, seld);
        __syncthreads();
    }
    for (int k = tid; k < m; k += 256) {
        idx_out[k] = sel[k];
        if (dist_out) dist_out[k] = seld[k];
    }
    SEL_MARK(1);
    // the hit code; with hm, whether this select also finishes the mean (the prediction it hit is
    // prepared).  Without it the host flag is written here; with it, after the mean.
    __shared__ int s_hm;
    if (hit_flag && wid == 0) {   // lane k compares entry k of the lists: one round trip, not m
        bool ne1 = false, ne2 = spec2_idx == nullptr;
        for (int k = lane; k < m; k += 64) {
            const int v = sel[k];
            ne1 |= v != spec_idx[k];
            if (spec2_idx) ne2 |= v != spec2_idx[k];
        }
        const bool hit1 = __ballot(ne1) == 0, hit2 = __ballot(ne2) == 0;
        const int hit = hit1 ? 1 : (hit2 ? 2 : 0);
        if (lane == 0) {
            *hit_flag = hit;
            int hmv = 0;
            if (hm && hit != 0) {
                const double *ap = hit == 1 ? hm->AP1 : hm->AP2;
                const int32_t *dn = hit == 1 ? hm->done1 : hm->done2;
                if (ap && __hip_atomic_load(dn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= hm->target) {
                    __threadfence();   // the prepared coordinates before their count
                    hmv = hit;
                }
            }
            s_hm = hmv;
            // a select that finishes the mean says so on the device too (code 3 / 4): it computes no
            // y_m / D2, so a mean kernel queued behind it (the look-ahead's form 1) must not run
            if (hmv != 0) *hit_flag = hmv + 2;
            if (host_flag && hmv == 0) __hip_atomic_store(host_flag, hit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    } else if (tid == 0) {
        s_hm = 0;
    }
    __syncthreads();
    const int hm_hit = s_hm;   // uniform: 1 / 2 = finish the mean from AP1 / AP2 below
    // the gathers of the m selected rows: SG loads in flight per thread before their stores (a
    // load -> store per trip would wait out one memory latency per element)
    constexpr int SG = 8;
    const int md = m * d;
    if (ymT && hm_hit == 0) {   // coalesced row reads, transposed writes (a finished hit reads none)
        for (int t0 = tid; t0 < md; t0 += 256 * SG) {
            double v[SG];
#pragma unroll
            for (int u = 0; u < SG; u++) {
                const int t = t0 + 256 * u, r = t / d, c = t - r * d;
                if (t < md) v[u] = Y[(int64_t)sel[r] * d + c];
            }
#pragma unroll
            for (int u = 0; u < SG; u++) {
                const int t = t0 + 256 * u, r = t / d, c = t - r * d;
                if (t < md) ymT[c * m + r] = v[u];
            }
        }
    }
    if (D2) {
        // lower triangle incl. diagonal, mirrored ((a-b)^2 == (b-a)^2 bitwise); the m neighbour
        // rows are staged in LDS with coalesced loads when they fit (xs_doubles), at a row stride
        // of d+1 doubles so that lanes reading different rows hit different banks
        extern __shared__ __attribute__((aligned(16))) double xs[];
        const int ds = d + 1;
        const bool staged = (int64_t)m * ds <= xs_doubles;
        if (staged)
            for (int t0 = tid; t0 < md; t0 += 256 * SG) {
                double v[SG];
#pragma unroll
                for (int u = 0; u < SG; u++) {
                    const int t = t0 + 256 * u, r = t / d, c = t - r * d;
                    if (t < md) v[u] = X[(int64_t)sel[r] * d + c];
                }
#pragma unroll
                for (int u = 0; u < SG; u++) {
                    const int t = t0 + 256 * u, r = t / d, c = t - r * d;
                    if (t < md) xs[r * ds + c] = v[u];
                }
            }
        __syncthreads();
        SEL_MARK(2);
        // the pairs, then kd2 on the next tasks
        const int npairs = m * (m + 1) / 2;
        const int ntask = npairs + (kd2 ? m : 0);
        if (staged && d >= 8 && d <= 128) {   // an octet of lanes per pair (pw_leaf_octet)
            const int j8 = tid & 7;
            // a finished hit needs kd2 only (its D2 is the prepared prediction's): tasks npairs..
            const int t0 = hm_hit != 0 ? npairs : 0;
            const int nrnd = (ntask - t0 + 31) / 32;   // whole octets iterate together
            for (int rd = 0; rd < nrnd; rd++) {
                const int t = t0 + rd * 32 + (tid >> 3);
                const bool valid = t < ntask;
                const bool is_kd = valid && t >= npairs;
                int r = 0, jj = 0;
                if (valid && !is_kd) {
                    while ((r + 1) * (r + 2) / 2 <= t) r++;
                    jj = t - r * (r + 1) / 2;
                } else if (is_kd) {
                    r = t - npairs;
                }
                const double *xr = xs + (size_t)r * ds;
                const double *xj = is_kd ? q : xs + (size_t)jj * ds;
                const double v = pw_leaf_octet(xr, xj, d, j8);
                if (valid && j8 == 0) {
                    if (is_kd) {
                        kd2[r] = v;
                    } else {
                        D2[r * m + jj] = v;
                        D2[jj * m + r] = v;
                    }
                }
            }
        } else if constexpr (GENERIC_D2) {   // the fused chain: any d, staged or not
        for (int t = tid; t < ntask; t += 256) {
            if (t >= npairs) {
                const int r = t - npairs;
                kd2[r] = pw_sqdiff(staged ? xs + (size_t)r * ds : X + (int64_t)sel[r] * d, q, d);
                continue;
            }
            int r = 0;
            while ((r + 1) * (r + 2) / 2 <= t) r++;
            const int j = t - r * (r + 1) / 2;
            const double *xr = staged ? xs + (size_t)r * ds : X + (int64_t)sel[r] * d;
            const double *xj = staged ? xs + (size_t)j * ds : X + (int64_t)sel[j] * d;
            const double v = pw_sqdiff(xr, xj, d);
            D2[r * m + j] = v;
            D2[j * m + r] = v;
        }
        } else {   // d < 8, staged (the host's contract for this kernel): pw_leaf's sequential branch
        for (int t = tid; t < ntask; t += 256) {
            int r = 0, j = 0;
            const double *xj = q;
            if (t >= npairs) {
                r = t - npairs;
            } else {
                while ((r + 1) * (r + 2) / 2 <= t) r++;
                j = t - r * (r + 1) / 2;
                xj = xs + (size_t)j * ds;
            }
            const double *xr = xs + (size_t)r * ds;
            double res = 0.;
            for (int i = 0; i < d; i++) {
                const double u = xr[i] - xj[i];
                res += u * u;
            }
            if (t >= npairs) {
                kd2[r] = res;
            } else {
                D2[r * m + j] = res;
                D2[j * m + r] = res;
            }
        }
        }
    }
    __syncthreads();
    SEL_MARK(3);
#undef SEL_MARK
    if (hm_hit != 0) {   // gp_mean_dev's output for every coordinate, from the prepared halves
        const double *AP = hm_hit == 1 ? hm->AP1 : hm->AP2;
        const int l = tid & 15, grp = tid >> 4, maxm = hm->maxm, rpl = (maxm + 15) / 16, st = HM_STRIDE(maxm);
        const bool big = maxm > 32;
        double kd[4];
#pragma unroll
        for (int s = 0; s < 4; s++) kd[s] = kd2[l + 16 * s < m ? l + 16 * s : 0];
        // CH coordinates per group at a time, all their loads issued before the sums; every group
        // runs every trip (the DPP row sums)
        constexpr int CH = 4;
        for (int c0 = 0; c0 < d; c0 += 16 * CH) {
            double al[CH][4], cq[CH], ps[CH], okv[CH];
#pragma unroll
            for (int u = 0; u < CH; u++) {
                const int c = c0 + 16 * u + grp;
                const double *ap = AP + (int64_t)(c < d ? c : 0) * st;
#pragma unroll
                for (int s = 0; s < 4; s++) {
                    const int row = l + 16 * s;
                    al[u][s] = (s < rpl && row < maxm) ? ap[row] : 0.0;
                }
                cq[u] = ap[maxm];
                ps[u] = ap[maxm + 1];
                okv[u] = ap[maxm + 2];
            }
#pragma unroll
            for (int u = 0; u < CH; u++) {
                const int c = c0 + 16 * u + grp;
                const double mean = gp_mean_finish<4>(m, l, rpl, big, kd, cq[u], ps[u], al[u], okv[u] != 0.0);
                if (c < d && l == 0) {
                    hm->preds[c] = mean;
                    hm->out[c] = mean + hm->bias[c];
                }
            }
        }
        __syncthreads();
        if (tid == 0 && host_flag) {   // the mean is in U1[i+1] (stream-ordered for the next slice)
            __threadfence();
            __hip_atomic_store(host_flag, hm_hit + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

template <int K>
__global__ void __launch_bounds__(256) knn_select_kernel(
    const double *__restrict__ dist, int64_t rows, int m, const double *__restrict__ X,
    const double *__restrict__ Y, int d, const double *__restrict__ q, int32_t *__restrict__ idx_out,
    double *__restrict__ dist_out, double *__restrict__ ymT, double *__restrict__ D2,
    double *__restrict__ kd2, const int32_t *__restrict__ spec_idx, int32_t *__restrict__ hit_flag,
    int xs_doubles, const int32_t *__restrict__ spec2_idx, int32_t *host_flag, HitMean hm, int key_lds) {
    __shared__ SelShm sh;
    const int qy = blockIdx.y;
    dist += (size_t)qy * rows;
    q += (size_t)qy * d;
    idx_out += (size_t)qy * m;
    if (dist_out) dist_out += (size_t)qy * m;
    if (ymT) ymT += (size_t)qy * d * m;
    if (D2) D2 += (size_t)qy * m * m;
    if (kd2) kd2 += (size_t)qy * m;
    uint64_t *mk = hm.marks;
    if (mk && threadIdx.x == 0) {
        const uint64_t t0 = wall_clock64();
        for (int k = 0; k < 5; k++) mk[k] -= t0;
        mk[5] += 1;
    }
    knn_select_dev<K, false>(sh, dist, rows, m, X, Y, d, q, idx_out, dist_out, ymT, D2, kd2, spec_idx, hit_flag,
                      xs_doubles, spec2_idx, host_flag, mk, hm.out ? &hm : nullptr,
                      K == 0 && key_lds != 0);
    if (mk && threadIdx.x == 0) mk[4] += wall_clock64();
}

static uint64_t *g_sel_marks = nullptr;
static int g_sel_marks_dev = -1;

uint64_t *sel_prof_marks() {
    if (env_int("NNGP_SEL_PROF", 0) == 0) return nullptr;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    if (g_sel_marks_dev != dev) {
        if (hipMalloc((void **)&g_sel_marks, 6 * sizeof(uint64_t)) != hipSuccess) return nullptr;
        if (hipMemset(g_sel_marks, 0, 6 * sizeof(uint64_t)) != hipSuccess) return nullptr;
        g_sel_marks_dev = dev;
    }
    return g_sel_marks;
}

void sel_prof_report(const char *what) {
    uint64_t *mk = sel_prof_marks();
    if (!mk) return;
    uint64_t h[6] = {0, 0, 0, 0, 0, 0};
    if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(h, mk, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return;
    (void)hipMemset(mk, 0, sizeof(h));
    const double n = h[5] ? (double)h[5] : 1.0, us = 1e3 / device_wallclock_khz();
    fprintf(stderr, "select profile %s: %llu launches, us per launch from its start: rounds %.2f merges %.2f "
            "gathers %.2f D2/kd2 %.2f end %.2f\n", what, (unsigned long long)h[5], (int64_t)h[0] * us / n,
            (int64_t)h[1] * us / n, (int64_t)h[2] * us / n, (int64_t)h[3] * us / n, (int64_t)h[4] * us / n);
}

// D2 / kd2 of the selected rows by one thread per pair (pw_sqdiff, reading X): the select's former
// in-kernel path for rows it cannot stage or d > 128, kept for NNGP_D2_WAVES=0 (query blockIdx.y;
// kd2 may be null).  Out of the select kernel its recursion stack no longer sets the select's
// register count (288 VGPRs with it, ~40 without: the select then fits beside the overlapped
// batch's fit waves).
__global__ void __launch_bounds__(256) d2_pairs_kernel(const double *__restrict__ X, const int32_t *__restrict__ idx,
                                                       int m, int d, const double *__restrict__ q,
                                                       double *__restrict__ D2, double *__restrict__ kd2) {
    const int qy = blockIdx.y;
    idx += (size_t)qy * m;
    q += (size_t)qy * d;
    D2 += (size_t)qy * m * m;
    if (kd2) kd2 += (size_t)qy * m;
    const int npairs = m * (m + 1) / 2;
    const int ntask = npairs + (kd2 ? m : 0);
    for (int t = blockIdx.x * 256 + threadIdx.x; t < ntask; t += gridDim.x * 256) {
        if (t >= npairs) {
            const int r = t - npairs;
            kd2[r] = pw_sqdiff(X + (int64_t)idx[r] * d, q, d);
            continue;
        }
        int r = 0;
        while ((r + 1) * (r + 2) / 2 <= t) r++;
        const int j = t - r * (r + 1) / 2;
        const double v = pw_sqdiff(X + (int64_t)idx[r] * d, X + (int64_t)idx[j] * d, d);
        D2[r * m + j] = v;
        D2[j * m + r] = v;
    }
}

// D2 / kd2 of the m selected rows when d > 128 or the rows do not fit the select's LDS staging:
// ONE WAVE per pair (blockIdx.x < m(m+1)/2) or per kd2 row (the next m blocks), query blockIdx.y.
// The pair's numpy leaves (pw_walk) go to the wave's 8 octets (pw_leaf_octet; a leaf is >= 64
// terms here), their values to LDS, and lane 0 combines them in the recursion's order: bitwise
// pw_sqdiff, with 64 lanes and all loads in flight instead of one lane walking d terms
// (FHN-PDE d = 800, m = 20: 230 such sums per prediction).
__global__ void __launch_bounds__(64) d2_wave_kernel(const double *__restrict__ X, const int32_t *__restrict__ idx,
                                                     int m, int d, const double *__restrict__ q,
                                                     double *__restrict__ D2, double *__restrict__ kd2) {
    __shared__ double leafv[16];
    __shared__ int leafo[16], leafl[16];
    __shared__ int nleaf;
    const int qy = blockIdx.y;
    idx += (size_t)qy * m;
    q += (size_t)qy * d;
    D2 += (size_t)qy * m * m;
    if (kd2) kd2 += (size_t)qy * m;
    const int t = blockIdx.x, lane = threadIdx.x;
    const int npairs = m * (m + 1) / 2;
    int r = 0, j = 0;
    const bool is_kd = t >= npairs;
    if (!is_kd) {
        while ((r + 1) * (r + 2) / 2 <= t) r++;
        j = t - r * (r + 1) / 2;
    } else {
        r = t - npairs;
    }
    const double *a = X + (int64_t)idx[r] * d;
    const double *b = is_kd ? q : X + (int64_t)idx[j] * d;
    if (lane == 0) {   // the leaves, left to right
        int k = 0;
        pw_walk(d, [&](int o, int l) {
            leafo[k] = o;
            leafl[k] = l;
            k++;
            return 0.0;
        });
        nleaf = k;
    }
    __syncthreads();
    const int nl = nleaf;
    for (int base = 0; base < nl; base += 8) {   // octet o computes leaf base + o
        const int lf = base + (lane >> 3);
        const bool ok = lf < nl;
        const int o = ok ? leafo[lf] : 0, l = ok ? leafl[lf] : 8;
        double v;
        if (l >= 8) v = pw_leaf_octet(a + o, b + o, l, lane & 7);
        else v = pw_leaf(a + o, b + o, l);   // (d < 8: one leaf)
        if (ok && (lane & 7) == 0) leafv[lf] = v;
    }
    __syncthreads();
    if (lane == 0) {
        int k = 0;
        const double v = pw_walk(d, [&](int, int) { return leafv[k++]; });
        if (is_kd) {
            kd2[r] = v;
        } else {
            D2[r * m + j] = v;
            D2[j * m + r] = v;
        }
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


// Nelder-Mead state machine: nngp_nm.h

// register budget: MAXM <= 16 fits 256 VGPRs (<= 512 threads), MAXM <= 32 needs up to 512 (256);
// MAXM > 32 (3-4 rows per lane) runs one wave per workgroup (LDS: four fit images, all registers)
// (a 168-VGPR cap at MAXM <= 16 -- 3 waves per SIMD, a few spills -- made the Burgers batch fits
// 12 % faster but starved the sweep's G launches running beside them: 0.258 -> 0.282 s end to end,
// tools/sessions/r4n.sh)
template <int MAXM> struct NMBound { static constexpr int T = (MAXM <= 16) ? 512 : (MAXM <= 32 ? 256 : 64); };
// threads of the wave-per-fit speculative kernel and of the mean kernel
template <int MAXM> struct WGT { static constexpr int T = MAXM > 32 ? 64 : 256; };

template <int MAXM, bool FUSED>
__global__ void __launch_bounds__(NMBound<MAXM>::T) nm_fit_kernel(NMArgs a) {
    constexpr int RPL = GP<MAXM>::RPL, IMG = GP<MAXM>::IMG;
    extern __shared__ __attribute__((aligned(16))) double sm[];
    if (a.skip && *a.skip) return;   // uniform: the whole grid exits
    nm_batch_offsets(a);
    const int m = a.m;
    const int nfc = a.nj * a.R;                         // fits per coordinate
    const int galloc = blockDim.x / 16;                 // groups incl. padding lanes
    const int ngroups = FUSED ? a.cpw * nfc : galloc;
    double *sD2 = sm;
    double *skd2 = sD2 + m * m;
    double *sRes = skd2 + m;                            // [galloc][4]
    double *sK = sRes + galloc * 4;                     // [galloc][IMG]
    const int tid = threadIdx.x;
    const int g = tid / 16;                             // group (= DPP row) in block
    const int l = tid % 16;

    __shared__ double sJit[MAX_JIT];   // the jitter powers, so a refill reads one LDS word
    for (int i = tid; i < m * m; i += blockDim.x) sD2[i] = a.D2[i];
    if (FUSED)
        for (int i = tid; i < m; i += blockDim.x) skd2[i] = a.kd2[i];
    if (tid < MAX_JIT) sJit[tid] = jit_lookup(a, tid);
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
            if (valid && a.jmajor && !a.coord) f = (f % a.d) * nfc + f / a.d;
        }
    }
    double y[RPL];
    double jit = 1.0;
    double *Kimg = sK + (size_t)g * IMG;
    GPLane<MAXM> P;
    gp_lane_init<MAXM>(P, m, l);
    gp_image_init<MAXM>(Kimg, m, l);
    NMCfg cfg{a.fatol, a.xatol, a.maxfev, a.maxfev};
    NM St;
    bool parked = false;
    // (re)start this row on fit f: its coordinate column, jitter and initial simplex
    auto start_fit = [&]() {
        parked = false;
        if (!FUSED && valid) {
            if (a.coord) {
                coord = a.coord[f];
                jidx = a.jitter_idx[f];
            } else {   // product(coord, jitter, restart) order (models.py:186)
                coord = f / nfc;
                jidx = (f % nfc) / a.R;
            }
        }
#pragma unroll
        for (int s2 = 0; s2 < RPL; s2++) {
            const int row = l + 16 * s2;
            y[s2] = (valid && row < m) ? a.Y[(int64_t)coord * a.ys_c + (int64_t)row * a.ys_r] : 0.0;
        }
        jit = valid ? sJit[jidx] : 1.0;
        St.f0 = St.f1 = St.f2 = INFINITY;
        St.xbx = St.xby = St.xrx = St.xry = St.fxr = 0.0;
        if (valid) {
            nm_start(St, cfg, a.theta0[2 * f], a.theta0[2 * f + 1]);
        } else {
            St.s0x = St.s0y = St.s1x = St.s1y = St.s2x = St.s2y = 0.0;
            St.px = St.py = 0.0;
            St.fcalls = St.iters = 0;
            St.st = ST_DONE;
        }
    };
    auto write_fit = [&]() {
        const double fval = (St.f1 != St.f1 || St.f2 != St.f2) ? NAN : St.f0;
        if (valid && l == 0 && !parked) {
            if (a.theta_out) { a.theta_out[2 * f] = St.s0x; a.theta_out[2 * f + 1] = St.s0y; }
            if (a.fval_out) a.fval_out[f] = fval;
            if (a.nfev_out) a.nfev_out[f] = St.fcalls;
            if (a.fits_out) {
                a.fits_out[4 * f + 0] = St.s0x;
                a.fits_out[4 * f + 1] = St.s0y;
                a.fits_out[4 * f + 2] = fval;
                a.fits_out[4 * f + 3] = (double)St.fcalls;
            }
            if (!FUSED && a.done) {   // the fit is visible device-wide before it is counted
                __threadfence();
                __hip_atomic_fetch_add(a.done + blockIdx.y, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            if (FUSED) {
                sRes[4 * g + 0] = St.s0x;
                sRes[4 * g + 1] = St.s0y;
                sRes[4 * g + 2] = fval;
            }
        }
    };
    start_fit();
    // every group of the wave evaluates once per trip until the wave's last fit is done, so the
    // evaluation code never diverges (finished groups evaluate a dummy point).  With a work queue
    // a finished group first takes the next unassigned fit of its prediction (a fit's arithmetic
    // does not depend on which group runs it), so the wave's groups stay busy to the end.
    bool can_take = !FUSED && a.queue != nullptr && g < ngroups;
    while (true) {
        if (!FUSED && can_take && St.st == ST_DONE) {   // uniform within the group
            write_fit();
            int fn = 0;
            if (l == 0) fn = (int)(gridDim.x * ngroups) + atomicAdd(a.queue + blockIdx.y, 1);
            fn = __builtin_amdgcn_mov_dpp(fn, 0x150, 0xF, 0xF, false);   // row_newbcast:0
            f = fn;
            valid = fn < a.n_fits;
            if (valid && a.jmajor && !a.coord) f = (fn % a.d) * nfc + fn / a.d;
            can_take = valid;
            start_fit();
        }
        const bool need = St.st != ST_DONE;
        if (!__any(need)) break;
        const double fv = gp_nlml<MAXM>(m, l, P, sD2, St.px, St.py, jit, y, Kimg);
        if (need) {
            nm_consume(St, cfg, fv);
            if (!FUSED && a.park_cap && St.st != ST_DONE && St.fcalls >= a.park_cap) {
                // a long fit: park it (state with its pending request) for the speculative kernel,
                // which finishes it a wave per fit in ~1.5x fewer rounds, so this wave's tail does
                // not set the launch's length (uniform within the group)
                // (finite simplices from the front of park_list, all-+inf ones -- which run to
                // maxfev -- from the back: the resume gives them different shapes)
                if (l == 0) {
                    a.park[f] = St;
                    if (St.f0 == INFINITY && St.f1 == INFINITY && St.f2 == INFINITY)
                        a.park_list[a.n_fits - 1 - atomicAdd(a.park_count + 1, 1)] = f;
                    else
                        a.park_list[atomicAdd(a.park_count, 1)] = f;
                }
                parked = true;
                St.st = ST_DONE;
            }
        }
    }
    write_fit();
    if constexpr (!FUSED) return;
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
        const double jb = sJit[best / a.R];
        const double mean = gp_mean<MAXM>(m, l, P, sD2, skd2, sx, sy, jb, y, Kimg);
        if (l == 0) {
            a.preds[coord] = mean;
            if (a.out) a.out[coord] = a.bias ? mean + a.bias[coord] : mean;
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Speculative Nelder-Mead: one WAVE per fit, its four 16-lane rows evaluating up to four points
// per round.  A Nelder-Mead iteration of scipy's algorithm needs f at the reflection and then,
// depending on it, at the expansion, the outside or the inside contraction -- all four computable
// from the same centroid and worst vertex -- so a round evaluates all of them and the unchanged
// state machine (nm_consume) then consumes them in scipy's order, taking each value from the round
// as if it had just been requested.  Shrinks (two new vertices) and the initial simplex (three
// points) are one round each.  Only requested points count towards nfev / maxfev, so every fit
// returns exactly what the one-row kernel (and scipy) returns, in ~1.5x fewer sequential rounds.
// Used when there are few enough fits that a wave per fit does not oversubscribe the SIMDs.
// ---------------------------------------------------------------------------------------------
struct NMCand {
    double x, y;
    int st;   // the state whose request this value answers (-1: none / consumed)
};

// candidate set for the pending request of S (cand[0] is the request itself)
__device__ __forceinline__ int nm_candidates(const NM &S, NMCand (&c)[4]) {
    c[0] = NMCand{S.px, S.py, S.st};
    c[1] = c[2] = c[3] = NMCand{S.px, S.py, -1};
    switch (S.st) {
    case ST_INIT0:   // x0 -> x1, x2 (the initial simplex)
        c[1] = NMCand{S.s1x, S.s1y, ST_INIT1};
        c[2] = NMCand{S.s2x, S.s2y, ST_INIT2};
        return 3;
    case ST_REFLECT:   // same expressions as nm_consume's ST_REFLECT branch
        if (S.f0 == INFINITY && S.f1 == INFINITY && S.f2 == INFINITY) {
            // an all-+inf simplex (the jittered kernel fails the Cholesky at every vertex so far;
            // ~8 % of an FHN-PDE d = 800 correction's fits, which then run to maxfev): if the
            // reflection is +inf too, scipy takes the inside contraction (fxr >= f2), and if that
            // is +inf the shrink's two points -- one iteration in ONE round instead of two.  A finite
            // reflection takes the expansion instead, answered in the next round as before.
            c[1] = NMCand{0.5 * S.xbx + 0.5 * S.s2x, 0.5 * S.xby + 0.5 * S.s2y, ST_ICONTRACT};
            c[2] = NMCand{S.s0x + 0.5 * (S.s1x - S.s0x), S.s0y + 0.5 * (S.s1y - S.s0y), ST_SHRINK1};
            c[3] = NMCand{S.s0x + 0.5 * (S.s2x - S.s0x), S.s0y + 0.5 * (S.s2y - S.s0y), ST_SHRINK2};
            return 4;
        }
        c[1] = NMCand{3 * S.xbx - 2 * S.s2x, 3 * S.xby - 2 * S.s2y, ST_EXPAND};
        c[2] = NMCand{1.5 * S.xbx - 0.5 * S.s2x, 1.5 * S.xby - 0.5 * S.s2y, ST_CONTRACT};
        c[3] = NMCand{0.5 * S.xbx + 0.5 * S.s2x, 0.5 * S.xby + 0.5 * S.s2y, ST_ICONTRACT};
        return 4;
    case ST_SHRINK1:   // the second shrunk vertex, as nm_consume's ST_SHRINK1 computes it
        c[1] = NMCand{S.s0x + 0.5 * (S.s2x - S.s0x), S.s0y + 0.5 * (S.s2y - S.s0y), ST_SHRINK2};
        return 2;
    default:
        return 1;
    }
}

template <int MAXM>
__global__ void __launch_bounds__(WGT<MAXM>::T) nm_spec_kernel(NMArgs a) {
    constexpr int RPL = GP<MAXM>::RPL, IMG = GP<MAXM>::IMG;
    extern __shared__ __attribute__((aligned(16))) double sm[];
    if (a.skip && *a.skip) return;   // uniform: the whole grid exits (speculation hit)
    nm_batch_offsets(a);
    const int m = a.m;
    const int nfc = a.nj * a.R;
    double *sD2 = sm;
    double *sK = sD2 + m * m;                           // [blockDim/16][IMG]
    const int tid = threadIdx.x;
    const int g = (tid & 63) / 16;                      // row of the wave = candidate slot
    const int l = tid % 16;
    int f = blockIdx.x * (blockDim.x / 64) + tid / 64;   // one fit per wave
    for (int i = tid; i < m * m; i += blockDim.x) sD2[i] = a.D2[i];
    __syncthreads();
    if (a.resume) {                                      // the parked fits of the packed kernel
        const int nf = a.park_count[0];                  // finite ones first, then the all-+inf
        if (f >= nf + a.park_count[1]) return;
        f = f < nf ? a.park_list[f] : a.park_list[a.n_fits - 1 - (f - nf)];
    } else if (f >= a.n_fits) {
        return;                                          // whole wave exits together
    }
    int coord, jidx;
    if (a.coord) {
        coord = a.coord[f];
        jidx = a.jitter_idx[f];
    } else {   // product(coord, jitter, restart) order (models.py:186)
        coord = f / nfc;
        jidx = (f % nfc) / a.R;
    }
    double y[RPL];
#pragma unroll
    for (int s = 0; s < RPL; s++) {
        const int row = l + 16 * s;
        y[s] = (row < m) ? a.Y[(int64_t)coord * a.ys_c + (int64_t)row * a.ys_r] : 0.0;
    }
    const double jit = jit_lookup(a, jidx);
    double *Kimg = sK + (size_t)(tid / 16) * IMG;
    GPLane<MAXM> P;
    gp_lane_init<MAXM>(P, m, l);
    gp_image_init<MAXM>(Kimg, m, l);

    NMCfg cfg{a.fatol, a.xatol, a.maxfev, a.maxfev};
    NM St;
    if (a.resume) {
        St = a.park[f];   // pending request included: the loop below continues it unchanged
    } else {
        St.fcalls = 0;
        St.iters = 0;
        St.f0 = St.f1 = St.f2 = INFINITY;
        St.xbx = St.xby = St.xrx = St.xry = St.fxr = 0.0;
        const double t0x = a.theta0[2 * f], t0y = a.theta0[2 * f + 1];
        St.s0x = t0x; St.s0y = t0y;
        St.s1x = (t0x != 0) ? (1 + 0.05) * t0x : 0.00025; St.s1y = t0y;   // nonzdelt / zdelt
        St.s2x = t0x; St.s2y = (t0y != 0) ? (1 + 0.05) * t0y : 0.00025;
        St.st = ST_INIT0;
        if (!nm_req(St, cfg, St.s0x, St.s0y, ST_INIT0)) St.st = ST_DONE;
    }
    while (St.st != ST_DONE) {   // wave-uniform
        NMCand c[4];
        const int nc = nm_candidates(St, c);
        double mx = c[0].x, my = c[0].y;   // this row's candidate (static indices: no scratch)
#pragma unroll
        for (int k = 1; k < 4; k++)
            if (g == k && k < nc) {
                mx = c[k].x;
                my = c[k].y;
            }
        const double fv = gp_nlml<MAXM>(m, l, P, sD2, mx, my, jit, y, Kimg);
        double val[4];
#pragma unroll
        for (int k = 0; k < 4; k++) val[k] = wave_lane_double(fv, 16 * k);
        // consume every answered request in scipy's order
        while (St.st != ST_DONE) {
            int hit = -1;
#pragma unroll
            for (int k = 0; k < 4; k++)
                if (hit < 0 && k < nc && c[k].st == St.st && c[k].x == St.px && c[k].y == St.py) hit = k;
            if (hit < 0) break;
            double v = val[0];
#pragma unroll
            for (int k = 1; k < 4; k++)
                if (hit == k) v = val[k];
            nm_consume(St, cfg, v);
#pragma unroll
            for (int k = 0; k < 4; k++)
                if (hit == k) c[k].st = -1;
        }
    }
    const double fval = (St.f1 != St.f1 || St.f2 != St.f2) ? NAN : St.f0;
    if ((tid & 63) == 0) {
        if (a.theta_out) { a.theta_out[2 * f] = St.s0x; a.theta_out[2 * f + 1] = St.s0y; }
        if (a.fval_out) a.fval_out[f] = fval;
        if (a.nfev_out) a.nfev_out[f] = St.fcalls;
        if (a.fits_out) {
            a.fits_out[4 * f + 0] = St.s0x;
            a.fits_out[4 * f + 1] = St.s0y;
            a.fits_out[4 * f + 2] = fval;
            a.fits_out[4 * f + 3] = (double)St.fcalls;
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Two-level speculative Nelder-Mead: W waves (4 W rows) per fit, for few fits (a latency-bound
// correction: the slowest fit's chain of rounds is the correction's time).  Rows 0-3 take the
// one-level candidates above; while the request is a reflection from a finite simplex, rows 4..
// also take the NEXT iteration's reflection, expansion and both contractions for the likeliest
// outcomes of this one, each of which fixes the sorted simplex the next centroid is formed from:
//   set 1 (W >= 2): the reflection is accepted between the best and the middle vertex
//                   (f0 <= f(r) < f1: simplex s0, r, s1);
//   set 2 (W == 4): the inside contraction is accepted and is the new best (s_ic, s0, s1);
//   set 3 (W == 4): the inside contraction is accepted and stays the worst (s0, s1, s_ic).
// (Outcome frequencies on trajectory-like fits, tests/nm_spec_sim.py: reflection accepted 21 %,
// inside contraction 19-20 % best / 16-21 % worst, expansions 25-30 %.)  The candidates are formed
// with nm_check's own expressions, and the unchanged state machine consumes whatever was
// requested and answered, so a fit is bitwise the one-level kernel's (and scipy's); only requested
// points count towards nfev.  Simulated on those fits: the slowest fit's rounds 50 -> 28 (W = 4),
// 50 -> 36 (W = 2).  A round's candidates and values go through LDS; every wave of a fit runs the
// state machine redundantly on the same values.
// ---------------------------------------------------------------------------------------------
struct NMCand2 {
    double x, y, f;
    int st;
};

// the next iteration's candidates after p replaces the worst vertex and sorts to `rank` among
// (s0, s1) -- nm_end_iter + nm_check's expressions for that simplex
__device__ __forceinline__ void nm_next_set(const NM &S, double px, double py, int rank, NMCand2 *c) {
    double ax = S.s0x, ay = S.s0y, bx = S.s1x, by = S.s1y, wx = px, wy = py;   // rank 2
    if (rank == 0) { ax = px; ay = py; bx = S.s0x; by = S.s0y; wx = S.s1x; wy = S.s1y; }
    else if (rank == 1) { ax = S.s0x; ay = S.s0y; bx = px; by = py; wx = S.s1x; wy = S.s1y; }
    const double xbx = (ax + bx) / 2, xby = (ay + by) / 2;
    c[0] = NMCand2{2 * xbx - 1 * wx, 2 * xby - 1 * wy, 0.0, ST_REFLECT};
    c[1] = NMCand2{3 * xbx - 2 * wx, 3 * xby - 2 * wy, 0.0, ST_EXPAND};
    c[2] = NMCand2{1.5 * xbx - 0.5 * wx, 1.5 * xby - 0.5 * wy, 0.0, ST_CONTRACT};
    c[3] = NMCand2{0.5 * xbx + 0.5 * wx, 0.5 * xby + 0.5 * wy, 0.0, ST_ICONTRACT};
}

// this row's candidate (slot 0 .. 4W-1; st = -1: none).  Every lane forms all sets from the
// fit's (uniform) state and keeps its own slot's with static selects: a few dozen VALU per round
// against a likelihood evaluation's ~2 500, and no serial hand-off through one lane.
__device__ __forceinline__ NMCand2 nm_candidate_slot(const NM &S, const NMCfg &cfg, int slot, int W) {
    NMCand l1[4];
    if (W > 1 && slot >= 4 && S.st == ST_REFLECT && S.f0 == INFINITY && S.f1 == INFINITY && S.f2 == INFINITY) {
        // an all-+inf simplex (the fits that run to maxfev: the parked tail of a large correction):
        // wave w of the fit takes iteration w's requests as the state machine makes them if every
        // earlier request is +inf too -- it answers them on a copy with +inf (reflection, inside
        // contraction, both shrink points per iteration), so W iterations per round instead of one
        NM T = S;
        const int w = slot / 4;   // uniform over the wave
        for (int k = 0; k < 4 * w; k++)
            if (T.st != ST_DONE) nm_consume(T, cfg, INFINITY);
        NMCand2 c{S.px, S.py, 0.0, -1};
        if (T.st == ST_DONE) return c;
        const int nc = nm_candidates(T, l1);
#pragma unroll
        for (int k = 0; k < 4; k++)
            if ((slot & 3) == k && k < nc) c = NMCand2{l1[k].x, l1[k].y, 0.0, l1[k].st};
        return c;
    }
    nm_candidates(S, l1);
    NMCand2 c{S.px, S.py, 0.0, -1};
#pragma unroll
    for (int k = 0; k < 4; k++)
        if (slot == k) c = NMCand2{l1[k].x, l1[k].y, 0.0, l1[k].st};
    if (W == 1) return c;
    const bool lv2 = S.st == ST_REFLECT && !(S.f0 == INFINITY && S.f1 == INFINITY && S.f2 == INFINITY);
    if (!lv2 || slot < 4) return c;
    NMCand2 set[4];
    const int si = slot / 4;   // 1: reflection accepted (rank 1); 2 / 3: inside contraction best / worst
    const double xi = 0.5 * S.xbx + 0.5 * S.s2x, yi = 0.5 * S.xby + 0.5 * S.s2y;   // ST_ICONTRACT's point
    nm_next_set(S, si == 1 ? S.xrx : xi, si == 1 ? S.xry : yi, si == 1 ? 1 : (si == 2 ? 0 : 2), set);
#pragma unroll
    for (int k = 0; k < 4; k++)
        if ((slot & 3) == k) c = set[k];
    return c;
}

// W = 0: the resume of the packed kernel's parked fits, shapes chosen on the device from the
// parked counts -- the finite fits' workgroups first (4 waves per fit while they number <=
// resume_w4, 2 while <= resume_w2, else 1), then the all-+inf fits' (a wave each: one iteration
// is one round for them already, and their waves would only take issue slots from the finite
// chains); the grid covers the largest case and the rest of it exits at once.
template <int MAXM, int W>
__global__ void __launch_bounds__(256) nm_spec2_kernel(NMArgs a) {
    constexpr int RPL = GP<MAXM>::RPL, IMG = GP<MAXM>::IMG;
    extern __shared__ __attribute__((aligned(16))) double sm[];
    __shared__ NMCand2 sC[16];   // the round's candidates and their values: fit fs's at [4*Wr*fs, 4*Wr*(fs+1))
    if (a.skip && *a.skip) return;   // uniform: the whole grid exits (speculation hit)
    const int tid = threadIdx.x, wv = tid / 64;
    int Wr = W, f = 0;
    bool live = true;
    if (W == 0) {
        const int nf = a.park_count[0], ni = a.park_count[1];
        const int wf = nf <= a.resume_w4 ? 4 : (nf <= a.resume_w2 ? 2 : 1);
        const int nbf = (nf * wf + 3) / 4;   // workgroups of the finite fits
        const int b = blockIdx.x;
        if (b < nbf) {
            Wr = wf;
            const int i = b * (4 / wf) + wv / wf;
            live = i < nf;
            if (live) f = a.park_list[i];
        } else {
            if ((b - nbf) * 4 >= ni) return;   // uniform over the workgroup
            Wr = 1;
            const int i = (b - nbf) * 4 + wv;
            live = i < ni;
            if (live) f = a.park_list[a.n_fits - 1 - i];
        }
    } else {
        f = blockIdx.x * (4 / W) + wv / W;   // (never a resume: that is W = 0)
        live = f < a.n_fits;
    }
    nm_batch_offsets(a);
    const int m = a.m;
    const int nfc = a.nj * a.R;
    double *sD2 = sm;
    double *sK = sD2 + m * m;                           // [16][IMG]
    const int g = (tid & 63) / 16, l = tid % 16;
    const int fs = wv / Wr;                             // this wave's fit within the workgroup
    const int slot = (wv % Wr) * 4 + g;                 // this row's candidate slot
    NMCand2 *sCf = sC + 4 * Wr * fs;
    for (int i = tid; i < m * m; i += blockDim.x) sD2[i] = a.D2[i];
    const int fc = live ? f : 0;
    int coord, jidx;
    if (a.coord) {
        coord = a.coord[fc];
        jidx = a.jitter_idx[fc];
    } else {   // product(coord, jitter, restart) order (models.py:186)
        coord = fc / nfc;
        jidx = (fc % nfc) / a.R;
    }
    double y[RPL];
#pragma unroll
    for (int s = 0; s < RPL; s++) {
        const int row = l + 16 * s;
        y[s] = (row < m) ? a.Y[(int64_t)coord * a.ys_c + (int64_t)row * a.ys_r] : 0.0;
    }
    const double jit = jit_lookup(a, jidx);
    double *Kimg = sK + (size_t)(tid / 16) * IMG;
    GPLane<MAXM> P;
    gp_lane_init<MAXM>(P, m, l);
    gp_image_init<MAXM>(Kimg, m, l);

    NMCfg cfg{a.fatol, a.xatol, a.maxfev, a.maxfev};
    NM St;
    if (!live) {
        St.st = ST_DONE;
    } else if (a.resume) {
        St = a.park[f];
    } else {
        const double t0x = a.theta0[2 * f], t0y = a.theta0[2 * f + 1];
        St.f0 = St.f1 = St.f2 = INFINITY;
        St.xbx = St.xby = St.xrx = St.xry = St.fxr = 0.0;
        nm_start(St, cfg, t0x, t0y);
    }
    // workgroup-uniform rounds (a finished fit's rows evaluate a dummy point until all are done);
    // with one wave per fit (Wr == 1, uniform over the workgroup: the resume's one-wave fits) each
    // wave runs its own rounds and exchanges its candidates within the wave only
    const int lane = tid & 63;
    __syncthreads();   // sD2
    for (;;) {
        if (Wr == 1) {
            if (St.st == ST_DONE) break;
        } else if (!__syncthreads_or(St.st != ST_DONE)) {
            break;
        }
        const bool run = St.st != ST_DONE;   // uniform over the fit's waves
        const NMCand2 mine = run ? nm_candidate_slot(St, cfg, slot, Wr) : NMCand2{-1.0, -1.0, 0.0, -1};
        // unused slots evaluate the request itself (a duplicate; never matched)
        const double fv = gp_nlml<MAXM>(m, l, P, sD2, mine.st >= 0 ? mine.x : St.px,
                                        mine.st >= 0 ? mine.y : St.py, jit, y, Kimg);
        if (l == 0) sCf[slot] = NMCand2{mine.x, mine.y, fv, mine.st};
        if (Wr == 1) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        } else {
            __syncthreads();
        }
        // consume every answered request in scipy's order: lane k < 4W holds candidate k; the
        // lowest matching slot answers (the order a sequential scan would take)
        const NMCand2 ck = sCf[lane < 4 * Wr ? lane : 0];
        uint64_t used = 0;
        while (run && St.st != ST_DONE) {
            const bool match = lane < 4 * Wr && !((used >> lane) & 1) && ck.st == St.st && ck.x == St.px &&
                               ck.y == St.py;
            const uint64_t mk = __builtin_amdgcn_ballot_w64(match);
            if (!mk) break;
            const int hit = __builtin_ctzll(mk);
            used |= 1ull << hit;
            nm_consume(St, cfg, wave_lane_double(ck.f, hit));
        }
    }
    if (live && (tid & (64 * Wr - 1)) == 0) {
        const double fval = (St.f1 != St.f1 || St.f2 != St.f2) ? NAN : St.f0;
        if (a.theta_out) { a.theta_out[2 * f] = St.s0x; a.theta_out[2 * f + 1] = St.s0y; }
        if (a.fval_out) a.fval_out[f] = fval;
        if (a.nfev_out) a.nfev_out[f] = St.fcalls;
        if (a.fits_out) {
            a.fits_out[4 * f + 0] = St.s0x;
            a.fits_out[4 * f + 1] = St.s0y;
            a.fits_out[4 * f + 2] = fval;
            a.fits_out[4 * f + 3] = (double)St.fcalls;
        }
    }
}

// posterior mean per coordinate, one 16-lane group per coordinate (models.py:162-168, 217).
// (theta, jitter) either given (a.theta0[c], a.jitter_idx[c]: nngp_gp_mean) or the first arg-min
// of the coordinate's a.nj*a.R fits in a.fits_out (the unfused nngp_predict path, used when a
// coordinate's fits do not fit one workgroup).  Writes a.preds[c] and a.out[c] = mean (+ bias).
// workgroup blk's coordinates (the kernel's blockIdx.x; the correction chain loops over them).
// load_lds: stage D2/kd2 first (the chain stages them once per slice)
template <int MAXM>
__device__ __forceinline__ void gp_mean_dev(const NMArgs &a, int blk, bool load_lds) {
    constexpr int RPL = GP<MAXM>::RPL, IMG = GP<MAXM>::IMG;
    extern __shared__ __attribute__((aligned(16))) double sm[];
    const int m = a.m, d = a.d;
    double *sD2 = sm, *skd2 = sm + m * m, *sK = skd2 + m;
    const int tid = threadIdx.x, g = tid / 16, l = tid % 16;
    // the slice's select finished the mean itself (HitMean, hit code 3 / 4): nothing to do
    if (a.skip && __hip_atomic_load(a.skip, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= 3) return;
    if (a.wait_done) {   // a hit served by the overlapped batch: wait for its fits of this query
        __shared__ int s_late;
        if (tid == 0) {
            s_late = 0;
            if (__hip_atomic_load(a.skip, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 1) {
                // never a hang: past the deadline flag it and write nothing; the host redoes the
                // sweep without the overlap.  Once any slice has given up, later slices do not
                // wait at all (the rerun recomputes them).
                // wait_ticks == 0 (NNGP_SPEC_WAIT_US=0): give up at once, fits finished or not --
                // the deterministic way into the rerun path (tests)
                const uint64_t t0 = wall_clock64();
                while (a.wait_ticks == 0 ||
                       __hip_atomic_load(a.wait_done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < a.wait_n) {
                    if (a.wait_ticks == 0 || __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0 ||
                        wall_clock64() - t0 >= a.wait_ticks) {
                        s_late = 1;
                        __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(2);
                }
                __threadfence();
            }
        }
        __syncthreads();
        if (s_late) return;
    }
    if (load_lds) {
        for (int i = tid; i < m * m; i += blockDim.x) sD2[i] = a.D2[i];
        for (int i = tid; i < m; i += blockDim.x) skd2[i] = a.kd2[i];
        __syncthreads();
    }
    const int c = blk * (blockDim.x / 16) + g;
    const bool valid = c < d;
    const int cc = valid ? c : 0;
    double y[RPL];
#pragma unroll
    for (int s = 0; s < RPL; s++) {
        const int row = l + 16 * s;
        y[s] = (valid && row < m) ? a.Y[(int64_t)cc * a.ys_c + (int64_t)row * a.ys_r] : 0.0;
    }
    double sx, sy;
    int jidx;
    if (a.fits_out) {
        const int nfc = a.nj * a.R;
        const int sk = a.skip ? *a.skip : 0;
        const double *FB = sk == 0 ? a.fits_out : (sk == 2 ? a.fits_alt2 : a.fits_alt);
        const double *F = FB + (size_t)4 * cc * nfc;
        // arg-min of fval with the sequential scan's semantics (models.py:205-207 np.argmin over
        // a scan "if f < best"): a NaN first value wins, NaNs never do later, ties keep the first.
        // The row's lanes load the values together and reduce (key, index) pairs.
        uint64_t bk = ~0ull;
        int bi = -1;
        for (int t = l; t < nfc; t += 16) key_take(bk, bi, fval_key(F[4 * t + 2]), t);
        row_key_min(bk, bi);
        const double f0 = F[2];
        const int best = (f0 != f0) ? 0 : bi;
        sx = F[4 * best];
        sy = F[4 * best + 1];
        jidx = best / a.R;
    } else {
        sx = a.theta0[2 * cc];
        sy = a.theta0[2 * cc + 1];
        jidx = a.jitter_idx[cc];
    }
    GPLane<MAXM> P;
    gp_lane_init<MAXM>(P, m, l);
    double *Kimg = sK + (size_t)g * IMG;
    gp_image_init<MAXM>(Kimg, m, l);
    const double mean = gp_mean<MAXM>(m, l, P, sD2, skd2, sx, sy, jit_lookup(a, jidx), y, Kimg);
    if (valid && l == 0) {
        if (a.preds) a.preds[c] = mean;
        if (a.out) a.out[c] = a.bias ? mean + a.bias[c] : mean;
    }
}

template <int MAXM>
__global__ void __launch_bounds__(WGT<MAXM>::T) gp_mean_kernel(NMArgs a) {
    gp_mean_dev<MAXM>(a, blockIdx.x, true);
}

// The query-independent half of gp_mean_dev for every coordinate of a speculative batch's
// predictions (blockIdx.y = prediction, batched offsets as the fits kernels): the first arg-min
// over the prediction's fits, then gp_mean_prep.  AP[q][c] = alpha rows 0..MAXM-1 | c | psy | ok
// (HM_STRIDE(MAXM) doubles); pre_done[q] counts the finished workgroups.  A sweep slice whose
// ordered list hits this prediction finishes its mean in the select kernel (knn_select_dev's
// HitMean) from these values and its own kd2 -- bitwise gp_mean_dev, which computes the same
// arg-min and prep on the same D2, y and fits.
template <int MAXM>
__global__ void __launch_bounds__(WGT<MAXM>::T) gp_pre_kernel(NMArgs a, double *__restrict__ AP,
                                                              int32_t *__restrict__ pre_done) {
    constexpr int RPL = GP<MAXM>::RPL, IMG = GP<MAXM>::IMG;
    extern __shared__ __attribute__((aligned(16))) double sm[];
    nm_batch_offsets(a);
    const int m = a.m, d = a.d;
    double *sD2 = sm, *sK = sm + m * m;
    const int tid = threadIdx.x, g = tid / 16, l = tid % 16;
    for (int i = tid; i < m * m; i += blockDim.x) sD2[i] = a.D2[i];
    __syncthreads();
    const int c = blockIdx.x * (blockDim.x / 16) + g;
    const bool valid = c < d;
    const int cc = valid ? c : 0;
    double y[RPL];
#pragma unroll
    for (int s = 0; s < RPL; s++) {
        const int row = l + 16 * s;
        y[s] = (valid && row < m) ? a.Y[(int64_t)cc * a.ys_c + (int64_t)row * a.ys_r] : 0.0;
    }
    const int nfc = a.nj * a.R;
    const double *F = a.fits_out + (size_t)4 * cc * nfc;
    uint64_t bk = ~0ull;   // gp_mean_dev's arg-min
    int bi = -1;
    for (int t = l; t < nfc; t += 16) key_take(bk, bi, fval_key(F[4 * t + 2]), t);
    row_key_min(bk, bi);
    const double f0 = F[2];
    const int best = (f0 != f0) ? 0 : bi;
    const double sx = F[4 * best], sy = F[4 * best + 1];
    const int jidx = best / a.R;
    GPLane<MAXM> P;
    gp_lane_init<MAXM>(P, m, l);
    double *Kimg = sK + (size_t)g * IMG;
    gp_image_init<MAXM>(Kimg, m, l);
    double alpha[RPL], cq, psy;
    const bool ok = gp_mean_prep<MAXM>(m, l, P, sD2, sx, sy, jit_lookup(a, jidx), y, Kimg, alpha, cq, psy);
    if (valid) {
        double *ap = AP + ((int64_t)blockIdx.y * d + c) * HM_STRIDE(MAXM);
#pragma unroll
        for (int s = 0; s < RPL; s++)
            if (l + 16 * s < MAXM) ap[l + 16 * s] = alpha[s];
        if (l == 0) {
            ap[MAXM] = cq;
            ap[MAXM + 1] = psy;
            ap[MAXM + 2] = ok ? 1.0 : 0.0;
        }
    }
    __syncthreads();
    if (tid == 0) {   // the workgroup's coordinates are visible device-wide before they are counted
        __threadfence();
        __hip_atomic_fetch_add(pre_done + blockIdx.y, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// ---------------------------------------------------------------------------------------------
// Fused correction chain (reference parareal.py:359-382): the speculative
// sweep's per-slice hit path as ONE persistent kernel.  For i = i0, i0+1, ...:
//   1. G:      UG1[i+1] = G(U1[i])            workgroup 0 (one lane for an ODE, one wave for Burgers)
//   2. kNN:    distances of every training row to U1[i]                    all workgroups
//   3. select: the ordered m-neighbour list, y_m, D2, kd2; hit = list == the speculative batch's
//              list (1) or the re-speculated one (2)                      workgroup 0
//   4. on a hit: per coordinate the first arg-min over the batch's fits, the posterior mean and
//              U1[i+1] = mean + UG1[i+1]                                  all workgroups
// with a grid barrier between the phases.  A miss ends the kernel at slice i (its G and select
// outputs are in the workspace) and the host runs that slice's fits; so the host sees one
// round trip per MISS instead of ~5 launches and a host-flag wait per slice.  Every phase runs the
// same device code as the unfused launches (lane_slice / burgers_wave_slice, knn_dist_row,
// knn_select_dev, gp_mean_dev), so the sweep is bitwise unchanged.
// ---------------------------------------------------------------------------------------------
inline namespace exact {
#include "nngp_rk_dev.h"
}

static constexpr int CHAIN_QMAX = 256;   // largest state the chain handles (Burgers d <= 256)

struct ChainArgs {
    NMArgs a;                  // the mean phase: m, d, nj, R, jit_pow; D2 / kd2 / Y = the workspace
    LaneArgs la;               // G of an ODE (gkind 0)
    FieldArgs fa;              // G of Burgers (gkind 1)
    int gkind, sys, order, lin, norm, ept;
    int64_t g_steps;
    const double *t;           // [N+1] slice boundaries
    int I, N, i0;
    double *U1, *UG1;
    const double *X, *Yd;      // training inputs / targets [rows][d]
    int64_t rows;
    int kk;                    // select variant (keys per thread: 2/4/8/16, 0 = streaming)
    int xs_doubles;
    int n_mean_blk;            // 16-lane coordinate groups / 16
    double *dist;              // [rows]
    int32_t *idx;              // [m]
    int32_t *flags;            // [N-I] hit codes (0 = miss)
    const int32_t *spec_idx, *spec2_idx;   // [N-I][m] (spec2: re-speculated lists, or null)
    const double *spec_fits, *spec2_fits;  // [N-I][n_fits][4]
    int64_t n_fits;
    double *preds;             // [d]
    uint32_t *bar;             // grid-barrier arrivals (zeroed before the launch)
    int32_t *stop;             // host-mapped: the slice the chain stopped at (a miss), or N
    uint64_t *g_ticks;         // host-mapped: wall-clock ticks spent in G
    uint64_t *prof;            // host-mapped [4] or null (NNGP_CHAIN_PROF): ticks in G | kNN | select | mean
    int32_t *berr;             // host-mapped: a grid barrier timed out (every workgroup then leaves)
    uint64_t bar_ticks;        // that timeout, in wall-clock ticks (2 s)
};

// all workgroups of the (co-resident) grid: arrivals counted on one agent-scope
// counter; the fences make every workgroup's global writes before the barrier visible to every
// workgroup after it (L2 write-back / invalidate across the XCDs).  Bounded: a workgroup that waits
// longer than bar_ticks (the grid was not co-resident after all -- e.g. another process's kernels
// hold CUs), or that sees another workgroup's timeout, flags *berr and returns false; the kernel
// then ends and the host reruns the sweep on the launch chain (nngp_sweep.hip).
__device__ __forceinline__ bool chain_barrier(uint32_t *bar, uint32_t &target, int32_t *berr, uint64_t ticks) {
    __shared__ int s_bad;
    __syncthreads();
    if (gridDim.x == 1) return true;
    target += gridDim.x;
    if (threadIdx.x == 0) {
        s_bad = 0;
        __threadfence();
        __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t t0 = wall_clock64();
        while (__hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
            if (__hip_atomic_load(berr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0 ||
                wall_clock64() - t0 >= ticks) {
                __hip_atomic_store(berr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                s_bad = 1;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        // a workgroup arriving after the others gave up finds bar >= target at once: it must not
        // run the next phase on data the others never finished writing
        if (__hip_atomic_load(berr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) s_bad = 1;
        __threadfence();
    }
    __syncthreads();
    return s_bad == 0;
}

template <int SYS, int ORDER>
__device__ __forceinline__ void chain_lane_g2(const LaneArgs &la, bool lin, bool norm, double T0, double T1,
                                              int64_t steps, const double *u0, double *out) {
    if (lin) {
        if (norm) lane_slice<SYS, ORDER, true, true>(la, T0, T1, steps, steps, 0, u0, out);
        else lane_slice<SYS, ORDER, true, false>(la, T0, T1, steps, steps, 0, u0, out);
    } else {
        if (norm) lane_slice<SYS, ORDER, false, true>(la, T0, T1, steps, steps, 0, u0, out);
        else lane_slice<SYS, ORDER, false, false>(la, T0, T1, steps, steps, 0, u0, out);
    }
}

template <int SYS>
__device__ __forceinline__ void chain_lane_g1(const LaneArgs &la, int order, bool lin, bool norm, double T0,
                                              double T1, int64_t steps, const double *u0, double *out) {
    switch (order) {
    case 1: chain_lane_g2<SYS, 1>(la, lin, norm, T0, T1, steps, u0, out); break;
    case 2: chain_lane_g2<SYS, 2>(la, lin, norm, T0, T1, steps, u0, out); break;
    case 4: chain_lane_g2<SYS, 4>(la, lin, norm, T0, T1, steps, u0, out); break;
    default: chain_lane_g2<SYS, 8>(la, lin, norm, T0, T1, steps, u0, out); break;
    }
}

// G of one ODE slice by one lane (the G launch's lane form; bitwise its group form), compiled
// once and called from every chain instantiation
__device__ __attribute__((noinline)) void chain_lane_g(LaneArgs la, int sys, int order, int lin, int norm,
                                                       double T0, double T1, int64_t steps, const double *u0,
                                                       double *out) {
    switch (sys) {
    case NNGP_SYS_LORENZ: chain_lane_g1<NNGP_SYS_LORENZ>(la, order, lin, norm, T0, T1, steps, u0, out); break;
    case NNGP_SYS_HOPF: chain_lane_g1<NNGP_SYS_HOPF>(la, order, lin, norm, T0, T1, steps, u0, out); break;
    case NNGP_SYS_THOMAS_LABYRINTH:
        chain_lane_g1<NNGP_SYS_THOMAS_LABYRINTH>(la, order, lin, norm, T0, T1, steps, u0, out);
        break;
    case NNGP_SYS_FHN_ODE: chain_lane_g1<NNGP_SYS_FHN_ODE>(la, order, lin, norm, T0, T1, steps, u0, out); break;
    case NNGP_SYS_ROSSLER: chain_lane_g1<NNGP_SYS_ROSSLER>(la, order, lin, norm, T0, T1, steps, u0, out); break;
    case NNGP_SYS_BRUSSELATOR:
        chain_lane_g1<NNGP_SYS_BRUSSELATOR>(la, order, lin, norm, T0, T1, steps, u0, out);
        break;
    default: chain_lane_g1<NNGP_SYS_DBL_PEND>(la, order, lin, norm, T0, T1, steps, u0, out); break;
    }
}

template <int ORDER, int EPT>
__device__ __forceinline__ void chain_burgers_g2(const FieldArgs &fa, bool lin, bool norm, int l, double T0,
                                                 double T1, int64_t steps, const double *u0, double *out) {
    if (lin) {
        if (norm) burgers_wave_slice<ORDER, true, EPT, true>(fa, l, T0, T1, steps, steps, 0, u0, out);
        else burgers_wave_slice<ORDER, true, EPT, false>(fa, l, T0, T1, steps, steps, 0, u0, out);
    } else {
        if (norm) burgers_wave_slice<ORDER, false, EPT, true>(fa, l, T0, T1, steps, steps, 0, u0, out);
        else burgers_wave_slice<ORDER, false, EPT, false>(fa, l, T0, T1, steps, steps, 0, u0, out);
    }
}

template <int EPT>
__device__ __forceinline__ void chain_burgers_g1(const FieldArgs &fa, int order, bool lin, bool norm, int l,
                                                 double T0, double T1, int64_t steps, const double *u0,
                                                 double *out) {
    switch (order) {
    case 1: chain_burgers_g2<1, EPT>(fa, lin, norm, l, T0, T1, steps, u0, out); break;
    case 2: chain_burgers_g2<2, EPT>(fa, lin, norm, l, T0, T1, steps, u0, out); break;
    case 4: chain_burgers_g2<4, EPT>(fa, lin, norm, l, T0, T1, steps, u0, out); break;
    default: chain_burgers_g2<8, EPT>(fa, lin, norm, l, T0, T1, steps, u0, out); break;
    }
}

// G of one Burgers slice by one full wave (the G launch's wave form)
__device__ __attribute__((noinline)) void chain_burgers_g(FieldArgs fa, int ept, int order, int lin, int norm,
                                                          int l, double T0, double T1, int64_t steps,
                                                          const double *u0, double *out) {
    switch (ept) {
    case 1: chain_burgers_g1<1>(fa, order, lin, norm, l, T0, T1, steps, u0, out); break;
    case 2: chain_burgers_g1<2>(fa, order, lin, norm, l, T0, T1, steps, u0, out); break;
    case 3: chain_burgers_g1<3>(fa, order, lin, norm, l, T0, T1, steps, u0, out); break;
    default: chain_burgers_g1<4>(fa, order, lin, norm, l, T0, T1, steps, u0, out); break;
    }
}

template <int MAXM>
__global__ void __launch_bounds__(256) chain_kernel(ChainArgs c) {
    __shared__ SelShm sh;
    __shared__ __attribute__((aligned(16))) double qs[CHAIN_QMAX];   // U1[i], read once per slice
    const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
    const int d = c.a.d, m = c.a.m;
    uint32_t target = 0;
    uint64_t g_ticks = 0, pt[4] = {0, 0, 0, 0}, tp = 0, sm4[4] = {0, 0, 0, 0}, cyc = 0;
    const bool prof = c.prof != nullptr && blockIdx.x == 0;
#define CHAIN_MARK(k)                          \
    if (prof) {                                \
        const uint64_t now = wall_clock64();   \
        pt[k] += now - tp;                     \
        tp = now;                              \
    }
    int i = c.i0;
    for (; i < c.N; i++) {
        const size_t j = (size_t)(i - c.I);
        const double *ui = c.U1 + (size_t)i * d;
        double *ug_next = c.UG1 + (size_t)(i + 1) * d;
        double *u_next = c.U1 + (size_t)(i + 1) * d;
        // U1[i] was written by the previous slice's mean phase (another workgroup): atomic loads
        // keep the read on the vector path, past the barrier's cache invalidation
        if (prof) tp = wall_clock64();
        for (int e = tid; e < d; e += 256)
            qs[e] = __hip_atomic_load(ui + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        // 1) G
        if (blockIdx.x == 0) {
            const uint64_t w0 = wall_clock64();
            if (c.gkind == 0) {
                if (tid == 0)
                    chain_lane_g(c.la, c.sys, c.order, c.lin, c.norm, c.t[i], c.t[i + 1], c.g_steps, qs, ug_next);
            } else if (wid == 0) {
                chain_burgers_g(c.fa, c.ept, c.order, c.lin, c.norm, lane, c.t[i], c.t[i + 1], c.g_steps, qs,
                                ug_next);
            }
            __syncthreads();
            g_ticks += wall_clock64() - w0;
            CHAIN_MARK(0);
        }
        // 2) distances of every training row (grid-stride over the workgroups)
        for (int64_t r = (int64_t)blockIdx.x * 256 + tid; r < c.rows; r += (int64_t)gridDim.x * 256)
            c.dist[r] = knn_dist_row(c.X, d, qs, r);
        if (!chain_barrier(c.bar, target, c.berr, c.bar_ticks)) break;
        CHAIN_MARK(1);
        // 3) ordered neighbour list, y_m, D2, kd2 and the hit code
        if (blockIdx.x == 0) {
            if (prof && tid == 0) {   // select sub-phases relative to its start
                const uint64_t now = wall_clock64();
                for (int k = 0; k < 4; k++) sm4[k] -= now;
                cyc -= clock64();
            }
            const int32_t *s2 = c.spec2_idx ? c.spec2_idx + j * m : nullptr;
            const int32_t *s1 = c.spec_idx + j * m;
            int32_t *fl = c.flags + j;
            double *ymT = const_cast<double *>(c.a.Y);
            double *D2 = const_cast<double *>(c.a.D2), *kd2 = const_cast<double *>(c.a.kd2);
            switch (c.kk) {
            case 2: knn_select_dev<2>(sh, c.dist, c.rows, m, c.X, c.Yd, d, qs, c.idx, nullptr, ymT, D2, kd2, s1, fl,
                                      c.xs_doubles, s2, nullptr, prof ? sm4 : nullptr); break;
            case 4: knn_select_dev<4>(sh, c.dist, c.rows, m, c.X, c.Yd, d, qs, c.idx, nullptr, ymT, D2, kd2, s1, fl,
                                      c.xs_doubles, s2, nullptr, prof ? sm4 : nullptr); break;
            case 8: knn_select_dev<8>(sh, c.dist, c.rows, m, c.X, c.Yd, d, qs, c.idx, nullptr, ymT, D2, kd2, s1, fl,
                                      c.xs_doubles, s2, nullptr, prof ? sm4 : nullptr); break;
            case 16: knn_select_dev<16>(sh, c.dist, c.rows, m, c.X, c.Yd, d, qs, c.idx, nullptr, ymT, D2, kd2, s1,
                                        fl, c.xs_doubles, s2, nullptr, prof ? sm4 : nullptr); break;
            default: knn_select_dev<0>(sh, c.dist, c.rows, m, c.X, c.Yd, d, qs, c.idx, nullptr, ymT, D2, kd2, s1,
                                       fl, c.xs_doubles, s2, nullptr, prof ? sm4 : nullptr); break;
            }
        }
        if (prof && tid == 0) cyc += clock64();
        if (!chain_barrier(c.bar, target, c.berr, c.bar_ticks)) break;
        CHAIN_MARK(2);
        const int hit = __hip_atomic_load(c.flags + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (hit == 0) break;   // uniform over the grid: the host runs this slice's fits
        // 4) arg-min over the batch's fits, posterior mean, U1[i+1] = mean + UG1[i+1]
        NMArgs a = c.a;   // the hit's fits, as gp_mean_kernel picks them through a.skip
        a.skip = nullptr;
        a.fits_out = const_cast<double *>(hit == 2 ? c.spec2_fits : c.spec_fits) + j * c.n_fits * 4;
        a.bias = ug_next;
        a.out = u_next;
        a.preds = c.preds;
        bool first = true;
        for (int blk = blockIdx.x; blk < c.n_mean_blk; blk += gridDim.x) {
            if (!first) __syncthreads();
            gp_mean_dev<MAXM>(a, blk, first);
            first = false;
        }
        if (!chain_barrier(c.bar, target, c.berr, c.bar_ticks)) break;
        CHAIN_MARK(3);
    }
#undef CHAIN_MARK
    if (prof && tid == 0)
        for (int k = 0; k < 4; k++) {
            __hip_atomic_store(c.prof + k, pt[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(c.prof + 4 + k, sm4[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(c.prof + 8, cyc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    if (blockIdx.x == 0 && tid == 0) {
        __hip_atomic_store(c.g_ticks, g_ticks, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(c.stop, i, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
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

// padded fit size: the kernel instantiations (8, 16, 18, 20, 24, 32, 48, 64).  18 is there so
// that 20 serves m = 19, 20 only, whose row set 0 never holds a tail row (GP<MAXM>::tail_set)
static constexpr int MAX_M = 64;
static int maxm_for(int m) {
    return m <= 8 ? 8 : (m <= 16 ? 16 : (m <= 18 ? 18 : (m <= 20 ? 20 : (m <= 24 ? 24 : (m <= 32 ? 32 : (m <= 48 ? 48 : 64))))));
}
static size_t k_image_doubles(int maxm) {
    switch (maxm) {
    case 8: return GP<8>::IMG;
    case 16: return GP<16>::IMG;
    case 18: return GP<18>::IMG;
    case 20: return GP<20>::IMG;
    case 24: return GP<24>::IMG;
    case 32: return GP<32>::IMG;
    case 48: return GP<48>::IMG;
    default: return GP<64>::IMG;
    }
}
static int wg_threads(int maxm) { return maxm > 32 ? 64 : 256; }

// f<MAXM>() for the padded size of m
template <typename F>
static int with_maxm(int m, F &&f) {
#ifdef NNGP_GP_ONLY_MAXM   // register/ISA experiments (tools): compile one padded size only
    return f(std::integral_constant<int, NNGP_GP_ONLY_MAXM>{});
#endif
    switch (maxm_for(m)) {
    case 8: return f(std::integral_constant<int, 8>{});
    case 16: return f(std::integral_constant<int, 16>{});
    case 18: return f(std::integral_constant<int, 18>{});
    case 20: return f(std::integral_constant<int, 20>{});
    case 24: return f(std::integral_constant<int, 24>{});
    case 32: return f(std::integral_constant<int, 32>{});
    case 48: return f(std::integral_constant<int, 48>{});
    default: return f(std::integral_constant<int, 64>{});
    }
}

template <int MAXM>
static int launch_nm(NMArgs &a, bool fused, int nblocks, int threads, size_t lds, hipStream_t st, int nq) {
    if (fused)
        hipLaunchKernelGGL((nm_fit_kernel<MAXM, true>), dim3(nblocks), dim3(threads), lds, st, a);
    else
        hipLaunchKernelGGL((nm_fit_kernel<MAXM, false>), dim3(nblocks, nq), dim3(threads), lds, st, a);
    NNGP_LAUNCH_CHECK();
    return NNGP_OK;
}

static int run_mean(NMArgs &a, hipStream_t st) {
    const int maxm = maxm_for(a.m);
    const int threads = wg_threads(maxm), per = threads / 16;
    const size_t lds = sizeof(double) * ((size_t)a.m * a.m + a.m + (size_t)per * k_image_doubles(maxm));
    const dim3 grid((a.d + per - 1) / per);
    return with_maxm(a.m, [&](auto mc) {
        hipLaunchKernelGGL(gp_mean_kernel<decltype(mc)::value>, grid, dim3(threads), lds, st, a);
        NNGP_LAUNCH_CHECK();
        return NNGP_OK;
    });
}

// speculative kernel: one wave per fit, 4 fits per 256-thread workgroup (1 per 64-thread
// workgroup for m > 32)
// waves per fit of the two-level kernel for a launch of `total` fits: 4 while every fit's four
// waves get a SIMD of their own (total <= #CU), 2 up to twice that -- and, for two row sets per
// lane (MAXM 18..32, whose one-level evaluation is twice as long), up to four times that: the
// FHN-PDE d = 800 8-GPU share (100 coordinates, 900 fits at m = 20) 0.711 -> 0.644 ms per
// correction, 4 waves 0.836 (profiles/r05/fhn_corr/level2.txt) -- else the one-level kernel.
// (Resumed parked fits take their shape on the device instead: run_nm_spec / resume_bounds.)
// NNGP_NM_LEVEL2=0 disables it.
static int spec_waves(int total, int maxm, bool resume) {
    const int e = env_int("NNGP_NM_LEVEL2", 1);
    if (maxm > 32 || resume || e == 0) return 1;
    if (e == 2 || e == 4) return e;   // forced (measurements)
    const int ncu = device_cus();
    return total <= ncu ? 4 : (total <= (maxm > 16 ? 4 : 2) * ncu ? 2 : 1);
}

// Finite parked-fit counts up to which the resume gives each finite fit 4 / 2 waves of the
// two-level kernel (NNGP_RESUME_W4 / NNGP_RESUME_W2; both 0 = the one-level kernel, one wave per
// fit, as NNGP_NM_LEVEL2=0)
static void resume_bounds(int maxm, int &t4, int &t2) {
    t4 = t2 = 0;
    if (maxm > 32 || env_int("NNGP_NM_LEVEL2", 1) == 0) return;
    const int ncu = device_cus();
    t4 = std::max(0, env_int("NNGP_RESUME_W4", ncu));
    t2 = std::max(t4, env_int("NNGP_RESUME_W2", 2 * ncu));
}

static int run_nm_spec(NMArgs &a, hipStream_t st, int nq = 1) {
    const int maxm = maxm_for(a.m);
    const int threads = wg_threads(maxm);
    const size_t lds = sizeof(double) * ((size_t)a.m * a.m + (size_t)(threads / 16) * k_image_doubles(maxm));
    if (a.resume && nq == 1) {
        // the parked fits: their counts are only known on the device, so the grid covers the
        // largest case -- finite fits on 4 waves each (<= t4 of them), 2 (<= t2) or 1, then the
        // all-+inf fits a wave each -- and the workgroups past the counts exit at once
        int t4, t2;
        resume_bounds(maxm, t4, t2);
        if (t2 > 0) {
            a.resume_w4 = t4;
            a.resume_w2 = t2;
            const int q4 = (a.n_fits + 3) / 4;
            const dim3 grid2(std::max(std::min(t4, a.n_fits), std::max((std::min(t2, a.n_fits) + 1) / 2, q4)) + q4);
            return with_maxm(a.m, [&](auto mc) {
                constexpr int M = decltype(mc)::value;
                if constexpr (M <= 32) {
                    hipLaunchKernelGGL((nm_spec2_kernel<M, 0>), grid2, dim3(256), lds, st, a);
                    NNGP_LAUNCH_CHECK();
                }
                return NNGP_OK;
            });
        }
    }
    const int W = spec_waves(a.n_fits * nq, maxm, a.resume != 0);
    if (W > 1) {
        const dim3 grid2((a.n_fits + 4 / W - 1) / (4 / W), nq);
        return with_maxm(a.m, [&](auto mc) {
            constexpr int M = decltype(mc)::value;
            if constexpr (M <= 32) {
                if (W == 4) hipLaunchKernelGGL((nm_spec2_kernel<M, 4>), grid2, dim3(256), lds, st, a);
                else hipLaunchKernelGGL((nm_spec2_kernel<M, 2>), grid2, dim3(256), lds, st, a);
                NNGP_LAUNCH_CHECK();
            }
            return NNGP_OK;
        });
    }
    const dim3 grid((a.n_fits + threads / 64 - 1) / (threads / 64), nq);
    return with_maxm(a.m, [&](auto mc) {
        hipLaunchKernelGGL(nm_spec_kernel<decltype(mc)::value>, grid, dim3(threads), lds, st, a);
        NNGP_LAUNCH_CHECK();
        return NNGP_OK;
    });
}

// Speculative (a wave per fit) while the fits fit ~2 waves per SIMD (MAXM <= 16) or ~1 (MAXM 24/32,
// two K rows per lane: twice the VGPRs and issue per evaluation); beyond that the packed kernel
// (4 fits per wave) has the better throughput.  Crossover measured on the box with
// `tools/nm_probe.py sweep` (profiles/r01/nm_sweep.txt): m=15 spec wins to 1728 fits, loses at
// 2304; m=20 spec wins at 864 fits (0.67 vs 0.98 ms), loses from 1152 (1.10 vs 0.98 ms).
// NNGP_NM_SPEC=0/1 forces either (tuning).
static bool use_spec(int n_fits, int m) {
    const int forced = env_int("NNGP_NM_SPEC", -1);
    if (forced >= 0) return forced != 0;
    const int ncu = device_cus();
    const int mm = maxm_for(m);   // m > 32: one fit per 64-thread workgroup, ~1 workgroup per CU (LDS)
    return n_fits <= (mm <= 16 ? 8 : (mm <= 32 ? 4 : 1)) * ncu;
}

// fits per 16-lane group in the unfused kernel's work-queue mode (NNGP_NM_REFILL; 0/1 = off)
static int nm_fits_per_row() {
    return std::max(0, env_int("NNGP_NM_REFILL", 8));
}

// qslot: the workspace slot of the work-queue counters -- its own per concurrent stream (the
// sweep's fits: 4; the overlapped speculative batch: 7; the re-speculation window: 8)
static int run_nm(NMArgs &a, bool fused, hipStream_t st, int nq = 1, int qslot = 4) {
    const int maxm = maxm_for(a.m);
    const size_t kimg = k_image_doubles(maxm);
    const int tmax = maxm <= 16 ? NMBound<16>::T : (maxm <= 32 ? NMBound<32>::T : NMBound<64>::T);
    auto lds_of = [&](int threads) {
        const int galloc = threads / 16;
        return sizeof(double) * ((size_t)a.m * a.m + a.m + 4 * (size_t)galloc + (size_t)galloc * kimg);
    };
    int threads, nblocks;
    if (fused) {
        // whole coordinates per workgroup (the arg-min needs all fits of a coordinate); few per
        // workgroup so the latency-bound fits spread over every CU, capped by LDS / threads
        const int nfc = a.nj * a.R;
        const int ncu = device_cus();
        auto thr = [&](int c) { return ((c * nfc * 16 + 63) / 64) * 64; };
        int cpw = std::max(1, std::min((a.d + ncu - 1) / ncu, a.d));
        while (cpw > 1 && (lds_of(thr(cpw)) > 150 * 1024 || thr(cpw) > tmax)) cpw--;
        if (lds_of(thr(cpw)) > 150 * 1024 || thr(cpw) > tmax) {
            set_error("m=%d with %d fits per coordinate exceeds the fused kernel's LDS/threads", a.m, nfc);
            return NNGP_E_UNSUPPORTED;
        }
        a.cpw = cpw;
        threads = thr(cpw);
        nblocks = (a.d + cpw - 1) / cpw;
    } else if (a.park_cap && nq == 1) {
        // one prediction with the tail hand-off: a wave (4 fits) per workgroup so the fits spread
        // over every CU like the fused kernel's; no work queue -- the long fits are parked instead
        threads = 64;
        nblocks = (a.n_fits + 3) / 4;
        a.cpw = 1;
        a.queue = nullptr;
    } else {
        // big batches (the speculative sweep's: Burgers 128 x 1 152 fits) on the throughput
        // kernel, LPF lanes per fit (nngp_nmlane.hip); NNGP_NM_LANES: -1 auto (>= 16 384 fits in
        // the launch), 0 never, 1 whenever m is instantiated
        const int lanes = env_int("NNGP_NM_LANES", -1);
        if (lanes != 0 && nm_lanes_supported(a.m) &&
            (lanes == 1 || (int64_t)a.n_fits * nq >= 16384))
            return run_nm_lanes(a, st, nq, qslot);
        threads = std::min(256, tmax);
        nblocks = (a.n_fits + threads / 16 - 1) / (threads / 16);
        a.cpw = 1;
        a.queue = nullptr;
        const int per_row = nm_fits_per_row();
        if (per_row > 1 && nblocks > 1) {   // work queues: ~per_row fits per group on average
            int err = 0;
            int32_t *qbuf = (int32_t *)workspace(sizeof(int32_t) * (size_t)nq, &err, qslot);
            if (err) return err;
            NNGP_HIP_CHECK(hipMemsetAsync(qbuf, 0, sizeof(int32_t) * (size_t)nq, st));
            a.queue = qbuf;
            nblocks = std::max(1, (nblocks + per_row - 1) / per_row);
        }
    }
    const size_t lds = lds_of(threads);
    return with_maxm(a.m, [&](auto mc) {
        return launch_nm<decltype(mc)::value>(a, fused, nblocks, threads, lds, st, nq);
    });
}

// evaluation count at which the packed kernel parks a fit for the speculative kernel
// (NNGP_NM_PARK; 0 = never)
static int nm_park_cap() {
    return std::max(0, env_int("NNGP_NM_PARK", 70));
}

// packed fits of ONE prediction with the tail hand-off: fits still running at nm_park_cap()
// evaluations are parked and finished by the speculative kernel (bitwise the same fits)
static int run_nm_parked(NMArgs a, hipStream_t st) {
    // NNGP_NM_LANES=1: the throughput kernel whenever m is instantiated (no tail hand-off)
    if (env_int("NNGP_NM_LANES", -1) == 1 && nm_lanes_supported(a.m)) {
        a.jmajor = env_int("NNGP_NM_JMAJOR", 1);
        return run_nm_lanes(a, st, 1, 4);
    }
    const int cap = nm_park_cap();
    if (cap <= 0) return run_nm(a, false, st);
    int err = 0;
    char *ws = (char *)workspace(sizeof(NM) * (size_t)a.n_fits + sizeof(int32_t) * ((size_t)a.n_fits + 2), &err, 5);
    if (err) return err;
    NM *park = (NM *)ws;
    int32_t *cnt = (int32_t *)(park + a.n_fits);   // [finite parked, all-+inf parked], list
    NNGP_HIP_CHECK(hipMemsetAsync(cnt, 0, 2 * sizeof(int32_t), st));
    a.park_cap = cap;
    // jitter-major rows (NNGP_NM_JMAJOR=0: product order): fits sharing a jitter run similar
    // evaluation counts, so a wave's rows finish together (d = 800 synthetic correction
    // 2.99 -> 2.72 ms; profiles/r02/jmajor_probe.txt)
    a.jmajor = env_int("NNGP_NM_JMAJOR", 1);
    a.park = park;
    a.park_count = cnt;
    a.park_list = cnt + 2;
    int rc = run_nm(a, false, st);
    if (rc) return rc;
    a.park_cap = 0;
    a.resume = 1;
    return run_nm_spec(a, st);
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
    launch_knn_select(dim3(1), 0, st, dist, rows, m, X, (const double *)nullptr, d, q, idx_out, dist_out,
                      (double *)nullptr, (double *)nullptr, (double *)nullptr, (const int32_t *)nullptr,
                      (int32_t *)nullptr, 0, (const int32_t *)nullptr, (int32_t *)nullptr, HitMean{});
    NNGP_LAUNCH_CHECK();
    return NNGP_OK;
}

extern "C" int nngp_nm_fit_batch(int m, int d, const double *xm, const double *ym, int n_fits,
                                 const int32_t *coord, const int32_t *jitter_idx, int n_jitter,
                                 const double *jitter_exp_host, const double *theta0, double fatol,
                                 double xatol, int maxfev, double *theta_out, double *fval_out,
                                 int32_t *nfev_out, void *stream) {
    NNGP_REQUIRE(m >= 1 && m <= MAX_M, "need 1 <= m <= %d (got %d)", MAX_M, m);
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
    if (use_spec(n_fits, m)) return run_nm_spec(a, st);
    return run_nm_parked(a, st);
}

extern "C" int nngp_gp_mean(int m, int d, const double *xm, const double *ym, const double *new_x,
                            const double *theta, const int32_t *jitter_idx, int n_jitter,
                            const double *jitter_exp_host, double *out, void *stream) {
    NNGP_REQUIRE(m >= 1 && m <= MAX_M, "need 1 <= m <= %d (got %d)", MAX_M, m);
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
    NMArgs ma{};
    rc = fill_jitters(ma, n_jitter, jitter_exp_host);
    if (rc) return rc;
    ma.m = m; ma.d = d; ma.D2 = D2; ma.kd2 = kd2; ma.Y = ym; ma.ys_c = 1; ma.ys_r = d;
    ma.theta0 = theta; ma.jitter_idx = jitter_idx; ma.R = 1; ma.preds = out;
    return run_mean(ma, st);
}

namespace nngp {

// One prediction (NNGP_p.predict).  With spec_idx (the ordered neighbour list a speculative batch
// assumed for this query), spec_fits (that batch's fits for it) and hit_flag (device int):
// knn_select sets *hit_flag = (actual list == spec_idx); the fits launch then exits at once on a
// hit and the arg-min/mean kernel reads spec_fits -- bitwise what it would have computed, since a
// fit depends only on (the ordered neighbours, its coordinate, jitter and theta0).
int predict_impl(const double *X, const double *Y, int64_t rows, int d, const double *new_x, int m,
                 int n_jitter, const double *jitter_exp_host, int n_restarts, const double *theta0,
                 double fatol, double xatol, int maxfev, double *preds_out, const double *bias,
                 double *out, double *fits_out, const int32_t *spec_idx, const double *spec_fits,
                 int32_t *hit_flag, const int32_t *spec2_idx, const double *spec2_fits, int32_t *host_flag,
                 hipStream_t st, int c0, int c1, const int32_t *wait_done, int32_t *wait_err, int phase,
                 const HitMean *hm, hipEvent_t bias_ready) {
    NNGP_REQUIRE(X && Y && new_x && theta0 && preds_out, "null array argument");
    NNGP_REQUIRE(phase >= PREDICT_ALL && phase <= PREDICT_SELECT_ONLY, "bad predict phase %d", phase);
    if (c1 < 0) c1 = d;
    NNGP_REQUIRE(0 <= c0 && c0 < c1 && c1 <= d, "bad coordinate range [%d, %d) of d=%d", c0, c1, d);
    NNGP_REQUIRE(m >= 1 && m <= MAX_M, "need 1 <= m <= %d (got %d)", MAX_M, m);
    NNGP_REQUIRE(m <= rows, "m=%d exceeds training rows=%lld", m, (long long)rows);
    NNGP_REQUIRE(d >= 1 && n_restarts >= 1 && maxfev >= 1, "bad d / n_restarts / maxfev");
    const bool spec = spec_idx && spec_fits && hit_flag;
    NMArgs a{};
    int rc = fill_jitters(a, n_jitter, jitter_exp_host);
    if (rc) return rc;
    // workspace: dist[rows] | D2[m*m] | kd2[m] | ymT[d*m] | idx[m] (int32) | fits[n_fits][4]
    // (the fits scratch serves the unfused paths when the caller passes no fits_out)
    const size_t nd = (size_t)rows + (size_t)m * m + m + (size_t)d * m;
    const size_t n_fits = (size_t)d * n_jitter * n_restarts;
    int err = 0;
    char *ws = (char *)workspace(sizeof(double) * nd + sizeof(int32_t) * 64 + sizeof(double) * 4 * n_fits, &err);
    if (err) return err;
    double *dist = (double *)ws;
    double *D2 = dist + rows;
    double *kd2 = D2 + (size_t)m * m;
    double *ymT = kd2 + m;
    int32_t *idx = (int32_t *)(ymT + (size_t)d * m);
    double *fits_ws = (double *)(ws + sizeof(double) * nd + sizeof(int32_t) * 64);
    if (phase == PREDICT_ALL || phase == PREDICT_SELECT || phase == PREDICT_SELECT_ONLY) {
        if (phase != PREDICT_SELECT_ONLY) {   // (SELECT_ONLY: gdist wrote the distances)
            hipLaunchKernelGGL(knn_dist_kernel, dim3((unsigned)((rows + 63) / 64)), dim3(64), 0, st, X, rows,
                               d, new_x, dist);
            NNGP_LAUNCH_CHECK();
        }
        const bool wave_d2 = d2_by_waves(m, d), pair_d2 = d2_by_pairs(m, d);
        const bool sel_d2 = !wave_d2 && !pair_d2;
        launch_knn_select(dim3(1), knn_xs_bytes(m, d), st, dist, rows, m, X, Y, d, new_x, idx, (double *)nullptr,
                          ymT, sel_d2 ? D2 : (double *)nullptr, sel_d2 ? kd2 : (double *)nullptr,
                          spec ? spec_idx : (const int32_t *)nullptr,
                          spec ? hit_flag : (int32_t *)nullptr, knn_xs_doubles(m, d),
                          spec ? spec2_idx : (const int32_t *)nullptr, spec ? host_flag : (int32_t *)nullptr,
                          [&] {
                              HitMean h = (spec && host_flag && hm && sel_d2 && kd2) ? *hm : HitMean{};
                              h.marks = sel_prof_marks();
                              return h;
                          }());
        NNGP_LAUNCH_CHECK();
        if (wave_d2) {
            hipLaunchKernelGGL(d2_wave_kernel, dim3((unsigned)(m * (m + 1) / 2 + m)), dim3(64), 0, st, X, idx, m,
                               d, new_x, D2, kd2);
            NNGP_LAUNCH_CHECK();
        } else if (pair_d2) {
            hipLaunchKernelGGL(d2_pairs_kernel, dim3((unsigned)((m * (m + 1) / 2 + m + 255) / 256)), dim3(256), 0, st, X,
                               idx, m, d, new_x, D2, kd2);
            NNGP_LAUNCH_CHECK();
        }
        if (phase != PREDICT_ALL) return NNGP_OK;
    }
    // coordinates [c0, c1) only (the multi-rank sweep's share): the fits and means of those
    // columns, in the same product(coord, jitter, restart) order with their own theta0 draws
    const int dc = c1 - c0;
    const size_t nfc = (size_t)n_jitter * n_restarts;
    a.m = m; a.d = dc; a.n_fits = (int)(dc * nfc);
    a.D2 = D2; a.kd2 = kd2; a.Y = ymT + (size_t)c0 * m; a.ys_c = m; a.ys_r = 1;
    a.theta0 = theta0 + (size_t)c0 * nfc * 2; a.fatol = fatol; a.xatol = xatol; a.maxfev = maxfev;
    a.R = n_restarts;
    a.fits_out = fits_out ? fits_out : fits_ws;
    a.preds = preds_out; a.bias = bias; a.out = out;
    if (spec) {
        a.skip = hit_flag;
        a.fits_alt = spec_fits;
        a.fits_alt2 = spec2_fits;
        if (wait_done) {   // the batch's fits may still be running (overlapped sweep)
            a.wait_done = wait_done;
            a.wait_n = (int)n_fits;
            a.err = wait_err;
            const double us = std::max(0, env_int("NNGP_SPEC_WAIT_US", 2000000));
            a.wait_ticks = (uint64_t)(us * device_wallclock_khz() / 1e3);
        }
    }
    // bias_ready: the bias (UG1[i+1] = G(U1[i])) comes from another stream; the mean waits for it
    auto mean = [&](NMArgs &ma) -> int {
        if (bias_ready) NNGP_HIP_CHECK(hipStreamWaitEvent(st, bias_ready, 0));
        return run_mean(ma, st);
    };
    if (phase == PREDICT_MEAN) {   // the select's hit is known: the fits are the speculative batch's
        NNGP_REQUIRE(spec, "predict: the mean-only phase needs the speculative fits");
        return mean(a);
    }
    if (use_spec(a.n_fits, a.m)) {   // fits (a wave each), then arg-min + mean (+ bias) per coordinate
        rc = run_nm_spec(a, st);
        if (rc) return rc;
        return mean(a);
    }
    if (!spec && nm_park_cap() == 0) {
        NMArgs fu = a;
        fu.fits_out = fits_out;
        if (bias_ready) NNGP_HIP_CHECK(hipStreamWaitEvent(st, bias_ready, 0));   // (the mean is in the fits)
        rc = run_nm(fu, true, st);
        if (rc != NNGP_E_UNSUPPORTED) return rc;
    }
    // the packed fits with the tail hand-off (or: a coordinate's fits exceed one workgroup, or
    // speculation), then the per-coordinate arg-min + posterior mean kernel
    NMArgs u = a;
    u.preds = nullptr; u.out = nullptr; u.bias = nullptr;
    rc = run_nm_parked(u, st);
    if (rc) return rc;
    return mean(a);
}

// gp_pre_kernel over nq predictions of a batch (p: the batch's fits arguments with its per-prediction
// strides): the query-independent half of every coordinate's mean, for the sweep's select to finish
static int run_pre(const NMArgs &p, double *AP, int32_t *pre_done, int nq, hipStream_t st) {
    const int maxm = maxm_for(p.m);
    const int threads = wg_threads(maxm), per = threads / 16;
    const size_t lds = sizeof(double) * ((size_t)p.m * p.m + (size_t)per * k_image_doubles(maxm));
    const dim3 grid((unsigned)((p.d + per - 1) / per), (unsigned)nq);
    return with_maxm(p.m, [&](auto mc) {
        hipLaunchKernelGGL(gp_pre_kernel<decltype(mc)::value>, grid, dim3(threads), lds, st, p, AP, pre_done);
        NNGP_LAUNCH_CHECK();
        return NNGP_OK;
    });
}

// The speculative batch: for nq guessed queries Q[nq][d] at once, the ordered kNN lists
// (idx_out[nq][m]) and every fit of every prediction (fits_out[nq][n_fits][4]), with each
// prediction's own theta0 draws (theta0[nq][n_fits][2]).  One kNN-distance launch, one
// kNN-select launch (a workgroup per query) and ONE packed fits launch (4 fits per wave over
// all nq*n_fits fits) -- the throughput-shaped work that the sequential sweep then only looks up.
int spec_batch(const double *X, const double *Y, int64_t rows, int d, const double *Q, int nq, int m,
               int n_jitter, const double *jitter_exp_host, int n_restarts, const double *theta0,
               double fatol, double xatol, int maxfev, int32_t *idx_out, double *fits_out, bool latency,
               hipStream_t st, int slot, int32_t *done, hipEvent_t ev_select, double *pre_AP, int32_t *pre_done) {
    NNGP_REQUIRE(nq >= 1 && m >= 1 && m <= MAX_M && m <= rows, "bad speculative batch shape");
    NMArgs a{};
    int rc = fill_jitters(a, n_jitter, jitter_exp_host);
    if (rc) return rc;
    const size_t nfp = (size_t)d * n_jitter * n_restarts;
    // slot-1 workspace: dist[nq][rows] | D2[nq][m*m] | ymT[nq][d*m]
    int err = 0;
    double *dist = (double *)workspace(sizeof(double) * (size_t)nq * ((size_t)rows + (size_t)m * m + (size_t)d * m),
                                       &err, slot);
    if (err) return err;
    double *D2 = dist + (size_t)nq * rows;
    double *ymT = D2 + (size_t)nq * m * m;
    if (done) NNGP_HIP_CHECK(hipMemsetAsync(done, 0, sizeof(int32_t) * (size_t)nq, st));
    if (pre_AP) NNGP_HIP_CHECK(hipMemsetAsync(pre_done, 0, sizeof(int32_t) * (size_t)nq, st));
    hipLaunchKernelGGL(knn_dist_kernel, dim3((unsigned)((rows + 63) / 64), (unsigned)nq), dim3(64), 0, st, X,
                       rows, d, Q, dist);
    NNGP_LAUNCH_CHECK();
    const bool wave_d2 = d2_by_waves(m, d), pair_d2 = d2_by_pairs(m, d);
    launch_knn_select(dim3(1, (unsigned)nq), knn_xs_bytes(m, d), st, dist, rows, m, X, Y, d, Q, idx_out,
                      (double *)nullptr, ymT, (wave_d2 || pair_d2) ? (double *)nullptr : D2, (double *)nullptr,
                      (const int32_t *)nullptr, (int32_t *)nullptr, knn_xs_doubles(m, d), (const int32_t *)nullptr,
                      (int32_t *)nullptr, HitMean{});
    NNGP_LAUNCH_CHECK();
    if (wave_d2) {
        hipLaunchKernelGGL(d2_wave_kernel, dim3((unsigned)(m * (m + 1) / 2), (unsigned)nq), dim3(64), 0, st, X,
                           idx_out, m, d, Q, D2, (double *)nullptr);
        NNGP_LAUNCH_CHECK();
    }
    if (pair_d2) {
        hipLaunchKernelGGL(d2_pairs_kernel, dim3((unsigned)((m * (m + 1) / 2 + 255) / 256), (unsigned)nq), dim3(256), 0,
                           st, X, idx_out, m, d, Q, D2, (double *)nullptr);
        NNGP_LAUNCH_CHECK();
    }
    // the counters are zeroed (above) before the event the sweep's mean kernels wait behind
    if (ev_select) NNGP_HIP_CHECK(hipEventRecord(ev_select, st));   // the lists are ready
    a.m = m; a.d = d; a.n_fits = (int)nfp;
    a.D2 = D2; a.Y = ymT; a.ys_c = m; a.ys_r = 1;
    a.theta0 = theta0; a.fatol = fatol; a.xatol = xatol; a.maxfev = maxfev; a.R = n_restarts;
    a.fits_out = fits_out;
    a.qs_D2 = (int64_t)m * m; a.qs_Y = (int64_t)d * m; a.qs_th = (int64_t)nfp * 2; a.qs_fits = (int64_t)nfp * 4;
    a.jmajor = env_int("NNGP_NM_JMAJOR", 1);   // (run_nm_parked; Burgers 0.328 -> 0.317 s)
    a.done = done;
    const NMArgs p = a;   // (run_nm adjusts its copy's launch fields)
    // latency: a wave per fit (the re-speculation window the sweep waits on); else packed fits.
    // (The window on the packed or the 4-lanes kernel: Burgers 0.297 / 0.281 s against 0.221 s,
    // profiles/r05/nm_lanes/respec_shape_not_kept.txt -- the next slice waits on its slowest fit.)
    rc = latency ? run_nm_spec(a, st, nq) : run_nm(a, false, st, nq, slot == 1 ? 7 : 8);
    if (rc || !pre_AP) return rc;
    return run_pre(p, pre_AP, pre_done, nq, st);
}

int pre_target(int d, int m) {
    const int per = wg_threads(maxm_for(m)) / 16;
    return (d + per - 1) / per;
}

int pre_maxm(int m) { return maxm_for(m); }

// ---- the fused correction chain, host side ----------------------------------------------------
struct ChainRes {
    int dev = -1;
    double tick_khz = 0;      // wall_clock64 rate
    uint32_t *bar = nullptr;  // device: grid-barrier counter
    int32_t *stop = nullptr;  // host-mapped: stop slice | G ticks (u64)
};
static ChainRes g_chain;
static std::mutex g_chain_mu;
static int64_t g_chain_launches = 0, g_chain_slices = 0;   // nngp_chain_stats (under g_chain_mu)

// nngp_shutdown: release the chain's buffers (re-created on next use)
void chain_release() {
    std::lock_guard<std::mutex> lk(g_chain_mu);
    if (g_chain.bar) (void)hipFree(g_chain.bar);
    if (g_chain.stop) (void)hipHostFree(g_chain.stop);
    g_chain = ChainRes{};
}

static int chain_resources(ChainRes **out) {
    std::lock_guard<std::mutex> lk(g_chain_mu);
    ChainRes &r = g_chain;
    int dev = 0;
    NNGP_HIP_CHECK(hipGetDevice(&dev));
    if (r.dev != dev) {
        if (r.bar) (void)hipFree(r.bar);
        if (r.stop) (void)hipHostFree(r.stop);
        r = ChainRes{};
        int khz = 0;
        NNGP_HIP_CHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev));
        r.tick_khz = khz > 0 ? khz : 100000.0;
        NNGP_HIP_CHECK(hipMalloc((void **)&r.bar, 256));
        NNGP_HIP_CHECK(hipHostMalloc((void **)&r.stop, 128, hipHostMallocMapped | hipHostMallocCoherent));
        r.dev = dev;
    }
    *out = &r;
    return NNGP_OK;
}

// G of one slice in-kernel (the chain and the guess chain): the G launch's system, tableau and grid
struct GArgs {
    LaneArgs la;    // an ODE (gkind 0): one lane
    FieldArgs fa;   // Burgers (gkind 1): one wave, d = 64 * ept
    int gkind, sys, order, lin, norm, ept;
    int64_t g_steps;
};

static int g_args(const nngp_system *sys, int g_tableau, int g_step_mode, int64_t g_steps, GArgs &g) {
    g = GArgs{};
    const int d = sys->d, kind = sys->kind;
    if (kind == NNGP_SYS_BURGERS) {
        g.gkind = 1;
        g.ept = d / 64;
        g.fa.d = d; g.fa.nx = sys->nx; g.fa.normalized = sys->normalized; g.fa.norm = sys->norm;
        const double dx = (1.0 - (-1.0)) / (sys->d - 1);   // as field_args (nngp_rk_dev.h users)
        const double nu = sys->param[0];
        g.fa.c_off = nu / (dx * dx);
        g.fa.c_diag = g.fa.c_off * -2.0;
        g.fa.c_grad = 1 / (2 * dx);
    } else {
        g.gkind = 0;
        g.la.normalized = sys->normalized;
        for (int k = 0; k < 4; k++) g.la.param[k] = sys->param[k];
        g.la.rparam0 = 1.0 / sys->param[0];
        g.la.norm = sys->norm;
    }
    NNGP_REQUIRE(!sys->normalized || sys->norm, "normalized system needs norm[3d]");
    NNGP_REQUIRE(g_tableau == 1 || g_tableau == 2 || g_tableau == 4 || g_tableau == 8, "bad G tableau %d", g_tableau);
    g.sys = kind; g.order = g_tableau;
    g.lin = (g_step_mode & ~NNGP_STEP_CONTRACT) == NNGP_STEP_LINSPACE;
    g.norm = sys->normalized != 0;
    g.g_steps = g_steps;
    return NNGP_OK;
}

// systems whose G runs in-kernel: every ODE (lane form) and Burgers with d = 64*EPT <= 256 (wave
// form); exact G only (the contracted build's G is another kernel)
static bool g_in_kernel(const nngp_system *sys, int g_step_mode) {
    if (g_step_mode & NNGP_STEP_CONTRACT) return false;
    switch (sys->kind) {
    case NNGP_SYS_LORENZ: case NNGP_SYS_HOPF: case NNGP_SYS_THOMAS_LABYRINTH: case NNGP_SYS_FHN_ODE:
    case NNGP_SYS_ROSSLER: case NNGP_SYS_BRUSSELATOR: case NNGP_SYS_DBL_PEND:
        return true;
    case NNGP_SYS_BURGERS:
        return sys->nx == sys->d && sys->d % 64 == 0 && sys->d <= CHAIN_QMAX;
    default:
        return false;
    }
}

// The speculative sweep's guesses along the coarse chain (nngp_sweep.hip), ONE wave for all of them:
//   Q[j+1] = (UF[I+j+1] - UG[I+j+1]) + G(Q[j]),   j = 0 .. nq-2
// with the G launch's own device code (lane_slice / burgers_wave_slice) and nngp_parareal_update's
// expression, so Q is bitwise the launch loop's (2 launches per slice: ~19 us of host issue each
// pair, 2.4 ms per Burgers N = 128 iteration).  Every element is written and re-read by the lane
// that owns it (lane 0 for an ODE, lane l for Burgers elements l*ept ..), so no barrier is needed.
__global__ void __launch_bounds__(64) guess_chain_kernel(GArgs g, const double *__restrict__ t, int I, int nq, int d,
                                                         const double *__restrict__ UF, const double *__restrict__ UG,
                                                         double *Q, double *gtmp) {
    const int l = threadIdx.x;
    for (int j = 0; j + 1 < nq; j++) {
        const int i = I + j;
        const double *q = Q + (size_t)j * d;
        double *qn = Q + (size_t)(j + 1) * d;
        const double *uf = UF + (size_t)(i + 1) * d, *ug = UG + (size_t)(i + 1) * d;
        if (g.gkind == 1) {
            chain_burgers_g(g.fa, g.ept, g.order, g.lin, g.norm, l, t[i], t[i + 1], g.g_steps, q, gtmp);
            for (int r = 0; r < g.ept; r++) {
                const int e = l * g.ept + r;
                const double p = uf[e] - ug[e];
                qn[e] = p + gtmp[e];
            }
        } else if (l == 0) {
            chain_lane_g(g.la, g.sys, g.order, g.lin, g.norm, t[i], t[i + 1], g.g_steps, q, gtmp);
            for (int e = 0; e < d; e++) {
                const double p = uf[e] - ug[e];
                qn[e] = p + gtmp[e];
            }
        }
    }
}

// false: the caller keeps the launch loop (a system without in-kernel G, or NNGP_GUESS_FUSED=0)
bool guess_chain_supported(const nngp_system *sys, int g_step_mode) {
    return env_int("NNGP_GUESS_FUSED", 1) != 0 && g_in_kernel(sys, g_step_mode);
}

int guess_chain(const nngp_system *sys, int g_tableau, int g_step_mode, int64_t g_steps, const double *t, int I,
                int nq, const double *UF, const double *UG, double *Q, double *gtmp, hipStream_t st) {
    NNGP_REQUIRE(g_in_kernel(sys, g_step_mode), "guess chain: no in-kernel G for this system");
    if (nq < 2) return NNGP_OK;
    GArgs g;
    const int rc = g_args(sys, g_tableau, g_step_mode, g_steps, g);
    if (rc) return rc;
    hipLaunchKernelGGL(guess_chain_kernel, dim3(1), dim3(64), 0, st, g, t, I, nq, sys->d, UF, UG, Q, gtmp);
    NNGP_LAUNCH_CHECK();
    return NNGP_OK;
}

// The sweep's slice head in ONE launch: G(U1[i]) -> UG1[i+1] and the query's kNN distances, which
// both only read U1[i].  Blocks 0 .. nb-1 are knn_dist_kernel's (a row per thread), the last block
// runs the G launch's device code (guess_chain_kernel's: a wave for Burgers, lane 0 for an ODE) --
// bitwise the two launches it replaces, at one host launch (~7 us of host issue) less per slice.
__global__ void __launch_bounds__(64) gdist_kernel(GArgs g, double T0, double T1, const double *__restrict__ X,
                                                   int64_t rows, int d, const double *q, double *__restrict__ dist,
                                                   double *ug_next) {
    const int l = threadIdx.x;
    if (blockIdx.x == gridDim.x - 1) {
        if (g.gkind == 1) chain_burgers_g(g.fa, g.ept, g.order, g.lin, g.norm, l, T0, T1, g.g_steps, q, ug_next);
        else if (l == 0) chain_lane_g(g.la, g.sys, g.order, g.lin, g.norm, T0, T1, g.g_steps, q, ug_next);
        return;
    }
    const int64_t r = (int64_t)blockIdx.x * 64 + l;
    if (r < rows) dist[r] = knn_dist_row(X, d, q, r);
}

bool gdist_supported(const nngp_system *sys, int g_step_mode) {
    return env_int("NNGP_GDIST", 1) != 0 && g_in_kernel(sys, g_step_mode);
}

// G on a side stream beside a slice's prediction (the systems without an in-kernel G: the PDE field
// kernels, whose one-slice G is tens of microseconds -- FHN-PDE d = 800: ~75 us of a ~1.8 ms
// correction); NNGP_G_SIDE=0: on the sweep's stream
bool g_side_supported(const nngp_system *sys, int g_step_mode) {
    return env_int("NNGP_G_SIDE", 1) != 0 && !g_in_kernel(sys, g_step_mode);
}

// G of slice i and its query's distances into predict_impl's workspace (the same slot-0 layout and
// size, so the select of PREDICT_SELECT_ONLY that follows finds them)
int gdist(const nngp_system *sys, int g_tableau, int g_step_mode, int64_t g_steps, const double *t, int i,
          const double *X, int64_t rows, int d, int m, int n_jitter, int n_restarts, const double *ui,
          double *ug_next, hipStream_t st) {
    GArgs g;
    const int rc = g_args(sys, g_tableau, g_step_mode, g_steps, g);
    if (rc) return rc;
    const size_t nd = (size_t)rows + (size_t)m * m + m + (size_t)d * m;
    const size_t n_fits = (size_t)d * n_jitter * n_restarts;
    int err = 0;
    double *dist = (double *)workspace(sizeof(double) * nd + sizeof(int32_t) * 64 + sizeof(double) * 4 * n_fits, &err);
    if (err) return err;
    hipLaunchKernelGGL(gdist_kernel, dim3((unsigned)((rows + 63) / 64 + 1)), dim3(64), 0, st, g, t[i], t[i + 1], X,
                       rows, d, ui, dist, ug_next);
    NNGP_LAUNCH_CHECK();
    return NNGP_OK;
}

// the systems / shapes the chain's in-kernel G covers (the rest keep the launch chain):
// every ODE (lane form) and Burgers with d = 64*EPT <= 256 (wave form); exact G, m <= 24 (at the
// padded size 32 the mean phase's 16 fit images -- K/L plus the per-row scalars -- and the select's
// LDS no longer fit one CU's 160 KiB together).
// Opt-in (NNGP_CHAIN=1): measured on the box it is bitwise the launch chain but not faster --
// 0.90-1.00x on Lorenz / FHN-ODE / Hopf / Burgers (tools/chain_probe.py).
bool chain_supported(const nngp_system *sys, int g_step_mode, int m) {
    const char *e = getenv("NNGP_CHAIN");
    if (!e || atoi(e) == 0) return false;
    if (m < 1 || m > 24 || sys->d > CHAIN_QMAX) return false;
    return g_in_kernel(sys, g_step_mode);
}

// An ordinary launch.  The grid barrier needs every workgroup resident at once: nb <= 64
// workgroups of 256 threads, checked against the kernel's occupancy, and nothing else runs on the
// device meanwhile (the overlapped batch is off in chain mode; the re-speculation window is
// launched only after the kernel has drained) -- and a workgroup that had to wait for a CU would
// still be scheduled once the kernels ahead of it finish, since none of them waits on the chain.
// (A cooperative launch gave the same guarantee through a separate HIP device queue, whose
// teardown at process exit crashed under rocprofv3: profiles/r03/chain_exit_crash.txt.)
template <int MAXM>
static int chain_launch(ChainArgs &c, int nb, size_t lds, hipStream_t st) {
    const int ncu = device_cus();
    int per_cu = 0;
    NNGP_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, chain_kernel<MAXM>, 256, lds));
    NNGP_REQUIRE(per_cu >= 1 && (int64_t)per_cu * ncu >= nb, "chain: %d workgroups cannot be co-resident", nb);
    hipLaunchKernelGGL(chain_kernel<MAXM>, dim3(nb), dim3(256), lds, st, c);
    NNGP_LAUNCH_CHECK();
    return NNGP_OK;
}

// Run the chain from slice i0 on stream st until the first miss (or N).  *stop_out = that slice:
// its G output (UG1[stop+1]) and its select workspace (chain_miss_fits) are in place.  The call
// returns after the kernel has drained; *g_ms_out += the in-kernel G time.
int chain_sweep(const nngp_system *sys, int g_tableau, int g_step_mode, int64_t g_steps, const double *t, int I,
                int N, int i0, double *U1, double *UG1, const double *X, const double *Y, int64_t rows, int m,
                int n_jitter, const double *jitter_exp_host, int n_restarts, int32_t *flags,
                const int32_t *spec_idx, const double *spec_fits, const int32_t *spec2_idx,
                const double *spec2_fits, double *preds, int *stop_out, float *g_ms_out, hipStream_t st) {
    const int d = sys->d;
    NNGP_REQUIRE(chain_supported(sys, g_step_mode, m) && I <= i0 && i0 < N && m <= rows, "chain: unsupported shape");
    ChainRes *res = nullptr;
    int rc = chain_resources(&res);
    if (rc) return rc;
    ChainArgs c{};
    rc = fill_jitters(c.a, n_jitter, jitter_exp_host);
    if (rc) return rc;
    // slot-0 workspace, predict_impl's layout: dist[rows] | D2[m*m] | kd2[m] | ymT[d*m] | idx[64] | fits
    const size_t nd = (size_t)rows + (size_t)m * m + m + (size_t)d * m;
    const size_t n_fits = (size_t)d * n_jitter * n_restarts;
    int err = 0;
    char *ws = (char *)workspace(sizeof(double) * nd + sizeof(int32_t) * 64 + sizeof(double) * 4 * n_fits, &err);
    if (err) return err;
    double *dist = (double *)ws;
    double *D2 = dist + rows, *kd2 = D2 + (size_t)m * m, *ymT = kd2 + m;
    c.a.m = m; c.a.d = d; c.a.n_fits = (int)n_fits; c.a.D2 = D2; c.a.kd2 = kd2; c.a.Y = ymT;
    c.a.ys_c = m; c.a.ys_r = 1; c.a.R = n_restarts;
    GArgs ga;
    rc = g_args(sys, g_tableau, g_step_mode, g_steps, ga);
    if (rc) return rc;
    c.la = ga.la; c.fa = ga.fa; c.gkind = ga.gkind; c.ept = ga.ept;
    c.sys = ga.sys; c.order = ga.order; c.lin = ga.lin; c.norm = ga.norm; c.g_steps = ga.g_steps;
    c.t = t; c.I = I; c.N = N; c.i0 = i0;
    c.U1 = U1; c.UG1 = UG1; c.X = X; c.Yd = Y; c.rows = rows;
    const int64_t per = (rows + 255) / 256;
    c.kk = per <= 2 ? 2 : (per <= 4 ? 4 : (per <= 8 ? 8 : (per <= 16 ? 16 : 0)));
    c.xs_doubles = knn_xs_doubles(m, d);
    c.n_mean_blk = (d + 15) / 16;
    c.dist = dist; c.idx = (int32_t *)(ymT + (size_t)d * m);
    c.flags = flags; c.spec_idx = spec_idx; c.spec2_idx = spec2_idx;
    c.spec_fits = spec_fits; c.spec2_fits = spec2_fits; c.n_fits = (int64_t)n_fits;
    c.preds = preds;
    c.bar = res->bar;
    c.stop = res->stop;
    c.g_ticks = (uint64_t *)(res->stop + 2);
    const bool prof = env_int("NNGP_CHAIN_PROF", 0) != 0;
    c.prof = prof ? (uint64_t *)(res->stop + 4) : nullptr;
    c.berr = res->stop + 28;   // byte 112 of the 128-byte host-mapped block (prof: bytes 16..87)
    // the grid-barrier timeout: other workgroups wait at barrier 1 while block 0 integrates G, so
    // it scales with the coarse step count (4 us per step covers every G kernel here, RK8 Burgers
    // ~1.4 us) and is never below NNGP_CHAIN_BARRIER_US (default 2 s)
    const double bar_us = std::max((double)std::max(0, env_int("NNGP_CHAIN_BARRIER_US", 2000000)), 4.0 * (double)g_steps);
    c.bar_ticks = (uint64_t)(bar_us * res->tick_khz / 1e3);
    const int maxm = maxm_for(m);
    const size_t lds = std::max(knn_xs_bytes(m, d),
                                sizeof(double) * ((size_t)m * m + m + 16 * k_image_doubles(maxm)));
    NNGP_REQUIRE(lds + sizeof(SelShm) + sizeof(double) * CHAIN_QMAX <= 160 * 1024, "chain: LDS");
    // workgroups: one per 16 coordinates of the mean phase (a single workgroup, i.e. no grid
    // barrier, measured slower: 65 us per slice, 0.387 s for Burgers N=128)
    const int nb = std::max(1, std::min(c.n_mean_blk, 64));
    res->stop[0] = -1;
    __atomic_store_n(c.berr, 0, __ATOMIC_RELEASE);
    NNGP_HIP_CHECK(hipMemsetAsync(res->bar, 0, sizeof(uint32_t), st));
    switch (maxm) {
    case 8: rc = chain_launch<8>(c, nb, lds, st); break;
    case 16: rc = chain_launch<16>(c, nb, lds, st); break;
    case 18: rc = chain_launch<18>(c, nb, lds, st); break;
    case 20: rc = chain_launch<20>(c, nb, lds, st); break;
    case 24: rc = chain_launch<24>(c, nb, lds, st); break;
    default: rc = chain_launch<32>(c, nb, lds, st); break;
    }
    if (rc) return rc;
    NNGP_HIP_CHECK(hipStreamSynchronize(st));
    if (__atomic_load_n(c.berr, __ATOMIC_ACQUIRE) != 0) {   // not co-resident: the caller reruns
        set_error("chain: a grid barrier timed out (NNGP_CHAIN=1 needs the device to itself)");
        *stop_out = -2;
        return NNGP_E_HIP;
    }
    const int stop = __atomic_load_n(res->stop, __ATOMIC_ACQUIRE);
    if (stop < i0 || stop > N) {
        set_error("chain: the kernel reported no stop slice (%d)", stop);
        return NNGP_E_HIP;
    }
    *stop_out = stop;
    if (g_ms_out) *g_ms_out += (float)((double)*c.g_ticks / res->tick_khz);
    if (c.prof)
        fprintf(stderr,
                "chain i0=%d stop=%d d=%d rows=%lld nb=%d us: G %.1f kNN %.1f select %.1f mean %.1f"
                " | select marks %.1f %.1f %.1f %.1f | select shader cycles %.0f\n",
                i0, stop, d, (long long)rows, nb, c.prof[0] / res->tick_khz * 1e3, c.prof[1] / res->tick_khz * 1e3,
                c.prof[2] / res->tick_khz * 1e3, c.prof[3] / res->tick_khz * 1e3, (double)(int64_t)c.prof[4] / res->tick_khz * 1e3,
                (double)(int64_t)c.prof[5] / res->tick_khz * 1e3, (double)(int64_t)c.prof[6] / res->tick_khz * 1e3,
                (double)(int64_t)c.prof[7] / res->tick_khz * 1e3, (double)c.prof[8]);
    {
        std::lock_guard<std::mutex> lk(g_chain_mu);
        g_chain_launches++;
        g_chain_slices += stop - i0;
    }
    return NNGP_OK;
}

// The fits of the slice the chain stopped at (a miss), from the chain's select workspace, then
// the arg-min, mean and U1[stop+1] = mean + UG1[stop+1]: predict_impl's launches after its select
// on a speculation miss, so the result is bitwise the unfused sweep's.
int chain_miss_fits(int64_t rows, int d, int m, int n_jitter, const double *jitter_exp_host, int n_restarts,
                    const double *theta0, double fatol, double xatol, int maxfev, double *preds,
                    const double *bias, double *out, hipStream_t st) {
    NMArgs a{};
    int rc = fill_jitters(a, n_jitter, jitter_exp_host);
    if (rc) return rc;
    const size_t nd = (size_t)rows + (size_t)m * m + m + (size_t)d * m;
    const size_t n_fits = (size_t)d * n_jitter * n_restarts;
    int err = 0;
    char *ws = (char *)workspace(sizeof(double) * nd + sizeof(int32_t) * 64 + sizeof(double) * 4 * n_fits, &err);
    if (err) return err;
    double *D2 = (double *)ws + rows, *kd2 = D2 + (size_t)m * m, *ymT = kd2 + m;
    double *fits_ws = (double *)(ws + sizeof(double) * nd + sizeof(int32_t) * 64);
    a.m = m; a.d = d; a.n_fits = (int)n_fits;
    a.D2 = D2; a.kd2 = kd2; a.Y = ymT; a.ys_c = m; a.ys_r = 1;
    a.theta0 = theta0; a.fatol = fatol; a.xatol = xatol; a.maxfev = maxfev;
    a.R = n_restarts;
    a.fits_out = fits_ws;
    a.preds = preds; a.bias = bias; a.out = out;
    if (use_spec(a.n_fits, a.m)) {
        rc = run_nm_spec(a, st);
        if (rc) return rc;
        return run_mean(a, st);
    }
    NMArgs u = a;
    u.preds = nullptr; u.out = nullptr; u.bias = nullptr;
    rc = run_nm_parked(u, st);
    if (rc) return rc;
    return run_mean(a, st);
}

}  // namespace nngp

extern "C" int64_t nngp_chain_stats(int64_t *slices_out) {
    std::lock_guard<std::mutex> lk(nngp::g_chain_mu);
    if (slices_out) *slices_out = nngp::g_chain_slices;
    return nngp::g_chain_launches;
}

extern "C" int nngp_predict(const double *X, const double *Y, int64_t rows, int d, const double *new_x,
                            int m, int n_jitter, const double *jitter_exp_host, int n_restarts,
                            const double *theta0, double fatol, double xatol, int maxfev,
                            double *preds_out, const double *bias, double *out, double *fits_out,
                            void *stream) {
    return nngp::predict_impl(X, Y, rows, d, new_x, m, n_jitter, jitter_exp_host, n_restarts, theta0, fatol,
                              xatol, maxfev, preds_out, bias, out, fits_out, nullptr, nullptr, nullptr, nullptr,
                              nullptr, nullptr, (hipStream_t)stream, 0, d, nullptr, nullptr);
}

extern "C" int nngp_predict_range(const double *X, const double *Y, int64_t rows, int d, const double *new_x,
                                  int m, int n_jitter, const double *jitter_exp_host, int n_restarts,
                                  const double *theta0, int c0, int c1, double fatol, double xatol, int maxfev,
                                  double *preds_out, void *stream) {
    return nngp::predict_impl(X, Y, rows, d, new_x, m, n_jitter, jitter_exp_host, n_restarts, theta0, fatol,
                              xatol, maxfev, preds_out, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                              nullptr, nullptr, nullptr, (hipStream_t)stream, c0, c1, nullptr, nullptr);
}
