// nngp_nmlane.hip -- the throughput-shaped Nelder-Mead fits kernels: LPF = 4 lanes per fit
// (nm_lane_kernel, the default) or one (nm_lane1_kernel, NNGP_NM_LPF=1), the exact neighbour count
// M as a compile-time constant (no padding).
//
// Reference: NNGP_p.get_preds fans d*9*R independent fits out through pool.map (models.py:185-202);
// each is scipy's Nelder-Mead (models.py:254-260) on the -LML of _fit_gp_jit (models.py:86-92,
// 240-252).  The speculative correction sweep (nngp_sweep.hip) batches every slice's fits of one
// Parareal iteration into ONE launch -- Burgers N = 128: 128 predictions x 1 152 fits = 147 456
// independent fits.  That is throughput work; nm_fit_kernel (nngp_gp.hip) runs a fit on a 16-lane
// DPP row, a layout built for the latency of one fit (~1 830 VALU per wave-evaluation of 4 fits,
// ~29 k issued lane-slots per fit-evaluation, profiles/r04/pmc_burgers_nm_r4c.txt).  Here a fit
// owns LPF lanes of a wave (a quad, or a pair inside one):
//   * lane q holds rows q, q+LPF, q+2 LPF, ... of the M x M kernel matrix (slot s = row / LPF) in
//     VGPRs, only the lower-triangle columns a slot can have (k < LPF s + LPF);
//   * the triangle's exps are the owners' own (no redistribution);
//   * the left-looking Cholesky broadcasts row j's entries L_jk from its owner lane by one
//     quad_perm DPP move (two v_mov_b32_dpp per double) and every lane updates its own rows;
//   * the forward solve runs fused into the columns; the back solve reads the transposed L from a
//     per-fit LDS image (each lane writes its rows once);
//   * the -LML sums use the oracle's butterfly order: xor-partner DPP levels inside the group,
//     the remaining levels inside the lane.
// Every row's arithmetic is the oracle's gp_factor / orc_nlml (oracle/nngp_oracle.c) in the same
// order -- OpenBLAS dpotf2_L's ddot pivot and dgemv_n vector/tail rows, successive-subtraction
// solves with Markstein quotients, the 16-slot butterfly sums -- so the fits are bitwise the
// packed kernel's and the oracle's (tests/test_gpu_kernels.py::test_nm_lanes_kernel_*).
#include <math.h>

#include <algorithm>

#include "common.h"
#include "nngp_gpeval.h"
#include "nngp_math.h"
#include "nngp_nm.h"
#include "nngp_nmargs.h"

namespace nngp {

template <int M, int LPF> struct LaneFit {
    static_assert(LPF == 2 || LPF == 4, "2 or 4 lanes per fit");
    static constexpr int RPL = (M + LPF - 1) / LPF;          // row slots per lane
    static constexpr int NB = 16 / LPF;                      // slots of the 16-entry butterfly
    // columns slot s can hold: rows LPF s .. LPF s + LPF - 1 have entries k <= row
    static constexpr int ncol(int s) { return LPF * s + LPF < M ? LPF * s + LPF : M; }
    // the back solve's LDS image of L, per fit: entry (slot s, column k) of lane q at
    // (off(s, k)) LPF + q -- every lane's addresses are its base plus compile-time offsets
    static constexpr int off(int s, int k) { return s == 0 ? k : off(s - 1, ncol(s - 1)) + k; }
    static constexpr int IMG = (off(RPL - 1, ncol(RPL - 1)) + LPF) * LPF;   // (+ a slot of padding)
    // dpotf2's tail rows of column j start here (the last (M-1-j) & 3 rows under j)
    static constexpr int tail_start(int j) { return j + 1 + ((M - 1 - j) & ~3); }
};

// every lane of the group <- lane SRC of the group (quad_perm)
template <int LPF, int SRC, typename T>
__device__ __forceinline__ T gbcast(T v) {
    if constexpr (LPF == 4) {
        return __builtin_amdgcn_mov_dpp(v, SRC | (SRC << 2) | (SRC << 4) | (SRC << 6), 0xF, 0xF, false);
    } else {
        return __builtin_amdgcn_mov_dpp(v, SRC | (SRC << 2) | ((2 + SRC) << 4) | ((2 + SRC) << 6), 0xF, 0xF, false);
    }
}

// gbcast of a double as ONE volatile asm (two v_mov_b32_dpp, s_nop 1 first for the DPP read
// hazard), which also takes two values of the previous k's updates (dep0, dep1; unused): the
// broadcast of x_k then waits for them, so at most one or two x's are live -- left free, LLVM
// computed every column's broadcasts up front (~34 broadcast doubles live at M = 15's peak)
template <int LPF, int SRC>
__device__ __forceinline__ double gbcast_pinned(double v, double dep0, double dep1) {
    constexpr int Q0 = SRC, Q2 = LPF == 4 ? SRC : 2 + SRC;
    static_assert(Q0 < 4 && Q2 < 4, "quad lane");
    uint32_t lo = (uint32_t)__double_as_longlong(v), hi = (uint32_t)(__double_as_longlong(v) >> 32);
    uint32_t olo, ohi;
    if constexpr (Q0 == 0 && Q2 == 0)
        asm volatile("s_nop 1\n\tv_mov_b32_dpp %0, %2 quad_perm:[0,0,0,0] row_mask:0xf bank_mask:0xf\n\t"
                     "v_mov_b32_dpp %1, %3 quad_perm:[0,0,0,0] row_mask:0xf bank_mask:0xf"
                     : "=&v"(olo), "=&v"(ohi) : "v"(lo), "v"(hi), "v"(dep0), "v"(dep1));
    else if constexpr (Q0 == 1 && Q2 == 1)
        asm volatile("s_nop 1\n\tv_mov_b32_dpp %0, %2 quad_perm:[1,1,1,1] row_mask:0xf bank_mask:0xf\n\t"
                     "v_mov_b32_dpp %1, %3 quad_perm:[1,1,1,1] row_mask:0xf bank_mask:0xf"
                     : "=&v"(olo), "=&v"(ohi) : "v"(lo), "v"(hi), "v"(dep0), "v"(dep1));
    else if constexpr (Q0 == 2 && Q2 == 2)
        asm volatile("s_nop 1\n\tv_mov_b32_dpp %0, %2 quad_perm:[2,2,2,2] row_mask:0xf bank_mask:0xf\n\t"
                     "v_mov_b32_dpp %1, %3 quad_perm:[2,2,2,2] row_mask:0xf bank_mask:0xf"
                     : "=&v"(olo), "=&v"(ohi) : "v"(lo), "v"(hi), "v"(dep0), "v"(dep1));
    else if constexpr (Q0 == 3 && Q2 == 3)
        asm volatile("s_nop 1\n\tv_mov_b32_dpp %0, %2 quad_perm:[3,3,3,3] row_mask:0xf bank_mask:0xf\n\t"
                     "v_mov_b32_dpp %1, %3 quad_perm:[3,3,3,3] row_mask:0xf bank_mask:0xf"
                     : "=&v"(olo), "=&v"(ohi) : "v"(lo), "v"(hi), "v"(dep0), "v"(dep1));
    else if constexpr (Q0 == 0)
        asm volatile("s_nop 1\n\tv_mov_b32_dpp %0, %2 quad_perm:[0,0,2,2] row_mask:0xf bank_mask:0xf\n\t"
                     "v_mov_b32_dpp %1, %3 quad_perm:[0,0,2,2] row_mask:0xf bank_mask:0xf"
                     : "=&v"(olo), "=&v"(ohi) : "v"(lo), "v"(hi), "v"(dep0), "v"(dep1));
    else
        asm volatile("s_nop 1\n\tv_mov_b32_dpp %0, %2 quad_perm:[1,1,3,3] row_mask:0xf bank_mask:0xf\n\t"
                     "v_mov_b32_dpp %1, %3 quad_perm:[1,1,3,3] row_mask:0xf bank_mask:0xf"
                     : "=&v"(olo), "=&v"(ohi) : "v"(lo), "v"(hi), "v"(dep0), "v"(dep1));
    return __longlong_as_double((long long)(((uint64_t)ohi << 32) | olo));
}

// xor partner inside the group: 1 -> quad_perm [1,0,3,2], 2 -> [2,3,0,1]
template <int X>
__device__ __forceinline__ double xor_dpp(double v) {
    return __builtin_amdgcn_mov_dpp(v, X == 1 ? 0xB1 : 0x4E, 0xF, 0xF, false);
}

// x / L_ii as the oracle's Markstein quotient: q = x RN(1/L_ii), fma(fma(-q, L_ii, x), RN(1/L_ii), q)
__device__ __forceinline__ double mk_div(double x, double lii, double ri) {
    const double q = x * ri;
    return fma(fma(-q, lii, x), ri, q);
}

// ljj = sqrt(x), ri = 1.0/ljj, both correctly rounded, for every x > 0 (the pivots that pass):
// the short mid-range sequences (nngp_math.h sqrt_mid / rcp_mid, exact on [2^-500, 2^500]) on x
// scaled by 4^k, k in {300, 0, -300}, and the results scaled back by 2^-k / 2^k -- exact, since
// sqrt(x 4^k) = sqrt(x) 2^k and both results stay normal (sqrt(x) in [2^-537, 2^512]).  x = +inf
// gives (inf, 0) as sqrt / division do.  Branch-free: a uniform branch to the full sequences was
// if-converted by LLVM, which then ran both (and held both's registers) at every column.
__device__ __forceinline__ void sqrt_rcp_exact(double x, double &ljj, double &ri) {
    const int k = x < 0x1p-500 ? 300 : (x > 0x1p+500 ? -300 : 0);
    const double s = sqrt_mid(ldexp(x, 2 * k));
    const double r = rcp_mid(s);
    // +inf -> (inf, 0) by bit masks, not a select: LLVM turned the select into a branch around the
    // whole sequence (a divergent branch per column, values spilled across it)
    const long long m = -(long long)(x == __builtin_huge_val());   // all ones for +inf
    const long long ls = __double_as_longlong(ldexp(s, -k)), lr = __double_as_longlong(ldexp(r, k));
    ljj = __longlong_as_double((ls & ~m) | (0x7FF0000000000000ll & m));
    ri = __longlong_as_double(lr & ~m);
}

// oracle butterfly_sum over the fit's rows r < M of v[r] (row r = LPF s + q in slot s of lane q):
// fold rows >= 16 into rows r mod 16 (adding the oracle's 0.0 for missing ones), then levels
// 1, 2, 4, 8 -- the ones below LPF across the group's lanes, the rest inside the lane
template <int M, int LPF>
__device__ __forceinline__ double lane_bsum(const double (&v)[LaneFit<M, LPF>::RPL], int q) {
    constexpr int NB = LaneFit<M, LPF>::NB, RPL = LaneFit<M, LPF>::RPL;
    double p[NB];
#pragma unroll
    for (int s = 0; s < NB; s++) {
        p[s] = (s < RPL && LPF * s + q < M) ? v[s < RPL ? s : 0] : 0.0;
#pragma unroll
        for (int f = 1; 16 * f < M; f++) {
            const int s2 = s + f * NB;
            p[s] = p[s] + ((s2 < RPL && LPF * s2 + q < M) ? v[s2 < RPL ? s2 : 0] : 0.0);
        }
    }
#pragma unroll
    for (int s = 0; s < NB; s++) {
        p[s] = p[s] + xor_dpp<1>(p[s]);
        if constexpr (LPF == 4) p[s] = p[s] + xor_dpp<2>(p[s]);
    }
#pragma unroll
    for (int st = 1; st < NB; st <<= 1)
#pragma unroll
        for (int s = 0; s < NB; s += 2 * st) p[s] = p[s] + p[s + st];
    return p[0];
}

// -LML (models.py:240-252) of the fit this lane's group owns at (sx, sy); +inf on NaN or a failed
// Cholesky.  ys: the group's y rows of this lane; sD2: [M][M]; img: the group's LDS image.
template <int M, int LPF>
__device__ __forceinline__ double lane_nlml(int q, const double *sD2, double sx, double sy, double jit,
                                            const double (&ys)[LaneFit<M, LPF>::RPL], double *img) {
    using LF = LaneFit<M, LPF>;
    constexpr int RPL = LF::RPL;
    const double c = -0.5 * (1 / nn_pow10(sx));
    const double psy = nn_pow10(sy);
    double a[RPL][M];
    // the owners' triangle entries: K_rk = psy exp(c D2_rk) (+ jit on the diagonal), models.py:146-155, 88
    // (D2 row LPF s + q at this lane's base q M plus a constant; rows >= M read harmless LDS)
    // The exps run as a chain, at most two in flight: entry t's D2 load waits (a "memory" pin)
    // until entry t-2's exp is done.  Left free, LLVM interleaves all ~40 independent exps of the
    // lane for ILP and holds their ~6 VGPRs each at once (256 VGPRs + 194 AGPRs at M = 15); a wave's
    // dependent fp64 ops issue as fast as independent ones (tools/ubench_fp64.hip), so nothing is lost.
    const double *d2q = sD2 + q * M;
    double e1 = 0.0, e2 = 0.0;   // the last two entries
#pragma unroll
    for (int s = 0; s < RPL; s++) {
#pragma unroll
        for (int k = 0; k < M; k++) {
            if (k >= LF::ncol(s)) continue;
            asm volatile("" ::"v"(e2) : "memory");
            double e = psy * nn_exp_nonpos(c * d2q[LPF * s * M + k]);
            if (k >= LPF * s) e = (k == LPF * s + q) ? e + jit : e;
            a[s][k] = e;
            e2 = e1;
            e1 = e;
        }
    }
    double acc[RPL], dg[RPL], rv[RPL];
#pragma unroll
    for (int s = 0; s < RPL; s++) {
        acc[s] = ys[s];
        dg[s] = 1.0;
        rv[s] = 1.0;
    }
    bool bad = false;
    static_for<0, M>([&](auto jc) {
        constexpr int j = decltype(jc)::value, SJ = j / LPF, QJ = j % LPF;
        constexpr int TS = LF::tail_start(j), JB = j & ~3;
        // pivot: a_jj - ddot(row j) (potf2_dot: two accumulators over groups of 4, fma tail)
        double t1 = 0.0, t2 = 0.0;
#pragma unroll
        for (int k = 0; k + 4 <= j; k += 4) {
            t1 = t1 + fma(a[SJ][k], a[SJ][k], a[SJ][k + 2] * a[SJ][k + 2]);
            t2 = t2 + fma(a[SJ][k + 1], a[SJ][k + 1], a[SJ][k + 3] * a[SJ][k + 3]);
        }
#pragma unroll
        for (int k = JB; k < j; k++) t1 = fma(a[SJ][k], a[SJ][k], t1);
        const double pv = gbcast<LPF, QJ>(a[SJ][j] - (t1 + t2));
        bad = bad || !(pv > 0.0);
        double ljj, ri;
        sqrt_rcp_exact(pv, ljj, ri);
        dg[SJ] = (q == QJ) ? ljj : dg[SJ];
        rv[SJ] = (q == QJ) ? ri : rv[SJ];
        // rows below j (dgemv_n, then * RN(1/ajj)): vector rows y -= 4-column fma blocks, leftover
        // columns y -= a x; tail rows y -= one fma chain.  x_k = L_jk from the owner, k ascending.
        double yv[RPL], bk[RPL], tt[RPL];
#pragma unroll
        for (int s = SJ; s < RPL; s++) {
            yv[s] = a[s][j];
            bk[s] = 0.0;
            tt[s] = 0.0;
        }
#pragma unroll
        for (int k = 0; k < j; k++) {
            // (the first broadcast of a column also waits for the previous column's last-slot
            // result: most of a left-looking column's products do not depend on the column before,
            // and LLVM otherwise ran columns ahead, holding their partial sums and x's)
            const double xk = gbcast_pinned<LPF, QJ>(a[SJ][k], (k == 0 && j > 0) ? a[RPL - 1][j > 0 ? j - 1 : 0]
                                                                                 : bk[RPL - 1], tt[RPL - 1]);
#pragma unroll
            for (int s = SJ; s < RPL; s++) {
                const bool vec = LPF * s < TS, tail = LPF * s + LPF - 1 >= TS;
                const double ak = a[s][k];
                if (vec) {
                    if (k < JB) {
                        bk[s] = (k % 4 == 0) ? ak * xk : fma(ak, xk, bk[s]);
                        if (k % 4 == 3) yv[s] = yv[s] - bk[s];
                    } else {
                        yv[s] = yv[s] - ak * xk;
                    }
                }
                if (tail) tt[s] = fma(ak, xk, tt[s]);
            }
        }
#pragma unroll
        for (int s = SJ; s < RPL; s++) {
            const bool vec = LPF * s < TS, tail = LPF * s + LPF - 1 >= TS;
            double y = vec ? yv[s] : a[s][j] - tt[s];
            if (vec && tail) y = (LPF * s + q < TS) ? yv[s] : a[s][j] - tt[s];
            // (rows <= j of slot SJ store garbage here: their entry j is above the diagonal, or --
            // for row j itself -- the diagonal K_jj, which nothing reads after the pivot; the back
            // solve's image takes the strictly lower entries only.  A select kept the old values
            // alive: 64 VGPRs at M = 15.)
            a[s][j] = y * ri;
        }
        // forward solve, fused: z_j = acc_j / L_jj, then rows below subtract L_ij z_j (models.py:90)
        const double zj = mk_div(gbcast<LPF, QJ>(acc[SJ]), ljj, ri);
        acc[SJ] = (q == QJ) ? zj : acc[SJ];   // acc of row j becomes z_j
#pragma unroll
        for (int s = SJ; s < RPL; s++) {
            if (s > SJ) acc[s] = acc[s] - a[s][j] * zj;
            else acc[s] = (q > QJ) ? acc[s] - a[s][j] * zj : acc[s];
        }
    });
    // back solve L^T alpha = z: the lanes' rows of L into the fit's LDS image, then alpha_i
    // (descending) from its owner, and every lane subtracts L_ir alpha_i from its rows r < i (k
    // descending, the oracle's order), L_ir read back from the image.  The image is rewritten every
    // evaluation: the first sync orders these writes after the previous evaluation's reads.
    wave_lds_sync();
    double *imw = img + q;
#pragma unroll
    for (int s = 0; s < RPL; s++)
#pragma unroll
        for (int k = 0; k < M - 1; k++)
            if (k < LF::ncol(s)) imw[LF::off(s, k) * LPF] = a[s][k];
    wave_lds_sync();
    const double *imr = img + q * LPF;   // + (off(SI, LPF s) ) LPF + QI: row i's column LPF s + q
    double al[RPL];
#pragma unroll
    for (int s = 0; s < RPL; s++) al[s] = 0.0;
    static_for<0, M>([&](auto ic) {
        constexpr int i = M - 1 - decltype(ic)::value, SI = i / LPF, QI = i % LPF;
        const double ai = gbcast<LPF, QI>(mk_div(acc[SI], dg[SI], rv[SI]));
        al[SI] = (q == QI) ? ai : al[SI];
#pragma unroll
        for (int s = 0; s <= SI; s++) {
            if (LPF * s >= i) continue;   // no row of the slot is below i
            const double lir = imr[LF::off(SI, LPF * s) * LPF + QI];
            if (LPF * s + LPF - 1 < i) acc[s] = acc[s] - lir * ai;
            else acc[s] = (LPF * s + q < i) ? acc[s] - lir * ai : acc[s];
        }
    });
    double ya[RPL], lg[RPL];
#pragma unroll
    for (int s = 0; s < RPL; s++) {
        ya[s] = ys[s] * al[s];
        lg[s] = nn_log(dg[s]);
    }
    const double ydot = lane_bsum<M, LPF>(ya, q);
    const double slog = lane_bsum<M, LPF>(lg, q);
    const double res = -(((-0.5 * ydot) - slog) - ((double)M / 2) * LOG_2PI);
    // every lane of the group has the same bits: the pivots and sums are broadcast / symmetric
    return (bad || res != res) ? INFINITY : res;
}

// One fit per LPF lanes; unfused batched mode (blockIdx.y = prediction, product-order fits or
// explicit coord / jitter arrays), work queue per prediction.
template <int M, int LPF>
__global__ void __launch_bounds__(256) nm_lane_kernel(NMArgs a) {
    using LF = LaneFit<M, LPF>;
    constexpr int RPL = LF::RPL;
    extern __shared__ __attribute__((aligned(16))) double sm[];
    if (a.skip && *a.skip) return;
    nm_batch_offsets(a);
    const int nfc = a.nj * a.R;
    const int ngroups = blockDim.x / LPF;
    double *sD2 = sm;
    double *sImg = sD2 + M * M;
    __shared__ double sJit[MAX_JIT];
    const int tid = threadIdx.x;
    for (int i = tid; i < M * M; i += blockDim.x) sD2[i] = a.D2[i];
    if (tid < MAX_JIT) sJit[tid] = jit_lookup(a, tid);
    __syncthreads();
    const int g = tid / LPF;
    int q = tid % LPF;
    asm volatile("" : "+v"(q));   // opaque: per-column lane masks stay one compare where used
    double *img = sImg + (size_t)g * LF::IMG;
    NMCfg cfg{a.fatol, a.xatol, a.maxfev, a.maxfev};
    NM St;
    double ys[RPL];
    double jit = 1.0;
    int fn = blockIdx.x * ngroups + g, f = 0;
    bool valid = false;
    auto start_fit = [&]() {
        valid = fn < a.n_fits;
        f = fn;
        if (valid && a.jmajor && !a.coord) f = (fn % a.d) * nfc + fn / a.d;
        int coord = 0, jidx = 0;
        if (valid) {
            if (a.coord) {
                coord = a.coord[f];
                jidx = a.jitter_idx[f];
            } else {   // product(coord, jitter, restart) order (models.py:186)
                coord = f / nfc;
                jidx = (f % nfc) / a.R;
            }
        }
#pragma unroll
        for (int s = 0; s < RPL; s++) {
            const int row = LPF * s + q;
            ys[s] = (valid && row < M) ? a.Y[(int64_t)coord * a.ys_c + (int64_t)row * a.ys_r] : 0.0;
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
        if (!valid || q != 0) return;
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
        if (a.done) {   // the fit is visible device-wide before it is counted
            __threadfence();
            __hip_atomic_fetch_add(a.done + blockIdx.y, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    };
    start_fit();
    bool can_take = a.queue != nullptr && valid;
    // every group of the wave evaluates once per trip until the wave's last fit is done (finished
    // groups evaluate a dummy point, so the evaluation never diverges); a finished group first
    // takes the next unassigned fit of its prediction from the queue
    while (true) {
        if (can_take && St.st == ST_DONE) {   // uniform within the group
            write_fit();
            int nf = 0;
            if (q == 0) nf = (int)(gridDim.x * ngroups) + atomicAdd(a.queue + blockIdx.y, 1);
            fn = gbcast<LPF, 0>(nf);
            start_fit();
            can_take = valid;
        }
        const bool need = St.st != ST_DONE;
        if (!__any(need)) break;
        const double fv = lane_nlml<M, LPF>(q, sD2, St.px, St.py, jit, ys, img);
        if (need) nm_consume(St, cfg, fv);
    }
    write_fit();
}

// ---------------------------------------------------------------------------------------------
// One fit per lane (LPF = 1): 64 fits per wave, no cross-lane traffic at all.
//
// A lane holds its fit's whole lower triangle (M(M+1)/2 doubles, K overwritten in place by L, the
// diagonal by L_jj) in registers -- more than 256 VGPRs from M = 15 on, so the kernel runs one
// wave per SIMD with the AGPR half of the register file; a wave's dependent fp64 ops issue as fast
// as independent ones (tools/ubench_fp64.hip), so one wave keeps the SIMD's VALU busy.  The D^2
// entries are wave-uniform (a workgroup serves one prediction): LDS reads every lane of a wave
// makes at the same address (a broadcast, no bank conflicts).  The arithmetic of every
// entry is lane_nlml's / the oracle's (gp_factor, orc_nlml), only scheduled row by row:
//   * L_ij, i > j: dpotf2_L's vector-row / tail-row forms, chosen at compile time (M is exact);
//   * z: acc_i = y_i - L_i0 z_0 - L_i1 z_1 - ... (k ascending), z_i = acc_i / L_ii (Markstein) --
//     the fused forward solve's order;
//   * alpha: acc_r = z_r - L_{M-1,r} alpha_{M-1} - ... (i descending), the back solve's order;
//   * the two sums: the 16-slot butterfly, all levels inside the lane.
// Issued instructions per fit-evaluation drop ~3x against LPF = 4 (no replicated pivots, no
// broadcasts, no masked rows, no DPP hazards; tools/nm_lanes_probe.py).
// ---------------------------------------------------------------------------------------------
template <int M> struct Lane1 {
    static constexpr int T = M * (M + 1) / 2;
    static constexpr int at(int r, int k) { return r * (r + 1) / 2 + k; }
    static constexpr int tail_start(int j) { return j + 1 + ((M - 1 - j) & ~3); }
};

// threads of the one-fit-per-lane kernel's workgroup = the row stride of its LDS y columns
static constexpr int LANE1_THREADS = 256;

// ys: this lane's y column in LDS, row r at ys[r * LANE1_THREADS]
template <int M>
__device__ __forceinline__ double lane1_nlml(const double *D2, double sx, double sy, double jit, const double *ys) {
    using LF = Lane1<M>;
    const double c = -0.5 * (1 / nn_pow10(sx));
    const double psy = nn_pow10(sy);
    double a[LF::T];
    // K_rk = psy exp(c D2_rk) (+ jit on the diagonal), models.py:146-155, 88; the exps as a chain
    // (see lane_nlml): at most two in flight
    double e1 = 0.0, e2 = 0.0;
    static_for<0, M>([&](auto rc) {
        constexpr int r = decltype(rc)::value;
        static_for<0, r + 1>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            asm volatile("" ::"v"(e2) : "memory");
            double e = psy * nn_exp_nonpos(c * D2[r * M + k]);
            if constexpr (k == r) e = e + jit;
            a[LF::at(r, k)] = e;
            e2 = e1;
            e1 = e;
        });
    });
    bool bad = false;
    double ri[M];
    static_for<0, M>([&](auto jc) {
        constexpr int j = decltype(jc)::value, JB = j & ~3, TS = LF::tail_start(j);
        // pivot: a_jj - ddot(row j) (potf2_dot)
        double t1 = 0.0, t2 = 0.0;
#pragma unroll
        for (int k = 0; k + 4 <= j; k += 4) {
            t1 = t1 + fma(a[LF::at(j, k)], a[LF::at(j, k)], a[LF::at(j, k + 2)] * a[LF::at(j, k + 2)]);
            t2 = t2 + fma(a[LF::at(j, k + 1)], a[LF::at(j, k + 1)], a[LF::at(j, k + 3)] * a[LF::at(j, k + 3)]);
        }
#pragma unroll
        for (int k = JB; k < j; k++) t1 = fma(a[LF::at(j, k)], a[LF::at(j, k)], t1);
        const double pv = a[LF::at(j, j)] - (t1 + t2);
        bad = bad || !(pv > 0.0);
        double ljj, rj;
        sqrt_rcp_exact(pv, ljj, rj);
        a[LF::at(j, j)] = ljj;
        ri[j] = rj;
        // rows below j: dgemv_n's vector rows (y -= 4-column fma blocks, leftover y -= a x) and
        // tail rows (y -= one fma chain), then * RN(1/L_jj)
        static_for<j + 1, M>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            double y;
            if constexpr (i < TS) {
                double yv = a[LF::at(i, j)], bk = 0.0;
#pragma unroll
                for (int k = 0; k < j; k++) {
                    const double p = a[LF::at(i, k)], x = a[LF::at(j, k)];
                    if (k < JB) {
                        bk = (k % 4 == 0) ? p * x : fma(p, x, bk);
                        if (k % 4 == 3) yv = yv - bk;
                    } else {
                        yv = yv - p * x;
                    }
                }
                y = yv;
            } else {
                double tt = 0.0;
#pragma unroll
                for (int k = 0; k < j; k++) tt = fma(a[LF::at(i, k)], a[LF::at(j, k)], tt);
                y = a[LF::at(i, j)] - tt;
            }
            a[LF::at(i, j)] = y * rj;
        });
    });
    // forward solve L z = y (models.py:90), row by row in the fused solve's order
    double z[M];
    static_for<0, M>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        double acc = ys[i * LANE1_THREADS];
#pragma unroll
        for (int k = 0; k < i; k++) acc = acc - a[LF::at(i, k)] * z[k];
        z[i] = mk_div(acc, a[LF::at(i, i)], ri[i]);
    });
    // back solve L^T alpha = z, rows descending, each row's terms i descending (alpha over z)
    static_for<0, M>([&](auto rc) {
        constexpr int r = M - 1 - decltype(rc)::value;
        double acc = z[r];
#pragma unroll
        for (int i = M - 1; i > r; i--) acc = acc - a[LF::at(i, r)] * z[i];
        z[r] = mk_div(acc, a[LF::at(r, r)], ri[r]);
    });
    // -LML: the oracle's 16-slot butterflies of y_r alpha_r and log L_rr
    double py[16], pl[16];
#pragma unroll
    for (int s = 0; s < 16; s++) {
        py[s] = s < M ? ys[(s < M ? s : 0) * LANE1_THREADS] * z[s < M ? s : 0] : 0.0;
        pl[s] = s < M ? nn_log(a[LF::at(s < M ? s : 0, s < M ? s : 0)]) : 0.0;
#pragma unroll
        for (int f = 1; 16 * f < M; f++) {
            const int r = s + 16 * f;
            py[s] = py[s] + (r < M ? ys[(r < M ? r : 0) * LANE1_THREADS] * z[r < M ? r : 0] : 0.0);
            pl[s] = pl[s] + (r < M ? nn_log(a[LF::at(r < M ? r : 0, r < M ? r : 0)]) : 0.0);
        }
    }
#pragma unroll
    for (int st = 1; st < 16; st <<= 1)
#pragma unroll
        for (int s = 0; s < 16; s += 2 * st) {
            py[s] = py[s] + py[s + st];
            pl[s] = pl[s] + pl[s + st];
        }
    const double res = -(((-0.5 * py[0]) - pl[0]) - ((double)M / 2) * LOG_2PI);
    return (bad || res != res) ? INFINITY : res;
}

// One fit per lane; unfused batched mode (blockIdx.y = prediction), work queue per prediction.
template <int M>
__global__ void __launch_bounds__(LANE1_THREADS) nm_lane1_kernel(NMArgs a) {
    if (a.skip && *a.skip) return;
    nm_batch_offsets(a);
    const int nfc = a.nj * a.R;
    extern __shared__ __attribute__((aligned(16))) double sm[];
    double *sD2 = sm;
    const int tid = threadIdx.x;
    double *ys = sm + M * M + tid;   // this lane's y column, row r at ys[r * LANE1_THREADS]
    for (int i = tid; i < M * M; i += blockDim.x) sD2[i] = a.D2[i];
    __syncthreads();
    NMCfg cfg{a.fatol, a.xatol, a.maxfev, a.maxfev};
    NM St;
    double jit = 1.0;
    int fn = blockIdx.x * blockDim.x + tid, f = 0;
    bool valid = false;
    auto start_fit = [&]() {
        valid = fn < a.n_fits;
        f = fn;
        if (valid && a.jmajor && !a.coord) f = (fn % a.d) * nfc + fn / a.d;
        int coord = 0, jidx = 0;
        if (valid) {
            if (a.coord) {
                coord = a.coord[f];
                jidx = a.jitter_idx[f];
            } else {   // product(coord, jitter, restart) order (models.py:186)
                coord = f / nfc;
                jidx = (f % nfc) / a.R;
            }
        }
#pragma unroll
        for (int r = 0; r < M; r++) ys[r * LANE1_THREADS] = valid ? a.Y[(int64_t)coord * a.ys_c + (int64_t)r * a.ys_r] : 0.0;
        jit = valid ? jit_lookup(a, jidx) : 1.0;
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
        if (!valid) return;
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
        if (a.done) {   // the fit is visible device-wide before it is counted
            __threadfence();
            __hip_atomic_fetch_add(a.done + blockIdx.y, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    };
    start_fit();
    bool can_take = a.queue != nullptr && valid;
    // every lane evaluates once per trip until the wave's last fit is done (finished lanes
    // evaluate their last point again, discarded); a finished lane first takes the next
    // unassigned fit of its prediction from the queue
    while (true) {
        if (can_take && St.st == ST_DONE) {
            write_fit();
            fn = (int)(gridDim.x * blockDim.x) + atomicAdd(a.queue + blockIdx.y, 1);
            start_fit();
            can_take = valid;
        }
        const bool need = St.st != ST_DONE;
        if (!__any(need)) break;
        const double fv = lane1_nlml<M>(sD2, St.px, St.py, jit, ys);
        if (need) nm_consume(St, cfg, fv);
    }
    write_fit();
}

// instantiated neighbour counts: the speculative batches of the BASELINE configs (Burgers nn = 15,
// Hopf / Lorenz 10-15).  LPF = 4 (lane_nlml) or 1 (lane1_nlml, NNGP_NM_LPF=1).  (m >= 17 needs
// more than a lane's 256 VGPRs at LPF = 4 -- the packed kernel serves it.)
template <typename F>
static int with_lane_m(int m, F &&f) {
    switch (m) {
    case 10: return f(std::integral_constant<int, 10>{});
    case 15: return f(std::integral_constant<int, 15>{});
    default: return NNGP_E_UNSUPPORTED;
    }
}

bool nm_lanes_supported(int m) {
    return with_lane_m(m, [](auto) { return NNGP_OK; }) == NNGP_OK;
}

static int lanes_lpf() {
    return env_int("NNGP_NM_LPF", 4) == 1 ? 1 : 4;
}

// Grid of a batched launch: the work queue lets a group (LPF lanes) that finished its fit take the
// next unassigned fit of its prediction, so the grid only has to fill the chip once -- the
// workgroups the occupancy calculator says fit at a time (registers and LDS: at 256 threads the
// 4-lane kernel's LDS images allow one workgroup per CU), spread over the nq predictions -- and
// never needs more workgroups than a prediction has fits (one fit per group, no queue).  A
// fixed "8 fits per group" grid, round 5's first cut, left a one-prediction batch of 18 432 fits
// on 144 waves (profiles/r05/nm_lanes/).  NNGP_NM_LANES_FILL (percent, default 100) sizes the
// grid to that share of the resident workgroups: the batch shares the chip with the sweep it
// feeds.  NNGP_NM_REFILL = 0 / 1: no queue, one fit per group.
template <typename K>
static int lanes_grid(NMArgs &a, hipStream_t st, int nq, int qslot, K kernel, int threads, size_t lds, int ngroups,
                      int &nblocks) {
    const int full = (a.n_fits + ngroups - 1) / ngroups;   // one fit per group
    nblocks = full;
    a.queue = nullptr;
    if (env_int("NNGP_NM_REFILL", 8) <= 1 || full <= 1) return NNGP_OK;
    int per_cu = 0;
    NNGP_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, threads, lds));
    const int fill = std::min(100, std::max(1, env_int("NNGP_NM_LANES_FILL", 100)));
    const int64_t resident = std::max<int64_t>(1, (int64_t)std::max(per_cu, 1) * device_cus() * fill / 100);
    // (rounded down: a rounded-up share left the last predictions' workgroups waiting for a slot
    // and running after everything else -- Burgers' 125-prediction batch, 3 x 125 workgroups for
    // 256 slots, took 9 ms in the run against 6.4 ms for one prediction of the same fit count)
    const int per_pred = (int)std::max<int64_t>(1, resident / nq);
    if (per_pred >= full) return NNGP_OK;
    int err = 0;
    int32_t *qbuf = (int32_t *)workspace(sizeof(int32_t) * (size_t)nq, &err, qslot);
    if (err) return err;
    NNGP_HIP_CHECK(hipMemsetAsync(qbuf, 0, sizeof(int32_t) * (size_t)nq, st));
    a.queue = qbuf;
    nblocks = per_pred;
    return NNGP_OK;
}

int run_nm_lanes(NMArgs &a, hipStream_t st, int nq, int qslot) {
    if (lanes_lpf() == 1) {
        return with_lane_m(a.m, [&](auto mc) {
            constexpr int M = decltype(mc)::value;
            const int threads = LANE1_THREADS;
            const size_t lds = sizeof(double) * (M * M + LANE1_THREADS * M);
            int nblocks = 0;
            const int err = lanes_grid(a, st, nq, qslot, nm_lane1_kernel<M>, threads, lds, threads, nblocks);
            if (err) return err;
            hipLaunchKernelGGL((nm_lane1_kernel<M>), dim3(nblocks, nq), dim3(threads), lds, st, a);
            NNGP_LAUNCH_CHECK();
            return NNGP_OK;
        });
    }
    return with_lane_m(a.m, [&](auto mc) {
        constexpr int M = decltype(mc)::value, LPF = 4;
        // workgroup size (NNGP_NM_LANES_WG: 64 / 128 / 256): the LDS images allow 1 / 3 / 7
        // workgroups of 256 / 128 / 64 threads per CU.  Burgers N = 128 to convergence (medians of
        // 3, profiles/r05/nm_lanes/grid_floor_ab_wg.txt): 0.231 / 0.221 / 0.223 s
        const int wg = env_int("NNGP_NM_LANES_WG", 128);
        const int threads = (wg == 64 || wg == 128) ? wg : 256, ngroups = threads / LPF;
        const size_t lds = sizeof(double) * ((size_t)M * M + (size_t)ngroups * LaneFit<M, LPF>::IMG);
        int nblocks = 0;
        const int err = lanes_grid(a, st, nq, qslot, nm_lane_kernel<M, LPF>, threads, lds, ngroups, nblocks);
        if (err) return err;
        hipLaunchKernelGGL((nm_lane_kernel<M, LPF>), dim3(nblocks, nq), dim3(threads), lds, st, a);
        NNGP_LAUNCH_CHECK();
        return NNGP_OK;
    });
}

}  // namespace nngp
