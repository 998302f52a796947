// nngp_gpeval.h -- the GP likelihood of one fit on one 16-lane DPP row (factor, solves, -LML,
// posterior mean): the evaluation core shared by the fit / mean / chain kernels of nngp_gp.hip
// (and by the micro-benchmarks under tools/).
#pragma once

#include <type_traits>

#include "common.h"
#include "nngp_math.h"

namespace nngp {

static constexpr double LOG_2PI = 1.8378770664093453;   // np.log(2*np.pi)

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---------------------------------------------------------------------------------------------
// GP likelihood of one fit on ONE 16-lane DPP row
//
// A fit owns one row of a wave (lanes 16g .. 16g+15).  Lane l holds rows l and, for m > 16
// (RPL = 2), l+16 of the m x m kernel matrix in VGPRs.  Every cross-lane move of the
// factorisation is a broadcast of one lane to its row -- `v_mov_b64_dpp row_newbcast:L` on
// gfx950, one VALU op, no LDS round trip -- and the two reductions are 4-level DPP butterflies.
// The wave is VALU-issue-bound (tools/ubench_fp64.hip), so the design goal is the smallest
// instruction count per likelihood evaluation:
//   * K's lower triangle (m(m+1)/2 exps) is spread evenly over the 16 lanes (lane l builds
//     entries l, l+16, ... of the flattened triangle, with their D2 values preloaded once per fit)
//     and redistributed to the row owners through a small LDS image;
//   * left-looking Cholesky with row broadcasts; forward solve with broadcasts; back solve from
//     the transposed L read back from the same LDS image.
// Arithmetic order (restated in oracle/nngp_oracle.c gp_factor / butterfly_sum):
//   K_rj = psy*exp(c*D2_rj) (+ jit on the diagonal)                 models.py:146-155, 88
//   L_ij = (K_ij - sum_k L_ik L_jk) * RN(1/L_jj), the sums in OpenBLAS dpotf2_L's order (ddot
//          for the pivot, dgemv_n's 4-column fma blocks / tail-row fma chain below; gp_factor)
//   z, alpha: successive subtraction, k ascending / descending; x/L_ii as Markstein x*RN(1/L_ii)
//   sums over rows: lane pairs (l, l+16) first, then butterfly levels 1, 2, 4, 8
// ---------------------------------------------------------------------------------------------
template <int L>
__device__ __forceinline__ double row_bcast(double v) {   // every lane <- lane L of its 16-row
    return __builtin_amdgcn_mov_dpp(v, 0x150 + L, 0xF, 0xF, false);
}

template <int CTRL>
__device__ __forceinline__ double dpp_mov(double v) {
    return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, false);
}

// sum over the 16 lanes of a row, xor-butterfly order: quad_perm [1,0,3,2], quad_perm [2,3,0,1],
// row_half_mirror, row_mirror.  After level s every lane of an aligned 2s-block holds the same
// partial sum, so the mirrors deliver exactly the xor partner's value; a+b == b+a keeps every
// lane bit-identical.
__device__ __forceinline__ double row_sum(double v) {
    v = v + dpp_mov<0xB1>(v);
    v = v + dpp_mov<0x4E>(v);
    v = v + dpp_mov<0x141>(v);
    v = v + dpp_mov<0x140>(v);
    return v;
}

template <int I, int N, typename F>
__device__ __forceinline__ void static_for(F &&f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for<I + 1, N>(f);
    }
}

// A fit of size m runs padded to MAXM (one of 8, 16, 18, 20, 24, 32, 48, 64): rows m..MAXM-1 are
// identity rows of K with y = 0.  The padded factorisation is exact -- L = [[L_m, 0], [0, I]], z
// and alpha pad with exact zeros, every real row's arithmetic is untouched -- so every loop has a
// compile-time trip count and no per-j branches.
// MAXM <= 32 (one or two rows per lane): the triangle's exps are spread evenly over the 16 lanes
// and redistributed through a full LDS image (stride S).  MAXM > 32 (m > 32: the adaptive
// m = max(10, k+2) past k = 30, or an explicit nn, models.py:172-175): three or four rows per
// lane, each lane builds its own rows' exps in registers (no redistribution), and the LDS image
// is the PACKED lower triangle (row r at r(r+1)/2) that only the back solve reads -- a full image
// would not fit four fits per workgroup in LDS at m = 64.
// the padded sizes, and the smallest m each one serves
__host__ __device__ constexpr int gp_mmin(int maxm) {
    return maxm <= 8 ? 1 : maxm <= 16 ? 9 : maxm <= 18 ? 17 : maxm <= 20 ? 19 : maxm <= 24 ? 21
         : maxm <= 32 ? 25 : maxm <= 48 ? 33 : 49;
}

template <int MAXM_> struct GP {
    static constexpr int MAXM = MAXM_;
    static constexpr int MMIN = gp_mmin(MAXM_);
    static constexpr int RPL = (MAXM + 15) / 16;                        // rows per lane
    static constexpr bool BIG = MAXM > 32;
    static constexpr int S = MAXM + 1;                                  // LDS row stride (pad)
    static constexpr int XOFF = BIG ? 8 * RPL * (16 * RPL + 1)          // K/L image doubles / fit
                                    : MAXM * S;                         // (rows >= MAXM: no image)
    // then the fit's per-row scalars, L_jj | RN(1/L_jj) | z | alpha, MAXM each (gp_factor)
    static constexpr int IMG = XOFF + 4 * MAXM;
    // two row sets per lane (MAXM 20..32): the column pins of gp_factor (see there)
    static constexpr bool PIN = RPL == 2 && !BIG;
    static constexpr int NQ = BIG ? 1 : (MAXM * (MAXM + 1) / 2 + 15) / 16;   // triangle entries / lane
    // can row set s hold a "tail row" of dpotf2's column update (the last (m-1-j) & 3 rows under
    // column j, all >= m - 3 >= MMIN - 3)?  If not, its rows always take the vector-row form and
    // the tail form's fma chain and select are not evaluated: for MAXM = 20 (m = 19, 20) set 0
    // skips 120 fma and 16 selects per evaluation.
    static constexpr bool tail_set(int s) { return 16 * s + 15 >= MMIN - 3; }
};
// LDS offset of K/L entry (r, j), j <= r, in a fit's image
template <int MAXM>
__device__ __forceinline__ int img_at(int r, int j) {
    if constexpr (GP<MAXM>::BIG) return r * (r + 1) / 2 + j;
    else return r * GP<MAXM>::S + j;
}

// per-lane, theta-independent part of a fit: where its share of the triangle lives
// (idxq[q] = diagonal << 30 | D2 index << 16 | K-image slot; D2 index < 2^10, slot < 2^16)
template <int MAXM> struct GPLane {
    int idxq[GP<MAXM>::NQ];
    int nq;           // entries this lane builds (<= NQ)
};

template <int MAXM>
__device__ __forceinline__ void gp_lane_init(GPLane<MAXM> &P, int m, int l) {
    constexpr int S = GP<MAXM>::S;
    const int T = m * (m + 1) / 2;
    P.nq = 0;
    if constexpr (GP<MAXM>::BIG) return;   // rows are built by their owners (gp_factor)
    int r = 0;
#pragma unroll
    for (int q = 0; q < GP<MAXM>::NQ; q++) {
        const int t = l + 16 * q;
        P.idxq[q] = 0;
        if (t < T) {
            while ((r + 1) * (r + 2) / 2 <= t) r++;
            const int j = t - r * (r + 1) / 2;
            P.idxq[q] = ((j == r) << 30) | ((r * m + j) << 16) | (r * S + j);
            P.nq = q + 1;
        }
    }
}

// The fit's LDS image: rows >= m (the pad) are identity rows, written once per kernel and never
// overwritten (the triangle build and the L write-back touch rows < m only).
template <int MAXM>
__device__ __forceinline__ void gp_image_init(double *Kimg, int m, int l) {
    constexpr int RPL = GP<MAXM>::RPL, S = GP<MAXM>::S;
    if constexpr (GP<MAXM>::BIG) {   // packed triangle: every pad-row entry (i >= m, j < i) is 0
        for (int t = l; t < GP<MAXM>::IMG; t += 16) Kimg[t] = 0.0;
        wave_lds_sync();
        return;
    }
#pragma unroll
    for (int s = 0; s < RPL; s++) {
        const int row = l + 16 * s;
        if (row < MAXM)
#pragma unroll
            for (int j = 0; j < MAXM; j++) Kimg[row * S + j] = (row >= m && j == row) ? 1.0 : 0.0;
    }
    wave_lds_sync();
}

// Factor K = psy*exp(c*D2) + jit*I and solve; returns false if potrf fails (jax: NaN).
// alpha[s], diag[s] are those of row l + 16 s (meaningful for rows < m).
template <int MAXM>
__device__ __forceinline__ bool gp_factor(int m, int l, const GPLane<MAXM> &P, const double *sD2,
                                          double c, double psy, double jit,
                                          const double (&y)[GP<MAXM>::RPL], double *Kimg,
                                          double (&alpha)[GP<MAXM>::RPL],
                                          double (&diag)[GP<MAXM>::RPL]) {
    constexpr int RPL = GP<MAXM>::RPL, S = GP<MAXM>::S, NQ = GP<MAXM>::NQ;
    double a[RPL][MAXM];
    if constexpr (!GP<MAXM>::BIG) {
        // 1) this lane's share of the triangle -> LDS image K[r*S + j]
        wave_lds_sync();
#pragma unroll
        for (int q = 0; q < NQ; q++) {
            if (q < P.nq) {
                const int ix = P.idxq[q];
                double e = psy * nn_exp_nonpos(c * sD2[(ix >> 16) & 0x3FF]);   // k_gauss, models.py:146-148
                if (ix >> 30) e = e + jit;                                // + eye*10**jitter, :88
                Kimg[ix & 0xFFFF] = e;
            }
        }
        wave_lds_sync();
        // 2) own rows into registers (pad rows are the image's identity rows, or identity rows
        //    outright past MAXM, which the image does not hold; the upper triangle is never used)
#pragma unroll
        for (int s = 0; s < RPL; s++) {
            const int row = l + 16 * s;
#pragma unroll
            for (int j = 0; j < MAXM; j++)
                if (j < 16 * (s + 1)) a[s][j] = row < MAXM ? Kimg[row * S + j] : (j == row ? 1.0 : 0.0);
        }
    } else {
        // 1+2) each lane builds its own rows (the same expressions, models.py:146-148, 88); pad
        //      rows are identity rows, the upper triangle zeros (never used)
#pragma unroll
        for (int s = 0; s < RPL; s++) {
            const int row = l + 16 * s;
#pragma unroll
            for (int j = 0; j < MAXM; j++) {
                if (j >= 16 * (s + 1)) continue;
                double e = (row >= m && j == row) ? 1.0 : 0.0;
                if (row < m && j <= row) {
                    e = psy * nn_exp_nonpos_sep(c * sD2[row * m + j]);
                    if (j == row) e = e + jit;
                }
                a[s][j] = e;
            }
        }
    }
    // 3) left-looking Cholesky, row j broadcast from lane j%16 of set j/16.  The pivot is
    //    broadcast, so every lane computes L_jj and RN(1/L_jj) identically, and every lane of the
    //    row stores them to the fit's scalar slots Kx[j], Kx[MAXM + j] (the same value to the same
    //    address from all 16 lanes: no lane mask, no VALU -- the owner-only select it replaces
    //    was a v_cmp and two v_cndmask per value, or two v_readlane when LLVM spilled the masks;
    //    z_i and alpha_i of the solves likewise).  Updates of rows < j (upper triangle) are
    //    computed and ignored: fewer instructions than masking them.
    // The lane index, opaque to LLVM: every per-column lane mask ((lane == j % 16), row >=
    // tail_start) is then one v_cmp where it is used.  Visible, LLVM hoisted all of them out of
    // the Nelder-Mead loop as 64-bit SGPR masks, ran out of SGPRs and spilled them to VGPR lanes:
    // two v_readlane per use instead of one compare (and VGPRs held for the spill slots).
    // m likewise (wave-uniform, an SGPR): the per-column tail_start is then two SALU ops where
    // it is used instead of a spilled constant read back by v_readlane.
    int lo = l, mo = m;
    asm volatile("" : "+v"(lo), "+s"(mo));
    // failed pivots as a wave mask (SGPRs): a per-lane bool OR-ed across columns is rebuilt into
    // a mask by a v_cndmask / v_cmp pair at every __all
    uint64_t fmask = 0;
    double *Kx = Kimg + GP<MAXM>::XOFF;   // L_jj | RN(1/L_jj) | z | (spare)
    // the forward solve L z = y (models.py:90, inner solve_triangular) runs fused into the
    // columns: z_j needs row j's accumulator after columns 0..j-1 -- exactly when column j
    // finishes -- so it is formed there, with column j's L_jj / RN(1/L_jj) still in registers
    double acc[RPL];
#pragma unroll
    for (int s = 0; s < RPL; s++) acc[s] = y[s];
    // OpenBLAS dpotf2_L's sums (the reference's LAPACK; oracle potf2_dot / potf2_gemv_row):
    //   pivot   a_jj - ddot(row j): accumulators t1/t2 over groups of 4, fma(x0,x0,x2^2) etc.;
    //   below   "vector rows" (the first ((m-1-j) & -4) rows under j): y -= 4-column fma chains,
    //           leftover columns y -= a*x; "tail rows" (the last (m-1-j) & 3): y -= one fma chain.
    //   Each lane evaluates both row forms (their operation counts add up to the old successive
    //   subtraction's) and keeps the one its row takes.
    // Once EVERY row of the wave has a failed pivot (each row is a fit, or a candidate of one
    // fit), the -LML of all of them is +inf whatever follows: the remaining columns, both solves
    // and the L write-back are skipped (a scalar branch per column).  Fits that wander where the
    // kernel is singular for their jitter -- near-duplicate neighbours, FHN-PDE at its steady
    // state -- evaluate +inf until maxfev (~8 % of a d = 800 correction's fits, the whole tail).
    bool dead = false;   // wave-uniform
    // The pivot's ddot, carried: ddot's accumulators over whole 4-column blocks depend only on the
    // block, so each lane adds every finished block of its OWN rows (D1, D2 per row set) once, as
    // the block's last column completes; column j then needs only D*[SJ] and its 0-3 tail
    // columns (same sums, same order: one block's terms per step instead of all of row j's).
    double D1[RPL], D2[RPL];
#pragma unroll
    for (int s = 0; s < RPL; s++) {
        D1[s] = 0.0;
        D2[s] = 0.0;
    }
    static_for<0, MAXM>([&](auto jc) {
        constexpr int j = decltype(jc)::value, SJ = j / 16, LJ = j % 16;
        if (dead) return;
        const int tail_start = j + 1 + ((mo - 1 - j) & ~3);
        double yv[RPL], tt[RPL], blk[RPL];
#pragma unroll
        for (int s = 0; s < RPL; s++)
            if (16 * (s + 1) > j) {
                yv[s] = a[s][j];
                tt[s] = 0.0;
                blk[s] = 0.0;
            }
#pragma unroll
        for (int k = 0; k < j; k++) {
            const double ljk = row_bcast<LJ>(a[SJ][k]);
#pragma unroll
            for (int s = 0; s < RPL; s++)
                if (16 * (s + 1) > j) {
                    const double ak = a[s][k];
                    if (k < (j & ~3)) {   // whole 4-column blocks of the vector-row form
                        blk[s] = (k % 4 == 0) ? ak * ljk : fma(ak, ljk, blk[s]);
                        if (k % 4 == 3) yv[s] = yv[s] - blk[s];
                    } else {
                        yv[s] = yv[s] - ak * ljk;
                    }
                    if (GP<MAXM>::tail_set(s)) tt[s] = fma(ak, ljk, tt[s]);
                }
        }
        // pivot ddot of the row-j owner's own entries L_jk (its set SJ): the carried blocks, then
        // the tail columns (j & ~3) .. j-1
        double d1 = D1[SJ], d2 = D2[SJ];
#pragma unroll
        for (int k = j & ~3; k < j; k++) d1 = fma(a[SJ][k], a[SJ][k], d1);
        // Pins (two row sets per lane): an empty asm that takes and returns each column's sums,
        // then each finished column.  Nothing is recomputed or reordered arithmetically -- the
        // asm is the identity on the bits -- but LLVM may no longer sink a row set's updates
        // (set 1 never feeds set 0 while j < 16) past later columns, which kept every broadcast
        // L_jk live until then: MAXM = 20 went from 256 VGPRs + 190 AGPRs to 210 VGPRs, i.e. two
        // waves per SIMD instead of one (tools/ubench_gpeval.hip).
        if constexpr (GP<MAXM>::PIN) {
#pragma unroll
            for (int s = 0; s < RPL; s++)
                if (16 * (s + 1) > j) {
                    if (GP<MAXM>::tail_set(s)) asm volatile("" : "+v"(yv[s]), "+v"(tt[s]));
                    else asm volatile("" : "+v"(yv[s]));
                }
        }
        double t[RPL];
#pragma unroll
        for (int s = 0; s < RPL; s++)
            if (16 * (s + 1) > j)
                t[s] = (GP<MAXM>::tail_set(s) && lo + 16 * s >= tail_start) ? a[s][j] - tt[s] : yv[s];
        // every lane forms the ddot pivot of its own set-SJ row; lane LJ's is row j's
        const double piv = row_bcast<LJ>(a[SJ][j] - (d1 + d2));
        fmask |= __builtin_amdgcn_ballot_w64(!(piv > 0.0));
        const uint64_t live = __builtin_amdgcn_read_exec();
        dead = fmask == live;
        // the pivot's sqrt and reciprocal: the short sequences when every live row's pivot is in
        // their range (always, in practice), the full ones otherwise -- the same bits either way
        double ljj, ri;
        if ((fmask | __builtin_amdgcn_ballot_w64(in_mid_range(piv))) == live) {
            ljj = sqrt_mid(piv);
            ri = rcp_mid(ljj);
        } else {
            ljj = sqrt(piv);
            ri = 1.0 / ljj;
        }
        Kx[j] = ljj;
        Kx[MAXM + j] = ri;
        // (the owner's diagonal entry a[SJ][j] becomes t*ri too: nothing reads it -- the solves
        // take L_jj from Kx, and the row-j updates they make after capturing z_j / alpha_j are
        // the harmless ones noted there)
#pragma unroll
        for (int s = 0; s < RPL; s++)
            if (16 * (s + 1) > j) a[s][j] = t[s] * ri;
        if constexpr (GP<MAXM>::PIN) {
#pragma unroll
            for (int s = 0; s < RPL; s++)
                if (16 * (s + 1) > j) asm volatile("" : "+v"(a[s][j]));
        }
        // forward-solve step j: z_j = acc_j / L_jj (Markstein: x * RN(1/L_jj), corrected; every
        // lane divides the broadcast accumulator by the row's L_jj, bitwise the row owner doing it),
        // then the rows below subtract L_ij z_j (rows <= j update harmlessly)
        {
            const double zb = row_bcast<LJ>(acc[SJ]);
            const double q = zb * ri;
            const double zj = fma(fma(-q, ljj, zb), ri, q);
            Kx[2 * MAXM + j] = zj;
#pragma unroll
            for (int s = 0; s < RPL; s++)
                if (16 * (s + 1) > j + 1) acc[s] = acc[s] - a[s][j] * zj;
        }
        // a finished 4-column block: fold it into the carried ddot of every set with rows past j
        if constexpr (j % 4 == 3) {
#pragma unroll
            for (int s = 0; s < RPL; s++)
                if (16 * (s + 1) - 1 > j) {
                    D1[s] = D1[s] + fma(a[s][j - 3], a[s][j - 3], a[s][j - 1] * a[s][j - 1]);
                    D2[s] = D2[s] + fma(a[s][j - 2], a[s][j - 2], a[s][j] * a[s][j]);
                }
        }
    });
    if (dead) {
#pragma unroll
        for (int s = 0; s < RPL; s++) alpha[s] = 0.0;
        return false;
    }
    // 5) back solve L^T alpha = z: L to the LDS image, column of this lane's row(s) back.  L_ii
    //    and RN(1/L_ii) come from the scalar slots (no LDS store in this loop, so LLVM issues
    //    those reads ahead of the chain); alpha_i stays with its row owner by a select.
    wave_lds_sync();
#pragma unroll
    for (int s = 0; s < RPL; s++) {
        const int row = l + 16 * s;
        if (row < m) {   // real rows only: the pad rows of the image stay identity (zero)
#pragma unroll
            for (int j = 0; j < MAXM; j++) {
                if (j >= 16 * (s + 1)) continue;
                if constexpr (GP<MAXM>::BIG) {
                    if (j <= row) Kimg[img_at<MAXM>(row, j)] = a[s][j];
                } else {
                    Kimg[row * S + j] = a[s][j];
                }
            }
        }
    }
    wave_lds_sync();
    // this lane's z and L_ii (rows past MAXM: the pad's exact 0 and 1)
    double acc2[RPL];
#pragma unroll
    for (int s = 0; s < RPL; s++) {
        const int row = l + 16 * s;
        const bool in = 16 * (s + 1) <= MAXM || row < MAXM;
        const int r = min(row, MAXM - 1);
        acc2[s] = in ? Kx[2 * MAXM + r] : 0.0;
        diag[s] = in ? Kx[r] : 1.0;
        alpha[s] = 0.0;
    }
    static_for<0, MAXM>([&](auto ic) {
        constexpr int i = MAXM - 1 - decltype(ic)::value, SI = i / 16, LI = i % 16;
        const double ab = row_bcast<LI>(acc2[SI]);
        const double li = Kx[i], ri = Kx[MAXM + i];
        const double q = ab * ri;
        const double ai = fma(fma(-q, li, ab), ri, q);   // ab / L_ii, as the forward step
        alpha[SI] = (lo == LI) ? ai : alpha[SI];
#pragma unroll
        for (int s = 0; s < RPL; s++)
            if (16 * s < i)   // L[i][row]; rows past MAXM (pads, never read) clamp to the image
                acc2[s] = acc2[s] - Kimg[img_at<MAXM>(i, min(l + 16 * s, MAXM - 1))] * ai;
    });
    return !((fmask >> (__lane_id() & 63)) & 1);
}

// sum over the fit's rows r < m of v[r]: each lane adds its rows l, l+16, l+32, ... left to right
// first, then the row butterfly (oracle butterfly_sum)
template <int RPL>
__device__ __forceinline__ double gp_rows_sum(int m, int l, const double (&v)[RPL]) {
    double p = (l < m) ? v[0] : 0.0;
#pragma unroll
    for (int s = 1; s < RPL; s++) p = p + ((l + 16 * s < m) ? v[s] : 0.0);
    return row_sum(p);
}

// -LML (models.py:240-252): NaN (incl. failed Cholesky) -> +inf
template <int MAXM>
__device__ __forceinline__ double gp_nlml(int m, int l, const GPLane<MAXM> &P, const double *sD2,
                                          double sx, double sy,
                                          double jit, const double (&y)[GP<MAXM>::RPL], double *Kimg) {
    constexpr int RPL = GP<MAXM>::RPL;
    const double c = -0.5 * (1 / nn_pow10(sx));
    const double psy = nn_pow10(sy);
    double alpha[RPL], diag[RPL], ya[RPL], lg[RPL];
    const bool ok = gp_factor<MAXM>(m, l, P, sD2, c, psy, jit, y, Kimg, alpha, diag);
#pragma unroll
    for (int s = 0; s < RPL; s++) {
        ya[s] = y[s] * alpha[s];
        lg[s] = nn_log(diag[s]);
    }
    const double ydot = gp_rows_sum<RPL>(m, l, ya);
    const double slog = gp_rows_sum<RPL>(m, l, lg);
    const double res = -(((-0.5 * ydot) - slog) - ((double)m / 2) * LOG_2PI);
    return (!ok || res != res) ? INFINITY : res;
}

// posterior mean K(xm, new_x)^T alpha (models.py:162-168); NaN on Cholesky failure.  Two parts:
// gp_mean_prep, everything that does not depend on the query (c, psy, alpha and potrf's success),
// and gp_mean_finish, the query's kernel row against alpha -- so a sweep can prepare a hit slice's
// coordinates ahead (gp_pre_kernel) and finish them in its select (bitwise gp_mean: the same
// expressions, and doubles stored and reloaded unchanged).
template <int MAXM>
__device__ __forceinline__ bool gp_mean_prep(int m, int l, const GPLane<MAXM> &P, const double *sD2, double sx,
                                             double sy, double jit, const double (&y)[GP<MAXM>::RPL], double *Kimg,
                                             double (&alpha)[GP<MAXM>::RPL], double &c, double &psy) {
    c = -0.5 * (1 / nn_pow10(sx));
    psy = nn_pow10(sy);
    double diag[GP<MAXM>::RPL];
    return gp_factor<MAXM>(m, l, P, sD2, c, psy, jit, y, Kimg, alpha, diag);
}

// rpl rows per lane (GP<MAXM>::RPL), big = GP<MAXM>::BIG (the exp variant): run-time here, so the
// select kernel can finish a mean for any padded size without one instantiation per size
// kd[s] = kd2 of row l + 16 s (row 0's for rows >= m)
template <int RPLMAX>
__device__ __forceinline__ double gp_mean_finish(int m, int l, int rpl, bool big, const double (&kd)[RPLMAX],
                                                 double c, double psy, const double (&alpha)[RPLMAX], bool ok) {
    double ka[RPLMAX];
#pragma unroll
    for (int s = 0; s < RPLMAX; s++) {
        const double x = c * kd[s];
        ka[s] = (psy * (big ? nn_exp_nonpos_sep(x) : nn_exp_nonpos(x))) * alpha[s];
    }
    // gp_rows_sum<rpl>: the lane's rows left to right, then the row butterfly
    double p = (l < m) ? ka[0] : 0.0;
#pragma unroll
    for (int s = 1; s < RPLMAX; s++)
        if (s < rpl) p = p + ((l + 16 * s < m) ? ka[s] : 0.0);
    const double mean = row_sum(p);
    return ok ? mean : NAN;
}

template <int MAXM>
__device__ __forceinline__ double gp_mean(int m, int l, const GPLane<MAXM> &P, const double *sD2,
                                          const double *skd2,
                                          double sx, double sy, double jit,
                                          const double (&y)[GP<MAXM>::RPL], double *Kimg) {
    constexpr int RPL = GP<MAXM>::RPL;
    double alpha[RPL], c, psy;
    const bool ok = gp_mean_prep<MAXM>(m, l, P, sD2, sx, sy, jit, y, Kimg, alpha, c, psy);
    double kd[RPL];
#pragma unroll
    for (int s = 0; s < RPL; s++) kd[s] = skd2[l + 16 * s < m ? l + 16 * s : 0];
    return gp_mean_finish<RPL>(m, l, RPL, GP<MAXM>::BIG, kd, c, psy, alpha, ok);
}

}  // namespace nngp
