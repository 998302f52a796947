// nngp_rk_dev.h -- device building blocks of the RK propagators, shared by nngp_rk.hip (the
// batched F/G kernels, exact and contracted builds) and nngp_gp.hip (the fused correction chain,
// whose in-kernel G step must be bitwise the G launch).  Included INSIDE
// `namespace nngp { inline namespace <variant> {`; needs common.h, nngp_math.h and tableau.h.
#pragma once

// ---------------------------------------------------------------------------------------------
// ODE right-hand sides (systems.py), one lane = one state
// ---------------------------------------------------------------------------------------------
struct LaneArgs {
    double mn[4], hw[4], sc[4];  // '-11' wrapper: mn, (mx-mn)/2, 2/(mx-mn)   (utils.py:14-33)
    double param[4];
    double rparam0;              // RN(1/param[0]) for the Markstein division below
    int normalized;
    const double *norm;          // device [3D], loaded into the fields above by each lane
};

// x / b for a constant divisor b with r = RN(1/b) precomputed: q = x*r corrected by one fma
// (Markstein's theorem: r within 1/2 ulp of 1/b => RN(q + r*(x - q*b)) == RN(x/b)); bitwise the
// IEEE quotient (checked on 2e8 random operands), 3 dependent ops instead of the ~10-op
// v_div_scale/v_rcp/v_div_fmas/v_div_fixup sequence on the RK critical path.
__device__ __forceinline__ double div_const(double x, double b, double r) {
    const double q = x * r;
    return fma(fma(-q, b, x), r, q);
}

template <int SYS> struct LaneSys;

template <> struct LaneSys<NNGP_SYS_LORENZ> {   // systems.py:232-238
    static constexpr int D = 3;
    __device__ static void f(const double *u, double *o, const LaneArgs &) {
        o[0] = 10 * (u[1] - u[0]);
        o[1] = (28 * u[0] - u[1]) - u[0] * u[2];
        o[2] = u[0] * u[1] - (8.0 / 3) * u[2];
    }
};
template <> struct LaneSys<NNGP_SYS_HOPF> {     // systems.py:148-154
    static constexpr int D = 3;
    __device__ static void f(const double *u, double *o, const LaneArgs &a) {
        const double g = (div_const(u[2], a.param[0], a.rparam0) - u[0] * u[0]) - u[1] * u[1];
        o[0] = -u[1] + u[0] * g;
        o[1] = u[0] + u[1] * g;
        o[2] = 1.0;
    }
};
template <> struct LaneSys<NNGP_SYS_THOMAS_LABYRINTH> {   // systems.py:257-271
    static constexpr int D = 3;
    __device__ static void f(const double *u, double *o, const LaneArgs &) {
        o[0] = -0.5 * u[0] + 10.0 * nn_sin_pi(u[1]);
        o[1] = -0.5 * u[1] + 10.0 * nn_sin_pi(u[2]);
        o[2] = -0.5 * u[2] + 10.0 * nn_sin_pi(u[0]);
    }
};
template <> struct LaneSys<NNGP_SYS_FHN_ODE> {  // systems.py:87-95 (u**3 = u*(u*u), jax)
    static constexpr int D = 2;
    __device__ static void f(const double *u, double *o, const LaneArgs &) {
        const double c = 3;
        o[0] = c * ((u[0] - div_const(u[0] * (u[0] * u[0]), 3.0, 1.0 / 3)) + u[1]);
        o[1] = -(1 / c) * ((u[0] - 0.2) + 0.2 * u[1]);
    }
};
template <> struct LaneSys<NNGP_SYS_ROSSLER> {  // systems.py:116-125
    static constexpr int D = 3;
    __device__ static void f(const double *u, double *o, const LaneArgs &) {
        o[0] = -u[1] - u[2];
        o[1] = u[0] + (0.2 * u[1]);
        o[2] = 0.2 + u[2] * (u[0] - 5.7);
    }
};
template <> struct LaneSys<NNGP_SYS_BRUSSELATOR> {  // systems.py:209-214
    static constexpr int D = 2;
    __device__ static void f(const double *u, double *o, const LaneArgs &) {
        o[0] = (1 + (u[0] * u[0]) * u[1]) - (3 + 1) * u[0];
        o[1] = 3 * u[0] - (u[0] * u[0]) * u[1];
    }
};
template <> struct LaneSys<NNGP_SYS_DBL_PEND> {  // systems.py:182-189
    static constexpr int D = 4;
    __device__ static void f(const double *u, double *o, const LaneArgs &) {
        double s, c;
        nn_sincos(u[0] - u[2], s, c);
        const double s0 = nn_sin(u[0]), s2 = nn_sin(u[2]);
        const double pre = -1 / (2 - c * c);
        o[0] = u[1];
        o[1] = pre * ((((u[1] * u[1]) * c) * s + (u[3] * u[3]) * s) + 2 * s0 - c * s2);
        o[2] = u[3];
        o[3] = pre * ((((-2 * (u[1] * u[1])) * s - ((u[3] * u[3]) * s) * c) - (2 * c) * s0) + 2 * s2);
    }
};

// f_n(u) = f(inverse(u)) * scale   (systems.py:36-40), inverse(u) = ((u+1)/2)*(mx-mn) + mn
// (utils.py:24) evaluated as (u+1)*((mx-mn)/2) + mn: halving is exact for normal numbers, so
// RN(RN(u+1)/2 * w) == RN(RN(u+1) * (w/2)) bit for bit, one multiply fewer per component.  NORM is a template parameter so the RK
// step loop carries no branches: the lane kernel is VALU-issue-bound (one wave per SIMD, ~4.5
// cycles per fp64 instruction, dependent or not -- tools/ubench_fp64.hip), so every instruction
// and every taken scalar branch inside the step is paid in full on the critical path.
template <int SYS, bool NORM>
__device__ __forceinline__ void lane_rhs(const double *u, double *o, const LaneArgs &a) {
    constexpr int D = LaneSys<SYS>::D;
    if constexpr (NORM) {
        double v[D];
#pragma unroll
        for (int c = 0; c < D; c++) v[c] = (u[c] + 1) * a.hw[c] + a.mn[c];
        LaneSys<SYS>::f(v, o, a);
#pragma unroll
        for (int c = 0; c < D; c++) o[c] = o[c] * a.sc[c];
    } else {
        LaneSys<SYS>::f(u, o, a);
    }
}

// stage input  u + sum_{j<s} a_sj k_j  over the non-zero a_sj in ascending j (RK.py:153-166).
// The reference starts the sum from 0.0 (`temp = jnp.zeros(dim)`); starting from the first term
// instead is identical up to the sign of an exact zero and saves one dependent add per stage.
// k is indexed k[j*KS + c]; s is a compile-time constant after unrolling.
template <typename T, int KS>
__device__ __forceinline__ double stage_input(int s, double u, const double *k, int c) {
    double t = 0.0;
    bool first = true;
#pragma unroll
    for (int j = 0; j < T::S; j++) {
        if (j >= s || T::A[s][j] == 0.0) continue;
        const double v = T::A[s][j] * k[j * KS + c];
        t = first ? v : t + v;
        first = false;
    }
    return first ? u : u + t;
}

// stage_input split at j = s - 1, for kernels that form the terms not involving k_{s-1} early:
// stage_partial = the sum over the non-zero a_sj with j < s - 1 (0.0 if none), stage_finish adds
// a_{s,s-1} k_{s-1} and u -- the same additions in the same order as stage_input.
template <typename T>
__host__ __device__ constexpr bool stage_has_partial(int s) {
    for (int j = 0; j + 1 < s; j++)
        if (T::A[s][j] != 0.0) return true;
    return false;
}
template <typename T, int KS>
__device__ __forceinline__ double stage_partial(int s, const double *k, int c) {
    double t = 0.0;
    bool first = true;
#pragma unroll
    for (int j = 0; j < T::S; j++) {
        if (j + 1 >= s || T::A[s][j] == 0.0) continue;
        const double v = T::A[s][j] * k[j * KS + c];
        t = first ? v : t + v;
        first = false;
    }
    return t;
}
template <typename T, int KS>
__device__ __forceinline__ double stage_finish(int s, double u, double partial, const double *k, int c) {
    const bool hp = stage_has_partial<T>(s), hl = s >= 1 && T::A[s][s - 1] != 0.0;
    if (!hp && !hl) return u;
    double t = partial;
    if (hl) {
        const double v = T::A[s][s - 1] * k[(s - 1) * KS + c];
        t = hp ? t + v : v;
    }
    return u + t;
}
// step_update accumulated stage by stage: acc after stage s (the same order, non-zero b_s only;
// acc is unset until the first non-zero b_s, which every tableau has at s = 0 or 1)
template <typename T>
__device__ __forceinline__ void step_accumulate(int s, double &acc, double ks) {
    if (T::B[s] == 0.0) return;
    bool first = true;
#pragma unroll
    for (int j = 0; j < T::S; j++)
        if (j < s && T::B[j] != 0.0) first = false;
    const double v = T::B[s] * ks;
    acc = first ? v : acc + v;
}

// u + sum_s b_s k_s over the non-zero b_s in ascending s (jnp.sum(b*k, 1), RK.py:170)
template <typename T, int KS>
__device__ __forceinline__ double step_update(double u, const double *k, int c) {
    double acc = 0.0;
    bool first = true;
#pragma unroll
    for (int s = 0; s < T::S; s++) {
        if (T::B[s] == 0.0) continue;
        const double v = T::B[s] * k[s * KS + c];
        acc = first ? v : acc + v;
        first = false;
    }
    return u + acc;
}

// FIXED:    h = dt = (t1-t0)/steps (RK.py:103).
// LINSPACE: step n of slice i is step j = j0 + n of the grid np.linspace(t0, t1, gsteps+1):
//           t[j] = j*gstep + t0 (gstep = (t1-t0)/gsteps), t[gsteps] = t1, h = t[j+1]-t[j]
//           (RK.py:91-99, 121; new_lib.py:87-137).  j0 = 0, gsteps = steps is the per-slice grid;
//           j0 > 0 walks one global grid (the legacy initial coarse sweep, new_lib.py:902-906).
// The grid is walked with loop-carried state: jd = (double)j is bumped by an exact +1.0 (j < 2^53)
// and t[j+1] of one step is t[j] of the next, so a step costs one grid point (add, mul, add, the
// last-point select, sub) instead of two int64 -> double conversions and two grid points -- the
// same values bit for bit, off the lane/group kernels' issue-bound step (TomLab RK4 267 -> 256
// VALU per step).
struct LinGrid {
    double jd, tn;     // (double)j, t[j]
    int64_t nlast;     // the step n with j + 1 == gsteps (its right end is t1 itself)
    __device__ __forceinline__ void init(int64_t j0, int64_t gsteps, double t0, double dt) {
        jd = (double)j0;
        tn = jd * dt + t0;
        nlast = gsteps - 1 - j0;
    }
    __device__ __forceinline__ double next(int64_t n, double t0, double t1, double dt) {
        jd = jd + 1.0;
        const double tn1 = (n == nlast) ? t1 : jd * dt + t0;
        const double h = tn1 - tn;
        tn = tn1;
        return h;
    }
};

// ---------------------------------------------------------------------------------------------
// PDE fields
// ---------------------------------------------------------------------------------------------
struct FieldArgs {
    int d, nx, normalized;
    const double *norm;   // device [3d] = mn | w | sc, or nullptr
    double c_off, c_diag, c_grad;   // Burgers: nu/dx^2, -2 nu/dx^2, 1/(2dx)
    double a_off, a_diag, b_off, b_diag;   // FHN-PDE: a*L and b*L entries
};

__device__ __forceinline__ double wave_prev(double v) {   // lane i <- lane i-1 (lane 0 <- 63)
    return __builtin_amdgcn_mov_dpp(v, 0x13C, 0xF, 0xF, false);
}
__device__ __forceinline__ double wave_next(double v) {   // lane i <- lane i+1 (lane 63 <- 0)
    return __builtin_amdgcn_mov_dpp(v, 0x134, 0xF, 0xF, false);
}

// ---------------------------------------------------------------------------------------------
// Per-slice bodies.  The batched kernels (nngp_rk.hip) call them with their slice's row; the
// correction chain (nngp_gp.hip) calls them for its in-kernel G step, so both are the same code.
// ---------------------------------------------------------------------------------------------

// one lane integrates one ODE slice (rk_lane_kernel): u0/uF are the slice's [D] rows
template <int SYS, int ORDER, bool LINSPACE, bool NORM>
__device__ __forceinline__ void lane_slice(LaneArgs args, double T0, double T1, int64_t steps, int64_t gsteps,
                                           int64_t j0, const double *__restrict__ u0, double *__restrict__ uF) {
    using T = Tableau<ORDER>;
    constexpr int S = T::S;
    constexpr int D = LaneSys<SYS>::D;
    if constexpr (NORM) {
#pragma unroll
        for (int c = 0; c < D; c++) {
            args.mn[c] = args.norm[c];
            args.hw[c] = 0.5 * args.norm[D + c];
            args.sc[c] = args.norm[2 * D + c];
        }
    }
    double u[D], k[S * D], tmp[D];
#pragma unroll
    for (int c = 0; c < D; c++) u[c] = u0[c];
    const double dt = (T1 - T0) / (double)(LINSPACE ? gsteps : steps);
    LinGrid grid;
    if constexpr (LINSPACE) grid.init(j0, gsteps, T0, dt);
    for (int64_t n = 0; n < steps; n++) {
        const double h = LINSPACE ? grid.next(n, T0, T1, dt) : dt;
        // k_0 = h f(u); k_s = h f(u + sum_{j<s} a_sj k_j)     (RK.py:153-170)
#pragma unroll
        for (int s = 0; s < S; s++) {
#pragma unroll
            for (int c = 0; c < D; c++) tmp[c] = stage_input<T, D>(s, u[c], k, c);
            lane_rhs<SYS, NORM>(tmp, k + s * D, args);
#pragma unroll
            for (int c = 0; c < D; c++) k[s * D + c] = h * k[s * D + c];
        }
#pragma unroll
        for (int c = 0; c < D; c++) u[c] = step_update<T, D>(u[c], k, c);   // RK.py:170
    }
#pragma unroll
    for (int c = 0; c < D; c++) uF[c] = u[c];
}

// one wave integrates one Burgers slice, d = 64*EPT (rk_burgers_wave_kernel): lane l owns the
// contiguous elements l*EPT .. l*EPT+EPT-1; u0/uF are the slice's [d] rows.  Every lane of the
// wave must be active (the stencil's outer neighbours are wave_ror/wave_rol DPP moves).
template <int ORDER, bool LINSPACE, int EPT, bool NORM>
__device__ __forceinline__ void burgers_wave_slice(const FieldArgs &fa, int l, double T0, double T1, int64_t steps,
                                                   int64_t gsteps, int64_t j0, const double *__restrict__ u0,
                                                   double *__restrict__ uF) {
    using T = Tableau<ORDER>;
    constexpr int S = T::S;
    constexpr int d = 64 * EPT;
    double u[EPT], k[S * EPT], mn[EPT], w[EPT], sc[EPT];
#pragma unroll
    for (int r = 0; r < EPT; r++) {
        const int e = l * EPT + r;
        u[r] = u0[e];
        mn[r] = NORM ? fa.norm[e] : 0.0;
        w[r] = NORM ? 0.5 * fa.norm[d + e] : 1.0;   // (mx-mn)/2, see lane_rhs
        sc[r] = NORM ? fa.norm[2 * d + e] : 1.0;
    }
    const bool first = l == 0, last = l == 63;     // rows 0 and d-1 live in lanes 0 and 63
    const double cxx = fa.c_off, cdg = fa.c_diag, q = fa.c_grad;
    const double dt = (T1 - T0) / (double)(LINSPACE ? gsteps : steps);
    LinGrid grid;
    if constexpr (LINSPACE) grid.init(j0, gsteps, T0, dt);
    for (int64_t n = 0; n < steps; n++) {
        const double h = LINSPACE ? grid.next(n, T0, T1, dt) : dt;
#pragma unroll
        for (int s = 0; s < S; s++) {
            double V[EPT];
#pragma unroll
            for (int r = 0; r < EPT; r++) {
                const double x = stage_input<T, EPT>(s, u[r], k, r);
                V[r] = NORM ? (x + 1) * w[r] + mn[r] : x;
            }
            const double Vl = wave_prev(V[EPT - 1]);   // element l*EPT - 1
            const double Vr = wave_next(V[0]);         // element l*EPT + EPT
#pragma unroll
            for (int r = 0; r < EPT; r++) {
                const double L = r > 0 ? V[r - 1] : Vl;
                const double C = V[r];
                const double R = r < EPT - 1 ? V[r + 1] : Vr;
                const double pL = cxx * L, pC = cdg * C, pR = cxx * R;
                // row 0: (cdg C + cxx R) + cxx L; row d-1: (cxx R + cxx L) + cdg C; else
                // (cxx L + cdg C) + cxx R
                const bool b0 = (r == 0) && first, b1 = (r == EPT - 1) && last;
                const double a1 = b0 ? pC : (b1 ? pR : pL);
                const double a2 = b0 ? pR : (b1 ? pL : pC);
                const double a3 = b0 ? pL : (b1 ? pC : pR);
                const double lap = (a1 + a2) + a3;
                const double grad = (-q) * L + q * R;
                double f = lap - C * grad;
                if (NORM) f = f * sc[r];
                k[s * EPT + r] = h * f;
            }
        }
#pragma unroll
        for (int r = 0; r < EPT; r++) u[r] = step_update<T, EPT>(u[r], k, r);   // RK.py:170
    }
#pragma unroll
    for (int r = 0; r < EPT; r++) uF[l * EPT + r] = u[r];
}
