// nngp_rk.hip -- batched fine/coarse Runge-Kutta propagator for gfx950 (MI355X).
//
// Replaces the reference's per-slice fine solve SolverRK.run_F -> RK.run_get_last ->
// _RK_jax_last (solver.py:86-107, RK.py:101-109, 146-174), fanned over the unconverged slices by
// pool.map at parareal.py:310-315 (legacy: RK_last / RK_jax_, new_lib.py:57-137, 939-945).
//
// One launch integrates ALL slices of one Parareal iteration.  Two kernel shapes:
//   * lane kernel  (ODEs, d <= 4): one lane = one slice, state + all S stage vectors in VGPRs,
//     no LDS, no barriers.  The RHS is a handful of dependent fp64 ops, so a slice is a serial
//     chain of 10^3..10^9 RK steps: this shape is latency-bound by construction.
//   * field kernel (Burgers d=nx, FHN-PDE d=2 nx^2): one workgroup = one slice, thread t owns
//     elements t, t+BT, ... (EPT per thread, u and the S stage vectors in VGPRs).  The stage input
//     is staged (already inverse-normalised) in a double-buffered LDS image so the stencil reads
//     neighbours from LDS; exactly one __syncthreads per stage.
// HBM traffic is 16*d bytes per slice per launch (read u0, write uF); everything else stays on
// chip, so the roofline is FP64 VALU, not HBM.
//
// Numerics: compiled with -ffp-contract=off; every add/mul is rounded in the order of the
// reference expression it restates (cited inline).  Zero tableau entries are skipped at compile
// time, which is exact for finite stages (t + 0*k == t).
//
// This file is compiled TWICE (csrc/Makefile): the exact build above, and -- with NNGP_RK_FMA
// defined and -ffp-contract=fast -- the opt-in contracted propagator (NNGP_STEP_CONTRACT,
// include/nngp.h): the same kernels with every a*b+c fused, in the inline namespace `contracted`
// so the two code objects' kernels never share a symbol.  Only the exact build exports the C-ABI;
// the contracted one exports nngp_rk_dispatch_contracted, which nngp_rk_batch calls.

#include <algorithm>
#include <type_traits>

#include "common.h"
#include "nngp_math.h"
#include "tableau.h"

#ifdef NNGP_RK_FMA
#define NNGP_RK_VARIANT contracted
#else
#define NNGP_RK_VARIANT exact
#endif

namespace nngp {
inline namespace NNGP_RK_VARIANT {

#include "nngp_rk_dev.h"


template <int SYS, int ORDER, bool LINSPACE, bool NORM>
__global__ void __launch_bounds__(64) rk_lane_kernel(LaneArgs args, int n_slices,
                                                     const double *__restrict__ t0,
                                                     const double *__restrict__ t1, int64_t steps,
                                                     int64_t gsteps, const int64_t *__restrict__ j0s,
                                                     const double *__restrict__ u0,
                                                     double *__restrict__ uF) {
    constexpr int D = LaneSys<SYS>::D;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_slices) return;
    lane_slice<SYS, ORDER, LINSPACE, NORM>(args, t0[i], t1[i], steps, gsteps, j0s ? j0s[i] : 0, u0 + (size_t)i * D,
                                           uF + (size_t)i * D);
}

// ---------------------------------------------------------------------------------------------
// Lane-group kernel: one slice = one group of G lanes, each component on its own lanes: G = 16
// (components in DPP banks, below) for every ODE but Thomas labyrinth, G = 4 (lane c = component c,
// lane 3 padding) for Thomas labyrinth's rotation.
// The lane kernel above runs every component's stage sums, (de)normalisation, h*k and final update
// in one lane; here each of those is one instruction per step-part for all components at once, and
// only the RHS coupling crosses lanes: `v_mov_b64_dpp row_newbcast` (gfx950's 64-bit DPP, one VALU
// op) for G = 16, or a quad_perm rotation (two 32-bit DPP ops) for G = 4.
// At few slices the step is one wave's instruction issue (a wave with 1 active
// lane costs the same as 64), so fewer instructions per step is the whole gain, measured on the
// box (tools/lane_group_probe.py): Hopf RK4 119 -> 97 VALU, 0.250 -> 0.201
// us/step; Lorenz 0.29 -> 0.19; Thomas labyrinth one sin per lane instead of three, 1.45 -> 0.47;
// double pendulum one sincos per bank instead of three, 1.82 -> 0.91.
// Bitwise the lane kernel: each component is rounded by the same expression in the same order.
// ---------------------------------------------------------------------------------------------
template <int CTRL>
__device__ __forceinline__ double quad_mov(double v) {
    return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, false);
}
constexpr int QROT = 0xC9;   // quad_perm [1,2,0,3]: lane c reads lane c+1 mod 3

// G = 16: component c lives in DPP bank c (lanes 4c..4c+3 of the row hold the same value; lane 4c
// writes it), so every cross-lane step is one 64-bit `v_mov_b64_dpp row_newbcast` -- the only DPP
// control gfx950 allows on 64-bit operands:
//   bcast<c>(v)            component c's value in every lane;
//   take<L, BANKS>(o, v)   lanes of the banks in BANKS take lane L's v, the others keep o -- a
//                          per-component select in one op (bank_mask), where a 64-bit v_cndmask
//                          is two.
template <int C>
__device__ __forceinline__ double bcast(double v) {
    return __builtin_amdgcn_mov_dpp(v, 0x150 + 4 * C, 0xF, 0xF, false);
}
template <int L, int BANKS>
__device__ __forceinline__ double take(double old, double v) {
    return __builtin_amdgcn_update_dpp(old, v, 0x150 + L, 0xF, BANKS, false);
}

// f(x = own de-normalised component, c = its index, one = 1.0) -> own component of f.  G16 (bank
// layout above) for the broadcast-coupled fields, G4 (lane c = component c) for Thomas
// labyrinth's rotation (quad_perm, two 32-bit DPP ops).
template <int SYS> struct GroupSys;

template <> struct GroupSys<NNGP_SYS_LORENZ> {   // systems.py:232-238, as LaneSys<LORENZ>
    static constexpr int G = 16;
    __device__ static double f(double x, int, double, const LaneArgs &) {
        const double A = bcast<0>(x), B = bcast<1>(x), C = bcast<2>(x);
        const double o0 = 10 * (B - A);
        const double o1 = (28 * A - B) - A * C;
        const double o2 = A * B - (8.0 / 3) * C;
        return take<8, 0x4>(take<4, 0x2>(o0, o1), o2);
    }
};
template <> struct GroupSys<NNGP_SYS_HOPF> {     // systems.py:148-154, as LaneSys<HOPF>
    static constexpr int G = 16;
    // g = (u2/mu - u0*u0) - u1*u1; component 0: -u1 + u0*g, component 1: u0 + u1*g, component 2: 1.
    // Fewer ops than broadcasting u0, u1, u2 and squaring the broadcasts: every lane squares its
    // own component (sq = x*x, the same rounded products), and bank-masked `take`s into registers
    // carried from stage to stage move only what banks 0 and 1 need -- u2 (for u2/mu), u0^2, u1^2
    // and the coupling term P (bank 0: u1, bank 1: u0) -- while bank 2's lanes keep what `init`
    // put there: 0 in C, A2, B2, so g = +-0 and x*g = +-0 (u2 is always finite), and 1.0 in P.
    // The sum p + x*g is one fma(S, P, x*g) with S = -1 in bank 0 and +1 elsewhere: S*P is exact,
    // so the fma is the correctly rounded x*g -+ P, bitwise the reference's addition (signed zeros
    // included: the fma's exact-sum rule is the addition's); bank 2: +-0 + 1 = 1.
    // 13 VALU per RHS instead of 16.  (The contracted build keeps the broadcast form, whose
    // p + x*g contracts to one fma there.)
#ifdef NNGP_RK_FMA
    __device__ static double f(double x, int c, double one, const LaneArgs &a) {
        const double A = bcast<0>(x), B = bcast<1>(x), C = bcast<2>(x);
        const double g = (div_const(C, a.param[0], a.rparam0) - A * A) - B * B;
        const double p = c == 0 ? -B : A;
        return take<8, 0x4>(p + x * g, one);
    }
#else
    struct St {
        double C, A2, B2, P, S;
    };
    __device__ static St init(int c) { return St{0.0, 0.0, 0.0, c == 2 ? 1.0 : 0.0, c == 0 ? -1.0 : 1.0}; }
    __device__ static double f(double x, St &s, double, const LaneArgs &a) {
        const double sq = x * x;
        s.C = take<8, 0x3>(s.C, x);
        s.A2 = take<0, 0x3>(s.A2, sq);
        s.B2 = take<4, 0x3>(s.B2, sq);
        s.P = take<0, 0x2>(take<4, 0x1>(s.P, x), x);
        const double g = (div_const(s.C, a.param[0], a.rparam0) - s.A2) - s.B2;
        return __builtin_fma(s.S, s.P, x * g);
    }
#endif
};
template <> struct GroupSys<NNGP_SYS_THOMAS_LABYRINTH> {   // systems.py:257-271
    static constexpr int G = 4;
    __device__ static double f(double x, int, double, const LaneArgs &) {
        const double sn = quad_mov<QROT>(nn_sin_pi(x));   // sin(u[c+1 mod 3])
        return -0.5 * x + 10.0 * sn;
    }
};
template <> struct GroupSys<NNGP_SYS_ROSSLER> {  // systems.py:116-125
    static constexpr int G = 16;
    __device__ static double f(double x, int, double, const LaneArgs &) {
        const double A = bcast<0>(x), B = bcast<1>(x), C = bcast<2>(x);
        return take<8, 0x4>(take<4, 0x2>(-B - C, A + (0.2 * B)), 0.2 + C * (A - 5.7));
    }
};

template <> struct GroupSys<NNGP_SYS_FHN_ODE> {  // systems.py:87-95, as LaneSys<FHN_ODE>
    static constexpr int G = 16;
    __device__ static double f(double x, int, double, const LaneArgs &) {
        const double A = bcast<0>(x), B = bcast<1>(x);
        const double c = 3;
        const double o0 = c * ((A - div_const(A * (A * A), 3.0, 1.0 / 3)) + B);
        const double o1 = -(1 / c) * ((A - 0.2) + 0.2 * B);
        return take<4, 0x2>(o0, o1);
    }
};
template <> struct GroupSys<NNGP_SYS_BRUSSELATOR> {  // systems.py:209-214, as LaneSys<BRUSSELATOR>
    static constexpr int G = 16;
    __device__ static double f(double x, int, double, const LaneArgs &) {
        const double A = bcast<0>(x), B = bcast<1>(x);
        const double o0 = (1 + (A * A) * B) - (3 + 1) * A;
        const double o1 = 3 * A - (A * A) * B;
        return take<4, 0x2>(o0, o1);
    }
};
template <> struct GroupSys<NNGP_SYS_DBL_PEND> {  // systems.py:182-189, as LaneSys<DBL_PEND>
    static constexpr int G = 16;
    __device__ static double f(double x, int, double, const LaneArgs &) {
        const double A = bcast<0>(x), B = bcast<1>(x), C = bcast<2>(x), D = bcast<3>(x);
        // the lane kernel's three sincos (of u0-u2, u0, u2) as one per bank: bank 0 takes u0-u2,
        // bank 1 u0 (lane 0's x), bank 2 u2 (lane 8's x)
        const double arg = take<8, 0x4>(take<0, 0x2>(A - C, x), x);
        double sn, cs;
        nn_sincos(arg, sn, cs);
        const double s = bcast<0>(sn), c = bcast<0>(cs), s0 = bcast<1>(sn), s2 = bcast<2>(sn);
        const double pre = -1 / (2 - c * c);
        const double o1 = pre * ((((B * B) * c) * s + (D * D) * s) + 2 * s0 - c * s2);
        const double o3 = pre * ((((-2 * (B * B)) * s - ((D * D) * s) * c) - (2 * c) * s0) + 2 * s2);
        // component 0: u1, 1: o1, 2: u3 (lane 12's x), 3: o3
        return take<12, 0x8>(take<12, 0x4>(take<4, 0x2>(B, o1), x), o3);
    }
};

// Per-lane state a group RHS carries from stage to stage (GroupSys<SYS>::St, made by its init(c));
// a field without one gets its component index.
template <class GS, class = void> struct GroupState {
    using T = int;
    __device__ static int init(int c) { return c; }
};
template <class GS> struct GroupState<GS, std::void_t<typename GS::St>> {
    using T = typename GS::St;
    __device__ static T init(int c) { return GS::init(c); }
};

template <int SYS> struct has_group { static constexpr bool value = false; };
template <> struct has_group<NNGP_SYS_LORENZ> { static constexpr bool value = true; };
template <> struct has_group<NNGP_SYS_HOPF> { static constexpr bool value = true; };
template <> struct has_group<NNGP_SYS_THOMAS_LABYRINTH> { static constexpr bool value = true; };
template <> struct has_group<NNGP_SYS_ROSSLER> { static constexpr bool value = true; };
template <> struct has_group<NNGP_SYS_FHN_ODE> { static constexpr bool value = true; };
template <> struct has_group<NNGP_SYS_BRUSSELATOR> { static constexpr bool value = true; };
template <> struct has_group<NNGP_SYS_DBL_PEND> { static constexpr bool value = true; };

template <int SYS, int ORDER, bool LINSPACE, bool NORM>
__global__ void __launch_bounds__(64) rk_group_kernel(LaneArgs args, int n_slices,
                                                     const double *__restrict__ t0,
                                                     const double *__restrict__ t1, int64_t steps,
                                                     int64_t gsteps, const int64_t *__restrict__ j0s,
                                                     const double *__restrict__ u0,
                                                     double *__restrict__ uF) {
    using T = Tableau<ORDER>;
    constexpr int S = T::S;
    constexpr int D = LaneSys<SYS>::D;
    static_assert(D <= (GroupSys<SYS>::G == 16 ? 4 : 3), "group kernel: one DPP bank (G=16) or lane (G=4) per component");
    constexpr int G = GroupSys<SYS>::G;
    const int tid = blockIdx.x * blockDim.x + threadIdx.x;
    const int i = tid / G, c = (G == 16) ? (tid % 16) >> 2 : tid % G;   // component of this lane
    if (i >= n_slices) return;   // group-uniform: the DPP partners of a live lane are live
    const bool own = c < D;
    const bool writer = own && (G != 16 || (tid & 3) == 0);
    const double one = 1.0;
    typename GroupState<GroupSys<SYS>>::T gst = GroupState<GroupSys<SYS>>::init(c);
    double mn = 0, hw = 0, sc = 0;
    if constexpr (NORM) {
        if (own) {
            mn = args.norm[c];
            hw = 0.5 * args.norm[D + c];
            sc = args.norm[2 * D + c];
        }
    }
    double u = own ? u0[(size_t)i * D + c] : 0.0, k[S];
    const double T0 = t0[i], T1 = t1[i];
    const double dt = (T1 - T0) / (double)(LINSPACE ? gsteps : steps);
    const int64_t j0 = j0s ? j0s[i] : 0;
    LinGrid grid;
    if constexpr (LINSPACE) grid.init(j0, gsteps, T0, dt);
    for (int64_t n = 0; n < steps; n++) {
        const double h = LINSPACE ? grid.next(n, T0, T1, dt) : dt;
#pragma unroll
        for (int s = 0; s < S; s++) {
            const double tmp = stage_input<T, 1>(s, u, k, 0);
            double o;
            if constexpr (NORM) o = GroupSys<SYS>::f((tmp + 1) * hw + mn, gst, one, args) * sc;
            else o = GroupSys<SYS>::f(tmp, gst, one, args);
            k[s] = h * o;
        }
        u = step_update<T, 1>(u, k, 0);
    }
    if (writer) uF[(size_t)i * D + c] = u;
}

// ---------------------------------------------------------------------------------------------
// PDE right-hand sides (Burgers, FHN-PDE), one workgroup = one slice
// ---------------------------------------------------------------------------------------------

// Burgers row i: (Dxx@u)_i - u_i (Dx@u)_i with non-zeros summed in ascending column order
// (systems.py:421-446)
__device__ __forceinline__ double burgers_elem(const double *__restrict__ V, int i, int d,
                                               const FieldArgs &fa) {
    const double cxx = fa.c_off, cdg = fa.c_diag, q = fa.c_grad;
    double lap, grad;
    if (i == 0) {
        lap = (cdg * V[0] + cxx * V[1]) + cxx * V[d - 1];
        grad = q * V[1] + (-q) * V[d - 1];
    } else if (i == d - 1) {
        lap = (cxx * V[0] + cxx * V[d - 2]) + cdg * V[d - 1];
        grad = q * V[0] + (-q) * V[d - 2];
    } else {
        lap = (cxx * V[i - 1] + cdg * V[i]) + cxx * V[i + 1];
        grad = (-q) * V[i - 1] + q * V[i + 1];
    }
    return lap - V[i] * grad;
}

// 5-point periodic neighbourhood of grid point p = y*nx + x with its columns in ascending order
// and a flag for the diagonal slot; precomputed once per element (a 9-comparator sorting
// network on named registers -- no runtime-indexed arrays, so nothing spills to scratch).
struct Nbr5 {
    int c0, c1, c2, c3, c4;
    bool d0, d1, d2, d3, d4;
};

__device__ __forceinline__ void cswap(int &a, bool &fa, int &b, bool &fb) {
    if (a > b) {
        const int t = a; a = b; b = t;
        const bool u = fa; fa = fb; fb = u;
    }
}

__device__ inline Nbr5 fhn_neighbours(int nx, int p) {
    const int y = p / nx, x = p - y * nx;
    const int ym = (y == 0) ? nx - 1 : y - 1, yp = (y == nx - 1) ? 0 : y + 1;
    const int xm = (x == 0) ? nx - 1 : x - 1, xp = (x == nx - 1) ? 0 : x + 1;
    Nbr5 r{ym * nx + x, y * nx + xm, p, y * nx + xp, yp * nx + x, false, false, true, false, false};
    // optimal 5-input sorting network
    cswap(r.c0, r.d0, r.c1, r.d1); cswap(r.c3, r.d3, r.c4, r.d4);
    cswap(r.c2, r.d2, r.c4, r.d4); cswap(r.c2, r.d2, r.c3, r.d3);
    cswap(r.c0, r.d0, r.c3, r.d3); cswap(r.c0, r.d0, r.c2, r.d2);
    cswap(r.c1, r.d1, r.c4, r.d4); cswap(r.c1, r.d1, r.c3, r.d3);
    cswap(r.c1, r.d1, r.c2, r.d2);
    return r;
}

// ((a L)@v)_p with the 5 terms in ascending column order (systems.py:365-366: `a*(DXX+DYY)@u1`
// multiplies the matrix by a first)
__device__ __forceinline__ double fhn_lap(const double *__restrict__ V, const Nbr5 &nb, double off,
                                          double diag) {
    double s = (nb.d0 ? diag : off) * V[nb.c0];
    s = s + (nb.d1 ? diag : off) * V[nb.c1];
    s = s + (nb.d2 ? diag : off) * V[nb.c2];
    s = s + (nb.d3 ? diag : off) * V[nb.c3];
    s = s + (nb.d4 ? diag : off) * V[nb.c4];
    return s;
}

// <= 256 threads per slice leaves ~170 VGPRs for u, the S stage vectors and the neighbour table
template <int SYS, int ORDER, bool LINSPACE, int EPT, bool NORM>
__global__ void __launch_bounds__(EPT == 1 ? 1024 : (EPT == 2 ? 512 : 256)) rk_field_kernel(FieldArgs fa, int n_slices,
                                                        const double *__restrict__ t0,
                                                        const double *__restrict__ t1,
                                                        int64_t steps, int64_t gsteps,
                                                        const int64_t *__restrict__ j0s,
                                                        const double *__restrict__ u0,
                                                        double *__restrict__ uF) {
    using T = Tableau<ORDER>;
    constexpr int S = T::S;
    extern __shared__ __attribute__((aligned(16))) double smem[];   // [2][d]
    const int slice = blockIdx.x;
    const int tid = threadIdx.x, BT = blockDim.x;
    const int d = fa.d;
    const int half = d / 2;   // FHN-PDE: u1 | u2

    double u[EPT], k[S * EPT], mn[EPT], w[EPT], sc[EPT];
    int e_[EPT];
    Nbr5 nb[(SYS == NNGP_SYS_FHN_PDE) ? EPT : 1];
#pragma unroll
    for (int r = 0; r < EPT; r++) {
        const int e = tid + r * BT;
        e_[r] = e;
        const bool ok = e < d;
        u[r] = ok ? u0[(size_t)slice * d + e] : 0.0;
        if (NORM && ok) {
            mn[r] = fa.norm[e];
            w[r] = 0.5 * fa.norm[d + e];   // (mx-mn)/2, see lane_rhs
            sc[r] = fa.norm[2 * d + e];
        } else {
            mn[r] = 0.0; w[r] = 1.0; sc[r] = 1.0;
        }
        if constexpr (SYS == NNGP_SYS_FHN_PDE) nb[r] = fhn_neighbours(fa.nx, ok ? (e % half) : 0);
    }
    const double T0 = t0[slice], T1 = t1[slice];
    const double dt = (T1 - T0) / (double)(LINSPACE ? gsteps : steps);
    const int64_t j0 = j0s ? j0s[slice] : 0;
    int buf = 0;
    LinGrid grid;
    if constexpr (LINSPACE) grid.init(j0, gsteps, T0, dt);
    for (int64_t n = 0; n < steps; n++) {
        const double h = LINSPACE ? grid.next(n, T0, T1, dt) : dt;
#pragma unroll
        for (int s = 0; s < S; s++) {
            double *V = smem + buf * d;
#pragma unroll
            for (int r = 0; r < EPT; r++) {
                if (e_[r] < d) {
                    const double x = stage_input<T, EPT>(s, u[r], k, r);
                    V[e_[r]] = NORM ? (x + 1) * w[r] + mn[r] : x;
                }
            }
            __syncthreads();
#pragma unroll
            for (int r = 0; r < EPT; r++) {
                const int e = e_[r];
                double f = 0.0;
                if (e < d) {
                    if constexpr (SYS == NNGP_SYS_BURGERS) {
                        f = burgers_elem(V, e, d, fa);
                    } else {   // FHN_PDE, systems.py:365-366
                        if (e < half) {
                            const double lu = fhn_lap(V, nb[r], fa.a_off, fa.a_diag);
                            const double u1 = V[e], u1c = u1 * (u1 * u1);
                            f = (((lu + u1) - u1c) - V[half + e]) + -5E-3 * 1.0;
                        } else {
                            const double lv = fhn_lap(V + half, nb[r], fa.b_off, fa.b_diag);
                            f = (1 / 0.1) * ((lv + V[e - half]) - V[e]);
                        }
                    }
                    if (NORM) f = f * sc[r];
                }
                k[s * EPT + r] = h * f;
            }
            buf ^= 1;
        }
#pragma unroll
        for (int r = 0; r < EPT; r++) u[r] = step_update<T, EPT>(u[r], k, r);   // RK.py:170
    }
#pragma unroll
    for (int r = 0; r < EPT; r++)
        if (e_[r] < d) uF[(size_t)slice * d + e_[r]] = u[r];
}

// ---------------------------------------------------------------------------------------------
// FHN-PDE with one thread per grid point: thread p owns u[p] and v[p] (elements p and half + p)
// with all their stage values.  The reaction terms couple u and v at the SAME point and the
// Laplacian's centre is the point itself, so a stage reads from LDS only the two 5-point
// Laplacians (the own and partner values come from registers): 1 write + 10 reads per point
// instead of the element-per-thread kernel's 2 writes + 14 reads.  Same expressions, same order
// (systems.py:365-366) -- bitwise rk_field_kernel<FHN_PDE>.  d = 2 nx^2 <= 2048.
//
// LDS layout: FhnPairImages::N images of [point][u, v] (below), and a stage's image fixed at
// compile time (stage s of every step uses image s & 1, the last of an odd stage count image 2, so
// the image a stage writes was last read two barriers earlier).  Every LDS access of the step loop
// is then one of five per-thread neighbour addresses plus an immediate offset: no address
// arithmetic per stage.  Threads past the grid (the last wave's idle lanes) compute point 0's
// stencil on their own zeros and write their garbage to the images' padding, so the step loop has
// no branch either.
// ---------------------------------------------------------------------------------------------
template <int S> struct FhnPairImages {
    static constexpr int N = (S % 2 == 1 && S > 1) ? 3 : 2;
    // image of stage s (S == 1 alternates at run time)
    static constexpr int of(int s) { return (S % 2 == 1 && s == S - 1) ? 2 : (s & 1); }
};

// ((a L)@v)_p as fhn_lap, from the five neighbour values (ascending column order) and the five
// coefficients selected once per thread
__device__ __forceinline__ double fhn_sum5(const double (&v)[5], double k0, double k1, double k2, double k3,
                                           double k4) {
    double s = k0 * v[0];
    s = s + k1 * v[1];
    s = s + k2 * v[2];
    s = s + k3 * v[3];
    s = s + k4 * v[4];
    return s;
}

// Images interleaved [point][u, v], 16 bytes per point: a neighbour's u and v arrive by ONE
// ds_read_b128 (4 LDS-array cycles per wave-instruction, 256 B/clk) and a point's two stage inputs
// leave by one ds_write_b128.  Round 3's split [u | v] images needed a ds_read2st64_b64 (8 cycles,
// 128 B/clk) per neighbour; PMC at 512 slices (profiles/r04/pmc_fhn_pair_r4c.txt) had the CU's LDS
// ~70 % busy under it (66 LDS instructions per wave per RK8 step, 20 % of their cycles bank
// conflicts) beside a 64 % busy VALU.  Measured (profiles/r04/fhn_pair_il_r4d.txt), us per RK8
// step at d = 800: 512 slices 5.54 -> 4.91, 64 slices 3.53 -> 2.98; bitwise unchanged.  The image
// stride is the block size (points past the grid write their own padding slots).
template <int ORDER, bool LINSPACE, bool NORM>
__global__ void __launch_bounds__(1024) rk_fhn_pair_kernel(FieldArgs fa, int n_slices,
                                                           const double *__restrict__ t0,
                                                           const double *__restrict__ t1, int64_t steps,
                                                           int64_t gsteps, const int64_t *__restrict__ j0s,
                                                           const double *__restrict__ u0,
                                                           double *__restrict__ uF) {
    using T = Tableau<ORDER>;
    using IM = FhnPairImages<T::S>;
    constexpr int S = T::S;
    extern __shared__ __attribute__((aligned(16))) double smem[];   // [IM::N][blockDim.x][2]
    const int slice = blockIdx.x;
    const int p = threadIdx.x;
    const int d = fa.d, half = d / 2;
    const bool ok = p < half;
    double u[2], k[S * 2], mn[2], w[2], sc[2];
#pragma unroll
    for (int r = 0; r < 2; r++) {
        const int e = p + r * half;
        u[r] = ok ? u0[(size_t)slice * d + e] : 0.0;
        if (NORM && ok) {
            mn[r] = fa.norm[e];
            w[r] = 0.5 * fa.norm[d + e];   // (mx-mn)/2, see lane_rhs
            sc[r] = fa.norm[2 * d + e];
        } else {
            mn[r] = 0.0; w[r] = 1.0; sc[r] = 1.0;
        }
    }
    const Nbr5 nb = fhn_neighbours(fa.nx, ok ? p : 0);   // the same stencil for u and v
    const double ka0 = nb.d0 ? fa.a_diag : fa.a_off, ka1 = nb.d1 ? fa.a_diag : fa.a_off,
                 ka2 = nb.d2 ? fa.a_diag : fa.a_off, ka3 = nb.d3 ? fa.a_diag : fa.a_off,
                 ka4 = nb.d4 ? fa.a_diag : fa.a_off;
    const double kb0 = nb.d0 ? fa.b_diag : fa.b_off, kb1 = nb.d1 ? fa.b_diag : fa.b_off,
                 kb2 = nb.d2 ? fa.b_diag : fa.b_off, kb3 = nb.d3 ? fa.b_diag : fa.b_off,
                 kb4 = nb.d4 ? fa.b_diag : fa.b_off;
    const double T0 = t0[slice], T1 = t1[slice];
    const double dt = (T1 - T0) / (double)(LINSPACE ? gsteps : steps);
    const int64_t j0 = j0s ? j0s[slice] : 0;
    LinGrid grid;
    if constexpr (LINSPACE) grid.init(j0, gsteps, T0, dt);
    // stage 0's input is u itself (RK.py:153-166: no a_0j terms)
    double xw[2];
#pragma unroll
    for (int r = 0; r < 2; r++) xw[r] = NORM ? (u[r] + 1) * w[r] + mn[r] : u[r];
    const int ISTR = 2 * (int)blockDim.x;   // doubles per image
    for (int64_t n = 0; n < steps; n++) {
        const double h = LINSPACE ? grid.next(n, T0, T1, dt) : dt;
        double acc[2];   // sum_s b_s k_s, accumulated as the stages finish (step_update's order)
#pragma unroll
        for (int s = 0; s < S; s++) {
            const int img = (S == 1) ? (int)(n & 1) : IM::of(s);
            double va[5], vb[5];
            double2 *V2 = reinterpret_cast<double2 *>(smem + img * ISTR);
            V2[p] = make_double2(xw[0], xw[1]);
            __syncthreads();
            const double2 w0 = V2[nb.c0], w1 = V2[nb.c1], w2 = V2[nb.c2], w3 = V2[nb.c3], w4 = V2[nb.c4];
            va[0] = w0.x; va[1] = w1.x; va[2] = w2.x; va[3] = w3.x; va[4] = w4.x;
            vb[0] = w0.y; vb[1] = w1.y; vb[2] = w2.y; vb[3] = w3.y; vb[4] = w4.y;
            // the next stage's input terms that do not involve this stage's k, computed while the
            // neighbour reads are in flight (pinned before the stencil: the reads' results pass
            // through the same empty asm, so LLVM can neither sink these sums past the stencil
            // nor start the stencil before them; profiles/r03: 47 % of a 64-slice step's wave
            // cycles were spent waiting, mostly on these reads and the barrier)
            double pn[2] = {0.0, 0.0};
            if (s + 1 < S) {
#pragma unroll
                for (int r = 0; r < 2; r++) pn[r] = stage_partial<T, 2>(s + 1, k, r);
            }
            // systems.py:365-366, as rk_field_kernel with V[e] / V[half+e] / V[e-half] in registers
            const double lu = fhn_sum5(va, ka0, ka1, ka2, ka3, ka4);
            const double u1 = xw[0], u1c = u1 * (u1 * u1);
            double fu = (((lu + u1) - u1c) - xw[1]) + -5E-3 * 1.0;
            const double lv = fhn_sum5(vb, kb0, kb1, kb2, kb3, kb4);
            double fv = (1 / 0.1) * ((lv + xw[0]) - xw[1]);
            if (NORM) {
                fu = fu * sc[0];
                fv = fv * sc[1];
            }
            k[s * 2 + 0] = h * fu;
            k[s * 2 + 1] = h * fv;
#pragma unroll
            for (int r = 0; r < 2; r++) {
                step_accumulate<T>(s, acc[r], k[s * 2 + r]);   // RK.py:170, in its order
                if (s + 1 < S) {
                    const double x = stage_finish<T, 2>(s + 1, u[r], pn[r], k, r);
                    xw[r] = NORM ? (x + 1) * w[r] + mn[r] : x;
                }
            }
        }
#pragma unroll
        for (int r = 0; r < 2; r++) {
            u[r] = u[r] + acc[r];   // RK.py:170
            xw[r] = NORM ? (u[r] + 1) * w[r] + mn[r] : u[r];
        }
    }
    if (ok) {
        uF[(size_t)slice * d + p] = u[0];
        uF[(size_t)slice * d + half + p] = u[1];
    }
}

// ---------------------------------------------------------------------------------------------
// Burgers with d = 64*EPT: ONE WAVE per slice, no LDS, no barriers.
// Lane l owns the contiguous elements l*EPT .. l*EPT+EPT-1; the periodic stencil's outer
// neighbours come from lanes l-1 / l+1 by `wave_ror:1` / `wave_rol:1` DPP moves, which wrap around
// the wave exactly like the periodic boundary wraps around the grid.  The general kernel above
// pays an LDS round trip and a workgroup barrier per stage instead (11 per RK8 step).
// Summation order = burgers_elem (systems.py:421-446, non-zeros in ascending column order): the
// three Laplacian terms of rows 0 and d-1 associate differently from the interior rows, so the
// operands are selected per element; the two gradient terms commute (a+b == b+a bitwise).
// ---------------------------------------------------------------------------------------------

template <int ORDER, bool LINSPACE, int EPT, bool NORM>
__global__ void __launch_bounds__(64) rk_burgers_wave_kernel(FieldArgs fa, int n_slices,
                                                              const double *__restrict__ t0,
                                                              const double *__restrict__ t1,
                                                              int64_t steps, int64_t gsteps,
                                                              const int64_t *__restrict__ j0s,
                                                              const double *__restrict__ u0,
                                                              double *__restrict__ uF) {
    constexpr int d = 64 * EPT;
    const int slice = blockIdx.x;
    burgers_wave_slice<ORDER, LINSPACE, EPT, NORM>(fa, threadIdx.x, t0[slice], t1[slice], steps, gsteps,
                                                   j0s ? j0s[slice] : 0, u0 + (size_t)slice * d,
                                                   uF + (size_t)slice * d);
}

// ---------------------------------------------------------------------------------------------
// single RHS evaluations (ODE.get_vector_field()(t, u)) and the elementwise Parareal update
// ---------------------------------------------------------------------------------------------
template <int SYS>
__global__ void __launch_bounds__(64) rhs_lane_kernel(LaneArgs args, int n, const double *__restrict__ u,
                                                      double *__restrict__ out) {
    constexpr int D = LaneSys<SYS>::D;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (args.normalized)
        for (int c = 0; c < D; c++) {
            args.mn[c] = args.norm[c];
            args.hw[c] = 0.5 * args.norm[D + c];
            args.sc[c] = args.norm[2 * D + c];
        }
    double x[D], o[D];
    for (int c = 0; c < D; c++) x[c] = u[(size_t)i * D + c];
    if (args.normalized)
        lane_rhs<SYS, true>(x, o, args);
    else
        lane_rhs<SYS, false>(x, o, args);
    for (int c = 0; c < D; c++) out[(size_t)i * D + c] = o[c];
}

template <int SYS>
__global__ void __launch_bounds__(256) rhs_field_kernel(FieldArgs fa, const double *__restrict__ u,
                                                        double *__restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) double V[];
    const int d = fa.d, half = d / 2, s = blockIdx.x;
    for (int e = threadIdx.x; e < d; e += blockDim.x) {
        const double x = u[(size_t)s * d + e];
        V[e] = fa.normalized ? ((x + 1) / 2) * fa.norm[d + e] + fa.norm[e] : x;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < d; e += blockDim.x) {
        double f;
        if constexpr (SYS == NNGP_SYS_BURGERS) {
            f = burgers_elem(V, e, d, fa);
        } else if (e < half) {
            const Nbr5 nb = fhn_neighbours(fa.nx, e);
            const double u1 = V[e];
            f = (((fhn_lap(V, nb, fa.a_off, fa.a_diag) + u1) - u1 * (u1 * u1)) - V[half + e]) + -5E-3 * 1.0;
        } else {
            const Nbr5 nb = fhn_neighbours(fa.nx, e - half);
            f = (1 / 0.1) * ((fhn_lap(V + half, nb, fa.b_off, fa.b_diag) + V[e - half]) - V[e]);
        }
        out[(size_t)s * d + e] = fa.normalized ? f * fa.norm[2 * d + e] : f;
    }
}

__global__ void __launch_bounds__(256) update_kernel(int64_t n, const double *__restrict__ a,
                                                     const double *__restrict__ b,
                                                     const double *__restrict__ c,
                                                     double *__restrict__ out) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const double p = a[i] - b[i];
        out[i] = c ? p + c[i] : p;
    }
}

// ---------------------------------------------------------------------------------------------
// host dispatch
// ---------------------------------------------------------------------------------------------
template <int SYS, int ORDER, bool LIN>
static int launch_lane(const nngp_system *sys, int n, const double *t0, const double *t1,
                       int64_t steps, int64_t gsteps, const int64_t *j0, const double *u0, double *uF,
                       hipStream_t st) {
    LaneArgs a{};
    constexpr int D = LaneSys<SYS>::D;
    NNGP_REQUIRE(sys->d == D, "system kind %d has d=%d, got d=%d", SYS, D, sys->d);
    a.normalized = sys->normalized;
    for (int c = 0; c < 4; c++) a.param[c] = sys->param[c];
    a.rparam0 = 1.0 / sys->param[0];
    a.norm = sys->norm;
    NNGP_REQUIRE(!sys->normalized || sys->norm != nullptr, "normalized system needs norm[3d]");
    const int bs = 64;
    if constexpr (has_group<SYS>::value) {
        // group kernel while all slices' lane groups fit one wave per SIMD (G*n <= 64 * 1024): there
        // the step time is one wave's issue and the group form issues fewer instructions per step;
        // beyond it waves share SIMDs and the lane kernel's G-fold fewer waves win.
        // NNGP_RK_GROUP=0 forces the lane kernel (A/B tool, tests).
        const char *ge = getenv("NNGP_RK_GROUP");
        const int group_on = ge ? atoi(ge) : 1;
        constexpr int G = GroupSys<SYS>::G;
        if (group_on && (int64_t)n * G <= 64 * 1024) {
            const int nb = (int)(((int64_t)G * n + bs - 1) / bs);
            if (sys->normalized)
                hipLaunchKernelGGL((rk_group_kernel<SYS, ORDER, LIN, true>), dim3(nb), dim3(bs), 0, st,
                                   a, n, t0, t1, steps, gsteps, j0, u0, uF);
            else
                hipLaunchKernelGGL((rk_group_kernel<SYS, ORDER, LIN, false>), dim3(nb), dim3(bs), 0, st,
                                   a, n, t0, t1, steps, gsteps, j0, u0, uF);
            NNGP_LAUNCH_CHECK();
            return NNGP_OK;
        }
    }
    if (sys->normalized)
        hipLaunchKernelGGL((rk_lane_kernel<SYS, ORDER, LIN, true>), dim3((n + bs - 1) / bs), dim3(bs), 0, st,
                           a, n, t0, t1, steps, gsteps, j0, u0, uF);
    else
        hipLaunchKernelGGL((rk_lane_kernel<SYS, ORDER, LIN, false>), dim3((n + bs - 1) / bs), dim3(bs), 0,
                           st, a, n, t0, t1, steps, gsteps, j0, u0, uF);
    NNGP_LAUNCH_CHECK();
    return NNGP_OK;
}

template <int SYS, int ORDER, bool LIN, int EPT>
static int launch_field_ept(const FieldArgs &fa, int bt, int n, const double *t0,
                            const double *t1, int64_t steps, int64_t gsteps, const int64_t *j0,
                            const double *u0, double *uF, hipStream_t st) {
    const size_t lds = sizeof(double) * 2 * (size_t)fa.d;
    if (fa.normalized)
        hipLaunchKernelGGL((rk_field_kernel<SYS, ORDER, LIN, EPT, true>), dim3(n), dim3(bt), lds, st, fa, n,
                           t0, t1, steps, gsteps, j0, u0, uF);
    else
        hipLaunchKernelGGL((rk_field_kernel<SYS, ORDER, LIN, EPT, false>), dim3(n), dim3(bt), lds, st, fa, n,
                           t0, t1, steps, gsteps, j0, u0, uF);
    NNGP_LAUNCH_CHECK();
    return NNGP_OK;
}

// threads per slice: env NNGP_RK_THREADS overrides (tuning), else the fewest whole waves that
// keep EPT <= 4 (d=128 -> 64 threads x 2, d=800 -> 256 threads x 4)
static int pick_threads(int d, int n_slices) {
    const char *env = getenv("NNGP_RK_THREADS");
    if (env) {
        int v = atoi(env);
        if (v >= 64 && v <= 1024 && v % 64 == 0) return v;
    }
    int bt = 64;
    while (bt < 256 && (d + bt - 1) / bt > 4) bt += 64;
    // up to 1024 elements: one element per thread while all slices' waves fit ~4 per SIMD (few
    // slices: the per-step latency is the stage chain, FHN-PDE d=800 at 64 slices 5.2 -> 4.0
    // us/step), else <= 2 per thread in 512 threads (512 slices: 8.6 -> 6.7 us/step)
    if ((d + bt - 1) / bt > 2 && d <= 1024) {
        const int64_t waves1 = (int64_t)n_slices * ((d + 63) / 64);
        bt = (waves1 <= 4 * 1024) ? ((d + 63) / 64) * 64 : 512;
    }
    return bt;
}

static int field_args(const nngp_system *sys, FieldArgs &fa) {
    fa = FieldArgs{};
    fa.d = sys->d;
    fa.nx = sys->nx;
    fa.normalized = sys->normalized;
    fa.norm = sys->norm;
    NNGP_REQUIRE(!sys->normalized || sys->norm, "normalized system needs norm[3d]");
    if (sys->kind == NNGP_SYS_BURGERS) {
        NNGP_REQUIRE(sys->nx == sys->d && sys->d >= 3, "Burgers needs nx == d >= 3");
        const double dx = (1.0 - (-1.0)) / (sys->d - 1);
        const double nu = sys->param[0];
        fa.c_off = nu / (dx * dx);   // (nu/dx**2)*Txx
        fa.c_diag = fa.c_off * -2.0;
        fa.c_grad = 1 / (2 * dx);    // (1/(2*dx))*Tx
    } else {
        NNGP_REQUIRE(sys->nx >= 3 && sys->d == 2 * sys->nx * sys->nx, "FHN_PDE needs d = 2 nx^2, nx >= 3");
        const double dx = (1.0 - (-1.0)) / (sys->nx - 1);
        const double c1 = 1 / (dx * dx);
        const double ldiag = c1 * -2.0 + c1 * -2.0;   // (DXX + DYY) diagonal
        fa.a_off = 2.8E-4 * c1;
        fa.a_diag = 2.8E-4 * ldiag;
        fa.b_off = 5E-3 * c1;
        fa.b_diag = 5E-3 * ldiag;
    }
    NNGP_REQUIRE(sizeof(double) * 2 * (size_t)sys->d <= 160 * 1024, "LDS image too large");
    return NNGP_OK;
}

template <int ORDER, bool LIN, int EPT>
static int launch_burgers_wave(const FieldArgs &fa, int n, const double *t0, const double *t1, int64_t steps,
                               int64_t gsteps, const int64_t *j0, const double *u0, double *uF, hipStream_t st) {
    if (fa.normalized)
        hipLaunchKernelGGL((rk_burgers_wave_kernel<ORDER, LIN, EPT, true>), dim3(n), dim3(64), 0, st, fa, n, t0,
                           t1, steps, gsteps, j0, u0, uF);
    else
        hipLaunchKernelGGL((rk_burgers_wave_kernel<ORDER, LIN, EPT, false>), dim3(n), dim3(64), 0, st, fa, n, t0,
                           t1, steps, gsteps, j0, u0, uF);
    NNGP_LAUNCH_CHECK();
    return NNGP_OK;
}

template <int SYS, int ORDER, bool LIN>
static int launch_field(const nngp_system *sys, int n, const double *t0, const double *t1,
                        int64_t steps, int64_t gsteps, const int64_t *j0, const double *u0, double *uF,
                        hipStream_t st) {
    FieldArgs fa;
    int rc = field_args(sys, fa);
    if (rc) return rc;
    if (SYS == NNGP_SYS_BURGERS && sys->d % 64 == 0 && sys->d <= 256 && !getenv("NNGP_BURGERS_LDS")) {
        const int e = sys->d / 64;
        if (e == 1) return launch_burgers_wave<ORDER, LIN, 1>(fa, n, t0, t1, steps, gsteps, j0, u0, uF, st);
        if (e == 2) return launch_burgers_wave<ORDER, LIN, 2>(fa, n, t0, t1, steps, gsteps, j0, u0, uF, st);
        if (e == 3) return launch_burgers_wave<ORDER, LIN, 3>(fa, n, t0, t1, steps, gsteps, j0, u0, uF, st);
        return launch_burgers_wave<ORDER, LIN, 4>(fa, n, t0, t1, steps, gsteps, j0, u0, uF, st);
    }
    // FHN-PDE from 16x16 grid points: one thread per point (u and v of the point) unless
    // NNGP_FHN_PAIR=0 or a thread count is forced.  Measured (tools/contract_probe.py): d = 800 at
    // 512 slices 7.50 -> 6.75 us/step, at 64 slices unchanged; d = 200 (100 points: 28 of 128
    // lanes idle) 3.65 -> 4.25, so small grids keep the element kernel's 64 threads x 4
    if (SYS == NNGP_SYS_FHN_PDE && sys->d / 2 >= 256 && sys->d / 2 <= 1024 && !getenv("NNGP_RK_THREADS")) {
        const char *pe = getenv("NNGP_FHN_PAIR");
        if (!pe || atoi(pe) != 0) {
            const int bt = ((sys->d / 2 + 63) / 64) * 64;
            const size_t lds = sizeof(double) * 2 * bt * FhnPairImages<Tableau<ORDER>::S>::N;
            if (fa.normalized)
                hipLaunchKernelGGL((rk_fhn_pair_kernel<ORDER, LIN, true>), dim3(n), dim3(bt), lds, st, fa, n, t0, t1,
                                   steps, gsteps, j0, u0, uF);
            else
                hipLaunchKernelGGL((rk_fhn_pair_kernel<ORDER, LIN, false>), dim3(n), dim3(bt), lds, st, fa, n, t0, t1,
                                   steps, gsteps, j0, u0, uF);
            NNGP_LAUNCH_CHECK();
            return NNGP_OK;
        }
    }
    const int bt = pick_threads(sys->d, n);
    const int ept = (sys->d + bt - 1) / bt;
    NNGP_REQUIRE(ept <= 8, "d=%d with %d threads per slice exceeds the field kernel's 8 elements per thread",
                 sys->d, bt);
    // each EPT variant is compiled for at most 1024 / 512 / 256 / 256 threads (launch bounds): a
    // larger block (only reachable through NNGP_RK_THREADS) would fail to launch
    const int bound = ept <= 1 ? 1024 : (ept <= 2 ? 512 : 256);
    NNGP_REQUIRE(bt <= bound, "%d threads per slice exceed the field kernel's bound %d at %d elements per thread "
                 "(d=%d)", bt, bound, ept <= 2 ? ept : (ept <= 4 ? 4 : 8), sys->d);
    if (ept <= 1) return launch_field_ept<SYS, ORDER, LIN, 1>(fa, bt, n, t0, t1, steps, gsteps, j0, u0, uF, st);
    if (ept <= 2) return launch_field_ept<SYS, ORDER, LIN, 2>(fa, bt, n, t0, t1, steps, gsteps, j0, u0, uF, st);
    if (ept <= 4) return launch_field_ept<SYS, ORDER, LIN, 4>(fa, bt, n, t0, t1, steps, gsteps, j0, u0, uF, st);
    return launch_field_ept<SYS, ORDER, LIN, 8>(fa, bt, n, t0, t1, steps, gsteps, j0, u0, uF, st);
}

template <int ORDER, bool LIN>
static int dispatch_sys(const nngp_system *s, int n, const double *t0, const double *t1,
                        int64_t steps, int64_t gsteps, const int64_t *j0, const double *u0,
                        double *uF, hipStream_t st) {
    switch (s->kind) {
    case NNGP_SYS_LORENZ: return launch_lane<NNGP_SYS_LORENZ, ORDER, LIN>(s, n, t0, t1, steps, gsteps, j0, u0, uF, st);
    case NNGP_SYS_HOPF: return launch_lane<NNGP_SYS_HOPF, ORDER, LIN>(s, n, t0, t1, steps, gsteps, j0, u0, uF, st);
    case NNGP_SYS_THOMAS_LABYRINTH:
        return launch_lane<NNGP_SYS_THOMAS_LABYRINTH, ORDER, LIN>(s, n, t0, t1, steps, gsteps, j0, u0, uF, st);
    case NNGP_SYS_FHN_ODE: return launch_lane<NNGP_SYS_FHN_ODE, ORDER, LIN>(s, n, t0, t1, steps, gsteps, j0, u0, uF, st);
    case NNGP_SYS_ROSSLER: return launch_lane<NNGP_SYS_ROSSLER, ORDER, LIN>(s, n, t0, t1, steps, gsteps, j0, u0, uF, st);
    case NNGP_SYS_BRUSSELATOR:
        return launch_lane<NNGP_SYS_BRUSSELATOR, ORDER, LIN>(s, n, t0, t1, steps, gsteps, j0, u0, uF, st);
    case NNGP_SYS_DBL_PEND: return launch_lane<NNGP_SYS_DBL_PEND, ORDER, LIN>(s, n, t0, t1, steps, gsteps, j0, u0, uF, st);
    case NNGP_SYS_BURGERS: return launch_field<NNGP_SYS_BURGERS, ORDER, LIN>(s, n, t0, t1, steps, gsteps, j0, u0, uF, st);
    case NNGP_SYS_FHN_PDE: return launch_field<NNGP_SYS_FHN_PDE, ORDER, LIN>(s, n, t0, t1, steps, gsteps, j0, u0, uF, st);
    default: set_error("unknown system kind %d", s->kind); return NNGP_E_ARG;
    }
}

template <bool LIN>
static int dispatch_tab(const nngp_system *s, int tab, int n, const double *t0, const double *t1,
                        int64_t steps, int64_t gsteps, const int64_t *j0, const double *u0,
                        double *uF, hipStream_t st) {
    switch (tab) {
    case NNGP_RK1: return dispatch_sys<1, LIN>(s, n, t0, t1, steps, gsteps, j0, u0, uF, st);
    case NNGP_RK2: return dispatch_sys<2, LIN>(s, n, t0, t1, steps, gsteps, j0, u0, uF, st);
    case NNGP_RK4: return dispatch_sys<4, LIN>(s, n, t0, t1, steps, gsteps, j0, u0, uF, st);
    case NNGP_RK8: return dispatch_sys<8, LIN>(s, n, t0, t1, steps, gsteps, j0, u0, uF, st);
    default: set_error("unknown tableau %d (RK1/2/4/8)", tab); return NNGP_E_ARG;
    }
}

template <int SYS>
static int launch_rhs_lane(const nngp_system *sys, int n, const double *u, double *out, hipStream_t st) {
    LaneArgs a{};
    NNGP_REQUIRE(sys->d == LaneSys<SYS>::D, "system kind %d has d=%d, got d=%d", SYS, LaneSys<SYS>::D, sys->d);
    NNGP_REQUIRE(!sys->normalized || sys->norm != nullptr, "normalized system needs norm[3d]");
    a.normalized = sys->normalized;
    a.norm = sys->norm;
    for (int c = 0; c < 4; c++) a.param[c] = sys->param[c];
    a.rparam0 = 1.0 / sys->param[0];
    hipLaunchKernelGGL(rhs_lane_kernel<SYS>, dim3((n + 63) / 64), dim3(64), 0, st, a, n, u, out);
    NNGP_LAUNCH_CHECK();
    return NNGP_OK;
}

template <int SYS>
static int launch_rhs_field(const nngp_system *sys, int n, const double *u, double *out, hipStream_t st) {
    FieldArgs fa;
    int rc = field_args(sys, fa);
    if (rc) return rc;
    hipLaunchKernelGGL(rhs_field_kernel<SYS>, dim3(n), dim3(256), sizeof(double) * sys->d, st, fa, u, out);
    NNGP_LAUNCH_CHECK();
    return NNGP_OK;
}

}  // namespace NNGP_RK_VARIANT
}  // namespace nngp

#ifdef NNGP_RK_FMA
// the contracted code object's one entry (not part of include/nngp.h): same arguments as the exact
// build's dispatch below
extern "C" __attribute__((visibility("hidden"))) int nngp_rk_dispatch_contracted(
    const nngp_system *sys, int tableau, int linspace, int n_slices, const double *t0, const double *t1,
    int64_t steps, int64_t gsteps, const int64_t *j0, const double *u0, double *uF, void *stream) {
    using namespace nngp;
    hipStream_t st = (hipStream_t)stream;
    if (linspace) return dispatch_tab<true>(sys, tableau, n_slices, t0, t1, steps, gsteps, j0, u0, uF, st);
    return dispatch_tab<false>(sys, tableau, n_slices, t0, t1, steps, gsteps, j0, u0, uF, st);
}
#else
extern "C" int nngp_rk_dispatch_contracted(const nngp_system *sys, int tableau, int linspace, int n_slices,
                                           const double *t0, const double *t1, int64_t steps, int64_t gsteps,
                                           const int64_t *j0, const double *u0, double *uF, void *stream);

extern "C" int nngp_rhs_batch(const nngp_system *sys, int n, const double *u, double *out, void *stream) {
    using namespace nngp;
    NNGP_REQUIRE(sys != nullptr && n >= 0, "bad sys / n");
    if (n == 0) return NNGP_OK;
    NNGP_REQUIRE(u && out, "null array argument");
    hipStream_t st = (hipStream_t)stream;
    switch (sys->kind) {
    case NNGP_SYS_LORENZ: return launch_rhs_lane<NNGP_SYS_LORENZ>(sys, n, u, out, st);
    case NNGP_SYS_HOPF: return launch_rhs_lane<NNGP_SYS_HOPF>(sys, n, u, out, st);
    case NNGP_SYS_THOMAS_LABYRINTH: return launch_rhs_lane<NNGP_SYS_THOMAS_LABYRINTH>(sys, n, u, out, st);
    case NNGP_SYS_FHN_ODE: return launch_rhs_lane<NNGP_SYS_FHN_ODE>(sys, n, u, out, st);
    case NNGP_SYS_ROSSLER: return launch_rhs_lane<NNGP_SYS_ROSSLER>(sys, n, u, out, st);
    case NNGP_SYS_BRUSSELATOR: return launch_rhs_lane<NNGP_SYS_BRUSSELATOR>(sys, n, u, out, st);
    case NNGP_SYS_DBL_PEND: return launch_rhs_lane<NNGP_SYS_DBL_PEND>(sys, n, u, out, st);
    case NNGP_SYS_BURGERS: return launch_rhs_field<NNGP_SYS_BURGERS>(sys, n, u, out, st);
    case NNGP_SYS_FHN_PDE: return launch_rhs_field<NNGP_SYS_FHN_PDE>(sys, n, u, out, st);
    default: set_error("unknown system kind %d", sys->kind); return NNGP_E_ARG;
    }
}

extern "C" int nngp_parareal_update(int64_t n, const double *a, const double *b, const double *c,
                                    double *out, void *stream) {
    using namespace nngp;
    NNGP_REQUIRE(n >= 0, "n < 0");
    if (n == 0) return NNGP_OK;
    NNGP_REQUIRE(a && b && out, "null array argument");
    const int64_t blocks = std::min<int64_t>((n + 255) / 256, 2048);
    hipLaunchKernelGGL(update_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, n, a, b, c, out);
    NNGP_LAUNCH_CHECK();
    return NNGP_OK;
}

extern "C" int nngp_rk_batch(const nngp_system *sys, int tableau, int step_mode, int n_slices,
                             const double *t0, const double *t1, int64_t steps, const double *u0,
                             double *uF, void *stream) {
    using namespace nngp;
    NNGP_REQUIRE(sys != nullptr, "sys is NULL");
    NNGP_REQUIRE(n_slices >= 0, "n_slices < 0");
    NNGP_REQUIRE(steps >= 1, "steps must be >= 1 (got %lld)", (long long)steps);
    if (n_slices == 0) return NNGP_OK;
    NNGP_REQUIRE(t0 && t1 && u0 && uF, "null array argument");
    hipStream_t st = (hipStream_t)stream;
    const int mode = step_mode & ~NNGP_STEP_CONTRACT;
    NNGP_REQUIRE(mode == NNGP_STEP_FIXED || mode == NNGP_STEP_LINSPACE, "unknown step_mode %d", step_mode);
    if (step_mode & NNGP_STEP_CONTRACT)
        return nngp_rk_dispatch_contracted(sys, tableau, mode == NNGP_STEP_LINSPACE, n_slices, t0, t1, steps,
                                           steps, nullptr, u0, uF, stream);
    if (mode == NNGP_STEP_FIXED)
        return dispatch_tab<false>(sys, tableau, n_slices, t0, t1, steps, steps, nullptr, u0, uF, st);
    return dispatch_tab<true>(sys, tableau, n_slices, t0, t1, steps, steps, nullptr, u0, uF, st);
}

extern "C" int nngp_rk_batch_grid(const nngp_system *sys, int tableau, int n_slices,
                                  const double *g0, const double *g1, int64_t gsteps,
                                  const int64_t *j0, int64_t steps, const double *u0, double *uF,
                                  void *stream) {
    using namespace nngp;
    NNGP_REQUIRE(sys != nullptr, "sys is NULL");
    NNGP_REQUIRE(n_slices >= 0 && steps >= 1 && gsteps >= 1, "bad n_slices / steps / gsteps");
    if (n_slices == 0) return NNGP_OK;
    NNGP_REQUIRE(g0 && g1 && j0 && u0 && uF, "null array argument");
    return dispatch_tab<true>(sys, tableau, n_slices, g0, g1, steps, gsteps, j0, u0, uF,
                              (hipStream_t)stream);
}
#endif  // NNGP_RK_FMA
