// nngp_math.h -- exp / log / 10^x for the GP likelihood, with a fully specified operation order.
//
// The -LML (models.py:240-252) evaluates hundreds of exp's per Nelder-Mead step, and Nelder-Mead
// branches on comparisons of those values, so a single last-ulp difference between two libms
// (ocml on the GPU, glibc in the CPU oracle) redirects whole fits.  These routines are plain
// IEEE arithmetic + fma + ldexp + rint, all exactly specified, so the GPU and the oracle's copy
// (oracle/nngp_oracle.c, same algorithm and constants) agree bit for bit.  Accuracy ~1 ulp.
//   exp:  Cody-Waite reduction x = n ln2 + r (|r| <= ln2/2), degree-13 Taylor (Horner, fma)
//   10^x: the same with the argument x*ln10 carried as a double-double
//   log:  fdlibm __ieee754_log (Sun Microsystems, freely distributable): x = 2^k (1+f),
//         s = f/(2+f), polynomial in s^2
#pragma once

#include <hip/hip_runtime.h>

namespace nngp {

struct MathC {
    static constexpr double INV_LN2 = 0x1.71547652b82fep+0;
    static constexpr double LN2_HI = 0x1.62e42fefa3800p-1;    // ln2 with 13 trailing zero bits
    static constexpr double LN2_LO = 0x1.ef35793c76730p-45;
    static constexpr double LN10 = 0x1.26bb1bbb55516p+1;
    static constexpr double LN10_LO = -0x1.f48ad494ea3e9p-53;  // ln10 - (double)ln10
    static constexpr double EXP_OVF = 709.782712893384;
    static constexpr double EXP_UNF = -745.1332191019412;
};

// fma(a, b, c) as one 3-address v_fma_f64.  In a Horner step p = fma(p, r, C) with C a
// loop-invariant coefficient held in a VGPR (gfx950's VOP3 takes no 64-bit literal, and the
// SGPRs are taken), LLVM emits the 2-address v_fmac_f64, whose addend is its destination, and so
// first copies C there: a v_mov_b64 per step, ~130 per likelihood evaluation at m = 20.  Same
// operation, same bits.
__device__ __forceinline__ double fma3(double a, double b, double c) {
    double d;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}

// exp(hi + lo) with |lo| << |hi|.  Branch-free (selects) so it inlines cheaply inside the
// unrolled kernel-row loops; identical results to the oracle's branchy form.
// NONPOS: hi <= 0 or NaN, lo == 0 (the SE kernel's c*D2 with c < 0 <= D2, models.py:146-148) --
// the same bits with three ops fewer: the upper clamp and the overflow select are never taken
// there, and r + 0 only normalises the sign of a zero r, which no term of the polynomial sees
// (p = fma(p, +-0, c) = c).
// BLOCK: the Horner steps as one asm block (below); false keeps ten separate fma3 statements,
// which the register-starved m > 32 fit kernels schedule better (fewer spills).
template <bool NONPOS = false, bool BLOCK = true>
__device__ __forceinline__ double nn_exp_t(double hi, double lo) {
    const double xc = NONPOS ? fmax(hi, -746.0) : fmin(fmax(hi, -746.0), 710.0);   // NaN -> -746
    const double n = rint(xc * MathC::INV_LN2);
    double r = fma(-n, MathC::LN2_HI, xc);
    r = fma(-n, MathC::LN2_LO, r);
    if constexpr (!NONPOS) r = r + lo;
    // sum_{j=0}^{13} r^j / j!: the first ten Horner steps (1/13! .. 1/3!) as ONE asm block of
    // 3-address v_fma_f64 (see fma3; one block instead of ten, because LLVM's hazard recognizer
    // puts an s_nop after every inline asm statement), then three plain steps
    double p;
    if constexpr (!BLOCK) {
        p = fma3(1.0 / 6227020800.0, r, 1.0 / 479001600.0);
        p = fma3(p, r, 1.0 / 39916800.0);
        p = fma3(p, r, 1.0 / 3628800.0);
        p = fma3(p, r, 1.0 / 362880.0);
        p = fma3(p, r, 1.0 / 40320.0);
        p = fma3(p, r, 1.0 / 5040.0);
        p = fma3(p, r, 1.0 / 720.0);
        p = fma3(p, r, 1.0 / 120.0);
        p = fma3(p, r, 1.0 / 24.0);
        p = fma3(p, r, 1.0 / 6.0);
    } else
    asm("v_fma_f64 %0, %2, %1, %3\n\t"
        "v_fma_f64 %0, %0, %1, %4\n\tv_fma_f64 %0, %0, %1, %5\n\tv_fma_f64 %0, %0, %1, %6\n\t"
        "v_fma_f64 %0, %0, %1, %7\n\tv_fma_f64 %0, %0, %1, %8\n\tv_fma_f64 %0, %0, %1, %9\n\t"
        "v_fma_f64 %0, %0, %1, %10\n\tv_fma_f64 %0, %0, %1, %11\n\tv_fma_f64 %0, %0, %1, %12"
        : "=&v"(p)
        : "v"(r), "v"(1.0 / 6227020800.0), "v"(1.0 / 479001600.0), "v"(1.0 / 39916800.0),
          "v"(1.0 / 3628800.0), "v"(1.0 / 362880.0), "v"(1.0 / 40320.0), "v"(1.0 / 5040.0),
          "v"(1.0 / 720.0), "v"(1.0 / 120.0), "v"(1.0 / 24.0), "v"(1.0 / 6.0));
    p = fma(p, r, 0.5);
    p = fma(p, r, 1.0);
    p = fma(p, r, 1.0);
    double res = ldexp(p, (int)n);
    if constexpr (!NONPOS) res = (hi > MathC::EXP_OVF) ? __builtin_huge_val() : res;
    res = (hi < MathC::EXP_UNF) ? 0.0 : res;
    return (hi != hi) ? hi : res;
}

__device__ __forceinline__ double nn_exp_dd(double hi, double lo) { return nn_exp_t<false>(hi, lo); }
__device__ __forceinline__ double nn_exp(double x) { return nn_exp_t<false>(x, 0.0); }
// exp(x) for x <= 0 or NaN only (see NONPOS)
__device__ __forceinline__ double nn_exp_nonpos(double x) { return nn_exp_t<true>(x, 0.0); }
__device__ __forceinline__ double nn_exp_nonpos_sep(double x) { return nn_exp_t<true, false>(x, 0.0); }

// sqrt(x) and 1.0/x, correctly rounded, for x in [2^-500, 2^500]: the instruction sequences the
// compiler emits for sqrt() and 1.0/x on gfx950 (rsq + Goldschmidt with two corrections; rcp +
// two Newton steps + the Markstein quotient correction) without the range scaling (ldexp /
// v_div_scale) and special-value fixups (v_cmp_class / v_div_fixup), which are identities on that
// range -- the same bits, ~12 ops fewer per pair.  Callers check the range (wave-uniformly) and
// keep sqrt() / 1.0/x for everything else.
__device__ __forceinline__ double sqrt_mid(double x) {
    const double y = __builtin_amdgcn_rsq(x);
    double g = x * y, h = y * 0.5;
    const double r = fma(-h, g, 0.5);
    g = fma(g, r, g);
    h = fma(h, r, h);
    double d = fma(-g, g, x);
    g = fma(d, h, g);
    d = fma(-g, g, x);
    return fma(d, h, g);
}
__device__ __forceinline__ double rcp_mid(double b) {
    double y = __builtin_amdgcn_rcp(b);
    y = fma(y, fma(-b, y, 1.0), y);
    y = fma(y, fma(-b, y, 1.0), y);
    return fma(fma(-b, y, 1.0), y, y);   // q = 1*y; r = 1 - b q; q + r y
}
// x in [2^-500, 2^500] (NaN and negatives excluded): one compare on the high word
__device__ __forceinline__ bool in_mid_range(double x) {
    const unsigned hi = (unsigned)(__double_as_longlong(x) >> 32);
    return hi - 0x20B00000u <= 0x5F300000u - 0x20B00000u;
}

// 10^x = exp(x ln10), x ln10 as a double-double (models.py: 10**sigma)
__device__ __forceinline__ double nn_pow10(double x) {
    const double hi = x * MathC::LN10;
    const double lo = fma(x, MathC::LN10, -hi) + x * MathC::LN10_LO;
    return nn_exp_dd(hi, lo);
}

// natural log for x > 0 finite (the Cholesky diagonal); fdlibm e_log.c
__device__ __forceinline__ double nn_log(double x_in) {
    const bool pos = x_in > 0.0 && x_in != __builtin_huge_val();
    const double x = pos ? x_in : 1.0;
    const double Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01,
                 Lg3 = 2.857142874366239149e-01, Lg4 = 2.222219843214978396e-01,
                 Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
                 Lg7 = 1.479819860511658591e-01;
    const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
    int k;
    double m = frexp(x, &k);                   // x = m 2^k, m in [0.5, 1)
    if (m < 0.70710678118654752440) {          // bring 1+f into [sqrt(1/2), sqrt(2))
        m = m * 2.0;
        k -= 1;
    }
    const double f = m - 1.0;
    const double dk = (double)k;
    const double s = f / (2.0 + f);
    const double z = s * s;
    const double w = z * z;
    const double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
    const double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
    const double R = t2 + t1;
    const double hfsq = 0.5 * f * f;
    const double res = dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
    if (pos) return res;
    return x_in == 0.0 ? -__builtin_huge_val() : (x_in > 0.0 ? x_in : __builtin_nan(""));
}

// sin / cos for the trigonometric vector fields (ThomasLabyrinth systems.py:257-271, DblPend
// :182-189), fully specified like exp/log above so the GPU and the oracle agree bit for bit:
// x = n pi/2 + r by a three-term fma Cody-Waite reduction (fdlibm's 33-bit pi/2 pieces; exact
// n*PIO2_1 for |n| < 2^20), then fdlibm's __kernel_sin / __kernel_cos polynomials on |r| <= pi/4
// and the quadrant select.  ~1 ulp for the |x| < 1e5 these fields see.
struct TrigC {
    static constexpr double INVPIO2 = 6.36619772367581382433e-01;
    static constexpr double PIO2_1 = 1.57079632673412561417e+00;
    static constexpr double PIO2_2 = 6.07710050630396597660e-11;
    static constexpr double PIO2_3 = 2.02226624871116645580e-21;
    static constexpr double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                            S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                            S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    static constexpr double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                            C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                            C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
};

__device__ __forceinline__ void nn_sincos(double x, double &sn, double &cs) {
    const bool fin = x - x == 0.0;                 // finite
    // (the oracle zeroes a non-finite x before the reduction; its result is replaced by x - x below
    // on both sides, so the kernel reduces x itself)
    const double n = rint(x * TrigC::INVPIO2);
    double r = fma(-n, TrigC::PIO2_1, x);
    r = fma(-n, TrigC::PIO2_2, r);
    r = fma(-n, TrigC::PIO2_3, r);
    const double z = r * r;
    const double v = z * r;
    const double ps = TrigC::S2 + z * (TrigC::S3 + z * (TrigC::S4 + z * (TrigC::S5 + z * TrigC::S6)));
    const double ks = r + v * (TrigC::S1 + z * ps);
    const double pc = z * (TrigC::C1 + z * (TrigC::C2 + z * (TrigC::C3 + z * (TrigC::C4 + z * (TrigC::C5 + z * TrigC::C6)))));
    const double hz = 0.5 * z;
    const double w = 1.0 - hz;
    const double kc = w + (((1.0 - w) - hz) + z * pc);
    // quadrant n mod 4 from the bit pattern of n + 1.5*2^52 (for |n| < 2^51 its low mantissa bits
    // are n in two's complement; beyond, the same correctly rounded add on both sides): two ops
    // instead of n - 4*floor(n/4) and a conversion
    const int q = (int)((uint32_t)__double_as_longlong(n + 6755399441055744.0) & 3u);
    double s_ = (q & 1) ? kc : ks;
    double c_ = (q & 1) ? ks : kc;
    // sign flips as sign-bit xors (a negation is exactly that, so this is the oracle's `-s_`)
    s_ = __longlong_as_double(__double_as_longlong(s_) ^ ((long long)(q & 2) << 62));
    c_ = __longlong_as_double(__double_as_longlong(c_) ^ ((long long)((q + 1) & 2) << 62));
#ifdef NNGP_RK_FMA
    // contracted propagator build: an inf/NaN argument already gives r = NaN (fma(-inf, PIO2_1,
    // inf)), hence NaN polynomials; the exact build keeps the oracle's explicit select
    (void)fin;
    sn = s_;
    cs = c_;
    return;
#endif
    const double nanv = x - x;                     // NaN for inf / NaN arguments
    sn = fin ? s_ : nanv;
    cs = fin ? c_ : nanv;
}

// sin alone (ThomasLabyrinth, systems.py:257-271, whose three sines are all it evaluates): x = n pi
// + r by the same three-term fma reduction (fdlibm's 33-bit pieces, doubled), |r| <= pi/2, then ONE
// odd polynomial r + r^3 P(r^2) (8 coefficients, a weighted minimax fit of sin(r)/r - 1 on
// [0, (pi/2)^2] computed with mpmath, relative error 2.8e-19; tests/golden/sin_pi_fit.py) and the
// sign (-1)^n as a sign-bit xor.  No quadrant select between two polynomials, so ~20 VALU
// instead of ~40 per sine.  <= 2 ulp from glibc (tests/test_oracle_golden.py: |x| <= 40 and the
// field's whole attractor range |x| <= b/a = 20 with margin, 2e5 points on |x| <= 25; |x| <= 1e4).
// Range of validity: the parity trick needs |n| < 2^51, i.e. |x| < pi*2^51; the three-term
// reduction keeps the 2-ulp bound only while n*PI_3's rounding stays far below r's ulp (measured
// to |x| = 1e4; ThomasLabyrinth's states stay within |x| <= 20).
struct SinPiC {
    static constexpr double INVPI = 0x1.45f306dc9c883p-2;
    static constexpr double PI_1 = 2 * 1.57079632673412561417e+00, PI_2 = 2 * 6.07710050630396597660e-11,
                            PI_3 = 2 * 2.02226624871116645580e-21;
    static constexpr double S1 = -0x1.5555555555555p-3, S2 = 0x1.11111111110c1p-7, S3 = -0x1.a01a01a0148bbp-13,
                            S4 = 0x1.71de3a5287c12p-19, S5 = -0x1.ae6454cb54cccp-26, S6 = 0x1.6123cb28741dap-33,
                            S7 = -0x1.ae431d76c3814p-41, S8 = 0x1.88299fb2db5f9p-49;
};

__device__ __forceinline__ double nn_sin_pi(double x) {
    const double n = rint(x * SinPiC::INVPI);
    double r = fma(-n, SinPiC::PI_1, x);
    r = fma(-n, SinPiC::PI_2, r);
    r = fma(-n, SinPiC::PI_3, r);
    const double z = r * r;
    double p = fma(SinPiC::S8, z, SinPiC::S7);
    p = fma(p, z, SinPiC::S6);
    p = fma(p, z, SinPiC::S5);
    p = fma(p, z, SinPiC::S4);
    p = fma(p, z, SinPiC::S3);
    p = fma(p, z, SinPiC::S2);
    p = fma(p, z, SinPiC::S1);
    const double s = fma(r * z, p, r);
    // (-1)^n: the low bit of n + 1.5*2^52 (n in two's complement for |n| < 2^51), into the sign
    const long long par = __double_as_longlong(n + 6755399441055744.0) & 1;
    // inf / NaN arguments give NaN without a select, as sin does: n = rint(+-inf / pi) = +-inf, so
    // r = fma(-n, PI_1, x) = inf - inf = NaN (a NaN x propagates).  Finite x never takes the
    // select the round-2 form had (x - x == 0), so finite results are unchanged; only the NaN's
    // payload differs (4 VALU per sine, 16 per ThomasLabyrinth RK4 step)
    return __longlong_as_double(__double_as_longlong(s) ^ (par << 63));
}

__device__ __forceinline__ double nn_sin(double x) {
    double s, c;
    nn_sincos(x, s, c);
    return s;
}

__device__ __forceinline__ double nn_cos(double x) {
    double s, c;
    nn_sincos(x, s, c);
    return c;
}

}  // namespace nngp
