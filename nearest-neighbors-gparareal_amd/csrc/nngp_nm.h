// nngp_nm.h -- the Nelder-Mead state machine shared by the device fits (nngp_gp.hip) and the
// host-driven full-GP fits (nngp_gpfull.hip).  One evaluation request at a time (px, py); the
// caller evaluates it and calls nm_consume with the value.
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>

#define NN_HD __host__ __device__ __forceinline__

namespace nngp {

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

NN_HD bool nm_less(double a, double b) { return a < b || (b != b && a == a); }

NN_HD void nm_sort(NM &S) {   // stable insertion sort of 3 (numpy argsort)
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
NN_HD bool nm_req(NM &S, const NMCfg &c, double x, double y, int st) {
    if (S.fcalls >= c.maxfun) return false;
    S.fcalls++;
    S.px = x;
    S.py = y;
    S.st = st;
    return true;
}

// loop head of the while in _minimize_neldermead
NN_HD void nm_check(NM &S, const NMCfg &c) {
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

NN_HD void nm_abort(NM &S, const NMCfg &c) {
    nm_sort(S);
    nm_check(S, c);   // fcalls >= maxfun -> DONE
}

NN_HD void nm_end_iter(NM &S, const NMCfg &c) {
    S.iters += 1;
    nm_sort(S);
    nm_check(S, c);
}

NN_HD void nm_shrink_start(NM &S, const NMCfg &c) {
    S.s1x = S.s0x + 0.5 * (S.s1x - S.s0x);   // sim[j] = sim[0] + sigma*(sim[j]-sim[0])
    S.s1y = S.s0y + 0.5 * (S.s1y - S.s0y);
    if (!nm_req(S, c, S.s1x, S.s1y, ST_SHRINK1)) nm_abort(S, c);
}

NN_HD void nm_consume(NM &S, const NMCfg &c, double f) {
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


// the initial simplex (x0, x0 with x0[k] *= 1.05, or 0.00025 when x0[k] == 0) and the first
// request (scipy _minimize_neldermead, nonzdelt / zdelt)
NN_HD void nm_start(NM &S, const NMCfg &c, double t0x, double t0y) {
    S.s0x = t0x; S.s0y = t0y;
    S.s1x = (t0x != 0) ? (1 + 0.05) * t0x : 0.00025; S.s1y = t0y;
    S.s2x = t0x; S.s2y = (t0y != 0) ? (1 + 0.05) * t0y : 0.00025;
    S.fcalls = 0;
    S.iters = 0;
    S.st = ST_INIT0;
    if (!nm_req(S, c, S.s0x, S.s0y, ST_INIT0)) S.st = ST_DONE;
}

}  // namespace nngp
