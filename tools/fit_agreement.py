"""Fit-level agreement between the oracle's restatement and the reference, attributed by cause
("What's weak" 1 / "Next round" 6).  CPU only, test infrastructure.

The golden fits (tests/golden/preds_d128.npz: one NNGP_p.get_preds at d = 128, m = 15, 1 152
fits; tests/golden/nm.npz: 3 x 27 fits at m = 10 / 18 / 30) were produced by running the reference
(models.py:240-260 under tests/golden/gen_golden.py).  Their -LML is restated here twice in
Python:
  S0  the reference's own arithmetic: numpy's 10**x and exp (the generator's broadcast kernel),
      np.linalg.cholesky (OpenBLAS potrf), scipy solve_triangular, y @ alpha and np.sum(np.log(diag))
      -- this must reproduce the recorded fits (checked);
and then one component at a time replaced by the oracle's (oracle/nngp_oracle.c, which the GPU
reproduces bit for bit):
  S1  + 10**x and exp: nn_pow10 / nn_exp (csrc/nngp_math.h)
  S2  + the Cholesky: OpenBLAS dpotf2_L's order as restated (orc_potf2)
  S3  + the triangular solves: successive subtraction, Markstein quotients (orc_solves)
  S4  + log and the two sums: nn_log, the 16-lane butterfly order -- this IS orc_nlml (checked).
Each fit is re-run by scipy's Nelder-Mead (which the oracle's state machine reproduces bit for
bit) at every stage.  A fit whose S4 result differs from S0 is attributed to the FIRST stage that
changed it, and flagged "pass/fail" when the first differing evaluation along the two paths is
+inf on one side only (a Cholesky that passes on one side and fails on the other).

    python tools/fit_agreement.py [--json out.json]
"""
import json
import os
import sys
import time

import numpy as np
import scipy.linalg as sl
from scipy.optimize import minimize

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'oracle')]
import oracle as O  # noqa: E402

LIB = O.lib()
LOG_2PI = 1.8378770664093453
STAGES = ['S0 reference', 'S1 +exp/pow10', 'S2 +Cholesky', 'S3 +solves', 'S4 +log/sums (= oracle)']
CAUSE = {1: 'exp / 10^x ulp', 2: 'Cholesky summation order', 3: 'solve order', 4: 'log ulp / sum order'}


def _arr(f, x):
    x = np.ascontiguousarray(x, dtype=np.float64)
    out = np.empty_like(x)
    f(x.size, O._p(x), O._p(out))
    return out


def butterfly(v):
    """oracle butterfly_sum (nngp_oracle.c): rows i, i+16, ... folded first, then levels 1,2,4,8"""
    n = len(v)
    buf = [v[i] if i < n else 0.0 for i in range(16)]
    for i in range(16):
        s = 1
        while 16 * s < n:
            buf[i] = buf[i] + (v[i + 16 * s] if i + 16 * s < n else 0.0)
            s += 1
    s = 1
    while s < 16:
        for i in range(0, 16, 2 * s):
            buf[i] = buf[i] + buf[i + s]
        s <<= 1
    return buf[0]


def nlml(stage, D2, y, th, jitter):
    """-LML of models.py:240-252 at stage S<stage> (see the module docstring); NaN -> +inf."""
    sx, sy = np.float64(th[0]), np.float64(th[1])
    m = len(y)
    if stage >= 1:
        c = -0.5 * (1 / LIB.nn_pow10(float(sx)))
        K = LIB.nn_pow10(float(sy)) * _arr(LIB.orc_exp_array, c * D2)
    else:   # gen_golden._broadcast_kernel: 10**(sigma_y) * np.exp(-0.5 * (1/(10**sigma_x)) * sq)
        K = 10 ** (sy) * np.exp(-0.5 * (1 / (10 ** sx)) * D2)
    K = K + np.eye(m) * 10 ** np.float64(jitter)
    if stage >= 2:
        L = np.ascontiguousarray(np.tril(K))
        rinv = np.empty(m)
        if LIB.orc_potf2(m, O._p(L), O._p(rinv)):
            return np.inf
    else:
        try:
            L = np.linalg.cholesky(K)
        except np.linalg.LinAlgError:
            return np.inf
        rinv = 1.0 / np.diag(L)
    if stage >= 3:
        alpha = np.empty(m)
        yc = np.ascontiguousarray(y, dtype=np.float64)
        LIB.orc_solves(m, O._p(np.ascontiguousarray(L)), O._p(rinv), O._p(yc), O._p(alpha))
    else:
        alpha = sl.solve_triangular(L.T, sl.solve_triangular(L, y, lower=True, check_finite=False), lower=False,
                                    check_finite=False)
    if stage >= 4:
        ydot = butterfly(list(y * alpha))
        slog = butterfly(list(_arr(LIB.orc_log_array, np.diag(L).copy())))
        res = -(((-0.5 * ydot) - slog) - (m / 2) * LOG_2PI)
    else:
        res = -(-0.5 * y.T @ alpha - np.sum(np.log(np.diag(L))) - (m / 2) * np.log(2 * np.pi))
    return np.inf if np.isnan(res) else float(res)


def fit(stage, D2, y, th0, jitter, tol):
    path = []

    def f(th):
        v = nlml(stage, D2, y, th, jitter)
        path.append(v)
        return v
    r = minimize(f, np.asarray(th0, dtype=float), method='Nelder-Mead', options={'fatol': tol[0], 'xatol': tol[1]})
    return r.x, float(r.fun), path


def cases():
    P = np.load(os.path.join(ROOT, 'tests', 'golden', 'preds_d128.npz'))
    xm, ym = P['xm'], P['ym']
    D2 = ((xm[:, None, :] - xm[None, :, :]) ** 2).sum(-1)
    jit = np.arange(-20, -11, dtype=float)
    ins = [(j, jt) for j in range(128) for jt in jit]   # product(range(d), jitter, range(1)), models.py:186
    yield 'preds_d128 (m=15, d=128)', xm, D2, ym, ins, P['rnd'], (0.1, 0.1), P['fit_res']
    N = np.load(os.path.join(ROOT, 'tests', 'golden', 'nm.npz'))
    for tag in ('m10', 'm18tol3', 'm30'):
        xm, ym, ins, th0, tol, out = [N[tag + '__' + k] for k in ('xm', 'ym', 'ins', 'th0', 'tol', 'out')]
        D2 = ((xm[:, None, :] - xm[None, :, :]) ** 2).sum(-1)
        yield f'nm {tag} (m={xm.shape[0]}, d=3)', xm, D2, ym, [(int(j), jt) for j, jt in ins], th0, tuple(tol), out


def main():
    t0 = time.time()
    report = {}
    lim = int(os.environ.get('FIT_AGREEMENT_LIMIT', '0'))
    for name, xm, D2, ym, ins, th0, tol, ref in cases():
        assert np.array_equal(D2, O.d2_matrix(xm)), 'the oracle D2 is numpy pairwise order'
        if lim:
            ins = ins[:lim]
        n = len(ins)
        rows = {'fits': n, 'S0_reproduces_reference': 0, 'bitwise_equal_to_reference': 0,
                'fval_within_1e-6': 0, 'causes': {}, 'pass_fail': 0, 'oracle_is_S4': True}
        for q, (j, jt) in enumerate(ins):
            y = np.ascontiguousarray(ym[:, j])
            res = [fit(s, D2, y, th0[q], jt, tol) for s in range(5)]
            x0, f0, p0 = res[0]
            same_ref = np.array_equal(x0, ref[q, :2]) and (f0 == ref[q, 2] or (np.isinf(f0) and np.isinf(ref[q, 2])))
            rows['S0_reproduces_reference'] += bool(same_ref)
            x4, f4, p4 = res[4]
            if q % 97 == 0:   # S4 is the oracle: spot-check against orc_nm_fit
                th, fv, ne = O.nm_fit(D2, y, th0[q], jt, tol[0], tol[1])
                rows['oracle_is_S4'] &= bool(np.array_equal(th, x4) and (fv == f4 or (np.isinf(fv) and np.isinf(f4))))
            eq = np.array_equal(x4, ref[q, :2]) and (f4 == ref[q, 2] or (np.isinf(f4) and np.isinf(ref[q, 2])))
            rows['bitwise_equal_to_reference'] += bool(eq)
            rows['fval_within_1e-6'] += bool(abs(f4 - ref[q, 2]) <= 1e-6 * max(1.0, abs(ref[q, 2])) or
                                             (np.isinf(f4) and np.isinf(ref[q, 2])))
            if not eq:
                first = next(s for s in range(1, 5) if not (np.array_equal(res[s][0], x0) and
                                                            (res[s][1] == f0 or (np.isinf(res[s][1]) and np.isinf(f0)))))
                c = CAUSE[first]
                rows['causes'][c] = rows['causes'].get(c, 0) + 1
                pa, pb = res[first - 1][2], res[first][2]
                k = next((i for i in range(min(len(pa), len(pb))) if pa[i] != pb[i]), None)
                if k is not None and np.isinf(pa[k]) != np.isinf(pb[k]):
                    rows['pass_fail'] += 1
        report[name] = rows
        print(name, json.dumps(rows), f'({time.time() - t0:.0f} s)', flush=True)
    if len(sys.argv) > 2 and sys.argv[1] == '--json':
        with open(sys.argv[2], 'w') as f:
            json.dump(report, f, indent=1)


if __name__ == '__main__':
    main()
