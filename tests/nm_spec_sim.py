"""Rounds per Nelder-Mead fit under speculation schemes, on the oracle's -LML (test infrastructure:
a Python copy of the state machine of csrc/nngp_nm.h, scipy's rules, and of the kernels' candidate
sets).  Scheme '1' = one level (nm_spec_kernel), 'X2' = two levels with the next iteration's four
candidates for reflection-accepted / inside-contraction-best / -worst (nm_spec2_kernel, W = 4),
'H1' = reflection-accepted only (W = 2).  Run from the repository root: python tests/nm_spec_sim.py
(DESIGN.md §3.3 quotes its output)."""
import sys, math
import numpy as np
import os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'oracle')); sys.path.insert(0, ROOT)
import oracle as O
INIT0, INIT1, INIT2, REFLECT, EXPAND, CONTRACT, ICONTRACT, SHRINK1, SHRINK2, DONE = range(10)
INF = float('inf')

def less(a, b): return a < b or (b != b and a == a)

class NM:
    def __init__(s, t0x, t0y, fatol, xatol, maxf=400):
        s.fatol, s.xatol, s.maxf = fatol, xatol, maxf
        s.s0x, s.s0y = t0x, t0y
        s.s1x = (1 + 0.05) * t0x if t0x != 0 else 0.00025; s.s1y = t0y
        s.s2x = t0x; s.s2y = (1 + 0.05) * t0y if t0y != 0 else 0.00025
        s.f0 = s.f1 = s.f2 = INF; s.xbx = s.xby = s.xrx = s.xry = s.fxr = 0.0
        s.fcalls = 0; s.iters = 0; s.st = INIT0
        if not s.req(s.s0x, s.s0y, INIT0): s.st = DONE
    def copy(s):
        n = NM.__new__(NM); n.__dict__ = dict(s.__dict__); return n
    def req(s, x, y, st):
        if s.fcalls >= s.maxf: return False
        s.fcalls += 1; s.px, s.py, s.st = x, y, st; return True
    def sort(s):
        if less(s.f1, s.f0):
            s.f0, s.f1 = s.f1, s.f0; s.s0x, s.s1x = s.s1x, s.s0x; s.s0y, s.s1y = s.s1y, s.s0y
        if less(s.f2, s.f1):
            f, x, y = s.f2, s.s2x, s.s2y
            s.f2, s.s2x, s.s2y = s.f1, s.s1x, s.s1y
            if less(f, s.f0):
                s.f1, s.s1x, s.s1y = s.f0, s.s0x, s.s0y; s.f0, s.s0x, s.s0y = f, x, y
            else:
                s.f1, s.s1x, s.s1y = f, x, y
    def check(s):
        if not (s.fcalls < s.maxf and s.iters < s.maxf): s.st = DONE; return
        xok = abs(s.s1x - s.s0x) <= s.xatol and abs(s.s1y - s.s0y) <= s.xatol and abs(s.s2x - s.s0x) <= s.xatol and abs(s.s2y - s.s0y) <= s.xatol
        fok = abs(s.f0 - s.f1) <= s.fatol and abs(s.f0 - s.f2) <= s.fatol
        if xok and fok: s.st = DONE; return
        s.xbx = (s.s0x + s.s1x) / 2; s.xby = (s.s0y + s.s1y) / 2
        s.xrx = 2 * s.xbx - 1 * s.s2x; s.xry = 2 * s.xby - 1 * s.s2y
        if not s.req(s.xrx, s.xry, REFLECT): s.sort(); s.st = DONE
    def abort(s): s.sort(); s.check()
    def end_iter(s): s.iters += 1; s.sort(); s.check()
    def shrink_start(s):
        s.s1x = s.s0x + 0.5 * (s.s1x - s.s0x); s.s1y = s.s0y + 0.5 * (s.s1y - s.s0y)
        if not s.req(s.s1x, s.s1y, SHRINK1): s.abort()
    def consume(s, f):
        st = s.st
        if st == INIT0:
            s.f0 = f
            if not s.req(s.s1x, s.s1y, INIT1): s.sort(); s.st = DONE
        elif st == INIT1:
            s.f1 = f
            if not s.req(s.s2x, s.s2y, INIT2): s.sort(); s.st = DONE
        elif st == INIT2:
            s.f2 = f; s.sort(); s.iters = 1; s.check()
        elif st == REFLECT:
            s.fxr = f
            if f < s.f0:
                if not s.req(3 * s.xbx - 2 * s.s2x, 3 * s.xby - 2 * s.s2y, EXPAND): s.abort()
            elif f < s.f1:
                s.s2x, s.s2y, s.f2 = s.xrx, s.xry, f; s.end_iter()
            elif f < s.f2:
                if not s.req(1.5 * s.xbx - 0.5 * s.s2x, 1.5 * s.xby - 0.5 * s.s2y, CONTRACT): s.abort()
            else:
                if not s.req(0.5 * s.xbx + 0.5 * s.s2x, 0.5 * s.xby + 0.5 * s.s2y, ICONTRACT): s.abort()
        elif st == EXPAND:
            if f < s.fxr: s.s2x, s.s2y, s.f2 = s.px, s.py, f
            else: s.s2x, s.s2y, s.f2 = s.xrx, s.xry, s.fxr
            s.end_iter()
        elif st == CONTRACT:
            if f <= s.fxr: s.s2x, s.s2y, s.f2 = s.px, s.py, f; s.end_iter()
            else: s.shrink_start()
        elif st == ICONTRACT:
            if f < s.f2: s.s2x, s.s2y, s.f2 = s.px, s.py, f; s.end_iter()
            else: s.shrink_start()
        elif st == SHRINK1:
            s.f1 = f; s.s2x = s.s0x + 0.5 * (s.s2x - s.s0x); s.s2y = s.s0y + 0.5 * (s.s2y - s.s0y)
            if not s.req(s.s2x, s.s2y, SHRINK2): s.abort()
        elif st == SHRINK2:
            s.f2 = f; s.end_iter()

def level1(S):
    c = [(S.st, S.px, S.py)]
    if S.st == INIT0: return c + [(INIT1, S.s1x, S.s1y), (INIT2, S.s2x, S.s2y)]
    if S.st == REFLECT:
        if S.f0 == INF and S.f1 == INF and S.f2 == INF:
            return c + [(ICONTRACT, 0.5 * S.xbx + 0.5 * S.s2x, 0.5 * S.xby + 0.5 * S.s2y),
                        (SHRINK1, S.s0x + 0.5 * (S.s1x - S.s0x), S.s0y + 0.5 * (S.s1y - S.s0y)),
                        (SHRINK2, S.s0x + 0.5 * (S.s2x - S.s0x), S.s0y + 0.5 * (S.s2y - S.s0y))]
        return c + [(EXPAND, 3 * S.xbx - 2 * S.s2x, 3 * S.xby - 2 * S.s2y),
                    (CONTRACT, 1.5 * S.xbx - 0.5 * S.s2x, 1.5 * S.xby - 0.5 * S.s2y),
                    (ICONTRACT, 0.5 * S.xbx + 0.5 * S.s2x, 0.5 * S.xby + 0.5 * S.s2y)]
    if S.st == SHRINK1: return c + [(SHRINK2, S.s0x + 0.5 * (S.s2x - S.s0x), S.s0y + 0.5 * (S.s2y - S.s0y))]
    return c

def next_reflect(S, px, py, rank, full):
    """the next iteration's candidates if (px,py) replaces s2 and lands at rank 0/1/2 (no convergence)"""
    v = [(S.s0x, S.s0y), (S.s1x, S.s1y)]
    v.insert(rank, (px, py))
    (a, b), (c, d), (e, f) = v
    xbx = (a + c) / 2; xby = (b + d) / 2
    out = [(REFLECT, 2 * xbx - 1 * e, 2 * xby - 1 * f)]
    if full:
        out += [(EXPAND, 3 * xbx - 2 * e, 3 * xby - 2 * f), (CONTRACT, 1.5 * xbx - 0.5 * e, 1.5 * xby - 0.5 * f),
                (ICONTRACT, 0.5 * xbx + 0.5 * e, 0.5 * xby + 0.5 * f)]
    return out

def level2(S, scheme):
    c = level1(S)
    if S.st != REFLECT or (S.f0 == INF and S.f1 == INF and S.f2 == INF): return c
    xr, yr = S.xrx, S.xry
    xe, ye = 3 * S.xbx - 2 * S.s2x, 3 * S.xby - 2 * S.s2y
    xo, yo = 1.5 * S.xbx - 0.5 * S.s2x, 1.5 * S.xby - 0.5 * S.s2y
    xi, yi = 0.5 * S.xbx + 0.5 * S.s2x, 0.5 * S.xby + 0.5 * S.s2y
    if scheme == 'X':   # full next iteration for expansion(e), expansion(r), reflection
        c += next_reflect(S, xe, ye, 0, True) + next_reflect(S, xr, yr, 0, True) + next_reflect(S, xr, yr, 1, True)
    elif scheme == 'Y':   # next reflection for every single-point outcome; expansions for A/B
        for (x, y, ranks) in ((xe, ye, [0]), (xr, yr, [0, 1]), (xo, yo, [0, 1, 2]), (xi, yi, [0, 1, 2])):
            for r in ranks: c += next_reflect(S, x, y, r, False)
        c += [t for t in next_reflect(S, xr, yr, 1, True)[1:2]]   # e' for the accepted reflection
    elif scheme in ('X2', 'X3', 'X4', 'H1', 'H2', 'H3'):
        sets = {'X2': [(xr, yr, 1), (xi, yi, 0), (xi, yi, 2)], 'X3': [(xr, yr, 1), (xi, yi, 0), (xe, ye, 0)],
                'X4': [(xr, yr, 1), (xi, yi, 0), (xi, yi, 2), (xe, ye, 0)],
                'H1': [(xr, yr, 1)], 'H2': [(xi, yi, 0)], 'H3': [(xi, yi, 2)]}[scheme]
        for x, y, r in sets: c += next_reflect(S, x, y, r, True)
    elif scheme == 'W8':   # 8 rows: level 1 + r' for e/r-best/r-mid + ic-rank... (2 waves)
        c += next_reflect(S, xe, ye, 0, False) + next_reflect(S, xr, yr, 0, False) + next_reflect(S, xr, yr, 1, False)
        c += next_reflect(S, xi, yi, 2, False)
    return c

def run(obj, t0, scheme, fatol=0.1, xatol=0.1):
    S = NM(t0[0], t0[1], fatol, xatol)
    rounds = 0
    while S.st != DONE:
        cands = level1(S) if scheme == '1' else level2(S, scheme)
        rounds += 1
        cs = set(cands)
        n = 0
        while S.st != DONE and (S.st, S.px, S.py) in cs:
            S.consume(obj(S.px, S.py)); n += 1
        assert n > 0
    return rounds, S.fcalls, len(cands)

def rounds_table():
  rng = np.random.default_rng(0)
  for d, m, R, rows in ((3, 15, 2, 600), (3, 10, 1, 600), (128, 15, 1, 1200), (800, 20, 1, 4000)):
      base = rng.uniform(-0.5, 0.5, size=d)
      X = base + np.cumsum(0.02 * rng.standard_normal((rows, d)), axis=0)
      Y = 0.01 * np.sin(3 * X) + 1e-5 * rng.standard_normal((rows, d))
      q = X[rows // 2] + 0.005
      idx, _ = O.knn(X, q, m)
      D2 = O.d2_matrix(X[idx])
      th0 = rng.integers(-8, 0, (d * 9 * R, 2)).astype(float)
      res = {k: [] for k in ('1', 'H1', 'H2', 'H3', 'X2')}
      f = 0
      coords = range(d) if d <= 3 else rng.choice(d, 6, replace=False)
      for c in coords:
          y = Y[idx, c].copy()
          for ji, je in enumerate(O.JITTERS):
              for r in range(R):
                  t0 = th0[(c * 9 + ji) * R + r]
                  cache = {}
                  def obj(x, yy, je=je):
                      k = (x, yy)
                      if k not in cache: cache[k] = O.nlml(D2, y, (x, yy), je)
                      return cache[k]
                  for k in res: res[k].append(run(obj, t0, k))
      for k, v in res.items():
          rr = np.array([a for a, b, c in v]); nf = np.array([b for a, b, c in v])
          print(f'd={d} m={m} scheme {k:2s}: rounds mean {rr.mean():6.1f} max {rr.max():4d}  nfev mean {nf.mean():5.1f} max {nf.max()}  cands<= {max(c for a,b,c in v)}')



def outcome_stats():
    """frequencies of a finite-simplex reflection iteration's outcomes (A: expansion tried, e or r
    kept; B: reflection accepted; C/D: outside / inside contraction accepted at rank 0/1/2, or
    shrink)"""
    import collections
    stats = collections.Counter()
    rng = np.random.default_rng(1)
    for d, m, rows in ((3, 15, 600), (800, 20, 4000)):
        base = rng.uniform(-0.5, 0.5, size=d)
        X = base + np.cumsum(0.02 * rng.standard_normal((rows, d)), axis=0)
        Y = 0.01 * np.sin(3 * X) + 1e-5 * rng.standard_normal((rows, d))
        idx, _ = O.knn(X, X[rows // 2] + 0.005, m)
        D2 = O.d2_matrix(X[idx])
        for c in (range(d) if d <= 3 else rng.choice(d, 6, replace=False)):
            y = Y[idx, c].copy()
            for je in O.JITTERS:
                obj = lambda x, yy, je=je: O.nlml(D2, y, (x, yy), je)
                t0 = rng.integers(-8, 0, 2).astype(float)
                S = NM(t0[0], t0[1], 0.1, 0.1)
                while S.st != DONE:
                    if S.st == REFLECT and not (S.f0 == INF and S.f1 == INF and S.f2 == INF):
                        fr = obj(S.xrx, S.xry)
                        if fr < S.f0:
                            stats['A_e' if obj(3 * S.xbx - 2 * S.s2x, 3 * S.xby - 2 * S.s2y) < fr else 'A_r'] += 1
                        elif fr < S.f1:
                            stats['B'] += 1
                        else:
                            tag, (px, py) = ('C', (1.5 * S.xbx - 0.5 * S.s2x, 1.5 * S.xby - 0.5 * S.s2y)) if fr < S.f2 \
                                else ('D', (0.5 * S.xbx + 0.5 * S.s2x, 0.5 * S.xby + 0.5 * S.s2y))
                            fp = obj(px, py)
                            ok = fp <= fr if tag == 'C' else fp < S.f2
                            stats[tag + (str(0 if fp < S.f0 else (1 if fp < S.f1 else 2)) if ok else '_shrink')] += 1
                    S.consume(obj(S.px, S.py))
        tot = sum(stats.values())
        print(d, {k: round(v / tot, 3) for k, v in sorted(stats.items())})
        stats.clear()


if len(sys.argv) > 1 and sys.argv[1] == '--stats':
    outcome_stats()
else:
    rounds_table()
