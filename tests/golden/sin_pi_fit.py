"""How the coefficients of nn_sin_pi (csrc/nngp_math.h, oracle/nngp_oracle.c) were computed: a
weighted minimax fit (Lawson's iteratively reweighted least squares, mpmath at 60 digits) of
P(z) = (sin(sqrt z)/sqrt z - 1)/z on [0, (pi/2)^2], weighted by the relative error it causes in
sin(r) = r + r z P(z).  The 8-coefficient fit's weighted error is 2.8e-19 (the 9-coefficient one's
4e-22).  Prints the coefficients as hex doubles.  Not run by the tests."""
import mpmath as mp
mp.mp.dps = 60
Z = (mp.pi/2)**2
def g(z):
    if z == 0: return mp.mpf(-1)/6
    r = mp.sqrt(z)
    return (mp.sin(r)/r - 1)/z
def fit(ncoef, iters=30, npts=400):
    # Lawson IRLS for weighted minimax of P(z) - g(z), weight = z*sqrt(z)/sin(sqrt(z)) (relative error of sin)
    pts = [Z*(1-mp.cos(mp.pi*(i+0.5)/npts))/2 for i in range(npts)]
    w = [ (z*mp.sqrt(z)/mp.sin(mp.sqrt(z))) if z>0 else mp.mpf(0) for z in pts]
    gv = [g(z) for z in pts]
    lw = [mp.mpf(1)]*npts
    for it in range(iters):
        A = mp.matrix(ncoef, ncoef); b = mp.matrix(ncoef,1)
        for z, ww, gg, l in zip(pts, w, gv, lw):
            W = l*(ww**2 + mp.mpf('1e-40'))
            powz = [z**k for k in range(ncoef)]
            for i in range(ncoef):
                b[i] += W*powz[i]*gg
                for j in range(ncoef):
                    A[i,j] += W*powz[i]*powz[j]
        c = mp.lu_solve(A, b)
        err = [abs(sum(c[k]*z**k for k in range(ncoef)) - gg)*ww for z, ww, gg in zip(pts, w, gv)]
        e = max(err)
        s = sum(l*er for l, er in zip(lw, err))
        lw = [l*er/s for l, er in zip(lw, err)]
        lw = [max(l, mp.mpf('1e-30')) for l in lw]
    return [c[k] for k in range(ncoef)], e
for n in (8, 9):
    c, e = fit(n)
    print(n, mp.nstr(e, 5))
    for k, v in enumerate(c):
        print(f'  S{k+1} = {float(v).hex()}  # {mp.nstr(v, 20)}')
