"""Cell pieces (binary64 interior C_D/C_L) checked on the host, no GPU: the records
libpdenv builds (pd_cell_piece_info) against an independent numpy restatement of the thin-plate
interpolant of scipy's RBFInterpolator(neighbors=50, kernel='thin_plate_spline', degree=1)
(aerodynamic_coefficients.py:57-66): the 50 nearest table points of the cell centre, the
[[K, P], [P^T, 0]] solve with scipy's shift/scale of the polynomial part, and the sum of all 50
terms in long double at random points of the cell whose 50-NN set is the centre's."""
import ctypes as C
import math

import numpy as np
import pytest

LD = np.longdouble


@pytest.fixture(scope="module")
def lib_params():
    from pdenv import _lib, params
    return _lib.load(), params.Params()


def _table(pk, name):
    t = pk[name]
    m = np.array(t["mach"], dtype=float)
    a = np.zeros_like(m)
    for col in t["cols"]:
        a[col["start"]:col["start"] + col["len"]] = col["aoa"]
    return np.stack([m, a], 1), np.array(t["coef"], dtype=float)


def _solve(Y, f):
    n = len(Y)
    r2 = ((Y[:, None, :] - Y[None, :, :]) ** 2).sum(-1)
    K = np.where(r2 > 0, 0.5 * r2 * np.log(np.where(r2 > 0, r2, 1.0)), 0.0)
    lo, hi = Y.min(0), Y.max(0)
    shift, scale = (hi + lo) / 2, (hi - lo) / 2
    scale[scale == 0] = 1.0
    P = np.hstack([np.ones((n, 1)), (Y - shift) / scale])
    A = np.zeros((n + 3, n + 3))
    A[:n, :n], A[:n, n:], A[n:, :n] = K, P, P.T
    sol = np.linalg.solve(A, np.concatenate([f, np.zeros(3)]))
    return sol[:n], sol[n:], shift, scale


def _info(L, P, tb, piece=-1):
    out = (C.c_double * (16 + 64))()
    assert L.pd_cell_piece_info(C.byref(P.struct), tb, piece, out, 80) == 0
    return np.array(out[:])


def _eval_piece(rec, deg, nex, M, A, u, v):
    """The device's order (pd_step_impl.h cell_eval), numpy log for the exact terms."""
    f, q = 0.0, 0
    for i in range(deg, -1, -1):
        qi = rec[q]
        q += 1
        for _ in range(deg - i):
            qi = math.fma(qi, v, rec[q]) if hasattr(math, "fma") else qi * v + rec[q]
            q += 1
        f = qi if i == deg else (math.fma(f, u, qi) if hasattr(math, "fma") else f * u + qi)
    ncoef = (deg + 1) * (deg + 2) // 2
    for e in range(nex):
        m, c8, a = rec[ncoef + 3 * e:ncoef + 3 * e + 3]
        d2 = (M - m) ** 2 + (A - a) ** 2
        if d2 > 0:
            f += c8 * d2 * 4.0 * math.log(d2)
    return f


@pytest.mark.parametrize("tb,name", [(0, "aero_cd"), (1, "aero_cl")])
def test_cell_pieces_vs_numpy_restatement(lib_params, tb, name):
    from pdenv.params import load_pack
    L, P = lib_params
    info = _info(L, P, tb)
    pieces, rejected, max_rel = info[0], info[1], info[2]
    nm, na, a0, a1, deg, nex, stride = int(info[5]), int(info[6]), info[7], info[8], int(info[9]), int(info[10]), int(info[11])
    assert (deg, nex, stride) == (8, 4, 58)
    assert pieces > nm * na * 0.8 and rejected <= 0.001 * pieces
    assert max_rel <= 1e-15          # the build's own check (kCellTol 1e-14 rejects)
    Y, coef = _table(load_pack(), name)
    dm, da = 10.0 / nm, (a1 - a0) / na
    rng = np.random.default_rng(7 + tb)
    errs = []
    for _ in range(24):
        im, ia = int(rng.integers(0, int(5.5 / dm))), int(rng.integers(0, na))
        rec = _info(L, P, tb, im * na + ia)[16:16 + stride]
        if not rec.any():
            continue                 # a refined cell: its pieces are reached through its sub-cells
        cm, ca = (im + 0.5) * dm, a0 + (ia + 0.5) * da
        nn = np.argsort(np.sqrt(((Y - [cm, ca]) ** 2).sum(1)), kind="stable")[:50]
        cf, p, sh, sc = _solve(Y[nn], coef[nn])
        for _ in range(12):
            u, v = rng.random() * 2 - 1, rng.random() * 2 - 1
            M, A = cm + u * dm / 2, ca + v * da / 2
            dq = np.sqrt(((Y - [M, A]) ** 2).sum(1))
            if set(np.argsort(dq, kind="stable")[:50]) != set(nn):
                continue
            f = _eval_piece(rec, deg, nex, M, A, u, v)
            r2 = ((np.array([M, A], dtype=LD) - Y[nn].astype(LD)) ** 2).sum(1)
            ph = np.where(r2 > 0, LD(0.5) * cf.astype(LD) * r2 * np.log(np.where(r2 > 0, r2, LD(1))), LD(0))
            ex = ph.sum() + LD(p[0]) + (LD(M) - LD(sh[0])) / LD(sc[0]) * LD(p[1]) + (LD(A) - LD(sh[1])) / LD(sc[1]) * LD(p[2])
            errs.append(float(abs(LD(f) - ex) / (np.abs(ph).sum() + abs(ex))))
    assert len(errs) >= 100
    # the same class as the binary64 direct sum's rounding (and the scipy solve's, which differs
    # from the library's LU in the last bits of the coefficients)
    assert max(errs) <= 2e-15, max(errs)


@pytest.mark.parametrize("tb", [0, 1])
def test_cell_pieces_binary32(lib_params, tb):
    """The binary32 handle's pieces (ensure_f32): every binary64-valid piece rounded to floats and
    evaluated as the binary32 kernel does (fmaf Horner, hardware log2 for the exact terms) at its
    check points; the ones within 2e-6 of sum |c_j phi_j| + |s| are used.  Nearly all pass, so the
    binary32 handle's interior queries take pieces (not the payload sums) almost everywhere."""
    L, P = lib_params
    info = _info(L, P, tb)
    pieces, rejected32, max32, ok64, ok32 = info[0], info[12], info[13], info[14], info[15]
    assert 0 < max32 <= 2e-6
    assert rejected32 <= 0.01 * pieces, (rejected32, pieces)
    assert ok32 >= 0.99 * ok64, (ok32, ok64)
