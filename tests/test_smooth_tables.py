"""The step kernel's tabulated smooth functions, checked on the host, no GPU:
pd_smooth_tables builds the tables as pd_create does and evaluates them in the device's order
and precision; they must equal the oracle's closed forms (oracle/pd_oracle.c orc_atmosphere,
the ISA of atmosphere_dynamics.py:5-27, and orc_inertia, the stage_inertia closure of
rocket_dimensions.py:167-196) to binary64 rounding -- over the whole altitude range, densely
around every layer boundary and cell edge, and over the whole fill range."""
import ctypes as C

import numpy as np
import pytest


@pytest.fixture(scope="module")
def lib_params():
    from pdenv import _lib, params
    return _lib.load(), params.Params()


def _tables(L, P, prec, alt, fill):
    alt = np.ascontiguousarray(alt, dtype=np.float64)
    fill = np.ascontiguousarray(fill, dtype=np.float64)
    atm = np.zeros((len(alt), 3))
    inr = np.zeros((len(fill), 2))
    err = np.zeros(2)
    ptr = lambda a: a.ctypes.data_as(C.c_void_p)
    assert L.pd_smooth_tables(C.byref(P.struct), prec, ptr(alt), len(alt), ptr(atm), ptr(fill), len(fill), ptr(inr),
                              ptr(err)) == 0
    return atm, inr, err


def _altitudes(P):
    r, top = P.struct.isa_r, P.struct.isa_alt_max
    hb = np.array(P.struct.isa_Hb[:])
    yb = r * hb[(hb > 0)] / (r - hb[(hb > 0)])            # layer boundaries in geometric altitude
    yb = yb[yb < top]
    rng = np.random.default_rng(3)
    pts = [np.linspace(0.0, top * (1 - 1e-12), 40001), rng.uniform(0, top, 40000),
           (yb[:, None] + np.linspace(-2.0, 2.0, 81)[None, :]).ravel(),
           (np.arange(1, int(top / 100)) * 100.0)[:, None] + np.array([-1e-6, 0.0, 1e-6])[None, :]]
    a = np.concatenate([p.ravel() for p in pts])
    return a[(a >= 0) & (a < top)]


def test_atmosphere_and_inertia_tables_binary64(lib_params):
    import oracle
    L, P = lib_params
    alt = _altitudes(P)
    fill = np.concatenate([np.linspace(1e-4, 1.0, 20001), np.random.default_rng(4).uniform(1e-6, 1.0, 20000),
                           [1.0 - 1e-6, 1.0]])
    atm, inr, err = _tables(L, P, 0, alt, fill)
    # the builders' own check against the long double closed forms (2e-16 typical)
    assert err[0] <= 5e-15 and err[1] <= 1e-15, err
    ol = oracle.lib()
    op = C.byref(oracle.params())
    ref = np.zeros_like(atm)
    r, p, a = C.c_double(), C.c_double(), C.c_double()
    for i, y in enumerate(alt):
        ol.orc_atmosphere(op, float(y), C.byref(r), C.byref(p), C.byref(a))
        ref[i] = (r.value, p.value, a.value)
    rel = np.abs(atm - ref) / np.abs(ref)
    # the oracle's closed form rounds 1 + b/Tb dH once and raises it to an exponent of about 34
    # (pow): up to 5e-15 from the exact function above 20 km; the table is within 2e-15 of it
    assert rel.max() <= 1e-14, (rel.max(0), alt[rel.max(1).argmax()])
    assert np.median(rel) <= 1e-15
    refi = np.zeros_like(inr)
    xc, ii = C.c_double(), C.c_double()
    for i, f in enumerate(fill):
        ol.orc_inertia(op, float(f), C.byref(xc), C.byref(ii))
        refi[i] = (xc.value, ii.value)
    reli = np.abs(inr - refi) / np.abs(refi)
    assert reli.max() <= 1e-15, (reli.max(0), fill[reli.max(1).argmax()])


def test_atmosphere_and_inertia_tables_binary32(lib_params):
    import oracle
    L, P = lib_params
    alt = _altitudes(P)[::7]
    # (binary32 H rounds by millimetres: within 5 cm of a layer boundary the binary32 handle's
    # layer, exact path or table, may differ from the binary64 oracle's -- across the pb jump)
    r = P.struct.isa_r
    hb = np.array(P.struct.isa_Hb[:])
    yb = r * hb[hb > 0] / (r - hb[hb > 0])
    alt = alt[np.abs(alt[:, None] - yb[None, :]).min(1) > 0.05]
    fill = np.linspace(1e-3, 1.0, 4001)
    atm, inr, err = _tables(L, P, 1, alt, fill)
    assert err[0] <= 4e-6 and err[1] <= 1e-6, err   # (binary32 y rounds by 8 mm at 80 km: 1e-6 of p)
    ol = oracle.lib()
    op = C.byref(oracle.params())
    r, p, a = C.c_double(), C.c_double(), C.c_double()
    worst = 0.0
    for i, y in enumerate(alt):
        ol.orc_atmosphere(op, float(np.float32(y)), C.byref(r), C.byref(p), C.byref(a))
        ref = np.array([r.value, p.value, a.value])
        worst = max(worst, float((np.abs(atm[i] - ref) / np.abs(ref)).max()))
    assert worst <= 5e-6, worst
