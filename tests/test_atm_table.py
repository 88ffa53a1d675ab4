"""The step kernel's tabulated ISA atmosphere, checked on the host, no GPU:
pd_atm_table builds the table as pd_create does and evaluates it in the device's order and
precision; it must equal the oracle's closed form (oracle/pd_oracle.c orc_atmosphere, the ISA of
atmosphere_dynamics.py:5-27) to binary64 rounding -- over the whole altitude range, densely
around every layer boundary (where the tabulated pb make p jump by ~4e-6: the table takes the
exact path's side) and every cell edge."""
import ctypes as C

import numpy as np
import pytest


@pytest.fixture(scope="module")
def lib_params():
    from pdenv import _lib, params
    return _lib.load(), params.Params()


def _table(L, P, prec, alt):
    alt = np.ascontiguousarray(alt, dtype=np.float64)
    atm = np.zeros((len(alt), 3))
    err = np.zeros(1)
    ptr = lambda a: a.ctypes.data_as(C.c_void_p)
    assert L.pd_atm_table(C.byref(P.struct), prec, ptr(alt), len(alt), ptr(atm), ptr(err)) == 0
    return atm, float(err[0])


def _boundaries(P):
    r = P.struct.isa_r
    hb = np.array(P.struct.isa_Hb[:])
    yb = r * hb[hb > 0] / (r - hb[hb > 0])
    return yb[yb < P.struct.isa_alt_max]


def _altitudes(P):
    top = P.struct.isa_alt_max
    rng = np.random.default_rng(3)
    pts = [np.linspace(0.0, top * (1 - 1e-12), 40001), rng.uniform(0, top, 40000),
           (_boundaries(P)[:, None] + np.linspace(-2.0, 2.0, 81)[None, :]).ravel(),
           (np.arange(1, int(top / 100)) * 100.0)[:, None] + np.array([-1e-6, 0.0, 1e-6])[None, :]]
    a = np.concatenate([p.ravel() for p in pts])
    return a[(a >= 0) & (a < top)]


def _oracle(alt):
    import oracle
    ol, op = oracle.lib(), C.byref(oracle.params())
    ref = np.zeros((len(alt), 3))
    r, p, a = C.c_double(), C.c_double(), C.c_double()
    for i, y in enumerate(alt):
        ol.orc_atmosphere(op, float(y), C.byref(r), C.byref(p), C.byref(a))
        ref[i] = (r.value, p.value, a.value)
    return ref


def test_atmosphere_table_binary64(lib_params):
    L, P = lib_params
    alt = _altitudes(P)
    atm, err = _table(L, P, 0, alt)
    assert err <= 5e-15, err        # the builder's check against the long double closed form
    ref = _oracle(alt)
    rel = np.abs(atm - ref) / np.abs(ref)
    # the oracle's closed form rounds 1 + b/Tb dH once and raises it to an exponent of about 34
    # (pow): up to 5e-15 from the exact function above 20 km; the table is within 2e-15 of it
    assert rel.max() <= 1e-14, (rel.max(0), alt[rel.max(1).argmax()])
    assert np.median(rel) <= 1e-15


def test_atmosphere_table_binary32(lib_params):
    L, P = lib_params
    alt = _altitudes(P)[::7]
    # (binary32 H rounds by millimetres: within 5 cm of a layer boundary the binary32 handle's
    # layer, exact path or table, may differ from the binary64 oracle's -- across the pb jump)
    alt = alt[np.abs(alt[:, None] - _boundaries(P)[None, :]).min(1) > 0.05]
    atm, err = _table(L, P, 1, alt)
    assert err <= 4e-6, err          # (binary32 y rounds by 8 mm at 80 km: 1e-6 of p)
    ref = _oracle(alt.astype(np.float32).astype(np.float64))
    assert (np.abs(atm - ref) / np.abs(ref)).max() <= 5e-6
