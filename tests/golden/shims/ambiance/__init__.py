"""Test-only stand-in for the third-party `ambiance` package (not installed here).

Used ONLY by tests/golden/make_golden.py when it imports the reference to generate
fixtures.  Restates ambiance's published ISA / US-1976 layer model (geopotential
altitude, 9-layer base table, lapse-rate / isothermal pressure laws).  Pinned by the
air_density / atmospheric_pressure / speed_of_sound columns the reference itself
recorded (tests/test_oracle_golden.py).
"""
import numpy as np

_G0, _R, _KAPPA, _RE = 9.80665, 287.05287, 1.4, 6356766.0
_LAYERS = np.array([
    [-5.00e3, 320.65, -6.5e-3, 1.77687e5],
    [0.0, 288.15, -6.5e-3, 1.01325e5],
    [11.0e3, 216.65, 0.0, 2.26320e4],
    [20.0e3, 216.65, 1.0e-3, 5.47487e3],
    [32.0e3, 228.65, 2.8e-3, 8.68014e2],
    [47.0e3, 270.65, 0.0, 1.10906e2],
    [51.0e3, 270.65, -2.8e-3, 6.69384e1],
    [71.0e3, 214.65, -2.0e-3, 3.95639e0],
    [80.0e3, 196.65, -2.0e-3, 8.86272e-1]])


class Atmosphere:
    def __init__(self, h):
        h = np.atleast_1d(np.asarray(h, dtype=float))
        H = _RE * h / (_RE + h)
        i = np.clip(np.searchsorted(_LAYERS[:, 0], H, side="right") - 1, 0, len(_LAYERS) - 1)
        Hb, Tb, b, pb = _LAYERS[i].T
        T = Tb + b * (H - Hb)
        with np.errstate(divide="ignore", invalid="ignore"):
            p = np.where(b != 0, pb * (1 + b / Tb * (H - Hb)) ** (-_G0 / (b * _R)),
                         pb * np.exp(-_G0 / (_R * T) * (H - Hb)))
        self.temperature = T
        self.pressure = p
        self.density = p / (_R * T)
        self.speed_of_sound = np.sqrt(_KAPPA * _R * T)
