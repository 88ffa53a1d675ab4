#!/usr/bin/env python3
"""Build the frozen parameter pack for the MI355X powered-descent env.

Runs ONLY in the build container (it reads the reference's data files under
/root/reference/data, read-only).  Output: psso-sac-for-powered-descent_amd/data/param_pack.json,
which is plain data (numbers), committed, and is all the product needs at run time.

Every number is parsed exactly the way the reference parses it, so the
resulting IEEE doubles are bit-identical to the reference's:

* sizing constants: csv.reader + float()            (rockets_physics.py:714-719)
* initial state: pandas.read_csv, last row          (load_initial_states.py:236-242)
* normalisation: pandas.read_csv max(|.|)+c         (input_normalisation.py:73-89)
* V2 aero tables: line.split(',') + float()         (aerodynamic_coefficients.py:8-49)
* grid-fin tables: pandas.read_csv                  (grid_fin_aerodynamics.py:7-46)
* wind profile: float() + interp1d node recompute   (HorizontalWindSpeed.py:5-114)
* von Karman filter: scipy.signal.cont2discrete     (vonkarman.py:9-39)
* stage-2 inertia closure constants: read STATICALLY out of
  data/rocket_parameters/rocket_functions.pkl with pickletools (opcode
  disassembly; nothing in the file is executed or unpickled).  They are the
  cell contents of `x_cog_inertia_subrocket_2_lambda`
  (rocket_dimensions.py:158-197, wired at rockets_physics.py:942-944).

The RBF neighbourhood keys (which 50-point neighbourhoods the kNN search of
scipy's RBFInterpolator(neighbors=50) can select over the reachable query
domain, aerodynamic_coefficients.py:57-66) are enumerated here on a dense grid
plus exact 1-D sweeps; the device table is only a cache - a miss is solved
exactly on the GPU at run time.
"""
import csv
import json
import math
import os
import pickletools
import struct
import sys

import numpy as np

REF = os.environ.get("PDENV_REFERENCE", "/root/reference")
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                   "psso-sac-for-powered-descent_amd", "data", "param_pack.json")

N_NEIGHBORS = 50
KEY_BITS_LO = 6
KEY_BITS_LEN = 6


def ref_path(*p):
    return os.path.join(REF, *p)


def read_sizing():
    d = {}
    with open(ref_path("data/rocket_parameters/sizing_results.csv")) as f:
        for row in csv.reader(f):
            d[row[0]] = row[2]
    return d


def read_closure_constants():
    """Static scan of the dill pickle: the 8 float64 cells of the
    stage_inertia closure stored under x_cog_inertia_subrocket_2_lambda are
    written (dill `_setattr(cell, 'cell_contents', numpy scalar)`) in reverse
    alphabetical order of the free variables: x_dry, m_ox, m_f, m_dry, h_ox,
    h_lower, h_f, I_dry."""
    data = open(ref_path("data/rocket_parameters/rocket_functions.pkl"), "rb").read()
    ops = list(pickletools.genops(data))
    start = end = None
    for i, (op, arg, pos) in enumerate(ops):
        if op.name.endswith("UNICODE") and arg == "x_cog_inertia_subrocket_2_lambda":
            start = i
        if start is not None and op.name.endswith("UNICODE") and arg == "d_cg_thrusters_subrocket_0_lambda":
            end = i
            break
    vals = [struct.unpack("<d", arg)[0] for (op, arg, pos) in ops[start:end]
            if op.name in ("SHORT_BINBYTES", "BINBYTES") and len(arg) == 8]
    assert len(vals) == 8, vals
    names = ["x_dry", "m_ox", "m_f", "m_dry", "h_ox", "h_lower", "h_f", "I_dry"]
    out = dict(zip(names, vals))
    # engine_height (rocket_dimensions.py:268) and the descent CoP
    # cop_func(lengths[2], .., d_0=0.75) = 0.75 * stage_1_height (main_sizing.py:217,
    # cop_estimation.py:20-21).  lengths[2] is the stage-1 height.
    out["engine_height"] = 3.1
    return out


def read_aero(fname):
    """aerodynamic_coefficients.py:8-49 restated (same float() parsing)."""
    with open(ref_path(fname)) as f:
        lines = f.readlines()
    header = lines[0].strip().split(",")
    aoa_values = [float(v.split("_")[0]) for v in header if "deg" in v]
    data = {a: ([], []) for a in aoa_values}
    for line in lines[2:]:
        if not line.strip():
            continue
        values = line.strip().split(",")
        if len(values) < len(header):
            continue
        col = 0
        for a in aoa_values:
            mi, ci = col, col + 1
            if ci < len(values) and values[mi].strip() and values[ci].strip():
                try:
                    m = float(values[mi]); c = float(values[ci])
                    data[a][0].append(m); data[a][1].append(c)
                except ValueError:
                    pass
            col += 2
    mach, aoa, coef = [], [], []
    for a in aoa_values:
        mach += data[a][0]; coef += data[a][1]; aoa += [a] * len(data[a][0])
    return np.array(mach), np.array(aoa), np.array(coef), aoa_values


def rbf_table(fname):
    mach, aoa, coef, cols = read_aero(fname)
    n = len(mach)
    table = {"n_pts": n, "cols": []}
    # points regrouped per AoA column, sorted by Mach (stable) inside a column
    pts_mach, pts_coef, pts_orig = [], [], []
    for c, a in enumerate(cols):
        idx = np.nonzero(aoa == a)[0]
        order = idx[np.argsort(mach[idx], kind="stable")]
        assert len(order) < (1 << KEY_BITS_LO)
        table["cols"].append({"aoa": a, "start": len(pts_mach), "len": int(len(order))})
        pts_mach += mach[order].tolist(); pts_coef += coef[order].tolist(); pts_orig += order.tolist()
    table["mach"] = pts_mach
    table["coef"] = pts_coef
    table["orig_index"] = [int(i) for i in pts_orig]
    # sanity: no exact duplicate points inside a column
    for col in table["cols"]:
        ms = pts_mach[col["start"]:col["start"] + col["len"]]
        assert len(set(ms)) == len(ms), "duplicate Mach inside a column"
    return table


def knn_keys(table, M, A):
    """Neighbourhood key of the 50-NN set (squared euclidean distance in raw
    (Mach, AoA-deg) space, the metric of scipy's cKDTree) for many queries."""
    pm = np.array(table["mach"]); n = len(pm)
    pa = np.concatenate([[c["aoa"]] * c["len"] for c in table["cols"]])
    col_of = np.concatenate([[ci] * c["len"] for ci, c in enumerate(table["cols"])])
    starts = np.array([c["start"] for c in table["cols"]])
    keys = np.zeros(len(M), dtype=np.uint64)
    B = 20000
    for s in range(0, len(M), B):
        m = M[s:s + B, None]; a = A[s:s + B, None]
        d2 = (m - pm[None, :]) ** 2 + (a - pa[None, :]) ** 2
        sel = np.argpartition(d2, N_NEIGHBORS - 1, axis=1)[:, :N_NEIGHBORS]
        k = np.zeros(sel.shape[0], dtype=np.uint64)
        for ci, c in enumerate(table["cols"]):
            inc = (col_of[sel] == ci)
            cnt = inc.sum(axis=1)
            lo = np.where(inc, sel, n + 1).min(axis=1) - starts[ci]
            lo = np.where(cnt > 0, lo, 0)
            field = (lo.astype(np.uint64) | (cnt.astype(np.uint64) << np.uint64(KEY_BITS_LO)))
            k |= field << np.uint64((KEY_BITS_LO + KEY_BITS_LEN) * ci)
        keys[s:s + B] = k
    return keys


def sweep_line_keys(table, a, mlo=0.0, mhi=10.0):
    """Exact enumeration along the line AoA=a: the kNN set only changes where
    two points swap distance order; visit every interval between consecutive
    pair-bisector crossings."""
    pm = np.array(table["mach"])
    pa = np.concatenate([[c["aoa"]] * c["len"] for c in table["cols"]])
    dz = (a - pa) ** 2
    i, j = np.triu_indices(len(pm), 1)
    den = 2.0 * (pm[j] - pm[i])
    ok = den != 0
    x = (pm[j][ok] ** 2 - pm[i][ok] ** 2 + dz[j][ok] - dz[i][ok]) / den[ok]
    x = np.unique(x[(x > mlo) & (x < mhi)])
    bps = np.concatenate([[mlo], x, [mhi]])
    mids = np.concatenate([[mlo], 0.5 * (bps[:-1] + bps[1:]), [mhi]])
    return knn_keys(table, mids, np.full(len(mids), a))


def vsweep_line_keys(table, M, a_lo, a_hi):
    """Exact enumeration along the vertical line Mach=M, a in [a_lo, a_hi]: bisectors of
    points in different AoA columns cross it once; same-column pairs never swap along it."""
    pm = np.array(table["mach"])
    pa = np.concatenate([[c["aoa"]] * c["len"] for c in table["cols"]])
    dm2 = (M - pm) ** 2
    i, j = np.triu_indices(len(pm), 1)
    den = 2.0 * (pa[j] - pa[i])
    ok = den != 0
    x = (dm2[j][ok] - dm2[i][ok] + pa[j][ok] ** 2 - pa[i][ok] ** 2) / den[ok]
    x = np.unique(x[(x > a_lo) & (x < a_hi)])
    bps = np.concatenate([[a_lo], x, [a_hi]])
    mids = np.concatenate([[a_lo], 0.5 * (bps[:-1] + bps[1:]), [a_hi]])
    return knn_keys(table, np.full(len(mids), M), mids)


def enumerate_keys(table, a_lo, a_hi, n_lines, extra_lines, n_vlines=2001, n_random=2000000):
    keys = set()
    for a in list(np.linspace(a_lo, a_hi, n_lines)) + list(extra_lines):
        keys.update(int(k) for k in sweep_line_keys(table, float(a)))
    for M in np.linspace(0.0, 10.0, n_vlines):
        keys.update(int(k) for k in vsweep_line_keys(table, float(M), a_lo, a_hi))
    rng = np.random.default_rng(1)
    keys.update(int(k) for k in knn_keys(table, rng.uniform(0, 10, n_random), rng.uniform(a_lo, a_hi, n_random)))
    # dense 2-D grid on top (cheap insurance for slivers between lines)
    M = np.linspace(0.0, 10.0, 2001)
    Aq = np.linspace(a_lo, a_hi, 4 * n_lines + 1)
    MM, AA = np.meshgrid(M, Aq)
    keys.update(int(k) for k in knn_keys(table, MM.ravel(), AA.ravel()))
    return sorted(keys)


def grid_fin_tables():
    import pandas as pd
    cd = pd.read_csv(ref_path("data/rocket_parameters/GridFin/C_D_grid_fin.csv"), header=None)
    mach_cd = cd[0].values; ca = cd[1].values
    # interp1d(assume_sorted=False) sorts with argsort(kind='mergesort')
    o = np.argsort(mach_cd, kind="mergesort")
    ca_tab = {"x": mach_cd[o].tolist(), "y": ca[o].tolist(),
              "min_mach": float(np.min(mach_cd)), "min_val": float(ca[np.argmin(mach_cd)])}
    cn = pd.read_csv(ref_path("data/rocket_parameters/GridFin/C_N_alpha_grid_fin.csv"), skiprows=2, header=None)
    m = cn[0].values; v = cn[1].values
    o = np.argsort(m, kind="mergesort")
    srt = np.argsort(m)
    mx, smx = srt[-1], srt[-2]
    slope = (v[mx] - v[smx]) / (m[mx] - m[smx])
    cn_tab = {"x": m[o].tolist(), "y": v[o].tolist(), "min_mach": float(np.min(m)),
              "max_mach": float(np.max(m)), "min_val": float(v[np.argmin(m)]),
              "max_val": float(v[mx]), "slope": float(slope)}
    return ca_tab, cn_tab


def call_linear_nodes(x, y):
    """scipy interp1d._call_linear evaluated at its own (sorted) nodes."""
    o = np.argsort(x, kind="mergesort")
    xs, ys = x[o], y[o]
    idx = np.searchsorted(xs, xs).clip(1, len(xs) - 1)
    lo, hi = idx - 1, idx
    slope = (ys[hi] - ys[lo]) / (xs[hi] - xs[lo])
    return xs, slope * (xs - xs[lo]) + ys[lo]


def wind_profiles():
    """HorizontalWindSpeed.py:5-114 for integer percentiles 50..99 (the
    drivers pass an int; WindModel draws float(randint(50, 99)))."""
    with open(ref_path("data/Wind/horizontal_wind.csv")) as f:
        lines = f.readlines()
    percs = [it for it in lines[0].strip().split(",") if it and not it.isspace()]
    wd = {p: ([], []) for p in percs}
    for line in lines[2:]:
        if not line.strip():
            continue
        values = line.strip().split(",")
        if len(values) < len(percs) * 2:
            continue
        for i, p in enumerate(percs):
            try:
                ws = float(values[2 * i]); alt = float(values[2 * i + 1])
                wd[p][0].append(ws); wd[p][1].append(alt)
            except (ValueError, IndexError):
                pass
    pvals = [float(p.split("_")[0]) for p in percs]
    profiles = []
    for req in range(50, 100):
        req_v = float(req)
        idx = int(np.searchsorted(pvals, req_v))
        if idx == 0:
            lo_p = up_p = percs[0]; w = 1.0
        elif idx == len(pvals):
            lo_p = up_p = percs[-1]; w = 0.0
        else:
            lo_p, up_p = percs[idx - 1], percs[idx]
            w = (req_v - pvals[idx - 1]) / (pvals[idx] - pvals[idx - 1])
        lo_alt = np.array(wd[lo_p][1]); up_alt = np.array(wd[up_p][1])
        all_alt = np.unique(np.concatenate([lo_alt, up_alt]))
        lo_sp = _interp_extrap(lo_alt, np.array(wd[lo_p][0]), all_alt)
        up_sp = _interp_extrap(up_alt, np.array(wd[up_p][0]), all_alt)
        sp = lo_sp * (1 - w) + up_sp * w
        o = np.argsort(all_alt)
        profiles.append({"percentile": req, "alt_km": all_alt[o].tolist(), "speed": sp[o].tolist()})
    return profiles


def _interp_extrap(x, y, xq):
    o = np.argsort(x, kind="mergesort")
    xs, ys = x[o], y[o]
    idx = np.searchsorted(xs, xq).clip(1, len(xs) - 1)
    lo, hi = idx - 1, idx
    slope = (ys[hi] - ys[lo]) / (xs[hi] - xs[lo])
    return slope * (xq - xs[lo]) + ys[lo]


def von_karman(dt=0.1, V=100.0):
    from scipy.signal import cont2discrete
    out = {}
    for name, L in (("u", 100.0), ("v", 30.0)):
        omega0 = V / L
        zeta = 1.0 / math.sqrt(2.0)
        scale = math.sqrt(math.pi / (2.0 * omega0 ** 3))
        A_c = np.array([[0.0, 1.0], [-omega0 ** 2, -2.0 * zeta * omega0]])
        B_c = np.array([[0.0], [1.0 * scale]])  # sigma = 1: Bd scales linearly in sigma
        C_c = np.array([[0.0, 1.0]]); D_c = np.zeros((1, 1))
        Ad, Bd, _, _, _ = cont2discrete((A_c, B_c, C_c, D_c), dt)
        out["Ad_" + name] = Ad.ravel().tolist()
        out["Bd_" + name] = Bd.ravel().tolist()
    return out


def read_full_rocket_constants():
    """Static scan of the dill pickle for the 13 float64 cells of
    `x_cog_inertia_subrocket_0_lambda` = full_rocket_inertia(...).func
    (rocket_dimensions.py:198-241, unpacked at main_sizing.py:209-212).  dill writes the
    cells in reverse alphabetical order of the closure's free variables; m_pay is a
    pickled Python float (BINFLOAT), the others numpy float64 scalars."""
    data = open(ref_path("data/rocket_parameters/rocket_functions.pkl"), "rb").read()
    ops = list(pickletools.genops(data))
    start = end = None
    for i, (op, arg, pos) in enumerate(ops):
        if op.name.endswith("UNICODE") and arg == "x_cog_inertia_subrocket_0_lambda":
            start = i
        if start is not None and op.name.endswith("UNICODE") and arg == "x_cog_inertia_subrocket_1_lambda":
            end = i
            break
    vals = []
    first_cell = next(i for i in range(start, end) if ops[i][0].name.endswith("UNICODE") and ops[i][1] == "cell_contents")
    for op, arg, pos in ops[first_cell:end]:   # the code object's own constants come before
        if op.name in ("SHORT_BINBYTES", "BINBYTES") and len(arg) == 8:
            vals.append(struct.unpack("<d", arg)[0])
        elif op.name == "BINFLOAT":
            vals.append(float(arg))
    names = ["x_wet_2_initial", "x_dry_1", "m_s_1", "m_pay", "m_2", "m_1_ox", "m_1_f", "h_lower_1",
             "h_1_ox", "h_1_f", "h_1", "I_wet_2_initial", "I_dry_1"]
    assert len(vals) == len(names), vals
    return dict(zip(names, vals))


STATE_NAMES = ["x[m]", "y[m]", "vx[m/s]", "vy[m/s]", "theta[rad]", "theta_dot[rad/s]",
               "gamma[rad]", "alpha[rad]", "mass[kg]", "mass_propellant[kg]", "time[s]"]


def phases_section(sz):
    """Constants of the flight phases other than the two landing-burn ones
    (rockets_physics.py:17-166,402-451,728-802,959-997; rtd_rl.py:11-188,353-534;
    load_initial_states.py:5-53; input_normalisation.py:5-71;
    reference_trajectory_interpolation.py:5-37)."""
    import pandas as pd
    tr = "data/reference_trajectory/"
    sub = pd.read_csv(ref_path(tr + "ascent_controls/subsonic_state_action_ascent_control.csv"))
    sup = pd.read_csv(ref_path(tr + "ascent_controls/supersonic_state_action_ascent_control.csv"))
    flip = pd.read_csv(ref_path(tr + "flip_over_and_boostbackburn_controls/state_action_flip_over_and_boostbackburn_control.csv"))
    ball = pd.read_csv(ref_path(tr + "ballistic_arc_descent_controls/state_action_ballistic_arc_descent_control.csv"))
    # load_initial_states.py:13-31 (np.array -> float64), :5-11, :33-45, :47-53
    state0 = {
        "subsonic": [0.0, 1.5, 0.0, 0.0, np.pi / 2, 0.0, 0.0, 0.0,
                     float(sz["Initial mass (subrocket 0)"]) * 1000,
                     float(sz["Actual propellant mass stage 1"]) * 1000, 0.0],
        "supersonic": [float(sub.iloc[-1][n]) for n in STATE_NAMES],
        "flip_over_boostbackburn": [float(sup.iloc[-1][n]) for n in STATE_NAMES],
        "ballistic_arc_descent": [float(flip.iloc[-1][n]) for n in STATE_NAMES],
    }
    state0["flip_over_boostbackburn"][8] = (float(sup.iloc[-1]["mass_propellant[kg]"])
                                            + float(sz["Actual structural mass stage 1"]) * 1000)

    def mx(df, cols):
        return np.max(np.abs(df[cols].values), axis=0)

    cols8 = ["x[m]", "y[m]", "vx[m/s]", "vy[m/s]", "theta[rad]", "theta_dot[rad/s]", "alpha[rad]", "mass[kg]"]
    m = mx(sub, cols8)
    r = math.radians
    norm = {
        "subsonic": [m[0] + 100, m[1] + 500, m[2] + 5, m[3] + 50, m[4] + r(2), m[5] * 2.5, m[6] + r(3), m[7]],
    }
    m = mx(sup, cols8)
    norm["supersonic"] = [m[0] + 2500, m[1] + 5000, m[2] + 100, m[3] + 150, m[4] + r(5), m[5] * 2.5, m[6] + r(3), m[7]]
    m = mx(flip, ["theta[rad]", "theta_dot[rad/s]"])
    norm["flip_over_boostbackburn"] = [m[0] + r(5), m[1] * 2.5]
    m = mx(ball, ["theta[rad]", "theta_dot[rad/s]", "alpha[rad]", "gamma[rad]"])
    norm["ballistic_arc_descent"] = [m[0] + r(5), m[1] * 2.5, m[3] + r(5), m[2] + r(5)]
    norm = {k: [float(v) for v in vs] for k, vs in norm.items()}
    # reference trajectory of the ascent rtd: interp1d(y, .) with extrapolation; scipy sorts
    # x with a stable argsort before building the interpolant
    ref = pd.read_csv(ref_path(tr + "ascent_controls/reference_trajectory_ascent_control.csv"))
    yv = ref["y[m]"].values
    order = np.argsort(yv, kind="mergesort")
    ascent_ref = {"y": yv[order].tolist()}
    for k, c in (("x", "x[m]"), ("vx", "vx[m/s]"), ("vy", "vy[m/s]"), ("m", "mass[kg]")):
        ascent_ref[k] = ref[c].values[order].tolist()
    # terminal Mach of the supersonic rtd (rtd_rl.py:580-589): the last reference row at the
    # restated ISA speed of sound (math.sqrt / Python float arithmetic)
    xt, yt, vxt, vyt = (float(ref[c].values[-1]) for c in ("x[m]", "y[m]", "vx[m/s]", "vy[m/s]"))
    _, _, a_t = isa(yt)
    mach_t = math.sqrt(vxt ** 2 + vyt ** 2) / a_t
    h1, h2 = float(sz["Stage 1 height "]), float(sz["Stage 2 height "])
    lb = [float(v) for v in ball.iloc[-1][STATE_NAMES]]
    return {
        "ascent_inertia": read_full_rocket_constants(),
        "cop_ascent": 0.25 * (h1 + h2),     # cop_func(lengths[0] = h_1 + h_2, d_0 = 0.25)
        "n_engines_stage1": int(sz["Number of engines stage 1"]),
        "rcs": {"max_force": float(sz["max_RCS_force_per_thruster"]),
                "d_bottom": float(sz["d_base_rcs_bottom"]), "d_top": float(sz["d_base_rcs_top"])},
        "state0": state0,
        "norm": norm,
        "ascent_ref": ascent_ref,
        "terminal_mach": {"subsonic": 1.0, "supersonic": mach_t},
        # rl_wrapped_env_pytorch (env_wrapped_rl_pytorch.py:107-110): speed of the landing
        # initial state, the v_ref scale of the Pcontrol phase
        "speed0_pcontrol": math.sqrt(lb[2] ** 2 + lb[3] ** 2),
        # rtd_rl.py:543-574 [mach, max_x, max_vy, max_vx, max_alpha_deg, w_alpha, w_x, w_vy, w_vx]
        "ascent_hyper": {
            "subsonic": [[0.0, 50, 10, 10, 0.5, 100, 100, 100, 100], [0.1, 50, 15, 10, 10, 100, 100, 100, 100]]
                        + [[m_, 50, 20, 5, 2, 100, 100, 100, 100] for m_ in (0.2, 0.3, 0.4, 0.5)]
                        + [[m_, 50, 20, 5, 1.75, 100, 100, 100, 100] for m_ in (0.6, 0.7, 0.8, 0.9, 1.0, 1.1)],
            "supersonic": [[1.0, 100, 50, 9, 8, 100, 100, 100, 100]]
                          + [[m_, 100, 60, vx_, 8, 100, 100, 100, 100] for m_, vx_ in
                             ((1.1, 20), (1.5, 20), (1.75, 30), (2.0, 40), (2.25, 50), (2.5, 60), (2.75, 70),
                              (3.0, 80), (3.25, 90), (3.5, 100), (3.75, 100))],
        },
    }


def isa(h):
    """The pack's ISA layer model (same constants as the "isa" section)."""
    g0, R, kappa, re = 9.80665, 287.05287, 1.4, 6356766.0
    L = [(-5.0e3, 320.65, -6.5e-3, 1.77687e5), (0.0, 288.15, -6.5e-3, 1.01325e5), (11.0e3, 216.65, 0.0, 2.26320e4),
         (20.0e3, 216.65, 1.0e-3, 5.47487e3), (32.0e3, 228.65, 2.8e-3, 8.68014e2), (47.0e3, 270.65, 0.0, 1.10906e2),
         (51.0e3, 270.65, -2.8e-3, 6.69384e1), (71.0e3, 214.65, -2.0e-3, 3.95639e0), (80.0e3, 196.65, -2.0e-3, 8.86272e-1)]
    H = re * h / (re + h)
    Hb, Tb, b, pb = [l for l in L if l[0] <= H][-1]
    T = Tb + b * (H - Hb)
    p = pb * (1 + b / Tb * (H - Hb)) ** (-g0 / (b * R)) if b != 0 else pb * math.exp(-g0 / (R * T) * (H - Hb))
    return p / (R * T), p, math.sqrt(kappa * R * T)


def main():
    import pandas as pd
    sz = read_sizing()
    cc = read_closure_constants()
    # initial state (load_initial_states.py:236-242): pandas parse, last row, by name
    df = pd.read_csv(ref_path("data/reference_trajectory/ballistic_arc_descent_controls/"
                              "state_action_ballistic_arc_descent_control.csv"))
    last = df.iloc[-1]
    names = ["x[m]", "y[m]", "vx[m/s]", "vy[m/s]", "theta[rad]", "theta_dot[rad/s]",
             "gamma[rad]", "alpha[rad]", "mass[kg]", "mass_propellant[kg]", "time[s]"]
    state0 = [float(last[n]) for n in names]
    st = df[["y[m]", "vy[m/s]", "theta[rad]", "theta_dot[rad/s]", "gamma[rad]", "x[m]", "vx[m/s]"]].values
    norm = {
        "y": float(np.max(np.abs(st[:, 0])) + 100),
        "vy": float(np.max(np.abs(st[:, 1])) + 50),
        "x": float(np.max(np.abs(st[:, 5])) + 1500),
        "vx": float(np.max(np.abs(st[:, 6])) + 30),
    }
    # size_gust_coefficients.py:3-22
    burnout_mass = (float(sz["Stage 1 Mass"]) - float(sz["Actual propellant mass stage 1"])) * 1000.0
    frontal = float(sz["Rocket frontal area"])
    C_gust_x = 2 * burnout_mass * (0.5 * 9.81) / (1.225 * (10 + 6.0) ** 2 * frontal)
    cd_tab = rbf_table("data/rocket_parameters/V2_aerodynamics/V2_drag_coefficient.csv")
    cl_tab = rbf_table("data/rocket_parameters/V2_aerodynamics/V2_lift_coefficient.csv")
    r10 = math.radians(10)
    print("enumerating C_D neighbourhoods ...", file=sys.stderr)
    cd_keys = enumerate_keys(cd_tab, -r10, r10, 41, [-r10, r10, 0.0])
    print("  ", len(cd_keys), file=sys.stderr)
    print("enumerating C_L neighbourhoods ...", file=sys.stderr)
    cl_keys = enumerate_keys(cl_tab, 0.0, 10.0, 401, [10.0, 1e-6])
    print("  ", len(cl_keys), file=sys.stderr)
    ca_tab, cn_tab = grid_fin_tables()
    pack = {
        "generator": "tools/make_param_pack.py",
        "sizing": {
            "thrust_per_engine": float(sz["Thrust engine stage 1"]),
            "nozzle_exit_pressure": float(sz["Nozzle exit pressure stage 1"]),
            "nozzle_exit_area": float(sz["Nozzle exit area"]),
            "n_engines_gimballed": int(sz["Number of engines gimballed stage 1"]),
            "v_exhaust": float(sz["Exhaust velocity stage 1"]),
            "grid_fin_area": float(sz["S_grid_fins"]),
            "d_base_grid_fin": float(sz["d_base_grid_fin"]),
            "rocket_radius": float(sz["Rocket Radius"]),
            "frontal_area": frontal,
            "m_prop0": float(sz["Actual propellant mass stage 1"]) * 1000,
            "stage_1_height": float(sz["Stage 1 height "]),
            "C_gust_x": C_gust_x,
            "C_gust_y": 0.0,
        },
        "inertia": cc,
        "cop": 0.75 * float(sz["Stage 1 height "]),
        "isa": {
            "Hb": [-5.0e3, 0.0, 11.0e3, 20.0e3, 32.0e3, 47.0e3, 51.0e3, 71.0e3, 80.0e3],
            "Tb": [320.65, 288.15, 216.65, 216.65, 228.65, 270.65, 270.65, 214.65, 196.65],
            "beta": [-6.5e-3, -6.5e-3, 0.0, 1.0e-3, 2.8e-3, 0.0, -2.8e-3, -2.0e-3, -2.0e-3],
            "pb": [1.77687e5, 1.01325e5, 2.26320e4, 5.47487e3, 8.68014e2, 1.10906e2, 6.69384e1,
                   3.95639e0, 8.86272e-1],
            "g0": 9.80665, "R": 287.05287, "kappa": 1.4, "r_earth": 6356766.0,
            "alt_max": 81020.0,
        },
        "gravity": {"R": 6371000.0, "g0": 9.80665},
        "aero_cd": cd_tab,
        "aero_cl": cl_tab,
        "rbf_keys_cd": [str(k) for k in cd_keys],
        "rbf_keys_cl": [str(k) for k in cl_keys],
        "grid_fin_ca": ca_tab,
        "grid_fin_cn": cn_tab,
        "wind_profiles": wind_profiles(),
        "von_karman": dict(von_karman(), V=100.0, L_u=100.0, L_v=30.0, dt=0.1,
                           y_threshold=15000.0, sigma_u=[0.5, 2.25], sigma_v=[1.25, 2.0]),
        "state0": state0,
        "norm": norm,
        "phases": phases_section(sz),
    }
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    with open(OUT, "w") as f:
        json.dump(pack, f, indent=1)
    print("wrote", os.path.normpath(OUT), file=sys.stderr)


def phases_only():
    """Refresh only the "phases" section of an existing pack (no key re-enumeration)."""
    with open(OUT) as f:
        pack = json.load(f)
    pack["phases"] = phases_section(read_sizing())
    with open(OUT, "w") as f:
        json.dump(pack, f, indent=1)
    print("updated phases in", os.path.normpath(OUT), file=sys.stderr)


if __name__ == "__main__":
    if "--phases-only" in sys.argv:
        phases_only()
    else:
        main()
