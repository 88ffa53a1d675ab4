"""Load the frozen parameter pack (data/param_pack.json) into the C `pd_params` struct.

The pack is plain data produced once by tools/make_param_pack.py from the reference's
data files (sizing_results.csv, V2 aero CSVs, grid-fin CSVs, wind CSV, initial state,
and the stage-2 inertia closure constants read statically from rocket_functions.pkl).
"""
import ctypes as C
import json
import os

import numpy as np

from ._lib import MAX_COLS, PdParams, U64

# pd_phase order (include/pdenv.h)
PHASE_NAMES = ["landing_burn_pure_throttle", "landing_burn", "landing_burn_pure_throttle_Pcontrol",
               "ballistic_arc_descent", "flip_over_boostbackburn", "subsonic", "supersonic", "landing_burn_ACS"]

PACK_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "data", "param_pack.json")

_pack_cache = {}


def load_pack(path=PACK_PATH):
    if path not in _pack_cache:
        with open(path) as f:
            _pack_cache[path] = json.load(f)
    return _pack_cache[path]


def _fill(arr, vals):
    for i, v in enumerate(vals):
        arr[i] = v


def _fill_table(t, tab):
    cols = tab["cols"]
    assert len(cols) == MAX_COLS
    t.n_cols = len(cols)
    t.n_pts = tab["n_pts"]
    for k, c in enumerate(cols):
        t.col_aoa[k] = c["aoa"]; t.col_start[k] = c["start"]; t.col_len[k] = c["len"]
    _fill(t.mach, tab["mach"]); _fill(t.coef, tab["coef"])


class Params:
    """Owns a PdParams struct and the key arrays it points to."""

    def __init__(self, path=PACK_PATH):
        pk = load_pack(path)
        p = PdParams()
        sz, inn = pk["sizing"], pk["inertia"]
        for k in ("thrust_per_engine", "nozzle_exit_pressure", "nozzle_exit_area", "v_exhaust",
                  "grid_fin_area", "d_base_grid_fin", "rocket_radius", "frontal_area", "m_prop0",
                  "C_gust_x", "C_gust_y"):
            setattr(p, k, sz[k])
        p.n_engines_gimballed = sz["n_engines_gimballed"]
        for k in ("h_ox", "h_f", "m_ox", "m_f", "h_lower", "m_dry", "x_dry", "I_dry", "engine_height"):
            setattr(p, k, inn[k])
        p.cop = pk["cop"]
        isa = pk["isa"]
        _fill(p.isa_Hb, isa["Hb"]); _fill(p.isa_Tb, isa["Tb"]); _fill(p.isa_beta, isa["beta"]); _fill(p.isa_pb, isa["pb"])
        p.isa_g0, p.isa_R, p.isa_kappa, p.isa_r, p.isa_alt_max = isa["g0"], isa["R"], isa["kappa"], isa["r_earth"], isa["alt_max"]
        p.grav_R, p.grav_g0 = pk["gravity"]["R"], pk["gravity"]["g0"]
        _fill_table(p.cd, pk["aero_cd"]); _fill_table(p.cl, pk["aero_cl"])
        ca, cn = pk["grid_fin_ca"], pk["grid_fin_cn"]
        p.ca_n = len(ca["x"]); _fill(p.ca_x, ca["x"]); _fill(p.ca_y, ca["y"])
        p.ca_min_mach, p.ca_min_val = ca["min_mach"], ca["min_val"]
        p.cn_n = len(cn["x"]); _fill(p.cn_x, cn["x"]); _fill(p.cn_y, cn["y"])
        p.cn_min_mach, p.cn_max_mach, p.cn_min_val, p.cn_max_val, p.cn_slope = (
            cn["min_mach"], cn["max_mach"], cn["min_val"], cn["max_val"], cn["slope"])
        for w, prof in enumerate(pk["wind_profiles"]):
            assert prof["percentile"] == 50 + w
            p.wind_n[w] = len(prof["alt_km"])
            _fill(p.wind_alt_km[w], prof["alt_km"]); _fill(p.wind_speed[w], prof["speed"])
        vk = pk["von_karman"]
        _fill(p.vk_Ad_u, vk["Ad_u"]); _fill(p.vk_Bd_u, vk["Bd_u"]); _fill(p.vk_Ad_v, vk["Ad_v"]); _fill(p.vk_Bd_v, vk["Bd_v"])
        p.vk_y_threshold = vk["y_threshold"]
        p.sigma_u_lo, p.sigma_u_hi = vk["sigma_u"]
        p.sigma_v_lo, p.sigma_v_hi = vk["sigma_v"]
        _fill(p.state0, pk["state0"])
        nm = pk["norm"]
        p.norm_y, p.norm_vy, p.norm_x, p.norm_vx = nm["y"], nm["vy"], nm["x"], nm["vx"]
        self.keys_cd = np.array([int(k) for k in pk["rbf_keys_cd"]], dtype=np.uint64)
        self.keys_cl = np.array([int(k) for k in pk["rbf_keys_cl"]], dtype=np.uint64)
        p.keys_cd = self.keys_cd.ctypes.data_as(C.POINTER(U64)); p.n_keys_cd = len(self.keys_cd)
        p.keys_cl = self.keys_cl.ctypes.data_as(C.POINTER(U64)); p.n_keys_cl = len(self.keys_cl)
        # the other flight phases (data/param_pack.json "phases", tools/make_param_pack.py)
        ph = pk["phases"]
        fr = ph["ascent_inertia"]
        _fill(p.full_rocket, [fr[k] for k in ("x_wet_2_initial", "x_dry_1", "m_s_1", "m_pay", "m_2", "m_1_ox",
                                              "m_1_f", "h_lower_1", "h_1_ox", "h_1_f", "h_1", "I_wet_2_initial",
                                              "I_dry_1")])
        p.cop_ascent = ph["cop_ascent"]
        p.n_engines_stage1 = ph["n_engines_stage1"]
        p.rcs_force, p.rcs_d_bottom, p.rcs_d_top = ph["rcs"]["max_force"], ph["rcs"]["d_bottom"], ph["rcs"]["d_top"]
        for k, name in enumerate(PHASE_NAMES):
            _fill(p.state0_phase[k], ph["state0"].get(name, pk["state0"]))
            _fill(p.norm_phase[k], ph["norm"].get(name, [nm["y"], nm["vy"]]))
        ref = ph["ascent_ref"]
        self.ref = [np.ascontiguousarray(ref[k], dtype=np.float64) for k in ("y", "x", "vx", "vy")]
        p.ref_y, p.ref_x, p.ref_vx, p.ref_vy = (a.ctypes.data_as(C.POINTER(C.c_double)) for a in self.ref)
        p.n_ref = len(ref["y"])
        for w, name in enumerate(("subsonic", "supersonic")):
            for r, row in enumerate(ph["ascent_hyper"][name]):
                _fill(p.hyper[w][r], [float(v) for v in row])
            p.terminal_mach[w] = ph["terminal_mach"][name]
        self.speed0_pcontrol = ph["speed0_pcontrol"]
        self.struct = p
        self.pack = pk

    def restrict_keys(self, n_cd, n_cl):
        """Keep only the first n_cd / n_cl pre-enumerated neighbourhoods (tests: forces the
        on-device exact solve for everything else)."""
        self.keys_cd = np.ascontiguousarray(self.keys_cd[:n_cd])
        self.keys_cl = np.ascontiguousarray(self.keys_cl[:n_cl])
        p = self.struct
        p.keys_cd = self.keys_cd.ctypes.data_as(C.POINTER(U64)); p.n_keys_cd = len(self.keys_cd)
        p.keys_cl = self.keys_cl.ctypes.data_as(C.POINTER(U64)); p.n_keys_cl = len(self.keys_cl)
        return self

    @property
    def state0(self):
        return np.array(self.pack["state0"])

    def state0_of(self, phase):
        """Initial state of a phase (load_initial_states.py), by pd_phase index or name."""
        k = PHASE_NAMES.index(phase) if isinstance(phase, str) else int(phase)
        return np.array(self.struct.state0_phase[k][:])
