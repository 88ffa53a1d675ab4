"""ctypes binding of libpdenv.so (include/pdenv.h).

The product path: every call goes to the HIP library.  There is no CPU fallback; loading
fails loudly when the library is missing or when no HIP device is visible.
"""
import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libpdenv.so")

D, I32, I64, U64 = C.c_double, C.c_int32, C.c_int64, C.c_uint64
MAX_PTS, MAX_COLS, MAX_TAB, MAX_WIND, N_PROF = 256, 5, 64, 16, 50
N_STATE, N_INFO = 11, 49

PD_OK, PD_ERR_INVALID, PD_ERR_HIP, PD_ERR_NOMEM, PD_ERR_UNSUPPORTED = range(5)
(PURE_THROTTLE, LANDING_BURN, PCONTROL, BALLISTIC_ARC, FLIP_OVER, SUBSONIC, SUPERSONIC,
 LANDING_BURN_ACS) = range(8)
RTD_RL, RTD_PSO, RTD_NONE = 0, 1, 2
F64, F32 = 0, 1
ACTOR_PARAMS = {0: 249, 1: 372}   # PD_ACTOR_PARAMS_PURE_THROTTLE / _LANDING_BURN

# pd_info_field order (include/pdenv.h): the last physics sub-step's quantities
INFO_FIELDS = ["air_density", "atmospheric_pressure", "speed_of_sound", "mach_number",
               "dynamic_pressure", "CL", "CD", "mass_flow", "x_cog", "inertia",
               "alpha_effective", "throttle", "g_load_1_sec_window", "ug", "vg", "gimbal_angle_deg",
               "mach_number_max", "drag", "lift", "d_cp_cg", "d_thrust_cg", "fuel_percentage_consumed",
               "control_force_parallel", "control_force_perpendicular", "control_force_x", "control_force_y",
               "aero_force_x", "aero_force_y", "gravity", "F_wind_x", "F_wind_y", "vx_dot", "vy_dot",
               "control_moment_z", "aero_moment_z", "M_wind_z", "moments_z", "theta_dot_dot",
               "delta_command_left_rad", "delta_command_right_rad", "delta_left_rad", "delta_right_rad",
               "C_a", "C_n_L", "C_n_R", "gf_F_perpendicular", "gf_F_parallel", "gf_Mz", "theta_in"]
assert len(INFO_FIELDS) == N_INFO


class PdAeroTable(C.Structure):
    _fields_ = [("n_cols", I32), ("n_pts", I32), ("col_aoa", D * MAX_COLS),
                ("col_start", I32 * MAX_COLS), ("col_len", I32 * MAX_COLS),
                ("mach", D * MAX_PTS), ("coef", D * MAX_PTS)]


class PdParams(C.Structure):
    _fields_ = [
        ("thrust_per_engine", D), ("nozzle_exit_pressure", D), ("nozzle_exit_area", D), ("v_exhaust", D),
        ("n_engines_gimballed", I32), ("pad0", I32),
        ("grid_fin_area", D), ("d_base_grid_fin", D), ("rocket_radius", D), ("frontal_area", D),
        ("m_prop0", D), ("C_gust_x", D), ("C_gust_y", D),
        ("h_ox", D), ("h_f", D), ("m_ox", D), ("m_f", D), ("h_lower", D), ("m_dry", D), ("x_dry", D),
        ("I_dry", D), ("engine_height", D), ("cop", D),
        ("isa_Hb", D * 9), ("isa_Tb", D * 9), ("isa_beta", D * 9), ("isa_pb", D * 9),
        ("isa_g0", D), ("isa_R", D), ("isa_kappa", D), ("isa_r", D), ("isa_alt_max", D),
        ("grav_R", D), ("grav_g0", D),
        ("cd", PdAeroTable), ("cl", PdAeroTable),
        ("ca_n", I32), ("cn_n", I32),
        ("ca_x", D * MAX_TAB), ("ca_y", D * MAX_TAB), ("ca_min_mach", D), ("ca_min_val", D),
        ("cn_x", D * MAX_TAB), ("cn_y", D * MAX_TAB), ("cn_min_mach", D), ("cn_max_mach", D),
        ("cn_min_val", D), ("cn_max_val", D), ("cn_slope", D),
        ("wind_n", I32 * N_PROF),
        ("wind_alt_km", (D * MAX_WIND) * N_PROF), ("wind_speed", (D * MAX_WIND) * N_PROF),
        ("vk_Ad_u", D * 4), ("vk_Bd_u", D * 2), ("vk_Ad_v", D * 4), ("vk_Bd_v", D * 2), ("vk_y_threshold", D),
        ("sigma_u_lo", D), ("sigma_u_hi", D), ("sigma_v_lo", D), ("sigma_v_hi", D),
        ("state0", D * N_STATE), ("norm_y", D), ("norm_vy", D), ("norm_x", D), ("norm_vx", D),
        ("keys_cd", C.POINTER(U64)), ("n_keys_cd", I64),
        ("keys_cl", C.POINTER(U64)), ("n_keys_cl", I64),
        # ABI 2: the other flight phases
        ("full_rocket", D * 13), ("cop_ascent", D), ("n_engines_stage1", I32), ("pad1", I32),
        ("rcs_force", D), ("rcs_d_bottom", D), ("rcs_d_top", D),
        ("state0_phase", (D * N_STATE) * 8), ("norm_phase", (D * 8) * 8),
        ("ref_y", C.POINTER(D)), ("ref_x", C.POINTER(D)), ("ref_vx", C.POINTER(D)), ("ref_vy", C.POINTER(D)),
        ("n_ref", I32), ("pad2", I32),
        ("hyper", ((D * 9) * 12) * 2), ("terminal_mach", D * 2),
    ]


class PdConfig(C.Structure):
    _fields_ = [("n_envs", I64), ("device", I32), ("phase", I32), ("rtd", I32), ("precision", I32),
                ("seed", U64), ("env_offset", U64), ("enable_wind", I32), ("stochastic_wind", I32),
                ("wind_percentile", I32), ("auto_reset", I32), ("tilt_sigma_rad", D),
                ("action_f64", I32), ("lanes_per_env", I32),
                ("dt", D), ("discount_factor", D), ("trajectory_length", I32), ("integrator", I32),
                ("table_flags", I32), ("pad3", I32)]


# pd_table_flags
TABLES_NO_CELL_PIECES, TABLES_NO_FINE_INDEX, TABLES_EXACT_ATMOSPHERE, TABLES_VERBOSE = 1, 2, 4, 8


class PdTuning(C.Structure):
    _fields_ = [("step_fuse", I32), ("policy_fuse", I32), ("policy_lanes", I32), ("policy_list", I32),
                ("policy_list_at", D), ("policy_refill", I32), ("policy_slots", I32),
                ("policy_refill_own", I32), ("pad_tuning", I32)]


EXPORTS = ["pd_abi_version", "pd_sizeof_params", "pd_sizeof_config", "pd_last_error", "pd_device_count", "pd_create",
           "pd_destroy", "pd_reset", "pd_step", "pd_step_n", "pd_rollout", "pd_rollout_policy", "pd_pso_step",
           "pd_flush_misses", "pd_observe", "pd_get_state", "pd_set_state", "pd_get_actuators", "pd_set_actuators",
           "pd_set_gload_window", "pd_get_gload_window", "pd_set_wind_sigmas", "pd_get_wind_state",
           "pd_set_wind_state", "pd_get_counters", "pd_set_counters", "pd_checkpoint_size", "pd_checkpoint_save",
           "pd_checkpoint_load", "pd_counters", "pd_stats", "pd_count_work", "pd_atmosphere", "pd_obs_dim",
           "pd_action_dim", "pd_step_sac", "pd_pso_swarm_minima", "pd_pso_update_bests", "pd_cell_piece_info",
           "pd_step_sac_ring", "pd_sac_actor", "pd_step_sac_fused", "pd_atm_table", "pd_set_tuning", "pd_get_tuning",
           "pd_pso_swarm_minima_scratch_bytes", "pd_step_n_info", "pd_pso_step_chunked", "pd_rollout_policy_chunked"]
ABI_VERSION = 11

_lib = None


class PdError(RuntimeError):
    pass


def load(path=None):
    """Load libpdenv.so (built in-tree by pdenv.build)."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or os.environ.get("PDENV_LIB") or LIB_PATH
    if not os.path.exists(path):
        raise PdError(f"libpdenv.so not found at {path}: run __graft_entry__.build() "
                      "(the HIP extension is required; there is no CPU fallback)")
    L = C.CDLL(path)
    vp, P = C.c_void_p, C.POINTER
    L.pd_abi_version.restype = C.c_int
    L.pd_last_error.restype = C.c_char_p
    L.pd_device_count.restype = C.c_int
    L.pd_create.argtypes = [P(PdParams), P(PdConfig), P(vp)]
    L.pd_destroy.argtypes = [vp]
    L.pd_reset.argtypes = [vp, vp, vp, vp]
    L.pd_step.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]
    L.pd_step_n.argtypes = [vp, vp, I32, vp, vp, vp, vp, vp, vp]
    L.pd_step_n_info.argtypes = [vp, vp, I32, vp, vp, vp, vp, vp, vp, U64, vp]
    L.pd_step_n_info.restype = C.c_int
    F32 = C.c_float
    L.pd_step_sac.argtypes = [vp, vp, vp, I32, vp, F32, F32, F32, vp, vp, vp, vp]
    L.pd_step_sac_ring.argtypes = [vp, vp, I32, F32, F32, F32, vp, vp, vp, I64, vp, vp, vp, vp, vp]
    L.pd_sac_actor.argtypes = [I64, I32, I32, I32, I32, vp, vp, vp, vp]
    L.pd_step_sac_fused.argtypes = [vp, I32, I32, I32, I32, vp, vp, I32, F32, F32, F32, vp, vp, vp, I64, vp, vp, vp,
                                    vp, vp]
    L.pd_set_tuning.argtypes = [vp, P(PdTuning)]
    L.pd_get_tuning.argtypes = [vp, P(PdTuning)]
    L.pd_rollout.argtypes = [vp, vp, I32, vp, vp]
    L.pd_rollout_policy.argtypes = [vp, vp, I32, I32, vp, vp, I32, vp]
    L.pd_rollout_policy_chunked.argtypes = [vp, vp, I32, I32, vp, vp, I32, vp]
    L.pd_pso_step.argtypes = [I64, I32, vp, vp, vp, vp, vp, vp, vp, vp, vp, C.c_double, C.c_double, C.c_double,
                              U64, C.c_uint32, U64, vp, vp]
    L.pd_pso_step_chunked.argtypes = L.pd_pso_step.argtypes
    L.pd_pso_swarm_minima.argtypes = [I64, I32, I32, vp, vp, vp, vp, vp, vp, C.c_size_t, vp]
    L.pd_pso_swarm_minima_scratch_bytes.argtypes = [I64, I32]
    L.pd_pso_swarm_minima_scratch_bytes.restype = C.c_size_t
    L.pd_pso_update_bests.argtypes = [I32, I32, vp, vp, vp, vp, vp, vp, vp]
    L.pd_observe.argtypes = [vp, vp, vp]
    L.pd_flush_misses.argtypes = [vp, vp]
    L.pd_get_state.argtypes = [vp, vp, vp]
    L.pd_set_state.argtypes = [vp, vp, vp]
    L.pd_get_actuators.argtypes = [vp, vp, vp]
    L.pd_set_actuators.argtypes = [vp, vp, vp]
    L.pd_set_wind_sigmas.argtypes = [vp, vp, vp]
    L.pd_set_gload_window.argtypes = [vp, vp, vp, vp, vp]
    L.pd_counters.argtypes = [vp, P(I64), P(I64), P(I64), P(I64)]
    L.pd_stats.argtypes = [vp, P(I64), I32]
    L.pd_count_work.argtypes = [vp, I32]
    L.pd_cell_piece_info.argtypes = [P(PdParams), I32, I64, P(C.c_double), I32]
    L.pd_atm_table.argtypes = [P(PdParams), I32, vp, I64, vp, vp]
    L.pd_atmosphere.argtypes = [vp, vp, vp, I64, vp]
    L.pd_get_gload_window.argtypes = [vp, vp, vp, vp, vp, vp]
    L.pd_get_wind_state.argtypes = [vp, vp, vp, vp, vp]
    L.pd_set_wind_state.argtypes = [vp, vp, vp, vp, vp]
    L.pd_get_counters.argtypes = [vp, vp, vp, vp, vp]
    L.pd_set_counters.argtypes = [vp, vp, vp, vp, vp]
    L.pd_checkpoint_size.argtypes = [vp]; L.pd_checkpoint_size.restype = C.c_size_t
    L.pd_checkpoint_save.argtypes = [vp, vp, vp]
    L.pd_checkpoint_load.argtypes = [vp, vp, vp]
    L.pd_obs_dim.argtypes = [vp]; L.pd_obs_dim.restype = C.c_int
    L.pd_action_dim.argtypes = [vp]; L.pd_action_dim.restype = C.c_int
    for name in ("pd_create", "pd_destroy", "pd_reset", "pd_step", "pd_step_n", "pd_step_sac", "pd_rollout", "pd_rollout_policy", "pd_pso_step",
                 "pd_rollout_policy_chunked", "pd_pso_step_chunked", "pd_pso_swarm_minima", "pd_pso_update_bests", "pd_flush_misses", "pd_observe",
                 "pd_get_state", "pd_set_state", "pd_get_actuators", "pd_set_actuators",
                 "pd_set_wind_sigmas", "pd_set_gload_window", "pd_counters", "pd_stats", "pd_count_work",
                 "pd_get_gload_window",
                 "pd_get_wind_state", "pd_set_wind_state", "pd_get_counters", "pd_set_counters",
                 "pd_checkpoint_save", "pd_checkpoint_load", "pd_atmosphere", "pd_cell_piece_info",
                 "pd_step_sac_ring", "pd_sac_actor", "pd_step_sac_fused", "pd_atm_table", "pd_set_tuning",
                 "pd_get_tuning"):
        getattr(L, name).restype = C.c_int
    L.pd_sizeof_params.restype = C.c_size_t
    L.pd_sizeof_config.restype = C.c_size_t
    if L.pd_abi_version() != ABI_VERSION:
        raise PdError("libpdenv ABI version mismatch")
    if L.pd_sizeof_params() != C.sizeof(PdParams) or L.pd_sizeof_config() != C.sizeof(PdConfig):
        raise PdError("pd_params/pd_config layout mismatch between ctypes and libpdenv.so")
    _lib = L
    return L


def check(status):
    if status != PD_OK:
        msg = load().pd_last_error().decode(errors="replace")
        raise PdError(f"libpdenv error {status}: {msg}")
