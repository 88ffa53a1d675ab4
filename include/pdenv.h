/* pdenv.h -- C ABI of the MI355X-native vectorised powered-descent environment (libpdenv.so).
 *
 * Drop-in boundary for the hot path of JvanZyl1/PSSO-SAC-for-powered-descent.  The reference
 * has no FFI: its seam is the Python object API, which this ABI replaces one-for-one for a
 * batch of N environments living in HBM:
 *
 *   pd_create   <- rocket_environment_pre_wrap.__init__ + compile_physics + compile_rtd_{rl,pso}
 *                  (src/envs/base_environment.py:13-78, src/envs/rockets_physics.py:707-998,
 *                   src/envs/rl/rtd_rl.py:537-604, src/envs/pso/rtd_pso.py:320-383)
 *   pd_reset    <- rocket_environment_pre_wrap.reset (base_environment.py:80-97)
 *   pd_step     <- rocket_environment_pre_wrap.step  (base_environment.py:99-154), i.e.
 *                  physics_step x4 sub-steps (rockets_physics.py:455-704, :857-860, :953-956),
 *                  g-load window, truncated_func -> done_func -> reward_func, plus the wrapper's
 *                  observation (env_wrapped_rl_pytorch.py:167-202 / env_wrapped_ea.py:97-123)
 *   pd_get_state/pd_set_state <- .state attribute (teacher forcing, checkpoint, perturbation)
 *   trunc_id output of pd_step <- rl_wrapped_env_pytorch.truncation_id (env_wrapped_rl_pytorch.py:117-118)
 *   pd_rollout_policy <- pso_wrapped_env.objective_function + simple_actor.forward for a batch of
 *                  particles (env_wrapped_ea.py:18-44, 200-222; particle_swarm_optimisation.py:334-350)
 *
 * Conventions: plain C, no torch types.  All array arguments are DEVICE pointers (HBM) owned by
 * the caller, laid out env-major [N] or [N][k]; `stream` is a hipStream_t (NULL = default).
 * Calls are asynchronous and stream-ordered; a handle is not thread-safe (one per GPU/shard).
 * Floating point buffers use the handle's precision: double for PD_F64, float for PD_F32.
 * Errors are returned as pd_status codes; pd_last_error() gives a thread-local message.
 */
#ifndef PDENV_H
#define PDENV_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PD_ABI_VERSION 11  /* 4: pd_config.integrator (was padding); 5: pd_count_work, pd_step_sac; 6: cell pieces (pd_cell_piece_info, stats word 44); 7: pd_step_sac_ring, pd_sac_actor, stats word 45; 8: pd_step_sac_fused, pd_atm_table; 9: pd_config.table_flags, pd_tuning, caller scratch for pd_pso_swarm_minima, state/action dims of pd_step_sac_fused; 10: step launches insert their own solved misses (pd_flush_misses optional), explicit list settings turn the auto refill off; 11: pd_pso_step_chunked, pd_rollout_policy_chunked */
#define PD_MAX_PTS 256      /* aero scatter points per table */
#define PD_MAX_COLS 5       /* AoA columns per aero table */
#define PD_MAX_TAB 64       /* grid-fin table length */
#define PD_MAX_WIND 16      /* nodes per wind profile */
#define PD_N_WIND_PROFILES 50   /* integer percentiles 50..99 */
#define PD_N_STATE 11       /* x y vx vy theta theta_dot gamma alpha mass mass_propellant time */
#define PD_N_INFO 49        /* see pd_info_field */
/* simple_actor sizes of the PSO drivers (env_wrapped_ea.py:18-36, 174-185):
 * pure throttle 2-8-(8-8)x3-1, landing_burn 5-8-(8-8)x4-4 */
#define PD_ACTOR_PARAMS_PURE_THROTTLE 249
#define PD_ACTOR_PARAMS_LANDING_BURN 372

typedef enum { PD_OK = 0, PD_ERR_INVALID = 1, PD_ERR_HIP = 2, PD_ERR_NOMEM = 3, PD_ERR_UNSUPPORTED = 4 } pd_status;
/* compile_physics flight phases (rockets_physics.py:707-998; base_environment.py:21).  Actions:
 * 1 (pure throttle: throttle; Pcontrol: v_ref; ballistic: RCS; flip-over: gimbal), 4 (landing_burn),
 * 2 (subsonic/supersonic: gimbal, throttle).  PD_PHASE_LANDING_BURN_ACS is accepted by the
 * enum but pd_create refuses it: the reference raises TypeError at its first step
 * (rockets_physics.py:867-891 calls the gimballed decomposer with ACS arguments;
 * base_environment.py:126-130 passes two prevs to a three-prev lambda). */
typedef enum {
    PD_PHASE_PURE_THROTTLE = 0, PD_PHASE_LANDING_BURN = 1, PD_PHASE_PCONTROL = 2,
    PD_PHASE_BALLISTIC_ARC = 3, PD_PHASE_FLIP_OVER = 4, PD_PHASE_SUBSONIC = 5, PD_PHASE_SUPERSONIC = 6,
    PD_PHASE_LANDING_BURN_ACS = 7
} pd_phase;
/* reward/truncated/done family: rtd_rl.py, rtd_pso.py, or none (compile_physics stepping only:
 * reward 0, never done/truncated).  Pairs the reference cannot step are refused by pd_create
 * with PD_ERR_UNSUPPORTED: RL + flip-over (rtd_rl.py:134 truncated_func takes one argument,
 * base_environment.py:150 passes three), PSO + any phase but the two landing burns (the same
 * arity mismatch in rtd_pso.py:38,107,141). */
typedef enum { PD_RTD_RL = 0, PD_RTD_PSO = 1, PD_RTD_NONE = 2 } pd_rtd;
typedef enum { PD_F64 = 0, PD_F32 = 1 } pd_precision;
/* Integrator of the physics sub-steps.  PD_INTEG_REFERENCE is the reference's semi-implicit Euler
 * (compile_physics, rockets_physics.py:909-957 / 803-861) and the only mode with reference
 * parity.  PD_INTEG_RK4 is NOT the reference: BASELINE config c2's "RK4 dt=0.01 s" (SURVEY 8(d)
 * c2, "benchmarked separately, labelled non-parity"), classical RK4 over (x, y, vx, vy, theta,
 * theta_dot, mass, mass_propellant) with rocket_physics_fcn's forces at every stage, 10 x 0.01 s
 * per 0.1 s env step; landing_burn_pure_throttle without wind only (the von Karman gusts are a
 * discrete-time process), no policy rollouts.  Checked against the oracle's restatement
 * (orc_physics, ORC_INTEG_RK4), not against the reference. */
typedef enum { PD_INTEG_REFERENCE = 0, PD_INTEG_RK4 = 1 } pd_integrator;
/* pd_config.table_flags: how the aero and atmosphere lookups are served (results agree within the
 * tolerances of DESIGN.md s4/s8; the cell-piece and fine-index switches give the same bits as
 * their default, which the GPU tests check).  0 = the defaults. */
typedef enum {
    PD_TABLES_NO_CELL_PIECES = 1,   /* interior C_D/C_L queries by payload sums, not cell pieces */
    PD_TABLES_NO_FINE_INDEX = 2,    /* cell pieces reached through the cell / sub-cell records only */
    PD_TABLES_EXACT_ATMOSPHERE = 4, /* the ISA closed form on the device, never the tabulated pieces */
    PD_TABLES_VERBOSE = 8           /* print the table builders' statistics to stderr at create */
} pd_table_flags;

/* One neighbourhood-aero table: scatter points grouped by AoA column, Mach-sorted inside. */
typedef struct {
    int32_t n_cols, n_pts;
    double col_aoa[PD_MAX_COLS];
    int32_t col_start[PD_MAX_COLS], col_len[PD_MAX_COLS];
    double mach[PD_MAX_PTS];
    double coef[PD_MAX_PTS];
} pd_aero_table;

/* Physical parameter pack (host memory); filled from data/param_pack.json by the loader. */
typedef struct {
    /* sizing_results.csv (rockets_physics.py:714-719, size_gust_coefficients.py:3-22) */
    double thrust_per_engine, nozzle_exit_pressure, nozzle_exit_area, v_exhaust;
    int32_t n_engines_gimballed, pad0;
    double grid_fin_area, d_base_grid_fin, rocket_radius, frontal_area, m_prop0, C_gust_x, C_gust_y;
    /* stage-2 stage_inertia closure constants (rocket_dimensions.py:158-197) */
    double h_ox, h_f, m_ox, m_f, h_lower, m_dry, x_dry, I_dry, engine_height, cop;
    /* ISA layer table (ambiance) + gravity (atmosphere_dynamics.py:5-33) */
    double isa_Hb[9], isa_Tb[9], isa_beta[9], isa_pb[9];
    double isa_g0, isa_R, isa_kappa, isa_r, isa_alt_max, grav_R, grav_g0;
    /* V2 aero (aerodynamic_coefficients.py:8-66) */
    pd_aero_table cd, cl;
    /* grid fins (grid_fin_aerodynamics.py:7-46), x sorted */
    int32_t ca_n, cn_n;
    double ca_x[PD_MAX_TAB], ca_y[PD_MAX_TAB], ca_min_mach, ca_min_val;
    double cn_x[PD_MAX_TAB], cn_y[PD_MAX_TAB], cn_min_mach, cn_max_mach, cn_min_val, cn_max_val, cn_slope;
    /* wind (HorizontalWindSpeed.py, vonkarman.py): profiles for percentiles 50..99 */
    int32_t wind_n[PD_N_WIND_PROFILES];
    double wind_alt_km[PD_N_WIND_PROFILES][PD_MAX_WIND], wind_speed[PD_N_WIND_PROFILES][PD_MAX_WIND];
    double vk_Ad_u[4], vk_Bd_u[2], vk_Ad_v[4], vk_Bd_v[2], vk_y_threshold;
    double sigma_u_lo, sigma_u_hi, sigma_v_lo, sigma_v_hi;
    /* initial state (load_initial_states.py:236-242) and observation normalisers */
    double state0[PD_N_STATE];
    double norm_y, norm_vy, norm_x, norm_vx;
    /* pre-enumerated neighbourhood keys of the two aero tables (host arrays, may be NULL) */
    const uint64_t* keys_cd; int64_t n_keys_cd;
    const uint64_t* keys_cl; int64_t n_keys_cl;
    /* ---- ABI 2: the other flight phases (rockets_physics.py:17-166,402-451,728-802,959-997) */
    /* full_rocket_inertia cells of x_cog_inertia_subrocket_0_lambda (rocket_dimensions.py:198-241):
     * x_wet_2_initial, x_dry_1, m_s_1, m_pay, m_2, m_1_ox, m_1_f, h_lower_1, h_1_ox, h_1_f, h_1,
     * I_wet_2_initial, I_dry_1 */
    double full_rocket[13];
    double cop_ascent;                  /* cop_func(h_1 + h_2, d_0 = 0.25) (main_sizing.py:215) */
    int32_t n_engines_stage1, pad1;     /* 42: 16 gimballed + 26 fixed in the ascent */
    double rcs_force, rcs_d_bottom, rcs_d_top;   /* RCS (rockets_physics.py:149-166, 784-786) */
    double state0_phase[8][PD_N_STATE]; /* initial state per pd_phase (load_initial_states.py) */
    double norm_phase[8][8];            /* RL observation normalisers (input_normalisation.py) */
    /* ascent reference trajectory sorted by y (reference_trajectory_interpolation.py:5-37) */
    const double* ref_y; const double* ref_x; const double* ref_vx; const double* ref_vy;
    int32_t n_ref, pad2;
    double hyper[2][12][9];             /* rtd_rl.py:543-574, subsonic / supersonic */
    double terminal_mach[2];            /* rtd_rl.py:576-589 */
} pd_params;

typedef struct {
    int64_t n_envs;
    int32_t device;            /* HIP device ordinal */
    int32_t phase;             /* pd_phase */
    int32_t rtd;               /* pd_rtd */
    int32_t precision;         /* pd_precision */
    uint64_t seed;             /* Philox key (wind normals, sigmas, percentiles, tilt) */
    uint64_t env_offset;       /* global index of env 0 (multi-GPU shards draw disjoint streams) */
    int32_t enable_wind, stochastic_wind;
    int32_t wind_percentile;   /* 50..99, or -1 = float(randint(50, 99)) per reset */
    int32_t auto_reset;        /* reset envs in-kernel when done|truncated */
    double tilt_sigma_rad;     /* initial pitch perturbation N(0, s) (0 = reference) */
    int32_t action_f64;        /* actions are double (f64 path, no float32 islands) */
    int32_t lanes_per_env;     /* step-kernel lanes per env: 1, 2, 4, 8 or 16 (0 = by n_envs: 16 up
                                  to 4 096 envs, 8 up to 8 192, 4 up to 16 384, else 2; policy
                                  rollouts use at most 8) */
    /* ---- ABI 2 */
    double dt;                 /* physics dt of phases 2..6, compile_physics(dt, phase) (0 = the env's 0.1) */
    double discount_factor;    /* rtd_rl landing_burn reward scale (1-g)/(1-g^L) and the Pcontrol
                                  alive bonus 0.01 (1-g) (rtd_rl.py:267, 472); rl_wrapped_env_pytorch kwargs */
    int32_t trajectory_length;
    int32_t integrator;        /* pd_integrator (ABI 4; 0 = the reference's) */
    int32_t table_flags;       /* pd_table_flags (ABI 9; 0 = the defaults) */
    int32_t pad3;
} pd_config;

/* Launch tuning of a handle (pd_set_tuning / pd_get_tuning; ABI 9).  Results never depend on it:
 * every setting steps the same envs through the same arithmetic. */
typedef struct {
    int32_t step_fuse;        /* env-steps per pd_step_n / pd_rollout launch, 1..256 (default 128) */
    int32_t policy_fuse;      /* policy steps per pd_rollout_policy launch: a power of two 1..64 (default 64) */
    int32_t policy_lanes;     /* lanes per env of the policy rollouts: 2 (default), 4 or 8 */
    int32_t policy_list;      /* live-list launches of the policy rollouts: -1 = when the grid exceeds
                                 one chip round (default), 0 = never, 1 = from the first launch */
    double policy_list_at;    /* > 0 (with policy_list -1 or 0): switch the list on once the live count
                                 read back falls to this fraction of n_envs (default 0: never) */
    int32_t policy_refill;    /* refill rollouts: -1 = every windless swarm of at least one wave's slots
                                 unless policy_list >= 0 or policy_list_at > 0 asks for the per-check
                                 launches (default; pool batch 3/4 of a wave's slots), 0 = never, k in
                                 1..64 = on (policy_list, policy_list_at and check_every then do nothing),
                                 pool batch k.  One launch of policy_slots env slots (0: the resident
                                 capacity) steps the whole swarm: a wave's slots take the next particles
                                 of its own range as their episodes end (no atomic; policy_refill_own),
                                 then the shared pool's once k of them wait (or none is live: a wave
                                 ballot, one atomic).  Windy handles: the per-check launches */
    int32_t policy_slots;     /* env slots of a refill rollout (0 = the chip's resident capacity; rounded
                                 down to whole waves) */
    int32_t policy_refill_own;/* refill rollouts: percent of the swarm handed out from the waves' own
                                 particle ranges (no atomic), the rest from the shared pool; -1 = 100 */
    int32_t pad_tuning;
} pd_tuning;

/* Info tap of pd_step: the quantities of the LAST physics sub-step that rocket_physics_fcn puts in
 * its info dict (rockets_physics.py:649-702, incl. acceleration_dict / moments_dict), the
 * action_info of the phase's control law and the ACS's acs_info (acs_model.py:62-86), and the
 * env's g_load_1_sec_window (base_environment.py:149).  Layout [PD_N_INFO][N].  Entries that are
 * arithmetic of these and the post-step state (accelerations, gravity_force_y, F_n_L = C_n_L qS,
 * ...) are formed by the caller (pdenv/wrappers.py builds the reference's dict). */
typedef enum {
    PD_INFO_AIR_DENSITY = 0, PD_INFO_PRESSURE, PD_INFO_SPEED_OF_SOUND, PD_INFO_MACH, PD_INFO_Q,
    PD_INFO_CL, PD_INFO_CD, PD_INFO_MASS_FLOW, PD_INFO_X_COG, PD_INFO_INERTIA, PD_INFO_ALPHA_EFF,
    PD_INFO_THROTTLE, PD_INFO_GLOAD, PD_INFO_UG, PD_INFO_VG, PD_INFO_GIMBAL_DEG,
    PD_INFO_MACH_MAX,                  /* sqrt(2 Qmax / rho) / a, Qmax 30000 (200 above the ISA) */
    PD_INFO_DRAG, PD_INFO_LIFT, PD_INFO_D_CP_CG, PD_INFO_D_THRUST_CG, PD_INFO_FUEL_CONSUMED,
    PD_INFO_CF_PAR, PD_INFO_CF_PERP, PD_INFO_CF_X, PD_INFO_CF_Y, PD_INFO_AERO_X, PD_INFO_AERO_Y,
    PD_INFO_GRAVITY,                   /* g at the sub-step's altitude */
    PD_INFO_F_WIND_X, PD_INFO_F_WIND_Y, PD_INFO_VX_DOT, PD_INFO_VY_DOT,
    PD_INFO_CONTROL_MOMENT, PD_INFO_AERO_MOMENT, PD_INFO_M_WIND, PD_INFO_MOMENTS, PD_INFO_THETA_DDOT,
    PD_INFO_DCMD_L, PD_INFO_DCMD_R,    /* fin deflection commands (rad) */
    PD_INFO_DELTA_L, PD_INFO_DELTA_R,  /* filtered fin deflections (rad) */
    PD_INFO_GF_CA, PD_INFO_GF_CN_L, PD_INFO_GF_CN_R,   /* grid-fin C_a, C_n of the left/right fin */
    PD_INFO_GF_F_PERP, PD_INFO_GF_F_PAR, PD_INFO_GF_MZ, /* grid-fin force perpendicular/parallel, moment */
    PD_INFO_THETA_IN                   /* pitch at the start of the sub-step (the ACS's pitch_angle) */
} pd_info_field;

typedef struct pd_env pd_env;

int pd_abi_version(void);
/* sizeof(pd_params) / sizeof(pd_config) as compiled, for binding-layout checks */
size_t pd_sizeof_params(void);
size_t pd_sizeof_config(void);
const char* pd_last_error(void);
/* Number of HIP devices visible (0 without a GPU); never aborts. */
int pd_device_count(void);

pd_status pd_create(const pd_params* params, const pd_config* cfg, pd_env** out);
pd_status pd_destroy(pd_env* env);
/* Launch tuning (see pd_tuning); PD_ERR_INVALID, changing nothing, for out-of-range fields. */
pd_status pd_set_tuning(pd_env* env, const pd_tuning* tuning);
pd_status pd_get_tuning(const pd_env* env, pd_tuning* tuning);
/* Reset envs (mask: device uint8[N], NULL = all).  obs may be NULL. */
pd_status pd_reset(pd_env* env, const uint8_t* mask, void* obs, void* stream);
/* One env step for all N envs.
 *  actions : [N][A] float32 (or double when cfg.action_f64), A = 1 or 4
 *  obs     : [N][O] (O = 2 pure throttle, 5 PSO landing_burn), post-step (pre-auto-reset)
 *  reward  : [N]; done, truncated: uint8 [N]; trunc_id: int8 [N]   (any output may be NULL)
 *  noise   : optional [N][8] double standard normals replacing the Philox wind stream
 *            (sub-step k uses noise[2k], noise[2k+1]; test injection), NULL = Philox
 *  info    : optional [PD_N_INFO][N] (last sub-step values), NULL = not written */
pd_status pd_step(pd_env* env, const void* actions, void* obs, void* reward, uint8_t* done,
                  uint8_t* truncated, int8_t* trunc_id, const double* noise, void* info, void* stream);
/* n_steps consecutive pd_step calls over device-resident actions [n_steps][N][A], landing-burn
 * phases: obs [n_steps][N][O], reward [n_steps][N], done/truncated/trunc_id [n_steps][N] receive
 * every step's outputs (any may be NULL).  Replaces a Python loop over
 * rocket_environment_pre_wrap.step (base_environment.py:99-154) with fused launches: each launch
 * runs up to 128 steps (pd_tuning.step_fuse, 1..256) of every env in one kernel, so the LDS table staging and the
 * launch tail are paid once per launch, followed by the miss flush.  Results are bit-identical
 * to n_steps pd_step calls.  No host synchronisation. */
pd_status pd_step_n(pd_env* env, const void* actions, int32_t n_steps, void* obs, void* reward, uint8_t* done,
                    uint8_t* truncated, int8_t* trunc_id, void* stream);
/* pd_step_n with the info tap in the fused launches (ABI 9): info [n_steps][k][N] (handle
 * precision) receives, for every step, the k = popcount(info_mask) fields of pd_info_field whose
 * bit is set in info_mask, in pd_info_field order -- the visualisation episodes' selected keys
 * (rockets_physics.py:649-702) without a launch per step.  The same values as pd_step's info. */
pd_status pd_step_n_info(pd_env* env, const void* actions, int32_t n_steps, void* obs, void* reward, uint8_t* done,
                         uint8_t* truncated, int8_t* trunc_id, void* info, uint64_t info_mask, void* stream);
/* One SAC data-collection step (sac_pytorch_powered_descent.py:160-183 for N envs) in one
 * launch.  The action is sampled in the kernel from the caller's actor heads, as Actor.sample
 * does it (sac_pytorch.py:161-179) in binary32: a = tanh(mean + exp(clamp(log_std, log_std_min,
 * log_std_max)) * eps) * max_action, or tanh(mean) * max_action when eps is NULL (deterministic);
 * mean, log_std: float32 rows of head_stride floats (0: A), e.g. both heads of one [N][2A] GEMM
 * with log_std = mean + A and head_stride 2A; eps [N][A] float32 standard normals (e.g.
 * torch.randn).  Then the env steps
 * as pd_step (auto-reset per config) and the kernel epilogue writes, all float32 and any of them
 * NULL: action [N][A]; slab [N][2 S + A + 2], the replay buffer's transition row
 * state | action | reward | next_state | done (sac_pytorch.py:27-35; next_state the terminal
 * observation before any reset, done without truncation, as the driver stores them,
 * sac_pytorch_powered_descent.py:170-176); obs32 [N][S], the observation the actor sees next
 * (after any auto-reset).  RL landing-burn handles (PD_PHASE_PURE_THROTTLE / PD_PHASE_LANDING_BURN,
 * rtd RL or NONE, reference integrator) with float32 actions only.  No host synchronisation. */
pd_status pd_step_sac(pd_env* env, const float* mean, const float* log_std, int32_t head_stride, const float* eps,
                      float log_std_min, float log_std_max, float max_action, float* action, float* slab, float* obs32,
                      void* stream);
/* pd_step_sac with the rest of the collection step folded into the same launch (c5):
 *  heads   : [N][2A] float32, mean | log_std as Actor.forward's two heads leave them (unclamped),
 *            e.g. from pd_sac_actor
 *  deterministic != 0: a = tanh(mean) * max_action; else eps ~ N(0, 1) is drawn in the kernel
 *            (torch.randn's role in Normal.rsample, sac_pytorch.py:170-172): Philox4x32-10 keyed
 *            by the handle's seed, counter (env, episode, step, tag 19 + a/2), Box-Muller as the
 *            wind gusts; eps_out [N][A] (may be NULL) receives the draws
 *  ring    : the replay buffer's transition rows [capacity][2S + A + 2] float32 (sac_pytorch.py:
 *            12-49); with ring_state != NULL env i's row goes to (ring_state[0] + i) mod capacity,
 *            priorities[row] = *max_priority (PrioritizedReplayBuffer.add, sac_pytorch.py:76-83;
 *            priorities may be NULL), and the launch's last workgroup sets ring_state[0] (position)
 *            += N mod capacity, ring_state[1] (size) = min(size + N, capacity); ring_state[2] is
 *            its workgroup counter and must be 0 between launches (capacity >= N).  With
 *            ring_state NULL, ring is a [N][2S + A + 2] slab (pd_step_sac's).
 *  action, obs32: as pd_step_sac.  No host synchronisation; the position lives on the device, so
 *  a captured graph replays correctly. */
pd_status pd_step_sac_ring(pd_env* env, const float* heads, int32_t deterministic, float log_std_min,
                           float log_std_max, float max_action, float* eps_out, float* action, float* ring,
                           int64_t capacity, long long* ring_state, float* priorities, const float* max_priority,
                           float* obs32, void* stream);
/* The SAC Actor's forward pass (sac_pytorch.py:129-159) for n float32 observations [n][state_dim]
 * in one launch: Linear(S, H) ReLU, (n_hidden_layers - 1) x [Linear(H, H) ReLU] on MFMA
 * (v_mfma_f32_16x16x4_f32), then the mean and log_std heads into heads [n][2A] (mean | log_std,
 * unclamped: pd_step_sac_ring clamps).  params: a host array of 2 (n_hidden_layers + 2) device
 * pointers, the torch parameters in named_parameters() order (weight [out][in] row-major, bias):
 * shared_net layers, then mean, then log_std.  hidden 128, 256 or 512 (else PD_ERR_UNSUPPORTED),
 * state_dim <= 16, action_dim <= 8, n_hidden_layers <= 8; every parameter 16-byte aligned (else
 * PD_ERR_UNSUPPORTED).  f32 sums in another order than torch's GEMMs: equal to f32 rounding.  Runs
 * on the current HIP device. */
pd_status pd_sac_actor(int64_t n, int32_t state_dim, int32_t hidden, int32_t n_hidden_layers, int32_t action_dim,
                       const float* obs, const float* const* params, float* heads, void* stream);
/* The whole SAC collection step (sac_pytorch_powered_descent.py:160-183: actor.sample on the
 * current observation, env.step, buffer.add) in ONE launch: pd_sac_actor's forward pass
 * (sac_pytorch.py:129-159) runs in the step kernel's prologue for each workgroup's 16 envs, on
 * obs32 [N][S] as the previous step (or pd_observe) left it, then pd_step_sac_ring follows with
 * those heads (same arguments and semantics; obs32 is overwritten with the next observation).
 * state_dim / action_dim / hidden / n_hidden_layers / params as pd_sac_actor (state_dim and
 * action_dim must equal the handle's pd_obs_dim / pd_action_dim: PD_ERR_INVALID otherwise); heads
 * [N][2A] (may be NULL) receives the heads.  Handles stepping 16 lanes per env (the default up to
 * 4 096 envs) with hidden <= 256 take the single launch; others run pd_sac_actor +
 * pd_step_sac_ring (two launches, the same bits).  No host synchronisation. */
pd_status pd_step_sac_fused(pd_env* env, int32_t state_dim, int32_t action_dim, int32_t hidden,
                            int32_t n_hidden_layers, const float* const* params,
                            float* heads, int32_t deterministic, float log_std_min, float log_std_max,
                            float max_action, float* eps_out, float* action, float* ring, int64_t capacity,
                            long long* ring_state, float* priorities, const float* max_priority, float* obs32,
                            void* stream);
/* Multi-step rollout with device-resident actions [T][N][A]: the fused launches of pd_step_n
 * (per-step launches for the other phases), rewards accumulated into reward_sum [N] (may be
 * NULL), no per-step outputs.  No host synchronisation. */
pd_status pd_rollout(pd_env* env, const void* actions, int32_t n_steps, void* reward_sum,
                     void* stream);
/* PSO objective for a batch of particles, one env per particle, on the device:
 * pso_wrapped_env.objective_function (env_wrapped_ea.py:200-222) driven by simple_actor
 * (env_wrapped_ea.py:18-44) evaluated inside the step kernel.  Resets every env, then steps
 * each until done or truncated (or max_steps), accumulating fitness = -sum(reward).
 *  weights : [n_params][N] float32, parameter-major (named_parameters() order per particle);
 *            the rollout first copies them into chunks of four parameters ([ceil(P/4)][N][4],
 *            handle-owned) that the step kernel's actor reads with 16-byte loads
 *  n_params: PD_ACTOR_PARAMS_* for the handle's phase; the handle must have rtd = PD_RTD_PSO
 *  fitness : [N] (handle precision); steps: [N] int32 episode lengths (may be NULL)
 *  check_every: >0 = read the live-env count every that many steps (at least once per launch),
 *            stop early when all envs are done, and size later launches to the live count (one
 *            host sync per check); 0 = always max_steps steps over the full grid.
 * Each launch runs up to 64 fused steps (pd_tuning.policy_fuse); a finished episode's lanes freeze
 * and a wave whose episodes have all ended leaves the launch.  Grids beyond one chip round of lanes
 * step only the live envs (pd_tuning.policy_list): a compacted index list, rebuilt inside the step
 * kernel (wave ballot + prefix count, one atomic per wave).  Results do not depend on either.
 * A refill rollout (pd_tuning.policy_refill; the default for windless swarms) is ONE launch that
 * steps the whole swarm: it reads no live count, so check_every, policy_list and policy_list_at
 * apply only when refill is off (an explicit policy_list >= 0 or policy_list_at > 0 with
 * policy_refill -1 turns it off). */
pd_status pd_rollout_policy(pd_env* env, const float* weights, int32_t n_params, int32_t max_steps,
                            void* fitness, int32_t* steps, int32_t check_every, void* stream);
/* pd_rollout_policy with the weights already in the chunked layout, weights4 [ceil(n_params/4)][N][4]
 * float32 (chunk c of particle i holds parameters 4c .. 4c+3, zeros past n_params; 16-byte aligned):
 * the layout pd_pso_step_chunked writes, so the rollout skips its copy pass.  Same results. (ABI 11) */
pd_status pd_rollout_policy_chunked(pd_env* env, const float* weights4, int32_t n_params, int32_t max_steps,
                                    void* fitness, int32_t* steps, int32_t check_every, void* stream);
/* One PSO generation's particle update on the device (particle_swarm_optimisation.py:437-441
 * personal best, :515-519 update_velocity_with_local_best, :112-118 update_position), binary64:
 *   if fitness < best_fitness: best_position = position;  best_fitness = min(best_fitness, fitness)
 *   v = w v + c1 r1 (best_position - x) + c2 r2 (swarm_best[swarm] - x);  x = clip(x + v, lower, upper)
 * r1, r2: one uniform per particle and generation (Philox4x32-10 keyed by seed, counter
 * (particle_offset + p, generation)).  Arrays are parameter-major [dim][n_particles]; swarm_best
 * [n_swarms][dim]; swarm [n_particles] int32 subswarm ids; lower/upper [dim].  position_f32
 * (optional, [dim][n_particles]) receives the new positions as the float32 actor weights
 * pd_rollout_policy reads.  Device pointers; runs on the current HIP device. */
pd_status pd_pso_step(int64_t n_particles, int32_t dim, const double* fitness, double* best_fitness,
                      double* position, double* velocity, double* best_position, const double* swarm_best,
                      const int32_t* swarm, const double* lower, const double* upper, double w, double c1,
                      double c2, uint64_t seed, uint32_t generation, uint64_t particle_offset,
                      float* position_f32, void* stream);
/* pd_pso_step with the float32 copy in the chunked layout of pd_rollout_policy_chunked:
 * position_f32_chunked (required) [ceil(dim/4)][n_particles][4], zeros past dim.  One thread per
 * (chunk, particle) updates its four parameters with the same operations as pd_pso_step (the same
 * bits in position, velocity, best_position and best_fitness) and stores the chunk with one 16-byte
 * store. (ABI 11) */
pd_status pd_pso_step_chunked(int64_t n_particles, int32_t dim, const double* fitness, double* best_fitness,
                              double* position, double* velocity, double* best_position, const double* swarm_best,
                              const int32_t* swarm, const double* lower, const double* upper, double w, double c1,
                              double c2, uint64_t seed, uint32_t generation, uint64_t particle_offset,
                              float* position_f32_chunked, void* stream);
/* Per subswarm s < n_swarms, the first particle of minimal fitness among those with swarm[p] ==
 * s: the result of particle_swarm_optimisation.py:437-441's sequential `if fitness <
 * subswarm_best` over the subswarm's particles in order (a NaN fitness never wins, ties keep the
 * lower index): min_fitness [n_swarms] and its position min_position [n_swarms][dim] (from
 * position [dim][n_particles]); +inf and zeros for a subswarm with no particle of non-NaN fitness.
 * A two-pass segmented argmin over blocks of 1 024 particles; no host synchronisation.  scratch:
 * a device buffer of at least pd_pso_swarm_minima_scratch_bytes(n_particles, n_swarms) bytes for
 * the first pass's partials, owned by the caller (calls that may overlap need their own). */
size_t pd_pso_swarm_minima_scratch_bytes(int64_t n_particles, int32_t n_swarms);
pd_status pd_pso_swarm_minima(int64_t n_particles, int32_t dim, int32_t n_swarms, const double* fitness,
                              const int32_t* swarm, const double* position, double* min_fitness,
                              double* min_position, void* scratch, size_t scratch_bytes, void* stream);
/* The subswarm and global bests after a generation (particle_swarm_optimisation.py:442-444,
 * :474-477), on the device: subswarm s takes (min_fitness[s], min_position[s]) if strictly better;
 * then the first subswarm holding the smallest best replaces global_best(_fitness) if strictly
 * better.  swarm_best [n_swarms][dim], global_best [dim], the fitnesses [n_swarms] / [1]. */
pd_status pd_pso_update_bests(int32_t n_swarms, int32_t dim, const double* min_fitness, const double* min_position,
                              double* swarm_best_fitness, double* swarm_best, double* global_best_fitness,
                              double* global_best, void* stream);
/* Insert the aero neighbourhoods solved on device and still queued into the handle's tables
 * (one tiny kernel; a no-op when nothing is queued).  Since ABI 10 every step launch (pd_step,
 * pd_step_n, pd_step_sac*, pd_rollout) inserts the neighbourhoods it solved itself, by its last
 * workgroup, and pd_rollout_policy flushes its own: a caller never needs this call any more.
 * It stays for callers written against ABI <= 9 (their periodic flush finds the queue empty). */
pd_status pd_flush_misses(pd_env* env, void* stream);
/* Current observation (post-reset) [N][O]. */
pd_status pd_observe(pd_env* env, void* obs, void* stream);
/* State SoA [11][N] in the handle's precision. */
pd_status pd_get_state(pd_env* env, void* state, void* stream);
pd_status pd_set_state(pd_env* env, const void* state, void* stream);
/* Landing-burn actuator memory [3][N] (gimbal deg, left/right fin command rad). */
pd_status pd_get_actuators(pd_env* env, void* act, void* stream);
pd_status pd_set_actuators(pd_env* env, const void* act, void* stream);
/* g-load history of every env (base_environment.py:137-149: |v| of previous_state and the
 * g_loads_window list, oldest first): vprev [N], window [10][N] (handle precision), len [N]
 * (0..10 valid entries).  Teacher forcing and checkpoint/restore. */
pd_status pd_set_gload_window(pd_env* env, const void* vprev, const void* window, const uint8_t* len,
                              void* stream);
/* g-load history read back: vprev [N], window [10][N] (ring slots), len and head [N] (the oldest
 * entry is slot head when len == 10, slot 0 otherwise). */
pd_status pd_get_gload_window(pd_env* env, void* vprev, void* window, uint8_t* len, uint8_t* head, void* stream);
/* Per-env wind state: sigma_u, sigma_v [2][N] (double). */
pd_status pd_set_wind_sigmas(pd_env* env, const double* sig, void* stream);
/* Wind state (vonkarman.py:33-36 filter states, full_wind_model.py percentile): filters [4][N]
 * (u0 u1 v0 v1, handle precision), sigmas [2][N] (handle precision), profile [N] uint8
 * (percentile - 50).  Any pointer may be NULL.  pd_set_wind_state returns PD_ERR_INVALID, writing
 * nothing, if a profile byte is >= PD_N_WIND_PROFILES (it synchronises the stream to check). */
pd_status pd_get_wind_state(pd_env* env, void* filters, void* sigmas, uint8_t* profile, void* stream);
pd_status pd_set_wind_state(pd_env* env, const void* filters, const void* sigmas, const uint8_t* profile, void* stream);
/* Episode bookkeeping: episode counter and step-within-episode [N] uint32 (the Philox counter
 * words of the wind and reset draws), truncation id [N] int8.  Any pointer may be NULL. */
pd_status pd_get_counters(pd_env* env, uint32_t* episode, uint32_t* step, int8_t* trunc_id, void* stream);
pd_status pd_set_counters(pd_env* env, const uint32_t* episode, const uint32_t* step, const int8_t* trunc_id,
                          void* stream);
/* Checkpoint of every per-env buffer (state, g-load window, actuator memory, wind, counters,
 * aero caches, episode flags) as one opaque device blob of pd_checkpoint_size() bytes: save
 * into, load from a device buffer.  Restoring into a handle of the same configuration continues
 * bit-identically (the Philox draws depend only on (seed, env, episode, step)).  Loading a blob
 * whose wind profile bytes are out of range returns PD_ERR_INVALID and loads nothing. */
size_t pd_checkpoint_size(const pd_env* env);
pd_status pd_checkpoint_save(pd_env* env, void* blob, void* stream);
pd_status pd_checkpoint_load(pd_env* env, const void* blob, void* stream);
/* Counters since create: aero-table misses solved on device, NaN guard hits. Host sync. */
pd_status pd_counters(pd_env* env, int64_t* rbf_misses, int64_t* table_entries_cd,
                      int64_t* table_entries_cl, int64_t* nan_events);
/* The handle's ISA atmosphere (endo_atmospheric_model, atmosphere_dynamics.py:5-27) at n device
 * altitudes [n] (handle precision): out [3][n] = density, pressure, speed of sound.  Used by the
 * facade's maximum_velocity (env_wrapped_rl_pytorch.py:60-66). */
pd_status pd_atmosphere(pd_env* env, const void* altitude, void* out, int64_t n, void* stream);
/* All device statistics words (up to n, at most PD_N_STATS): 0 misses, 1 NaN events, 2/3 table
 * entries C_D/C_L, 16 solved neighbourhoods not queued (queue full; solved again until a later
 * flush).  Workload counters of the step kernel, summed over every launch made with counting on
 * (pd_count_work) since create:
 * 32 env sub-steps inside the gust band (stochastic wind, y < 15 km), 33 in-kernel auto-resets;
 * with 2 lanes per env (one table query per lane and sub-step): 34 queries on a clamped line,
 * 35 queries whose candidate neighbourhood was verified by the swap search, 36 queries evaluated
 * from a Taylor piece, 37 by the balanced chunk sums, 38 missed (device solve), 39 balanced-sum
 * rounds, 40 interior queries in a refined grid cell, 41 ... in a sub-cell split by a bisector,
 * 42 / 43 wave sub-steps with at least one such query, 44 queries evaluated from a cell piece,
 * 45 wave sub-steps holding both clamped-line and interior queries.  Host sync. */
#define PD_N_STATS 48
pd_status pd_stats(pd_env* env, int64_t* out, int32_t n);
/* Workload counting (pd_stats words 32-45) on (enable != 0) or off (the default) for the handle's
 * following step launches with 2 lanes per env (the default above 16 384 envs; other launches
 * count nothing).  A diagnostic: on, the launches run a counting instantiation of the step kernel
 * (a ballot and an LDS add per counter per sub-step, a few per cent slower); off, the product
 * kernel has no counting code.  Results do not change. */
pd_status pd_count_work(pd_env* env, int32_t enable);
/* Cell pieces of one table (0: C_D, 1: C_L), host only (no device needed): the polynomial + exact-
 * term records that binary64 handles evaluate interior queries from (not a
 * reference interface: the test hook behind them).  Built once per process and table.
 * out[0] pieces, [1] rejected by the build's check, [2] worst checked error relative to
 * sum |c_j phi_j|, [3] build seconds, [4] records, [5] nm, [6] na, [7] a0, [8] a1 (the grid),
 * [9] degree, [10] exact terms, [11] record stride, [12] pieces the binary32 check rejects (of the
 * binary64-valid), [13] its worst error relative to sum |c_j phi_j| + |s|, [14] / [15] exact cells
 * with a valid binary64 / binary32 piece; piece >= 0 (an exact cell's piece is at its
 * cell index im na + ia): its record at out[16 ...] (n_out >= 16 + stride). */
pd_status pd_cell_piece_info(const pd_params* params, int32_t table, int64_t piece, double* out, int32_t n_out);
/* The step kernel's tabulated ISA atmosphere (atmosphere_dynamics.py:5-27), built and evaluated on
 * the host in the device's order and precision (test hook; no device needed): rho, p, a into
 * atm_out [n_alt][3] at geometric altitudes alt; max_rel: the builder's worst relative error
 * against the long double closed form. */
pd_status pd_atm_table(const pd_params* params, int32_t precision, const double* alt, int64_t n_alt,
                       double* atm_out, double* max_rel);
/* Observation / action widths of the handle. */
int pd_obs_dim(const pd_env* env);
int pd_action_dim(const pd_env* env);

#ifdef __cplusplus
}
#endif
#endif
