"""CPU checks of the C ABI: libpdenv.so loads without a GPU, exports every symbol the
header declares, and the ctypes mirror of pd_params / pd_config has the C layout."""
import ctypes as C
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    txt = open(os.path.join(REPO, "include", "pdenv.h")).read()
    return sorted(set(re.findall(r"^\s*(?:[\w\*\s]+?)\s\**(pd_\w+)\(", txt, re.M)))


def test_library_exports_header_symbols():
    import pdenv
    from pdenv import _lib
    L = pdenv.load()
    syms = header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(L, s), f"{s} declared in include/pdenv.h but not exported"
    assert set(_lib.EXPORTS) <= set(syms)


def test_struct_layout_and_abi():
    import pdenv
    from pdenv import _lib
    L = pdenv.load()
    assert L.pd_abi_version() == _lib.ABI_VERSION == 11
    assert L.pd_sizeof_params() == C.sizeof(_lib.PdParams)
    assert L.pd_sizeof_config() == C.sizeof(_lib.PdConfig)


def test_argument_checks_before_any_launch():
    """Entry points refuse bad arguments before touching the device (callable without a GPU;
    the pointers below are never dereferenced): a misaligned SAC actor parameter, a missing or
    short pd_pso_swarm_minima scratch, a null handle's tuning."""
    import pdenv
    from pdenv import _lib
    L = pdenv.load()
    vp = C.c_void_p
    params = (vp * 8)(*([0x10000] * 7 + [0x10004]))          # the last one 4-byte aligned only
    st = L.pd_sac_actor(64, 2, 256, 2, 1, vp(0x10000), params, vp(0x10000), None)
    assert st == _lib.PD_ERR_UNSUPPORTED and b"aligned" in L.pd_last_error()
    params[7] = 0
    assert L.pd_sac_actor(64, 2, 256, 2, 1, vp(0x10000), params, vp(0x10000), None) == _lib.PD_ERR_INVALID
    need = L.pd_pso_swarm_minima_scratch_bytes(5000, 3)
    assert need == 5 * 3 * 16                                  # 5 blocks of 1 024 particles x 3 subswarms
    for scratch, nb in ((None, 0), (vp(0x10000), need - 8), (vp(0x10004), need)):
        st = L.pd_pso_swarm_minima(5000, 10, 3, vp(0x10000), vp(0x10000), vp(0x10000), vp(0x10000), vp(0x10000),
                                   scratch, nb, None)
        assert st == _lib.PD_ERR_INVALID and b"scratch" in L.pd_last_error()
    # pd_pso_step_chunked: the chunked copy is required and 16-byte aligned
    a = [vp(0x10000)] * 9
    for x32c in (None, vp(0x10008)):
        st = L.pd_pso_step_chunked(5000, 372, *a, 0.7, 1.5, 1.5, 1, 0, 0, x32c, None)
        assert st == _lib.PD_ERR_INVALID and b"chunked" in L.pd_last_error()
    assert L.pd_rollout_policy_chunked(None, vp(0x10000), 372, 10, vp(0x10000), None, 0, None) == _lib.PD_ERR_INVALID
    t = _lib.PdTuning(128, 64, 2, -1, 0.0, -1, 0, -1, 0)
    assert L.pd_set_tuning(None, C.byref(t)) == _lib.PD_ERR_INVALID
    assert L.pd_get_tuning(None, C.byref(t)) == _lib.PD_ERR_INVALID


def test_no_gpu_create_fails_loudly():
    """Without a HIP device the product refuses to run (no CPU fallback)."""
    import torch
    import pdenv
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    with pytest.raises(pdenv.PdError):
        pdenv.PoweredDescentEnv(4)


def test_params_pack_consistency():
    import numpy as np
    import pdenv
    p = pdenv.Params()
    s = p.struct
    assert s.cd.n_pts == 191 and s.cl.n_pts == 138
    assert sum(s.cd.col_len[k] for k in range(5)) == 191
    # stage-2 inertia closure constants
    assert abs(s.x_dry - 5.50221) < 1e-5 and abs(s.I_dry - 20784441.14) < 0.01
    assert np.isclose(s.C_gust_x, 100.1717, atol=1e-4)
    assert len(p.keys_cd) > 0 and len(p.keys_cl) > 0
    # every key decodes to exactly 50 points
    for k in list(p.keys_cd) + list(p.keys_cl[:500]):
        k = int(k)
        tot = sum((k >> (12 * c + 6)) & 63 for c in range(5))
        assert tot == 50


def test_phase_pairs_the_reference_cannot_step():
    """landing_burn_ACS, RL flip-over and PSO outside the landing burns construct (no GPU needed)
    and raise TypeError at step(), as the reference's envs do; PSO + Pcontrol/ACS fails the
    reference's compile_rtd_pso assertion at construction."""
    import pdenv
    for phase, mode in (("landing_burn_ACS", "rl"), ("flip_over_boostbackburn", "rl"), ("subsonic", "pso"),
                        ("ballistic_arc_descent", "pso")):
        env = pdenv.PoweredDescentEnv(4, phase, mode=mode)
        assert env.reset() is None
        with pytest.raises(TypeError):
            env.step(None)
    with pytest.raises(AssertionError):
        pdenv.PoweredDescentEnv(4, "landing_burn_pure_throttle_Pcontrol", mode="pso")
    from pdenv.wrappers import rl_wrapped_env_pytorch
    w = rl_wrapped_env_pytorch("landing_burn_ACS", trajectory_length=100, discount_factor=0.99)
    assert (w.state_dim, w.action_dim) == (5, 3)
    with pytest.raises(TypeError):
        w.step([0.0, 0.0, 0.0])


def test_params_phases():
    """The other phases' constants from the pack (tools/make_param_pack.py "phases")."""
    import numpy as np
    import pdenv
    p = pdenv.Params()
    s = p.struct
    assert s.n_engines_stage1 == 42 and s.n_ref == 864
    assert np.allclose(p.state0_of("subsonic")[:5], [0, 1.5, 0, 0, np.pi / 2])
    assert np.allclose(p.state0_of("landing_burn_pure_throttle_Pcontrol"), p.state0)
    ys = np.array(s.ref_y[:s.n_ref])
    assert np.all(np.diff(ys) > 0)
    assert abs(s.terminal_mach[1] - 4.11865) < 1e-4
