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
    assert L.pd_abi_version() == 1
    assert L.pd_sizeof_params() == C.sizeof(_lib.PdParams)
    assert L.pd_sizeof_config() == C.sizeof(_lib.PdConfig)


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
