"""pdenv -- MI355X-native vectorised powered-descent environment.

Drop-in for the env hot path of JvanZyl1/PSSO-SAC-for-powered-descent: the physics step,
ISA atmosphere, exact local-RBF aerodynamics, grid fins, wind and the RL/PSO
reward/termination run as HIP kernels in libpdenv.so (C ABI: include/pdenv.h).
"""
from ._lib import PdError, INFO_FIELDS, load  # noqa: F401
from .env import PoweredDescentEnv  # noqa: F401
from .params import Params, load_pack  # noqa: F401

__all__ = ["PoweredDescentEnv", "Params", "load_pack", "PdError", "INFO_FIELDS", "load"]
