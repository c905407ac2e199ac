"""MI355X-native Procgen step path (coinrun first) behind the reference's libenv C ABI.

Import path: add ``<repo>/procgen-1_amd`` to ``sys.path``; ``import procgen_amd``.
"""
from .env import ENV_NAMES, ProcgenGym3Env, BaseProcgenEnv, ProcgenError  # noqa: F401
from . import catalog  # noqa: F401
from .adapters import ProcgenEnv, ToBaselinesVecEnv, ToGymEnv, make_env, register_environments  # noqa: F401

__all__ = ["ProcgenGym3Env", "BaseProcgenEnv", "ProcgenError", "ENV_NAMES", "catalog", "ProcgenEnv",
           "ToBaselinesVecEnv", "ToGymEnv", "make_env", "register_environments"]
