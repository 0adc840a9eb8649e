"""pandasim — MI355X-native batched Panda manipulation envs (PandaReach/Push/PickAndPlace-v3).

Host layer over libpandasim.so (HIP, gfx950).  See DESIGN.md.
"""
from ._lib import PandasimError, lib
from .envs import REGISTRY, PandaVecEnv, make
from .sim import PandaSim

__all__ = ["make", "PandaVecEnv", "PandaSim", "REGISTRY", "PandasimError", "lib"]
__version__ = "0.1.0"
