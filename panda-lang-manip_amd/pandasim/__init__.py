"""pandasim — MI355X-native batched Panda manipulation envs (PandaReach/Push/Slide/PickAndPlace/Stack/Flip-v3).

Host layer over libpandasim.so (HIP, gfx950).  See DESIGN.md.
"""
from ._lib import PandasimError, lib
from .core import PyBulletRobot, RobotTaskEnv, Task, TimeLimit
from .envs import REGISTRY, PandaVecEnv, make
from .panda_tasks import (PandaFlipEnv, PandaPickAndPlaceEnv, PandaPushEnv, PandaReachEnv, PandaSlideEnv,
                          PandaStackEnv)
from .robots import Panda
from .sim import PandaSim
from .tasks import Flip, PickAndPlace, Push, Reach, Slide, Stack

__all__ = ["make", "PandaVecEnv", "PandaSim", "REGISTRY", "PandasimError", "lib", "PyBulletRobot", "Task",
           "RobotTaskEnv", "TimeLimit", "Panda", "Reach", "Push", "PickAndPlace", "PandaReachEnv", "PandaPushEnv",
           "PandaPickAndPlaceEnv", "Slide", "Stack", "Flip", "PandaSlideEnv", "PandaStackEnv", "PandaFlipEnv"]
__version__ = "0.1.0"
