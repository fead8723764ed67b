"""drpo_amd -- MI355X-native hot path of Distributional Reachability Policy Optimization.

Drop-in for the reference's hot-path API (src/smbpo.py, src/ssac.py,
src/dynamics.py, src/sampling.py, src/policy.py): same classes, Config fields and
state_dict layout; compute runs in libdrpo_hip.so (hand-written HIP for gfx950).
"""
from .config import BaseConfig, Configurable, Optional, Require  # noqa: F401
from .buffers import SampleBuffer, SafetySampleBuffer, ConstraintSafetySampleBuffer, DummyModuleWrapper  # noqa
from .dynamics import BatchedGaussianEnsemble, Normalizer  # noqa: F401
from .policy import SquashedGaussianPolicy  # noqa: F401
from .ssac import SSAC, CriticEnsemble, ConstraintCritic, MLPMultiplier  # noqa: F401
from .smbpo import SMBPO  # noqa: F401
from .rng import DeviceNoise, TapeNoise  # noqa: F401
from .torch_util import set_seed, device  # noqa: F401
from .policy import UniformPolicy  # noqa: F401,E402
from .checkpoint import CheckpointableData, Checkpointer  # noqa: F401,E402
from .envs import ProductEnv  # noqa: F401,E402
from .sampling import sample_episodes_batched  # noqa: F401,E402
