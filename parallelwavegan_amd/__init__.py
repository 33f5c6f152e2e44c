"""MI355X-native Parallel WaveGAN generator inference engine.

Public surface (mirrors parallel_wavegan.models for the generator hot path):
  ParallelWaveGANGenerator  drop-in module, forward/inference run on HIP kernels
  Engine                    lower-level batch engine over the C-ABI (include/pwg.h)
"""

from .engine import Engine, HostHandle  # noqa: F401
from .models import ParallelWaveGANGenerator  # noqa: F401

__version__ = "0.1.0"
