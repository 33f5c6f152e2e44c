"""MI355X-native Parallel WaveGAN generator inference engine.

Public surface (mirrors parallel_wavegan.models for the generator hot path):
  ParallelWaveGANGenerator  drop-in module, forward/inference run on HIP kernels
  Engine                    lower-level batch engine over the C-ABI (include/pwg.h)
  GraphedRun                one plan's forward captured as a HIP graph (pwg_graph_create) for
                            repeated shapes
"""

from .engine import Engine, GraphedRun, HostHandle  # noqa: F401
from .models import ParallelWaveGANGenerator  # noqa: F401

__version__ = "0.1.0"
