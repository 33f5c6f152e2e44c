import glob
import json
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

GOLDEN_DIR = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X); run with -m gpu")


def load_golden(name):
    with np.load(os.path.join(GOLDEN_DIR, name + ".npz"), allow_pickle=False) as z:
        d = {k: z[k] for k in z.files}
    d["meta"] = json.loads(str(d["meta"]))
    return d


def _all_golden():
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN_DIR, "*.npz")))


def _meta(name):
    with np.load(os.path.join(GOLDEN_DIR, name + ".npz"), allow_pickle=False) as z:
        return json.loads(str(z["meta"]))


def golden_names():
    """ParallelWaveGAN fixtures."""
    return [n for n in _all_golden() if "vocoder" not in _meta(n)]


def vocoder_golden_names():
    """MelGAN / multi-band MelGAN / HiFiGAN fixtures (make_golden.py --vocoders)."""
    return [n for n in _all_golden() if "vocoder" in _meta(n)]


def vocoder_holder(meta):
    """(drop-in module with the fixture's weights loaded, generator params, folded state dict)."""
    import torch

    from parallelwavegan_amd import configs, synthetic
    from parallelwavegan_amd.engine import fold_weight_norm
    from parallelwavegan_amd.hifigan import HiFiGANGenerator
    from parallelwavegan_amd.melgan import PQMF, MelGANGenerator

    cls_name, params = configs.vocoder_params(meta["vocoder"])
    cls = {"MelGANGenerator": MelGANGenerator, "HiFiGANGenerator": HiFiGANGenerator}[cls_name]
    m = cls(**configs.vocoder_params(meta["vocoder"])[1])
    if not meta["weight_norm"]:
        m.remove_weight_norm()
    sd = synthetic.make_module_state_dict(m, seed=meta["weight_seed"])
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    if meta["options"].get("pqmf"):
        m.pqmf = PQMF(params["out_channels"])
    return m.eval(), params, fold_weight_norm(sd)


def golden_params(meta):
    from parallelwavegan_amd import configs

    return configs.generator_params(meta["config"], **meta["overrides"])


def golden_state(meta, params):
    from parallelwavegan_amd import synthetic

    return synthetic.make_state_dict(params, seed=meta["weight_seed"], weight_norm=meta["weight_norm"])


@pytest.fixture(scope="session")
def built_lib():
    """Build (if stale) and load libpwg_hip.so."""
    from parallelwavegan_amd import _lib

    _lib.build()
    return _lib.load()


@pytest.fixture(scope="session")
def cuda_device():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but no ROCm GPU is visible")
    return torch.device("cuda:0")
