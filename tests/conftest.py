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


def golden_names():
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN_DIR, "*.npz")))


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
