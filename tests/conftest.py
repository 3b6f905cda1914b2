import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "ert-conditional-diffusion-model_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG, GOLDEN):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and libertdiff_hip.so")


def load_golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


@pytest.fixture(scope="session")
def golden_weights():
    return dict(load_golden("weights_seed42.npz"))


@pytest.fixture(scope="session")
def fwd_kat():
    return load_golden("forward_kat.npz")


@pytest.fixture(scope="session")
def sampler_kat():
    return load_golden("sampler_kat.npz")


@pytest.fixture(scope="session")
def sched_kat():
    return load_golden("schedule.npz")


@pytest.fixture(scope="session")
def train_kat():
    return load_golden("train_kat.npz")


@pytest.fixture(scope="session")
def postproc_kat():
    return load_golden("postproc_kat.npz")


@pytest.fixture(scope="session")
def postproc_chain_kat():
    return load_golden("postproc_chain_kat.npz")


@pytest.fixture(scope="session")
def cuda_dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    return torch.device("cuda", 0)


@pytest.fixture(scope="session")
def gpu_model(golden_weights, cuda_dev):
    """Seed-42 reference weights loaded into the ertdiff model on the GPU."""
    import torch
    import ertdiff
    m = ertdiff.ConditionalDiffusionModel(29, 128)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in golden_weights.items()})
    return m.to(cuda_dev).eval()


@pytest.fixture(scope="session")
def kde_kat():
    return load_golden("kde_kat.npz")


@pytest.fixture(scope="session")
def unet_sampler_kat():
    return load_golden("unet_sampler_kat.npz")


def record_error(name: str, value: float) -> None:
    """Append a measured parity error to gpurun_out/parity_errors.jsonl (the
    numbers DESIGN.md quotes next to each gate); never fails a test."""
    import json
    try:
        d = os.path.join(ROOT, "gpurun_out")
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, "parity_errors.jsonl"), "a") as f:
            f.write(json.dumps({"test": name, "value": float(value)}) + "\n")
    except OSError:
        pass
