import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels through libcfa.so)")


def load_golden(name: str) -> dict:
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def ragged(keys, lens, vals):
    """Rebuild {tuple(key): list} from the (keys, lengths, concatenated values) fixture form."""
    out = {}
    pos = 0
    for key, n in zip(keys, lens):
        out[tuple(int(x) for x in key)] = [int(v) for v in vals[pos:pos + n]]
        pos += n
    return out


def normwise_close(y, r, rtol=1e-5):
    """The north-star tolerance: max|y - r| <= rtol * max|r| per tensor."""
    y = np.asarray(y, dtype=np.float64)
    r = np.asarray(r, dtype=np.float64)
    if y.shape != r.shape:
        return False
    scale = np.max(np.abs(r)) if r.size else 0.0
    return bool(np.max(np.abs(y - r), initial=0.0) <= rtol * max(scale, np.finfo(np.float32).tiny))


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from federated_amd.engine import get_engine
    return get_engine()
