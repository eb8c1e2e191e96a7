import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "zk-odst_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden", "blake2f_golden.json")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")


@pytest.fixture(scope="session")
def orc():
    import oracle

    oracle.lib()
    return oracle


@pytest.fixture(scope="session")
def golden():
    import json

    with open(GOLDEN) as fh:
        return json.load(fh)


@pytest.fixture(scope="session")
def engine():
    import b2f

    eng = b2f.Engine(0)
    yield eng
    eng.close()


@pytest.fixture(scope="session")
def diag_engine():
    """An engine on the diagnostics build (libb2f_diag.so): fused band sizes other than the
    product's, kernel floors. Never the product path."""
    import b2f

    eng = b2f.Engine(0, diag=True)
    yield eng
    eng.close()


def random_inputs(n, rounds_choices=(12,), seed=1):
    import b2f

    rng = np.random.default_rng(seed)
    x = np.zeros(n, dtype=b2f.INPUT_DTYPE)
    x["h"] = rng.integers(0, 2**64, (n, 8), dtype=np.uint64)
    x["m"] = rng.integers(0, 2**64, (n, 16), dtype=np.uint64)
    x["t"] = rng.integers(0, 2**64, (n, 2), dtype=np.uint64)
    x["f"] = rng.integers(0, 2, n)
    x["rounds"] = rng.choice(np.asarray(rounds_choices, dtype=np.uint32), n)
    return x


def words(hexlist):
    return np.array([int(w, 16) for w in hexlist], dtype=np.uint64)
