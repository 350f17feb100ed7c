import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
import maskclustering_amd  # noqa: E402,F401  (HIP queue setting before the first HIP call)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI library)")


GOLDEN = os.path.join(REPO, "tests", "golden")
CASES = ["tiny_scannet", "edge_scannet", "edge_scannetpp", "c1_scannet", "c1_scannetpp", "mid_tasmap"]


def load_case(name):
    import numpy as np
    return dict(np.load(os.path.join(GOLDEN, name + ".npz")))


@pytest.fixture(scope="session")
def golden_cases():
    return {n: load_case(n) for n in CASES}
