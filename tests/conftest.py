import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP C-ABI)")


@pytest.fixture(scope="session")
def golden():
    import json

    d = os.path.join(ROOT, "tests", "golden")
    with open(os.path.join(d, "kat_published.json")) as f:
        kat = json.load(f)
    with open(os.path.join(d, "openssl_vectors.json")) as f:
        ossl = json.load(f)
    return kat, ossl
