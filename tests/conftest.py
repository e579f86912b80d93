import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

ATMOSPHERE_GZ = os.path.join(ROOT, "airiceraytracing_amd", "data", "Atmosphere.dat.gz")
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running (full-size) case")


@pytest.fixture(scope="session")
def atmosphere_text():
    import gzip
    with open(ATMOSPHERE_GZ, "rb") as f:
        return gzip.decompress(f.read())


@pytest.fixture(scope="session")
def oracle_medium(atmosphere_text):
    import oracle
    return oracle.parse_atmosphere(atmosphere_text, oracle.PI_MULTIRAY)


@pytest.fixture(scope="session")
def oracle_medium_py(atmosphere_text):
    import oracle
    return oracle.parse_atmosphere(atmosphere_text, oracle.PI_EXACT)
