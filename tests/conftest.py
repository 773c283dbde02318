import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); parity tests of the HIP path")
    config.addinivalue_line("markers", "slow: long-running CPU oracle case")


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import oracle
    if not os.path.exists(oracle.LIB):
        oracle.build()
    return oracle


@pytest.fixture(scope="session")
def gpu_lib():
    lib_path = os.path.join(ROOT, "libmems_amd", "libmums_hip.so")
    if not os.path.exists(lib_path):
        subprocess.run(["make", "-s", "-j8", "-C", os.path.join(ROOT, "libmems_amd")], check=True)
    import libmems_amd
    libmems_amd.load_library()
    return libmems_amd
