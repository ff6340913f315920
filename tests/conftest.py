import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running case")


@pytest.fixture(scope="session")
def oracle():
    from oracle import pyoracle
    pyoracle.build()
    return pyoracle


@pytest.fixture(scope="session")
def mdx():
    import motion_detection_amd as m
    if not os.path.exists(m.LIB_PATH):
        m.build()
    m.lib()
    return m


@pytest.fixture(scope="session")
def ctx(mdx):
    c = mdx.Context(0, 1920, 1080, 1)
    yield c
    c.close()
