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


def _lib_stamp(path):
    """The src_sha256 compiled into a libmdx.so (csrc/Makefile's mdx_build_info string), read from
    the file's bytes without loading it."""
    with open(path, "rb") as f:
        data = f.read()
    i = data.find(b"src_sha256=")
    return data[i + 11:i + 75].decode() if i >= 0 else None


@pytest.fixture(scope="session")
def mdx():
    """The in-tree libmdx.so, rebuilt from the tree (make -B) whenever it is missing or its stamp
    does not match the sources here, so a test never runs a library built from other sources."""
    import motion_detection_amd as m
    if os.environ.get("MDX_LIB_PATH"):
        # an explicitly chosen library (scripts/build_variant.sh A/B runs: this tree's sources
        # with extra -D flags, so its stamp differs by construction)
        m.lib()
        return m
    if not os.path.exists(m.LIB_PATH) or _lib_stamp(m.LIB_PATH) != m._lib.source_sha256():
        m.build()
    m.lib()
    assert m._lib.build_info()["matches_tree"], "libmdx.so does not match the sources in the tree"
    return m


@pytest.fixture(scope="session")
def ctx(mdx):
    c = mdx.Context(0, 1920, 1080, 1)
    yield c
    c.close()
