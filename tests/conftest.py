import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cassandra-accord_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")


@pytest.fixture(scope="session")
def oracle():
    import pyoracle
    pyoracle.build()
    return pyoracle


@pytest.fixture(autouse=True)
def _device_guard_bands(request):
    """AD_GUARD=1|2 (debug, accord_deps.h ad_debug_guard_check): after every GPU test, no device
    allocation's guard band may have been overwritten -- a write past the end of a buffer fails the test
    that did it instead of corrupting a later one."""
    yield
    if not os.environ.get("AD_GUARD") or request.node.get_closest_marker("gpu") is None:
        return
    import gc
    gc.collect()
    from accord_deps import native
    bad, report = native.guard_check()
    assert bad == 0, "device guard bands overwritten:\n" + report
