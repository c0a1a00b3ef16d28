import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def _build_lib():
    """(Re)build libwsgpu.so if stale, before any test module imports snf4j_amd
    (build.py is loaded by path: the package import would load the old library)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("_wsgpu_build", os.path.join(ROOT, "snf4j_amd", "build.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.build()


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libwsgpu.so on the device)")
    _build_lib()


@pytest.fixture(scope="session")
def oracle():
    from oracle import pyoracle
    pyoracle.build()
    return pyoracle
