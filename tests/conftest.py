import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


_CONFIG = None


def pytest_configure(config):
    global _CONFIG
    _CONFIG = config
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) and libmml_hip.so")


def progress(msg):
    """A progress line written past pytest's output capture, so a long test (minutes of oracle
    work) shows it is alive under a plain `pytest -q` too."""
    cm = _CONFIG.pluginmanager.getplugin("capturemanager") if _CONFIG is not None else None
    if cm is None:
        print(msg, flush=True)
        return
    with cm.global_and_fixture_disabled():
        print(msg, flush=True)


@pytest.fixture(scope="session", autouse=True)
def _built():
    """Build libmml_hip.so / the oracle if they are missing (never a fallback: a build failure
    fails the session)."""
    so = os.path.join(ROOT, "mymedialite_amd", "lib", "libmml_hip.so")
    ora = os.path.join(ROOT, "oracle", "build", "libmml_oracle.so")
    if not (os.path.exists(so) and os.path.exists(ora)):
        import __graft_entry__
        __graft_entry__.build()
    yield
