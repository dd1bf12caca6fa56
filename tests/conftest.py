"""Shared pytest configuration: the `gpu` marker and repo paths."""
import os
import sys
import threading
import time

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "lzma-java_amd")
for p in (REPO, PKG, os.path.join(REPO, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")


def pytest_collection_modifyitems(config, items):
    # gpu tests are selected explicitly with -m gpu; when a run selects them
    # without a device present they must fail loudly, not skip silently.
    pass


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(REPO, "tests", "golden")


@pytest.fixture
def heartbeat(capsys):
    """A line on the real stdout every 30 s (output capture suspended for it) while a
    long GPU call runs: a single-stream encode of tens of MiB is one wave's serial
    parse and takes minutes, and a run that prints nothing for minutes looks hung."""
    stop = threading.Event()

    def beat():
        t0 = time.time()
        while not stop.wait(30.0):
            with capsys.disabled():
                print("\n[heartbeat] %.0f s" % (time.time() - t0), flush=True)

    th = threading.Thread(target=beat, daemon=True)
    th.start()
    yield
    stop.set()
    th.join()
