"""Shared pytest setup.

Markers: ``gpu`` = needs a real MI355X (run with ``-m gpu`` on the GPU box);
everything else runs on CPU here.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "metabodecon-rust_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: test needs an MI355X GPU (HIP device)")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


class EngineEnv:
    """MDG_* engine switches for a test: set in the environment and re-read by every
    live engine context (the engine reads the environment only when a context is
    created or on mdg_ctx_reload_switches, never on a call's path)."""

    def __init__(self, mp):
        self.mp = mp

    def setenv(self, name, value):
        self.mp.setenv(name, value)
        self.reload()

    def delenv(self, name, raising=True):
        self.mp.delenv(name, raising=raising)
        self.reload()

    @staticmethod
    def reload():
        nat = sys.modules.get("metabodecon._native")
        if nat is not None:
            nat.reload_switches()


@pytest.fixture
def engine_env(monkeypatch):
    e = EngineEnv(monkeypatch)
    yield e
    monkeypatch.undo()  # the switches the other tests expect, then re-read them
    e.reload()
