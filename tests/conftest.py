"""Shared test set-up: marker registration, import paths and in-tree builds."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "i-emic_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the C ABI on cuda:0)")
    config.addinivalue_line("markers", "slow: larger CPU cases")


def _make(path):
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, path)], check=True,
                   stdout=subprocess.DEVNULL)


@pytest.fixture(scope="session")
def oracle_lib():
    """oracle/_build/liboracle.so (the CPU checker)."""
    _make("oracle")
    from oracle import oracle as orc
    return orc


@pytest.fixture(scope="session")
def emul():
    """tests/_build/libstencil_emul.so (device assembly logic run on the CPU)."""
    _make("tests/emul")
    from helpers import Emul
    return Emul
