"""pytest configuration.

* ``gpu`` marker: needs an MI355X (the driver runs ``-m gpu`` on a GPU box and
  ``-m "not gpu"`` here).
* ``mpi`` marker + ``--with-mpi`` flag: the pytest-mpi contract the reference
  tests use (README.md:189,200,212: ``mpirun -n N python -m pytest ... --with-mpi``).
  pytest-mpi is not installed in this image, so the flag and marker are
  provided here; without the flag, mpi tests are skipped (they only make sense
  inside a multi-rank launch — tests/test_reference_suite.py launches them).
"""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_addoption(parser):
    parser.addoption("--with-mpi", action="store_true", default=False,
                     help="run tests marked mpi (inside scripts/mpirun -n N)")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: requires an AMD MI355X GPU")
    config.addinivalue_line("markers", "mpi: multi-rank test, run under scripts/mpirun with --with-mpi")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    if config.getoption("--with-mpi"):
        return
    skip = pytest.mark.skip(reason="needs --with-mpi (run under scripts/mpirun -n N)")
    for item in items:
        if "mpi" in item.keywords:
            item.add_marker(skip)
