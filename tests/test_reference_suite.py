"""Runs the reference-style multi-rank tests under the framework launcher with
the rank counts the reference uses (README.md:189,200,212): get_info at 8
ranks, forward/backward collects at 4 ranks."""
import pytest

from _launch import py, run_ranks


@pytest.mark.parametrize("n,path", [
    (8, "tests/test_get_info.py"),
    (4, "tests/test_transformer_forward.py"),
    (4, "tests/test_transformer_backward.py"),
])
def test_reference_mpi_suite(n, path):
    r = run_ranks(n, py("-m", "pytest", path, "--with-mpi", "-q", "-p", "no:cacheprovider"), timeout=240)
    assert "passed" in r.stdout
