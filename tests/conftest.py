import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "mpi.jl_amd"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: beyond parity coverage (repeats, soaks, long late-rank waits); "
                                       "deselected unless --run-slow or MPIGX_RUN_SLOW=1")


def pytest_addoption(parser):
    parser.addoption("--run-slow", action="store_true", default=False,
                     help="also run tests marked slow (deselected by default)")


def pytest_collection_modifyitems(config, items):
    """The GPU suite's budget: `-m gpu` on the driver's
    box must stay under ~600 s, so cases beyond parity coverage are marked
    `slow` and deselected unless asked for (tests/test_suite_budget_cpu.py
    keeps every parity case unmarked)."""
    if config.getoption("--run-slow") or os.environ.get("MPIGX_RUN_SLOW") == "1":
        return
    keep, drop = [], []
    for it in items:
        (drop if it.get_closest_marker("slow") else keep).append(it)
    if drop:
        config.hook.pytest_deselected(items=drop)
        items[:] = keep
