import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.dirname(os.path.abspath(__file__))):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_addoption(parser):
    parser.addoption("--run-perf", action="store_true", default=False,
                     help="run the wall-clock checks (marker perf; scripts/perf_checks.sh)")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI library)")
    config.addinivalue_line("markers", "slow: CPU test that takes more than ~20 s")
    config.addinivalue_line("markers", "perf: wall-clock check on an MI355X; deselected unless --run-perf")


def pytest_collection_modifyitems(config, items):
    """Wall-clock checks stay out of the parity gates (`-m gpu` / `-m "not gpu"`): a noisy box must
    not stop the parity run, so `perf` tests are deselected unless --run-perf is given."""
    if config.getoption("--run-perf"):
        return
    keep = [it for it in items if it.get_closest_marker("perf") is None]
    if len(keep) != len(items):
        config.hook.pytest_deselected(items=[it for it in items if it.get_closest_marker("perf") is not None])
        items[:] = keep
