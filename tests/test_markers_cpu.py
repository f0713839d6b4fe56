"""The parity gate `pytest -m gpu` holds no wall-clock assertion: collect it
(collect-only, no GPU needed) and check that no collected test, nor a helper of its module that it
calls, reads a clock.  Timing checks live in tests/test_perf_gpu.py under the `perf` marker, which
conftest.py deselects unless --run-perf is given."""
import ast
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLOCKS = ("elapsed_time", "perf_counter", "time.time(", "monotonic")


def _collect(*args):
    r = subprocess.run([sys.executable, "-m", "pytest", "--collect-only", "-q", "-p", "no:cacheprovider", *args,
                        os.path.join(ROOT, "tests")], capture_output=True, text=True, cwd=ROOT, timeout=600)
    assert r.returncode in (0, 5), r.stdout[-2000:] + r.stderr[-2000:]
    return [ln.strip() for ln in r.stdout.splitlines() if "::" in ln]


def _functions(path):
    tree = ast.parse(open(path).read())
    src = open(path).read()
    return {n.name: (ast.get_source_segment(src, n), {c.func.id for c in ast.walk(n) if isinstance(c, ast.Call)
                                                       and isinstance(c.func, ast.Name)})
            for n in tree.body if isinstance(n, ast.FunctionDef)}


def _reads_clock(name, funcs, seen=None):
    seen = seen if seen is not None else set()
    if name in seen or name not in funcs:
        return False
    seen.add(name)
    body, calls = funcs[name]
    return any(c in body for c in CLOCKS) or any(_reads_clock(c, funcs, seen) for c in calls)


@pytest.mark.slow
def test_gpu_gate_has_no_timing_assertions():
    ids = _collect("-m", "gpu")
    assert len(ids) > 100, ids[:5]
    bad, cache = [], {}
    for nid in ids:
        path, func = nid.split("::")[0], nid.split("::")[-1].split("[")[0]
        full = os.path.join(ROOT, path)
        funcs = cache.setdefault(full, _functions(full))
        if _reads_clock(func, funcs):
            bad.append(nid)
    assert not bad, bad
    assert not any("test_perf_gpu" in nid for nid in ids)


@pytest.mark.slow
def test_perf_checks_collected_only_on_request():
    assert not _collect("-m", "perf")
    ids = _collect("--run-perf", "-m", "perf")
    assert ids and all("test_perf_gpu.py" in nid for nid in ids)
