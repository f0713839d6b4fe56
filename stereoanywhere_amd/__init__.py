"""MI355X (gfx950) build of the Stereo Anywhere cost-volume hot path.

Importing the package points MIOpen at the in-repo find/perf database (miopen_db/), so the
dense convolutions that stay on MIOpen use the algorithms measured on MI355X for these
shapes instead of immediate-mode heuristics; without entries MIOpen falls back to its
heuristics.  Override with MIOPEN_USER_DB_PATH / MIOPEN_CUSTOM_CACHE_DIR (compiled-kernel
cache for the chosen solvers).  Regenerate with `bench.py --miopen-find 1` on the box.
"""
import os as _os

_DB = _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))), "miopen_db")
if _os.path.isdir(_DB):
    _os.environ.setdefault("MIOPEN_USER_DB_PATH", _DB)
    _os.environ.setdefault("MIOPEN_CUSTOM_CACHE_DIR", _os.path.join(_DB, "cache"))
