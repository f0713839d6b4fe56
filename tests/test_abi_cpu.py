"""C-ABI library checks that need no GPU: it loads, exports every symbol the header
declares, the ctypes table matches the header, and argument validation fails cleanly
(no HIP call is made before validation)."""
import ctypes
import re

import pytest

from stereoanywhere_amd import _native as N


def header_functions():
    src = open(N.HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    out = {}
    for m in re.finditer(r"^\s*(?:const\s+)?[\w\s\*]+?\b(sa_\w+)\s*\(([^)]*)\)\s*;", src, flags=re.M):
        args = [a.strip() for a in m.group(2).split(",") if a.strip() and a.strip() != "void"]
        out[m.group(1)] = len(args)
    return out


def test_library_exports_every_declared_symbol():
    lib = N.lib()
    decl = header_functions()
    assert len(decl) >= 20
    for name in decl:
        assert hasattr(lib, name), f"{name} declared in the header but not exported"


def test_ctypes_table_matches_header():
    decl = header_functions()
    assert set(decl) == set(N.SIGNATURES), set(decl) ^ set(N.SIGNATURES)
    for name, nargs in decl.items():
        assert len(N.SIGNATURES[name][1]) == nargs, name


def test_pyramid_geometry():
    lib = N.lib()
    assert [lib.sa_pyramid_level_width(240, i) for i in range(4)] == [240, 120, 60, 30]
    assert [lib.sa_pyramid_level_offset(240, i) for i in range(4)] == [0, 240, 360, 420]
    assert lib.sa_pyramid_row_stride(240, 4) == 452
    # odd widths floor at every halving (avg_pool2d [1,2], corr.py:88-91)
    assert [lib.sa_pyramid_level_width(37, i) for i in range(4)] == [37, 18, 9, 4]
    assert lib.sa_pyramid_row_stride(37, 4) == 68


def test_argument_errors_are_reported():
    lib = N.lib()
    rc = lib.sa_corr_volume_pyramid(None, None, 1, 1, 1, 1, 1, 1.0, None, None, 0.9, 4, None, 4, None)
    assert rc == -1
    assert b"null pointer" in lib.sa_last_error()
    with pytest.raises(N.NativeError, match="num_levels"):
        N.call("sa_corr_lookup", 8, None, 32, 60, 7, 4, 8, 0, 1, 1, 1, 8, 100, None)


def test_timing_api_without_gpu():
    N.timing_enable(False)
    assert N.timing_read("corr_lookup") == (0.0, 0)
