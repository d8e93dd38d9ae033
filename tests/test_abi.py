"""CPU: the C-ABI library loads, exports every entry point include/ofx.h declares, struct layouts
match, and argument errors come back as status codes + ofx_last_error (no GPU work)."""
import ctypes
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "ofx.h")


def _declared():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+char\s*\*|int)\s+(ofx_\w+)\s*\(", txt, re.M)))


def test_header_declares_entry_points():
    names = _declared()
    for must in ("ofx_integrate", "ofx_skin_volume", "ofx_skin_points", "ofx_gn_solve", "ofx_gn_linearize",
                 "ofx_gn_step", "ofx_deform_points", "ofx_last_error"):
        assert must in names


def test_library_exports_every_declared_symbol():
    from occlusionfusion_amd import _lib
    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = [n for n in _declared() if not hasattr(lib, n)]
    assert not missing, missing
    assert set(_declared()) == set(_lib.EXPORTED)


def test_library_not_built_from_torch_extension():
    from occlusionfusion_amd import _lib
    assert _lib.LIB_PATH.startswith(ROOT)      # in-tree .so, loaded through the C ABI


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_struct_layouts_match_ctypes(tmp_path):
    from occlusionfusion_amd import _lib
    src = tmp_path / "sz.c"
    src.write_text('#include <stdio.h>\n#include "ofx.h"\nint main(){printf("%zu %zu %zu %zu %zu\\n",'
                   'sizeof(ofx_volume_desc),sizeof(ofx_camera),sizeof(ofx_gn_params),sizeof(ofx_gn_problem),'
                   'sizeof(ofx_gn_result));}\n')
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    c_sizes = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True).stdout.split()]
    py = [ctypes.sizeof(t) for t in (_lib.VolumeDesc, _lib.Camera, _lib.GnParams, _lib.GnProblem, _lib.GnResult)]
    assert c_sizes == py


def test_errors_are_status_codes_not_exceptions():
    from occlusionfusion_amd import _lib
    d = _lib.VolumeDesc()
    d.dim[:] = [16, 16, 16]
    d.brick_x0, d.brick_x1 = 0, 3            # only 2 bricks along x exist
    n = ctypes.c_int64()
    st = _lib.lib.ofx_volume_num_slots(ctypes.byref(d), ctypes.byref(n))
    assert st == -1
    assert b"shard range" in _lib.lib.ofx_last_error()
    with pytest.raises(_lib.OfxError):
        _lib.call("ofx_volume_num_slots", ctypes.byref(d), ctypes.byref(n))
    d.brick_x1 = 2
    _lib.call("ofx_volume_num_slots", ctypes.byref(d), ctypes.byref(n))
    assert n.value == 2 * 2 * 2 * 512
    assert _lib.lib.ofx_gn_create(20000, 10, ctypes.byref(ctypes.c_void_p())) == -3   # > 16384 nodes
