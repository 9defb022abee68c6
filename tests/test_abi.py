"""The C-ABI library loads (no GPU needed) and exports every symbol include/*.h declares."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "h-slam_amd", "lib", "libhslam_amd.so")


def declared_symbols():
    names = set()
    inc = os.path.join(ROOT, "include")
    for fn in sorted(os.listdir(inc)):
        if not fn.endswith(".h"):
            continue
        txt = open(os.path.join(inc, fn)).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        for m in re.finditer(r"^[A-Za-z_][\w \*]*?\b(hs_\w+)\s*\(", txt, flags=re.M):
            names.add(m.group(1))
    return sorted(names)


def test_headers_declare_entry_points():
    names = declared_symbols()
    assert "hs_ba_optimize" in names and "hs_create" in names
    assert len(names) >= 17


def test_library_exports_all_declared():
    if not os.path.exists(LIB):
        subprocess.run(["make", "-C", os.path.join(ROOT, "h-slam_amd", "csrc")], check=True, capture_output=True)
    lib = ctypes.CDLL(LIB)  # loads without a GPU: no device work at load time
    missing = [n for n in declared_symbols() if not hasattr(lib, n)]
    assert not missing, missing


def test_params_default_and_no_device_error():
    import sys
    sys.path.insert(0, os.path.join(ROOT, "h-slam_amd"))
    from hslam_amd import _lib
    p = _lib.default_params()
    assert p.huberTH == 9 and abs(p.frameEnergyTHN - 0.7) < 1e-7 and p.initialCalibHessian == 5e9
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:
        has_gpu = False
    if not has_gpu:
        h = ctypes.c_void_p()
        rc = _lib.load().hs_create(ctypes.byref(h), ctypes.byref(p), 0)
        assert rc != 0  # fails loudly: no CPU fallback
        assert b"device" in _lib.load().hs_last_error()


def test_ctypes_structs_match_c_layout(tmp_path):
    """The ctypes mirrors (hslam_amd._lib, oracle_ffi) have the C structs' sizes (compiled here with gcc)."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "h-slam_amd"))
    from hslam_amd import _lib
    src = tmp_path / "sz.c"
    src.write_text('#include <stdio.h>\n#include "hs_types.h"\n#include "hs_trace.h"\n'
                   'int main(void){printf("%zu %zu %zu %zu %zu %zu\\n", sizeof(hs_params), sizeof(hs_camera),'
                   ' sizeof(hs_frame), sizeof(hs_points), sizeof(hs_residuals), sizeof(hs_trace_host));return 0;}\n')
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    sizes = list(map(int, subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()))
    py = [ctypes.sizeof(c) for c in (_lib.hs_params, _lib.hs_camera, _lib.hs_frame, _lib.hs_points,
                                     _lib.hs_residuals)] + [14 * 4]
    assert sizes == py, (sizes, py)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_ffi
    assert ctypes.sizeof(oracle_ffi.hs_params) == sizes[0]


def test_built_libraries_are_current():
    """The in-tree .so files (they travel to the GPU box prebuilt) are newer than every source they are built from:
    a stale library would make GPU parity compare two stale builds."""
    def newest(paths):
        return max(os.path.getmtime(p) for p in paths)

    def files(d, exts):
        return [os.path.join(d, f) for f in os.listdir(d) if f.endswith(exts)]

    csrc = os.path.join(ROOT, "h-slam_amd", "csrc")
    inc = os.path.join(ROOT, "include")
    ora = os.path.join(ROOT, "oracle")
    lib_src = files(csrc, (".hip", ".cpp", ".h")) + files(inc, (".h",)) + [os.path.join(csrc, "Makefile")]
    ora_src = files(ora, (".cpp", ".h")) + files(inc, (".h",)) + [os.path.join(ora, "Makefile")]
    assert os.path.getmtime(LIB) >= newest(lib_src), "libhslam_amd.so is stale: make -C h-slam_amd/csrc"
    for so in ("liboracle.so", "liboracle_fast.so"):
        p = os.path.join(ora, "_build", so)
        assert os.path.getmtime(p) >= newest(ora_src), f"{so} is stale: make -C oracle"


def test_c_caller_is_built_against_the_headers():
    """tests/c/ba_caller.c is a plain C99 program (gcc -Wall -Wextra, no HIP headers) against include/hs_ba.h, built
    by h-slam_amd/csrc/Makefile next to the library: the boundary compiles and links from C.  The GPU suite runs it
    (tests/test_gpu_c_caller.py)."""
    exe = os.path.join(ROOT, "h-slam_amd", "lib", "ba_caller")
    src = os.path.join(ROOT, "tests", "c", "ba_caller.c")
    assert os.path.exists(exe), "make -C h-slam_amd/csrc"
    assert os.path.getmtime(exe) >= max(os.path.getmtime(src), os.path.getmtime(os.path.join(ROOT, "include", "hs_ba.h")))


def test_lin8_offset_limit():
    """hs_k_lin8's taps use 32-bit buffer offsets formed by 24-bit multiplies (hs_lin8_kernels.hip interp33_8b): a
    window runs it only while W * H < 2^23 and all HS_MAXF packed slots stay below 2^31 bytes (lin8_supported,
    hs_ba_ctx.h); larger images fall back to hs_k_lin.  Pure host rule, checked at the limit without a GPU."""
    lib = ctypes.CDLL(LIB)
    f = lib.hs_debug_lin8_supported
    f.argtypes, f.restype = [ctypes.c_int, ctypes.c_int], ctypes.c_int
    assert f(640, 480) == 1 and f(1232, 368) == 1
    assert f(4096, 2047) == 1          # 2^23 - 4096 texels
    assert f(4096, 2048) == 0          # 2^23 texels: the 24-bit texel index would wrap
    assert f(3840, 2160) == 1 and f(4096, 2160) == 0
    assert f(1 << 23, 1) == 0
