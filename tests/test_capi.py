"""CPU: the C-ABI library builds, loads and exports every symbol include/*.h declares
(no compute calls without a GPU)."""
import ctypes
import glob
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    syms = set()
    for hdr in glob.glob(os.path.join(ROOT, "include", "*.h")):
        txt = open(hdr).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        syms |= set(re.findall(r"\b(m3s_\w+)\s*\(", txt))
    return syms


def test_library_exports_every_declared_symbol():
    from monst3r_slam_amd import _lib
    lib = _lib.load()
    syms = declared_symbols()
    assert len(syms) >= 15
    missing = [s for s in sorted(syms) if not hasattr(lib, s)]
    assert not missing, missing
    # python signature table covers the header
    assert syms <= set(_lib.SIGNATURES), sorted(syms - set(_lib.SIGNATURES))


def test_status_strings_and_version():
    from monst3r_slam_amd import _lib
    lib = _lib.load()
    assert _lib.status_string(0) == "ok"
    assert "invalid" in _lib.status_string(-1)
    assert lib.m3s_version() >= (0 << 16) | (1 << 8)


def test_invalid_args_rejected_without_device():
    from monst3r_slam_amd import _lib
    lib = _lib.load()
    # null pointers / bad sizes are rejected before any HIP call
    assert lib.m3s_iter_proj(None, None, None, None, None, 1, 8, 8, 64, 10, 1e-8, 1e-6,
                             None) == -1
    assert lib.m3s_refine_matches(None, None, None, None, 1, 8, 8, 64, 24, 3, 5, None) == -1
    assert lib.m3s_iter_proj(None, None, None, None, None, 0, 8, 8, 0, 10, 1e-8, 1e-6,
                             None) == 0
    assert lib.m3s_gn_workspace_bytes(10, 20, 100) > 16 * 10 * 100 + 4 * 20 * 100


def test_dropin_module_surface():
    import mast3r_slam_backends as mb
    for name in ("iter_proj", "refine_matches", "gauss_newton_rays", "gauss_newton_calib",
                 "gauss_newton_points"):
        assert callable(getattr(mb, name))
    import torch
    x = torch.zeros(1, 4, 4, 9)[..., ::1].transpose(1, 2)
    with pytest.raises(RuntimeError, match="must be contiguous"):
        mb.iter_proj(x, torch.zeros(1, 16, 3), torch.zeros(1, 16, 2), 10, 1e-8, 1e-6)


def test_gemm_desc_layout_matches_header(tmp_path):
    """The ctypes mirror of m3s_gemm_desc (_lib.GemmDesc) has the C header's size and field
    offsets (gcc on include/monst3r_slam_amd.h): a drifted mirror would hand the library
    garbage in the fields past the first mismatch (ABI 0.5 appended ln_c3 / ln_shift /
    ln_qscale)."""
    import shutil
    import subprocess
    from monst3r_slam_amd import _lib
    if shutil.which("gcc") is None:
        pytest.skip("no gcc")
    names = [f[0] for f in _lib.GemmDesc._fields_]
    src = tmp_path / "layout.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "monst3r_slam_amd.h"\n'
                   "int main(void) {\n"
                   '  printf("%zu\\n", sizeof(m3s_gemm_desc));\n' +
                   "".join(f'  printf("%zu\\n", offsetof(m3s_gemm_desc, {n}));\n' for n in names) +
                   "  return 0;\n}\n")
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)],
                   check=True)
    out = [int(v) for v in subprocess.run([str(exe)], check=True, capture_output=True,
                                          text=True).stdout.split()]
    assert out[0] == ctypes.sizeof(_lib.GemmDesc)
    assert out[1:] == [getattr(_lib.GemmDesc, n).offset for n in names]
