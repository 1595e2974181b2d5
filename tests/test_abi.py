"""The C-ABI library loads and exports exactly what include/dp_mi355x.h declares (no GPU needed)."""

import ctypes
import os
import re
import subprocess

import pytest

from depth_pro import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "dp_mi355x.h")


def declared():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^int (dp_\w+)\(", src, flags=re.M)))


def test_header_and_python_export_lists_agree():
    assert declared() == sorted(_lib.EXPORTS)


def test_library_loads_and_exports_every_symbol():
    lib = _lib.load()
    for name in declared():
        assert hasattr(lib, name), name
    assert lib.dp_abi_version() == _lib.DP_ABI_VERSION


def test_gemm_args_struct_layout_matches_c(tmp_path):
    """ctypes GemmArgs == sizeof/offsetof of the C struct (compiled with gcc)."""
    fields = [f for f, _ in _lib.GemmArgs._fields_]
    prog = tmp_path / "lay.c"
    body = "".join(f'printf("%zu\\n", offsetof(dp_gemm_args, {f}));' for f in fields)
    prog.write_text(f'#include <stdio.h>\n#include <stddef.h>\n#include "{HEADER}"\n'
                    f'int main(void){{printf("%zu\\n", sizeof(dp_gemm_args));{body}return 0;}}\n')
    exe = tmp_path / "lay"
    subprocess.run(["gcc", "-std=c11", str(prog), "-o", str(exe)], check=True)
    vals = [int(v) for v in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    assert vals[0] == ctypes.sizeof(_lib.GemmArgs)
    for f, off in zip(fields, vals[1:]):
        assert getattr(_lib.GemmArgs, f).offset == off, f


def test_argument_errors_are_reported_before_launch():
    """Shape/alignment errors return DP_ERR_* without touching the GPU (null stream, no device)."""
    lib = _lib.load()
    a = _lib.GemmArgs()
    a.M, a.N, a.K = 16, 16, 60  # K % 64 != 0
    a.A = a.B = a.C = 16
    a.lda = a.ldb = 64
    assert lib.dp_gemm(ctypes.byref(a), None) == 1001
    a.K = 64
    a.ldb = 12
    assert lib.dp_gemm(ctypes.byref(a), None) == 1002
    assert lib.dp_attention(16, 16, 1, 577, 16, 128, 0.1, 0, None) == 1001
    with pytest.raises(_lib.DPError, match="DP_ERR_SHAPE"):
        _lib.check(1001, "x")
