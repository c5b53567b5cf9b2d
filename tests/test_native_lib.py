"""CPU tests of the C-ABI library: it builds for gfx950, loads, exports every symbol the header
declares, and fails loudly (no crash, no fallback) where no GPU is present."""
import ctypes as C
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "shd_accel.h")


def header_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(shd_[a-z_0-9]+)\s*\(", text)))


def test_library_builds_and_loads():
    from shadow_amd import build
    path = build.build(verbose=False)
    assert os.path.exists(path)
    C.CDLL(path)


def test_exports_every_header_symbol():
    from shadow_amd import _native as N
    from shadow_amd import build
    path = build.build(verbose=False)
    out = subprocess.check_output(["nm", "-D", "--defined-only", path], text=True)
    exported = set(re.findall(r"\bT (shd_[a-z_0-9]+)$", out, flags=re.M))
    declared = header_functions()
    assert declared, "no functions parsed from the header"
    missing = [f for f in declared if f not in exported]
    assert not missing, missing
    assert sorted(N.EXPORTED) == declared


def test_code_object_is_gfx950(tmp_path):
    from shadow_amd import build
    path = build.build(verbose=False)
    fb = tmp_path / "fatbin.bin"
    subprocess.check_call(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", path, str(fb)])
    out = subprocess.check_output(["/opt/rocm/lib/llvm/bin/clang-offload-bundler", "--list",
                                   "--type=o", f"--input={fb}"], text=True)
    targets = [t for t in out.split() if "amdgcn" in t]
    assert targets == ["hipv4-amdgcn-amd-amdhsa--gfx950"]


def test_status_strings_and_no_gpu_open_fails_loudly():
    import torch
    from shadow_amd import _native as N
    lib = N.load()
    assert lib.shd_status_str(0) == b"ok"
    assert b"gfx950" in lib.shd_version()
    if torch.cuda.is_available():
        pytest.skip("a GPU is present; covered by the gpu tests")
    st = C.c_int32(0)
    assert lib.shd_open(0, C.byref(st)) is None
    assert st.value == 6  # SHD_ERR_HIP
