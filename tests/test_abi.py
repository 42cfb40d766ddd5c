"""C-ABI checks that need no GPU: the library loads, exports exactly what include/rein48.h
declares, the ctypes signatures cover every export, and argument errors come back as
R48_EINVAL with a message (no HIP call is made on these paths)."""
import ctypes as C
import os
import re
import subprocess

import pytest

from rein48_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "rein48.h")


def declared():
    text = open(HEADER).read()
    return set(re.findall(r"^\s*(?:const\s+)?[\w]+\s*\*?\s*(r48_\w+)\s*\(", text, re.M))


def test_header_parses():
    names = declared()
    assert "r48_env_step" in names and "r48_last_error" in names and len(names) >= 20


def test_binding_constants_mirror_the_header():
    text = open(HEADER).read()
    consts = {k: int(v, 0) for k, v in
              re.findall(r"^#define (R48_\w+)\s+\(?(-?(?:0x[0-9a-fA-F]+|\d+))u?\)?", text, re.M)}
    assert consts["R48_DRAW_CONTRACT"] == _lib.DRAW_CONTRACT
    assert (consts["R48_AUTO_RESET"], consts["R48_RANDOM_POLICY"], consts["R48_MERGE_REWARD"]) == \
        (_lib.AUTO_RESET, _lib.RANDOM_POLICY, _lib.MERGE_REWARD)


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    out = subprocess.check_output(["nm", "-D", "--defined-only", _lib.LIB_PATH], text=True)
    exported = set(re.findall(r" T (r48_\w+)$", out, re.M))
    assert declared() == exported
    for name in declared():
        assert hasattr(lib, name)
    assert set(_lib.SIGNATURES) == declared()


def prototypes():
    """name -> parameter count of every r48_ prototype in the header (comments stripped)."""
    text = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    out = {}
    for m in re.finditer(r"(r48_\w+)\s*\(([^;{]*?)\)\s*;", text, re.S):
        params = m.group(2).strip()
        out[m.group(1)] = 0 if params in ("", "void") else params.count(",") + 1
    return out


def test_ctypes_signatures_match_the_header_arity():
    """Every ctypes argtypes list has exactly as many entries as the header prototype has
    parameters (an entry point that gained an argument in include/rein48.h but not in _lib.py would
    otherwise shift every later argument silently)."""
    protos = prototypes()
    assert set(protos) == declared()
    bad = {n: (len(_lib.SIGNATURES[n][1]), k) for n, k in protos.items() if len(_lib.SIGNATURES[n][1]) != k}
    assert not bad, bad


def test_library_is_gfx950_code_object():
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data  # the embedded offload bundle's target triple


def test_argument_errors_without_gpu():
    lib = _lib.load()
    env = C.c_void_p()
    assert lib.r48_env_create(C.byref(env), 0, 0, 1, 0) == _lib.R48_EINVAL
    assert b"n_boards" in lib.r48_last_error()
    assert lib.r48_env_create(None, 0, 16, 1, 0) == _lib.R48_EINVAL
    assert lib.r48_env_bind_boards(None, None) == _lib.R48_EINVAL
    assert lib.r48_env_step(None, None, 0, None, None, None, None, None) == _lib.R48_EINVAL
    assert lib.r48_values_check(None, 1, 4, 4, None, None, None) == _lib.R48_EINVAL
    assert lib.r48_env_fill_random(None, 7, None) == _lib.R48_EINVAL
    assert lib.r48_values_move(None, None, 1, None, None, None) == _lib.R48_EINVAL
    assert lib.r48_env_destroy(None) == _lib.R48_OK
    with pytest.raises(_lib.Rein48Error):
        _lib.check(lib.r48_env_create(C.byref(env), 0, -5, 1, 0))
    assert lib.r48_version().startswith(b"rein48")


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "nope.so"))
    with pytest.raises(_lib.Rein48LibraryError):
        _lib.load()
