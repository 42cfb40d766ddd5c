"""Host build of the kernel's per-lane board logic (r48_board.h) vs the C oracle (CPU).

Compiles tests/native/board_logic_test.cpp with g++ (the same source the gfx950 kernels
include, with v_perm_b32 emulated) and runs: exhaustive 18^4-line table in every direction,
400k random moves with merge reward and game-over, 200k full steps with injected draws and
3 x 200k Philox-mode steps with auto-reset.
"""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_board_logic_matches_oracle(tmp_path):
    orc = tmp_path / "orc.o"
    exe = tmp_path / "board_logic_test"
    subprocess.check_call(["gcc", "-O2", "-std=c11", "-c", "-o", str(orc), os.path.join(ROOT, "oracle", "r48_oracle.c")])
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-Wall", "-Werror", "-o", str(exe),
                           os.path.join(ROOT, "tests", "native", "board_logic_test.cpp"), str(orc)])
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK (0 failures)" in r.stdout


def test_cnn_fragment_schedules_compile_time_checks():
    """r48_cnn_common.h's weight-fragment read schedules (grouped inference order, chain order)
    checked by static_asserts in tests/native/cnn_schedule_test.cpp (host-only syntax pass)."""
    hipcc = "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        import pytest
        pytest.skip("hipcc not available")
    r = subprocess.run([hipcc, "-std=c++17", "--offload-host-only", "-fsyntax-only",
                        os.path.join(ROOT, "tests", "native", "cnn_schedule_test.cpp")],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
