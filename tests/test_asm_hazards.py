"""The inline-asm MFMAs of the fused A3C update (csrc/r48_a3c_train.hip) are outside hipcc's
hazard padding; compile the kernel to gfx950 assembly exactly as the Makefile does and check the
wait states around every one of them (tools/check_asm_hazards.py). CPU-only (hipcc cross-compiles)."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_train_kernel_asm_mfma_wait_states(tmp_path):
    asm = tmp_path / "r48_a3c_train.s"
    subprocess.check_call([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC", "--cuda-device-only", "-S",
                           "-mllvm", "-amdgpu-mfma-vgpr-form=1", "-o", str(asm),
                           os.path.join(ROOT, "rein48_amd", "csrc", "r48_a3c_train.hip")], cwd=str(tmp_path))
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "check_asm_hazards.py"), str(asm)],
                         capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "asm MFMAs checked" in out.stdout and " 0 violations" in out.stdout
