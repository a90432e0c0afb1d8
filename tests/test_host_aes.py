"""Host CPU self-test of the device AES T-table round structure (tests/host/*.cpp): the
exact template in csrc/aes_ttable.h instantiated with emulated v_perm_b32 / LDS loads."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_aes_ttable_host(tmp_path):
    if not shutil.which("hipcc"):
        pytest.skip("hipcc not available")
    exe = tmp_path / "aes_host"
    subprocess.run(["hipcc", "--offload-arch=gfx950", "-O2", "-std=c++17",
                    os.path.join(ROOT, "tests", "host", "aes_ttable_host_test.cpp"), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True)
    assert out.returncode == 0 and out.stdout.strip() == "OK", out.stdout + out.stderr


def test_transpose32_host(tmp_path):
    """The 32 x 32 bit transpose (csrc/bitslice.h) of the OT hashes and the garbled-table kernels."""
    if not shutil.which("hipcc"):
        pytest.skip("hipcc not available")
    exe = tmp_path / "transpose_host"
    subprocess.run(["hipcc", "--offload-arch=gfx950", "-O1", "-std=c++17",
                    os.path.join(ROOT, "tests", "host", "transpose_host_test.cpp"), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True)
    assert out.returncode == 0 and out.stdout.strip() == "OK", out.stdout + out.stderr


def test_item_layout_host(tmp_path):
    """k_expand's two-phase work decomposition covers every (job, entry, word) exactly once."""
    if not shutil.which("hipcc"):
        pytest.skip("hipcc not available")
    exe = tmp_path / "item_layout"
    subprocess.run(["hipcc", "--offload-arch=gfx950", "-O1", "-std=c++17",
                    os.path.join(ROOT, "tests", "host", "item_layout_host_test.cpp"), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True)
    assert out.returncode == 0 and out.stdout.strip() == "OK", out.stdout + out.stderr
