"""The traversal kernels' claim order (device_common.h claim_perm, used by
k_shadow's job claims, RTG_CLAIM_PERM): a bijection of [0, n) that keeps each
64-claim block contiguous, for queue lengths around every power of two and
the bench's sizes.  Frames do not depend on it (the closest hit and the
any-hit answer are schedule-independent); a non-bijective order would trace
some jobs twice and skip others."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")


def test_claim_order_is_a_block_preserving_bijection(tmp_path):
    exe = tmp_path / "claim_perm"
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "tests", "host_emu"),
                    os.path.join(ROOT, "tests", "claim_perm_emu.cpp"), "-o", str(exe)], check=True)
    ns = {0, 1, 63, 64, 65, 127, 128, 129, 1000, 4095, 4096, 4097, 123457, 810000, 3 * 1024 * 1024 + 17}
    for k in range(7, 21):
        ns |= {(1 << k) - 1, 1 << k, (1 << k) + 1, (1 << k) * 3 // 2}
    out = subprocess.run([str(exe)] + [str(n) for n in sorted(ns)], capture_output=True, text=True)
    assert out.returncode == 0 and out.stdout.strip() == "ok", out.stdout
