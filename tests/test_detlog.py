"""The volume free-flight logarithm (volume.go:66, -(1/rho)*ln(U)) is computed
without libm on both sides: device_common.h rt_logf (the kernels) and the
oracle's fp32 restatement o_logf.  Checked here over every RNG value
U = k*2^-24, k in [0, 2^24): the two agree bit for bit, and both are within
2 ulp of the float64 logarithm.  This is what makes fog hit ids bit-exact on
the GPU (tests/test_gpu_parity.py has no mismatch allowance)."""
import ctypes as C
import os
import shutil
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")


def test_device_log_equals_oracle_log_on_every_rng_value(O, tmp_path):
    exe = tmp_path / "detlog"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-I", os.path.join(ROOT, "tests", "host_emu"),
                    os.path.join(ROOT, "tests", "detlog_emu.cpp"), "-o", str(exe)], check=True)
    out = tmp_path / "log.f32"
    subprocess.run([str(exe), str(out)], check=True)
    dev = np.fromfile(out, np.float32)
    u = np.arange(1 << 24, dtype=np.float64) * 2.0 ** -24
    uf = u.astype(np.float32)
    assert np.array_equal(uf.astype(np.float64), u)          # every RNG value is exact in fp32
    orc = np.zeros_like(uf)
    O.lib().oracle_logf32(uf.ctypes.data_as(C.POINTER(C.c_float)), orc.ctypes.data_as(C.POINTER(C.c_float)),
                          C.c_int64(uf.size))
    assert np.array_equal(dev.view(np.uint32), orc.view(np.uint32))
    assert dev[0] == -np.inf
    ref = np.log(u[1:])
    got = dev[1:].astype(np.float64)
    ulp = np.spacing(np.abs(ref).astype(np.float32)).astype(np.float64)
    ulp[ref == 0] = np.spacing(np.float32(0))
    err = np.abs(got - ref) / ulp
    assert err.max() <= 2.0, float(err.max())
    assert got[-1] < 0 and np.all(np.diff(got) >= 0)         # monotone on the RNG grid
