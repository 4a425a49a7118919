"""The C-ABI libraries load and export every symbol their headers declare
(no compute calls: this container has no GPU)."""
import ctypes as C
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared(header):
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"\b((?:rt|rts)_[a-z0-9_]+)\s*\(", src)
    return sorted(set(names))


@pytest.mark.parametrize("header,lib", [("rtgpu.h", "librtgpu.so"), ("rtscene.h", "librtscene.so")])
def test_exports_every_declared_symbol(g, header, lib):
    names = _declared(header)
    assert len(names) >= 10
    so = C.CDLL(os.path.join(g.LIB_DIR, lib))
    missing = [n for n in names if not hasattr(so, n)]
    assert not missing, missing


def test_abi_version(g):
    assert g.rtgpu().rt_abi_version() == 1


def test_no_silent_cpu_fallback_without_gpu(g):
    """Without a usable device the product path fails loudly (no CPU path)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(g.RTError):
        g.Context(0)


def test_kernels_built_for_gfx950(g):
    data = open(os.path.join(g.LIB_DIR, "librtgpu.so"), "rb").read()
    assert b"gfx950" in data


def test_scene_desc_struct_sizes(g):
    # layout the Go side mirrors in INTEGRATION.md
    assert C.sizeof(g.RtHittable) == 4 * 4 + 6 * 8 + 16 * 8
    assert C.sizeof(g.RtMaterial) == 8 + 5 * 8
    assert C.sizeof(g.RtTexture) == 16 + 4 * 8
