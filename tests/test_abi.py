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
    assert g.rtgpu().rt_abi_version() == 8


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
    assert C.sizeof(g.RtTexture) == 16 + 5 * 8 + 8
    assert C.sizeof(g.RtPerlin) == 256 * 3 * 8 + 3 * 256 * 4


def test_ctypes_mirror_matches_c_header(g, tmp_path):
    """sizeof of every ABI struct as gcc sees include/rtgpu.h == the ctypes mirror."""
    import shutil
    import subprocess
    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    names = {"rt_hittable": g.RtHittable, "rt_material": g.RtMaterial, "rt_texture": g.RtTexture,
             "rt_work_counts": g.RtWorkCounts, "rt_kernel_times": g.RtKernelTimes,
             "rt_scene_info": g.RtSceneInfo, "rt_camera_desc": g.RtCameraDesc,
             "rt_render_params": g.RtRenderParams, "rt_scene_desc": g.RtSceneDesc, "rt_stats": g.RtStats,
             "rt_image": g.RtImage, "rt_perlin": g.RtPerlin, "rts_scene_options": g.RtsSceneOptions}
    src = tmp_path / "probe.c"
    inc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include")
    body = "".join(f'  printf("{n} %zu\\n", sizeof({n}));\n' for n in names)
    src.write_text(f'#include <stdio.h>\n#include "rtscene.h"\nint main(void) {{\n{body}  return 0;\n}}\n')
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-I", inc, str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    sizes = dict(line.split() for line in out if line)
    for n, cls in names.items():
        assert int(sizes[n]) == C.sizeof(cls), n
