"""go-raytracing_amd — MI355X-native path tracer for byvfx/go-raytracing scenes.

Python binding (ctypes) over the two native libraries built in ``lib/``:

* ``librtgpu.so``  — the drop-in C-ABI of ``include/rtgpu.h`` (scene graph
  upload, GPU render, tonemap, parity probes).  This is what the Go host binds
  through cgo.
* ``librtscene.so`` — the C++ mirror of the reference's host-side ``rt`` API
  (``scenes.go`` builders, ``NewBVHNode``, loaders, ``NewBucketRenderer``;
  ``include/rtscene.h``), standing in for the Go host (no Go toolchain here).

There is no CPU fallback: if the libraries are missing or no GPU is present the
calls fail loudly.  The package directory has a hyphen, so import it with
``load_package()`` from ``__graft_entry__`` / tests (importlib by path).
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional, Sequence

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
# RTGPU_LIB_DIR: an alternative in-tree build (A/B experiments), e.g. lib_w5
LIB_DIR = os.path.join(PKG_DIR, os.environ.get("RTGPU_LIB_DIR", "lib"))
REPO_DIR = os.path.dirname(PKG_DIR)
ASSET_DIR = os.path.join(REPO_DIR, "assets")

RT_OK = 0
RT_OPT_BLAS_BUILDER, RT_OPT_TLAS_BUILDER, RT_OPT_NODE_FORMAT = 1, 2, 3
RT_OPT_BATCH_SLOTS, RT_OPT_REFILL, RT_OPT_MAX_BLOCKS, RT_OPT_STREAMS = 4, 5, 6, 7
RT_OPT_VOLUMES = 8
RT_VOLUMES_LIFTED, RT_VOLUMES_IN_BVH = 0, 1
RT_OPT_BVH4_COLLAPSE = 9
RT_COLLAPSE_SAH, RT_COLLAPSE_GREEDY = 0, 1
RT_BLAS_REFERENCE, RT_BLAS_SAH, RT_BLAS_DEVICE = 0, 1, 2
RT_NODES_FP32, RT_NODES_QUANT8, RT_NODES_WIDE8 = 0, 1, 2
RT_OPT_DEALING, RT_OPT_DEAL_FIRST = 10, 11
RT_OPT_TAIL = 12
RT_OPT_OVERLAP = 13
RT_DEAL_STATIC, RT_DEAL_DYNAMIC = 0, 1
STATUS = {0: "RT_OK", -1: "RT_ERR_INVALID", -2: "RT_ERR_UNSUPPORTED", -3: "RT_ERR_HIP", -4: "RT_ERR_OOM",
          -5: "RT_ERR_NO_SCENE", -6: "RT_ERR_DEVICE"}

# hittable kinds (rtgpu.h)
RT_SPHERE, RT_QUAD, RT_TRIANGLE, RT_PLANE, RT_LIST, RT_BVH_NODE, RT_BVH_LEAF = 1, 2, 3, 4, 5, 6, 7
RT_TRANSLATE, RT_ROTATE_X, RT_ROTATE_Y, RT_ROTATE_Z, RT_SCALE, RT_VOLUME = 8, 9, 10, 11, 12, 13
RT_LAMBERTIAN, RT_METAL, RT_DIELECTRIC, RT_DIFFUSE_LIGHT, RT_ISOTROPIC = 1, 2, 3, 4, 5
RT_TEX_SOLID, RT_TEX_CHECKER, RT_TEX_NOISE, RT_TEX_IMAGE = 1, 2, 3, 4


class RtHittable(C.Structure):
    _fields_ = [("kind", C.c_int32), ("material", C.c_int32), ("a", C.c_int32), ("b", C.c_int32),
                ("bbox", C.c_double * 6), ("p", C.c_double * 16)]


class RtMaterial(C.Structure):
    _fields_ = [("kind", C.c_int32), ("texture", C.c_int32), ("albedo", C.c_double * 3), ("fuzz", C.c_double),
                ("refraction_index", C.c_double)]


class RtTexture(C.Structure):
    _fields_ = [("kind", C.c_int32), ("even", C.c_int32), ("odd", C.c_int32), ("albedo", C.c_double * 3),
                ("inv_scale", C.c_double), ("scale", C.c_double), ("perlin", C.c_int32), ("image", C.c_int32)]


class RtImage(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("rgb", C.POINTER(C.c_double))]


class RtPerlin(C.Structure):
    _fields_ = [("randvec", (C.c_double * 3) * 256), ("perm_x", C.c_int32 * 256), ("perm_y", C.c_int32 * 256),
                ("perm_z", C.c_int32 * 256)]


class RtEnvironment(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("rgb", C.POINTER(C.c_double)),
                ("rotation", C.c_double), ("use_importance_sampling", C.c_int32)]


class RtSceneDesc(C.Structure):
    _fields_ = [("hittables", C.POINTER(RtHittable)), ("num_hittables", C.c_int32),
                ("children", C.POINTER(C.c_int32)), ("num_children", C.c_int32), ("root", C.c_int32),
                ("materials", C.POINTER(RtMaterial)), ("num_materials", C.c_int32),
                ("textures", C.POINTER(RtTexture)), ("num_textures", C.c_int32),
                ("lights", C.POINTER(C.c_int32)), ("num_lights", C.c_int32),
                ("environment", C.POINTER(RtEnvironment)),
                ("images", C.POINTER(RtImage)), ("num_images", C.c_int32),
                ("perlins", C.POINTER(RtPerlin)), ("num_perlins", C.c_int32)]


class RtCameraDesc(C.Structure):
    _fields_ = [("image_width", C.c_int32), ("image_height", C.c_int32), ("samples_per_pixel", C.c_int32),
                ("max_depth", C.c_int32), ("center", C.c_double * 3), ("pixel00", C.c_double * 3),
                ("pixel_delta_u", C.c_double * 3), ("pixel_delta_v", C.c_double * 3),
                ("defocus_angle", C.c_double), ("defocus_disk_u", C.c_double * 3),
                ("defocus_disk_v", C.c_double * 3), ("background", C.c_double * 3),
                ("use_sky_gradient", C.c_int32), ("phantom_hdri", C.c_int32), ("camera_motion", C.c_int32),
                ("free_camera", C.c_int32), ("center_motion_orig", C.c_double * 3),
                ("center_motion_dir", C.c_double * 3), ("look_at_motion_orig", C.c_double * 3),
                ("look_at_motion_dir", C.c_double * 3), ("vup", C.c_double * 3), ("forward", C.c_double * 3),
                ("viewport_width", C.c_double), ("viewport_height", C.c_double), ("focus_dist", C.c_double),
                ("defocus_radius", C.c_double)]


class RtBucket(C.Structure):
    _fields_ = [("x", C.c_int32), ("y", C.c_int32), ("width", C.c_int32), ("height", C.c_int32)]


class RtRenderParams(C.Structure):
    _fields_ = [("samples_per_pixel", C.c_int32), ("max_depth", C.c_int32), ("sample_offset", C.c_int32),
                ("seed", C.c_uint32), ("buckets", C.POINTER(RtBucket)), ("num_buckets", C.c_int32),
                ("accumulate", C.c_int32)]


class RtStats(C.Structure):
    _fields_ = [("kernel_ms", C.c_double), ("samples", C.c_uint64)]


class RtWorkCounts(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in ("samples", "rays", "shadow_rays", "node_visits", "sphere_tests",
                                          "quad_tests", "tri_tests", "plane_tests", "instance_visits",
                                          "volume_tests", "material_fetches", "env_lookups",
                                          "instance_box_tests", "stack_spills")]


class RtKernelTimes(C.Structure):
    _fields_ = [("extend_ms", C.c_double), ("shade_ms", C.c_double), ("shadow_ms", C.c_double),
                ("extend_launches", C.c_int32), ("shade_launches", C.c_int32), ("shadow_launches", C.c_int32),
                ("twins", C.c_int32)]


class RtSceneInfo(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("nodes", "leaves", "refs", "spheres", "quads", "triangles", "planes",
                                         "instances", "blases", "volumes", "materials", "textures", "lights",
                                         "stack_needed", "tlas_depth", "blas_depth")] + [("device_bytes", C.c_int64)] + \
        [("node_format", C.c_int32), ("nodes8", C.c_int32)]


class RtsSceneOptions(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("width", C.c_int32), ("aspect", C.c_double), ("spp", C.c_int32),
                ("max_depth", C.c_int32), ("asset_dir", C.c_char_p), ("obj_path", C.c_char_p),
                ("lucy_rings", C.c_int32), ("lucy_cols", C.c_int32), ("camera_motion", C.c_int32),
                ("look_from2", C.c_double * 3), ("look_at2", C.c_double * 3), ("free_camera", C.c_int32),
                ("forward", C.c_double * 3)]


_rtgpu = None
_rtscene = None


def _load(name: str) -> C.CDLL:
    path = os.path.join(LIB_DIR, name)
    if not os.path.exists(path):
        raise RuntimeError(f"{path} is missing: build it first (python -c 'import __graft_entry__ as g; g.build()')")
    return C.CDLL(path, mode=C.RTLD_GLOBAL)


def rtgpu() -> C.CDLL:
    """The C-ABI library (include/rtgpu.h)."""
    global _rtgpu
    if _rtgpu is None:
        lib = _load("librtgpu.so")
        P, I32, U32 = C.c_void_p, C.c_int32, C.c_uint32
        lib.rt_abi_version.restype = C.c_int
        lib.rt_ctx_create.argtypes = [C.c_int, C.POINTER(P)]
        # (A/B builds of older revisions, RTGPU_LIB_DIR, may lack the newer entry points)
        if hasattr(lib, "rt_ctx_create_multi"):
            lib.rt_ctx_create_multi.argtypes = [C.POINTER(I32), I32, C.POINTER(P)]
            lib.rt_ctx_num_devices.argtypes = [P]
            lib.rt_device_count.argtypes = [C.POINTER(I32)]
        if hasattr(lib, "rt_last_dealing"):
            lib.rt_last_dealing.argtypes = [P, C.POINTER(I32), C.POINTER(I32), I32]
        lib.rt_ctx_destroy.argtypes = [P]
        lib.rt_ctx_destroy.restype = None
        lib.rt_last_error.argtypes = [P]
        lib.rt_last_error.restype = C.c_char_p
        lib.rt_scene_upload.argtypes = [P, C.POINTER(RtSceneDesc)]
        lib.rt_scene_get_info.argtypes = [P, C.POINTER(RtSceneInfo)]
        lib.rt_last_build_ms.argtypes = [P, C.POINTER(C.c_double)]
        lib.rt_render.argtypes = [P, C.POINTER(RtCameraDesc), C.POINTER(RtRenderParams), C.POINTER(C.c_float),
                                  C.POINTER(RtStats)]
        lib.rt_render_device.argtypes = [P, C.POINTER(RtCameraDesc), C.POINTER(RtRenderParams), P, P]
        lib.rt_last_render_kernel_ms.argtypes = [P, C.POINTER(C.c_double)]
        lib.rt_sync.argtypes = [P]
        lib.rt_count_work.argtypes = [P, C.POINTER(RtCameraDesc), C.POINTER(RtRenderParams),
                                      C.POINTER(RtWorkCounts)]
        lib.rt_count_work_by_kernel.argtypes = [P, C.POINTER(RtCameraDesc), C.POINTER(RtRenderParams),
                                                C.POINTER(RtWorkCounts)]
        lib.rt_set_kernel_timing.argtypes = [P, C.c_int]
        if hasattr(lib, "rt_measure_read_bandwidth"):
            lib.rt_measure_read_bandwidth.argtypes = [P, C.c_uint64, I32, C.POINTER(C.c_double)]
        lib.rt_ctx_set_option.argtypes = [P, I32, I32]
        lib.rt_last_kernel_times.argtypes = [P, C.POINTER(RtKernelTimes)]
        lib.rt_tonemap_rgba8.argtypes = [P, C.POINTER(C.c_float), I32, I32, I32, C.POINTER(C.c_uint8)]
        lib.rt_primary_hits.argtypes = [P, C.POINTER(RtCameraDesc), U32, I32, C.POINTER(I32), C.POINTER(I32),
                                        C.POINTER(C.c_float)]
        if hasattr(lib, "rt_render_rgba8"):
            lib.rt_render_rgba8.argtypes = [P, C.POINTER(RtCameraDesc), C.POINTER(RtRenderParams),
                                            C.POINTER(C.c_uint8), C.POINTER(RtStats)]
            lib.rt_read_frame_sums.argtypes = [P, C.POINTER(C.c_float), C.c_int64]
        if hasattr(lib, "rt_extend_first_hits"):
            lib.rt_extend_first_hits.argtypes = [P, C.POINTER(RtCameraDesc), U32, I32, C.POINTER(I32),
                                                 C.POINTER(I32), C.POINTER(C.c_float)]
        if hasattr(lib, "rt_extend_hits"):
            lib.rt_extend_hits.argtypes = [P, C.POINTER(RtCameraDesc), U32, I32, I32, C.POINTER(I32), C.POINTER(I32),
                                           C.POINTER(C.c_float), C.POINTER(C.c_float)]
            lib.rt_shadow_visibility.argtypes = [P, C.POINTER(RtCameraDesc), U32, I32, I32, C.POINTER(I32)]
        _rtgpu = lib
    return _rtgpu


def rtscene() -> C.CDLL:
    """The host rt mirror (include/rtscene.h)."""
    global _rtscene
    if _rtscene is None:
        rtgpu()
        lib = _load("librtscene.so")
        P, I32 = C.c_void_p, C.c_int32
        lib.rts_scene_create.argtypes = [C.c_char_p, C.POINTER(RtsSceneOptions), C.POINTER(P), C.c_char_p, I32]
        lib.rts_scene_destroy.argtypes = [P]
        lib.rts_scene_destroy.restype = None
        lib.rts_scene_get_desc.argtypes = [P]
        lib.rts_scene_get_desc.restype = C.POINTER(RtSceneDesc)
        lib.rts_scene_get_camera.argtypes = [P]
        lib.rts_scene_get_camera.restype = C.POINTER(RtCameraDesc)
        lib.rts_scene_world_objects.argtypes = [P, C.POINTER(I32), I32]
        lib.rts_scene_world_objects.restype = I32
        lib.rts_renderer_create.argtypes = [P, I32, I32, I32, C.c_uint32, C.POINTER(P), C.c_char_p, I32]
        lib.rts_renderer_destroy.argtypes = [P]
        lib.rts_renderer_destroy.restype = None
        lib.rts_renderer_render_pass.argtypes = [P, I32]
        lib.rts_renderer_render_all.argtypes = [P]
        lib.rts_renderer_is_completed.argtypes = [P]
        lib.rts_renderer_framebuffer.argtypes = [P]
        lib.rts_renderer_framebuffer.restype = C.POINTER(C.c_uint8)
        lib.rts_renderer_accum.argtypes = [P]
        lib.rts_renderer_accum.restype = C.POINTER(C.c_float)
        lib.rts_renderer_duration_ms.argtypes = [P]
        lib.rts_renderer_duration_ms.restype = C.c_double
        lib.rts_renderer_save_png.argtypes = [P, C.c_char_p]
        lib.rts_renderer_last_error.argtypes = [P]
        lib.rts_renderer_last_error.restype = C.c_char_p
        if hasattr(lib, "rts_renderer_timings"):
            lib.rts_renderer_timings.argtypes = [P, C.POINTER(C.c_double)]
        lib.rts_load_hdr.argtypes = [C.c_char_p, C.POINTER(I32), C.POINTER(I32), C.POINTER(C.c_double), C.c_int64]
        lib.rts_write_synthetic_lucy_obj.argtypes = [C.c_char_p, I32, I32]
        lib.rts_obj_triangle_count.argtypes = [C.c_char_p]
        lib.rts_write_png.argtypes = [C.c_char_p, C.POINTER(C.c_uint8), I32, I32]
        _rtscene = lib
    return _rtscene


class RTError(RuntimeError):
    def __init__(self, code: int, msg: str = ""):
        super().__init__(f"{STATUS.get(code, code)}: {msg}")
        self.code = code


def _f32p(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def _i32p(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_int32))


# ---------------------------------------------------------------------------
# Scenes (scenes.go builders, via librtscene)
# ---------------------------------------------------------------------------
class Scene:
    """A BASELINE scene built by the host rt mirror; world wrapped in
    NewBVHNodeFromList like main.go:77."""

    def __init__(self, name: str, *, seed: int = 0x5EED, width: int = 0, aspect: float = 0.0, spp: int = 0,
                 max_depth: int = 0, asset_dir: Optional[str] = None, obj_path: Optional[str] = None,
                 lucy_rings: int = 0, lucy_cols: int = 0, motion: Optional[Sequence[Sequence[float]]] = None,
                 free_forward: Optional[Sequence[float]] = None):
        """`motion=(look_from2, look_at2)` applies Camera.SetMotion and
        `free_forward=(x, y, z)` Camera.EnableFreeCamera(LookFrom, forward,
        Vup) to the scene's camera before Build() (camera.go:204-232)."""
        lib = rtscene()
        self.name = name
        opt = RtsSceneOptions(seed, width, aspect, spp, max_depth, (asset_dir or ASSET_DIR).encode(),
                              obj_path.encode() if obj_path else None, lucy_rings, lucy_cols)
        if motion is not None:
            opt.camera_motion = 1
            opt.look_from2[:] = [float(x) for x in motion[0]]
            opt.look_at2[:] = [float(x) for x in motion[1]]
        if free_forward is not None:
            opt.free_camera = 1
            opt.forward[:] = [float(x) for x in free_forward]
        h = C.c_void_p()
        err = C.create_string_buffer(512)
        rc = lib.rts_scene_create(name.encode(), C.byref(opt), C.byref(h), err, 512)
        if rc != RT_OK:
            raise RTError(rc, err.value.decode())
        self._h = h
        self._lib = lib

    def __del__(self):
        if getattr(self, "_h", None):
            self._lib.rts_scene_destroy(self._h)
            self._h = None

    @property
    def desc(self):
        return self._lib.rts_scene_get_desc(self._h)

    @property
    def camera(self) -> RtCameraDesc:
        return self._lib.rts_scene_get_camera(self._h).contents

    @property
    def width(self) -> int:
        return self.camera.image_width

    @property
    def height(self) -> int:
        return self.camera.image_height

    def world_objects(self) -> np.ndarray:
        n = self._lib.rts_scene_world_objects(self._h, None, 0)
        out = np.zeros(max(n, 1), np.int32)
        self._lib.rts_scene_world_objects(self._h, _i32p(out), n)
        return out[:n]

    def hittables(self) -> np.ndarray:
        d = self.desc.contents
        return np.ctypeslib.as_array(C.cast(d.hittables, C.POINTER(C.c_byte)),
                                     shape=(d.num_hittables * C.sizeof(RtHittable),)).view(
            np.dtype([("kind", "<i4"), ("material", "<i4"), ("a", "<i4"), ("b", "<i4"), ("bbox", "<f8", 6),
                      ("p", "<f8", 16)])).copy()

    def children(self) -> np.ndarray:
        d = self.desc.contents
        if d.num_children == 0:
            return np.zeros(0, np.int32)
        return np.ctypeslib.as_array(d.children, shape=(d.num_children,)).copy()


def buckets_array(buckets: Sequence[Sequence[int]]):
    arr = (RtBucket * max(len(buckets), 1))()
    for i, b in enumerate(buckets):
        arr[i] = RtBucket(*[int(v) for v in b])
    return arr


def generate_buckets(width: int, height: int, bucket_size: int = 32):
    """rt.generateBuckets (bucket_renderer.go:77-125): centre-out order (stable)."""
    bs = []
    for y in range(0, height, bucket_size):
        for x in range(0, width, bucket_size):
            bs.append((x, y, min(bucket_size, width - x), min(bucket_size, height - y)))
    cx, cy = width // 2, height // 2
    bs.sort(key=lambda b: (b[0] + b[2] // 2 - cx) ** 2 + (b[1] + b[3] // 2 - cy) ** 2)
    return bs


def split_buckets(buckets, tile: int = 16):
    """Each bucket cut into tile x tile sub-buckets, in bucket order (the
    kernels' own work tiles are 16x16, api.cpp make_tiles)."""
    out = []
    for x, y, w, h in buckets:
        for ty in range(y, y + h, tile):
            for tx in range(x, x + w, tile):
                out.append((tx, ty, min(tile, x + w - tx), min(tile, y + h - ty)))
    return out


def shard_buckets(buckets, rank: int, world: int, tile: int = 0):
    """Round-robin tile sharding across ranks (bucket k -> rank k mod world):
    the centre-heavy cost of the centre-out bucket order is spread evenly
    (SURVEY.md §8(e)).  tile > 0 deals tile x tile sub-buckets instead (finer
    grain, better balance).  The RNG is keyed by global pixel id, so the
    combined frame is identical for any world size and grain."""
    if tile:
        buckets = split_buckets(buckets, tile)
    return [b for i, b in enumerate(buckets) if i % world == rank]


def make_params(spp: int, depth: int, seed: int = 1, sample_offset: int = 0, buckets=None, accumulate: bool = False):
    keep = None
    if buckets is not None:
        keep = buckets_array(buckets)
        p = RtRenderParams(spp, depth, sample_offset, seed, C.cast(keep, C.POINTER(RtBucket)), len(buckets),
                           1 if accumulate else 0)
    else:
        p = RtRenderParams(spp, depth, sample_offset, seed, None, 0, 1 if accumulate else 0)
    p._keep = keep
    return p


# ---------------------------------------------------------------------------
# GPU context (rt_ctx)
# ---------------------------------------------------------------------------
def device_count() -> int:
    """Visible HIP devices (rt_device_count)."""
    n = C.c_int32()
    rc = rtgpu().rt_device_count(C.byref(n))
    if rc != RT_OK:
        raise RTError(rc, "rt_device_count failed (no GPU?)")
    return n.value


class Context:
    """One device's flattened scene + render entry points (rtgpu.h).  With
    `devices=[d0, d1, ...]` one context over several devices
    (rt_ctx_create_multi): renders deal the buckets round-robin over them."""

    def __init__(self, device: int = 0, devices: Optional[Sequence[int]] = None):
        self._lib = rtgpu()
        h = C.c_void_p()
        if devices is not None and len(devices) > 0:
            arr = (C.c_int32 * len(devices))(*[int(d) for d in devices])
            rc = self._lib.rt_ctx_create_multi(arr, len(devices), C.byref(h))
            if rc != RT_OK:
                raise RTError(rc, f"rt_ctx_create_multi(devices={list(devices)}) failed")
            device = int(devices[0])
        else:
            rc = self._lib.rt_ctx_create(device, C.byref(h))
            if rc != RT_OK:
                raise RTError(rc, f"rt_ctx_create(device={device}) failed (no GPU?)")
        self._h = h
        self.device = device

    @property
    def num_devices(self) -> int:
        return int(self._lib.rt_ctx_num_devices(self._h))

    def set_dealing(self, mode: str = "static", first_share: int = 0):
        """Multi-device tile dealing (RT_OPT_DEALING): "static" (tile k to
        device k mod n) or "dynamic" (runs claimed from a shared counter as
        devices finish, bucket_renderer.go:193-213); first_share = the first
        run in percent of a fair share (0: default)."""
        self.set_option(RT_OPT_DEALING, {"static": RT_DEAL_STATIC, "dynamic": RT_DEAL_DYNAMIC}[mode])
        self.set_option(RT_OPT_DEAL_FIRST, first_share)

    def last_dealing(self):
        """(tiles, runs) per device of the last multi-device render."""
        n = self.num_devices
        tiles, runs = (C.c_int32 * n)(), (C.c_int32 * n)()
        self._check(self._lib.rt_last_dealing(self._h, tiles, runs, n))
        return list(tiles), list(runs)

    def close(self):
        if getattr(self, "_h", None):
            self._lib.rt_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def _check(self, rc: int):
        if rc != RT_OK:
            raise RTError(rc, self._lib.rt_last_error(self._h).decode())

    def upload(self, scene_desc) -> None:
        self._check(self._lib.rt_scene_upload(self._h, scene_desc))

    def info(self) -> RtSceneInfo:
        i = RtSceneInfo()
        self._check(self._lib.rt_scene_get_info(self._h, C.byref(i)))
        return i

    def render(self, camera: RtCameraDesc, params: RtRenderParams, accum: Optional[np.ndarray] = None):
        if accum is None:
            accum = np.zeros((camera.image_height, camera.image_width, 3), np.float32)
        st = RtStats()
        self._check(self._lib.rt_render(self._h, C.byref(camera), C.byref(params), _f32p(accum), C.byref(st)))
        return accum, st

    def render_rgba8(self, camera: RtCameraDesc, params: RtRenderParams):
        """One progressive pass (rt_render_rgba8): render + device quantisation;
        returns the (H, W, 4) RGBA8 framebuffer and the stats."""
        out = np.zeros((camera.image_height, camera.image_width, 4), np.uint8)
        st = RtStats()
        self._check(self._lib.rt_render_rgba8(self._h, C.byref(camera), C.byref(params),
                                              out.ctypes.data_as(C.POINTER(C.c_uint8)), C.byref(st)))
        return out, st

    def frame_sums(self, camera: RtCameraDesc) -> np.ndarray:
        """The device frame sums behind render_rgba8's framebuffer."""
        out = np.zeros((camera.image_height, camera.image_width, 3), np.float32)
        self._check(self._lib.rt_read_frame_sums(self._h, _f32p(out), out.size))
        return out

    def render_device(self, camera: RtCameraDesc, params: RtRenderParams, dev_ptr: int, stream: int = 0):
        self._check(self._lib.rt_render_device(self._h, C.byref(camera), C.byref(params), C.c_void_p(dev_ptr),
                                               C.c_void_p(stream)))

    def sync(self) -> None:
        """Wait for every enqueued render; raises RTError(RT_ERR_DEVICE) on a device error."""
        self._check(self._lib.rt_sync(self._h))

    def last_render_kernel_ms(self) -> float:
        ms = C.c_double()
        self._check(self._lib.rt_last_render_kernel_ms(self._h, C.byref(ms)))
        return ms.value

    def count_work(self, camera: RtCameraDesc, params: RtRenderParams) -> dict:
        w = RtWorkCounts()
        self._check(self._lib.rt_count_work(self._h, C.byref(camera), C.byref(params), C.byref(w)))
        return {n: int(getattr(w, n)) for n, _ in RtWorkCounts._fields_}

    def count_work_by_kernel(self, camera: RtCameraDesc, params: RtRenderParams) -> dict:
        """{"extend": counts, "shade": counts, "shadow": counts} (rt_count_work_by_kernel)."""
        w = (RtWorkCounts * 3)()
        self._check(self._lib.rt_count_work_by_kernel(self._h, C.byref(camera), C.byref(params), w))
        return {k: {n: int(getattr(w[i], n)) for n, _ in RtWorkCounts._fields_}
                for i, k in enumerate(("extend", "shade", "shadow"))}

    def set_option(self, key: int, value: int):
        self._check(self._lib.rt_ctx_set_option(self._h, key, value))

    def set_blas_builder(self, builder: str):
        """Mesh BLAS layout, next upload: "sah" (default, host binned SAH), "reference" (the
        caller's BVH topology) or "device" (LBVH built on the GPU, build.hip)."""
        self.set_option(RT_OPT_BLAS_BUILDER,
                        {"reference": RT_BLAS_REFERENCE, "sah": RT_BLAS_SAH, "device": RT_BLAS_DEVICE}[builder])

    def last_build_ms(self) -> float:
        """Wall time of the device BVH builds of the last upload (0 for host-built BLASes)."""
        ms = C.c_double()
        self._check(self._lib.rt_last_build_ms(self._h, C.byref(ms)))
        return ms.value

    def set_tlas_builder(self, builder: str):
        """World BVH layout: "sah" (default) or "reference"; next upload."""
        self.set_option(RT_OPT_TLAS_BUILDER, {"reference": RT_BLAS_REFERENCE, "sah": RT_BLAS_SAH}[builder])

    def set_node_format(self, fmt: str):
        """BVH4 node records: "fp32" (default, 128 B) or "quant8" (64 B,
        8-bit child planes with a conservative margin); next upload."""
        self.set_option(RT_OPT_NODE_FORMAT, {"fp32": RT_NODES_FP32, "quant8": RT_NODES_QUANT8, "wide8": RT_NODES_WIDE8}[fmt])

    def set_collapse(self, collapse: str):
        """BVH2 -> BVH4 collapse: "sah" (default, least total node area) or
        "greedy" (largest-area child first); same hits; next upload."""
        self.set_option(RT_OPT_BVH4_COLLAPSE, {"sah": RT_COLLAPSE_SAH, "greedy": RT_COLLAPSE_GREEDY}[collapse])

    def set_schedule(self, batch_slots: int = 0, refill: int = 0, max_blocks: int = 0, streams: int = 0):
        """Schedule options (0 = automatic) for the next renders: path slots per
        batch, idle lanes before a wave claims more rays, cap on the persistent
        traversal grids, one or two twin streams.  They never change the image
        (DESIGN.md §3)."""
        self.set_option(RT_OPT_BATCH_SLOTS, batch_slots)
        self.set_option(RT_OPT_REFILL, refill)
        self.set_option(RT_OPT_MAX_BLOCKS, max_blocks)
        self.set_option(RT_OPT_STREAMS, streams)

    def set_tail(self, paths: int = 0):
        """RT_OPT_TAIL for the next renders: 0 automatic, 1 off (every bounce
        through the per-bounce kernels), n > 1 = hand the paths left to the
        long-tail kernel once at most n remain (deep scenes without lights).
        Never changes the image."""
        self.set_option(RT_OPT_TAIL, paths)

    def set_overlap(self, mode: int = 0):
        """RT_OPT_OVERLAP for the next renders: 0 automatic (off), 1 off, 2 on
        (scenes with lights).  Bounce b's shadow rays and NEE adds run beside
        bounce b + 1's closest-hit kernel on a second stream per part.  Never
        changes the image."""
        self.set_option(RT_OPT_OVERLAP, mode)

    def measure_read_bandwidth(self, nbytes: int = 4 << 30, reps: int = 10) -> float:
        """The measured HBM read peak (GB/s): `reps` coalesced passes over a
        fresh `nbytes` device buffer (rt_measure_read_bandwidth)."""
        gbs = C.c_double(0.0)
        self._check(self._lib.rt_measure_read_bandwidth(self._h, C.c_uint64(nbytes), reps, C.byref(gbs)))
        return float(gbs.value)

    def set_kernel_timing(self, enable: bool = True):
        self._check(self._lib.rt_set_kernel_timing(self._h, 1 if enable else 0))

    def last_kernel_times(self) -> dict:
        t = RtKernelTimes()
        self._check(self._lib.rt_last_kernel_times(self._h, C.byref(t)))
        return {n: getattr(t, n) for n, _ in RtKernelTimes._fields_}

    def tonemap(self, accum: np.ndarray, spp: int) -> np.ndarray:
        h, w = accum.shape[:2]
        a = np.ascontiguousarray(accum, np.float32)
        out = np.zeros((h, w, 4), np.uint8)
        self._check(self._lib.rt_tonemap_rgba8(self._h, _f32p(a), w, h, spp,
                                               out.ctypes.data_as(C.POINTER(C.c_uint8))))
        return out

    def primary_hits(self, camera: RtCameraDesc, seed: int, sample: int = 0):
        n = camera.image_width * camera.image_height
        top = np.zeros(n, np.int32)
        prim = np.zeros(n, np.int32)
        t = np.zeros(n, np.float32)
        self._check(self._lib.rt_primary_hits(self._h, C.byref(camera), seed, sample, _i32p(top), _i32p(prim),
                                              _f32p(t)))
        return top, prim, t

    def extend_first_hits(self, camera: RtCameraDesc, seed: int, sample: int = 0):
        """primary_hits' ids from the production pipeline's first k_extend."""
        n = camera.image_width * camera.image_height
        top = np.zeros(n, np.int32)
        prim = np.zeros(n, np.int32)
        t = np.zeros(n, np.float32)
        self._check(self._lib.rt_extend_first_hits(self._h, C.byref(camera), seed, sample, _i32p(top), _i32p(prim),
                                                   _f32p(t)))
        return top, prim, t

    def extend_hits(self, camera: RtCameraDesc, seed: int, sample: int, bounce: int):
        """Closest hit of every pixel's bounce-`bounce` ray from the production
        k_extend (rt_extend_hits): top, prim (-1 miss, -2 path ended), t, and
        the incoming ray (n, 6) float32 (origin, direction)."""
        n = camera.image_width * camera.image_height
        top = np.zeros(n, np.int32)
        prim = np.zeros(n, np.int32)
        t = np.zeros(n, np.float32)
        ray = np.zeros((n, 6), np.float32)
        self._check(self._lib.rt_extend_hits(self._h, C.byref(camera), seed, sample, bounce, _i32p(top), _i32p(prim),
                                             _f32p(t), _f32p(ray)))
        return top, prim, t, ray

    def shadow_visibility(self, camera: RtCameraDesc, seed: int, sample: int, bounce: int) -> np.ndarray:
        """NEE shadow rays of bounce `bounce` per pixel (rt_shadow_visibility):
        bits 0/1 area/HDRI ray traced, bits 2/3 unoccluded."""
        n = camera.image_width * camera.image_height
        nee = np.zeros(n, np.int32)
        self._check(self._lib.rt_shadow_visibility(self._h, C.byref(camera), seed, sample, bounce, _i32p(nee)))
        return nee


# ---------------------------------------------------------------------------
# rt.NewBucketRenderer analogue (progressive 3-pass, RGBA8 framebuffer)
# ---------------------------------------------------------------------------
class BucketRenderer:
    """NewBucketRenderer(camera, world, bucketSize, numWorkers) on the GPU
    (bucket_renderer.go:54-74); passes as in renderPass (:170-214)."""

    def __init__(self, scene: Scene, bucket_size: int = 32, num_workers: int = 0, device: int = 0, seed: int = 1):
        self._lib = rtscene()
        self.scene = scene
        h = C.c_void_p()
        err = C.create_string_buffer(512)
        rc = self._lib.rts_renderer_create(scene._h, bucket_size, num_workers, device, seed, C.byref(h), err, 512)
        if rc != RT_OK:
            raise RTError(rc, err.value.decode())
        self._h = h

    def __del__(self):
        if getattr(self, "_h", None):
            self._lib.rts_renderer_destroy(self._h)
            self._h = None

    def _check(self, rc):
        if rc != RT_OK:
            raise RTError(rc, self._lib.rts_renderer_last_error(self._h).decode())

    def render_pass(self, p: int):
        self._check(self._lib.rts_renderer_render_pass(self._h, p))

    def render_all(self):
        self._check(self._lib.rts_renderer_render_all(self._h))

    def is_completed(self) -> bool:
        return bool(self._lib.rts_renderer_is_completed(self._h))

    def framebuffer(self) -> np.ndarray:
        w, h = self.scene.width, self.scene.height
        p = self._lib.rts_renderer_framebuffer(self._h)
        return np.ctypeslib.as_array(p, shape=(h, w, 4)).copy()

    def accum(self) -> np.ndarray:
        w, h = self.scene.width, self.scene.height
        return np.ctypeslib.as_array(self._lib.rts_renderer_accum(self._h), shape=(h, w, 3)).copy()

    def duration_ms(self) -> float:
        return float(self._lib.rts_renderer_duration_ms(self._h))

    def timings(self) -> dict:
        """Construction ms (context + scene upload), each pass's wall ms (host
        buffers + tonemap) and its device render ms."""
        t = (C.c_double * 7)()
        self._check(self._lib.rts_renderer_timings(self._h, t))
        return {"create_ms": t[0], "pass_wall_ms": [t[1], t[2], t[3]], "pass_render_ms": [t[4], t[5], t[6]]}

    def save_image(self, path: str):
        self._check(self._lib.rts_renderer_save_png(self._h, path.encode()))


def load_hdr(path: str):
    lib = rtscene()
    w = C.c_int32()
    h = C.c_int32()
    rc = lib.rts_load_hdr(path.encode(), C.byref(w), C.byref(h), None, 0)
    if rc != RT_OK:
        raise RTError(rc, path)
    out = np.zeros((h.value, w.value, 3), np.float64)
    rc = lib.rts_load_hdr(path.encode(), C.byref(w), C.byref(h), out.ctypes.data_as(C.POINTER(C.c_double)),
                          out.size)
    if rc != RT_OK:
        raise RTError(rc, path)
    return out


def write_png(path: str, rgba: np.ndarray):
    a = np.ascontiguousarray(rgba, np.uint8)
    rc = rtscene().rts_write_png(path.encode(), a.ctypes.data_as(C.POINTER(C.c_uint8)), a.shape[1], a.shape[0])
    if rc != RT_OK:
        raise RTError(rc, path)
