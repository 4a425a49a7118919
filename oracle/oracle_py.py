"""ctypes binding of the CPU oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg as the checker / CPU baseline — never by the
product path (go-raytracing_amd/).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        path = os.path.join(HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        P = C.c_void_p
        L.oracle_render.argtypes = [P, P, P, C.c_int, C.c_int, C.POINTER(C.c_double)]
        L.oracle_primary_hits.argtypes = [P, P, C.c_uint32, C.c_int32, C.c_int, C.POINTER(C.c_int32),
                                          C.POINTER(C.c_int32), C.POINTER(C.c_double)]
        L.oracle_path_records.argtypes = [P, P, C.c_uint32, C.c_int32, C.c_int32, C.c_int, C.c_int,
                                          C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(C.c_double),
                                          C.POINTER(C.c_double), C.POINTER(C.c_int32)]
        L.oracle_tonemap.argtypes = [C.POINTER(C.c_float), C.c_int64, C.c_int32, C.POINTER(C.c_uint8)]
        L.oracle_tonemap.restype = None
        L.oracle_rng_uniform.argtypes = [C.c_uint32] * 4
        L.oracle_rng_uniform.restype = C.c_double
        L.oracle_logf32.argtypes = [C.POINTER(C.c_float), C.POINTER(C.c_float), C.c_int64]
        L.oracle_logf32.restype = None
        L.oracle_build_bvh.argtypes = [C.POINTER(C.c_double), C.c_int32, C.POINTER(C.c_int32), C.c_int32]
        L.oracle_load_hdr.argtypes = [C.c_char_p, C.POINTER(C.c_int32), C.POINTER(C.c_int32),
                                      C.POINTER(C.c_double), C.c_int64]
        L.oracle_hdri_total_power.argtypes = [C.POINTER(C.c_double), C.c_int32, C.c_int32]
        L.oracle_hdri_total_power.restype = C.c_double
        _lib = L
    return _lib


def _ptr(x):
    if isinstance(x, C._Pointer):
        return C.cast(x, C.c_void_p)
    return C.cast(C.pointer(x), C.c_void_p)


def render(scene_desc, camera, params, fp32: bool = False, threads: int = 0, accum=None) -> np.ndarray:
    """Sum of per-sample radiance (H, W, 3) float64."""
    if accum is None:
        accum = np.zeros((camera.image_height, camera.image_width, 3), np.float64)
    threads = threads or os.cpu_count() or 1
    rc = lib().oracle_render(_ptr(scene_desc), _ptr(camera), _ptr(params), 1 if fp32 else 0, threads,
                             accum.ctypes.data_as(C.POINTER(C.c_double)))
    if rc != 0:
        raise RuntimeError(f"oracle_render failed: {rc}")
    return accum


def primary_hits(scene_desc, camera, seed: int, sample: int = 0, fp32: bool = True):
    n = camera.image_width * camera.image_height
    top = np.zeros(n, np.int32)
    prim = np.zeros(n, np.int32)
    t = np.zeros(n, np.float64)
    rc = lib().oracle_primary_hits(_ptr(scene_desc), _ptr(camera), seed, sample, 1 if fp32 else 0,
                                   top.ctypes.data_as(C.POINTER(C.c_int32)),
                                   prim.ctypes.data_as(C.POINTER(C.c_int32)), t.ctypes.data_as(C.POINTER(C.c_double)))
    if rc != 0:
        raise RuntimeError(f"oracle_primary_hits failed: {rc}")
    return top, prim, t


def path_records(scene_desc, camera, seed: int, sample: int, num_bounces: int, fp32: bool = True, threads: int = 0):
    """Per bounce b < num_bounces (arrays of shape (num_bounces, W*H)): top,
    prim (-1 miss, -2 path ended), t, the incoming ray (..., 6) and the NEE
    bits (oracle.h oracle_path_records)."""
    n = camera.image_width * camera.image_height
    top = np.zeros((num_bounces, n), np.int32)
    prim = np.zeros((num_bounces, n), np.int32)
    t = np.zeros((num_bounces, n), np.float64)
    ray = np.zeros((num_bounces, n, 6), np.float64)
    nee = np.zeros((num_bounces, n), np.int32)
    threads = threads or min(16, os.cpu_count() or 1)
    rc = lib().oracle_path_records(_ptr(scene_desc), _ptr(camera), seed, sample, num_bounces, 1 if fp32 else 0, threads,
                                   top.ctypes.data_as(C.POINTER(C.c_int32)), prim.ctypes.data_as(C.POINTER(C.c_int32)),
                                   t.ctypes.data_as(C.POINTER(C.c_double)), ray.ctypes.data_as(C.POINTER(C.c_double)),
                                   nee.ctypes.data_as(C.POINTER(C.c_int32)))
    if rc != 0:
        raise RuntimeError(f"oracle_path_records failed: {rc}")
    return top, prim, t, ray, nee


def tonemap(accum_f32: np.ndarray, spp: int) -> np.ndarray:
    a = np.ascontiguousarray(accum_f32, np.float32)
    h, w = a.shape[:2]
    out = np.zeros((h, w, 4), np.uint8)
    lib().oracle_tonemap(a.ctypes.data_as(C.POINTER(C.c_float)), h * w, spp, out.ctypes.data_as(C.POINTER(C.c_uint8)))
    return out


def rng_uniform(seed, pixel, sample, counter) -> float:
    return lib().oracle_rng_uniform(seed, pixel, sample, counter)


def build_bvh(boxes: np.ndarray) -> list:
    b = np.ascontiguousarray(boxes, np.float64)
    n = b.shape[0]
    cap = 4 * n + 16
    out = np.zeros(cap, np.int32)
    ln = lib().oracle_build_bvh(b.ctypes.data_as(C.POINTER(C.c_double)), n, out.ctypes.data_as(C.POINTER(C.c_int32)),
                                cap)
    if ln < 0:
        raise RuntimeError("oracle_build_bvh: capacity")
    return out[:ln].tolist()


def load_hdr(path: str) -> np.ndarray:
    w = C.c_int32()
    h = C.c_int32()
    if lib().oracle_load_hdr(path.encode(), C.byref(w), C.byref(h), None, 0) != 0:
        raise RuntimeError("oracle_load_hdr header")
    out = np.zeros((h.value, w.value, 3), np.float64)
    if lib().oracle_load_hdr(path.encode(), C.byref(w), C.byref(h), out.ctypes.data_as(C.POINTER(C.c_double)),
                             out.size) != 0:
        raise RuntimeError("oracle_load_hdr data")
    return out


def hdri_total_power(rgb: np.ndarray) -> float:
    a = np.ascontiguousarray(rgb, np.float64)
    return lib().oracle_hdri_total_power(a.ctypes.data_as(C.POINTER(C.c_double)), a.shape[1], a.shape[0])
