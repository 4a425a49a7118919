"""Tiny Python builder of rt_scene_desc graphs (same fields the Go
constructors fill, scenes built by hand) for oracle known-answer tests."""
import ctypes as C

import numpy as np


class Builder:
    def __init__(self, g):
        self.g = g
        self.h = []
        self.children = []
        self.mats = []
        self.texs = []
        self.lights = []

    # materials / textures -------------------------------------------------
    def solid(self, rgb):
        t = self.g.RtTexture(self.g.RT_TEX_SOLID, -1, -1, (C.c_double * 3)(*rgb), 0.0)
        self.texs.append(t)
        return len(self.texs) - 1

    def checker(self, scale, even, odd):
        e, o = self.solid(even), self.solid(odd)
        self.texs.append(self.g.RtTexture(self.g.RT_TEX_CHECKER, e, o, (C.c_double * 3)(0, 0, 0), 1.0 / scale))
        return len(self.texs) - 1

    def mat(self, kind, tex=-1, albedo=(0, 0, 0), fuzz=0.0, ior=0.0):
        self.mats.append(self.g.RtMaterial(kind, tex, (C.c_double * 3)(*albedo), min(fuzz, 1.0), ior))
        return len(self.mats) - 1

    def lambertian(self, rgb):
        return self.mat(self.g.RT_LAMBERTIAN, self.solid(rgb))

    def light(self, rgb):
        return self.mat(self.g.RT_DIFFUSE_LIGHT, self.solid(rgb))

    # hittables --------------------------------------------------------------
    def _add(self, kind, mat, a, b, bbox, p):
        e = self.g.RtHittable()
        e.kind, e.material, e.a, e.b = kind, mat, a, b
        for i, v in enumerate(bbox):
            e.bbox[i] = v
        for i, v in enumerate(p):
            e.p[i] = v
        self.h.append(e)
        return len(self.h) - 1

    @staticmethod
    def _pad(b):
        b = list(b)
        for a in range(3):
            if b[2 * a + 1] - b[2 * a] < 1e-4:
                b[2 * a] -= 1e-4
                b[2 * a + 1] += 1e-4
        return b

    def sphere(self, c, r, mat, vel=(0, 0, 0)):
        c = np.array(c, float)
        c2 = c + np.array(vel, float)
        lo, hi = np.minimum(c, c2) - r, np.maximum(c, c2) + r
        return self._add(self.g.RT_SPHERE, mat, 0, 0, self._pad([lo[0], hi[0], lo[1], hi[1], lo[2], hi[2]]),
                         list(c) + list(vel) + [r])

    def quad(self, Q, u, v, mat):
        Q, u, v = (np.array(x, float) for x in (Q, u, v))
        n = np.cross(u, v)
        normal = n / np.linalg.norm(n)
        D = float(normal @ Q)
        w = n / float(n @ n)
        pts = np.array([Q, Q + u + v, Q + u, Q + v])
        lo, hi = pts.min(0), pts.max(0)
        b = [lo[0], hi[0], lo[1], hi[1], lo[2], hi[2]]
        return self._add(self.g.RT_QUAD, mat, 0, 0, self._pad(b), list(Q) + list(u) + list(v) + list(w) + list(normal) + [D])

    def triangle(self, a, b, c, mat):
        a, b, c = (np.array(x, float) for x in (a, b, c))
        n = np.cross(b - a, c - a)
        n = n / np.linalg.norm(n)
        pts = np.array([a, b, c])
        lo, hi = pts.min(0), pts.max(0)
        return self._add(self.g.RT_TRIANGLE, mat, 0, 0, self._pad([lo[0], hi[0], lo[1], hi[1], lo[2], hi[2]]),
                         list(a) + list(b) + list(c) + list(n))

    def plane(self, p, n, mat):
        n = np.array(n, float)
        n = n / np.linalg.norm(n)
        inf = float("inf")
        return self._add(self.g.RT_PLANE, mat, 0, 0, [-inf, inf, -inf, inf, -inf, inf], list(p) + list(n))

    def listing(self, kids, kind=None):
        kind = kind or self.g.RT_LIST
        first = len(self.children)
        self.children.extend(kids)
        bb = [min(self.h[k].bbox[0] for k in kids), max(self.h[k].bbox[1] for k in kids),
              min(self.h[k].bbox[2] for k in kids), max(self.h[k].bbox[3] for k in kids),
              min(self.h[k].bbox[4] for k in kids), max(self.h[k].bbox[5] for k in kids)]
        return self._add(kind, -1, first, len(kids), bb, [])

    def leaf_node(self, kids):
        """BVHNode{leaf, leaf} (bvh.go:141)."""
        lf = self.listing(kids, self.g.RT_BVH_LEAF)
        return self._add(self.g.RT_BVH_NODE, -1, lf, lf, list(self.h[lf].bbox), [])

    def translate(self, child, off):
        b = list(self.h[child].bbox)
        bb = self._pad([b[0] + off[0], b[1] + off[0], b[2] + off[1], b[3] + off[1], b[4] + off[2], b[5] + off[2]])
        return self._add(self.g.RT_TRANSLATE, -1, child, 0, bb, list(off))

    def rotate_y(self, child, sin_t, cos_t):
        """RotateY (transform.go:113-157): bbox = the child's corners rotated."""
        b = self.h[child].bbox
        pts = np.array([[x, y, z] for x in b[0:2] for y in b[2:4] for z in b[4:6]], float)
        nx = cos_t * pts[:, 0] + sin_t * pts[:, 2]
        nz = -sin_t * pts[:, 0] + cos_t * pts[:, 2]
        bb = [nx.min(), nx.max(), pts[:, 1].min(), pts[:, 1].max(), nz.min(), nz.max()]
        return self._add(self.g.RT_ROTATE_Y, -1, child, 0, self._pad(bb), [sin_t, cos_t])

    def rotate_x(self, child, sin_t, cos_t):
        """RotateX (transform.go:201-237): bbox = the child's corners rotated about x."""
        b = self.h[child].bbox
        pts = np.array([[x, y, z] for x in b[0:2] for y in b[2:4] for z in b[4:6]], float)
        ny = cos_t * pts[:, 1] - sin_t * pts[:, 2]
        nz = sin_t * pts[:, 1] + cos_t * pts[:, 2]
        bb = [pts[:, 0].min(), pts[:, 0].max(), ny.min(), ny.max(), nz.min(), nz.max()]
        return self._add(self.g.RT_ROTATE_X, -1, child, 0, self._pad(bb), [sin_t, cos_t])

    def bvh_node(self, left, right):
        """BVHNode{left, right} (bvh.go): bbox = the union of the children's."""
        l, r = self.h[left].bbox, self.h[right].bbox
        bb = [min(l[0], r[0]), max(l[1], r[1]), min(l[2], r[2]), max(l[3], r[3]), min(l[4], r[4]), max(l[5], r[5])]
        return self._add(self.g.RT_BVH_NODE, -1, left, right, bb, [])

    def scale(self, child, f):
        """Scale (transform.go:360-403): bbox corners times the factor."""
        b = self.h[child].bbox
        lo = [b[0] * f[0], b[2] * f[1], b[4] * f[2]]
        hi = [b[1] * f[0], b[3] * f[1], b[5] * f[2]]
        bb = []
        for a in range(3):
            bb += [min(lo[a], hi[a]), max(lo[a], hi[a])]
        return self._add(self.g.RT_SCALE, -1, child, 0, self._pad(bb), list(f) + [1.0 / x for x in f])

    def volume(self, boundary, density, mat):
        return self._add(self.g.RT_VOLUME, mat, boundary, 0, list(self.h[boundary].bbox), [-1.0 / density])

    # desc -------------------------------------------------------------------
    def desc(self, root, env=None):
        self._harr = (self.g.RtHittable * len(self.h))(*self.h)
        self._carr = (C.c_int32 * max(len(self.children), 1))(*self.children)
        self._marr = (self.g.RtMaterial * max(len(self.mats), 1))(*self.mats)
        self._tarr = (self.g.RtTexture * max(len(self.texs), 1))(*self.texs)
        self._larr = (C.c_int32 * max(len(self.lights), 1))(*self.lights)
        d = self.g.RtSceneDesc()
        d.hittables = C.cast(self._harr, C.POINTER(self.g.RtHittable))
        d.num_hittables = len(self.h)
        d.children = C.cast(self._carr, C.POINTER(C.c_int32))
        d.num_children = len(self.children)
        d.root = root
        d.materials = C.cast(self._marr, C.POINTER(self.g.RtMaterial))
        d.num_materials = len(self.mats)
        d.textures = C.cast(self._tarr, C.POINTER(self.g.RtTexture))
        d.num_textures = len(self.texs)
        d.lights = C.cast(self._larr, C.POINTER(C.c_int32))
        d.num_lights = len(self.lights)
        d.environment = None
        self._desc = d
        return d


def pinhole(g, w, h, origin, pixel00, du, dv, max_depth=5, sky=False, bg=(0, 0, 0)):
    c = g.RtCameraDesc()
    c.image_width, c.image_height, c.samples_per_pixel, c.max_depth = w, h, 1, max_depth
    for i in range(3):
        c.center[i], c.pixel00[i], c.pixel_delta_u[i], c.pixel_delta_v[i] = origin[i], pixel00[i], du[i], dv[i]
        c.background[i] = bg[i]
    c.use_sky_gradient = 1 if sky else 0
    return c
