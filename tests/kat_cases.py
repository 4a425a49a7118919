"""Hand-derived known-answer cases for the parts of the path the reference
holds no fixture for (NEE, instance transforms, volumes).  Each case builds a
tiny scene with the Builder and derives its expected values in closed form
from the cited Go code, independently of the oracle's restatement.  The
oracle (both modes, tests/test_oracle_kat.py) and the GPU (through the C-ABI,
tests/test_gpu_kat.py) are held to the same expected values.

These are not reference-held fixtures: parity for these features stays
"partial" (DESIGN.md §5)."""
import math

import numpy as np

from tests.scene_builder import Builder, pinhole

SEED = 3
DOM_SCATTER, DOM_NEE, DOM_VOL = 1, 3, 4


def lowbias32(x):
    x &= 0xFFFFFFFF
    x ^= x >> 16
    x = (x * 0x7FEB352D) & 0xFFFFFFFF
    x ^= x >> 15
    x = (x * 0x846CA68B) & 0xFFFFFFFF
    x ^= x >> 16
    return x


def rnd(seed, pixel, sample, bounce, dom, idx):
    """DESIGN.md §3 RNG: u = (draw >> 8) * 2^-24 for counter (bounce, domain, index)."""
    k = lowbias32(seed ^ 0xA511E9B3)
    k = lowbias32(k ^ pixel)
    k = lowbias32((k + sample * 0x9E3779B9) & 0xFFFFFFFF)
    ctr = (bounce << 16) | (dom << 12) | idx
    return (lowbias32(k ^ lowbias32(ctr ^ 0x632BE5AB)) >> 8) * 2.0 ** -24


def random_unit_vector(seed, pixel, sample, bounce):
    """RandomUnitVector (vec3.go:45-54): rejection in the cube, draws
    3k, 3k+1, 3k+2 of the scatter domain."""
    for k in range(64):
        p = np.array([-1 + 2 * rnd(seed, pixel, sample, bounce, DOM_SCATTER, 3 * k + i) for i in range(3)])
        l2 = float(p @ p)
        if 1e-160 < l2 <= 1:
            return p / math.sqrt(l2)
    return np.array([0.0, 0.0, 1.0])


def straight_camera(g, n, origin, direction, depth):
    """n x 1 pixels that all shoot the same ray (zero pixel deltas; the RNG
    is still keyed per pixel)."""
    p00 = tuple(o + d for o, d in zip(origin, direction))
    return pinhole(g, n, 1, origin, p00, (0, 0, 0), (0, 0, 0), max_depth=depth)


# --------------------------------------------------------------------------
# 1. sampleAreaLight (camera.go:610-678) over a Lambertian floor.
#    Floor y = 0 (normal +y), hit point P = origin from a camera at (0, 1, 0)
#    looking down (t = 1); two unit-area lights facing down at y = 2, so for a
#    light point at distance d: cos(theta) = cos(light) = 2/d, pdfL =
#    d^2 / (cos(light) * 1) = d^3 / 2, pdfB = cos(theta)/pi = 2/(pi d), and
#    emission * cos(theta)/pdfL * w = E * 4/d^4 / (1 + 4/(pi d^4)); times the
#    albedo and the number of lights (2), each component clamped to 20.
#    Depth 1: the bounce's indirect term is 0 and L = direct.
# --------------------------------------------------------------------------
AREA_LIGHTS = [((-0.5, 2.0, -0.5), (1.0, 0.0, 0.0), (0.0, 0.0, 1.0)),
               ((3.0, 2.0, -0.5), (1.0, 0.0, 0.0), (0.0, 0.0, 1.0))]
AREA_E = (400.0, 2.0, 1.0)
AREA_ALBEDO = (0.5, 0.25, 0.125)
AREA_N = 64


def area_light_scene(g):
    b = Builder(g)
    floor = b.quad((-5, 0, 5), (10, 0, 0), (0, 0, -10), b.lambertian(AREA_ALBEDO))
    lm = b.light(AREA_E)
    lights = [b.quad(Q, u, v, lm) for Q, u, v in AREA_LIGHTS]
    b.lights = lights
    root = b.listing([floor] + lights)
    cam = straight_camera(g, AREA_N, (0, 1, 0), (0, -1, 0), 1)
    return b, b.desc(root), cam


def area_light_expected(spp=1):
    """(AREA_N, 3) per-pixel radiance sums of `spp` samples."""
    out = np.zeros((AREA_N, 3))
    for pix in range(AREA_N):
        for s in range(spp):
            li = min(int(rnd(SEED, pix, s, 0, DOM_NEE, 0) * 2), 1)
            al, be = rnd(SEED, pix, s, 0, DOM_NEE, 1), rnd(SEED, pix, s, 0, DOM_NEE, 2)
            Q, u, v = (np.array(x) for x in AREA_LIGHTS[li])
            lp = Q + al * u + be * v                      # Quad.SamplePoint (quad.go:87-92)
            d = float(np.linalg.norm(lp))
            f = 4.0 / d ** 4 / (1.0 + 4.0 / (math.pi * d ** 4))
            out[pix] += np.minimum(np.array(AREA_E) * f * np.array(AREA_ALBEDO) * 2.0, 20.0)
    return out


# --------------------------------------------------------------------------
# 2. Translate(RotateY(Scale(quad))) (transform.go:93-106, 159-191,
#    408-444).  The object-space quad Q = (-1,-1,0), u = (2,0,0), v = (0,2,2)
#    (normal (0,-1,1)/sqrt 2) is scaled by (1, 2, 0.5), rotated by
#    sin 0.6 / cos 0.8 and moved by (0, 0, -5).  The camera ray from the
#    origin aims at the world image of the object point (0.25, 0.5, 1.5)
#    (alpha 0.625, beta 0.75), with direction = that point, so t = 1 in
#    every space (the transforms map the ray, not t).  The hit point is the
#    world point; the normal is (0,-1,1) flipped to face the object-space ray,
#    times the inverse factor, renormalised (Scale), then rotated back.  The
#    bounce-1 ray starts at P with direction N + RandomUnitVector (Lambertian,
#    material.go:57-68).
# --------------------------------------------------------------------------
INST_F = (1.0, 2.0, 0.5)
INST_SIN, INST_COS = 0.6, 0.8
INST_OFF = (0.0, 0.0, -5.0)
INST_OBJ_POINT = np.array([0.25, 0.5, 1.5])


def _rot_back(p):          # RotateY.Hit's back-map of P and N (transform.go:175-184)
    return np.array([INST_COS * p[0] + INST_SIN * p[2], p[1], -INST_SIN * p[0] + INST_COS * p[2]])


def _rot_in(p):            # RotateY.Hit's ray map (transform.go:163-167)
    return np.array([INST_COS * p[0] - INST_SIN * p[2], p[1], INST_SIN * p[0] + INST_COS * p[2]])


def instance_world_point():
    return _rot_back(INST_OBJ_POINT * np.array(INST_F)) + np.array(INST_OFF)


def instance_scene(g):
    b = Builder(g)
    q = b.quad((-1, -1, 0), (2, 0, 0), (0, 2, 2), b.lambertian((0.5, 0.5, 0.5)))
    top = b.translate(b.rotate_y(b.scale(q, INST_F), INST_SIN, INST_COS), INST_OFF)
    root = b.listing([top])
    cam = straight_camera(g, 8, (0, 0, 0), tuple(instance_world_point()), 2)
    return b, b.desc(root), cam, top, q


def instance_expected_normal():
    d_world = instance_world_point()
    d_obj = _rot_in(d_world) / np.array(INST_F)              # Translate leaves d; RotateY; Scale by 1/f
    n = np.array([0.0, -1.0, 1.0]) / math.sqrt(2.0)
    n = n if float(d_obj @ n) < 0 else -n                   # SetFaceNormal (hittable.go:20-30)
    n = n / np.array(INST_F)
    n = n / np.linalg.norm(n)                               # Scale: Normal * InvFactor, Unit()
    return _rot_back(n)


# --------------------------------------------------------------------------
# 3. Volume.Hit (volume.go:34-79) with the free flight from a fixed draw.
#    A slab boundary z in [-4, -2] (two quads) around the -z camera ray: t1 =
#    2, t2 = 4, |d| = 1, so the ray scatters iff -ln(U)/rho <= 2 and then at
#    t = 2 - ln(U)/rho, U = the draw (bounce 0, DOM_VOL, 4 * vol_id); else it
#    hits the back wall at t = 10.  One test per traversal (list root).
# --------------------------------------------------------------------------
VOL_RHO = 0.35
VOL_N = 256


def volume_scene(g):
    b = Builder(g)
    wm = b.lambertian((0.5, 0.5, 0.5))
    faces = [b.quad((-1, -1, -2), (2, 0, 0), (0, 2, 0), wm), b.quad((-1, -1, -4), (2, 0, 0), (0, 2, 0), wm)]
    boundary = b.listing(faces)
    vol = b.volume(boundary, VOL_RHO, b.mat(g.RT_ISOTROPIC, b.solid((1, 1, 1))))
    back = b.quad((-5, -5, -10), (10, 0, 0), (0, 10, 0), wm)
    root = b.listing([vol, back])
    cam = straight_camera(g, VOL_N, (0, 0, 0), (0, 0, -1), 5)
    return b, b.desc(root), cam, vol, back


def volume_expected(sample=0):
    """(prim ids, t) per pixel: the volume at 2 - ln(U)/rho, else the back wall at 10."""
    ids, ts = [], []
    for pix in range(VOL_N):
        u = rnd(SEED, pix, sample, 0, DOM_VOL, 0)
        hd = -math.log(u) / VOL_RHO if u > 0 else math.inf
        if hd <= 2.0:
            ids.append("vol")
            ts.append(2.0 + hd)
        else:
            ids.append("back")
            ts.append(10.0)
    return ids, np.array(ts)
