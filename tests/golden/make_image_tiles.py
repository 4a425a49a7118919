"""Fixture from the reference's only output artifact, /root/reference/image.png.

HDRITestScene (scenes.go:415-455) rendered by the Go BucketRenderer at
800x450, 200 spp, depth 20 (stats bar burned into the bottom 30 rows,
bucket_renderer.go:396-403).  The Go RNG is unseeded, so only
statistics can be compared: this script stores the mean 8-bit RGB of 50x50
tiles over rows 0..399 (16 x 8 tiles).  Run once in the build container
(the reference is not on the GPU box); the JSON is the committed data.

    python tests/golden/make_image_tiles.py
"""
import json
import os

import numpy as np
from PIL import Image

SRC = "/root/reference/image.png"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "hdri_test_image_tiles.json")


def tile_means(rgb: np.ndarray, tile: int = 50, rows: int = 400) -> np.ndarray:
    h, w = rows // tile, rgb.shape[1] // tile
    a = rgb[:rows, : w * tile, :3].astype(np.float64)
    return a.reshape(h, tile, w, tile, 3).mean(axis=(1, 3))


def main():
    img = np.asarray(Image.open(SRC).convert("RGB"))
    assert img.shape == (450, 800, 3), img.shape
    m = tile_means(img)
    json.dump({"source": "reference image.png (HDRITestScene 800x450, 200 spp, depth 20, Go CPU renderer)",
               "tile": 50, "rows": 400, "means_rgb8": np.round(m, 3).tolist(),
               "image_mean_rgb8": np.round(img[:400].reshape(-1, 3).mean(axis=0), 3).tolist()},
              open(OUT, "w"), indent=0)
    print("wrote", OUT, m.shape)


if __name__ == "__main__":
    main()
