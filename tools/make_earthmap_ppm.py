"""Converts the reference's texture asset assets/images/earthmap.jpg (EarthScene,
scenes.go:216) to the 8-bit binary PPM the C++ scene mirror loads
(assets/images/earthmap.ppm).  JPEG decoding is PIL's (libjpeg); Go's
image/jpeg may differ from it by one 8-bit level in some pixels."""
import sys

from PIL import Image

src = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/assets/images/earthmap.jpg"
dst = sys.argv[2] if len(sys.argv) > 2 else "assets/images/earthmap.ppm"
Image.open(src).convert("RGB").save(dst, format="PPM")
print(dst)
