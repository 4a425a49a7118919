"""SaveImage (bucket_renderer.go:417-438) PNG writer of the host mirror
(librtscene rts_write_png): decodes back to the exact RGBA8 buffer, CRCs valid,
multi-block (>64 KiB) zlib stream included.  CPU only."""
import numpy as np
import pytest

from tests.pngdec import read_png


@pytest.mark.parametrize("w,h", [(1, 1), (37, 53), (300, 200)])
def test_png_round_trip(g, tmp_path, w, h):
    rng = np.random.default_rng(w * 1000 + h)
    img = rng.integers(0, 256, (h, w, 4), dtype=np.uint8)
    path = tmp_path / "img.png"
    g.write_png(str(path), img)
    assert np.array_equal(read_png(str(path)), img)
