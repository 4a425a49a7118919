"""Minimal PNG reader for the tests (8-bit RGBA, non-interlaced; all five
scanline filters), checking every chunk CRC: enough to decode the renderer's
SaveImage output (bucket_renderer.go:417-438) back to the framebuffer."""
import struct
import zlib

import numpy as np


def _paeth(a, b, c):
    p = a + b - c
    pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
    if pa <= pb and pa <= pc:
        return a
    return b if pb <= pc else c


def read_png(path):
    data = open(path, "rb").read()
    assert data[:8] == b"\x89PNG\r\n\x1a\n", "not a PNG"
    pos, idat, hdr, seen_end = 8, b"", None, False
    while pos < len(data):
        n, = struct.unpack(">I", data[pos:pos + 4])
        typ = data[pos + 4:pos + 8]
        body = data[pos + 8:pos + 8 + n]
        crc, = struct.unpack(">I", data[pos + 8 + n:pos + 12 + n])
        assert zlib.crc32(typ + body) & 0xFFFFFFFF == crc, f"bad CRC in {typ!r}"
        if typ == b"IHDR":
            hdr = struct.unpack(">IIBBBBB", body)
        elif typ == b"IDAT":
            idat += body
        elif typ == b"IEND":
            seen_end = True
        pos += 12 + n
    assert hdr is not None and seen_end
    w, h, depth, ctype, comp, filt, interlace = hdr
    assert (depth, ctype, comp, filt, interlace) == (8, 6, 0, 0, 0), hdr
    raw = zlib.decompress(idat)
    stride = w * 4
    assert len(raw) == h * (stride + 1)
    out = np.zeros((h, stride), np.uint8)
    prev = np.zeros(stride, np.int64)
    for y in range(h):
        f = raw[y * (stride + 1)]
        line = np.frombuffer(raw, np.uint8, stride, y * (stride + 1) + 1).astype(np.int64)
        cur = np.zeros(stride, np.int64)
        if f == 0:
            cur = line
        elif f == 2:
            cur = (line + prev) & 255
        else:
            for i in range(stride):
                a = cur[i - 4] if i >= 4 else 0
                c = prev[i - 4] if i >= 4 else 0
                pred = {1: a, 3: (a + prev[i]) // 2, 4: _paeth(a, prev[i], c)}[f]
                cur[i] = (line[i] + pred) & 255
        out[y] = cur
        prev = cur
    return out.reshape(h, w, 4)
