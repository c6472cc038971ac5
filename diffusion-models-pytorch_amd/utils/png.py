"""Minimal PNG writer (torchvision is absent here).

Matches torchvision.utils.save_image for a single image: float [0, 1] ->
uint8 via x * 255 + 0.5 clamped and truncated; 1-channel images are
replicated to RGB (make_grid does this for one image, no padding).
"""
import struct
import zlib

import numpy as np
import torch


def _chunk(tag: bytes, data: bytes) -> bytes:
    return struct.pack('>I', len(data)) + tag + data + struct.pack('>I', zlib.crc32(tag + data) & 0xFFFFFFFF)


def to_uint8(image: torch.Tensor) -> np.ndarray:
    """[C, H, W] float in [0, 1] -> [H, W, 3] uint8."""
    x = image.detach().to('cpu', torch.float32)
    if x.shape[0] == 1:
        x = torch.cat((x, x, x), 0)
    return x.mul(255).add_(0.5).clamp_(0, 255).permute(1, 2, 0).to(torch.uint8).numpy()


def save_image(image: torch.Tensor, path: str):
    rgb = to_uint8(image)
    h, w, _ = rgb.shape
    raw = b''.join(b'\x00' + rgb[y].tobytes() for y in range(h))
    png = b'\x89PNG\r\n\x1a\n' + _chunk(b'IHDR', struct.pack('>IIBBBBB', w, h, 8, 2, 0, 0, 0)) + \
        _chunk(b'IDAT', zlib.compress(raw, 6)) + _chunk(b'IEND', b'')
    with open(path, 'wb') as f:
        f.write(png)


def read_png_rgb(path: str) -> np.ndarray:
    """Decode PNGs written by save_image (8-bit RGB, filter 0) — for tests."""
    with open(path, 'rb') as f:
        data = f.read()
    assert data[:8] == b'\x89PNG\r\n\x1a\n'
    pos, idat, w, h = 8, b'', 0, 0
    while pos < len(data):
        n = struct.unpack('>I', data[pos:pos + 4])[0]
        tag = data[pos + 4:pos + 8]
        body = data[pos + 8:pos + 8 + n]
        if tag == b'IHDR':
            w, h = struct.unpack('>II', body[:8])
        elif tag == b'IDAT':
            idat += body
        pos += 12 + n
    raw = zlib.decompress(idat)
    rows = [raw[y * (3 * w + 1) + 1:(y + 1) * (3 * w + 1)] for y in range(h)]
    return np.frombuffer(b''.join(rows), dtype=np.uint8).reshape(h, w, 3)
