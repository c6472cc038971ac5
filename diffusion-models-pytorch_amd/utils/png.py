"""Minimal PNG writer (torchvision is absent here).

Restates torchvision 0.16 utils.make_grid / save_image (torchvision is absent, so
byte parity with it is unpinned): a [B, C, H, W] tensor or a list of [C, H, W]
images is tiled nrow per row with `padding` pixels of `pad_value` around every
tile (a single image is returned as is, no padding); 1-channel images are
replicated to RGB; float [0, 1] -> uint8 via x * 255 + 0.5 clamped and truncated.
"""
import struct
import zlib

import numpy as np
import torch


def _chunk(tag: bytes, data: bytes) -> bytes:
    return struct.pack('>I', len(data)) + tag + data + struct.pack('>I', zlib.crc32(tag + data) & 0xFFFFFFFF)


def make_grid(tensor, nrow: int = 8, padding: int = 2, pad_value: float = 0.0) -> torch.Tensor:
    """torchvision/utils.py make_grid (0.16), normalize=False."""
    if isinstance(tensor, (list, tuple)):
        tensor = torch.stack(list(tensor), dim=0)
    if tensor.dim() == 2:
        tensor = tensor.unsqueeze(0)
    if tensor.dim() == 3:
        if tensor.shape[0] == 1:
            tensor = torch.cat((tensor, tensor, tensor), 0)
        tensor = tensor.unsqueeze(0)
    if tensor.dim() == 4 and tensor.shape[1] == 1:
        tensor = torch.cat((tensor, tensor, tensor), 1)
    if tensor.shape[0] == 1:
        return tensor.squeeze(0)
    n = tensor.shape[0]
    xmaps = min(nrow, n)
    ymaps = (n + xmaps - 1) // xmaps
    height, width = tensor.shape[2] + padding, tensor.shape[3] + padding
    grid = tensor.new_full((tensor.shape[1], height * ymaps + padding, width * xmaps + padding), pad_value)
    k = 0
    for y in range(ymaps):
        for x in range(xmaps):
            if k >= n:
                break
            grid[:, y * height + padding:(y + 1) * height, x * width + padding:(x + 1) * width] = tensor[k]
            k += 1
    return grid


def to_uint8(image: torch.Tensor) -> np.ndarray:
    """[C, H, W] float in [0, 1] -> [H, W, 3] uint8."""
    x = image.detach().to('cpu', torch.float32)
    if x.shape[0] == 1:
        x = torch.cat((x, x, x), 0)
    return x.mul(255).add_(0.5).clamp_(0, 255).permute(1, 2, 0).to(torch.uint8).numpy()


def save_image(image, path: str, nrow: int = 8, padding: int = 2, pad_value: float = 0.0):
    """torchvision/utils.py save_image (0.16): make_grid, then one 8-bit RGB PNG."""
    if isinstance(image, (list, tuple)) or image.dim() == 4:
        image = make_grid(image, nrow=nrow, padding=padding, pad_value=pad_value)
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
