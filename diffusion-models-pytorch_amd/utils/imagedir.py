"""Image-directory input for the DDIM reconstruction mode (reference scripts/sample_uncond.py:279-312).

`ImageDir` follows the reference's datasets/ImageDir.py:6-35 (every .jpg/.jpeg/.png/.bmp/.tiff under
root, sorted paths, PIL `convert('RGB')`). torchvision is absent from this image, so the transform chain
the reference builds at sample_uncond.py:281-286 —
    Resize(img_size) -> CenterCrop(img_size) -> ToTensor() -> Normalize([0.5]*3, [0.5]*3)
— is restated on PIL directly with torchvision 0.16's documented arithmetic: the shorter side goes to
`size` and the longer to int(size * long / short) with PIL bilinear (no-op when already that size), the
crop offsets are int(round((H - size) / 2)), ToTensor divides uint8 by 255, Normalize is (x - 0.5) / 0.5.
Parity of the resize against torchvision itself is unpinned (no torchvision here); for inputs already at
img_size the chain is exact.
"""
import os
from typing import List

import numpy as np
import torch

IMG_EXT = ('.jpg', '.jpeg', '.png', '.bmp', '.tiff')


def extract_images(root: str) -> List[str]:
    """datasets/ImageDir.py:6-16."""
    root = os.path.expanduser(root)
    paths = []
    for curdir, _, files in os.walk(root):
        for file in files:
            if os.path.splitext(file)[1].lower() in IMG_EXT:
                paths.append(os.path.join(curdir, file))
    return sorted(paths)


def resize_center_crop_normalize(img, size: int) -> torch.Tensor:
    """PIL RGB image -> [3, size, size] float32 in [-1, 1] (sample_uncond.py:281-286)."""
    from PIL import Image
    w, h = img.size
    short, long = (w, h) if w <= h else (h, w)
    new_short, new_long = size, int(size * long / short)
    new_w, new_h = (new_short, new_long) if w <= h else (new_long, new_short)
    if (new_w, new_h) != (w, h):
        img = img.resize((new_w, new_h), Image.BILINEAR)
    top = int(round((new_h - size) / 2.0))
    left = int(round((new_w - size) / 2.0))
    img = img.crop((left, top, left + size, top + size))
    x = torch.from_numpy(np.asarray(img, dtype=np.uint8).copy()).permute(2, 0, 1).float().div(255)
    return (x - 0.5) / 0.5


class ImageDir(torch.utils.data.Dataset):
    """datasets/ImageDir.py:19-35 with the reconstruction transform built in."""

    def __init__(self, root: str, img_size: int):
        root = os.path.expanduser(root)
        if not os.path.isdir(root):
            raise ValueError(f'{root} is not a valid directory')
        self.img_size = img_size
        self.img_paths = extract_images(root)

    def __len__(self):
        return len(self.img_paths)

    def __getitem__(self, item):
        from PIL import Image
        with Image.open(self.img_paths[item]) as im:
            return resize_center_crop_normalize(im.convert('RGB'), self.img_size)
