"""Host-side image I/O of the sampling scripts: utils.png.make_grid / save_image (torchvision 0.16
utils.py restated; torchvision is absent, so byte parity with it is unpinned) and utils.imagedir
(reference datasets/ImageDir.py + the sample_uncond.py:281-286 transform chain)."""
import numpy as np
import torch

from utils.imagedir import ImageDir, extract_images, resize_center_crop_normalize
from utils.png import make_grid, read_png_rgb, save_image


def test_make_grid_layout():
    x = torch.rand(3, 1, 4, 5)
    g = make_grid(x, nrow=2, padding=2, pad_value=0.5)
    # 2 columns x 2 rows of (4+2)x(5+2) cells plus the leading padding; 1 channel -> RGB
    assert g.shape == (3, 2 * 6 + 2, 2 * 7 + 2)
    for k in range(3):
        r, c = divmod(k, 2)
        tile = g[:, r * 6 + 2:r * 6 + 6, c * 7 + 2:c * 7 + 7]
        assert torch.equal(tile, x[k].expand(3, -1, -1))
    assert torch.all(g[:, 8:12, 9:14] == 0.5)      # the empty 4th cell keeps pad_value
    assert torch.equal(make_grid(x[:1]), x[0].expand(3, -1, -1))   # one image: no padding


def test_save_image_grid_png(tmp_path):
    a, b = torch.rand(3, 6, 6), torch.rand(3, 6, 6)
    p = str(tmp_path / 'g.png')
    save_image([a, b], p, nrow=2)
    rgb = read_png_rgb(p)
    assert rgb.shape == (10, 18, 3)
    exp = make_grid([a, b], nrow=2).mul(255).add(0.5).clamp(0, 255).permute(1, 2, 0).to(torch.uint8).numpy()
    assert np.array_equal(rgb, exp)


def test_imagedir_transform(tmp_path):
    from PIL import Image
    rng = np.random.default_rng(0)
    exact = rng.integers(0, 256, (8, 8, 3), dtype=np.uint8)
    Image.fromarray(exact).save(tmp_path / 'b.png')
    wide = rng.integers(0, 256, (10, 16, 3), dtype=np.uint8)
    (tmp_path / 'sub').mkdir()
    Image.fromarray(wide).save(tmp_path / 'sub' / 'a.PNG')
    (tmp_path / 'notes.txt').write_text('x')
    assert [p.split('/')[-1] for p in extract_images(str(tmp_path))] == ['b.png', 'a.PNG']
    ds = ImageDir(str(tmp_path), 8)
    assert len(ds) == 2
    x = ds[0]   # already img_size: ToTensor + Normalize only, exact
    assert torch.equal(x, (torch.from_numpy(exact).permute(2, 0, 1).float() / 255 - 0.5) / 0.5)
    y = ds[1]   # 16x10 -> short side 8 (12x8, PIL bilinear) -> center crop columns 2..9
    ref = np.asarray(Image.fromarray(wide).resize((12, 8), Image.BILINEAR))[:, 2:10]
    assert torch.equal(y, (torch.from_numpy(ref.copy()).permute(2, 0, 1).float() / 255 - 0.5) / 0.5)
    assert resize_center_crop_normalize(Image.fromarray(exact), 8).shape == (3, 8, 8)
