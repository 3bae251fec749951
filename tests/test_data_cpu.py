"""Data pipeline: the FramesDataset item layout on a PNG frame tree, the
augmentation restatement (facevae_amd.augmentation; the reference's skimage / cv2 / torchvision
calls cannot run here -- parity unpinned, so the geometric maps are checked against
scipy.ndimage on the same coordinates and the transforms against their invariants)."""
import random

import numpy as np
import torch

import fvamd  # noqa: F401
from facevae_amd import augmentation as A
from facevae_amd.data import DatasetRepeater, FramesDataset


def test_rotate_matches_scipy_map_coordinates():
    from scipy import ndimage
    rng = np.random.default_rng(0)
    img = rng.random((17, 23, 3)).astype(np.float32)
    angle = 23.0
    out = A.rotate(img, angle)
    H, W = img.shape[:2]
    cy, cx = (H - 1) / 2, (W - 1) / 2
    t = np.deg2rad(angle)
    yy, xx = np.mgrid[0:H, 0:W].astype(np.float64)
    xs = np.cos(t) * (xx - cx) - np.sin(t) * (yy - cy) + cx
    ys = np.sin(t) * (xx - cx) + np.cos(t) * (yy - cy) + cy
    for c in range(3):
        ref = ndimage.map_coordinates(img[..., c].astype(np.float64), [ys, xs], order=1, mode="constant", cval=0.0)
        inside = (ys >= 0) & (ys <= H - 1) & (xs >= 0) & (xs <= W - 1)
        assert np.abs(out[..., c][inside] - ref[inside]).max() < 1e-5
    assert np.allclose(A.rotate(img, 0.0), img, atol=1e-6)


def test_perspective_transform_and_warp():
    src = np.array([[0, 0], [0, 10], [10, 0], [10, 10]], dtype=np.float64)
    dst = np.array([[1, 2], [0, 11], [12, 1], [9, 9]], dtype=np.float64)
    M = A.perspective_transform(src, dst)
    for (x, y), (u, v) in zip(src, dst):
        p = M @ np.array([x, y, 1.0])
        assert abs(p[0] / p[2] - u) < 1e-9 and abs(p[1] / p[2] - v) < 1e-9
    img = np.random.default_rng(1).random((256, 256, 3)).astype(np.float32)
    assert np.allclose(A.warp_perspective(img, np.eye(3), (256, 256)), img, atol=1e-6)
    np.random.seed(0)
    out = A.RandomPerspective(30, 40)([img.copy()])[0]
    assert out.shape == (256, 256, 3) and np.isfinite(out).all() and out.min() >= 0 and out.max() <= 1


def test_color_jitter_identity_and_range():
    img = np.random.default_rng(2).random((32, 32, 3)).astype(np.float32)
    u8 = (img * 255 + 0.5).astype(np.uint8)
    assert np.array_equal(A.adjust_brightness(u8, 1.0), u8)
    assert np.array_equal(A.adjust_contrast(u8, 1.0), u8)
    assert np.array_equal(A.adjust_saturation(u8, 1.0), u8)
    random.seed(0)
    out = A.ColorJitter(0.1, 0.1, 0.1, 0.1)([img])[0]
    assert out.dtype == np.float32 and out.shape == img.shape and 0 <= out.min() and out.max() <= 1
    assert np.abs(out - img).mean() < 0.15


def test_resize_crop_flip():
    img = np.random.default_rng(3).random((40, 30, 3)).astype(np.float32)
    assert A.resize(img, (80, 60)).shape == (80, 60, 3)
    assert np.allclose(A.resize(img, (40, 30)), img, atol=1e-6)
    random.seed(1)
    c = A.RandomCrop(32)([img, img])
    assert c[0].shape == (32, 32, 3) and np.array_equal(c[0], c[1])
    random.seed(3)
    f = A.RandomFlip(horizontal_flip=True)
    outs = [f([img])[0] for _ in range(8)]
    assert any(np.array_equal(o, img[:, ::-1]) for o in outs)


def test_frames_dataset_items(tmp_path):
    from PIL import Image
    rng = np.random.default_rng(4)
    for vid in ("id0#a.mp4", "id0#b.mp4", "id1#c.mp4"):
        for split in ("train", "test"):
            d = tmp_path / split / vid
            d.mkdir(parents=True)
            for f in range(3):
                Image.fromarray((rng.random((64, 64, 3)) * 255).astype(np.uint8)).save(d / f"{f:07d}.png")
    ds = FramesDataset(str(tmp_path), frame_shape=(64, 64, 3), id_sampling=True, is_train=True)
    assert sorted(ds.videos) == ["id0", "id1"]
    np.random.seed(0)
    random.seed(0)
    s, d, sa, da = ds[0]
    for t in (s, d, sa, da):
        assert t.dtype == np.float32 and 0 <= t.min() and t.max() <= 1
    assert s.shape == d.shape == (3, 64, 64)
    # RandomPerspective warps into a fixed 256 x 256 canvas (augmentation.py:333, crop_size = 256)
    assert sa.shape == da.shape == (3, 256, 256)
    ev = FramesDataset(str(tmp_path), frame_shape=(64, 64, 3), id_sampling=False, is_train=False)
    assert ev[0].shape == (3, 3, 64, 64)
    rep = DatasetRepeater(ds, 5)
    assert len(rep) == 10
    loader = torch.utils.data.DataLoader(rep, batch_size=4, num_workers=2)
    b = next(iter(loader))
    assert [tuple(t.shape) for t in b] == [(4, 3, 64, 64)] * 2 + [(4, 3, 256, 256)] * 2
