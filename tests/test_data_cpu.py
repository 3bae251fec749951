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
    # 96-px frames: RandomPerspective moves the corners by |enlarge| <= 39 px, which on a 64-px
    # frame can make two source corners coincide (enlarge = -32) -- a singular system
    rng = np.random.default_rng(4)
    for vid in ("id0#a.mp4", "id0#b.mp4", "id1#c.mp4"):
        for split in ("train", "test"):
            d = tmp_path / split / vid
            d.mkdir(parents=True)
            for f in range(3):
                Image.fromarray((rng.random((96, 96, 3)) * 255).astype(np.uint8)).save(d / f"{f:07d}.png")
    ds = FramesDataset(str(tmp_path), frame_shape=(96, 96, 3), id_sampling=True, is_train=True)
    assert sorted(ds.videos) == ["id0", "id1"]
    np.random.seed(0)
    random.seed(0)
    s, d, sa, da = ds[0]
    for t in (s, d, sa, da):
        assert t.dtype == np.float32 and 0 <= t.min() and t.max() <= 1
    assert s.shape == d.shape == (3, 96, 96)
    # RandomPerspective warps into a fixed 256 x 256 canvas (augmentation.py:333, crop_size = 256)
    assert sa.shape == da.shape == (3, 256, 256)
    ev = FramesDataset(str(tmp_path), frame_shape=(96, 96, 3), id_sampling=False, is_train=False)
    assert ev[0].shape == (3, 3, 96, 96)
    rep = DatasetRepeater(ds, 5)
    assert len(rep) == 10
    loader = torch.utils.data.DataLoader(rep, batch_size=4, num_workers=2)
    b = next(iter(loader))
    assert [tuple(t.shape) for t in b] == [(4, 3, 96, 96)] * 2 + [(4, 3, 256, 256)] * 2


def _tree(tmp_path, H=32, frames=5):
    from PIL import Image
    rng = np.random.default_rng(5)
    for vid in ("id0#a.mp4", "id1#b.mp4"):
        for split in ("train", "test"):
            d = tmp_path / split / vid
            d.mkdir(parents=True)
            for f in range(frames):
                Image.fromarray((rng.random((H, H, 3)) * 255).astype(np.uint8)).save(d / f"{f:07d}.png")
    return tmp_path


def test_training_frames_follow_os_listdir_order(tmp_path, monkeypatch):
    """dataset.py:102-105: the two sorted random indices select from os.listdir(path) as it
    comes (test items read_video: sorted by name)."""
    import os
    from facevae_amd import data as D
    _tree(tmp_path)
    real = os.listdir
    seen = []

    def rev(p):
        out = real(p)
        if str(p).endswith(".mp4"):
            out = sorted(out, reverse=True)        # a directory order that is not name order
            seen.append(out)
        return out
    monkeypatch.setattr(D.os, "listdir", rev)
    ds = D.FramesDataset(str(tmp_path), frame_shape=(32, 32, 3), id_sampling=False, is_train=True,
                         augmentation_params=None, output="uint8")
    np.random.seed(3)
    s, d = ds[0]
    np.random.seed(3)
    fidx = np.sort(np.random.choice(5, replace=True, size=2))
    frames = seen[-1]
    path = os.path.join(str(tmp_path), "train", ds.videos[0])
    assert np.array_equal(s, D._read_frame_u8(os.path.join(path, frames[fidx[0]])).transpose(2, 0, 1))
    assert np.array_equal(d, D._read_frame_u8(os.path.join(path, frames[fidx[1]])).transpose(2, 0, 1))


def test_uint8_feed_matches_float32_items(tmp_path):
    """output="uint8" + to_device_frames (here on the CPU) gives the float32 frames of the
    reference layout bit for bit (x * fp32(1/255) = img_as_float32)."""
    from facevae_amd import data as D
    _tree(tmp_path)
    f32 = D.FramesDataset(str(tmp_path), frame_shape=(32, 32, 3), id_sampling=True, is_train=True,
                          augmentation_params=None)
    u8 = D.FramesDataset(str(tmp_path), frame_shape=(32, 32, 3), id_sampling=True, is_train=True,
                         augmentation_params=None, output="uint8")
    for i in range(2):
        np.random.seed(10 + i)
        s, d, _, _ = f32[i]
        np.random.seed(10 + i)
        s8, d8 = u8[i]
        assert s8.dtype == np.uint8 and s8.shape == (3, 32, 32)
        assert torch.equal(D.to_device_frames(torch.from_numpy(s8), "cpu"), torch.from_numpy(s))
        assert torch.equal(D.to_device_frames(torch.from_numpy(d8), "cpu"), torch.from_numpy(d))
    loader = torch.utils.data.DataLoader(DatasetRepeater(u8, 2), batch_size=4, num_workers=2)
    b = next(iter(loader))
    assert len(b) == 2 and b[1].dtype == torch.uint8 and tuple(b[1].shape) == (4, 3, 32, 32)
    ev = D.FramesDataset(str(tmp_path), frame_shape=(32, 32, 3), id_sampling=False, is_train=False, output="uint8")
    assert ev[0].shape == (3, 5, 32, 32) and ev[0].dtype == np.uint8


def test_gif_video(tmp_path):
    """read_video of a .gif (dataset.py:24-30, PIL frames instead of imageio.mimread)."""
    from PIL import Image
    from facevae_amd import data as D
    rng = np.random.default_rng(6)
    frames = [Image.fromarray((rng.random((16, 16, 3)) * 255).astype(np.uint8)).convert("P", palette=Image.ADAPTIVE)
              for _ in range(4)]
    p = tmp_path / "v.gif"
    frames[0].save(p, save_all=True, append_images=frames[1:])
    v = D.read_video_u8(str(p))
    assert v.shape == (4, 16, 16, 3) and v.dtype == np.uint8
    for i, f in enumerate(frames):
        assert np.array_equal(v[i], np.asarray(f.convert("RGB")))
    import pytest
    with pytest.raises(NotImplementedError):
        D.read_video_u8(str(tmp_path / "x.mp4"))



def test_driving_feed_is_the_reference_driving_frame(tmp_path):
    """output="driving_uint8": the same two random draws as the reference item, only the
    driving frame decoded -- equal to the float32 item's `driving` after the uint8 -> float conversion."""
    from facevae_amd import data as D
    _tree(tmp_path)
    f32 = D.FramesDataset(str(tmp_path), frame_shape=(32, 32, 3), is_train=True, augmentation_params=None)
    dv = D.FramesDataset(str(tmp_path), frame_shape=(32, 32, 3), is_train=True, output="driving_uint8")
    for i in range(2):
        np.random.seed(20 + i)
        _, d, _, _ = f32[i]
        np.random.seed(20 + i)
        d8 = dv[i]
        assert d8.dtype == np.uint8 and d8.shape == (3, 32, 32)
        assert torch.equal(D.to_device_frames(torch.from_numpy(d8), "cpu"), torch.from_numpy(d))


def test_uint8_conversion_is_img_as_float32():
    """skimage.util.img_as_float32 on uint8 is np.multiply(x, 1. / 255, dtype=float32)
    (skimage/util/dtype.py `_convert`, unsigned -> float; skimage is not importable here, so this
    restates its arithmetic -- parity unpinned by a reference fixture).  x / 255 differs from it in
    the last bit for 126 of the 256 byte values; the CPU items and the GPU feed both use the
    fp32 reciprocal."""
    import numpy as np
    import torch
    import fvamd  # noqa: F401
    from facevae_amd import data as D
    x = np.arange(256, dtype=np.uint8)
    ref = np.multiply(x, 1. / 255, dtype=np.float32)
    assert np.array_equal(D.u8_to_float(x), ref)
    assert int((x.astype(np.float32) / 255.0 != ref).sum()) == 126
    assert torch.equal(D.to_device_frames(torch.from_numpy(x), "cpu"), torch.from_numpy(ref))


def test_resize_is_skimage_antialiased_constant_mode():
    """augmentation.py:58-59 calls skimage resize with anti_aliasing=True, mode='constant' (skimage
    is not importable here: parity unpinned, properties only).  A 1-pixel checkerboard shrunk 4x
    comes out near its mean (the Gaussian pre-filter; plain bilinear sampling would alias to the
    extremes); the zero fill darkens the border rows of a constant image when upscaling."""
    cb = (np.indices((64, 64)).sum(0) % 2).astype(np.float32)[..., None]
    small = A.resize(cb, (16, 16))
    assert abs(small[4:-4, 4:-4].mean() - 0.5) < 0.02 and small[4:-4, 4:-4].std() < 0.05
    one = np.ones((8, 8, 1), np.float32)
    big = A.resize(one, (16, 16))
    assert np.allclose(big[4:-4, 4:-4], 1.0) and big[0, 8, 0] < 0.9      # grid-constant: 0 outside
    assert big.min() >= 0.0 and big.max() <= 1.0                         # clipped to [min(0, lo), hi]
    q = A.resize((np.arange(16).reshape(4, 4, 1) * 10).astype(np.uint8), (8, 8), order=0)
    assert q.dtype == np.float64                                         # preserve_range on integers
