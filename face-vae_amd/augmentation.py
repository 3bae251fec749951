"""Clip augmentations of the training data (augmentation.py:22-418 of Luh1124/face-vae),
restated on numpy + PIL: the reference calls skimage (rotate, resize, img_as_ubyte), cv2
(getPerspectiveTransform, warpPerspective) and torchvision's functional colour adjustments,
none of which is in this image.  Same classes, constructor arguments and call convention
(a list of HxWxC float32 frames in [0, 1] -> list), the same random draws in the same order
(python `random` for rotation / flip / jitter parameters, numpy for the perspective), and the
same arithmetic:

  RandomRotation   skimage.transform.rotate(img, angle, preserve_range=True): rotation about
                   the centre ((cols - 1) / 2, (rows - 1) / 2), bilinear, constant 0 outside
  RandomPerspective cv2.getPerspectiveTransform on the reference's four point pairs, then
                   cv2.warpPerspective(..., (256, 256), BORDER_REPLICATE): bilinear inverse map
  RandomFlip       np.fliplr / time reversal
  RandomResize / RandomCrop  skimage resize (order 0 / 1, anti-aliased, zero fill) / random crop + pad
  ColorJitter      torchvision.transforms.functional.adjust_{brightness, saturation, hue,
                   contrast} on the uint8 PIL image (ImageEnhance blends; hue via PIL HSV),
                   in a random order, as augmentation.py:245-281

Parity: the reference's augmentation cannot run here (skimage / cv2 / torchvision absent), so
this restatement is "parity unpinned"; tests/test_data_cpu.py checks the geometric maps
against scipy.ndimage on the same inverse maps and the transforms' invariants.
"""
from __future__ import annotations

import numbers
import random

import numpy as np


def _bilinear(img: np.ndarray, ys: np.ndarray, xs: np.ndarray, mode: str) -> np.ndarray:
    """Sample img [H, W, C] at fractional (ys, xs) [h, w]; mode 'constant' (0 outside) or 'edge'."""
    H, W = img.shape[:2]
    if mode == "edge":
        ys = np.clip(ys, 0, H - 1)
        xs = np.clip(xs, 0, W - 1)
    y0 = np.floor(ys).astype(np.int64)
    x0 = np.floor(xs).astype(np.int64)
    ty = (ys - y0)[..., None].astype(np.float32)
    tx = (xs - x0)[..., None].astype(np.float32)
    out = np.zeros(ys.shape + img.shape[2:], dtype=np.float32)
    for dy, wy in ((0, 1 - ty), (1, ty)):
        for dx, wx in ((0, 1 - tx), (1, tx)):
            yy, xx = y0 + dy, x0 + dx
            ok = (yy >= 0) & (yy < H) & (xx >= 0) & (xx < W)
            v = img[np.clip(yy, 0, H - 1), np.clip(xx, 0, W - 1)]
            out += np.where(ok[..., None], v, 0.0) * (wy * wx)
    return out


def rotate(img: np.ndarray, angle: float) -> np.ndarray:
    """skimage.transform.rotate(img, angle, preserve_range=True) (order 1, constant 0)."""
    H, W = img.shape[:2]
    cy, cx = (H - 1) / 2.0, (W - 1) / 2.0
    t = np.deg2rad(angle)
    yy, xx = np.mgrid[0:H, 0:W].astype(np.float64)
    # skimage rotates counter-clockwise: the output pixel (x, y) samples the input at the
    # inverse rotation about the centre
    xs = np.cos(t) * (xx - cx) - np.sin(t) * (yy - cy) + cx
    ys = np.sin(t) * (xx - cx) + np.cos(t) * (yy - cy) + cy
    return _bilinear(img, ys, xs, "constant").astype(img.dtype)


def perspective_transform(src: np.ndarray, dst: np.ndarray) -> np.ndarray:
    """cv2.getPerspectiveTransform: the 3x3 M with dst ~ M src for four (x, y) point pairs."""
    A = np.zeros((8, 8))
    b = np.zeros(8)
    for i in range(4):
        x, y = src[i]
        u, v = dst[i]
        A[i] = [x, y, 1, 0, 0, 0, -x * u, -y * u]
        A[i + 4] = [0, 0, 0, x, y, 1, -x * v, -y * v]
        b[i], b[i + 4] = u, v
    m = np.linalg.solve(A, b)
    return np.append(m, 1.0).reshape(3, 3)


def warp_perspective(img: np.ndarray, M: np.ndarray, size) -> np.ndarray:
    """cv2.warpPerspective(img, M, size=(w, h), INTER_LINEAR, BORDER_REPLICATE)."""
    w, h = size
    Mi = np.linalg.inv(M)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float64)
    den = Mi[2, 0] * xx + Mi[2, 1] * yy + Mi[2, 2]
    xs = (Mi[0, 0] * xx + Mi[0, 1] * yy + Mi[0, 2]) / den
    ys = (Mi[1, 0] * xx + Mi[1, 1] * yy + Mi[1, 2]) / den
    return _bilinear(img, ys, xs, "edge").astype(img.dtype)


def resize(img: np.ndarray, size, order: int = 1) -> np.ndarray:
    """skimage.transform.resize(img, size, order, preserve_range=True, mode='constant',
    anti_aliasing=True) (augmentation.py:58-59), restated on scipy.ndimage as skimage computes it:
    a Gaussian pre-filter with sigma = max(0, (in / out - 1) / 2) per axis (zero padding; a no-op
    when upscaling), ndimage.zoom with grid_mode=True (pixel-centre mapping) in 'grid-constant'
    mode (samples past the border blend with 0), then the output clipped to the input's range
    extended by the 0 fill.  Float input keeps its dtype, integer input comes back float64
    (preserve_range)."""
    from scipy import ndimage as ndi
    x = img if img.dtype.char in "df" else img.astype(np.float64)
    out_shape = tuple(int(v) for v in size) + x.shape[2:]
    factors = np.divide(x.shape, out_shape)
    sigma = np.maximum(0, (factors - 1) / 2)
    filtered = ndi.gaussian_filter(x, sigma, cval=0, mode="constant")
    out = ndi.zoom(filtered, [1 / f for f in factors], order=order, mode="grid-constant", cval=0, grid_mode=True)
    lo, hi = min(float(x.min()), 0.0), float(x.max())
    return np.clip(out, lo, hi)


class RandomFlip:
    """augmentation.py:202-213."""

    def __init__(self, time_flip=False, horizontal_flip=False):
        self.time_flip, self.horizontal_flip = time_flip, horizontal_flip

    def __call__(self, clip):
        if random.random() < 0.5 and self.time_flip:
            return clip[::-1]
        if random.random() < 0.5 and self.horizontal_flip:
            return [np.fliplr(img) for img in clip]
        return clip


class RandomRotation:
    """augmentation.py:161-199: one angle ~ U(degrees) for the whole clip."""

    def __init__(self, degrees):
        if isinstance(degrees, numbers.Number):
            if degrees < 0:
                raise ValueError("If degrees is a single number, must be positive")
            degrees = (-degrees, degrees)
        elif len(degrees) != 2:
            raise ValueError("If degrees is a sequence, it must be of len 2.")
        self.degrees = degrees

    def __call__(self, clip):
        angle = random.uniform(self.degrees[0], self.degrees[1])
        return [rotate(img, angle) for img in clip]


class RandomPerspective:
    """augmentation.py:315-353 (the reference's point pairs, 256x256 output, replicate border)."""

    def __init__(self, pers_num, enlarge_num):
        self.pers_num, self.enlarge_num = pers_num, enlarge_num

    def __call__(self, clip):
        out = clip
        for i in range(len(clip)):
            pers = np.random.randint(20, self.pers_num) * pow(-1, np.random.randint(2))
            enl = np.random.randint(20, self.enlarge_num) * pow(-1, np.random.randint(2))
            h, w, _ = clip[i].shape
            dst = np.array([[-enl, -enl], [-enl + pers, w + enl], [h + enl, -enl], [h + enl - pers, w + enl]],
                           dtype=np.float32)
            src = np.array([[-enl, -enl], [-enl, w + enl], [h + enl, -enl], [h + enl, w + enl]], dtype=np.float32)
            out[i] = warp_perspective(clip[i], perspective_transform(src, dst), (256, 256))
        return out


class RandomResize:
    """augmentation.py:93-120: scale ~ U(ratio), skimage resize of every frame."""

    def __init__(self, ratio=(3. / 4., 4. / 3.), interpolation="nearest"):
        self.ratio, self.interpolation = ratio, interpolation

    def __call__(self, clip):
        s = random.uniform(self.ratio[0], self.ratio[1])
        h, w = clip[0].shape[:2]
        order = 1 if self.interpolation == "bilinear" else 0        # augmentation.py:58
        return [resize(img, (int(h * s), int(w * s)), order) for img in clip]


class RandomCrop:
    """augmentation.py:123-158: pad to at least `size`, then one random crop for the clip."""

    def __init__(self, size):
        self.size = (size, size) if isinstance(size, numbers.Number) else size

    def __call__(self, clip):
        h, w = self.size
        im_h, im_w = clip[0].shape[:2]
        clip = [np.pad(img, ((0, max(0, h - im_h)), (0, max(0, w - im_w)), (0, 0)), mode="edge") for img in clip]
        im_h, im_w = clip[0].shape[:2]
        x1 = 0 if w == im_w else random.randint(0, im_w - w)
        y1 = 0 if h == im_h else random.randint(0, im_h - h)
        return [img[y1:y1 + h, x1:x1 + w] for img in clip]


def _blend(a: np.ndarray, b: np.ndarray, f: float) -> np.ndarray:
    """PIL ImageEnhance / Image.blend on uint8: clip(b + f (a - b)) rounded to uint8."""
    return np.clip(b.astype(np.float32) + f * (a.astype(np.float32) - b.astype(np.float32)), 0, 255).round()


def adjust_brightness(img: np.ndarray, f: float) -> np.ndarray:
    return _blend(img, np.zeros_like(img), f).astype(np.uint8)


def adjust_saturation(img: np.ndarray, f: float) -> np.ndarray:
    from PIL import Image
    gray = np.asarray(Image.fromarray(img).convert("L").convert("RGB"))
    return _blend(img, gray, f).astype(np.uint8)


def adjust_contrast(img: np.ndarray, f: float) -> np.ndarray:
    from PIL import Image
    mean = int(np.asarray(Image.fromarray(img).convert("L")).mean() + 0.5)
    return _blend(img, np.full_like(img, mean), f).astype(np.uint8)


def adjust_hue(img: np.ndarray, f: float) -> np.ndarray:
    from PIL import Image
    hsv = np.asarray(Image.fromarray(img).convert("HSV")).copy()
    hsv[..., 0] = ((hsv[..., 0].astype(np.int16) + np.int16(round(f * 255))) % 256).astype(np.uint8)
    return np.asarray(Image.fromarray(hsv, "HSV").convert("RGB"))


class ColorJitter:
    """augmentation.py:216-313 (numpy-frame branch): factors drawn with python `random`, the
    adjustments applied in a random order on the uint8 image, back to float in [0, 1]."""

    def __init__(self, brightness=0, contrast=0, saturation=0, hue=0):
        self.brightness, self.contrast, self.saturation, self.hue = brightness, contrast, saturation, hue

    @staticmethod
    def get_params(brightness, contrast, saturation, hue):
        b = random.uniform(max(0, 1 - brightness), 1 + brightness) if brightness > 0 else None
        c = random.uniform(max(0, 1 - contrast), 1 + contrast) if contrast > 0 else None
        s = random.uniform(max(0, 1 - saturation), 1 + saturation) if saturation > 0 else None
        h = random.uniform(-hue, hue) if hue > 0 else None
        return b, c, s, h

    def __call__(self, clip):
        b, c, s, h = self.get_params(self.brightness, self.contrast, self.saturation, self.hue)
        fns = []
        if b is not None:
            fns.append(lambda im: adjust_brightness(im, b))
        if s is not None:
            fns.append(lambda im: adjust_saturation(im, s))
        if h is not None:
            fns.append(lambda im: adjust_hue(im, h))
        if c is not None:
            fns.append(lambda im: adjust_contrast(im, c))
        random.shuffle(fns)
        out = []
        for img in clip:
            im = (np.clip(img, 0, 1) * 255 + 0.5).astype(np.uint8)       # img_as_ubyte
            for f in fns:
                im = f(im)
            out.append((im.astype(np.float32) / 255.0).astype("float32"))  # img_as_float
        return out


class AllAugmentationTransform:
    """augmentation.py:384-418: flip, rotation, perspective, resize, crop, colour jitter."""

    def __init__(self, resize_param=None, rotation_param=None, perspective_param=None, flip_param=None,
                 crop_param=None, jitter_param=None, blur_param=None, gray_param=None):
        self.transforms = []
        if flip_param is not None:
            self.transforms.append(RandomFlip(**flip_param))
        if rotation_param is not None:
            self.transforms.append(RandomRotation(**rotation_param))
        if perspective_param is not None:
            self.transforms.append(RandomPerspective(**perspective_param))
        if resize_param is not None:
            self.transforms.append(RandomResize(**resize_param))
        if crop_param is not None:
            self.transforms.append(RandomCrop(**crop_param))
        if jitter_param is not None:
            self.transforms.append(ColorJitter(**jitter_param))

    def __call__(self, clip):
        for t in self.transforms:
            clip = t(clip)
        return clip
