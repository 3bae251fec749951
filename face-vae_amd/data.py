"""Frame datasets for the FaceVAE trainer (dataset.py:13-193 of Luh1124/face-vae).

`FramesDataset` keeps the reference constructor, directory conventions and item layout:
`root_dir` holds one folder of PNG frames (or a .gif) per video (`<id>#<video>.mp4`),
optionally split into `train/` and `test/`; with `id_sampling` the training set is the set of
identities and an item picks a random video of the identity, then two random frames (sorted
indices into the folder's `os.listdir` order, dataset.py:102-105), returned as `(source,
driving, source_aug, driving_aug)` float32 CHW arrays in [0, 1] (dataset.py:91-129); a
test-split item is the whole video, frames sorted by name (read_video, dataset.py:20-23).
Frames are decoded with PIL (skimage / imageio are not in this image; for uint8 PNGs
`img_as_float32` is `np.multiply(x, 1. / 255, dtype=np.float32)`, i.e. x times the fp32
reciprocal of 255 -- NOT x / 255, which differs in the last bit for 126 of the 256 values).  The `*_aug` items go through
`augmentation.AllAugmentationTransform` with the reference's default parameters (rotation
30 degrees, perspective (30, 40), colour jitter 0.1, dataset.py:52-57), each frame on its own
as dataset.py:122-123; they feed the keypoint / contrastive losses, not the FaceVAE path.

`output="uint8"` keeps the item layout as bytes: training items are `(source, driving)` uint8
CHW arrays (no float conversion, no augmentation in the workers: 4x fewer bytes through the
DataLoader's worker IPC and collate).  `output="driving_uint8"` is the FaceVAE feed: the item
is the `driving` frame alone (the same two random draws, so the same frame as the reference
item's `driving`; `source` is not decoded -- the FaceVAE step never reads it).
`to_device_frames` turns a collated uint8 batch into the float32 NCHW [0, 1] tensor on the
GPU -- x times fp32(1/255), bit-identical to img_as_float32 on the CPU (`u8_to_float`).

`SyntheticFramesDataset` produces VoxCeleb-shaped frames x ~ U[0, 1) deterministically per
index (the benchmark / test input when no dataset is on disk).  The reference's
`PairedDataset` (dataset.py:154-193: source / driving pairs for the animation evaluation) is
not on the FaceVAE training path and is not provided.
"""
from __future__ import annotations

import glob
import os
from typing import Optional, Sequence

import numpy as np
from torch.utils.data import Dataset


def _read_frame_u8(path: str) -> np.ndarray:
    """HxWx3 uint8 (gray and RGBA frames converted as skimage's gray2rgb / [..., :3] would)."""
    from PIL import Image
    with Image.open(path) as im:
        if im.mode != "RGB":
            im = im.convert("RGB")
        return np.asarray(im)


# skimage.util.img_as_float32 on uint8 (skimage/util/dtype.py `_convert`: unsigned -> float
# multiplies by 1. / imax_in with dtype=float32, so the reciprocal is rounded to fp32 first)
INV255 = np.float32(1.0 / 255.0)


def u8_to_float(a: np.ndarray) -> np.ndarray:
    """img_as_float32 of a uint8 array."""
    return np.multiply(a, INV255, dtype=np.float32)


def _read_frame(path: str) -> np.ndarray:
    return u8_to_float(_read_frame_u8(path))


def _read_gif_u8(path: str) -> np.ndarray:
    """All frames of a .gif as [T, H, W, 3] uint8 (imageio.mimread + the RGBA -> RGB cut of
    dataset.py:25-29; here through PIL's frame iterator).  .mp4 needs a video decoder, which
    this image does not have."""
    from PIL import Image, ImageSequence
    with Image.open(path) as im:
        return np.stack([np.asarray(f.convert("RGB")) for f in ImageSequence.Iterator(im)])


def read_video_u8(name: str) -> np.ndarray:
    """dataset.py:13-34 read_video, as uint8 [T, H, W, 3]: a folder of frames sorted by name, or
    a .gif."""
    if os.path.isdir(name):
        return np.stack([_read_frame_u8(os.path.join(name, f)) for f in sorted(os.listdir(name))])
    if name.lower().endswith(".gif"):
        return _read_gif_u8(name)
    if name.lower().endswith(".mp4"):
        raise NotImplementedError(f"{name}: .mp4 decoding needs a video decoder (imageio / ffmpeg), "
                                  "not in this image; extract the frames to a folder")
    raise ValueError("Unknown file extensions  %s" % name)


def to_device_frames(t, device="cuda") -> "torch.Tensor":
    """A collated batch of frames -> float32 NCHW on `device`: uint8 (output="uint8") is moved
    as bytes and converted there (x * fp32(1/255), as u8_to_float); float32 is moved as is."""
    import torch
    t = torch.as_tensor(t)
    if t.dtype == torch.uint8:
        return t.to(device, non_blocking=True).float().mul_(float(INV255))
    return t.to(device, non_blocking=True)


def _train_test_split(videos: Sequence[str], random_seed: int, test_size: float = 0.2):
    """sklearn.model_selection.train_test_split(videos, random_state, test_size=0.2) ordering."""
    from sklearn.model_selection import train_test_split
    return train_test_split(list(videos), random_state=random_seed, test_size=test_size)


DEFAULT_AUGMENTATION = {
    "rotation_param": {"degrees": 30},
    "perspective_param": {"pers_num": 30, "enlarge_num": 40},
    "jitter_param": {"brightness": 0.1, "contrast": 0.1, "saturation": 0.1, "hue": 0.1},
}


class FramesDataset(Dataset):
    def __init__(self, root_dir: str, frame_shape=(256, 256, 3), id_sampling: bool = True, is_train: bool = True,
                 random_seed: int = 0, pairs_list: Optional[str] = None, augmentation_params=DEFAULT_AUGMENTATION,
                 output: str = "float32"):
        if output not in ("float32", "uint8", "driving_uint8"):
            raise ValueError("FramesDataset: output must be 'float32' (reference items), 'uint8' or "
                             "'driving_uint8' (FaceVAE feed)")
        self.output = output
        self.root_dir = root_dir
        self.videos = os.listdir(root_dir)
        self.frame_shape = tuple(frame_shape)
        self.pairs_list = pairs_list
        self.id_sampling = id_sampling
        if os.path.exists(os.path.join(root_dir, "train")):
            if not os.path.exists(os.path.join(root_dir, "test")):
                raise FileNotFoundError(os.path.join(root_dir, "test"))
            if id_sampling:
                train_videos = list({os.path.basename(v).split("#")[0]
                                     for v in os.listdir(os.path.join(root_dir, "train"))})
            else:
                train_videos = os.listdir(os.path.join(root_dir, "train"))
            test_videos = os.listdir(os.path.join(root_dir, "test"))
            self.root_dir = os.path.join(self.root_dir, "train" if is_train else "test")
        else:
            train_videos, test_videos = _train_test_split(self.videos, random_seed)
        self.videos = train_videos if is_train else test_videos
        self.is_train = is_train
        from .augmentation import AllAugmentationTransform
        self.transform = AllAugmentationTransform(**(augmentation_params or {})) \
            if is_train and output == "float32" else None

    def __len__(self):
        return len(self.videos)

    def __getitem__(self, idx):
        name = self.videos[idx]
        if self.is_train and self.id_sampling:
            path = str(np.random.choice(glob.glob(os.path.join(self.root_dir, name + "*.mp4"))))
        else:
            path = os.path.join(self.root_dir, name)
        if self.is_train and os.path.isdir(path):
            # dataset.py:102-105: two sorted random indices into the folder's os.listdir order
            frames = os.listdir(path)
            fidx = np.sort(np.random.choice(len(frames), replace=True, size=2))
            if self.output == "driving_uint8":
                return np.ascontiguousarray(_read_frame_u8(os.path.join(path, frames[fidx[1]])).transpose(2, 0, 1))
            arr = [_read_frame_u8(os.path.join(path, frames[i])) for i in fidx]
        else:
            video = read_video_u8(path)                # dataset.py:107-110
            fidx = np.sort(np.random.choice(len(video), replace=True, size=2)) if self.is_train else range(len(video))
            arr = video[fidx]
        if self.output == "driving_uint8" and self.is_train:
            return np.ascontiguousarray(arr[1].transpose(2, 0, 1))
        if self.output != "float32":
            if self.is_train:
                return (np.ascontiguousarray(arr[0].transpose(2, 0, 1)),
                        np.ascontiguousarray(arr[1].transpose(2, 0, 1)))
            return np.ascontiguousarray(np.asarray(arr).transpose(3, 0, 1, 2))
        arr = [u8_to_float(a) for a in arr]
        if self.is_train:
            source = np.ascontiguousarray(arr[0].transpose(2, 0, 1))
            driving = np.ascontiguousarray(arr[1].transpose(2, 0, 1))
            if self.transform is None:
                return source, driving, None, None
            s_aug = np.array(self.transform([arr[0].copy()])[0], dtype=np.float32)
            d_aug = np.array(self.transform([arr[1].copy()])[0], dtype=np.float32)
            return (source, driving, np.ascontiguousarray(s_aug.transpose(2, 0, 1)),
                    np.ascontiguousarray(d_aug.transpose(2, 0, 1)))
        video = np.stack(arr)
        return np.ascontiguousarray(video.transpose(3, 0, 1, 2))


class DatasetRepeater(Dataset):
    """dataset.py:132-145: several passes over the same dataset per epoch."""

    def __init__(self, dataset, num_repeats: int = 75):
        self.dataset = dataset
        self.num_repeats = num_repeats

    def __len__(self):
        return self.num_repeats * len(self.dataset)

    def __getitem__(self, idx):
        return self.dataset[idx % len(self.dataset)]


class SyntheticFramesDataset(Dataset):
    """`n` items of (source, driving, source_aug, driving_aug), each [3, H, H] float32 ~ U[0, 1),
    deterministic per index (seed = 1234 + index)."""

    def __init__(self, n: int, H: int = 256):
        self.n, self.H = n, H

    def __len__(self):
        return self.n

    def __getitem__(self, idx):
        g = np.random.default_rng(1234 + idx)
        s = g.random((3, self.H, self.H), dtype=np.float32)
        d = g.random((3, self.H, self.H), dtype=np.float32)
        return s, d, s.copy(), d.copy()
