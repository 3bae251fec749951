"""Frame datasets for the FaceVAE trainer (dataset.py:36-150 of Luh1124/face-vae).

`FramesDataset` keeps the reference constructor, directory conventions and item layout:
`root_dir` holds one folder of PNG frames per video (`<id>#<video>.mp4/`), optionally split
into `train/` and `test/`; with `id_sampling` the training set is the set of identities and an
item picks a random video of the identity, then two random frames (sorted indices), returned
as `(source, driving, source_aug, driving_aug)` float32 CHW arrays in [0, 1]
(dataset.py:91-129).  Frames are decoded with PIL (skimage is not in this image; for uint8
PNGs `img_as_float32` is the same division by 255).  The `*_aug` items go through
`augmentation.AllAugmentationTransform` with the reference's default parameters (rotation
30 degrees, perspective (30, 40), colour jitter 0.1, dataset.py:52-57), each frame on its own
as dataset.py:122-123; they feed the keypoint / contrastive losses, not the FaceVAE path.

`SyntheticFramesDataset` produces VoxCeleb-shaped frames x ~ U[0, 1) deterministically per
index (the benchmark / test input when no dataset is on disk).
"""
from __future__ import annotations

import glob
import os
from typing import Optional, Sequence

import numpy as np
from torch.utils.data import Dataset


def _read_frame(path: str) -> np.ndarray:
    from PIL import Image
    with Image.open(path) as im:
        a = np.asarray(im.convert("RGB"))
    return a.astype(np.float32) / 255.0


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
                 random_seed: int = 0, pairs_list: Optional[str] = None, augmentation_params=DEFAULT_AUGMENTATION):
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
        self.transform = AllAugmentationTransform(**(augmentation_params or {})) if is_train else None

    def __len__(self):
        return len(self.videos)

    def _frames(self, path):
        return sorted(os.listdir(path))

    def __getitem__(self, idx):
        name = self.videos[idx]
        if self.is_train and self.id_sampling:
            path = str(np.random.choice(glob.glob(os.path.join(self.root_dir, name + "*.mp4"))))
        else:
            path = os.path.join(self.root_dir, name)
        if not os.path.isdir(path):
            raise NotImplementedError("FramesDataset: frame folders only (.mp4/.gif decoding needs imageio, "
                                      "not in this image)")
        frames = self._frames(path)
        if self.is_train:
            fidx = np.sort(np.random.choice(len(frames), replace=True, size=2))
            arr = [_read_frame(os.path.join(path, frames[i])) for i in fidx]
            source = np.ascontiguousarray(arr[0].transpose(2, 0, 1))
            driving = np.ascontiguousarray(arr[1].transpose(2, 0, 1))
            if self.transform is None:
                return source, driving, None, None
            s_aug = np.array(self.transform([arr[0].copy()])[0], dtype=np.float32)
            d_aug = np.array(self.transform([arr[1].copy()])[0], dtype=np.float32)
            return (source, driving, np.ascontiguousarray(s_aug.transpose(2, 0, 1)),
                    np.ascontiguousarray(d_aug.transpose(2, 0, 1)))
        video = np.stack([_read_frame(os.path.join(path, f)) for f in frames])
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
