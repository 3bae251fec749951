"""Input-pipeline throughput: FramesDataset (PNG decode, two frames per item) through a
torch DataLoader, with and without the *_aug augmentation, on a synthetic frame tree.

    python tools/databench.py [--workers 16] [--videos 64] [--frames 8] [--items 4096]

Prints one JSON line: items/s and frames/s (an item = source + driving, 2 decoded frames) for
each mode: the FaceVAE feed (FramesDataset(output="driving_uint8"): the driving frame as bytes,
converted to float32 on the GPU when there is one; images/s), the (source, driving) uint8
items, the reference's float32 items without and with the *_aug augmentation.  The FaceVAE
step consumes `driving` only, so the feed rate is the one that bounds it; the
augmented rate bounds the full GeneratorFull inputs.
"""
import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import fvamd  # noqa: E402,F401
from facevae_amd.data import DatasetRepeater, FramesDataset  # noqa: E402


def make_tree(root, videos, frames, H):
    from PIL import Image
    rng = np.random.default_rng(0)
    for split in ("train", "test"):
        for v in range(videos):
            d = os.path.join(root, split, f"id{v // 2:05d}#vid{v:05d}.mp4")
            os.makedirs(d)
            for f in range(frames):
                # smooth-ish content so PNG compression behaves like face crops, not noise
                base = rng.random((H // 8, H // 8, 3))
                img = np.kron(base, np.ones((8, 8, 1))) + 0.05 * rng.random((H, H, 3))
                Image.fromarray((np.clip(img, 0, 1) * 255).astype(np.uint8)).save(os.path.join(d, f"{f:07d}.png"))


def rate(ds, workers, items, batch, to_gpu=False):
    """Items/s out of a DataLoader (shuffled, pinned memory as train.py); to_gpu: each batch's
    `driving` also goes through to_device_frames (H2D + the uint8 -> float32 division)."""
    from facevae_amd.data import to_device_frames
    loader = torch.utils.data.DataLoader(DatasetRepeater(ds, 1000), batch_size=batch, num_workers=workers,
                                         shuffle=True, drop_last=True, persistent_workers=workers > 0,
                                         pin_memory=to_gpu)
    it = iter(loader)
    next(it)                                   # worker start-up
    t0 = time.perf_counter()
    n = 0
    while n < items:
        b = next(it)
        d = b[1] if isinstance(b, (list, tuple)) else b
        if to_gpu:
            to_device_frames(d, "cuda")
        n += d.shape[0]
    if to_gpu:
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return n / dt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", type=int, default=min(16, os.cpu_count() or 1))
    ap.add_argument("--videos", type=int, default=64)
    ap.add_argument("--frames", type=int, default=8)
    ap.add_argument("--items", type=int, default=4096)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--res", type=int, default=256)
    a = ap.parse_args()
    with tempfile.TemporaryDirectory() as root:
        make_tree(root, a.videos, a.frames, a.res)
        out = {"workers": a.workers, "res": a.res}
        gpu = torch.cuda.is_available()
        feed = FramesDataset(root, frame_shape=(a.res, a.res, 3), output="driving_uint8")
        r = rate(feed, a.workers, a.items, a.batch, to_gpu=gpu)
        out.update(facevae_feed_images_per_s=round(r, 1), facevae_feed_to_gpu=gpu)
        feed = FramesDataset(root, frame_shape=(a.res, a.res, 3), output="uint8")
        r = rate(feed, a.workers, a.items, a.batch, to_gpu=gpu)
        out.update(uint8_items_per_s=round(r, 1), uint8_frames_per_s=round(2 * r, 1))
        plain = FramesDataset(root, frame_shape=(a.res, a.res, 3), augmentation_params=None)
        r = rate(plain, a.workers, a.items, a.batch)
        out.update(decode_items_per_s=round(r, 1), decode_frames_per_s=round(2 * r, 1))
        aug = FramesDataset(root, frame_shape=(a.res, a.res, 3))
        r = rate(aug, a.workers, max(a.batch, a.items // 4), a.batch)
        out.update(augmented_items_per_s=round(r, 1))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
