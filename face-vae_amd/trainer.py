"""Logger-compatible FaceVAE trainer (logger.py:24-184 of Luh1124/face-vae, restricted to the
FaceVAE hot path).

`FaceVAETrainer(ckp_dir, vis_dir, dataloader, lr, ...)` keeps the reference constructor and
the `.step()` / `.save_cpk()` / `.load_cpk(epoch)` surface.  One `train_step` is the
Logger.step iteration (logger.py:150-164): zero_grad -> forward -> loss = sum of weighted
losses -> backward (gradient all-reduce overlapped) -> Adam.step.  The batch element used
as the VAE input is `driving`.
"""
from __future__ import annotations

import collections
import os
from typing import Dict, Optional

import numpy as np
import torch
import torch.distributed as dist

from . import config as _config
from . import distributed
from .data import to_device_frames
from .losses import KLDivergenceLoss, ReconLoss
from .models import FaceVAE
from .optim import Adam


class FaceVAETrainer:
    def __init__(self, ckp_dir, vis_dir, dataloader, lr, checkpoint_freq=1, visualizer_params=None, zfill_num=8,
                 log_file_name="log_facevae.txt", cfg: Optional[_config.FaceVAEConfig] = None,
                 compute_dtype: Optional[torch.dtype] = None, seed: Optional[int] = None, graph: bool = False):
        self.cfg = cfg or _config.FaceVAEConfig(lr=lr)
        self.ckp_dir, self.vis_dir = ckp_dir, vis_dir
        self.dataloader = dataloader
        self.checkpoint_freq, self.zfill_num = checkpoint_freq, zfill_num
        self.epoch = 0
        self.g_losses = []
        self.loss_names = None
        self.log_file = None
        if distributed.is_master() and ckp_dir is not None:
            os.makedirs(ckp_dir, exist_ok=True)
            if vis_dir:
                os.makedirs(vis_dir, exist_ok=True)
            self.log_file = open(log_file_name, "a")
        if seed is not None:          # the reference seeds in train.py (init_seeds), not here
            torch.manual_seed(seed)
        self.model = FaceVAE(self.cfg).cuda()
        if compute_dtype is not None:
            self.model.set_compute_dtype(compute_dtype)
        # a process group initialised by the caller (e.g. the reference's init_dist, which
        # uses torch.distributed directly) gets its communicator here: the model is never
        # trained unsynchronised under a multi-rank launch
        self.comm = distributed.get_comm()
        if self.comm is None and dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            self.comm = distributed.comm_from_process_group(self.cfg.syncbn)
        multi = self.comm is not None and self.comm.world_size > 1
        self.ddp = distributed.DataParallel(self.model, self.comm) if multi else None
        self.net = self.ddp if self.ddp is not None else self.model
        # one Adam per model as logger.py:60 (elementwise: identical to one over all params)
        self.g_models = {"afe": self.model.afe, "generator": self.model.generator}
        self.g_optimizers = {k: Adam(m.parameters(), lr=lr, betas=self.cfg.betas) for k, m in self.g_models.items()}
        self.kl, self.recon = KLDivergenceLoss(), ReconLoss()
        self.weights = {"R": self.cfg.w_R, "K": self.cfg.w_K}
        self._eps_gen = None
        # graph=True: train_step replays one captured HIP graph per batch shape (graph.StepGraph;
        # under DataParallel the graph segments between the collectives); the batch is copied
        # into static input buffers first.  A batch of another shape (e.g. the last, smaller
        # one, the same on every rank) runs eagerly.
        self.graph = bool(graph)
        self._sg = None

    # ---------------------------------------------------------------- one iteration
    def train_step(self, x: torch.Tensor, eps: torch.Tensor) -> Dict[str, torch.Tensor]:
        if self.graph:
            return self._graph_step(x, eps)
        return self._eager_step(x, eps)

    def _graph_step(self, x, eps):
        from .graph import StepGraph
        key = (tuple(x.shape), x.dtype, tuple(eps.shape))
        if self._sg is None or self._sg[0] != key:
            if self._sg is not None:
                return self._eager_step(x, eps)          # one graph, for the first batch shape
            xs, es = x.detach().clone(), eps.detach().clone()
            sg = StepGraph(lambda: self._eager_step(xs, es), list(self.g_optimizers.values()), warmup=1)
            sg.capture()                                  # the warm-up step trains on this batch
            self._sg = (key, xs, es, sg)
            return sg.warm_out
        _, xs, es, sg = self._sg
        xs.copy_(x)
        es.copy_(eps)
        return {k: v.clone() for k, v in sg.replay().items()}

    def _eager_step(self, x: torch.Tensor, eps: torch.Tensor) -> Dict[str, torch.Tensor]:
        for opt in self.g_optimizers.values():
            opt.zero_grad(set_to_none=True)
        y, mu, logstd = self.net(x, eps)
        R, K = self.recon((x, y)), self.kl((mu, logstd))
        losses = {"R": self.weights["R"] * R.detach(), "K": self.weights["K"] * K.detach()}
        # backward of sum(w * loss): the weights seed the two terms directly (no ones-fill, add
        # or scalar multiplies in the captured backward)
        torch.autograd.backward([R, K], list(self._loss_seeds(x.device)))
        for opt in self.g_optimizers.values():
            opt.step()
        losses["y"] = y
        return losses

    def _loss_seeds(self, device):
        key = (device, float(self.weights["R"]), float(self.weights["K"]))
        seeds = getattr(self, "_seeds", None)
        if seeds is None or seeds[0] != key:
            seeds = (key, torch.tensor(key[1], device=device), torch.tensor(key[2], device=device))
            self._seeds = seeds
        return seeds[1:]

    def sample_eps(self, x: torch.Tensor) -> torch.Tensor:
        B = x.shape[0]
        h = self.cfg.latent_hw
        if self._eps_gen is None:
            self._eps_gen = torch.Generator(device=x.device)
            self._eps_gen.manual_seed(1 + distributed.get_rank())
        return torch.randn(B, self.cfg.latent, h, h, device=x.device, generator=self._eps_gen)

    # ---------------------------------------------------------------- Logger surface
    def step(self):
        """One epoch over the dataloader (logger.py:135-184)."""
        for idx, batch in enumerate(self.dataloader):
            # (source, driving, source_aug, driving_aug) float32 items, (source, driving) uint8, or
            # the driving frames alone (FramesDataset(output="driving_uint8")): the VAE trains on
            # `driving`
            d = to_device_frames(batch[1] if isinstance(batch, (list, tuple)) else batch, "cuda")
            out = self.train_step(d, self.sample_eps(d))
            self.log_iter({k: v.detach().float().cpu().numpy() for k, v in out.items() if k != "y"})
        self.log_epoch()
        self.epoch += 1

    def log_iter(self, losses):
        if not distributed.is_master():
            return
        losses = collections.OrderedDict(losses.items())
        if self.loss_names is None:
            self.loss_names = list(losses.keys())
        self.g_losses.append(list(losses.values()))

    def log_scores(self):
        if not distributed.is_master() or self.log_file is None or not self.g_losses:
            return
        loss_mean = np.array(self.g_losses).mean(axis=0)
        s = "; ".join("%s - %.5f" % (n, v) for n, v in zip(self.loss_names, loss_mean))
        print("G" + str(self.epoch).zfill(self.zfill_num) + ") " + s, file=self.log_file)
        self.log_file.flush()
        self.g_losses = []

    def log_epoch(self):
        if (self.epoch + 1) % self.checkpoint_freq == 0:
            self.save_cpk()
        self.log_scores()
        if self.ddp is not None:
            self.ddp.sync_buffers()

    def save_cpk(self):
        if not distributed.is_master() or self.ckp_dir is None:
            return
        ckp = {**{k: m.state_dict() for k, m in self.g_models.items()},
               **{"optimizer_" + k: o.state_dict() for k, o in self.g_optimizers.items()},
               "epoch": self.epoch}
        torch.save(ckp, os.path.join(self.ckp_dir, "%s-checkpoint.pth.tar" % str(self.epoch).zfill(self.zfill_num)))

    def load_cpk(self, epoch):
        path = os.path.join(self.ckp_dir, "%s-checkpoint.pth.tar" % str(epoch).zfill(self.zfill_num))
        ckp = torch.load(path, map_location="cpu", weights_only=True)
        for k, m in self.g_models.items():
            m.load_state_dict(ckp[k])
        for k, o in self.g_optimizers.items():
            o.load_state_dict(ckp["optimizer_" + k])
        self.epoch = ckp["epoch"] + 1
        self._sg = None            # new optimizer state tensors: the next graph step recaptures
