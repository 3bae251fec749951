"""FaceVAE training entry point with the reference CLI (train.py:10-54 of Luh1124/face-vae).

    python train.py --gpu_ids [0,1,2,3,4,5,6,7] --batch_size 32 --root_dir <vox-png> ...
    python train.py --gpu_ids [0] --synthetic 256 --num_epochs 1        # no dataset on disk

Same flags, the same seeding / rendezvous order (init_seeds before init_dist, so every rank
seeds 1), one process per GPU via mp.spawn, a DistributedSampler over
DatasetRepeater(FramesDataset(root_dir), 100), and the Logger surface (here FaceVAETrainer:
.load_cpk(ckp), .step() per epoch).  Extra flags: --synthetic N (N synthetic frames instead
of a dataset), --config toy|256|512, --backend nccl|gloo (gloo: several ranks on one GPU),
--feed driving_uint8|uint8|float32 (data feed format, see data.py), --dump_dir (each rank writes its final
state_dict; used by the tests).
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402
import torch.utils.data as data  # noqa: E402


def _config(name):
    import facevae_amd as fv
    return {"toy": fv.FaceVAEConfig.toy(), "256": fv.FaceVAEConfig(), "512": fv.FaceVAEConfig.hires()}[name]


def main(proc, args):
    import facevae_amd as fv
    from facevae_amd.data import DatasetRepeater, FramesDataset, SyntheticFramesDataset
    from facevae_amd.distributed import init_dist, init_seeds
    world_size = len(args.gpu_ids)
    init_seeds(not args.benchmark)
    if args.init == "torch":
        # what the reference's own init_dist does (distributed.py:24-31): only a torch process
        # group; FaceVAETrainer then builds the communicator from it
        torch.cuda.set_device(proc % torch.cuda.device_count())
        torch.distributed.init_process_group(backend=args.backend, init_method="env://", world_size=world_size,
                                             rank=proc)
    else:
        init_dist(proc, world_size, backend=args.backend)
    cfg = _config(args.config)
    cfg.lr = args.lr
    if args.synthetic:
        trainset = SyntheticFramesDataset(args.synthetic, cfg.H)
    else:
        # --feed driving_uint8 (default): the driving frame alone leaves the workers as bytes and
        # becomes float32 [0, 1] on the GPU (bit-identical to the reference's img_as_float32; the
        # FaceVAE step reads only `driving`, so neither `source` nor the *_aug copies are made);
        # --feed uint8: (source, driving) bytes; --feed float32: the reference items
        trainset = DatasetRepeater(FramesDataset(root_dir=args.root_dir, frame_shape=(cfg.H, cfg.H, 3),
                                                 output=args.feed), num_repeats=100)
    trainsampler = data.distributed.DistributedSampler(trainset, num_replicas=world_size, rank=proc)
    trainloader = data.DataLoader(trainset, batch_size=args.batch_size, num_workers=args.num_workers,
                                  pin_memory=True, sampler=trainsampler)
    logger = fv.FaceVAETrainer(args.ckp_dir, args.vis_dir, trainloader, args.lr, log_file_name=args.log_file,
                               cfg=cfg, graph=args.graph)
    if args.ckp > 0:
        logger.load_cpk(args.ckp)
    for _ in range(args.num_epochs):
        logger.step()
    if args.dump_dir:
        os.makedirs(args.dump_dir, exist_ok=True)
        torch.save({k: v.detach().cpu() for k, v in logger.model.state_dict().items()},
                   os.path.join(args.dump_dir, f"rank{proc}.pt"))
    if torch.distributed.is_initialized():
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()


def parse(argv=None):
    parser = argparse.ArgumentParser(description="face-vae (MI355X)")

    def str2bool(s):
        return s.lower().startswith("t")

    parser.add_argument("--batch_size", default=8, type=int, help="Batch size per GPU")
    parser.add_argument("--benchmark", type=str2bool, default=True, help="(reference: cuDNN benchmarking)")
    parser.add_argument("--gpu_ids", default=[0, 1, 2], type=eval, help="IDs of GPUs to use")
    parser.add_argument("--lr", default=0.00005, type=float, help="Learning rate")
    parser.add_argument("--num_epochs", default=150, type=int, help="Number of epochs to train")
    parser.add_argument("--num_workers", default=8, type=int, help="Number of data loader threads")
    parser.add_argument("--ckp_dir", type=str, default="ckp_1644_", help="Checkpoint dir")
    parser.add_argument("--vis_dir", type=str, default="vis_1644_", help="Visualization dir")
    parser.add_argument("--ckp", type=int, default=0, help="Checkpoint epoch")
    parser.add_argument("--log_file", type=str, default="log_1644_.txt", help="log file")
    parser.add_argument("--ext", type=str, default="add", help="extension")
    parser.add_argument("--root_dir", type=str, default="/home/lh/repo/datasets/face-video-preprocessing/vox-png",
                        help="data_path")
    parser.add_argument("--synthetic", type=int, default=0, help="N synthetic frames instead of root_dir")
    parser.add_argument("--config", default="256", choices=["toy", "256", "512"])
    parser.add_argument("--backend", default="nccl", choices=["nccl", "gloo"])
    parser.add_argument("--graph", type=str2bool, default=False,
                        help="replay each step as a captured HIP graph (FaceVAETrainer(graph=True); several GPUs: graph "
                             "segments between the collectives)")
    parser.add_argument("--feed", default="driving_uint8", choices=["driving_uint8", "uint8", "float32"],
                        help="FramesDataset output: uint8 frames converted on the GPU, or the reference's float32 items")
    parser.add_argument("--dump_dir", type=str, default="")
    parser.add_argument("--init", default="ours", choices=["ours", "torch"],
                        help="rendezvous: our init_dist, or a bare torch process group (reference style)")
    args = parser.parse_args(argv)
    # train.py:47-49, including its log-file naming (directory part of --log_file + ext + .txt)
    args.ckp_dir = args.ckp_dir + args.ext
    args.vis_dir = args.vis_dir + args.ext
    args.log_file = os.path.split(args.log_file)[0] + args.ext + ".txt"
    return args


if __name__ == "__main__":
    args = parse()
    os.environ["CUDA_VISIBLE_DEVICES"] = str(args.gpu_ids)[1:-1] if args.backend == "nccl" else \
        os.environ.get("CUDA_VISIBLE_DEVICES", "0")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "2345")
    if args.backend == "gloo":           # several ranks may share GPU 0
        args.gpu_ids = list(range(len(args.gpu_ids)))
    mp.spawn(main, nprocs=len(args.gpu_ids), args=(args,))
