"""Training entry point with the reference loop's shape (train.py:32-223), on the HIP path.

    python train.py [--backbone mit_b2 --height 480 --width 640 --batch-size 2 ...]
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 train.py ...

Same sequence per iteration as the reference: H2D copy, ``loss = model(rgb, modal_x, gt)``,
(distributed) loss all-reduce for logging, ``optimizer.zero_grad()`` (a no-op: backward
overwrites the flat gradient buffer), ``loss.backward()``, ``optimizer.step()`` (RCCL
gradient all-reduce + fused AdamW), THEN the WarmUpPolyLR update (the LR lands one step
late, as in the reference).  Differences: DistributedDataParallel is replaced by the flat
gradient all-reduce (dist.py); data is the synthetic dataset unless --dataset-path names one
in the reference's layout (then RGBXDataset + TrainPre on the GPU, augment.py);
TensorBoard logging is omitted (tensorboardX is not installed).
"""
from __future__ import annotations

import argparse
import os
import sys
import time
from types import SimpleNamespace

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from rgbx_semantic_segmentation_amd.engine.engine import Engine  # noqa: E402
from rgbx_semantic_segmentation_amd.engine.logger import get_logger  # noqa: E402
from rgbx_semantic_segmentation_amd.dataloader import RGBXDataset, SyntheticRGBXDataset, get_train_loader  # noqa: E402
from rgbx_semantic_segmentation_amd.utils.lr_policy import WarmUpPolyLR  # noqa: E402
from rgbx_semantic_segmentation_amd.utils.pyt_utils import all_reduce_tensor  # noqa: E402

logger = get_logger()


def build_parser():
    p = argparse.ArgumentParser()
    p.add_argument("--backbone", default="mit_b2")
    p.add_argument("--num-classes", type=int, default=40)
    p.add_argument("--height", type=int, default=480)
    p.add_argument("--width", type=int, default=640)
    p.add_argument("--batch-size", type=int, default=2, help="GLOBAL batch (divided by world size)")
    p.add_argument("--lr", type=float, default=6e-5)
    p.add_argument("--lr-power", type=float, default=0.9)
    p.add_argument("--weight-decay", type=float, default=0.01)
    p.add_argument("--nepochs", type=int, default=1)
    p.add_argument("--niters-per-epoch", type=int, default=10)
    p.add_argument("--warm-up-epoch", type=int, default=10)
    p.add_argument("--compute-dtype", default=None, choices=["bfloat16", "float32", "float16"],
                   help="default: float16 with --use-mixed-precision (the reference's fp16 autocast), else bfloat16")
    p.add_argument("--criterion", default="CrossEntropyLoss")
    p.add_argument("--optimizer", default="AdamW")
    p.add_argument("--seed", type=int, default=12345)
    p.add_argument("--use-mixed-precision", action="store_true",
                   help="config.use_mixed_precision (config.py:61): dynamic loss scaling (GradScaler, train.py:185-198)")
    p.add_argument("--dataset-path", default="",
                   help="a dataset in the reference's layout (config.py:19-33): RGB/, Label/, <x-folder>/, "
                        "<train-source>; empty: the synthetic dataset")
    p.add_argument("--x-folder", default="Thermal")
    p.add_argument("--train-source", default="train_val.txt")
    p.add_argument("--image-format", default=".png")
    p.add_argument("--x-multi-channel", action="store_true", help="config.x_is_single_channel = False")
    p.add_argument("--gt-transform", action="store_true", help="config.gt_transform (label - 1)")
    p.add_argument("--num-workers", type=int, default=2)
    p.add_argument("--checkpoint-dir", default="")
    p.add_argument("--checkpoint-start-epoch", type=int, default=1)
    p.add_argument("--checkpoint-step", type=int, default=1)
    return p


def resolve_precision(args):
    """(compute dtype, dynamic loss scaling on?).  The reference runs fp16 only under autocast
    with a GradScaler (train.py:185-198), so fp16 storage always turns loss scaling on, as in
    bench.py: fp16 training without it would let gradient under/overflow go undetected."""
    dtype = args.compute_dtype or ("float16" if args.use_mixed_precision else "bfloat16")
    return dtype, bool(args.use_mixed_precision or dtype == "float16")


def main(argv=None):
    parser = build_parser()
    with Engine(custom_parser=parser, argv=argv) as engine:
        args = engine.args
        seed = engine.local_rank if engine.distributed else args.seed
        torch.manual_seed(seed)
        if args.criterion != "CrossEntropyLoss":
            raise NotImplementedError(f"criterion {args.criterion} (only CrossEntropyLoss is on the HIP path)")
        if args.optimizer != "AdamW":
            raise NotImplementedError(f"optimizer {args.optimizer} (only AdamW is on the HIP path)")
        if not torch.cuda.is_available():
            raise RuntimeError("train.py runs the HIP path and needs a GPU")
        dev = torch.device("cuda", engine.local_rank)

        if args.dataset_path:
            # the reference's file dataset + TrainPre on the GPU (dataloader.py:129-165)
            root = args.dataset_path
            fmt = args.image_format
            config = SimpleNamespace(
                rgb_root_folder=os.path.join(root, "RGB"), rgb_format=fmt, gt_root_folder=os.path.join(root, "Label"),
                gt_format=fmt, gt_transform=args.gt_transform, x_root_folder=os.path.join(root, args.x_folder),
                x_format=fmt, x_is_single_channel=not args.x_multi_channel,
                train_source=os.path.join(root, args.train_source), eval_source=os.path.join(root, args.train_source),
                background=255, num_classes=args.num_classes, image_height=args.height, image_width=args.width,
                norm_mean=[0.485, 0.456, 0.406], norm_std=[0.229, 0.224, 0.225],
                train_scale_array=[0.5, 0.75, 1, 1.25, 1.5, 1.75], batch_size=args.batch_size,
                niters_per_epoch=args.niters_per_epoch, num_workers=args.num_workers)
            train_loader, train_sampler = get_train_loader(engine, RGBXDataset, config)
        else:
            config = SimpleNamespace(batch_size=args.batch_size, num_workers=0)
            dataset = SyntheticRGBXDataset(args.niters_per_epoch * args.batch_size, args.height, args.width,
                                           args.num_classes, seed=args.seed)
            train_loader, train_sampler = get_train_loader(engine, dataset, config)

        from rgbx_semantic_segmentation_amd.models.builder import EncoderDecoder
        from rgbx_semantic_segmentation_amd.optim import FusedAdamW, GradScaler
        from rgbx_semantic_segmentation_amd import dist as cdist

        norm = torch.nn.SyncBatchNorm if engine.distributed else torch.nn.BatchNorm2d
        dtype, loss_scaling = resolve_precision(args)
        cfg = dict(backbone=args.backbone, num_classes=args.num_classes, compute_dtype=dtype,
                   decoder_embed_dim=512)
        model = EncoderDecoder(cfg, norm_layer=norm).to(dev)
        sync = None
        if engine.distributed:
            group = torch.distributed.group.WORLD
            model.process_group = group
            cdist.broadcast_parameters(model, group)
            sync = cdist.BucketedGradSync(model.store, group)
            model.backbone.grad_sync = sync    # segment all-reduces overlap the backward
        optimizer = FusedAdamW(model, lr=args.lr, betas=(0.9, 0.999), weight_decay=args.weight_decay,
                               grad_sync=sync)
        total_iteration = args.nepochs * args.niters_per_epoch
        lr_policy = WarmUpPolyLR(args.lr, args.lr_power, total_iteration, args.niters_per_epoch * args.warm_up_epoch)

        scaler = GradScaler(enabled=loss_scaling, device=dev)
        engine.register_state(dataloader=train_loader, model=model, optimizer=optimizer)
        if engine.continue_state_object:
            engine.restore_checkpoint()

        optimizer.zero_grad()
        model.train()
        logger.info("begin training:")
        for epoch in range(engine.state.epoch, args.nepochs + 1):
            if train_sampler is not None:
                train_sampler.set_epoch(epoch)
            dataloader = iter(train_loader)
            sum_loss = 0.0
            t0 = time.time()
            for idx in range(args.niters_per_epoch):
                engine.update_iteration(epoch, idx)
                mb = next(dataloader)
                imgs = mb["data"].to(dev, non_blocking=True)
                gts = mb["label"].to(dev, non_blocking=True)
                modal_xs = mb["modal_x"].to(dev, non_blocking=True)
                loss = model(imgs, modal_xs, gts)
                reduce_loss = all_reduce_tensor(loss.detach(), world_size=engine.world_size) \
                    if engine.distributed else loss.detach()
                optimizer.zero_grad()
                if scaler.is_enabled():          # train.py:185-198 under use_mixed_precision
                    scaler.scale(loss).backward()
                    scaler.step(optimizer)
                    scaler.update()
                else:
                    loss.backward()
                    optimizer.step()
                current_idx = (epoch - 1) * args.niters_per_epoch + idx
                lr = lr_policy.get_lr(current_idx)
                for g in optimizer.param_groups:
                    g["lr"] = lr
                sum_loss += reduce_loss.item()
                if engine.local_rank == 0:
                    logger.info(f"Epoch {epoch}/{args.nepochs} Iter {idx + 1}/{args.niters_per_epoch}: lr={lr:.4e} "
                                f"loss={reduce_loss.item():.4f} total_loss={sum_loss / (idx + 1):.4f}")
            torch.cuda.synchronize()
            if engine.local_rank == 0:
                dt = time.time() - t0
                logger.info(f"epoch {epoch}: {args.niters_per_epoch * args.batch_size / dt:.2f} images/s (eager)")
            # the reference's schedule (train.py:310): from the start epoch on every step-th
            # epoch, and always the last epoch
            save = (epoch >= args.checkpoint_start_epoch and epoch % args.checkpoint_step == 0) or \
                epoch == args.nepochs
            if args.checkpoint_dir and engine.local_rank == 0 and save:
                engine.save_and_link_checkpoint(args.checkpoint_dir, args.checkpoint_dir,
                                                os.path.join(args.checkpoint_dir, "log_last"))
        return sum_loss / max(1, args.niters_per_epoch)


if __name__ == "__main__":
    main()
