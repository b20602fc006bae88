"""Drop-in ``Engine`` (reference: engine/engine.py:14-163).

Same surface as the reference: a context manager with ``.distributed``, ``.local_rank``,
``.world_size``, ``.devices``, ``.state``, ``.continue_state_object``, ``.args``; methods
``register_state``, ``update_iteration``, ``save_checkpoint``, ``save_and_link_checkpoint``,
``restore_checkpoint``, ``link_tb``; the ``-d/-c/--local_rank/-p`` flags; and checkpoint
dicts with keys ``model`` / ``optimizer`` / ``epoch`` / ``iteration``.

MI355X specifics:
  * one process per GPU; the rank's device comes from ``LOCAL_RANK`` (torchrun) or
    ``--local_rank`` (torch.distributed.launch); the process group is RCCL (backend "nccl")
    and binds the device at init (``device_id``) so collectives skip lazy setup;
  * checkpoints are read with ``torch.load(weights_only=True)`` onto the CPU and keys are
    normalised (a ``module.`` prefix is stripped whether or not the run is distributed,
    fixing the reference's non-DDP restore of DDP-written files).
"""
from __future__ import annotations

import argparse
import os
import os.path as osp
import time
from collections import OrderedDict

import torch
import torch.distributed as dist

from .logger import get_logger
from ..utils.pyt_utils import ensure_dir, extant_file, link_file, parse_devices

logger = get_logger()


class State:
    _KEYS = ("epoch", "iteration", "dataloader", "model", "optimizer")

    def __init__(self):
        self.epoch = 1
        self.iteration = 0
        self.dataloader = None
        self.model = None
        self.optimizer = None

    def register(self, **kwargs):
        for k, v in kwargs.items():
            if k not in self._KEYS:
                raise KeyError(f"unknown engine state '{k}' (expected one of {self._KEYS})")
            setattr(self, k, v)


def _strip_module(sd):
    out = OrderedDict()
    for k, v in sd.items():
        out[k[7:] if k.startswith("module.") else k] = v
    return out


class Engine:
    def __init__(self, custom_parser: argparse.ArgumentParser | None = None, argv=None):
        logger.info(f"PyTorch Version {torch.__version__}")
        self.state = State()
        self.devices = None
        self.distributed = False
        self.world_size = 1
        self.local_rank = 0
        if custom_parser is None:
            self.parser = argparse.ArgumentParser()
        else:
            if not isinstance(custom_parser, argparse.ArgumentParser):
                raise TypeError("custom_parser must be an argparse.ArgumentParser")
            self.parser = custom_parser
        self.inject_default_parser()
        self.args = self.parser.parse_args(argv)
        self.continue_state_object = self.args.continue_fpath

        if "WORLD_SIZE" in os.environ:
            self.distributed = int(os.environ["WORLD_SIZE"]) > 1
        if self.distributed:
            self.local_rank = int(os.environ.get("LOCAL_RANK", self.args.local_rank))
            self.world_size = int(os.environ["WORLD_SIZE"])
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", self.args.port)
            if torch.cuda.is_available():
                torch.cuda.set_device(self.local_rank)
                dist.init_process_group(backend="nccl", world_size=self.world_size, init_method="env://",
                                        device_id=torch.device("cuda", self.local_rank))
            else:   # CPU rehearsal of the DP path
                dist.init_process_group(backend="gloo", world_size=self.world_size, init_method="env://")
            self.devices = list(range(self.world_size))
        else:
            self.devices = parse_devices(self.args.devices)

    def inject_default_parser(self):
        p = self.parser
        p.add_argument("-d", "--devices", default="", help="set data parallel training")
        p.add_argument("-c", "--continue", type=extant_file, metavar="FILE", dest="continue_fpath",
                       help="continue from one certain checkpoint")
        p.add_argument("--local_rank", "--local-rank", default=0, type=int, help="process rank on node")
        p.add_argument("-p", "--port", type=str, default="16005", dest="port", help="port for init_process_group")

    def register_state(self, **kwargs):
        self.state.register(**kwargs)

    def update_iteration(self, epoch, iteration):
        self.state.epoch = epoch
        self.state.iteration = iteration

    def save_checkpoint(self, path):
        logger.info(f"Saving checkpoint to file {path}")
        t0 = time.time()
        state = {
            "model": _strip_module(self.state.model.state_dict()),
            "optimizer": self.state.optimizer.state_dict(),
            "epoch": self.state.epoch,
            "iteration": self.state.iteration,
        }
        t1 = time.time()
        torch.save(state, path)
        logger.info(f"Save checkpoint to file {path}, Time usage:\n\tprepare checkpoint: {t1 - t0}, "
                    f"IO: {time.time() - t1}")

    def link_tb(self, source, target):
        ensure_dir(source)
        ensure_dir(target)
        link_file(source, target)

    def save_and_link_checkpoint(self, checkpoint_dir, log_dir, log_dir_link):
        ensure_dir(checkpoint_dir)
        if not osp.exists(log_dir_link):
            link_file(log_dir, log_dir_link)
        current = osp.join(checkpoint_dir, f"epoch-{self.state.epoch}.pth")
        self.save_checkpoint(current)
        link_file(current, osp.join(checkpoint_dir, "epoch-last.pth"))

    def restore_checkpoint(self):
        t0 = time.time()
        tmp = torch.load(self.continue_state_object, map_location="cpu", weights_only=True)
        t1 = time.time()
        self.state.model.load_state_dict(_strip_module(tmp["model"]), strict=True)
        self.state.optimizer.load_state_dict(tmp["optimizer"])
        self.state.epoch = tmp["epoch"] + 1
        self.state.iteration = tmp["iteration"]
        logger.info(f"Load checkpoint from file {self.continue_state_object}, Time usage:\n\tIO: {t1 - t0}, "
                    f"restore checkpoint: {time.time() - t1}")

    def __enter__(self):
        return self

    def __exit__(self, exc_type, value, tb):
        if torch.cuda.is_available():
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
        # the communicator goes last, after the device has drained (a process
        # group torn down under live RCCL work was the one recorded hang); on an exception the
        # peers may never reach a barrier, so only the clean path waits for them
        if self.distributed and torch.distributed.is_available() and torch.distributed.is_initialized():
            if exc_type is None:
                torch.distributed.barrier()
            torch.distributed.destroy_process_group()
        if exc_type is not None:
            logger.warning("A exception occurred during Engine initialization, give up running process")
            return False
        return None
