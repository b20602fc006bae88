"""Host helpers used by the Engine and train loop (reference: utils/pyt_utils.py:110-246).

``link_file`` / ``ensure_dir`` use os calls instead of shelling out (`rm -rf`, `ln -s`);
``parse_devices('')`` returns [] (the reference raises on int('') when -d is omitted).
"""
from __future__ import annotations

import argparse
import os
import shutil

import torch
import torch.distributed as dist


def reduce_tensor(tensor, dst=0, op=dist.ReduceOp.SUM, world_size=1):
    """pyt_utils.py:110-116: reduce to dst, divided by world_size."""
    t = tensor.clone()
    dist.reduce(t, dst, op)
    if dist.get_rank() == dst:
        t.div_(world_size)
    return t


def all_reduce_tensor(tensor, op=dist.ReduceOp.SUM, world_size=1):
    """pyt_utils.py:119-124: all-reduce a copy, divided by world_size."""
    t = tensor.clone()
    dist.all_reduce(t, op)
    t.div_(world_size)
    return t


def parse_devices(input_devices: str):
    """'0,2-3' -> [0, 2, 3]; '*' -> every visible device; '' -> []."""
    if input_devices.endswith("*"):
        return list(range(torch.cuda.device_count()))
    devices = []
    for d in filter(None, (s.strip() for s in input_devices.split(","))):
        if "-" in d:
            a, b = (int(v) for v in d.split("-"))
            if not a < b:
                raise ValueError(f"bad device range {d}")
            devices.extend(range(a, b + 1))
        else:
            devices.append(int(d))
    return devices


def extant_file(x: str) -> str:
    if not os.path.exists(x):
        raise argparse.ArgumentTypeError(f"{x} does not exist")
    return x


def link_file(src: str, target: str) -> None:
    if os.path.islink(target) or os.path.isfile(target):
        os.remove(target)
    elif os.path.isdir(target):
        shutil.rmtree(target)
    os.symlink(src, target)


def ensure_dir(path: str) -> None:
    os.makedirs(path, exist_ok=True)
