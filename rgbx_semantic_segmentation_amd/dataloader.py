"""Train loader with the reference's interface (dataloader/dataloader.py:129-165).

``get_train_loader(engine, dataset, config) -> (loader, sampler | None)``: the global
``config.batch_size`` is split across ranks (dataloader.py:155), a DistributedSampler
shards the index space, and every minibatch is a dict with keys ``data`` / ``label`` /
``modal_x`` / ``fn`` / ``n`` (RGBXDataset.py:71).

``SyntheticRGBXDataset`` yields seeded samples with the reference's input semantics
(data.make_batch: ImageNet-normalised uint8 RGB, one replicated X plane, labels with a
25x25 ignore block).  Reading real NYUDepthv2/MFNet files (cv2-based augmentation
pipeline, RGBXDataset.py) is outside the hot-path scope; any
torch Dataset returning the same dict keys plugs in unchanged.
"""
from __future__ import annotations

import torch
from torch.utils.data import DataLoader, Dataset
from torch.utils.data.distributed import DistributedSampler

from .data import make_batch


class SyntheticRGBXDataset(Dataset):
    def __init__(self, length: int, H: int, W: int, num_classes: int, seed: int = 12345, background: int = 255):
        self.length, self.H, self.W, self.K, self.seed, self.background = length, H, W, num_classes, seed, background

    def __len__(self):
        return self.length

    def __getitem__(self, idx):
        rgb, x, lab = make_batch(1, self.H, self.W, self.K, seed=self.seed + idx, background=self.background)
        return {"data": rgb[0], "label": lab[0], "modal_x": x[0], "fn": f"synthetic_{idx:06d}", "n": self.length}


def get_train_loader(engine, dataset: Dataset, config):
    batch_size = int(config.batch_size)
    sampler = None
    shuffle = True
    if engine.distributed:
        sampler = DistributedSampler(dataset)
        batch_size = batch_size // engine.world_size
        shuffle = False
    loader = DataLoader(dataset, batch_size=batch_size, num_workers=int(getattr(config, "num_workers", 0)),
                        drop_last=True, shuffle=shuffle, pin_memory=torch.cuda.is_available(), sampler=sampler)
    return loader, sampler
