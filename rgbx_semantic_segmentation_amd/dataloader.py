"""Train loader with the reference's interface (dataloader/dataloader.py:129-165) and the
RGB-X file dataset (dataloader/RGBXDataset.py).

``get_train_loader(engine, dataset, config) -> (loader, sampler | None)``: the global
``config.batch_size`` is split across ranks (dataloader.py:155), a DistributedSampler
shards the index space, and every minibatch is a dict with keys ``data`` / ``label`` /
``modal_x`` / ``fn`` / ``n`` (RGBXDataset.py:71).

Two kinds of dataset:
  * ``RGBXDataset`` -- the reference's file dataset (same constructor ``(setting, split_name,
    preprocess=None, file_length=None)``, same file list / extension / gt_transform rules).
    Passed as the CLASS, like the reference's ``get_train_loader(engine, RGBXDataset)``
    (train.py:45), the loader builds it from ``config`` and runs TrainPre ON THE GPU
    (augment.TrainPre, csrc/augment.hip): workers only decode files into uint8 arrays, the
    main process uploads them and augments straight into device batch tensors.
  * any torch Dataset instance returning the dict keys above (``SyntheticRGBXDataset``: seeded
    samples with the reference's input semantics, data.make_batch).
"""
from __future__ import annotations

import os

import numpy as np
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


def _open_image(path: str, mode: str) -> np.ndarray:
    """cv2.imread equivalents (RGBXDataset._open_image, :111-114) with PIL (cv2 is not in this
    image): mode "color" = the reference's flag 4 (IMREAD_ANYCOLOR: 8-bit, BGR for colour files,
    HxW for grey ones), "gray" = IMREAD_GRAYSCALE.  PIL's palette / RGB -> L conversion uses the
    same ITU-R 601 weights as cv2 but its own rounding (label PNGs are single-channel, where
    both are the identity)."""
    from PIL import Image
    with Image.open(path) as im:
        if mode == "gray":
            if im.mode in ("I;16", "I;16B", "I"):
                return (np.asarray(im, dtype=np.uint32) >> 8).astype(np.uint8)
            return np.asarray(im.convert("L"), dtype=np.uint8)
        if im.mode == "L":
            return np.asarray(im, dtype=np.uint8)
        if im.mode in ("I;16", "I;16B", "I"):
            return (np.asarray(im, dtype=np.uint32) >> 8).astype(np.uint8)
        return np.ascontiguousarray(np.asarray(im.convert("RGB"), dtype=np.uint8)[:, :, ::-1])


class RGBXDataset(Dataset):
    """dataloader/RGBXDataset.py:10-73.  Without ``preprocess`` a train item carries the decoded
    uint8 arrays (rgb / modal_x HxWx3 BGR, label HxW) for the GPU TrainPre; with a CPU
    ``preprocess`` callable the item is converted like the reference (float / long tensors)."""

    def __init__(self, setting, split_name, preprocess=None, file_length=None):
        super().__init__()
        self._split_name = split_name
        self._rgb_path = setting["rgb_root"]
        self._rgb_format = setting["rgb_format"]
        self._gt_path = setting["gt_root"]
        self._gt_format = setting["gt_format"]
        self._transform_gt = setting["transform_gt"]
        self._x_path = setting["x_root"]
        self._x_format = setting["x_format"]
        self._x_single_channel = setting["x_single_channel"]
        self._train_source = setting["train_source"]
        self._eval_source = setting["eval_source"]
        self.class_names = setting.get("class_names")
        self._file_names = self._get_file_names(split_name)
        self._file_length = file_length
        self.preprocess = preprocess
        self.dataset_name = setting.get("dataset_name")
        self.background = setting.get("background", 255)
        self.num_classes = setting.get("num_classes")

    def __len__(self):
        return self._file_length if self._file_length is not None else len(self._file_names)

    def _get_file_names(self, split_name):
        assert split_name in ("train", "val")
        source = self._eval_source if split_name == "val" else self._train_source
        with open(source) as f:
            return [line.strip() for line in f.readlines()]

    def _construct_new_file_names(self, length):
        """RGBXDataset.py:91-101: the list repeated, the remainder a random subset."""
        assert isinstance(length, int)
        n = len(self._file_names)
        names = self._file_names * (length // n)
        names += [self._file_names[i] for i in torch.randperm(n).tolist()[:length % n]]
        return names

    def get_length(self):
        return self.__len__()

    @staticmethod
    def _gt_transform(gt):
        return gt - 1

    def __getitem__(self, index):
        # the reference rebuilds the repeated list (a fresh randperm for the remainder) per item (:38-40)
        if self._file_length is not None:
            name = self._construct_new_file_names(self._file_length)[index]
        else:
            name = self._file_names[index]
        rgb = _open_image(os.path.join(self._rgb_path, name + self._rgb_format), "color")
        if rgb.ndim == 2:                                  # cv2.COLOR_GRAY2RGB (:48-49)
            rgb = np.repeat(rgb[:, :, None], 3, axis=2)
        gt = _open_image(os.path.join(self._gt_path, name + self._gt_format), "gray")
        if self._transform_gt:
            gt = self._gt_transform(gt)
        if self._x_single_channel:                         # cv2.merge([x, x, x]) (:56-58)
            x = _open_image(os.path.join(self._x_path, name + self._x_format), "gray")
            x = np.repeat(x[:, :, None], 3, axis=2)
        else:
            x = _open_image(os.path.join(self._x_path, name + self._x_format), "color")
            if x.ndim == 2:
                x = np.repeat(x[:, :, None], 3, axis=2)
        if self.preprocess is not None:
            rgb, gt, x = self.preprocess(rgb, gt, x)
            if self._split_name == "train":
                rgb = torch.from_numpy(np.ascontiguousarray(rgb)).float()
                gt = torch.from_numpy(np.ascontiguousarray(gt)).long()
                x = torch.from_numpy(np.ascontiguousarray(x)).float()
        return dict(data=rgb, label=gt, modal_x=x, fn=str(name), n=len(self._file_names))


def _raw_collate(items):
    return items


class GPUAugmentLoader:
    """Iterates a DataLoader of raw uint8 items and yields the reference's minibatch dicts with
    ``data`` / ``label`` / ``modal_x`` already augmented on the device (augment.TrainPre)."""

    def __init__(self, loader: DataLoader, pre):
        self.loader = loader
        self.pre = pre
        self.sampler = loader.sampler

    def __len__(self):
        return len(self.loader)

    def __iter__(self):
        for items in self.loader:
            # host arrays go straight into TrainPre.batch's reused pinned staging buffer: one
            # host-to-device copy and one launch per augmentation stage for the whole minibatch
            samples = [tuple(it[k] for k in ("data", "label", "modal_x")) for it in items]
            rgb, gt, x = self.pre.batch(samples)
            yield dict(data=rgb, label=gt, modal_x=x, fn=[it["fn"] for it in items], n=items[0]["n"])


def data_setting(config) -> dict:
    """dataloader.py:130-144."""
    return {"rgb_root": config.rgb_root_folder, "rgb_format": config.rgb_format, "gt_root": config.gt_root_folder,
            "gt_format": config.gt_format, "transform_gt": config.gt_transform, "x_root": config.x_root_folder,
            "x_format": config.x_format, "x_single_channel": config.x_is_single_channel,
            "class_names": getattr(config, "class_names", None), "train_source": config.train_source,
            "eval_source": config.eval_source, "dataset_name": getattr(config, "dataset_name", None),
            "background": config.background, "num_classes": config.num_classes}


def get_train_loader(engine, dataset, config):
    batch_size = int(config.batch_size)
    sampler = None
    shuffle = True
    pre = None
    if isinstance(dataset, type):           # the reference passes the Dataset class (train.py:45)
        from .augment import TrainPre
        dataset = dataset(data_setting(config), "train", None, int(config.batch_size * config.niters_per_epoch))
        # the draws follow torch's seed like the reference's worker-seeded `random`
        # (train.py --seed -> torch.manual_seed): one generator per rank
        import random
        rank = torch.distributed.get_rank() if engine.distributed else 0
        rng = random.Random(torch.initial_seed() * 1000003 + rank)
        pre = TrainPre(config.norm_mean, config.norm_std, config.num_classes, config.image_height,
                       config.image_width, getattr(config, "train_scale_array", None), config.background, rng=rng)
    if engine.distributed:
        sampler = DistributedSampler(dataset)
        batch_size = batch_size // engine.world_size
        shuffle = False
    if pre is not None:
        loader = DataLoader(dataset, batch_size=batch_size, num_workers=int(getattr(config, "num_workers", 0)),
                            drop_last=True, shuffle=shuffle, sampler=sampler, collate_fn=_raw_collate)
        return GPUAugmentLoader(loader, pre), sampler
    loader = DataLoader(dataset, batch_size=batch_size, num_workers=int(getattr(config, "num_workers", 0)),
                        drop_last=True, shuffle=shuffle, pin_memory=torch.cuda.is_available(), sampler=sampler)
    return loader, sampler
