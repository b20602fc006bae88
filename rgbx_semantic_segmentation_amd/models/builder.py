"""Drop-in ``EncoderDecoder`` (reference: models/builder.py:14-253) on MI355X kernels.

API kept from the reference:
  ``EncoderDecoder(cfg, criterion=nn.CrossEntropyLoss(reduction='mean', ignore_index=255),
                   norm_layer=nn.BatchNorm2d)``
  attributes ``backbone``, ``decode_head``, ``criterion``, ``channels``, ``aux_head = None``;
  ``forward(rgb, modal_x, label=None)`` -> 0-dim loss (with autograd graph) if ``label`` is
  given, else fp32 logits (B, K, H, W); ``encode_decode``; ``init_weights``; ``state_dict``
  keys identical to the reference.

Differences by design:
  * ``model.cuda()`` / ``model.to(device)`` flattens the parameters into a ParamStore
    (one fp32 buffer + gradient buffer + bf16 / fp16 shadow); parameters remain ``nn.Parameter``
    views with reference shapes.  There is no CPU execution path: forward on a model that
    was not moved to a GPU raises.
  * Decoder input channels come from the encoder's ``embed_dims`` (the reference's
    hard-coded [96,192,384,768] for mit_b4/b5, builder.py:66-75, cannot run; its mit_b1
    entry builds mit_b0, :84-87).
  * compute dtype: ``cfg.compute_dtype`` ("float32" | "bfloat16" | "float16"); defaults to
    float16 when ``cfg.use_mixed_precision`` (the reference's fp16 autocast switch,
    config.py:61, train.py:185-198: fp16 storage, fp32 accumulation, with dynamic loss scaling
    by optim.GradScaler), else float32.
  * ``backward`` writes parameter gradients straight into the flat gradient buffer
    (overwrite, not accumulate); use the package's ``FusedAdamW``.
"""
from __future__ import annotations

import logging
from typing import Optional

import torch
import torch.nn as nn

from .. import functions as F
from .. import kernels as K
from ..params import ParamStore
from .decoders.MLPDecoder import DecoderHead
from .encoders.dual_segformer import BACKBONES, MIT_SPECS, load_dualpath_model

logger = logging.getLogger("cmx")

PE1_KPAD = 152  # 3*7*7 = 147 padded to a multiple of 8 (16-byte aligned GEMM rows)


def _get(cfg, name, default):
    if cfg is None:
        return default
    if isinstance(cfg, dict):
        return cfg.get(name, default)
    return getattr(cfg, name, default)


def backward_segment(name: str) -> int:
    """Backward-completion segment of a parameter: 0 = decode head + stage 4 (done first),
    1 = stage 3, 2 = stage 2, 3 = stage 1.  A stage's patch embed, blocks, norm, FRM and FFM
    all have their final gradients once the backward has passed that stage's patch embed."""
    import re
    if name.startswith("decode_head.") or name.startswith("aux_head."):
        return 0
    m = re.match(r"backbone\.(?:extra_)?(?:patch_embed|block|norm)(\d)\.", name)
    if m:
        return 4 - int(m.group(1))
    m = re.match(r"backbone\.(?:FRMs|FFMs)\.(\d)\.", name)
    if m:
        return 3 - int(m.group(1))
    return 0


class EncoderDecoder(nn.Module):
    # the forward is one stream-ordered sequence of library launches with no host sync: callers
    # may capture it in a HIP graph (the evaluator does, per crop-batch shape)
    cmx_capturable = True

    def __init__(self, cfg=None, criterion=None, norm_layer=nn.BatchNorm2d):
        super().__init__()
        backbone = _get(cfg, "backbone", "mit_b2")
        if backbone not in BACKBONES:
            raise NotImplementedError(f"backbone {backbone!r}: only the MiT family (mit_b0..b5) is on the "
                                      "CMX hot path")
        decoder = _get(cfg, "decoder", "MLPDecoder")
        if decoder != "MLPDecoder":
            raise NotImplementedError(f"decoder {decoder!r}: only MLPDecoder is on the CMX hot path")
        # config.py:57-58 selects the rectify / fusion blocks (dual_segformer.py:316-329: 'FRM' / 'FFM'
        # the originals, any other value the improved IFRM / IFFM, as there)
        frm = _get(cfg, "feature_rectify_module", "FRM")
        ffm = _get(cfg, "feature_fusion_module", "FFM")
        if criterion is None:
            criterion = nn.CrossEntropyLoss(reduction="mean", ignore_index=int(_get(cfg, "background", 255)))
        if not isinstance(criterion, nn.CrossEntropyLoss) or criterion.reduction != "mean" or \
                criterion.weight is not None or criterion.label_smoothing != 0.0:
            raise NotImplementedError("criterion: only CrossEntropyLoss(reduction='mean') is on the hot path")
        self.cfg = cfg
        self.norm_layer = norm_layer
        self.criterion = criterion
        self.ignore_index = int(criterion.ignore_index)
        self.backbone_name = backbone
        self.channels = list(MIT_SPECS[backbone]["embed_dims"])
        self.backbone = BACKBONES[backbone](norm_fuse=norm_layer, frm=frm, ffm=ffm)
        self.aux_head = None
        self.num_classes = int(_get(cfg, "num_classes", 40))
        self.decode_head = DecoderHead(in_channels=self.channels, num_classes=self.num_classes,
                                       norm_layer=norm_layer, embed_dim=int(_get(cfg, "decoder_embed_dim", 512)))
        self.bn_eps = float(_get(cfg, "bn_eps", 1e-3))
        self.bn_momentum = float(_get(cfg, "bn_momentum", 0.1))
        dt = _get(cfg, "compute_dtype", None)
        if dt is None:
            dt = "float16" if _get(cfg, "use_mixed_precision", False) else "float32"
        self.compute_dtype = {"float32": torch.float32, "fp32": torch.float32, "bfloat16": torch.bfloat16,
                              "bf16": torch.bfloat16, "float16": torch.float16, "fp16": torch.float16}[str(dt)]
        self.sync_bn = norm_layer is nn.SyncBatchNorm
        self.process_group = None
        # DDP's default (train.py:145-146): the BatchNorm running statistics of rank 0 are
        # broadcast at the start of every training forward when a process group is set
        self.broadcast_buffers = True
        self._bnbuf = None
        self.store: Optional[ParamStore] = None
        self.forced_masks = None
        self.init_weights(cfg, pretrained=_get(cfg, "pretrained_model", None))

    # ------------------------------------------------------------------ init / placement
    def init_weights(self, cfg, pretrained=None):
        """builder.py:199-210: optional MiT pretrained load + decoder init_weight."""
        if pretrained:
            logger.info("Loading pretrained model: %s", pretrained)
            load_dualpath_model(self.backbone, pretrained)
        for m in self.decode_head.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_in", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                m.eps, m.momentum = self.bn_eps, self.bn_momentum
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)
        if self.store is not None:
            self.store.refresh_shadow()

    def setup(self, device=None, compute_dtype=None):
        """Move buffers to ``device`` and flatten parameters into the ParamStore."""
        device = torch.device(device if device is not None else "cuda")
        if device.type != "cuda":
            raise RuntimeError("EncoderDecoder runs only on the GPU through libcmx_hip.so (no CPU path)")
        if compute_dtype is not None:
            self.compute_dtype = compute_dtype
        for mod in self.modules():
            for k, b in list(mod._buffers.items()):
                if b is not None:
                    mod._buffers[k] = b.to(device)
        if self.store is None:
            self.store = ParamStore(self, device, self.compute_dtype,
                                    conv_pad={"backbone.patch_embed1.proj.weight": PE1_KPAD,
                                              "backbone.extra_patch_embed1.proj.weight": PE1_KPAD},
                                    segment_of=backward_segment)
        from .. import deferred
        deferred.reserve()          # pinned launch-record tables for captured backward passes
        # every BatchNorm's num_batches_tracked is a view into one counter: one increment per
        # training forward instead of one launch per BN
        bns = [m for m in self.modules() if isinstance(m, nn.modules.batchnorm._BatchNorm)
               and m.num_batches_tracked is not None]
        if bns and getattr(self, "_nbt", None) is None:
            cnt = torch.stack([m.num_batches_tracked.to(device) for m in bns]).contiguous()
            for i, m in enumerate(bns):
                m._buffers["num_batches_tracked"] = cnt[i]
                m._nbt_shared = True
            self._nbt = cnt
        if self._bnbuf is None:      # running statistics as views of one tensor: one broadcast per forward
            from .. import dist as cdist
            self._bnbuf = cdist.flatten_bn_buffers(self, device)
        return self

    def cuda(self, device=None):
        return self.setup(torch.device("cuda", device) if isinstance(device, int) else device)

    def to(self, *args, **kwargs):
        device = kwargs.get("device", args[0] if args else None)
        if isinstance(device, (str, torch.device)) and torch.device(device).type == "cuda":
            return self.setup(device)
        if self.store is not None:
            raise RuntimeError("parameters are flattened on the GPU; .to() other than cuda is not supported")
        return super().to(*args, **kwargs)

    def load_state_dict(self, state_dict, strict=True, assign=False):
        r = super().load_state_dict(state_dict, strict=strict)
        if self.store is not None:
            self.store.refresh_shadow()
        return r

    # ------------------------------------------------------------------ stochastic masks
    def _stochastic(self, B, device):
        """DropPath per-sample scales (n_blocks, 2 [attn, mlp], 2*B) and Dropout2d (B, E)."""
        if not self.training:
            return None, None
        key = (B, str(device))
        cache = self.__dict__.setdefault("_keep_cache", {})
        if key not in cache:   # built once: no host->device copy inside a captured graph
            keep = torch.tensor(self.backbone.drop_path_keep_probs(), dtype=torch.float32)  # (nb, 2 streams)
            cache[key] = keep[:, None, :, None].expand(-1, 2, -1, B).reshape(len(keep), 2, 2 * B).to(device)
        keep = cache[key]
        p = self.decode_head.dropout_ratio
        E = self.decode_head.embed_dim
        if self.forced_masks is not None:
            dp = self.forced_masks["droppath"].to(device=device, dtype=torch.float32)
            d2 = self.forced_masks.get("dropout2d")
            d2 = (d2.to(device=device, dtype=torch.float32) / (1 - p)).contiguous() if (p > 0 and d2 is not None) \
                else None
            return (dp / keep).contiguous(), d2
        # one launch draws both masks (counter-based RNG, step counter on the device, so graph
        # replays draw fresh masks) and bumps num_batches_tracked: cmx_step_masks
        st = self.__dict__.get("_mask_state")
        if st is None or st[1].device != keep.device:
            seed = int(torch.randint(0, 2 ** 62, (1,)).item())       # from torch's host generator
            st = self.__dict__["_mask_state"] = (seed, torch.zeros(1, dtype=torch.int64, device=device))
        dp = torch.empty_like(keep)
        d2 = torch.empty(B, E, device=device) if p > 0 else None
        nbt = getattr(self, "_nbt", None)
        K.call("cmx_step_masks", K.ptr(keep), keep.numel(), K.ptr(dp), B * E if d2 is not None else 0, float(p),
               K.ptr(d2), st[0], K.ptr(st[1]), K.ptr(nbt), nbt.numel() if nbt is not None else 0, K.stream())
        self._nbt_bumped = True
        return dp, d2

    # ------------------------------------------------------------------ forward
    def _logits_lowres(self, rgb, modal_x):
        if self.store is None:
            raise RuntimeError("call model.cuda() first: EncoderDecoder has no CPU execution path")
        B, _, H, W = rgb.shape
        dev = self.store.device
        if self.training and torch.is_grad_enabled() and not torch.cuda.is_current_stream_capturing():
            self.store.ensure_grads()
        rgb = rgb.to(device=dev, dtype=torch.float32).contiguous()
        modal_x = modal_x.to(device=dev, dtype=torch.float32).contiguous()
        images = (rgb, modal_x)            # the stage-1 im2col reads both batches (no concat)
        self._nbt_bumped = False
        pg = self.process_group
        if self.training and self.broadcast_buffers and pg is not None and self._bnbuf is not None:
            import torch.distributed as tdist
            if tdist.get_world_size(pg) > 1:
                from .. import dist as cdist
                cdist.broadcast_buffers(self._bnbuf, pg)
        dp, d2 = self._stochastic(B, dev)
        group = self.process_group if (self.sync_bn and self.training) else None
        if self.training and getattr(self, "_nbt", None) is not None and not self._nbt_bumped:
            self._nbt.add_(1)
        feats, grids = self.backbone.run(self.store, images, B, H, W, self.training, dp)
        logits = self.decode_head.run(self.store, feats, grids, B, self.training, dscale=d2, group=group)
        return logits, grids[0]

    def encode_decode(self, rgb, modal_x):
        logits, (h, w) = self._logits_lowres(rgb, modal_x)
        B, _, H, W = rgb.shape
        return F.upsample_logits_nchw(logits, B, h, w, H, W, self.num_classes)

    def forward(self, rgb, modal_x, label=None):
        if label is None:
            return self.encode_decode(rgb, modal_x)
        logits, (h, w) = self._logits_lowres(rgb, modal_x)
        B, _, H, W = rgb.shape
        label = label.to(device=logits.device, dtype=torch.int64).contiguous()
        return F.UpsampleCEF.apply(logits, label, (B, h, w, H, W, self.num_classes), self.ignore_index)
