"""CPU-only tests: the oracle's two restatements agree, the C-ABI library loads and exports
every entry point include/cmx_hip.h declares (no compute without a GPU), host-side logic
(ParamStore layout, state_dict compatibility, FLOP counts, LR policy, optimizer groups)."""
import ctypes
import os

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_oracle_two_restatements_agree_fp64():
    from oracle.cmx_ref import EncoderDecoder, CMXConfig, DropPath
    from oracle import cmx_functional as FN
    torch.manual_seed(0)
    m = EncoderDecoder(CMXConfig(backbone="mit_b0", num_classes=5)).double()
    for n, b in m.named_buffers():
        if "running_mean" in n:
            b.uniform_(-0.1, 0.1)
        if "running_var" in n:
            b.uniform_(0.5, 1.5)
    rgb = torch.randn(2, 3, 64, 96, dtype=torch.float64)
    x = torch.randn(2, 3, 64, 96, dtype=torch.float64)
    m.eval()
    a = m(rgb, x)
    b = FN.forward(m.state_dict(), rgb, x, "mit_b0", "eval")
    assert ((a - b).abs().max() / a.abs().max()).item() < 1e-10
    m.train()
    for _, mod in m.stochastic_modules():
        mod.p = 0.0
    a = m(rgb, x)
    b = FN.forward(m.state_dict(), rgb, x, "mit_b0", "batch")
    assert ((a - b).abs().max() / a.abs().max()).item() < 1e-10


def test_header_symbols_exported():
    from rgbx_semantic_segmentation_amd import _lib
    sigs = _lib.parse_header(os.path.join(ROOT, "include", "cmx_hip.h"))
    assert len(sigs) > 40
    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = [n for n in sigs if not hasattr(lib, n)]
    assert not missing, missing
    assert lib.cmx_abi_version() == _lib.header_abi_version() == 6


def test_abi_rejects_bad_shapes_without_launching():
    """Shape validation happens on the host before any launch."""
    from rgbx_semantic_segmentation_amd import _lib
    st = _lib.LIB.cmx_layernorm_fwd(None, None, None, None, None, None, 10, 1, 30, 1e-5, 1, None)
    assert st == -1 and "layernorm_fwd" in _lib.last_error()
    st = _lib.LIB.cmx_sra_attn_fwd(None, None, None, None, None, 1, 4, 4, 1, 48, 64, 128, 64, 0.1, 1, None)
    assert st == -1
    st = _lib.LIB.cmx_upsample_ce_fwd(None, None, None, None, None, 1, 2, 2, 8, 8, 100, 255, 1, None)
    assert st == -1 and "K=100" in _lib.last_error()


def test_product_state_dict_matches_reference_keys_and_store_layout():
    from oracle.cmx_ref import EncoderDecoder as Ref, CMXConfig
    from rgbx_semantic_segmentation_amd.models.builder import EncoderDecoder, PE1_KPAD
    from rgbx_semantic_segmentation_amd.params import ParamStore
    torch.manual_seed(0)
    ref = Ref(CMXConfig(backbone="mit_b2", num_classes=40))
    m = EncoderDecoder(dict(backbone="mit_b2", num_classes=40))
    assert list(ref.state_dict().keys()) == list(m.state_dict().keys())
    m.load_state_dict(ref.state_dict())
    st = ParamStore(m, "cpu", torch.float32, conv_pad={"backbone.patch_embed1.proj.weight": PE1_KPAD,
                                                       "backbone.extra_patch_embed1.proj.weight": PE1_KPAD})
    sd = m.state_dict()
    for k, v in ref.state_dict().items():
        assert torch.equal(sd[k], v), k
    # modality pairs are stacked views
    q = m.backbone.block3[2].attn.q.weight
    assert torch.equal(st.w(q)[1], ref.backbone.extra_block3[2].attn.q.weight)
    kv = m.backbone.FFMs[1].cross.cross_attn.kv1.weight
    assert torch.equal(st.w(kv)[1], ref.backbone.FFMs[1].cross.cross_attn.kv2.weight)
    # gradients are views of the flat gradient buffer
    st.grad.fill_(3.0)
    assert all(float(p.grad.max()) == 3.0 for p in m.parameters())
    # all parameters sit 64-aligned pairs; decay flags follow group_weight
    assert st.numel % 64 == 0
    assert sum(p.numel() for p in m.parameters()) == 66581424


def test_flop_counts_match_survey():
    from rgbx_semantic_segmentation_amd.flops import forward_macs_per_image as f
    assert f("mit_b2", 480, 640, 40) == 78201854976
    assert f("mit_b0", 240, 320, 9) == 7134849664
    assert f("mit_b4", 480, 640, 9) == 157630872576
    assert f("mit_b5", 1024, 1024, 19) == 897432223744


def test_lr_policy_matches_reference_formula():
    from rgbx_semantic_segmentation_amd.utils.lr_policy import WarmUpPolyLR
    from oracle.train_ref import WarmUpPolyLR as Ref
    a, b = WarmUpPolyLR(6e-5, 0.9, 29600, 1480), Ref(6e-5, 0.9, 29600, 1480)
    for it in (0, 1, 700, 1479, 1480, 1481, 20000, 29599):
        assert a.get_lr(it) == b.get_lr(it)


def test_synthetic_batch_semantics():
    from rgbx_semantic_segmentation_amd.data import make_batch
    rgb, x, lab = make_batch(2, 64, 80, 40, seed=1)
    assert rgb.shape == (2, 3, 64, 80) and rgb.dtype == torch.float32
    # X is one uint8 plane replicated to 3 channels before the per-channel normalisation
    raw = x * torch.tensor([0.229, 0.224, 0.225])[None, :, None, None] + torch.tensor([0.485, 0.456, 0.406])[None, :, None, None]
    assert torch.allclose(raw[:, 0], raw[:, 1], atol=1e-5) and torch.allclose(raw[:, 1], raw[:, 2], atol=1e-5)
    assert ((lab == 255).sum(dim=(1, 2)) == 625).all()
    v = lab[lab != 255]
    assert v.min() >= 0 and v.max() < 40


def test_encoder_decoder_refuses_cpu_execution():
    from rgbx_semantic_segmentation_amd.models.builder import EncoderDecoder
    m = EncoderDecoder(dict(backbone="mit_b0", num_classes=3))
    with pytest.raises(RuntimeError):
        m(torch.zeros(1, 3, 32, 32), torch.zeros(1, 3, 32, 32))
    with pytest.raises(NotImplementedError):
        EncoderDecoder(dict(backbone="swin_s"))


def test_tune_knobs_roundtrip():
    """cmx_tune sets a launch-policy knob in-process (no GPU needed); unset knobs read -1."""
    from rgbx_semantic_segmentation_amd import kernels as K
    assert K.tune_get("TEST_ONLY_KNOB") == -1
    K.tune("TEST_ONLY_KNOB", 7)
    assert K.tune_get("TEST_ONLY_KNOB") == 7
    K.tune("TEST_ONLY_KNOB", 3)
    assert K.tune_get("TEST_ONLY_KNOB") == 3
    with pytest.raises(Exception):
        K.tune("X" * 40, 1)
