"""Host logic of the bench's in-step roofline (roofline.measure_in_step) on a synthetic kernel
trace: complete steps only, family attribution by kernel name, and the timed-step scaling (each
family's time = its share of the traced kernel time x the untraced timed step)."""
import pytest

from rgbx_semantic_segmentation_amd import roofline as R


def _trace(steps, stretch=1.0):
    recs, t = [], 0.0
    for _ in range(steps):
        for name, us in (("step_masks_kernel", 5.0), ("gemm_bf16_kernel<64>", 60.0), ("sra_fwd_fast<bf16>", 20.0),
                         ("adamw_kernel<bf16>", 15.0)):
            recs.append((name, t, us * stretch))
            t += us * stretch
    recs.append(("step_masks_kernel", t, 5.0))          # an incomplete trailing step: dropped
    return recs


@pytest.mark.parametrize("stretch", [1.0, 1.1])
def test_measure_in_step_scales_by_share(monkeypatch, stretch):
    monkeypatch.setattr(R, "trace_kernels", lambda run, steps: _trace(4, stretch))
    shape = dict(backbone="mit_b0", H=64, W=96, B=1, K=9)
    roof, fam = R.measure_in_step(None, "w", shape, 1e6, steps=4, step_us=200.0)
    assert fam["complete_steps_traced"] == 4
    g = fam["families"]["gemm"]
    assert g["share_of_busy"] == pytest.approx(0.6)
    assert g["us_per_step"] == pytest.approx(120.0)                 # 0.6 x 200 us, whatever the stretch
    assert g["profiled_us_per_step"] == pytest.approx(60.0 * stretch)
    assert roof["family"] == "gemm" and roof["total_us"] == pytest.approx(120.0)
    work = R.step_work(n_params=1e6, **shape)["gemm"]
    assert roof["achieved_hbm_gbs"] == pytest.approx(work[1] / 120e-6 / 1e9, rel=1e-3)
    # without a timed step the profiled durations stand
    roof2, fam2 = R.measure_in_step(None, "w", shape, 1e6, steps=4)
    assert fam2["families"]["gemm"]["us_per_step"] == pytest.approx(60.0 * stretch)
