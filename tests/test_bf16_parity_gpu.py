"""bf16 parity of the benchmarked (MFMA) path, per golden fixture, against the reference's fp32
outputs AND calibrated against the reference's own bf16 error: the same reference code run under
torch.autocast(bfloat16) (tests/golden/make_bf16_calibration.py -> bf16_reference_calibration.json).

The north star's "logits within 1e-2 bf16" is read as RELATIVE (relative L2 over the pinned logits):
the reference itself, in bf16, is 2.5e-2 .. 4.3e-2 off in max-abs on these fixtures (logit scale ~4),
so no bf16 implementation meets 1e-2 absolute; DESIGN.md §6 has the table. Bounds:
  logits   rel-L2 <= 1e-2 and <= 1.5x the reference-bf16 rel-L2; max-abs <= 1.5x the reference-bf16
           max-abs; argmax identical wherever the reference's top-1/top-2 margin > 5e-2
  encoder  rel-L2 <= 1.75x the reference-bf16 encoder error (the 12-layer ViT towers keep a bf16
           residual stream; autocast's is f32)
  step     loss within 5e-3, pre-clip grad norm within 1 %; per-tensor gradient error RMS / tensor RMS:
           median <= 1.4x reference-bf16 + 0.01, worst tensor <= 1.6x reference-bf16's worst; every
           tensor's norm within 10 %.
  The 24-layer CLIP-L configs (cfg2, cfg3: f32 encoder residual stream) are held tighter: logits
  rel-L2 <= 8e-3, encoder <= 1.3x and worst gradient tensor <= 1.5x the reference's bf16 error
  (measured round 3: 6.8e-3 / 7.4e-3, 1.00x / 0.98x, 1.05x / 1.22x; profiles/r03_bf16_parity.json). Since
  round 6 that worst-tensor bound is taken over 1024 pinned elements per tensor (tests/golden/
  make_grad_dense.py) with the largest 1 % of squared errors left out: over the fixtures' 64 pins a
  handful of elements carried each tensor's value (tools/grad_metric_report.py,
  profiles/r06_grad_metric_report.json).
  Margin: every fixture's logits rel-L2 <= 1.15x the reference's bf16 error and >= 10 %
  under the 1e-2 bound (<= 9e-3). Each case's metrics are written to gpurun_out/parity/<case>.json
  (and printed), so the margin of the tree under test is on record after every GPU run."""
import json
import os

import pytest
import torch

import fixtures as FX

pytestmark = pytest.mark.gpu

CAL = json.load(open(os.path.join(FX.GOLDEN, "bf16_reference_calibration.json")))


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.parametrize("name", FX.CASES)
def test_bf16_within_reference_bf16_envelope(name):
    from parity_metrics import case_metrics
    r = case_metrics(name, torch.bfloat16)
    c = CAL[name]
    print(f"{name}: logits rel {r['logits_rel_l2']:.2e} (ref-bf16 {c['logits_rel_l2']:.2e}) max-abs "
          f"{r['logits_max_abs']:.3f} ({c['logits_max_abs']:.3f}); enc {r['enc_rel_l2']:.2e} ({c['enc_rel_l2']:.2e}); "
          f"grad rms median {r['grad_rms_median']:.3f} ({c['grad_rms_median']:.3f}) max {r['grad_rms_max']:.3f} "
          f"({c['grad_rms_max']:.3f})")
    out = os.path.join(os.path.dirname(FX.GOLDEN), "..", "gpurun_out", "parity")
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, f"{name}.json"), "w") as f:
        json.dump({"ours": r, "reference_bf16": c,
                   "logits_ratio": r["logits_rel_l2"] / c["logits_rel_l2"]}, f, indent=1)
    assert r["logits_rel_l2"] <= 9e-3
    assert r["logits_rel_l2"] <= 1.15 * c["logits_rel_l2"]
    assert r["logits_max_abs"] <= 1.5 * c["logits_max_abs"]
    assert r["argmax_agree_margin_gt_5e-2"] == 1.0
    assert r["enc_rel_l2"] <= 1.75 * c["enc_rel_l2"]
    assert r["step1_loss_abs_err"] <= 5e-3
    assert r["grad_norm_rel_err"] <= 1e-2
    assert r["grad_rms_median"] <= 1.4 * c["grad_rms_median"] + 0.01
    assert r["grad_rms_max"] <= 1.6 * c["grad_rms_max"]
    assert r["grad_norm_rel_err_max"] <= 0.1
    if name.startswith(("cfg2", "cfg3")):  # 24-layer CLIP-L towers, f32 encoder residual stream
        assert r["logits_rel_l2"] <= 8e-3
        assert r["enc_rel_l2"] <= 1.3 * c["enc_rel_l2"]
        # the worst tensor over the 1024 denser pins, 1 % trimmed (round 6, profiles/r06_grad_metric_report.json):
        # on 64 pins one to four elements carry 70-93 % of a tensor's squared error, so the max over ~150
        # tensors jumped 1.3-1.7x under a 1-ulp quick_gelu change; this form moved 0.2-0.9 % under it
        assert r["grad_rms_max_trim"] <= 1.5 * c["grad_rms_max_trim"]
