"""bf16 (and fp32) parity of the MI355X path against the reference's golden outputs, per fixture (the
DESIGN.md §6 table), next to the reference's OWN bf16 error (torch.autocast, tests/golden/
bf16_reference_calibration.json). Writes gpurun_out/bf16_parity.json.
Run on the GPU box: python tools/bf16_parity_report.py [case ...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "multimodal-image-transformer_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import torch  # noqa: E402

import fixtures as FX  # noqa: E402
from parity_metrics import case_metrics  # noqa: E402


def main():
    out = {}
    for name in sys.argv[1:] or FX.CASES:
        out[name] = {"bf16": case_metrics(name, torch.bfloat16), "fp32": case_metrics(name, torch.float32)}
        print(name, json.dumps(out[name]), flush=True)
        torch.cuda.empty_cache()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "bf16_parity.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
