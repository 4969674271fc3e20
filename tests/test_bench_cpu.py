"""bench.py host logic on CPU: every train workload names an encoder the build knows, and the
algorithmic FLOPs per pair recorded in the committed bench lines follow the SURVEY.md §8d convention
(GEMMs 2MNK, dense attention 4·Lq·Lk·d, train = encoder fwd + 3 × decoder fwd)."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "multimodal-image-transformer_amd"))


def _encoder_flops(spec):
    n_p = (spec["image"] // spec["patch"]) ** 2
    N, e, m = n_p + 1, spec["hidden"], spec["mlp"]
    layer = 2 * N * 4 * e * e + 2 * N * 2 * e * m + 4 * N * N * e
    return spec["layers"] * layer + 2 * n_p * e * 3 * spec["patch"] ** 2, N, e


def _decoder_flops(T, S, d, ff, L, V):
    layer = (2 * T * 3 * d * d + 2 * T * d * d + 4 * T * T * d + 2 * T * d * d + 2 * S * 2 * d * d + 4 * T * S * d
             + 2 * T * d * d + 2 * T * 2 * d * ff)
    return L * layer + 2 * T * d * V


def _pair_gflop(workload, T=63, V=10000):
    import bench
    import config
    enc_name, d, _, L, ff, _ = bench.WORKLOADS[workload]
    enc, S, e = _encoder_flops(config.ENCODER_SPECS[enc_name])
    proj = 2 * S * e * d
    return (enc + 3 * (_decoder_flops(T, S, d, ff, L, V) + proj)) / 1e9


def test_workloads_name_known_encoders():
    import bench
    import config
    for name, (enc, d, heads, layers, ff, label) in bench.WORKLOADS.items():
        assert enc in config.ENCODER_SPECS, name
        assert d % heads == 0 and d // heads == 64, name  # the kernels' head dim
        assert label.startswith("configs["), name


@pytest.mark.parametrize("workload,survey,line", [
    ("train", 50.17, "r01_bench_run.json"),
    ("clip336", 406.37, "r01_bench_clip336_run.json"),
    ("cfg3", 227.66, "r01_bench_cfg3_run.json"),
])
def test_gflop_per_pair_matches_survey(workload, survey, line):
    got = _pair_gflop(workload)
    assert abs(got - survey) < 0.01, (workload, got)
    path = os.path.join(ROOT, "profiles", line)
    if os.path.exists(path):
        with open(path) as f:
            rec = json.load(f)
        assert abs(rec["config"]["gflop_per_pair"] - got) < 0.01
        assert rec["unit"] == "pairs/s" and rec["n_gpus"] >= 1
