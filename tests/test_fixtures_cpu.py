"""The denser gradient pins (tests/golden/<case>.grad_dense.safetensors, make_grad_dense.py) are consistent
with their fixture: the first 64 of each tensor's 1024 pins are the fixture's own 64, bit for bit (same seeded
permutation, same reference step), and every sampled tensor of more than 4096 elements has them."""
import pytest
import torch

import fixtures as FX


@pytest.mark.parametrize("name", ["cfg3_b2_patches", "cfg2_b2_patches"])
def test_dense_pins_extend_the_fixture(name):
    meta, T = FX.load(name)
    dense = FX.load_dense(name)
    assert dense is not None
    sampled = [k for k in FX.trainable_names(meta) if f"grad1.sample.{k}" in T]
    assert sampled and set(sampled) == set(dense)
    for k in sampled:
        idx, vals = dense[k]
        assert len(idx) == len(vals) == 1024 and len(set(idx.tolist())) == 1024
        assert torch.equal(idx[:64], torch.tensor(meta["sample_index"][k]))
        assert torch.equal(vals[:64], T[f"grad1.sample.{k}"])
