"""The native step replay (native.record / mit_plan_run: the train step's launches recorded once and
re-issued from C++) is the same computation as the eager step: from identical states, eager steps and
recorded + replayed steps give bit-identical losses and parameters (the step is deterministic), with
dropout, the encoder prefetch stream, the weight-gradient side stream and the optimizer in the plan."""
import pytest
import torch

import fixtures as FX
from model_util import build_model

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_replayed_steps_equal_eager_steps(dtype):
    import native
    import optim
    meta, _ = FX.load("tiny_vit_patches")
    imgs, di, tg = [t.cuda() for t in FX.inputs(meta, 0)]
    res = []
    for replay in (False, True):
        m, _ = build_model(meta, dtype, dropout=0.1)
        m.train()
        opt = optim.AdamW(m.parameters(), lr=1e-3)

        def step():
            loss = m.train_step(imgs, di, tg, next_images=imgs)
            opt.step(5.0)
            return loss
        losses = [step().item() for _ in range(2)]  # warm-up: arenas, prefetch steady state
        if replay:
            loss_t = m.decoder.acts(di.shape[0], di.shape[1], 197, True).loss
            progs = []
            for _ in range(2):  # two real steps, recorded (the prefetch alternates two arenas)
                progs.append(native.record(step))
                losses.append(loss_t.item())
            assert progs[0].launches() > 100
            for k in range(4):
                progs[k % 2].run()
                losses.append(loss_t.item())
        else:
            losses += [step().item() for _ in range(6)]
        res.append((losses, m.store.master.clone(), int(opt.step_t.item())))
    (l0, p0, s0), (l1, p1, s1) = res
    assert s0 == s1 == 8
    assert l0 == l1, (l0, l1)
    assert torch.equal(p0, p1)


@pytest.mark.parametrize("kind", ["cpu", "int32"])
def test_record_rejects_token_copies(kind):
    """A step fed CPU or int32 tokens converts them with a device copy / cast kernel inside train_step;
    a replay would not repeat it (it would read the recording run's temporary), so native.record
    raises instead of recording a silently wrong plan."""
    import native
    import optim
    meta, _ = FX.load("tiny_vit_patches")
    imgs, di, tg = [t.cuda() for t in FX.inputs(meta, 0)]
    m, _ = build_model(meta, torch.bfloat16, dropout=0.0)
    m.train()
    opt = optim.AdamW(m.parameters(), lr=1e-3)
    di_bad = di.cpu() if kind == "cpu" else di.to(torch.int32)

    def step():
        m.train_step(imgs, di_bad, tg)
        opt.step(5.0)
    step()
    with pytest.raises(native.NativeError, match="would enqueue GPU work"):
        native.record(step)
    torch.cuda.synchronize()
