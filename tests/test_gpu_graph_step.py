"""GPU: nsm_amd.GraphedTrainStep — the whole training step (forward, loss,
backward, the FlatAdamW device tail of main.py:287-423) replayed from one HIP
graph gives the eager step's results."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _setup(device, p, seed=3, B=2, C=7, H=64):
    import nsm_amd
    torch.manual_seed(seed)
    m = nsm_amd.Unet(in_ch=C, dropout_rate=p).to(device).train()
    opt = nsm_amd.FlatAdamW(m.parameters(), lr=1e-3, weight_decay=1e-3, max_grad_norm=1.0,
                            sanitize=True, seed=11)
    crit = nsm_amd.CustomLoss(device, 0.9, vgg_weights=False)
    g = torch.Generator(device=device).manual_seed(seed)
    x = torch.randn(B, C, H, H, device=device, generator=g)
    y = torch.rand(B, 1, H, H, device=device, generator=g)
    return m, opt, crit, x, y


def _state(m, opt):
    return [t.detach().clone() for t in [opt.flat, opt.exp_avg, opt.exp_avg_sq]
            + list(m.buffers())]


def test_graphed_step_equals_eager_steps(device):
    """Without dropout (no random masks) three replays equal three eager steps
    bitwise: parameters, AdamW moments, BN running statistics; and building the
    step (its warm-up runs real steps) leaves the training state untouched."""
    import nsm_amd
    m, opt, crit, x, y = _setup(device, 0.0)
    m2, opt2, crit2, _, _ = _setup(device, 0.0)
    before = _state(m, opt)
    step = nsm_amd.GraphedTrainStep(m, crit, opt, x, y, warmup=2)
    for a, b in zip(before, _state(m, opt)):
        assert torch.equal(a, b)
    losses = [step().item() for _ in range(3)]
    ref = []
    for _ in range(3):
        loss = crit2(m2(x), y, x)
        loss.backward()
        opt2.step()
        opt2.zero_grad()
        ref.append(loss.item())
    assert losses == ref, (losses, ref)
    for a, b in zip(_state(m, opt), _state(m2, opt2)):
        assert torch.equal(a, b)


def test_graphed_step_draws_new_masks_every_replay(device):
    """Dropout2d masks come from the graph-safe generator: with lr = 0 the
    parameters stay put, so two replays on the same batch differ only by
    their masks (train-mode BN uses the batch statistics)."""
    import nsm_amd
    m, opt, crit, x, y = _setup(device, 0.2)
    opt.param_groups[0]["lr"] = 0.0
    opt.param_groups[0]["weight_decay"] = 0.0
    step = nsm_amd.GraphedTrainStep(m, crit, opt, x, y, warmup=1)
    l1, l2, l3 = step().item(), step().item(), step().item()
    assert len({l1, l2, l3}) == 3, (l1, l2, l3)


def test_graphed_step_recaptures_on_lr_change(device):
    """A new learning rate (the LambdaLR schedule) re-captures: the replay then
    equals an eager step at that rate."""
    import nsm_amd
    m, opt, crit, x, y = _setup(device, 0.0)
    m2, opt2, crit2, _, _ = _setup(device, 0.0)
    step = nsm_amd.GraphedTrainStep(m, crit, opt, x, y, warmup=1)
    step()
    loss = crit2(m2(x), y, x)
    loss.backward()
    opt2.step()
    opt2.zero_grad()
    for o in (opt, opt2):
        o.param_groups[0]["lr"] = 3e-4
    step()
    loss = crit2(m2(x), y, x)
    loss.backward()
    opt2.step()
    opt2.zero_grad()
    for a, b in zip(_state(m, opt), _state(m2, opt2)):
        assert torch.equal(a, b)


def test_graphed_step_range_assert(device):
    """The CustomLoss range assert inside the graph: its sticky device flag is
    read by check_range_now()."""
    import nsm_amd
    m, opt, crit, x, y = _setup(device, 0.0)
    step = nsm_amd.GraphedTrainStep(m, crit, opt, x, y, warmup=1)
    step()
    crit.check_range_now()   # sigmoid output: in range, nothing raised
