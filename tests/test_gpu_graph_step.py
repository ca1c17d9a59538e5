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


def test_graphed_unet_follows_graphed_train_step(device):
    """A GraphedUnet built before training sees the weights and BN running
    statistics that GraphedTrainStep replays wrote (the replay bumps their
    version counters): its output equals an eager eval forward afterwards."""
    import nsm_amd
    m, opt, crit, x, y = _setup(device, 0.2)
    step = nsm_amd.GraphedTrainStep(m, crit, opt, x, y, warmup=1)
    gu = nsm_amd.GraphedUnet(m, x[:1])
    before = gu(x[:1]).clone()
    for _ in range(3):
        step()
    after = gu(x[:1]).clone()
    m.eval()
    with torch.no_grad():
        ref = m(x[:1])
    m.train()
    assert not torch.equal(before, after)
    torch.testing.assert_close(after, ref, rtol=0, atol=0)


def test_graphed_step_recapture_keeps_sticky_flag(device):
    """A re-capture (warmup=0) with a range check whose flag was never
    allocated: the flag is allocated before the capture, so a replay does not
    re-zero it (it stays sticky) and the step's every-2nd-replay check raises
    after an out-of-range output was seen."""
    import nsm_amd
    from nsm_amd import losses
    m, opt, crit, x, y = _setup(device, 0.0)
    step = nsm_amd.GraphedTrainStep(m, crit, opt, x, y, warmup=1, range_check_every=2)
    crit._range = losses._RangeCheck("CustomLoss")   # no flag yet
    opt.param_groups[0]["lr"] = 5e-4                 # the next call re-captures, warmup=0
    step()
    step()                      # replay 2 checks the flag: in range
    crit._range.flag.fill_(1)   # as if an output had left [0, 1]
    step()
    with pytest.raises(AssertionError):
        step()                  # replay 4 checks: the flag survived replay 3


def test_eager_steps_back_to_back_keep_memory_flat(device):
    """Eager steps queued back to back (the host ahead of the GPU) with the
    weight gradients on the side stream: after the first steps the caching
    allocator reserves no new device memory (the tensors the side stream
    reads are held until the main stream waited for it, not record_stream-ed,
    whose blocks return only once the allocator sees their events complete)."""
    import nsm_amd
    from nsm_amd import unet
    assert unet.WGRAD_STREAM
    m, opt, crit, x, y = _setup(device, 0.2, B=8, H=512)

    def step():
        loss = crit(m(x), y, x)
        loss.backward()
        opt.step()
        opt.zero_grad()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    r0 = torch.cuda.memory_stats()["num_device_alloc"]
    for _ in range(12):        # no synchronisation between the steps
        step()
    torch.cuda.synchronize()
    assert torch.cuda.memory_stats()["num_device_alloc"] == r0


def test_reserve_side_stream_is_the_backward_side_stream(device):
    """nsm_amd.reserve_side_stream (called before init_process_group by DP
    ranks, bench.py) creates and binds the very stream the Unet backward then
    runs its weight gradients on, once per device."""
    import nsm_amd
    from nsm_amd import unet
    s = nsm_amd.reserve_side_stream(device)
    assert unet._wg_streams[torch.device(device)] is s
    assert nsm_amd.reserve_side_stream(device) is s
