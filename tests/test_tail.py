"""CPU: the training-step tail and LR schedule of main.py, pinned by fixtures
made by running the reference's own train_model / main() (tests/golden/
make_golden_tail.py): the oracle restatement replays them exactly, the host
schedules of nsm_amd reproduce them, and FlatAdamW's checkpoint format is
torch.optim.AdamW's."""
import numpy as np
import pytest
import torch

from oracle import step_tail_ref as T
from util import load


def tail_fixture():
    fx = load("tail_steps")
    E, P = int(fx["meta/epochs"]), int(fx["meta/per_epoch"])
    nparam = len([k for k in fx if k.startswith("init/")])
    steps = []
    for b in range(E * P):
        grads = [torch.from_numpy(fx[f"g/{b}/{i}"].copy()) for i in range(nparam)]
        severe = any(((torch.isnan(g) | torch.isinf(g)).sum().item() / g.numel()) > 0.2
                     for g in grads)
        noise = T.replay_noise(torch.from_numpy(fx[f"rng/{b}"]), grads, severe)
        steps.append((b // P, grads, noise))
    return fx, E, P, nparam, steps


def test_oracle_tail_replays_reference_train_model():
    fx, E, P, nparam, steps = tail_fixture()
    params = [torch.nn.Parameter(torch.from_numpy(fx[f"init/{i}"].copy())) for i in range(nparam)]
    opt = torch.optim.AdamW(params, lr=float(fx["meta/base_lr"]), weight_decay=float(fx["meta/wd"]))
    sched = torch.optim.lr_scheduler.LambdaLR(opt, lr_lambda=lambda e: 1.0 / (1.0 + e))
    for b, (epoch, grads, noise) in enumerate(steps):
        for p, g in zip(params, grads):
            p.grad = g.clone()
        skip = T.sanitize_and_clip(params, epoch, E, 1.0, noise)
        assert skip == bool(fx["skipped"][b]), b
        if not skip:
            assert opt.param_groups[0]["lr"] == float(fx[f"lr/{b}"])
            for i, p in enumerate(params):
                assert torch.equal(p.grad, torch.from_numpy(fx[f"step_grad/{b}/{i}"])), (b, i)
            opt.step()
            for i, p in enumerate(params):
                assert torch.equal(p.detach(), torch.from_numpy(fx[f"param/{b}/{i}"])), (b, i)
        opt.zero_grad(set_to_none=True)
        if b % P == P - 1:
            sched.step()
    # the scripted cases really exercise every branch
    assert list(np.nonzero(fx["skipped"])[0]) == [3, 6, 10]


@pytest.mark.parametrize("tag,warm,epochs", [("w5_e200", 5, 200), ("w3_e10", 3, 10), ("w0_e7", 0, 7)])
def test_lr_schedule_matches_reference(tag, warm, epochs):
    import nsm_amd
    from nsm_amd.optim import lr_lambda, make_lambda_lr
    fx = load("lr_schedule")
    ref = fx[f"{tag}/lr"]
    lr0, wd, b1, b2, eps = fx[f"{tag}/hp"].tolist()
    assert ref[0] == (0.0 if warm > 0 else lr0)          # epoch-0 lr is 0
    lam = lr_lambda(warm, epochs)
    assert np.array_equal(np.array([lr0 * lam(e) for e in range(epochs)]), ref)
    # the same sequence through torch's LambdaLR on FlatAdamW (host-side lr)
    ps = [torch.nn.Parameter(torch.zeros(3)), torch.nn.Parameter(torch.zeros(2))]
    opt = nsm_amd.FlatAdamW(ps, lr=lr0, betas=(b1, b2), eps=eps, weight_decay=wd)
    sch = make_lambda_lr(opt, warm, epochs)
    got = []
    for _ in range(epochs):
        got.append(opt.param_groups[0]["lr"])
        sch.step()
    assert np.array_equal(np.array(got), ref)


def test_max_norm_schedule():
    from nsm_amd.optim import max_norm_for
    assert [max_norm_for(e, 10) for e in range(10)] == \
        [1.0] * 5 + [0.5, max(0.1, 1 - 0.6), max(0.1, 1 - 0.7), max(0.1, 1 - 0.8), 0.1]
    for e in range(200):
        assert max_norm_for(e, 200) == T.max_norm_for(e, 200)


def test_flat_adamw_checkpoint_format_is_torch_adamw():
    import nsm_amd
    torch.manual_seed(0)
    ps = [torch.nn.Parameter(torch.randn(4, 3)), torch.nn.Parameter(torch.randn(5))]
    ref_ps = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    ref = torch.optim.AdamW(ref_ps, lr=1e-3, weight_decay=1e-3)
    for p in ref_ps:
        p.grad = torch.randn_like(p)
    ref.step()
    sd = ref.state_dict()
    opt = nsm_amd.FlatAdamW(ps, lr=5.0, weight_decay=0.0)
    opt.load_state_dict(sd)
    assert opt.param_groups[0]["lr"] == 1e-3 and opt.param_groups[0]["weight_decay"] == 1e-3
    assert opt.steps_taken() == 1
    out = opt.state_dict()
    for i in range(2):
        assert torch.equal(out["state"][i]["exp_avg"], sd["state"][i]["exp_avg"])
        assert torch.equal(out["state"][i]["exp_avg_sq"], sd["state"][i]["exp_avg_sq"])
        assert float(out["state"][i]["step"]) == 1.0
    # and it loads back into torch's AdamW
    back = torch.optim.AdamW([torch.nn.Parameter(p.detach().clone()) for p in ps])
    back.load_state_dict(out)
    assert back.param_groups[0]["lr"] == 1e-3
    assert torch.equal(back.state_dict()["state"][1]["exp_avg"], sd["state"][1]["exp_avg"])


def test_fp32_norm_overflow_edge():
    """The oracle's fp32 norm (step_tail_ref.fp32_norm): torch.norm's value below
    the fp32 sum-of-squares overflow, +inf above it (~1.8e19) on every host."""
    g = torch.tensor([3.0, -4.0])
    assert T.fp32_norm(g).item() == torch.norm(g).item() == 5.0
    assert torch.isinf(T.fp32_norm(torch.tensor([1e20, -1e20, 1.0])))
    assert torch.isfinite(T.fp32_norm(torch.tensor([1e19, 1.0])))
