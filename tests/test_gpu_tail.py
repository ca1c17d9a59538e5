"""GPU: FlatAdamW(sanitize=True) — the device-side step tail (include/nsm.h
nsm_grad_tail + nsm_adamw_tail) — against the reference's own train_model
(fixture tests/golden/tail_steps.npz, made by tests/golden/make_golden_tail.py):
12 scripted steps over 4 epochs with NaN/Inf repairs, 20 % skips, per-parameter
pre-clip, the max_norm schedule and AdamW, with the repair noise the reference
drew injected."""
import numpy as np
import pytest
import torch

from test_tail import tail_fixture

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _replay(world=1, capture=False):
    import nsm_amd
    fx, E, P, nparam, steps = tail_fixture()
    params = [torch.nn.Parameter(torch.from_numpy(fx[f"init/{i}"].copy()).to(DEV))
              for i in range(nparam)]
    sizes = [p.numel() for p in params]
    opt = nsm_amd.FlatAdamW(params, lr=float(fx["meta/base_lr"]), weight_decay=float(fx["meta/wd"]),
                            max_grad_norm=1.0, sanitize=True, world_size=world)
    gflat = torch.empty(sum(sizes), device=DEV)
    noise = torch.empty_like(gflat)
    off = 0
    for p in params:
        p.grad = gflat[off:off + p.numel()].view_as(p)
        off += p.numel()
    got = {}
    graph = None
    for b, (epoch, grads, nz) in enumerate(steps):
        gflat.copy_(torch.cat([g.reshape(-1) for g in grads]).to(DEV) * world)
        noise.copy_(torch.cat([n.reshape(-1) for n in nz]).to(DEV))
        opt.param_groups[0]["lr"] = float(fx["meta/base_lr"]) / (1.0 + epoch)
        opt.set_epoch(epoch, E)
        if capture:
            # lr / max_norm are launch arguments: capture per epoch, replay within it
            if graph is None or b % P == 0:
                graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph):   # capture does not execute: replay runs it
                    opt.step(noise=noise)
            graph.replay()
        else:
            opt.step(noise=noise)
        torch.cuda.synchronize()
        got[b] = (opt.last_flags(), [p.detach().cpu().numpy().copy() for p in params])
    return fx, opt, got, nparam, params


@pytest.mark.parametrize("world", [1, 2])
def test_device_tail_matches_reference_train_model(world):
    fx, opt, got, nparam, params = _replay(world)
    worst = 0.0
    for b, (flags, ps) in got.items():
        assert flags["skip"] == int(fx["skipped"][b]), (b, flags)
        if b in (1, 5, 8):
            assert flags["repaired"] == 1, (b, flags)
        if b == 4:
            assert flags["total_norm"] <= 1e3 * 1.0001
        if not fx["skipped"][b]:
            for i in range(nparam):
                ref = fx[f"param/{b}/{i}"]
                err = np.abs(ps[i] - ref).max()
                worst = max(worst, float(err))
                np.testing.assert_allclose(ps[i], ref, rtol=1e-5, atol=2e-6, err_msg=f"step {b} p{i}")
    assert opt.steps_taken() == int(fx["opt_step/0"])
    sd = opt.state_dict()
    for i in range(nparam):
        np.testing.assert_allclose(sd["state"][i]["exp_avg"].cpu().numpy(), fx[f"exp_avg/{i}"],
                                   rtol=1e-4, atol=1e-7)
        np.testing.assert_allclose(sd["state"][i]["exp_avg_sq"].cpu().numpy(), fx[f"exp_avg_sq/{i}"],
                                   rtol=1e-4, atol=1e-10)
    print(f"world {world}: max |param - reference| over 9 steps = {worst:.3e}")


def test_device_tail_is_graph_capturable():
    """No host synchronisation anywhere in the tail: the whole step captures
    into a HIP graph and replays to the same result as eager."""
    _, _, eager, nparam, _ = _replay()
    _, _, graphed, _, _ = _replay(capture=True)
    for b in eager:
        assert eager[b][0]["skip"] == graphed[b][0]["skip"]
        for i in range(nparam):
            assert np.array_equal(eager[b][1][i], graphed[b][1][i]), (b, i)


def test_device_noise_repair_stays_finite_and_close():
    """Without injected noise the device draws its own normals: the repaired
    values must be distributed as mean + N(0,1) * 0.1 std."""
    import nsm_amd
    torch.manual_seed(0)
    p = torch.nn.Parameter(torch.zeros(20000, device=DEV))
    opt = nsm_amd.FlatAdamW([p], lr=1e-3, weight_decay=0.0, max_grad_norm=1e9, sanitize=True)
    g = torch.randn(20000, device=DEV) * 0.01
    bad = torch.randperm(20000, device=DEV)[:500]
    g[bad] = float("nan")
    p.grad = g.clone()
    opt.step()
    fl = opt.last_flags()
    assert fl["repaired"] == 1 and fl["skip"] == 0
    rep = p.grad[bad]
    assert torch.isfinite(rep).all()
    ok = torch.ones(20000, dtype=torch.bool, device=DEV)
    ok[bad] = False
    mu, sd = g[ok].mean(), g[ok].std()
    z = (rep - mu) / (sd * 0.1)
    assert abs(z.mean().item()) < 0.2 and 0.8 < z.std().item() < 1.2


def test_overflowing_norm_steps_like_reference():
    """A gradient whose values are finite but whose norm overflows fp32: the
    reference's pre-unscale clip factor 1/max(1, inf/1000) is 0 (main.py:
    361-365), the parameter's gradient becomes 0 and the step is taken; the
    device tail must decide the same and match the oracle's AdamW step."""
    import nsm_amd
    from oracle.step_tail_ref import sanitize_and_clip
    g0 = torch.tensor([3e38, 3e38, 1.0, -2.0])
    g1 = torch.tensor([0.5, -0.25, 0.125])
    init = [torch.tensor([0.1, -0.2, 0.3, 0.4]), torch.tensor([1.0, 2.0, -1.0])]
    # reference (oracle restatement of main.py:287-423 + torch AdamW)
    ref = [torch.nn.Parameter(t.clone()) for t in init]
    for p, g in zip(ref, (g0, g1)):
        p.grad = g.clone()
    assert not sanitize_and_clip(ref, 0, 200)
    assert torch.equal(ref[0].grad, torch.zeros(4))
    ropt = torch.optim.AdamW(ref, lr=1e-3, weight_decay=1e-3)
    ropt.step()
    # device
    ps = [torch.nn.Parameter(t.clone().to(DEV)) for t in init]
    opt = nsm_amd.FlatAdamW(ps, lr=1e-3, weight_decay=1e-3, max_grad_norm=1.0, sanitize=True,
                            seed=1)
    for p, g in zip(ps, (g0, g1)):
        p.grad = g.clone().to(DEV)
    opt.step()
    fl = opt.last_flags()
    assert fl["skip"] == 0 and fl["nonfinite"] == 0, fl
    assert opt.steps_taken() == 1
    for p, r in zip(ps, ref):
        torch.testing.assert_close(p.detach().cpu(), r.detach(), rtol=1e-6, atol=1e-7)


def test_large_finite_norm_zeroes_like_fp32_norm():
    """A gradient norm of ~1.4e20: above the ~1.8e19 where an fp32 sum of
    squares (torch.norm on the reference's CUDA device, main.py:95) overflows,
    below FLT_MAX. The tail takes the fp32 arithmetic on every host: the norm
    reads +inf, the pre-unscale clip's factor 1/max(1, inf) = 0 zeroes that
    gradient (main.py:361-365) and the step is taken, as the oracle
    (step_tail_ref.fp32_norm) decides."""
    import nsm_amd
    from oracle.step_tail_ref import sanitize_and_clip
    g0 = torch.tensor([1e20, -1e20, 1.0, -2.0])
    g1 = torch.tensor([0.5, -0.25, 0.125])
    assert g0.double().norm().item() > 1.8e19
    init = [torch.tensor([0.1, -0.2, 0.3, 0.4]), torch.tensor([1.0, 2.0, -1.0])]
    ref = [torch.nn.Parameter(t.clone()) for t in init]
    for p, g in zip(ref, (g0, g1)):
        p.grad = g.clone()
    assert not sanitize_and_clip(ref, 0, 200)
    assert ref[0].grad.abs().max().item() == 0      # zeroed by the clip
    assert ref[1].grad.abs().max().item() > 0
    ropt = torch.optim.AdamW(ref, lr=1e-3, weight_decay=1e-3)
    ropt.step()
    ps = [torch.nn.Parameter(t.clone().to(DEV)) for t in init]
    opt = nsm_amd.FlatAdamW(ps, lr=1e-3, weight_decay=1e-3, max_grad_norm=1.0, sanitize=True,
                            seed=1)
    for p, g in zip(ps, (g0, g1)):
        p.grad = g.clone().to(DEV)
    opt.step()
    fl = opt.last_flags()
    assert fl["skip"] == 0 and fl["nonfinite"] == 0, fl
    assert opt.steps_taken() == 1
    for p, r in zip(ps, ref):
        torch.testing.assert_close(p.detach().cpu(), r.detach(), rtol=1e-6, atol=1e-7)


def test_repair_noise_fresh_after_skipped_step():
    """The repair noise is keyed by the tail-call counter: a repaired step that
    is then skipped (post-clip norm > 10, main.py:408-418) does not advance
    the AdamW step, yet the next repair draws different normals."""
    import nsm_amd
    torch.manual_seed(1)
    n = 20000
    p = torch.nn.Parameter(torch.zeros(n, device=DEV))
    opt = nsm_amd.FlatAdamW([p], lr=1e-3, weight_decay=0.0, max_grad_norm=1e9, sanitize=True,
                            seed=7)
    G = torch.randn(n, device=DEV) * 100.0      # norm ~1.4e4: rescaled to 1e3, still > 10
    bad = torch.randperm(n, device=DEV)[:300]
    G[bad] = float("nan")
    draws = []
    for _ in range(2):
        p.grad = G.clone()
        opt.step()
        fl = opt.last_flags()
        assert fl["repaired"] == 1 and fl["skip"] == 1 and fl["postclip"] == 1, fl
        draws.append(p.grad[bad].clone())
    assert opt.steps_taken() == 0
    assert int(opt._step_dev[1].item()) == 2
    assert (draws[0] != draws[1]).float().mean().item() > 0.99
