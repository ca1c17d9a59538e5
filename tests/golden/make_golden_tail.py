"""Golden fixtures for the training-step tail and the LR schedule, made by
running the REFERENCE's own main.py (/root/reference, read-only) here.

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_tail.py

main.py imports tensorboard, colorama, torchvision, cv2, OpenEXR and Imath,
none of which this image has; they get import-only stubs (nothing on the
step path uses them). Two captures:

1. tail_steps.npz — `main.train_model` (main.py:132-581) itself runs 4 epochs
   x 3 batches on a stub model with 8 parameters (odd sizes, one spanning two
   kernel blocks, a 1-element one). After each backward a post-accumulate hook
   overwrites the gradients with scripted values: clean, NaN/Inf below and
   above the 20 % threshold, norms above 1e3 (the pre-unscale clip). A
   recording AdamW subclass stores the gradient the reference hands to
   `optimizer.step()` and the parameters after it; skipped steps never reach
   it. The RNG state at each loss call is stored so the NaN-repair noise
   (main.py:336) can be replayed.
2. lr_schedule.npz — `main.main()` runs with a scratch config.ini and a tiny
   .npy dataset, `train_model` replaced by a recorder that steps the
   reference's own LambdaLR (main.py:959-969) through all epochs.

The oracle restatement (oracle/step_tail_ref.py) is asserted against both
right here. Fixtures hold inputs and expected outputs only. Never shipped to
or run on the GPU box.
"""
import os
import sys
import tempfile
import types

import numpy as np
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.dont_write_bytecode = True
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

from oracle import step_tail_ref as T  # noqa: E402

SHAPES = [(16, 12, 3, 3), (16,), (32, 16, 1, 1), (37,), (9000,), (4,), (1,), (3, 3)]
EPOCHS, PER_EPOCH = 4, 3
BASE_LR = 1e-2


def install_main_stubs():
    from make_golden import install_stubs
    install_stubs()
    for name in ("cv2", "OpenEXR", "Imath"):
        sys.modules.setdefault(name, types.ModuleType(name))
    tvt = types.ModuleType("torchvision.transforms")
    tvt.transforms = tvt
    sys.modules["torchvision.transforms"] = tvt
    sys.modules["torchvision"].transforms = tvt
    col = types.ModuleType("colorama")
    col.init = lambda *a, **k: None
    col.Fore = types.SimpleNamespace(YELLOW="", RED="", GREEN="", WHITE="", CYAN="", MAGENTA="")
    col.Style = types.SimpleNamespace(RESET_ALL="")
    sys.modules["colorama"] = col
    tb = types.ModuleType("torch.utils.tensorboard")

    class SummaryWriter:
        def __init__(self, *a, **k):
            pass

        def __getattr__(self, name):
            return lambda *a, **k: None

    tb.SummaryWriter = SummaryWriter
    sys.modules["torch.utils.tensorboard"] = tb


def scripted_grads():
    """G[b][i]: the gradient of parameter i at global batch b."""
    rng = np.random.default_rng(2024)
    G = []
    for b in range(EPOCHS * PER_EPOCH):
        scale = {2: 1e-3, 7: 1e-2, 9: 1e4}.get(b, 1.0)
        g = [(rng.standard_normal(s) * 0.05 * scale).astype(np.float32) for s in SHAPES]
        flat = lambda i: g[i].reshape(-1)  # noqa: E731
        if b == 1:        # Inf in P0, NaN in P2: repair
            flat(0)[[3, 50, 700, 701, 1500]] = [np.inf, -np.inf, np.inf, -np.inf, np.inf]
            flat(2)[[0, 10, 511]] = np.nan
        elif b == 3:      # 30 % NaN in P4: severe -> skip
            flat(4)[rng.permutation(9000)[:2700]] = np.nan
        elif b == 4:      # P4 norm ~2.4e3: clipped to 1000 before unscaling
            g[4] *= 500.0
        elif b == 5:      # P3: 3 NaN + 2 Inf of 37 (13.5 %): repair
            flat(3)[[1, 2, 30]] = np.nan
            flat(3)[[5, 36]] = [np.inf, -np.inf]
        elif b == 6:      # P5: 1 Inf of 4 (25 %): severe -> skip
            flat(5)[2] = -np.inf
        elif b == 8:      # NaN in P1 (1/16), -Inf in P7 (1/9): repair
            flat(1)[7] = np.nan
            flat(7)[4] = -np.inf
        elif b == 10:     # P6 is a single NaN: 100 % -> skip
            flat(6)[0] = np.nan
        G.append(g)
    return G


class StubModel(nn.Module):
    def __init__(self):
        super().__init__()
        rng = np.random.default_rng(7)
        for i, s in enumerate(SHAPES):
            setattr(self, f"p{i}", nn.Parameter(torch.from_numpy(
                (rng.standard_normal(s) * 0.1).astype(np.float32))))

    def params(self):
        return [getattr(self, f"p{i}") for i in range(len(SHAPES))]

    def forward(self, x):
        return torch.sigmoid(x[:, :1])


def capture_tail():
    import main as ref_main
    G = scripted_grads()
    model = StubModel()
    state = {"b": -1, "rng": []}

    def hook_for(i):
        def hook(p):
            p.grad.copy_(torch.from_numpy(G[state["b"]][i]))
        return hook

    for i, p in enumerate(model.params()):
        p.register_post_accumulate_grad_hook(hook_for(i))

    class Crit(nn.Module):
        def __init__(self):
            super().__init__()
            self.alpha = 0.9
            self.l1 = nn.L1Loss()

        def forward(self, outputs, labels, inputs):
            state["b"] += 1
            state["rng"].append(torch.get_rng_state().numpy().copy())
            loss = 0.0 * outputs.float().sum()
            for p in model.params():
                loss = loss + p.sum()
            return loss

    records = {}

    class RecAdamW(torch.optim.AdamW):
        def step(self, closure=None):
            b = state["b"]
            rec = {"grad": [p.grad.detach().clone().numpy() for p in model.params()],
                   "lr": self.param_groups[0]["lr"]}
            r = super().step(closure)
            rec["param"] = [p.detach().clone().numpy() for p in model.params()]
            records[b] = rec
            return r

    class Loader:
        batch_size = 2

        def __init__(self):
            g = torch.Generator().manual_seed(3)
            self.batches = [(torch.randn(2, 4, 6, 6, generator=g).requires_grad_(True),
                             torch.rand(2, 1, 6, 6, generator=g)) for _ in range(PER_EPOCH)]

        def __len__(self):
            return len(self.batches)

        def __iter__(self):
            return iter(self.batches)

    init = [p.detach().clone().numpy() for p in model.params()]
    opt = RecAdamW(model.params(), lr=BASE_LR, weight_decay=1e-3)
    sched = torch.optim.lr_scheduler.LambdaLR(opt, lr_lambda=lambda e: 1.0 / (1.0 + e))
    torch.manual_seed(99)
    ref_main.train_model(model, Loader(), None, Crit(), opt, EPOCHS, torch.device("cpu"),
                         os.path.join(os.getcwd(), "best.pth"), sched)

    # oracle replay of the same 12 steps
    omodel = StubModel()
    with torch.no_grad():
        for p, v in zip(omodel.params(), init):
            p.copy_(torch.from_numpy(v))
    oopt = torch.optim.AdamW(omodel.params(), lr=BASE_LR, weight_decay=1e-3)
    osched = torch.optim.lr_scheduler.LambdaLR(oopt, lr_lambda=lambda e: 1.0 / (1.0 + e))
    skipped = []
    worst = 0.0
    for b in range(EPOCHS * PER_EPOCH):
        epoch = b // PER_EPOCH
        grads = [torch.from_numpy(x.copy()) for x in G[b]]
        severe = any(((torch.isnan(g) | torch.isinf(g)).sum().item() / g.numel()) > 0.2
                     for g in grads)
        noise = T.replay_noise(torch.from_numpy(state["rng"][b]), grads, severe)
        for p, g in zip(omodel.params(), grads):
            p.grad = g
        skip = T.sanitize_and_clip(omodel.params(), epoch, EPOCHS, 1.0, noise)
        skipped.append(skip)
        assert skip == (b not in records), (b, skip)
        if not skip:
            for ga, gb in zip(omodel.params(), records[b]["grad"]):
                worst = max(worst, float((ga.grad - torch.from_numpy(gb)).abs().max()))
            oopt.step()
            for pa, pb in zip(omodel.params(), records[b]["param"]):
                worst = max(worst, float((pa.detach() - torch.from_numpy(pb)).abs().max()))
        oopt.zero_grad(set_to_none=True)
        if b % PER_EPOCH == PER_EPOCH - 1:
            osched.step()
    print(f"tail: skipped {[b for b, s in enumerate(skipped) if s]}, oracle max|d| {worst:.3e}")
    assert worst == 0.0, worst

    out = {"meta/epochs": np.array(EPOCHS), "meta/per_epoch": np.array(PER_EPOCH),
           "meta/base_lr": np.array(BASE_LR), "meta/wd": np.array(1e-3),
           "skipped": np.array(skipped)}
    for i, v in enumerate(init):
        out[f"init/{i}"] = v
    for b in range(EPOCHS * PER_EPOCH):
        out[f"rng/{b}"] = state["rng"][b]
        for i in range(len(SHAPES)):
            out[f"g/{b}/{i}"] = G[b][i]
        if b in records:
            out[f"lr/{b}"] = np.array(records[b]["lr"])
            for i in range(len(SHAPES)):
                out[f"step_grad/{b}/{i}"] = records[b]["grad"][i]
                out[f"param/{b}/{i}"] = records[b]["param"][i]
    st = opt.state_dict()["state"]
    for i in range(len(SHAPES)):
        out[f"exp_avg/{i}"] = st[i]["exp_avg"].numpy()
        out[f"exp_avg_sq/{i}"] = st[i]["exp_avg_sq"].numpy()
        out[f"opt_step/{i}"] = np.array(float(st[i]["step"]))
    np.savez_compressed(os.path.join(HERE, "tail_steps.npz"), **out)


def capture_lr(d):
    import main as ref_main
    proc = os.path.join(d, "data", "processed")
    os.makedirs(proc, exist_ok=True)
    rng = np.random.default_rng(1)
    for split in ("train", "val"):
        np.save(os.path.join(proc, f"{split}_inputs.npy"),
                rng.standard_normal((2, 4, 8, 8)).astype(np.float32))
        np.save(os.path.join(proc, f"{split}_labels.npy"), rng.integers(0, 256, (2, 1, 8, 8)) / 255.0)
    np.save(os.path.join(proc, "train_stats.npy"), {"means": [0.0] * 4, "stds": [1.0] * 4})
    out = {}
    for tag, warm, epochs in (("w5_e200", 5, 200), ("w3_e10", 3, 10), ("w0_e7", 0, 7)):
        with open(os.path.join(d, "config.ini"), "w") as f:
            f.write(f"""[base]
batch_size=2
num_epochs={epochs}
learning_rate=0.0007
dropout_rate=0.2
optimizer_type=adamw
warmup_epochs={warm}
perturb_weight=0.1
save_dir=./checkpoints
processed_data_dir = ./data/processed
image_width=8
image_height=8
input_channels=4
output_channels=1
alpha=0.9
loss_type=standard
log_dir=./logs
""")
        seen = {}

        def recorder(model, train_loader, val_loader, criterion, optimizer, num_epochs, device,
                     save_path, scheduler):
            lrs = []
            for _ in range(num_epochs):
                lrs.append(optimizer.param_groups[0]["lr"])
                scheduler.step()
            seen["lrs"] = lrs
            g = optimizer.param_groups[0]
            seen["hp"] = [g["lr"] if False else g["initial_lr"], g["weight_decay"], g["betas"][0],
                          g["betas"][1], g["eps"]]
            seen["type"] = type(optimizer).__name__
            seen["alpha"] = criterion.alpha

        orig = ref_main.train_model
        ref_main.train_model = recorder
        argv = sys.argv
        sys.argv = ["main.py"]
        try:
            ref_main.main()
        finally:
            ref_main.train_model = orig
            sys.argv = argv
        lrs = np.array(seen["lrs"])
        lam = T.lr_lambda(warm, epochs)
        mine = np.array([0.0007 * lam(e) for e in range(epochs)])
        err = float(np.abs(lrs - mine).max())
        print(f"lr {tag}: {seen['type']} hp {seen['hp']} first {lrs[:7].tolist()} oracle max|d| {err:.2e}")
        assert seen["type"] == "AdamW" and err <= 1e-12
        out[f"{tag}/lr"] = lrs
        out[f"{tag}/hp"] = np.array(seen["hp"], dtype=np.float64)
        out[f"{tag}/alpha"] = np.array(seen["alpha"])
    np.savez_compressed(os.path.join(HERE, "lr_schedule.npz"), **out)


if __name__ == "__main__":
    install_main_stubs()
    sys.path.insert(0, REF)
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as d:
        os.chdir(d)  # main.py / setdata.py write logs and checkpoints into CWD
        try:
            import logging
            import main  # noqa: F401  (prints "Using device: cpu")
            logging.getLogger().setLevel(logging.ERROR)
            capture_tail()
            capture_lr(d)
        finally:
            os.chdir(cwd)
