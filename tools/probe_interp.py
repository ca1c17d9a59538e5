"""Diagnostic: which fp32 rounding of bilinear(align_corners) lambda does the
host ATen use here, and which does libnsm's resize kernel produce?"""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "pcss-unet_amd"))
import numpy as np, torch, torch.nn.functional as F
print("cpu capability", torch.backends.cpu.get_cpu_capability())


def emu(xn, Hi, Wi, Ho, Wo, mode):
    def idx(inn, outn, o):
        sc = np.float32(inn - 1) / np.float32(outn - 1)
        if mode == "f32":
            src = np.float32(sc * np.float32(o)); i0 = min(int(src), inn - 1); l1 = np.float32(src - np.float32(i0))
        else:
            srcd = np.float64(sc) * o; i0 = min(int(np.float32(srcd)), inn - 1); l1 = np.float32(srcd - i0)
        l1 = min(max(l1, np.float32(0)), np.float32(1)); l0 = np.float32(1) - l1; i1 = i0 + (1 if i0 < inn - 1 else 0)
        return i0, i1, l0, l1
    Y = [idx(Hi, Ho, o) for o in range(Ho)]; X = [idx(Wi, Wo, o) for o in range(Wo)]
    out = np.zeros((Ho, Wo), np.float32)
    for oy, (y0, y1, a0, a1) in enumerate(Y):
        for ox, (x0, x1, b0, b1) in enumerate(X):
            out[oy, ox] = a0 * (b0 * xn[y0, x0] + b1 * xn[y0, x1]) + a1 * (b0 * xn[y1, x0] + b1 * xn[y1, x1])
    return out


for (Hi, Wi, Ho, Wo) in [(67, 120, 134, 240), (134, 240, 135, 240), (64, 64, 32, 32)]:
    torch.manual_seed(0)
    x = torch.randn(1, 1, Hi, Wi)
    ref = F.interpolate(x, size=(Ho, Wo), mode="bilinear", align_corners=True)[0, 0].numpy()
    xn = x[0, 0].numpy()
    e = {m: emu(xn, Hi, Wi, Ho, Wo, m) for m in ("f32", "fma")}
    line = f"{(Hi, Wi, Ho, Wo)} aten-vs-f32 {np.abs(ref - e['f32']).max():.2e} aten-vs-fma {np.abs(ref - e['fma']).max():.2e}"
    if torch.cuda.is_available():
        from nsm_amd import ops
        y = ops.resize(x[0, 0].reshape(Hi * Wi, 1).cuda(), 1, Hi, Wi, Ho, Wo).cpu().numpy().reshape(Ho, Wo)
        g = F.interpolate(x.cuda(), size=(Ho, Wo), mode="bilinear", align_corners=True)[0, 0].cpu().numpy()
        line += f" | nsm-vs-f32 {np.abs(y - e['f32']).max():.2e} nsm-vs-fma {np.abs(y - e['fma']).max():.2e} torchgpu-vs-f32 {np.abs(g - e['f32']).max():.2e} torchgpu-vs-fma {np.abs(g-e['fma']).max():.2e}"
    print(line)
