"""Diagnostic (GPU box): per-parameter gradient error of the HIP backward vs an
fp64 CPU oracle, in backward order; and the upsample bitwise mismatch report."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "hulk-keypoints_amd"), os.path.join(REPO, "tests")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from oracle import cpu_ref, recipe  # noqa: E402


def grads_report(case):
    from src.model import KeypointsGauss
    from hkp import train
    g = np.load(os.path.join(REPO, "tests/golden/%s.npz" % case))
    bb, k = str(g["backbone"]), int(g["k"])
    dev = torch.device("cuda:0")
    x = recipe.to_tensor_nchw(g["images_u8"])
    uv = g["uv"]
    sd64 = {kk: (v.double() if v.is_floating_point() else v.clone())
            for kk, v in recipe.seeded_state_dict(bb, int(g["wseed"])).items()}
    L64, gr64, _ = cpu_ref.train_step(sd64, x.double(), uv, bb, k)
    sd32 = {kk: v.clone() for kk, v in recipe.seeded_state_dict(bb, int(g["wseed"])).items()}
    L32, gr32, _ = cpu_ref.train_step(sd32, x, uv, bb, k)
    m = KeypointsGauss(k, backbone=bb, pretrained=False)
    m.load_state_dict(recipe.seeded_state_dict(bb, int(g["wseed"])))
    m = m.to(dev)
    t = train.Trainer(m)
    L = t.forward_backward(x.to(dev), uv=torch.from_numpy(uv).to(dev))
    print("%s loss gpu %.12f cpu32 %.12f cpu64 %.12f" % (case, L.item(), L32.item(), L64.item()))
    named = dict(m.named_parameters())
    for n in reversed(list(gr64.keys())):
        ref = gr64[n]
        got = named[n].grad.detach().cpu().double()
        if got.shape != ref.shape:
            got = got.permute(0, 3, 1, 2)
        c32 = gr32[n].double()
        den = ref.abs().max().item() + 1e-30
        print("  %-52s gpu %.2e  cpu32 %.2e" % (n[len("resnet.%s_8s." % bb):], (got - ref).abs().max().item() / den,
                                                (c32 - ref).abs().max().item() / den))


def upsample_report():
    from hkp import ops
    from test_gpu_forward import upsample_emulated, rand
    for (n, k, h, w, H, W) in [(2, 4, 12, 16, 96, 128), (2, 3, 10, 13, 75, 100)]:
        low = rand(n, k, h, w, seed=16)
        raw, _ = ops.upsample_sigmoid(low.cuda(), H, W, heat=True, argmax=False, sigmoid=False)
        emu = upsample_emulated(low, H, W)
        ref = F.interpolate(low, size=(H, W), mode="bilinear", align_corners=True)
        bad = (raw.cpu() != emu)
        print("upsample", (h, w, H, W), "mismatch frac vs emu %.4f vs host-aten %.4f maxdiff %.3g" % (
            bad.float().mean().item(), (raw.cpu() != ref).float().mean().item(), (raw.cpu() - emu).abs().max().item()))
        idx = bad.nonzero()[:5]
        for i in idx.tolist():
            print("   at", i, "gpu %.9g emu %.9g" % (raw.cpu()[tuple(i)].item(), emu[tuple(i)].item()))
        rows = bad.any(-1).any(0).any(0).nonzero().flatten()[:10].tolist()
        cols = bad.any(-2).any(0).any(0).nonzero().flatten()[:10].tolist()
        print("   bad rows", rows, "bad cols", cols)


def calls_report(case):
    """Every backward conv / BN call of one step re-done in fp64 on CPU from the
    GPU call's own inputs: isolates kernel error from forward rounding."""
    from src.model import KeypointsGauss
    from hkp import net, train
    g = np.load(os.path.join(REPO, "tests/golden/%s.npz" % case))
    bb, k = str(g["backbone"]), int(g["k"])
    dev = torch.device("cuda:0")
    m = KeypointsGauss(k, backbone=bb, pretrained=False)
    m.load_state_dict(recipe.seeded_state_dict(bb, int(g["wseed"])))
    m = m.to(dev)
    log = []
    orig_conv, orig_bn = net._conv_backward, net._bn_backward

    def conv_spy(conv, x, dy, grads, need_dx=True, add=None):
        dx = orig_conv(conv, x, dy, grads, need_dx, add)
        log.append(("conv", conv, x, dy, add, dx, grads[conv.weight]))
        return dx

    def bn_spy(bn, gr, out_mask, y, mi, grads, want_dz=False):
        dy, dz = orig_bn(bn, gr, out_mask, y, mi, grads, want_dz)
        log.append(("bn", bn, gr, out_mask, y, mi, dy, grads[bn.weight], grads[bn.bias]))
        return dy, dz

    net._conv_backward, net._bn_backward = conv_spy, bn_spy
    try:
        t = train.Trainer(m)
        t.forward_backward(recipe.to_tensor_nchw(g["images_u8"]).to(dev), uv=torch.from_numpy(g["uv"]).to(dev))
        torch.cuda.synchronize()
    finally:
        net._conv_backward, net._bn_backward = orig_conv, orig_bn
    names = {mod: n for n, mod in m.named_modules()}
    D = torch.float64

    def rel(a, b):
        return ((a.double().cpu() - b).abs().max() / (b.abs().max() + 1e-30)).item()

    for rec in log:
        if rec[0] == "conv":
            _, conv, x, dy, add, dx, dw = rec
            st, pd, dl = (net._i(conv.stride), net._i(conv.padding), net._i(conv.dilation))
            w = conv.weight.detach().double().cpu().permute(0, 3, 1, 2)
            xc = x.double().cpu().permute(0, 3, 1, 2)
            dyc = dy.double().cpu().permute(0, 3, 1, 2)
            rdw = torch.nn.grad.conv2d_weight(xc, w.shape, dyc, st, pd, dl)
            s = "conv %-28s x%s w%s s%d d%d  dw %.2e" % (names[conv], tuple(x.shape), tuple(w.shape), st, dl,
                                                         rel(dw.permute(0, 3, 1, 2), rdw))
            if dx is not None:
                rdx = torch.nn.grad.conv2d_input(xc.shape, w, dyc, st, pd, dl)
                if add is not None:
                    rdx = rdx + add.double().cpu().permute(0, 3, 1, 2)
                s += "  dx %.2e" % rel(dx.permute(0, 3, 1, 2), rdx)
            print(s)
        else:
            _, bn, gr, out_mask, y, mi, dy, dgam, dbet = rec
            c = y.shape[-1]
            gc, yc = gr.double().cpu().reshape(-1, c), y.double().cpu().reshape(-1, c)
            dz = gc * (out_mask.double().cpu().reshape(-1, c) > 0) if out_mask is not None else gc
            mean, inv = mi[:c].double().cpu(), mi[c:].double().cpu()
            xh = (yc - mean) * inv
            n = yc.shape[0]
            db, dgm = dz.sum(0), (dz * xh).sum(0)
            rdy = bn.weight.detach().double().cpu() * inv * (dz - db / n - xh * dgm / n)
            print("bn   %-28s m%d c%d  dy %.2e dgamma %.2e dbeta %.2e" % (names[bn], n, c, rel(dy.reshape(-1, c), rdy),
                                                                        rel(dgam, dgm), rel(dbet, db)))


def two_step_report(case, steps=2):
    """GPU vs CPU-fp32 vs CPU-fp64 over `steps` Adam iterations (reference fit loop)."""
    from src.model import KeypointsGauss
    from hkp import ops
    g = np.load(os.path.join(REPO, "tests/golden/%s.npz" % case))
    bb, k = str(g["backbone"]), int(g["k"])
    dev = torch.device("cuda:0")
    x = recipe.to_tensor_nchw(g["images_u8"])
    uv = g["uv"]
    tr = {}
    for dt in (torch.float32, torch.float64):
        sd = {kk: (v.to(dt) if v.is_floating_point() else v.clone())
              for kk, v in recipe.seeded_state_dict(bb, int(g["wseed"])).items()}
        tr[dt] = cpu_ref.OracleTrainer(sd, bb, k)
    m = KeypointsGauss(k, backbone=bb, pretrained=False)
    m.load_state_dict(recipe.seeded_state_dict(bb, int(g["wseed"])))
    m = m.to(dev)
    opt = torch.optim.Adam(m.parameters(), lr=1e-4, weight_decay=1e-4)
    gt = ops.gauss_target(torch.from_numpy(uv).to(dev), x.shape[2], x.shape[3], 8)
    named = dict(m.named_parameters())
    for s in range(steps):
        L32, g32 = tr[torch.float32].step(x, uv)
        L64, g64 = tr[torch.float64].step(x.double(), uv)
        opt.zero_grad()
        L = torch.nn.BCELoss()(m(x.to(dev)).double(), gt)
        L.backward()
        print("%s step %d loss rel err: gpu %.2e cpu32 %.2e" % (case, s, abs(L.item() - L64.item()) / L64.item(),
                                                               abs(L32.item() - L64.item()) / L64.item()))
        worst = []
        for n, ref in g64.items():
            got = named[n].grad.detach().cpu().double()
            if got.shape != ref.shape:
                got = got.permute(0, 3, 1, 2)
            den = ref.abs().max().item() + 1e-30
            worst.append(((got - ref).abs().max().item() / den, (g32[n].double() - ref).abs().max().item() / den, n))
        worst.sort(reverse=True)
        for w in worst[:4]:
            print("   gpu %.2e cpu32 %.2e  %s" % w)
        # parameter state after the update
        opt.step()
        pw = []
        for n, p in tr[torch.float64].params.items():
            got = named[n].detach().cpu().double()
            if got.shape != p.shape:
                got = got.permute(0, 3, 1, 2)
            d = (got - p.detach()).abs()
            d32 = (tr[torch.float32].params[n].detach().double() - p.detach()).abs()
            pw.append(((d > 1e-5).sum().item(), (d32 > 1e-5).sum().item(), n))
        pw.sort(reverse=True)
        print("   params differing by >1e-5 after step (gpu, cpu32):", pw[:4])


if __name__ == "__main__":
    upsample_report()
    for c in sys.argv[1:] or ["train_r18_k2_64x80"]:
        two_step_report(c)
