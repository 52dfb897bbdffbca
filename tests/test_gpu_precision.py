"""Split-precision fp16 MFMA conv ("f16x3", fp32-accurate) and plain fp16 ("f16",
BASELINE config C4): accuracy vs an fp64 oracle, and full-network parity."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import cpu_ref, recipe

# every live HKP_TILE_* policy past AUTO (7, 8 and 14 are retired)
LIVE_TILES = (1, 2, 3, 4, 5, 6, 9, 10, 11, 13, 15, 16)

pytestmark = pytest.mark.gpu

CASES = [
    (2, 17, 23, 64, 64, 3, 1, 1, 1),
    (2, 30, 40, 64, 128, 3, 2, 1, 1),
    (1, 15, 20, 128, 256, 3, 1, 2, 2),
    (1, 15, 20, 512, 512, 3, 1, 4, 4),     # layer4 shape: K = 4608
    (3, 9, 11, 96, 192, 3, 1, 1, 1),
    (1, 12, 16, 256, 1024, 1, 1, 0, 1),
]


def rand(*shape, seed=0, scale=1.0):
    return torch.randn(*shape, generator=torch.Generator().manual_seed(seed)) * scale


def _unpack_x3(t):
    """packed split [.., C/32, hi32|lo32] → (hi, lo) [.., C] fp16."""
    g = t.reshape(*t.shape[:-1], t.shape[-1] // 64, 2, 32)
    return g[..., 0, :].reshape(*t.shape[:-1], -1), g[..., 1, :].reshape(*t.shape[:-1], -1)


def _bn_stats(part, m):
    """mean | invstd of a conv's BN tile partials (hkp_bn_finalize): compares
    partials of bodies whose tiles group the rows differently (the halo body's
    tiles are 8x32 pixel patches)."""
    from hkp import ops
    c = part.shape[1]
    one = torch.ones(c, device=part.device)
    return ops.bn_finalize(part, m, one, torch.zeros_like(one))[1]


def _pow2(t):
    m, _ = torch.frexp(t)
    return bool((m.abs() == 0.5).all())


def test_producer_split_layouts(cuda_device):
    """bn_apply / bn_relu_maxpool write exactly hi = f16(x), lo = f16(x-hi) in the
    packed layout (split=3) and the fp16 plane (split=1); keep_fp32=False writes the
    same split without the fp32 tensor.  Weight packs scale each output channel by
    a power of two (max -> [2^13, 2^14)) and return the inverse."""
    from hkp import ops
    y = rand(2, 15, 20, 128, seed=11).to(cuda_device)
    ss = torch.cat([rand(128, seed=12) * 0.5 + 1, rand(128, seed=13) * 0.1]).to(cuda_device)
    act = ops.bn_apply(y, ss, relu=True, split=3)
    sp, passes = ops.split_of(act)
    assert passes == 3 and sp.shape == (2, 15, 20, 256)
    hi, lo = _unpack_x3(sp)
    assert torch.equal(hi, act.half())
    assert torch.equal(lo, (act - act.half().float()).half())
    only = ops.bn_apply(y, ss, relu=True, split=3, keep_fp32=False)
    assert only.dtype == torch.float16 and torch.equal(only, sp) and ops.channels_of(only) == 128
    one = ops.bn_apply(y, ss, relu=True, split=1)
    assert torch.equal(ops.split_of(one)[0], act.half())
    pool = ops.bn_relu_maxpool(rand(2, 31, 41, 64, seed=15).to(cuda_device), ss[:64].repeat(2), split=3)
    ph, pl = _unpack_x3(ops.split_of(pool)[0])
    assert torch.equal(ph, pool.half()) and torch.equal(pl, (pool - pool.half().float()).half())
    w = rand(64, 3, 3, 96, seed=16, scale=0.02).to(cuda_device)
    wp = ops.weight_pack_x3(w)
    assert _pow2(wp.inv_scale)
    ws = w / wp.inv_scale.view(-1, 1, 1, 1)                         # exact: power-of-two scale
    mx = ws.abs().amax((1, 2, 3))
    assert bool(((mx >= 2 ** 13) & (mx < 2 ** 14)).all())
    wh, wl = _unpack_x3(wp.split)
    assert torch.equal(wh, ws.half()) and torch.equal(wl, (ws - ws.half().float()).half())
    fp = ops.weight_flip_pack_x3(w)                                 # [C, R, S, 2K], row = input channel
    wf = w.flip(1, 2).permute(3, 1, 2, 0) / fp.inv_scale.view(-1, 1, 1, 1)
    fh, fl = _unpack_x3(fp.split)
    assert _pow2(fp.inv_scale) and torch.equal(fh, wf.half()) and torch.equal(fl, (wf - wf.half().float()).half())


def test_split_residual_and_splitonly_maxpool(cuda_device):
    """bn_apply with a split-only (packed) residual adds exactly hi + lo; the
    split-only maxpool writes the same split as the fp32 one."""
    from hkp import ops
    y = rand(2, 9, 11, 96, seed=21).to(cuda_device)
    ss = torch.cat([rand(96, seed=22) * 0.5 + 1, rand(96, seed=23) * 0.1]).to(cuda_device)
    x = ops.bn_apply(rand(2, 9, 11, 96, seed=24).to(cuda_device), ss, relu=True, split=3, keep_fp32=False)
    hi, lo = _unpack_x3(x)
    got = ops.bn_apply(y, ss, res=x, relu=True, split=3)
    ref = ops.bn_apply(y, ss, res=(hi.float() + lo.float()).contiguous(), relu=True, split=3)
    assert torch.equal(got, ref) and torch.equal(ops.split_of(got)[0], ops.split_of(ref)[0])
    only = ops.bn_apply(y, ss, res=x, relu=True, split=3, keep_fp32=False)
    assert torch.equal(only, ops.split_of(ref)[0])
    yp = rand(2, 31, 41, 64, seed=25).to(cuda_device)
    full = ops.bn_relu_maxpool(yp, ss[:64].repeat(2), split=3)
    sp = ops.bn_relu_maxpool(yp, ss[:64].repeat(2), split=3, keep_fp32=False)
    assert sp.dtype == torch.float16 and torch.equal(sp, ops.split_of(full)[0])


def test_weight_pack_batch_bitexact(cuda_device):
    """hkp_weight_pack_x3_batch == the per-conv packs, bit for bit: 1x1 and 3x3,
    (tap, k) row counts off the 256-row tile, K = 2048 (many column partials),
    rows longer than the register-held 5120 floats, > 32 jobs (several launches),
    reuse of output buffers."""
    from hkp import ops
    shapes = [(64, 3, 3, 64), (128, 3, 3, 64), (64, 1, 1, 256), (2048, 1, 1, 512), (256, 3, 3, 1024),
              (96, 3, 3, 128), (512, 3, 3, 512), (128, 1, 1, 64)]
    ws = [rand(*s, seed=40 + i, scale=10.0 ** (i % 5 - 3)).to(cuda_device) for i, s in enumerate(shapes)]
    ws[2][5].zero_()                                   # an all-zero filter: scale 1
    items = []
    for i in range(40):
        w = ws[i % len(ws)]
        kind = "flip_x3" if (i % 3 == 1 and w.shape[-1] % 64 == 0) else "x3"
        items.append((kind, w))
    got = ops.weight_pack_x3_batch(items)
    for (kind, w), g in zip(items, got):
        ref = ops.weight_flip_pack_x3(w) if kind == "flip_x3" else ops.weight_pack_x3(w)
        assert torch.equal(g.split, ref.split) and torch.equal(g.inv_scale, ref.inv_scale), (kind, tuple(w.shape))
    for w in ws:
        w.mul_(-3.0)
    again = ops.weight_pack_x3_batch(items, got)
    for (kind, w), g, o in zip(items, again, got):
        assert g.split.data_ptr() == o.split.data_ptr()
        ref = ops.weight_flip_pack_x3(w) if kind == "flip_x3" else ops.weight_pack_x3(w)
        assert torch.equal(g.split, ref.split) and torch.equal(g.inv_scale, ref.inv_scale), (kind, tuple(w.shape))


X3_CASES = CASES + [
    (3, 13, 17, 64, 64, 3, 1, 1, 1),        # M = 663: ragged last 256-row tile (and 128-row half)
    (2, 31, 41, 64, 128, 1, 2, 0, 1),       # 1x1 stride-2 downsample
    (1, 9, 14, 32, 192, 3, 1, 2, 2),        # C = 32 (one channel group), K = 192 (BN 64)
    (2, 11, 13, 64, 256, 3, 1, 1, 1),       # 256x256 tiles, ragged M, C = 64
    (2, 16, 64, 64, 64, 3, 1, 1, 1),        # halo tiles (8x32 patches), Cin 64: 2 channel groups
    (1, 24, 96, 128, 128, 3, 1, 1, 1),      # halo tiles, 4 channel groups, 2 column tiles
]


@pytest.mark.parametrize("case", X3_CASES)
def test_x3_conv_fp32_accurate(cuda_device, case):
    """The deep-pipelined packed-operand conv: fp32-class vs fp64, BN partials as the
    fp32 kernel's, every kernel body (hkp_conv_desc.tile: 256x256, 256x128 with
    16x16x32 / 32x32x16 MFMAs, 256x64 pairs, stream-K) agrees to fp32 summation
    order, and stats=False gives the same output."""
    from hkp import ops
    n, h, w, cin, cout, k, st, pad, dil = case
    x = F.relu(rand(n, h, w, cin, seed=21))
    wt = rand(cout, k, k, cin, seed=22, scale=(2.0 / (k * k * cout)) ** 0.5)
    ref = F.conv2d(x.permute(0, 3, 1, 2).double(), wt.permute(0, 3, 1, 2).double(), None, st, pad, dil)
    d = cuda_device
    ss = torch.cat([torch.ones(cin), torch.zeros(cin)]).to(d)
    xs = ops.bn_apply(x.to(d), ss, relu=False, split=3, keep_fp32=False)      # identity BN → split of x
    wp = ops.weight_pack_x3(wt.to(d))
    y, p = ops.conv2d_fwd_x3(xs, wp, st, pad, dil)
    scale = ref.abs().max().item()
    err = (y.cpu().double().permute(0, 3, 1, 2) - ref).abs().max().item() / scale
    assert err < 2e-6, err
    y32, p32 = ops.conv2d_fwd(x.to(d), wt.to(d), st, pad, dil)
    m = y.numel() // cout
    assert torch.allclose(_bn_stats(p, m), _bn_stats(p32, m), rtol=1e-5, atol=1e-6)
    y3, p3 = ops.conv2d_fwd_x3(xs, wp, st, pad, dil, stats=False)
    assert p3 is None and torch.equal(y3, y)
    for tile in LIVE_TILES:
        yv, pv = ops.conv2d_fwd_x3(xs, wp, st, pad, dil, tile=tile)
        # every tile / stream-K variant is fp32-class vs fp64 (stream-K sums K
        # segments at the end, so variants differ by fp32 summation order)
        assert (yv.cpu().double().permute(0, 3, 1, 2) - ref).abs().max().item() < 2e-6 * scale, tile
        assert torch.allclose(_bn_stats(pv, m), _bn_stats(p, m), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("case", [c for c in X3_CASES if c[6] == 1 and c[3] % 64 == 0])
@pytest.mark.parametrize("gscale", [1.0, 1e-9])
def test_x3_dgrad_scaled(cuda_device, case, gscale):
    """dgrad on packed scaled dy (split_pack_x3 + conv_x3_kernel, flipped weights with
    per-channel power-of-two scales): fp32-class vs fp64, also for gradients far
    below fp16's normal range."""
    from hkp import ops
    n, h, w, cin, cout, k, st, pad, dil = case
    wt = rand(cout, cin, k, k, seed=5, scale=(2.0 / (k * k * cout)) ** 0.5)
    ho = (h + 2 * pad - dil * (k - 1) - 1) + 1
    wo = (w + 2 * pad - dil * (k - 1) - 1) + 1
    gy = rand(n, cout, ho, wo, seed=6) * gscale
    add = rand(n, cin, h, w, seed=7) * gscale
    ref = torch.nn.grad.conv2d_input((n, cin, h, w), wt.double(), gy.double(), 1, pad, dil) + add.double()
    d = cuda_device
    gy_d = gy.permute(0, 2, 3, 1).contiguous().to(d)
    amax = ops.absmax(gy_d)
    dx = ops.conv2d_bwd_data_x3(ops.split_pack_x3(gy_d, amax),
                                ops.weight_flip_pack_x3(wt.permute(0, 2, 3, 1).contiguous().to(d)),
                                (n, h, w, cin), pad, dil, add=add.permute(0, 2, 3, 1).contiguous().to(d), amax=amax)
    err = (dx.cpu().double().permute(0, 3, 1, 2) - ref).abs().max().item() / ref.abs().max().item()
    assert err < 2e-6, err


STRIDED_CASES = [
    (2, 30, 40, 64, 128, 3, 1),     # R34 layer2.0.conv1 shape class (3x3 s2 p1)
    (1, 31, 41, 64, 128, 3, 1),     # odd H, W: phases of unequal size, last dy row/col half-used
    (2, 30, 40, 64, 128, 1, 0),     # 1x1 s2 downsample: three phases are add-only
    (1, 15, 21, 128, 256, 3, 1),    # R50 layer2 conv2 (3x3 s2), Cout 256
]


@pytest.mark.parametrize("case", STRIDED_CASES)
@pytest.mark.parametrize("gscale", [1.0, 1e-9])
def test_x3_dgrad_strided(cuda_device, case, gscale):
    """stride-2 dgrad as one stride-1 x3 conv per output phase (phase packs from the
    batched packer, kind 2): fp32-class vs fp64, residual addend included."""
    from hkp import ops
    n, h, w, cin, cout, k, pad = case
    wt = rand(cout, cin, k, k, seed=15, scale=(2.0 / (k * k * cout)) ** 0.5)
    ho = (h + 2 * pad - (k - 1) - 1) // 2 + 1
    wo = (w + 2 * pad - (k - 1) - 1) // 2 + 1
    gy = rand(n, cout, ho, wo, seed=16) * gscale
    add = rand(n, cin, h, w, seed=17) * gscale
    ref = torch.nn.grad.conv2d_input((n, cin, h, w), wt.double(), gy.double(), 2, pad, 1) + add.double()
    d = cuda_device
    gy_d = gy.permute(0, 2, 3, 1).contiguous().to(d)
    wk = wt.permute(0, 2, 3, 1).contiguous().to(d)
    amax = ops.absmax(gy_d)
    phs = ops.weight_phase_pack_x3(wk, pad)
    assert sum(p is not None for p in phs) == (4 if k == 3 else 1)
    dx = ops.conv2d_bwd_data_x3_strided(ops.split_pack_x3(gy_d, amax), phs, (n, h, w, cin), tuple(wk.shape), pad,
                                        add=add.permute(0, 2, 3, 1).contiguous().to(d), amax=amax)
    err = (dx.cpu().double().permute(0, 3, 1, 2) - ref).abs().max().item() / ref.abs().max().item()
    assert err < 2e-6, err
    # each phase pack holds exactly the flipped filter's taps of that phase, same scales
    fp = ops.weight_flip_pack_x3(wk)
    fh, fl = _unpack_x3(fp.split)                     # [C, R, S, K], tap (i, j) = w tap (R-1-i, S-1-j)
    for ph, p in enumerate(phs):
        if p is None:
            continue
        assert torch.equal(p.inv_scale, fp.inv_scale)
        ph_h, ph_l = _unpack_x3(p.split)
        rows = [k - 1 - r for r in range(k - 1, -1, -1) if (((ph >> 1) + pad - r) % 2) == 0]
        cols = [k - 1 - s for s in range(k - 1, -1, -1) if (((ph & 1) + pad - s) % 2) == 0]
        assert torch.equal(ph_h, fh[:, rows][:, :, cols]) and torch.equal(ph_l, fl[:, rows][:, :, cols])


WG_X3_CASES = [c for c in X3_CASES if c[4] % 64 == 0] + [
    (2, 7, 9, 64, 64, 3, 1, 1, 1),          # Wo = 9 < 32: a K-step spans several rows/images
    (1, 30, 40, 96, 128, 3, 2, 1, 1),       # stride 2, RSC = 864 (ragged 256-column tile)
    (2, 30, 40, 256, 256, 3, 1, 2, 2),      # 256x256 tile (16-pixel stages), several pixel splits
    (1, 3, 5, 64, 256, 3, 1, 1, 1),         # Cout 256 with Wo = 5 < 16: the KA-128 fallback, one stage
    (1, 30, 40, 96, 256, 3, 2, 1, 1),       # 256x256 tile, RSC 864: column groups past R*S*Cin
    (2, 7, 9, 64, 256, 3, 1, 1, 1),         # Cout 256 with Wo = 9 < 16: the KA-128 fallback wraps rows
    (2, 9, 20, 64, 256, 3, 1, 1, 1),        # 256x256 tile, Wo = 20: 16-pixel stages wrap rows and images
    (2, 96, 128, 64, 64, 3, 1, 1, 1),       # 3 tiles over 24576 pixels: > 16 splits (the 4-wave slab reduce)
    # the halo body (3x3 stride 1 pad 1, C and K 64 / 128, 4x16-pixel patches)
    (3, 8, 16, 64, 64, 3, 1, 1, 1),         # Wo = 16: one patch per row band, images wrap
    (1, 24, 48, 64, 128, 3, 1, 1, 1),       # two K tiles
    (2, 12, 32, 128, 64, 3, 1, 1, 1),       # two channel tiles
    (1, 8, 16, 128, 128, 3, 1, 1, 1),       # 2 patches: fewer pixel ranges than CUs
    (2, 10, 32, 64, 64, 3, 1, 1, 1),        # Ho % 4 != 0: the tiled body
]


def _wg_halo(case):
    n, h, w, cin, cout, k, st, pad, dil = case
    return (k == 3 and st == 1 and pad == 1 and dil == 1 and cin % 64 == 0 and cout % 64 == 0 and cin <= 128
            and cout <= 128 and w % 16 == 0 and h % 4 == 0)


@pytest.mark.parametrize("case", WG_X3_CASES)
@pytest.mark.parametrize("gscale", [1.0, 1e-9])
def test_x3_wgrad_scaled(cuda_device, case, gscale):
    """wgrad on packed operands (transposed LDS reads, split-K over pixels): fp32-class
    accuracy vs fp64, also for gradients far below fp16's normal range."""
    from hkp import ops
    n, h, w, cin, cout, k, st, pad, dil = case
    x = F.relu(rand(n, cin, h, w, seed=8))
    ho = (h + 2 * pad - dil * (k - 1) - 1) // st + 1
    wo = (w + 2 * pad - dil * (k - 1) - 1) // st + 1
    gy = rand(n, cout, ho, wo, seed=9) * gscale
    ref = torch.nn.grad.conv2d_weight(x.double(), (cout, cin, k, k), gy.double(), st, pad, dil)
    d = cuda_device
    xd = x.permute(0, 2, 3, 1).contiguous().to(d)
    gy_d = gy.permute(0, 2, 3, 1).contiguous().to(d)
    xs = ops.split_pack_x3(xd)
    amax = ops.absmax(gy_d)
    dys = ops.split_pack_x3(gy_d, amax)
    dw = ops.conv2d_bwd_filter_x3(xs, dys, (cout, k, k, cin), st, pad, dil, amax=amax)
    err = (dw.cpu().double().permute(0, 3, 1, 2) - ref).abs().max().item() / ref.abs().max().item()
    assert err < 2e-6, err
    # a caller-chosen CU budget (Policy.wgrad_overlap_cus): the same sums over
    # another grouping of pixel ranges (1: a single split)
    # (one split over all M pixels accumulates M terms in fp32 inside one tile:
    # the bound grows like sqrt(M) past 4096 pixels — 24576 pixels: x2.45)
    m_px = n * ho * wo
    for cus in (1, 40, 96):
        dws = ops.conv2d_bwd_filter_x3(xs, dys, (cout, k, k, cin), st, pad, dil, amax=amax, cus=cus)
        e = (dws.cpu().double().permute(0, 3, 1, 2) - ref).abs().max().item() / ref.abs().max().item()
        assert e < 2e-6 * max(1.0, (m_px / 4096) ** 0.5), (cus, e)
        # the observer's symbol query takes the wgrad's CU budget in the same field
        from hkp._lib import HKP_KOP_WGRAD_X3, ConvDesc
        name = ops.kernel_name(ConvDesc(n, h, w, cin, cout, k, k, st, pad, dil, 0, cus), HKP_KOP_WGRAD_X3)
        assert name == "wgrad_x3_halo_kernel" if _wg_halo(case) else name.startswith("wgrad_x3_kernel<"), name
    if _wg_halo(case):
        # the tiled body on the same operands (tile -1): the same bound; the halo
        # body run twice: bit-identical (fixed-order slabs)
        dwt = ops.conv2d_bwd_filter_x3(xs, dys, (cout, k, k, cin), st, pad, dil, amax=amax, cus=-1)
        e = (dwt.cpu().double().permute(0, 3, 1, 2) - ref).abs().max().item() / ref.abs().max().item()
        assert e < 2e-6, e
        assert torch.equal(dw, ops.conv2d_bwd_filter_x3(xs, dys, (cout, k, k, cin), st, pad, dil, amax=amax))


@pytest.mark.parametrize("shape", [(2, 3, 50, 70), (3, 3, 33, 41), (1, 1, 20, 26), (2, 3, 480 // 4, 640 // 4)])
def test_stem_x3_fp32_accurate(cuda_device, shape):
    """f16x3 stem (zero-padded NHWC4 planes, one K-step per filter row): fp32-class
    accuracy vs fp64, BN partials as the fp32 stem kernel's; odd sizes, C < 3."""
    from hkp import ops
    n, c, h, w = shape
    x = torch.rand(*shape, generator=torch.Generator().manual_seed(3))
    wt = rand(64, c, 7, 7, seed=4, scale=(2.0 / (49 * 64)) ** 0.5)
    ref = F.conv2d(x.double(), wt.double(), None, 2, 3)
    xd, wd = x.to(cuda_device), wt.to(cuda_device)
    assert ops.stem_x3_ok(tuple(x.shape), tuple(wt.shape), 2, 3, 1)
    y, part = ops.conv2d_fwd_stem_x3(xd, ops.stem_weight_pack_x3(wd), 64)
    err = (y.cpu().double().permute(0, 3, 1, 2) - ref).abs().max().item() / ref.abs().max().item()
    assert err < 2e-6, err
    y32, p32 = ops.conv2d_fwd(xd, wd, 2, 3, 1, layout="nchw")
    assert torch.allclose(part, p32, rtol=1e-4, atol=1e-3)


def _merged_stats(part, count):
    """Per-channel mean and biased variance merged (fp64, Chan) from conv tile
    partials [tiles][C][2] (sum, M2 about the 128-row tile's mean)."""
    p = part.double().cpu()
    tiles = p.shape[0]
    n_t = torch.full((tiles, 1), 128.0, dtype=torch.float64)
    n_t[-1] = count - 128 * (tiles - 1)
    mean = p[:, :, 0].sum(0) / count
    m2 = (p[:, :, 1] + n_t * (p[:, :, 0] / n_t - mean) ** 2).sum(0)
    return mean, m2 / count


@pytest.mark.parametrize("shape", [(2, 3, 32, 64), (1, 3, 48, 128), (1, 1, 32, 64), (2, 3, 480, 640)])
def test_stem_patch_body(cuda_device, shape):
    """The stem patch body (conv_x3_stem_patch_kernel: patch-divisible outputs, the
    8 x 32 patch's padded input and all 7 weight rows staged once): fp32-class vs
    fp64, the one-tile stem's values to fp32 summation order (HKP_TILE_64_PAIR),
    and the same BN statistics merged from its patch-grouped tile partials."""
    from hkp import ops
    from hkp._lib import HKP_KOP_STEM_X3, HKP_LAYOUT_NCHW, HKP_TILE_64_PAIR, ConvDesc
    n, c, h, w = shape
    assert ops.kernel_name(ConvDesc(n, h, w, c, 64, 7, 7, 2, 3, 1, HKP_LAYOUT_NCHW, 0),
                           HKP_KOP_STEM_X3) == "conv_x3_stem_patch_kernel<0>"
    assert ops.kernel_name(ConvDesc(n, h, w, c, 64, 7, 7, 2, 3, 1, HKP_LAYOUT_NCHW, HKP_TILE_64_PAIR),
                           HKP_KOP_STEM_X3).startswith("conv_x3_kernel<64, true, true")
    x = torch.rand(*shape, generator=torch.Generator().manual_seed(5))
    wt = rand(64, c, 7, 7, seed=6, scale=(2.0 / (49 * 64)) ** 0.5)
    xd, wd = x.to(cuda_device), wt.to(cuda_device)
    wp = ops.stem_weight_pack_x3(wd)
    y, part = ops.conv2d_fwd_stem_x3(xd, wp, 64)                          # straight from the image
    yp, partp = ops.conv2d_fwd_stem_x3(xd, wp, 64, image_direct=False)    # packed planes, then the patch body
    assert torch.equal(y, yp) and torch.equal(part, partp)
    # the uint8 batch (ToTensor fused): image-direct vs packed, bit for bit
    img = (x.permute(0, 2, 3, 1) * 255).round().to(torch.uint8).contiguous().to(cuda_device)
    yu, pu = ops.conv2d_fwd_stem_x3(img, wp, 64)
    yup, pup = ops.conv2d_fwd_stem_x3(img, wp, 64, image_direct=False)
    assert torch.equal(yu, yup) and torch.equal(pu, pup)
    y1, part1 = ops.conv2d_fwd_stem_x3(xd, wp, 64, tile=HKP_TILE_64_PAIR)
    assert (y - y1).abs().max().item() <= 4e-6 * y1.abs().max().item()
    y2, _ = ops.conv2d_fwd_stem_x3(xd, wp, 64)
    assert torch.equal(y, y2)
    count = y.shape[0] * y.shape[1] * y.shape[2]
    (m0, v0), (m1, v1) = _merged_stats(part, count), _merged_stats(part1, count)
    assert torch.allclose(m0, m1, rtol=1e-5, atol=1e-6) and torch.allclose(v0, v1, rtol=1e-4, atol=1e-7)
    if n * h * w <= 2 * 48 * 128:                              # fp64 on the small shapes
        ref = F.conv2d(x.double(), wt.double(), None, 2, 3)
        err = (y.cpu().double().permute(0, 3, 1, 2) - ref).abs().max().item() / ref.abs().max().item()
        assert err < 2e-6, err
        ym = y.cpu().double().reshape(-1, 64)
        assert torch.allclose(m0, ym.mean(0), rtol=1e-5, atol=1e-7)
        assert torch.allclose(v0, ym.var(0, unbiased=False), rtol=1e-4, atol=1e-9)


def _model(bb, k, wseed, dev, precision="f16x3"):
    from src.model import KeypointsGauss
    m = KeypointsGauss(k, backbone=bb, pretrained=False, precision=precision)
    m.load_state_dict(recipe.seeded_state_dict(bb, wseed))
    return m.to(dev)


@pytest.mark.parametrize("case", ["fwd_r18_k2_96x128", "fwd_r34_k4_96x128", "fwd_r34_k4_75x100",
                                  "fwd_r50_k8_96x128", "fwd_r34_k4_480x640"])
def test_f16x3_forward_matches_golden(cuda_device, golden, case):
    g = golden(case)
    bb, k = str(g["backbone"]), int(g["k"])
    m = _model(bb, k, int(g["wseed"]), cuda_device)
    x = recipe.to_tensor_nchw(g["images_u8"]).to(cuda_device)
    with torch.no_grad():
        hm, yx = m.heatmaps_and_keypoints(x)
    assert np.array_equal(yx.cpu().numpy(), g["argmax_yx"])
    if "heat" in g:
        assert np.abs(hm.cpu().numpy() - g["heat"]).max() < 1e-3
    else:
        np.testing.assert_allclose(hm.double().sum(3).cpu().numpy(), g["heat_row_sum"], rtol=1e-4)


HALO_CASES = [(2, 16, 64, 64, 64), (1, 24, 96, 128, 128), (3, 8, 32, 64, 128), (1, 120, 160, 64, 64)]


@pytest.mark.parametrize("case", HALO_CASES)
@pytest.mark.parametrize("prec", ["x3", "f16"])
def test_halo_tiles_equal_pair_body(cuda_device, case, prec):
    """The halo-tile body (8x32 patches, the nine taps read from one staged
    halo image) runs the same MFMAs in the same order as the 256x64 pair body:
    outputs and BN partials bit-identical (forward, both operand layouts), and
    the stride-1 dgrad too; the planner picks it for 64-channel inputs (where it
    measured faster), HKP_TILE_HALO forces it elsewhere."""
    from hkp import ops
    from hkp._lib import HKP_KOP_DGRAD_X3, HKP_KOP_FWD_F16, HKP_KOP_FWD_X3, HKP_TILE_64_PAIR, HKP_TILE_HALO, ConvDesc
    n, h, w, cin, cout = case
    d = cuda_device
    x = F.relu(rand(n, h, w, cin, seed=31)).to(d)
    wt = rand(cout, 3, 3, cin, seed=32, scale=(2.0 / (9 * cout)) ** 0.5).to(d)
    halo = HKP_TILE_HALO
    desc = ConvDesc(n, h, w, cin, cout, 3, 3, 1, 1, 1, 0, 0)
    forced = ConvDesc(n, h, w, cin, cout, 3, 3, 1, 1, 1, 0, halo)
    if prec == "x3":
        assert ops.kernel_name(forced, HKP_KOP_FWD_X3) == "conv_x3_halo_kernel<3>"
        assert (ops.kernel_name(desc, HKP_KOP_FWD_X3) == "conv_x3_halo_kernel<3>") == (cin <= 64)
        ss = torch.cat([torch.ones(cin, device=d), torch.zeros(cin, device=d)])
        xs = ops.bn_apply(x, ss, relu=False, split=3, keep_fp32=False)
        wp = ops.weight_pack_x3(wt)
        y0, p0 = ops.conv2d_fwd_x3(xs, wp, 1, 1, 1, tile=halo)
        y1, p1 = ops.conv2d_fwd_x3(xs, wp, 1, 1, 1, tile=HKP_TILE_64_PAIR)
        ref = F.conv2d(x.permute(0, 3, 1, 2).double(), wt.permute(0, 3, 1, 2).double(), None, 1, 1, 1)
        assert (y0.double().permute(0, 3, 1, 2) - ref).abs().max().item() < 2e-6 * ref.abs().max().item()
        # dgrad (stride 1): dy of Cout channels, flipped weights
        gy = rand(n, h, w, cout, seed=33).to(d)
        amax = ops.absmax(gy)
        dys = ops.split_pack_x3(gy, amax)
        wf = ops.weight_flip_pack_x3(wt)
        add = rand(n, h, w, cin, seed=34).to(d)
        assert ops.kernel_name(forced, HKP_KOP_DGRAD_X3) == "conv_x3_halo_kernel<3>"
        assert (ops.kernel_name(desc, HKP_KOP_DGRAD_X3) == "conv_x3_halo_kernel<3>") == (cout <= 64)
        dx0 = ops.conv2d_bwd_data_x3(dys, wf, (n, h, w, cin), 1, 1, add=add, amax=amax, tile=halo)
        dx1 = ops.conv2d_bwd_data_x3(dys, wf, (n, h, w, cin), 1, 1, add=add, amax=amax, tile=HKP_TILE_64_PAIR)
        assert torch.equal(dx0, dx1)
    else:
        assert ops.kernel_name(forced, HKP_KOP_FWD_F16) == "conv_x3_halo_kernel<1>"
        assert (ops.kernel_name(desc, HKP_KOP_FWD_F16) == "conv_x3_halo_kernel<1>") == (cin <= 64)
        x16 = x.half()
        x16._hkp_split_passes = 1
        wp = ops.weight_pack_f16(wt)
        y0, p0 = ops.conv2d_fwd_f16(x16, wp, 1, 1, 1, tile=halo)
        y1, p1 = ops.conv2d_fwd_f16(x16, wp, 1, 1, 1, tile=HKP_TILE_64_PAIR)
    assert torch.equal(y0, y1)
    # BN partials: the same sums over differently grouped rows (patches vs row
    # runs) -> the same statistics to fp64 merge order
    m = y0.numel() // cout
    assert torch.allclose(_bn_stats(p0, m), _bn_stats(p1, m), rtol=1e-6, atol=1e-7)


def test_f16_forward_close_to_reference(cuda_device, golden):
    """Plain fp16 operands (config C4): heatmaps close, argmax reported not promised."""
    g = golden("fwd_r50_k8_96x128")
    m = _model("resnet50", 8, int(g["wseed"]), cuda_device, precision="f16")
    x = recipe.to_tensor_nchw(g["images_u8"]).to(cuda_device)
    with torch.no_grad():
        hm, yx = m.heatmaps_and_keypoints(x)
    err = np.abs(hm.cpu().numpy() - g["heat"]).max()
    agree = (yx.cpu().numpy() == g["argmax_yx"]).all(-1).mean()
    print("fp16 R50: max heat err %.3g, argmax agreement %.2f" % (err, agree))
    # fp16 operands through 53 train-mode-BN layers: gate at the measured values
    # (round 2: max err 0.057, 13 of 16 argmax (y, x) equal) with a small margin
    assert err < 0.075 and agree >= 0.75


SK_CASES = [
    (1, 240, 320, 64, 128, 3, 1, 1, 1),     # 300 256x128 tiles over 256 CUs: stream-K segments span tiles
    (2, 60, 80, 256, 512, 3, 1, 2, 2),      # layer4 class (dilation 2), 150 m-tiles x 4 column tiles
    (1, 20, 30, 64, 64, 1, 1, 0, 1),        # 3 tiles of two K-steps each (fewer units than CUs)
]


@pytest.mark.parametrize("case", SK_CASES)
def test_x3_stream_k(cuda_device, case):
    """Stream-K x3 conv (HKP_TILE_SK: split tiles x K-steps over one block per CU,
    fixed segment-order fp32 sum) vs one tile per block (HKP_TILE_NO_SK), forward
    and stride-1 dgrad: same values to fp32 summation order, same BN partials,
    deterministic run to run (the arrival counters are left zero)."""
    from hkp import ops
    from hkp._lib import HKP_KOP_FWD_X3, HKP_TILE_NO_SK, HKP_TILE_SK, ConvDesc
    n, h, w, cin, cout, k, st, pad, dil = case
    d = cuda_device
    x = F.relu(rand(n, h, w, cin, seed=31)).to(d)
    wt = rand(cout, k, k, cin, seed=32, scale=(2.0 / (k * k * cout)) ** 0.5).to(d)
    ss = torch.cat([torch.ones(cin), torch.zeros(cin)]).to(d)
    xs = ops.bn_apply(x, ss, relu=False, split=3, keep_fp32=False)
    wp = ops.weight_pack_x3(wt)
    ho, wo = ops.conv_out_hw(h, w, k, k, st, pad, dil)
    gy = rand(n, ho, wo, cout, seed=33).to(d)
    amax = ops.absmax(gy)
    dys = ops.split_pack_x3(gy, amax)
    wfp = ops.weight_flip_pack_x3(wt)
    add = rand(n, h, w, cin, seed=34).to(d)
    assert ops.kernel_name(ConvDesc(n, h, w, cin, cout, k, k, st, pad, dil, 0, HKP_TILE_SK),
                           HKP_KOP_FWD_X3).endswith(", true, 3>")          # really the stream-K body
    out = {}
    for tile in (HKP_TILE_NO_SK, HKP_TILE_SK, HKP_TILE_SK):
        y, p = ops.conv2d_fwd_x3(xs, wp, st, pad, dil, tile=tile)
        dx = ops.conv2d_bwd_data_x3(dys, wfp, (n, h, w, cin), pad, dil, add=add, amax=amax, tile=tile)
        out.setdefault(tile, []).append((y, p, dx))
    (y9, p9, dx9), = out[HKP_TILE_NO_SK]
    (y8, p8, dx8), (y8b, p8b, dx8b) = out[HKP_TILE_SK]
    assert torch.equal(y8, y8b) and torch.equal(p8, p8b) and torch.equal(dx8, dx8b)
    # both fp32-class (each within 2e-6 of fp64, test_x3_conv_fp32_accurate): K
    # segments summed at the end reorder the fp32 sum
    assert (y8 - y9).abs().max().item() <= 4e-6 * y9.abs().max().item()
    assert torch.allclose(p8, p9, rtol=1e-4, atol=1e-3)
    assert (dx8 - dx9).abs().max().item() <= 4e-6 * dx9.abs().max().item()


BODY_CASES = [
    (2, 11, 13, 64, 256, 3, 1, 1, 1),       # ragged M (286 rows: second tile mostly empty)
    (1, 15, 20, 512, 512, 3, 1, 4, 4),      # layer4 class, K = 4608
    (2, 12, 16, 256, 512, 1, 1, 0, 1),      # 1x1 (downsample class)
]


@pytest.mark.parametrize("case", BODY_CASES)
@pytest.mark.parametrize("tile", [3, 4, 5, 6, 9, 10, 11])
def test_x3_tile_bodies_dgrad(cuda_device, case, tile):
    """Every kernel body (256x256 / 256x128 16x16x32 / 256x128 32x32x16 / 256x64
    pairs) on the forward and the stride-1 dgrad with a residual addend:
    fp32-class vs fp64; BN partials agree with the planner's choice."""
    from hkp import ops
    n, h, w, cin, cout, k, st, pad, dil = case
    x = F.relu(rand(n, h, w, cin, seed=61))
    wt = rand(cout, k, k, cin, seed=62, scale=(2.0 / (k * k * cout)) ** 0.5)
    ref = F.conv2d(x.permute(0, 3, 1, 2).double(), wt.permute(0, 3, 1, 2).double(), None, st, pad, dil)
    d = cuda_device
    ss = torch.cat([torch.ones(cin), torch.zeros(cin)]).to(d)
    xs = ops.bn_apply(x.to(d), ss, relu=False, split=3, keep_fp32=False)
    wp = ops.weight_pack_x3(wt.to(d))
    ho, wo = ops.conv_out_hw(h, w, k, k, st, pad, dil)
    gy = rand(n, cout, ho, wo, seed=63)
    add = rand(n, cin, h, w, seed=64)
    dref = torch.nn.grad.conv2d_input((n, cin, h, w), wt.permute(0, 3, 1, 2).double(), gy.double(), 1, pad, dil) \
        + add.double()
    gy_d = gy.permute(0, 2, 3, 1).contiguous().to(d)
    amax = ops.absmax(gy_d)
    dys = ops.split_pack_x3(gy_d, amax)
    wfp = ops.weight_flip_pack_x3(wt.to(d))
    add_d = add.permute(0, 2, 3, 1).contiguous().to(d)
    y3, p3 = ops.conv2d_fwd_x3(xs, wp, st, pad, dil, sk=False)
    y, p = ops.conv2d_fwd_x3(xs, wp, st, pad, dil, sk=False, tile=tile)
    dx = ops.conv2d_bwd_data_x3(dys, wfp, (n, h, w, cin), pad, dil, add=add_d, amax=amax, sk=False, tile=tile)
    scale = ref.abs().max().item()
    assert (y.cpu().double().permute(0, 3, 1, 2) - ref).abs().max().item() < 2e-6 * scale
    assert torch.allclose(p, p3, rtol=1e-4, atol=1e-3)
    err = (dx.cpu().double().permute(0, 3, 1, 2) - dref).abs().max().item() / dref.abs().max().item()
    assert err < 2e-6, err


def test_x3_mf16_policy_large_grid(cuda_device):
    """The 256x128 16x16x32-MFMA body (HKP_TILE_128_MF16) agrees with the 32x32x16
    body (HKP_TILE_128_MF32) to fp32 summation order — forward and stride-1 dgrad —
    and hkp_conv_kernel_name (the observer's symbol) names each; AUTO plans a
    128-wide output that fills a round of 256x128 tiles on the 256x64
    two-blocks-per-CU tiles (round 5) and a one-round grid on the 16x16x32 body."""
    from hkp import ops
    from hkp._lib import HKP_KOP_DGRAD_X3, HKP_KOP_FWD_X3, HKP_TILE_128_MF16, HKP_TILE_128_MF32, ConvDesc
    # 585 tiles; Wo % 32 != 0 keeps the halo body (HKP_TILE_HALO) out of the choice
    n, h, w, cin, cout, k, st, pad, dil = (2, 240, 312, 128, 128, 3, 1, 1, 1)
    d = cuda_device
    x = F.relu(rand(n, h, w, cin, seed=71)).to(d)
    wt = rand(cout, k, k, cin, seed=72, scale=(2.0 / (k * k * cout)) ** 0.5).to(d)
    ss = torch.cat([torch.ones(cin), torch.zeros(cin)]).to(d)
    xs = ops.bn_apply(x, ss, relu=False, split=3, keep_fp32=False)
    wp = ops.weight_pack_x3(wt)
    desc = ConvDesc(n, h, w, cin, cout, k, k, st, pad, dil, 0)
    assert ops.kernel_name(desc, HKP_KOP_FWD_X3) == "conv_x3_kernel<64, false, true, 16, false, 3>"
    assert ops.kernel_name(desc, HKP_KOP_DGRAD_X3) == "conv_x3_kernel<64, false, true, 16, false, 3>"
    one = ConvDesc(2, 120, 150, cin, cout, k, k, st, pad, dil, 0)     # 141 tiles: under one round
    assert ops.kernel_name(one, HKP_KOP_FWD_X3) == "conv_x3_kernel<128, false, false, 16, false, 3>"
    desc.tile = HKP_TILE_128_MF16
    assert ops.kernel_name(desc, HKP_KOP_FWD_X3) == "conv_x3_kernel<128, false, false, 16, false, 3>"
    assert ops.kernel_name(desc, HKP_KOP_DGRAD_X3) == "conv_x3_kernel<128, false, false, 16, false, 3>"
    desc.tile = HKP_TILE_128_MF32
    assert ops.kernel_name(desc, HKP_KOP_FWD_X3) == "conv_x3_kernel<128, false, false, 32, false, 3>"
    gy = rand(n, h, w, cout, seed=73).to(d)
    amax = ops.absmax(gy)
    dys = ops.split_pack_x3(gy, amax)
    wfp = ops.weight_flip_pack_x3(wt)
    y16, p16 = ops.conv2d_fwd_x3(xs, wp, st, pad, dil, tile=HKP_TILE_128_MF16)
    dx16 = ops.conv2d_bwd_data_x3(dys, wfp, (n, h, w, cin), pad, dil, amax=amax, tile=HKP_TILE_128_MF16)
    y32, p32 = ops.conv2d_fwd_x3(xs, wp, st, pad, dil, tile=HKP_TILE_128_MF32)
    dx32 = ops.conv2d_bwd_data_x3(dys, wfp, (n, h, w, cin), pad, dil, amax=amax, tile=HKP_TILE_128_MF32)
    assert (y16 - y32).abs().max().item() <= 4e-6 * y32.abs().max().item()
    assert torch.allclose(p16, p32, rtol=1e-4, atol=1e-3)
    assert (dx16 - dx32).abs().max().item() <= 4e-6 * dx32.abs().max().item()


F16_CASES = [
    (2, 17, 23, 64, 64, 3, 1, 1, 1),
    (2, 30, 40, 64, 128, 3, 2, 1, 1),       # stride 2
    (1, 15, 20, 128, 256, 3, 1, 2, 2),      # dilation 2, 256x256 tiles
    (1, 15, 20, 512, 512, 3, 1, 4, 4),      # layer4 class (dilation 4), K = 4608
    (3, 13, 17, 256, 64, 1, 1, 0, 1),       # 1x1 reduce (bottleneck conv1), 256x64 pairs, ragged M
    (1, 12, 16, 256, 1024, 1, 1, 0, 1),     # 1x1 expand (bottleneck conv3)
    (2, 31, 41, 256, 512, 1, 2, 0, 1),      # 1x1 stride-2 downsample
    (3, 13, 17, 64, 256, 1, 1, 0, 1),       # K = 64 (one K-step: DUO's two half-line stages), ragged M
    (1, 12, 16, 128, 128, 1, 1, 0, 1),      # K = 128, one partly filled tile (DUO: rows past M)
    (2, 9, 11, 192, 384, 3, 1, 2, 2),       # DUO: 3 column tiles, dilated taps at the border
]


@pytest.mark.parametrize("case", F16_CASES)
def test_f16_conv_exact_products(cuda_device, case):
    """Plain-fp16 LDS-DMA conv (config C4): its operands are the fp16 roundings of
    x and of the power-of-two-scaled weights; products of fp16 values are exact in
    fp32, so against an fp64 conv of those same operands only fp32 accumulation
    error and the output's one fp16 rounding remain (every tile body; BN partials
    from the unrounded accumulators)."""
    from hkp import ops
    n, h, w, cin, cout, k, st, pad, dil = case
    x = F.relu(rand(n, h, w, cin, seed=81))
    wt = rand(cout, k, k, cin, seed=82, scale=(2.0 / (k * k * cout)) ** 0.5)
    d = cuda_device
    x16 = x.half().to(d)
    wp = ops.weight_pack_f16(wt.to(d))
    w_eff = (wp.split.double() * wp.inv_scale.double().view(-1, 1, 1, 1)).cpu()     # the weights it multiplies
    ref = F.conv2d(x.half().double().permute(0, 3, 1, 2), w_eff.permute(0, 3, 1, 2), None, st, pad, dil)
    scale = ref.abs().max().item()
    y16, p16 = ops.conv2d_fwd_f16(x16, wp, st, pad, dil)
    assert y16.dtype == torch.float16

    def err_ratio(y):          # fp32 accumulation error + one fp16 rounding of the output
        e = (y.cpu().double().permute(0, 3, 1, 2) - ref).abs()
        return (e / (2.0 ** -11 * ref.abs() + 2e-6 * scale)).max().item()
    assert err_ratio(y16) <= 1.0
    # BN partials (from the fp32 accumulators) as the fp32 conv's on the same fp16-rounded operands
    yr, pr = ops.conv2d_fwd(x.half().float().to(d), w_eff.float().to(d), st, pad, dil)
    assert torch.allclose(p16, pr, rtol=1e-4, atol=1e-3)
    from hkp._lib import HKP_KOP_FWD_F16, HKP_TILE_DUO, ConvDesc
    duo = ops.kernel_name(ConvDesc(n, h, w, cin, cout, k, k, st, pad, dil, 0, HKP_TILE_DUO), HKP_KOP_FWD_F16)
    assert duo == ("conv_x3_duo_kernel<1>" if cout % 128 == 0 else ops.kernel_name(
        ConvDesc(n, h, w, cin, cout, k, k, st, pad, dil, 0, 0), HKP_KOP_FWD_F16))
    for tile in LIVE_TILES:
        yv, pv = ops.conv2d_fwd_f16(x16, wp, st, pad, dil, tile=tile)
        assert err_ratio(yv) <= 1.0, tile
        assert torch.allclose(pv, p16, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("tile", [7, 8, 14])
def test_retired_tile_policies_rejected(cuda_device, tile):
    """Policies 7, 8 (the persistent conv) and 14 (the persistent A3 body), each
    measured slower than the one-tile grid and removed, are rejected with
    HKP_ERR_ARG, not silently re-planned."""
    from hkp import ops
    d = cuda_device
    x16 = torch.ones(1, 8, 8, 64, device=d, dtype=torch.float16)
    wp = ops.weight_pack_f16(torch.ones(64, 1, 1, 64, device=d))
    with pytest.raises(ops.HkpError, match="retired"):
        ops.conv2d_fwd_f16(x16, wp, tile=tile)


TAIL_CASES = [
    # (precision, n, h, w, cin, cout, k, stride, pad, dil): one full round + a split-K tail
    ("x3", 16, 60, 80, 256, 256, 3, 1, 2, 2),      # C2 layer3 class: 300 tiles = 256 + 44 halves
    ("x3", 9, 60, 80, 256, 512, 3, 1, 4, 4),       # two column tiles, 338 tiles, ragged M
    ("f16", 16, 60, 80, 512, 256, 1, 1, 0, 1),     # plain fp16, 8 K-steps per tile
    ("x3", 4, 60, 80, 256, 256, 3, 1, 2, 2),       # 75 tiles, no full round: a tail-only grid (S = 3)
]


@pytest.mark.parametrize("case", TAIL_CASES)
def test_split_k_tail(cuda_device, case):
    """HKP_TILE_256_TAIL: 256x256 tiles, the tiles past the last full round run as
    S split-K segments (conv_x3_tail_kernel, fixed-order sum by the last-arriving
    segment) — the same values as the plain one-tile grid (fp32 summation order),
    the same BN partials, and run to run bit-identical."""
    from hkp import ops
    from hkp._lib import HKP_TILE_256, HKP_TILE_256_A3, HKP_TILE_256_TAIL
    prec, n, h, w, cin, cout, k, st, pad, dil = case
    d = cuda_device
    g = torch.Generator(device=d).manual_seed(9)
    x = torch.relu(torch.randn(n, h, w, cin, device=d, generator=g))
    wt = torch.randn(cout, k, k, cin, device=d, generator=g) * (2.0 / (k * k * cout)) ** 0.5
    if prec == "f16":
        xs, wp, fwd = x.half(), ops.weight_pack_f16(wt), ops.conv2d_fwd_f16
    else:
        ss = torch.cat([torch.ones(cin, device=d), torch.zeros(cin, device=d)])
        xs = ops.bn_apply(x, ss, relu=False, split=3, keep_fp32=False)
        wp, fwd = ops.weight_pack_x3(wt), ops.conv2d_fwd_x3
    y0, p0 = fwd(xs, wp, st, pad, dil, sk=False, tile=HKP_TILE_256)
    tol = 2.0 ** -10 if prec == "f16" else 4e-6
    # 256_TAIL: a second launch (conv_x3_tail_kernel); 256_A3 / AUTO: the A3 kernel
    # with the tail's segments appended to the same launch
    for tile in (HKP_TILE_256_TAIL, HKP_TILE_256_A3, 0):
        y1, p1 = fwd(xs, wp, st, pad, dil, tile=tile)
        y2, _ = fwd(xs, wp, st, pad, dil, tile=tile)
        assert (y1.float() - y0.float()).abs().max().item() <= tol * y0.float().abs().max().item(), tile
        assert torch.allclose(p1, p0, rtol=1e-4, atol=1e-3), tile
        assert torch.equal(y1, y2), tile                       # counters back at zero, fixed order


A3_192_CASES = [
    # (n, h, w, cin, cout, k, stride, pad, dil)
    (8, 60, 80, 256, 256, 3, 1, 2, 2),      # the B=8 shard's layer3: 200 192-row tiles, one round
    (3, 37, 41, 128, 512, 3, 1, 1, 1),      # ragged M (4551 rows: a partial last tile and half tile)
    (2, 30, 40, 512, 256, 1, 1, 0, 1),      # 1x1, 2400 rows
    (1, 9, 11, 256, 256, 3, 2, 1, 1),       # stride 2, one partial tile (30 rows)
    (8, 60, 80, 128, 128, 3, 1, 1, 1),      # the B=8 shard's layer2: 128-wide (160x128 tiles; 192: AUTO)
    (3, 37, 41, 128, 128, 1, 1, 0, 1),      # 128-wide, ragged M
]


@pytest.mark.parametrize("bm", [192, 160])
@pytest.mark.parametrize("case", A3_192_CASES)
def test_a3_192_tiles(cuda_device, case, bm):
    """HKP_TILE_192_A3 / HKP_TILE_160_A3 (conv_x3_a3_192 / _160_kernel: the A3 body on
    192 x 256 / 160 x 256 tiles): every output is the 256-row A3 body's, bit for bit
    (the same MFMA sequence per output element), for f16x3 and both two-product
    sets; the BN partials come per 96- / 80-row tile (ceil(M / rows) of them) and
    finalize to the 128-row tiles' statistics; the stride-1 dgrad (with the
    residual addend) likewise."""
    from hkp import ops
    from hkp._lib import (HKP_KOP_FWD_X3, HKP_TILE_128_MF16, HKP_TILE_160_A3, HKP_TILE_192_A3, HKP_TILE_256_A3,
                          HKP_X3_W16, HKP_X3_X16, ConvDesc)
    tile, rows = (HKP_TILE_192_A3, 96) if bm == 192 else (HKP_TILE_160_A3, 80)
    n, h, w, cin, cout, k, st, pad, dil = case
    d = cuda_device
    g = torch.Generator(device=d).manual_seed(31)
    x = torch.relu(torch.randn(n, h, w, cin, device=d, generator=g))
    wt = torch.randn(cout, k, k, cin, device=d, generator=g) * (2.0 / (k * k * cout)) ** 0.5
    ss = torch.cat([torch.ones(cin, device=d), torch.zeros(cin, device=d)])
    xs = ops.bn_apply(x, ss, relu=False, split=3, keep_fp32=False)
    wp = ops.weight_pack_x3(wt)
    if cout % 256:                       # 128-wide: the 160x128 form; 192 rows plan as AUTO
        if bm == 192:
            return
        tile, ref = HKP_TILE_160_A3, HKP_TILE_128_MF16
        name = "conv_x3_a3_160x128_kernel<3>"
    else:
        ref, name = HKP_TILE_256_A3, "conv_x3_a3_%d_kernel<3>" % bm
    desc = ConvDesc(n, h, w, cin, cout, k, k, st, pad, dil, 0, tile)
    assert ops.kernel_name(desc, HKP_KOP_FWD_X3) == name
    # the 256-row reference without the split-K tail (its segment sums reorder the K loop)
    y0, p0 = ops.conv2d_fwd_x3(xs, wp, st, pad, dil, sk=False, tile=ref)
    y1, p1 = ops.conv2d_fwd_x3(xs, wp, st, pad, dil, tile=tile)
    m = y0.numel() // cout
    assert p1.shape == ((m + rows - 1) // rows, cout, 2) and ops.stat_tile_rows(p1) == rows
    assert torch.equal(y1, y0)
    assert torch.allclose(_bn_stats(p1, m), _bn_stats(p0, m), rtol=1e-6, atol=1e-7)
    for prod in (HKP_X3_W16, HKP_X3_X16):
        a, _ = ops.conv2d_fwd_x3(xs, wp, st, pad, dil, sk=False, tile=ref, products=prod)
        b, _ = ops.conv2d_fwd_x3(xs, wp, st, pad, dil, tile=tile, products=prod)
        assert torch.equal(a, b), prod
    if st == 1:
        gy = torch.randn(n, h, w, cout, device=d, generator=g) * 1e-3
        add = torch.randn(n, h, w, cin, device=d, generator=g) * 1e-3
        amax = ops.absmax(gy)
        dys = ops.split_pack_x3(gy, amax)
        wf = ops.weight_flip_pack_x3(wt)
        dref = HKP_TILE_256_A3 if cin % 256 == 0 else HKP_TILE_128_MF16 if bm == 160 else None
        if dref is not None:                # (dgrad outputs cin channels)
            dx0 = ops.conv2d_bwd_data_x3(dys, wf, (n, h, w, cin), pad, dil, add=add, amax=amax, sk=False,
                                         tile=dref)
            dx1 = ops.conv2d_bwd_data_x3(dys, wf, (n, h, w, cin), pad, dil, add=add, amax=amax, tile=tile)
            assert torch.equal(dx1, dx0)


def test_split_k_tail_dgrad_back_to_back(cuda_device):
    """The overlapped dgrad's policy (HKP_TILE_256_TAIL, with the stream-K
    workspace) on a stride-1 shape whose last round is partial (300 tiles = one
    round + 44 tail tiles in S segments): the tail's arrival counters must return
    to zero and its slabs must not leak into the next launch — two launches back
    to back on one stream give bit-identical dx, equal to the plain grid to fp32
    summation order, and fp32-class vs fp64."""
    from hkp import ops
    from hkp._lib import HKP_KOP_DGRAD_X3, HKP_TILE_256, HKP_TILE_256_A3, HKP_TILE_256_TAIL, ConvDesc
    n, h, w, cin, cout, k, pad, dil = 8, 60, 80, 512, 512, 3, 4, 4          # the C3 shard's layer4 dgrad
    d = cuda_device
    g = torch.Generator(device=d).manual_seed(21)
    wt = torch.randn(cout, k, k, cin, device=d, generator=g) * (2.0 / (k * k * cout)) ** 0.5
    gy = torch.randn(n, h, w, cout, device=d, generator=g) * 1e-3
    add = torch.randn(n, h, w, cin, device=d, generator=g) * 1e-3
    desc = ConvDesc(n, h, w, cin, cout, k, k, 1, pad, dil, 0, HKP_TILE_256_TAIL)
    assert ops.kernel_name(desc, HKP_KOP_DGRAD_X3).startswith("conv_x3_kernel<256,")
    amax = ops.absmax(gy)
    dys = ops.split_pack_x3(gy, amax)
    wf = ops.weight_flip_pack_x3(wt)
    dx1 = ops.conv2d_bwd_data_x3(dys, wf, (n, h, w, cin), pad, dil, add=add, amax=amax, tile=HKP_TILE_256_TAIL)
    dx2 = ops.conv2d_bwd_data_x3(dys, wf, (n, h, w, cin), pad, dil, add=add, amax=amax, tile=HKP_TILE_256_TAIL)
    dx0 = ops.conv2d_bwd_data_x3(dys, wf, (n, h, w, cin), pad, dil, add=add, amax=amax, sk=False, tile=HKP_TILE_256)
    assert torch.equal(dx1, dx2)
    assert (dx1 - dx0).abs().max().item() <= 4e-6 * dx0.abs().max().item()
    dx3 = ops.conv2d_bwd_data_x3(dys, wf, (n, h, w, cin), pad, dil, add=add, amax=amax, tile=HKP_TILE_256_A3)
    dx4 = ops.conv2d_bwd_data_x3(dys, wf, (n, h, w, cin), pad, dil, add=add, amax=amax, tile=HKP_TILE_256_A3)
    assert torch.equal(dx3, dx4)                                # the one-launch A3 + tail form
    assert (dx3 - dx0).abs().max().item() <= 4e-6 * dx0.abs().max().item()
    # fp64 on a slice of images
    ref = torch.nn.grad.conv2d_input((2, cin, h, w), wt.permute(0, 3, 1, 2).double(),
                                     gy[:2].permute(0, 3, 1, 2).double(), 1, pad, dil) + add[:2].permute(0, 3, 1, 2).double()
    err = (dx1[:2].permute(0, 3, 1, 2).double() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 2e-6, err


def test_bn_apply_f16(cuda_device):
    """fp16 BN apply (config C4): fp32 arithmetic on fp16 y / residuals, one fp16
    rounding of the result; the fp32 copy is the unrounded value."""
    from hkp import ops
    d = cuda_device
    y = rand(2, 9, 11, 96, seed=91).half().to(d)
    r = rand(2, 9, 11, 96, seed=92).half().to(d)
    ss = torch.cat([rand(96, seed=93) * 0.5 + 1, rand(96, seed=94) * 0.1]).to(d)
    rs = torch.cat([rand(96, seed=95) * 0.5 + 1, rand(96, seed=96) * 0.1]).to(d)
    c = 96
    base = y.float() * ss[:c] + ss[c:]
    for res, res_ss, want in ((None, None, base), (r, None, base + r.float()),
                              (r, rs, base + (r.float() * rs[:c] + rs[c:]))):
        o = ops.bn_apply_f16(y, ss, res=res, res_ss=res_ss, relu=True, keep_fp32=True)
        assert torch.equal(o, torch.relu(want))
        assert torch.equal(ops.split_of(o)[0], torch.relu(want).half())
        o16 = ops.bn_apply_f16(y, ss, res=res, res_ss=res_ss, relu=False)
        assert o16.dtype == torch.float16 and torch.equal(o16, want.half())


@pytest.mark.parametrize("case", X3_CASES)
@pytest.mark.parametrize("products", [2, 4])
def test_x3_product_subsets(cuda_device, case, products):
    """hkp_conv2d_fwd_x3_products: HKP_X3_W16 (2) = the activation exact x the
    weights rounded to fp16 after their power-of-two scale; HKP_X3_X16 (4) = the
    activation rounded to fp16 x the weights exact.  Each equals an fp64 conv of
    the correspondingly rounded operands to fp32-class accuracy (2e-6 of the output
    scale, as f16x3), on every live tile body; BN partials as the y they produced."""
    from hkp import ops
    n, h, w, cin, cout, k, st, pad, dil = case
    x = F.relu(rand(n, h, w, cin, seed=21))
    wt = rand(cout, k, k, cin, seed=22, scale=(2.0 / (k * k * cout)) ** 0.5)
    d = cuda_device
    ss = torch.cat([torch.ones(cin), torch.zeros(cin)]).to(d)
    xs = ops.bn_apply(x.to(d), ss, relu=False, split=3, keep_fp32=False)
    wp = ops.weight_pack_x3(wt.to(d))
    inv = wp.inv_scale.cpu().view(-1, 1, 1, 1)
    xr, wr = x.double(), wt.double()
    if products == 2:                                     # weights: hi of the scaled weight, unscaled
        wr = ((wt / inv).half().double()) * inv.double()
    else:                                                 # activation: hi = f16(x)
        xr = x.half().double()
    ref = F.conv2d(xr.permute(0, 3, 1, 2), wr.permute(0, 3, 1, 2), None, st, pad, dil)
    scale = ref.abs().max().item()
    y, p = ops.conv2d_fwd_x3(xs, wp, st, pad, dil, products=products)
    err = (y.cpu().double().permute(0, 3, 1, 2) - ref).abs().max().item() / scale
    full = F.conv2d(x.permute(0, 3, 1, 2).double(), wt.permute(0, 3, 1, 2).double(), None, st, pad, dil)
    err_full = (y.cpu().double().permute(0, 3, 1, 2) - full).abs().max().item() / scale
    print("products %d: vs rounded-operand fp64 %.3g, vs exact fp64 %.3g" % (products, err, err_full))
    assert err < 2e-6, err
    assert 1e-5 < err_full < 3e-3, err_full              # the fp16 rounding of one operand is visible
    m = y.numel() // cout
    y32 = y.reshape(m, cout).double()
    stats = _bn_stats(p, m)
    torch.testing.assert_close(stats[:cout].cpu().double(), y32.mean(0).cpu(), rtol=1e-5, atol=1e-6)
    for tile in LIVE_TILES:
        yv, pv = ops.conv2d_fwd_x3(xs, wp, st, pad, dil, tile=tile, products=products)
        assert (yv.cpu().double().permute(0, 3, 1, 2) - ref).abs().max().item() < 2e-6 * scale, tile



BNIN_CASES = [
    (2, 16, 64, 64, 64),        # 2 channel groups (f16x3) / 1 (fp16), 2 x 2 patches per image
    (1, 24, 96, 128, 128),      # 4 / 2 channel groups, 2 column tiles
    (1, 8, 32, 32, 64),         # one patch, one f16x3 channel group
]


@pytest.mark.parametrize("case", BNIN_CASES)
@pytest.mark.parametrize("prec", ["f16x3", "f16"])
def test_fused_input_bn_equals_apply_then_conv(cuda_device, case, prec):
    """hkp_conv2d_fwd_x3_bnin / _f16_bnin (the halo body applying its input's BN +
    ReLU to each halo image in LDS, out-of-image lines as NaN lines) == bn_apply /
    bn_apply_f16 followed by the halo conv: the same y and BN partials, bit for bit.
    Scale / shift include negative scales and large shifts (the NaN padding must
    give 0 whatever their sign)."""
    from hkp import ops
    n, h, w, c, k = case
    if prec == "f16" and c % 64:
        pytest.skip("plain fp16 needs Cin % 64")
    d = cuda_device
    y = (rand(n, h, w, c, seed=91) * 3 + 1).to(d)
    ss = torch.cat([rand(c, seed=92) * 0.7, rand(c, seed=93) * 2.0]).to(d)     # mixed signs
    wt = rand(k, 3, 3, c, seed=94, scale=(2.0 / (9 * k)) ** 0.5).to(d)
    if prec == "f16x3":
        wp = ops.weight_pack_x3(wt)
        a = ops.bn_apply(y, ss, relu=True, split=3, keep_fp32=False)
        ref, pref = ops.conv2d_fwd_x3(a, wp, 1, 1, 1, tile=10)                 # the halo body
        got, pgot = ops.conv2d_fwd_bnin(y, ss, wp, 1, 1, 1, tile=10)
    else:
        wp = ops.weight_pack_f16(wt)
        y16 = y.half()
        a = ops.bn_apply_f16(y16, ss, relu=True)
        ref, pref = ops.conv2d_fwd_f16(a, wp, 1, 1, 1, tile=10)
        got, pgot = ops.conv2d_fwd_bnin(y16, ss, wp, 1, 1, 1, tile=10)
    assert got.dtype == ref.dtype and torch.equal(got, ref)
    assert torch.equal(pgot, pref)
    _, pnone = ops.conv2d_fwd_bnin(y if prec == "f16x3" else y.half(), ss, wp, 1, 1, 1, stats=False, tile=10)
    assert pnone is None


def test_fused_input_bn_rejects_other_shapes(cuda_device):
    from hkp import ops
    d = cuda_device
    y = rand(1, 12, 32, 64, seed=95).to(d)                  # Ho % 8 != 0: no halo tiling
    ss = torch.cat([torch.ones(64), torch.zeros(64)]).to(d)
    wp = ops.weight_pack_x3(rand(64, 3, 3, 64, seed=96, scale=0.05).to(d))
    with pytest.raises(ops.HkpError, match="halo"):
        ops.conv2d_fwd_bnin(y, ss, wp, 1, 1, 1)
    # the A3 body has no fused form (round 5: removed)
    wp16 = ops.weight_pack_f16(rand(256, 1, 1, 64, seed=97, scale=0.05).to(d))
    with pytest.raises(ops.HkpError, match="halo"):
        ops.conv2d_fwd_bnin(y.half(), ss, wp16, 1, 0, 1, tile=11)
    assert ops.bnin_kernel(1, 12, 32, 64, 256, 1, 1, 1, 0, 1, f16=True, tile=11) is None
    assert ops.bnin_kernel(1, 12, 32, 64, 256, 1, 1, 1, 0, 1, tile=11) is None


@pytest.mark.parametrize("bb,prec,b,hw,fused", [
    ("resnet18", "f16x3", 2, (128, 256), "conv_x3_halo_bnin_kernel<3>"),
    ("resnet50", "f16", 2, (128, 256), "conv_x3_halo_bnin_kernel<1>"),
    ("resnet34", "f16x3", 32, (480, 640), "conv_x3_halo_bnin_kernel<3>")])     # C2 itself
def test_fused_input_bn_network_bitexact(cuda_device, bb, prec, b, hw, fused):
    """Whole inference forward (128x256: a halo-tiled layer1 at 32x64; C2 640x480
    B=32): fused == unfused, heatmaps and argmax bit for bit, and the fused
    kernels ran."""
    from hkp import net, ops
    m = _model(bb, 4, 7, cuda_device, precision=prec)
    x = recipe.to_tensor_nchw(recipe.seeded_images_u8(b, hw[0], hw[1], 8)).to(cuda_device)
    syms = set()

    def observe(sym, flops, nbytes, launch):
        syms.add(sym)
        launch()
    outs = []
    for fuse in (True, False):
        ops.set_observer(observe if fuse else None)
        try:
            with torch.no_grad():
                hm, yx = m.heatmaps_and_keypoints(x, policy=m.policy.with_(fuse_input_bn=fuse))
        finally:
            ops.set_observer(None)
        outs.append((hm, yx))
    assert fused in syms, syms
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


def test_stage_precision_plans(cuda_device, golden):
    """Policy.stage_precision (DESIGN "Per-stage precision"): an all-f16 plan gives
    the plain-fp16 network's bits and an all-f16x3 plan the f16x3 network's; a mixed
    plan converts the activation where two stages meet (f16 -> fp32 + packed split,
    f16x3 -> the fp16 plane) and its heatmap error against the reference fixture stays
    within the plain-fp16 network's own error on it (argmax reported, not promised —
    as for plain fp16, near-flat random-init heatmaps flip peaks)."""
    g = golden("fwd_r50_k8_480x640_b2")
    B, H, W, K, st = int(g["batch"]), int(g["height"]), int(g["width"]), int(g["k"]), int(g["step"])
    m = _model("resnet50", K, int(g["wseed"]), cuda_device, precision="f16")
    x = recipe.to_tensor_nchw(recipe.seeded_images_u8(B, H, W, int(g["iseed"]))).to(cuda_device)

    def run(**kw):
        with torch.no_grad():
            return m.heatmaps_and_keypoints(x, policy=m.policy.with_(**kw))
    f16, x3 = run(), run(precision="f16x3")
    a16 = run(stage_precision=("f16",) * 4)
    a3 = run(stage_precision=("f16x3",) * 4)
    assert torch.equal(a16[0], f16[0]) and torch.equal(a16[1], f16[1])
    assert torch.equal(a3[0], x3[0]) and torch.equal(a3[1], x3[1])

    def score(out):
        err = float(np.abs(out[0][:, :, ::st, ::st].cpu().numpy() - g["heat_sub"]).max())
        return err, float((out[1].cpu().numpy() == g["argmax_yx"]).all(-1).mean())
    e16, g16 = score(f16)
    print("plain f16: max heat err %.3g, argmax agreement %.2f" % (e16, g16))
    for plan in (("f16", "f16", "f16x3", "f16x3"), ("f16x3", "f16", "f16x3", "f16")):
        out = run(stage_precision=plan)
        err, agree = score(out)
        print("%s: max heat err %.3g, argmax agreement %.2f" % (",".join(plan), err, agree))
        # round 6 on MI355X: the first plan 0.068 / 0.69; gate: no worse than plain fp16
        # on the same fixture plus 10 %
        assert torch.isfinite(out[0]).all() and err < max(e16, 0.02) * 1.1, (plan, err, e16)
    # the offered accuracy point (DESIGN "Per-stage precision"): layer1-2 at f16x3 —
    # measured 0.0049 max heat error and 15/16 keypoints (plain f16: 0.069, 12/16)
    out = run(stage_precision=("f16x3", "f16x3", "f16", "f16"))
    err, agree = score(out)
    print("f16x3,f16x3,f16,f16: max heat err %.3g, argmax agreement %.2f" % (err, agree))
    assert err < 0.01 and err < e16 / 5 and agree >= 0.8, (err, agree)
