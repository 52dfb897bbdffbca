"""CPU-only checks of the boundary: the C-ABI library loads, exports every
symbol include/hulkkp.h declares, and the Python module tree speaks the
reference's state_dict (no GPU compute here)."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

from conftest import REPO

HEADER = os.path.join(REPO, "include", "hulkkp.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(hkp_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    from hkp import _lib
    L = _lib.lib()
    names = declared_functions()
    assert len(names) >= 10
    for n in names:
        assert hasattr(L, n), "missing export " + n
    assert set(names) == set(_lib.SIGNATURES), "ctypes signature table out of sync with the header"
    assert _lib.version().startswith("hulkkp")


def test_product_library_has_no_ab_knobs():
    """The A/B instruments (hkp_debug_*, include/hulkkp_ab.h) exist only in the tools
    build: the product library exports none of them and its header declares none."""
    from hkp import _lib
    path = os.path.join(REPO, "hulk-keypoints_amd", "hkp", "libhulkkp.so")
    L = ctypes.CDLL(path)
    assert _lib.AB_SIGNATURES
    for n in _lib.AB_SIGNATURES:
        assert not hasattr(L, n), "product library exports the A/B knob " + n
    assert not [n for n in declared_functions() if n.startswith("hkp_debug_")]
    syms = open(path, "rb").read()
    assert b"hkp_debug_" not in syms


def _kernel_scratch(blob):
    """(symbol, private_segment_fixed_size) of every gfx950 kernel in a library's
    embedded code objects, read from the msgpack kernel metadata (uncompressed)."""
    key = b".private_segment_fixed_size"
    out = []
    for m in re.finditer(re.escape(key), blob):
        i = m.end()
        t = blob[i]
        size = t if t < 0x80 else int.from_bytes(blob[i + 1:i + 1 + {0xcc: 1, 0xcd: 2, 0xce: 4}[t]], "big")
        j = blob.find(b".symbol", i, i + 4096)
        sym = "?"
        if j >= 0:
            k = j + len(b".symbol")
            if 0xa0 <= blob[k] <= 0xbf:
                sym = blob[k + 1:k + 1 + (blob[k] & 0x1f)].decode(errors="replace")
            elif blob[k] == 0xd9:
                sym = blob[k + 2:k + 2 + blob[k + 1]].decode(errors="replace")
        out.append((sym, size))
    return out


def test_no_kernel_uses_scratch():
    """No kernel of libhulkkp.so spills or keeps an array in scratch (a runtime
    accumulator index once put the 256x256 conv's whole tile there: 528 B per lane)."""
    lib = os.path.join(REPO, "hulk-keypoints_amd", "hkp", "libhulkkp.so")
    ks = _kernel_scratch(open(lib, "rb").read())
    assert len(ks) >= 100
    bad = [(s, n) for s, n in ks if n]
    assert not bad, bad


def test_bad_arguments_raise_not_crash():
    from hkp import _lib
    d = _lib.ConvDesc(1, 8, 8, 30, 64, 3, 3, 1, 1, 1, 0)  # Cin=30 is unsupported on the NHWC path
    with pytest.raises(_lib.HkpError, match="multiple of 32"):
        _lib.call("hkp_conv2d_fwd", ctypes.byref(d), ctypes.c_void_p(1), ctypes.c_void_p(1), ctypes.c_void_p(1),
                  None, None)
    ho, wo = ctypes.c_int32(), ctypes.c_int32()
    d = _lib.ConvDesc(2, 60, 80, 256, 256, 3, 3, 1, 2, 2, 0)
    _lib.call("hkp_conv_out_hw", ctypes.byref(d), ctypes.byref(ho), ctypes.byref(wo))
    assert (ho.value, wo.value) == (60, 80)
    assert _lib.lib().hkp_conv_stat_tiles(ctypes.byref(d)) == (2 * 60 * 80 + 127) // 128


@pytest.mark.parametrize("bb", ["resnet18", "resnet34", "resnet50"])
def test_state_dict_is_reference_compatible(bb):
    from oracle import cpu_ref, recipe
    from src.model import KeypointsGauss
    m = KeypointsGauss(4, backbone=bb, pretrained=False)
    spec = cpu_ref.state_dict_spec(bb)
    sd = m.state_dict()
    assert list(sd.keys()) == [k for k, _, _ in spec]
    for k, shape, _ in spec:
        assert tuple(sd[k].shape) == tuple(shape), k
    # parameters() order == reference parameters() order (Adam state / DDP buckets line up)
    names = [n for n, _ in m.named_parameters()]
    assert names == cpu_ref.param_keys(bb)
    # load → save round trip is exact (OIHW ↔ KRSC repack)
    ref_sd = recipe.seeded_state_dict(bb, 11)
    m.load_state_dict(ref_sd)
    back = m.state_dict()
    for k in ref_sd:
        assert torch.equal(back[k], ref_sd[k]), k
    w = m.resnet.net.layer1[0].conv1.weight
    assert tuple(w.shape[1:3]) == ((1, 1) if bb == "resnet50" else (3, 3))  # stored KRSC


def test_reference_init_statistics():
    from src.model import KeypointsGauss
    torch.manual_seed(0)
    m = KeypointsGauss(4, pretrained=False)
    w = m.resnet.net.layer4[0].conv2.weight  # 512x3x3x512, std sqrt(2/(9*512))
    assert abs(w.std().item() - np.sqrt(2 / (9 * 512))) < 2e-4
    assert abs(m.resnet.net.fc.weight.std().item() - 0.01) < 2e-4
    assert m.resnet.net.fc.bias.abs().sum().item() == 0


def test_weight_pack_batch_host_side():
    """hkp_pack_job layout, workspace sizing and argument checks (host only)."""
    from hkp import _lib
    assert ctypes.sizeof(_lib.PackJob) == 56
    jobs = (_lib.PackJob * 3)()
    for j, (kind, k, rs, c) in zip(jobs, [(0, 64, 9, 64), (1, 512, 9, 512), (1, 2048, 1, 512)]):
        j.w, j.out, j.inv_scale, j.kind, j.k, j.rs, j.c = 16, 16, 16, kind, k, rs, c
    assert _lib.lib().hkp_weight_pack_x3_batch_ws_bytes(3, jobs) == 4 * (512 // 8 * 512 + 2048 // 8 * 512)
    with pytest.raises(_lib.HkpError, match="workspace"):
        _lib.call("hkp_weight_pack_x3_batch", 3, jobs, None, 0, None)
    jobs[1].c = 96                                     # flip needs c % 64 == 0
    with pytest.raises(_lib.HkpError, match="c%64==0"):
        _lib.call("hkp_weight_pack_x3_batch", 3, jobs, None, 0, None)
    assert _lib.call("hkp_weight_pack_x3_batch", 0, jobs, None, 0, None) == 0


def test_adam_abi_host_side():
    """hkp_adam_tensor layout and argument checks (host only, no launch)."""
    from hkp import _lib
    assert ctypes.sizeof(_lib.AdamTensor) == 40
    ts = (_lib.AdamTensor * 2)()
    ts[0].param, ts[0].grad, ts[0].exp_avg, ts[0].exp_avg_sq, ts[0].n = 16, 16, 16, 16, 8
    ts[1].n = 8                                        # null pointers with n > 0
    with pytest.raises(_lib.HkpError, match="null pointer"):
        _lib.call("hkp_adam_step", 2, ts, 0.999, 0.1, 0.001, 1e-8, 0.0, -1e-3, 1.0, None)
    with pytest.raises(_lib.HkpError, match="bias_correction2_sqrt"):
        _lib.call("hkp_adam_step", 1, ts, 0.999, 0.1, 0.001, 1e-8, 0.0, -1e-3, 0.0, None)
    assert _lib.call("hkp_adam_step", 0, ts, 0.999, 0.1, 0.001, 1e-8, 0.0, -1e-3, 1.0, None) == 0


def test_fused_adam_rejects_unsupported_options():
    from hkp.optim import FusedAdam
    from hkp._lib import HkpError
    p = [torch.nn.Parameter(torch.zeros(4))]
    with pytest.raises(HkpError):
        FusedAdam(p, amsgrad=True)
    opt = FusedAdam(p, lr=1e-4, weight_decay=1e-4)
    p[0].grad = torch.zeros(4)
    with pytest.raises(HkpError, match="CUDA"):       # no CPU path
        opt.step()


def test_kernel_name_query():
    """hkp_conv_kernel_name: the tile planner's choice for a descriptor, as the
    kernel symbol rocprofv3 reports — per call (hkp_conv_desc.tile), no global knob."""
    from hkp import _lib, ops
    # C2 layer4 conv (R34, 640x480, B=32, dilation 4): 1200 256x256 tiles
    d = _lib.ConvDesc(32, 60, 80, 512, 512, 3, 3, 1, 4, 4, 0)
    assert ops.kernel_name(d, _lib.HKP_KOP_FWD_X3) == "conv_x3_a3_kernel<3>"        # 256x256 on the A3 body
    assert ops.kernel_name(d, _lib.HKP_KOP_FWD_F16) == "conv_x3_a3_kernel<1>"
    d.tile = _lib.HKP_TILE_256
    assert ops.kernel_name(d, _lib.HKP_KOP_FWD_X3) == "conv_x3_kernel<256, false, false, 16, false, 3>"
    assert ops.kernel_name(d, _lib.HKP_KOP_WGRAD_X3) == "wgrad_x3_kernel<256>"
    # the C3 shard's layer1 / layer2 3x3 wgrads: the halo body; tile -1 keeps the tiled one
    for c, h, w in ((64, 120, 160), (128, 60, 80)):
        dw = _lib.ConvDesc(8, h, w, c, c, 3, 3, 1, 1, 1, 0)
        assert ops.kernel_name(dw, _lib.HKP_KOP_WGRAD_X3) == "wgrad_x3_halo_kernel"
        dw.tile = -1
        assert ops.kernel_name(dw, _lib.HKP_KOP_WGRAD_X3) == "wgrad_x3_kernel<%d>" % (64 if c == 64 else 128)
    # stride 2 / dilation 2 / Wo % 16 != 0: the tiled body
    for dw in (_lib.ConvDesc(8, 120, 160, 64, 128, 3, 3, 2, 1, 1, 0), _lib.ConvDesc(8, 60, 80, 128, 128, 3, 3, 1, 2, 2, 0),
               _lib.ConvDesc(2, 17, 23, 64, 64, 3, 3, 1, 1, 1, 0)):
        assert ops.kernel_name(dw, _lib.HKP_KOP_WGRAD_X3).startswith("wgrad_x3_kernel<")
    d.tile = _lib.HKP_TILE_AUTO_A3                                  # AUTO without the DUO choices
    assert ops.kernel_name(d, _lib.HKP_KOP_FWD_X3) == "conv_x3_a3_kernel<3>"
    # plain fp16: the DUO body at K-depth 64 and for 128-wide outputs (AUTO), not under AUTO_A3
    l1 = _lib.ConvDesc(128, 120, 160, 64, 256, 1, 1, 1, 0, 1, 0)
    l2 = _lib.ConvDesc(128, 60, 80, 128, 128, 3, 3, 1, 1, 1, 0)
    for dd in (l1, l2):
        assert ops.kernel_name(dd, _lib.HKP_KOP_FWD_F16) == "conv_x3_duo_kernel<1>"
        assert ops.kernel_name(dd, _lib.HKP_KOP_FWD_X3) != "conv_x3_duo_kernel<1>"
        dd.tile = _lib.HKP_TILE_AUTO_A3
        assert ops.kernel_name(dd, _lib.HKP_KOP_FWD_F16) != "conv_x3_duo_kernel<1>"
    assert ops.kernel_name(_lib.ConvDesc(128, 60, 80, 512, 2048, 1, 1, 1, 0, 1, 0),
                           _lib.HKP_KOP_FWD_F16) == "conv_x3_a3_kernel<1>"
    d.tile = _lib.HKP_TILE_256_A3
    assert ops.kernel_name(d, _lib.HKP_KOP_FWD_X3) == "conv_x3_a3_kernel<3>"
    assert ops.kernel_name(d, _lib.HKP_KOP_FWD_X3_W16) == "conv_x3_a3_kernel<2>"
    assert ops.kernel_name(d, _lib.HKP_KOP_FWD_X3_X16) == "conv_x3_a3_kernel<4>"
    # the 192-row A3 tiles: packed operands with Cout % 256 == 0 (forward and dgrad), 96-row
    # BN statistic tiles; plain fp16 and narrower outputs plan as AUTO (128-row tiles)
    d.tile = _lib.HKP_TILE_192_A3
    assert ops.kernel_name(d, _lib.HKP_KOP_FWD_X3) == "conv_x3_a3_192_kernel<3>"
    assert ops.kernel_name(d, _lib.HKP_KOP_FWD_X3_W16) == "conv_x3_a3_192_kernel<2>"
    assert ops.kernel_name(d, _lib.HKP_KOP_FWD_F16) == ops.kernel_name(
        _lib.ConvDesc(*[getattr(d, f) for f, _ in d._fields_[:-1]], 0), _lib.HKP_KOP_FWD_F16)
    rows = _lib.lib().hkp_conv_x3_stat_tile_rows
    assert rows(ctypes.byref(d), _lib.HKP_KOP_FWD_X3) == 96 and rows(ctypes.byref(d), _lib.HKP_KOP_FWD_F16) == 128
    b8 = _lib.ConvDesc(8, 60, 80, 256, 256, 3, 3, 1, 2, 2, 0, _lib.HKP_TILE_192_A3)
    assert ops.kernel_name(b8, _lib.HKP_KOP_DGRAD_X3) == "conv_x3_a3_192_kernel<3>"
    narrow = _lib.ConvDesc(8, 60, 80, 256, 128, 3, 3, 1, 2, 2, 0, _lib.HKP_TILE_192_A3)
    assert "a3_192" not in ops.kernel_name(narrow, _lib.HKP_KOP_FWD_X3)
    assert rows(ctypes.byref(narrow), _lib.HKP_KOP_FWD_X3) == 128
    narrow.tile = _lib.HKP_TILE_160_A3                                 # 128-wide: the 160x128 form
    assert ops.kernel_name(narrow, _lib.HKP_KOP_FWD_X3) == "conv_x3_a3_160x128_kernel<3>"
    assert rows(ctypes.byref(narrow), _lib.HKP_KOP_FWD_X3) == 80
    b8.tile = _lib.HKP_TILE_160_A3
    assert ops.kernel_name(b8, _lib.HKP_KOP_FWD_X3) == "conv_x3_a3_160_kernel<3>"
    assert rows(ctypes.byref(b8), _lib.HKP_KOP_FWD_X3) == 80
    b8.tile = 0
    assert rows(ctypes.byref(b8), _lib.HKP_KOP_FWD_X3) == 128
    d.tile = _lib.HKP_TILE_64_PAIR
    assert ops.kernel_name(d, _lib.HKP_KOP_FWD_X3) == "conv_x3_kernel<64, false, true, 16, false, 3>"
    d.tile = 99
    with pytest.raises(_lib.HkpError, match="tile policy"):
        ops.kernel_name(d, _lib.HKP_KOP_FWD_X3)
    stem = _lib.ConvDesc(32, 480, 640, 3, 64, 7, 7, 2, 3, 1, _lib.HKP_LAYOUT_NCHW)
    assert ops.kernel_name(stem, _lib.HKP_KOP_STEM_X3) == "conv_x3_stem_patch_kernel<0>"    # 240x320: 8x32 patches
    assert ops.kernel_name(stem, _lib.HKP_KOP_STEM_X3_IMAGE) == "conv_x3_stem_patch_kernel<1>"  # straight from the image
    assert ops.kernel_name(stem, _lib.HKP_KOP_STEM_X3_IMAGE_U8) == "conv_x3_stem_patch_kernel<2>"
    assert _lib.lib().hkp_stem_x3_image_ok(ctypes.byref(stem)) == 1
    stem.tile = _lib.HKP_TILE_64_PAIR
    assert ops.kernel_name(stem, _lib.HKP_KOP_STEM_X3) == "conv_x3_kernel<64, true, true, 16, false, 3>"
    odd = _lib.ConvDesc(2, 120, 160, 3, 64, 7, 7, 2, 3, 1, _lib.HKP_LAYOUT_NCHW)              # 60x80: no patch tiling
    assert ops.kernel_name(odd, _lib.HKP_KOP_STEM_X3) == "conv_x3_kernel<64, true, true, 16, false, 3>"
    assert _lib.lib().hkp_stem_x3_image_ok(ctypes.byref(odd)) == 0
    with pytest.raises(_lib.HkpError, match="patch body"):
        ops.kernel_name(odd, _lib.HKP_KOP_STEM_X3_IMAGE)


def test_bnin_kernel_eligibility():
    """ops.bnin_kernel names the fused-input-BN kernel from the unfused launch's own
    tile choice (hkp_conv_kernel_name; no GPU): the halo body at 64-channel 3x3
    stride-1 shapes, None elsewhere (the A3 body's fused form was removed in round
    5: measured slower, and its untracked in-flight loads faulted an instrument
    build — DESIGN "BN apply folded into the consumer")."""
    from hkp import ops
    # C2 layer1 conv2 (halo default at 64 channels)
    assert ops.bnin_kernel(32, 120, 160, 64, 64, 3, 3, 1, 1, 1) == "conv_x3_halo_bnin_kernel<3>"
    assert ops.bnin_kernel(32, 120, 160, 64, 64, 3, 3, 1, 1, 1, f16=True) == "conv_x3_halo_bnin_kernel<1>"
    # C2 layer3 / layer4 conv2 (the A3 body): no fused form
    assert ops.bnin_kernel(32, 60, 80, 256, 256, 3, 3, 1, 2, 2) is None
    assert ops.bnin_kernel(32, 60, 80, 512, 512, 3, 3, 1, 4, 4) is None
    assert ops.bnin_kernel(32, 60, 80, 512, 512, 3, 3, 1, 4, 4, f16=True, tile=11) is None
    # 128-wide outputs (layer2) and the forced 2-stage body: no fused form
    assert ops.bnin_kernel(32, 60, 80, 128, 128, 3, 3, 1, 1, 1) is None
    assert ops.bnin_kernel(32, 60, 80, 256, 256, 3, 3, 1, 2, 2, tile=1) is None
    # channel counts the operand layouts cannot take
    assert ops.bnin_kernel(1, 16, 32, 48, 64, 3, 3, 1, 1, 1) is None


def test_policy_fusion_and_overlap_fields():
    from hkp.policy import DEFAULT, TUNING_FIELDS
    assert DEFAULT.fuse_input_bn
    assert DEFAULT.overlap_wgrad and DEFAULT.overlap_min_gflop == 0.0
    for f in ("fuse_input_bn", "overlap_min_gflop"):
        assert f in TUNING_FIELDS
