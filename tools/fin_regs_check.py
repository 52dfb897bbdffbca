#!/usr/bin/env python3
"""A/B check on the tools build (tools/ab_lib/libhulkkp_ab.so): the BN finalize
merges' register-held form (hkp_debug_fin_regs 1, the product's only form) gives
the batched-load loops' bits, forward (scale/shift, mean/invstd, running
statistics) and backward (dgamma, dbeta, the apply coefficients, the split-scale
bound), over random partials with ragged counts.  Run by
tests/test_gpu_backward.py::test_bn_finalize_register_form_same_bits."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "hulk-keypoints_amd")]

import torch  # noqa: E402

CASES = [(64, 1), (64, 2047), (128, 1200), (256, 1200), (512, 1200), (512, 300), (1024, 600), (2048, 150),
         (256, 3000)]


def main():
    from hkp import _lib
    _lib.use_ab_library()
    from hkp import ops
    from hkp._lib import lib
    d = torch.device("cuda", 0)
    for c, tiles in CASES:
        g = torch.Generator(device=d).manual_seed(c * 7 + tiles)
        rows = tiles * 128 - 37
        part = torch.stack([torch.randn(tiles, c, device=d, generator=g) * 100,
                            torch.rand(tiles, c, device=d, generator=g) * 1000], -1).contiguous()
        gamma = torch.rand(c, device=d, generator=g) + 0.5
        beta = torch.rand(c, device=d, generator=g) - 0.5
        mrows = tiles * 64 - 5                       # the backward's 64-row tiles
        bpart = torch.randn(tiles, c, 2, device=d, generator=g) * 50
        bmax = torch.rand(tiles, c, 2, device=d, generator=g) * 10
        mi = torch.cat([torch.randn(c, device=d, generator=g), torch.rand(c, device=d, generator=g) + 0.1])
        outs = []
        try:
            for on in (0, 1):
                lib().hkp_debug_fin_regs(on)
                rm, rv = torch.zeros(c, device=d), torch.ones(c, device=d)
                nbt = torch.zeros(1, device=d, dtype=torch.int64)
                ss, mio = ops.bn_finalize(part, rows, gamma, beta, rm, rv, nbt, two_level_tiles=1 << 40)
                dgamma, dbeta = torch.empty(c, device=d), torch.empty(c, device=d)
                coef = torch.empty(3 * c, device=d)
                amax = torch.zeros(1, device=d, dtype=torch.int32)
                ops.call("hkp_bn_bwd_finalize", c, mrows, ops._ptr(bpart), ops._ptr(bmax), ops._ptr(mi),
                         ops._ptr(gamma), ops._ptr(dgamma), ops._ptr(dbeta), ops._ptr(coef), ops._ptr(amax),
                         ops._stream())
                outs.append((ss, mio, rm, rv, nbt, dgamma, dbeta, coef, amax))
            torch.cuda.synchronize()
        finally:
            lib().hkp_debug_fin_regs(1)
        for a, b in zip(*outs):
            assert torch.equal(a, b), (c, tiles)
        assert outs[1][4].item() == 1 and outs[1][8].item() != 0
        print("c=%d tiles=%d: same bits" % (c, tiles))
    print("fin_regs_check ok")


if __name__ == "__main__":
    main()
