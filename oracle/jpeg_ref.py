"""TEST INFRASTRUCTURE — CPU restatement of the data-parallel half of a JPEG
decode, the checker for hkp_jpeg_reconstruct (csrc/jpeg.hip).  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may use it.

The reference decodes its images with cv2.imread (/root/reference/src/
dataset.py:71); OpenCV and Pillow both decode JPEG with libjpeg-turbo (here
Pillow's bundled 3.1.4, API 6.2 — cv2 itself is not installed).  With the
library defaults (JDCT_ISLOW, do_fancy_upsampling) libjpeg-turbo computes, per
8x8 block and pixel, the integer arithmetic of the IJG reference sources it
keeps (its SIMD paths are bit-exact with them):

  idct_islow     jidctint.c jpeg_idct_islow: LL&M 1-D IDCT, CONST_BITS 13,
                 PASS1_BITS 2, columns then rows, DESCALE rounding, the
                 post-IDCT range-limit table of jdmaster.c
                 (prepare_range_limit_table: index & 1023, so clamp to [0,255]
                 for every value a valid stream produces)
  upsample       jdsample.c h2v1_fancy_upsample / h2v2_fancy_upsample (the
                 triangle filter, biases 1/2 and 8/7) for components wider
                 than 2 samples, the box upsamplers h2v1/h2v2_upsample
                 otherwise; rows outside the image repeat the edge row
                 (jdmainct.c context rows)
  ycc_to_bgr     jdcolor.c ycc_rgb_convert: SCALEBITS 16 tables
                 (1.40200, 1.77200, 0.71414, 0.34414), range-limited

Pinned, not restated blind: tests/test_jpeg_cpu.py decodes Pillow-encoded JPEGs
(every supported subsampling, qualities, odd sizes, restart intervals,
optimised Huffman tables, grayscale) with the host entropy decoder plus this
module and requires the pixels to equal Pillow's decode exactly.
"""
import numpy as np

CONST_BITS, PASS1_BITS = 13, 2
FIX_0_298631336, FIX_0_390180644, FIX_0_541196100 = 2446, 3196, 4433
FIX_0_765366865, FIX_0_899976223, FIX_1_175875602 = 6270, 7373, 9633
FIX_1_501321110, FIX_1_847759065, FIX_1_961570560 = 12299, 15137, 16069
FIX_2_053119869, FIX_2_562915447, FIX_3_072711026 = 16819, 20995, 25172


def _descale(x, n):
    return (x + (1 << (n - 1))) >> n


def _idct_1d(s0, s1, s2, s3, s4, s5, s6, s7):
    """jidctint.c's even / odd parts on int64 arrays: returns the 8 outputs before
    descaling (both passes share this)."""
    z2, z3 = s2, s6
    z1 = (z2 + z3) * FIX_0_541196100
    tmp2 = z1 + z3 * (-FIX_1_847759065)
    tmp3 = z1 + z2 * FIX_0_765366865
    tmp0 = (s0 + s4) << CONST_BITS
    tmp1 = (s0 - s4) << CONST_BITS
    tmp10, tmp13 = tmp0 + tmp3, tmp0 - tmp3
    tmp11, tmp12 = tmp1 + tmp2, tmp1 - tmp2
    t0, t1, t2, t3 = s7, s5, s3, s1
    z1, z2, z3, z4 = t0 + t3, t1 + t2, t0 + t2, t1 + t3
    z5 = (z3 + z4) * FIX_1_175875602
    t0 = t0 * FIX_0_298631336
    t1 = t1 * FIX_2_053119869
    t2 = t2 * FIX_3_072711026
    t3 = t3 * FIX_1_501321110
    z1 = z1 * (-FIX_0_899976223)
    z2 = z2 * (-FIX_2_562915447)
    z3 = z3 * (-FIX_1_961570560) + z5
    z4 = z4 * (-FIX_0_390180644) + z5
    t0 = t0 + z1 + z3
    t1 = t1 + z2 + z4
    t2 = t2 + z2 + z3
    t3 = t3 + z1 + z4
    return (tmp10 + t3, tmp11 + t2, tmp12 + t1, tmp13 + t0, tmp13 - t0, tmp12 - t1, tmp11 - t2, tmp10 - t3)


def _range_limit_idct(v):
    """jdmaster.c's post-IDCT table indexed by v & 1023 (= clamp(v + 128, 0, 255)
    for -512 <= v < 512)."""
    i = v & 1023
    out = np.where(i < 128, i + 128, np.where(i < 512, 255, np.where(i < 896, 0, i - 896)))
    return out.astype(np.uint8)


def idct_islow(coefs, qt):
    """coefs int16 [nb,64] (natural order), qt [64] → uint8 [nb,8,8] samples."""
    c = coefs.astype(np.int64).reshape(-1, 8, 8) * qt.astype(np.int64).reshape(1, 8, 8)
    # pass 1: columns (index [row] within a column), results scaled by 2^PASS1_BITS
    outs = _idct_1d(*[c[:, r, :] for r in range(8)])
    ws = np.stack([_descale(o, CONST_BITS - PASS1_BITS) for o in outs], axis=1)     # [nb, row, col]
    # pass 2: rows
    outs = _idct_1d(*[ws[:, :, k] for k in range(8)])
    px = np.stack([_descale(o, CONST_BITS + PASS1_BITS + 3) for o in outs], axis=2)  # [nb, row, col]
    return _range_limit_idct(px)


def component_planes(coefs, qt, g):
    """Per component: uint8 [bh*8, bw*8] plane of IDCT'd blocks (geometry dict g)."""
    planes = []
    for c in range(g["ncomp"]):
        bw, bh, off = g["bw"][c], g["bh"][c], g["blk_off"][c]
        blk = idct_islow(coefs[off:off + bw * bh], qt[c]).reshape(bh, bw, 8, 8)
        planes.append(blk.transpose(0, 2, 1, 3).reshape(bh * 8, bw * 8))
    return planes


def _fancy_h2(row, dw):
    """h2v1_fancy_upsample of one sample row (int64 [dw]) → [2*dw]."""
    x = row[:dw].astype(np.int64)
    out = np.empty(2 * dw, np.int64)
    left = np.concatenate([x[:1], x[:-1]])
    right = np.concatenate([x[1:], x[-1:]])
    out[0::2] = (3 * x + left + 1) >> 2
    out[1::2] = (3 * x + right + 2) >> 2
    out[0], out[-1] = x[0], x[-1]
    return out


def upsample(plane, dw, dh, fh, fv, width, height):
    """One component to full resolution [height, width] (jdsample.c)."""
    p = plane[:dh, :dw].astype(np.int64)
    if fh == 1 and fv == 1:
        return p[:height, :width]
    if dw <= 2:                                        # box upsampling (no fancy method for narrow components)
        return np.repeat(np.repeat(p, fv, axis=0), fh, axis=1)[:height, :width]
    if fv == 1:                                        # h2v1
        return np.stack([_fancy_h2(r, dw) for r in p])[:height, :width]
    # h2v2: column sums with the row above (even output rows) / below (odd)
    above = np.concatenate([p[:1], p[:-1]])
    below = np.concatenate([p[1:], p[-1:]])
    out = np.empty((2 * dh, 2 * dw), np.int64)
    for par, nb in ((0, above), (1, below)):
        cs = 3 * p + nb
        left = np.concatenate([cs[:, :1], cs[:, :-1]], axis=1)
        right = np.concatenate([cs[:, 1:], cs[:, -1:]], axis=1)
        o = out[par::2]
        o[:, 0::2] = (3 * cs + left + 8) >> 4
        o[:, 1::2] = (3 * cs + right + 7) >> 4
        o[:, 0] = (4 * cs[:, 0] + 8) >> 4
        o[:, -1] = (4 * cs[:, -1] + 7) >> 4
    return out[:height, :width]


def ycc_to_bgr(y, cb, cr):
    """jdcolor.c ycc_rgb_convert, channels reordered B, G, R (cv2.imread)."""
    one_half = 1 << 15
    x_cb, x_cr = cb.astype(np.int64) - 128, cr.astype(np.int64) - 128
    r = y + ((91881 * x_cr + one_half) >> 16)
    gch = y + ((-22554 * x_cb + one_half - 46802 * x_cr) >> 16)
    b = y + ((116130 * x_cb + one_half) >> 16)
    return np.stack([np.clip(v, 0, 255) for v in (b, gch, r)], -1).astype(np.uint8)


def reconstruct(coefs, qt, g):
    """(coefficients, quantisation tables, geometry) of one image → uint8 [H,W,3] BGR."""
    planes = component_planes(coefs, qt, g)
    W, H = g["width"], g["height"]
    full = [upsample(planes[c], g["dw"][c], g["dh"][c], g["hmax"] // g["hs"][c], g["vmax"] // g["vs"][c], W, H)
            for c in range(g["ncomp"])]
    if g["ncomp"] == 1:
        return np.repeat(full[0].astype(np.uint8)[:, :, None], 3, axis=2)
    return ycc_to_bgr(*full)
