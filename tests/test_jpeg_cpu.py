"""Hybrid JPEG decode, host half + oracle (CPU): the C entropy decoder
(libhkpjpeg.so) followed by oracle/jpeg_ref.py's restatement of libjpeg-turbo's
islow IDCT / fancy upsampling / YCbCr→BGR must reproduce Pillow's decode
(libjpeg-turbo 3.1, the library behind the reference's cv2.imread,
dataset.py:71) pixel for pixel — over every supported subsampling, several
qualities, odd sizes, restart intervals and optimised Huffman tables.  This pins
the oracle that tests/test_gpu_jpeg.py holds the GPU kernels to."""
import ctypes
import io
import os
import re

import numpy as np
import pytest

from conftest import REPO

PIL = pytest.importorskip("PIL.Image")


def _image(h, w, seed, gray=False):
    """Smooth gradients + edges + noise: exercises DC, AC and clipping."""
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    base = np.stack([128 + 100 * np.sin(xx / (7 + 3 * c) + yy / (11 + c)) for c in range(3)], -1)
    base[h // 3:h // 2, :] = [250, 5, 128]                            # a hard edge, saturated colours
    img = np.clip(base + rng.normal(0, 18, base.shape), 0, 255).astype(np.uint8)
    return img[:, :, 0] if gray else img


def _jpeg(img, **kw):
    b = io.BytesIO()
    PIL.fromarray(img).save(b, "JPEG", **kw)
    return b.getvalue()


def _pil_bgr(data):
    with PIL.open(io.BytesIO(data)) as im:
        return np.asarray(im.convert("RGB"))[:, :, ::-1]


CASES = [
    # (h, w, gray, save kwargs)
    (48, 64, False, dict(quality=75, subsampling=2)),                  # 4:2:0
    (48, 64, False, dict(quality=75, subsampling=1)),                  # 4:2:2
    (48, 64, False, dict(quality=75, subsampling=0)),                  # 4:4:4
    (37, 53, False, dict(quality=90, subsampling=2)),                  # odd sizes, partial MCUs
    (37, 53, False, dict(quality=50, subsampling=1)),
    (23, 5, False, dict(quality=85, subsampling=2)),                   # chroma 3 wide: narrowest fancy case
    (9, 3, False, dict(quality=85, subsampling=2)),                    # chroma 2 wide: box upsampling
    (64, 80, False, dict(quality=95, subsampling=2, restart_marker_blocks=3)),
    (64, 80, False, dict(quality=60, subsampling=0, restart_marker_rows=1)),
    (48, 64, False, dict(quality=80, subsampling=2, optimize=True)),   # per-image Huffman tables
    (40, 56, False, dict(quality=100, subsampling=0)),                 # quantiser 1: large coefficients
    (37, 53, True, dict(quality=80)),                                  # grayscale
    (120, 160, False, dict(quality=92, subsampling=2)),
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: "%dx%d%s-%s" % (c[0], c[1], "g" if c[2] else "",
                                                                       "-".join("%s%s" % kv for kv in c[3].items())))
def test_entropy_decode_plus_oracle_equals_libjpeg(case):
    from hkp import jpeg
    from oracle import jpeg_ref
    h, w, gray, kw = case
    data = _jpeg(_image(h, w, h * w, gray), **kw)
    coefs, qt, g = jpeg.entropy_decode(data)
    assert (g.width, g.height, g.ncomp) == (w, h, 1 if gray else 3)
    got = jpeg_ref.reconstruct(coefs, qt, g.as_dict())
    ref = _pil_bgr(data)
    assert got.shape == ref.shape
    diff = np.abs(got.astype(int) - ref.astype(int))
    assert diff.max() == 0, "max diff %d at %s" % (diff.max(), np.unravel_index(diff.argmax(), diff.shape))


def test_geometry_fields():
    from hkp import jpeg
    g = jpeg.probe(_jpeg(_image(37, 53, 1), quality=80, subsampling=2))
    assert (g.hs[0], g.vs[0], g.hs[1], g.vs[1], g.hmax, g.vmax) == (2, 2, 1, 1, 2, 2)
    assert (g.bw[0], g.bh[0], g.bw[1], g.bh[1]) == (8, 6, 4, 3)       # MCU-padded grids (4 x 3 MCUs of 16x16)
    assert (g.dw[1], g.dh[1]) == (27, 19)
    assert g.nblocks == 8 * 6 + 2 * 4 * 3
    assert list(g.blk_off) == [0, 48, 60]


@pytest.mark.parametrize("kind", ["progressive", "truncated", "not_jpeg"])
def test_rejects(kind):
    from hkp import jpeg
    img = _image(32, 32, 3)
    if kind == "progressive":
        with pytest.raises(jpeg.JpegUnsupported, match="SOF2"):
            jpeg.entropy_decode(_jpeg(img, quality=80, progressive=True))
    elif kind == "truncated":
        data = _jpeg(img, quality=80)
        with pytest.raises(jpeg.JpegError):
            jpeg.entropy_decode(data[:100])
    else:
        with pytest.raises(jpeg.JpegError, match="SOI"):
            jpeg.entropy_decode(b"\x89PNG\r\n\x1a\n" + bytes(64))


def test_truncated_scan_reads_zeros_like_libjpeg():
    """Entropy-coded data cut short: the missing bits read as zeros (libjpeg's
    behaviour after a premature marker / end of data), no crash."""
    from hkp import jpeg
    data = _jpeg(_image(64, 64, 5), quality=85)
    cut = data[:len(data) * 2 // 3] + b"\xff\xd9"
    coefs, qt, g = jpeg.entropy_decode(cut)
    assert coefs.shape == (g.nblocks, 64)


def test_host_library_exports_header():
    from hkp import jpeg
    text = open(os.path.join(REPO, "include", "hkp_jpeg.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = set(re.findall(r"\b(hkpj_[a-z0-9_]+)\s*\(", text))
    assert names == set(jpeg.HOST_SIGNATURES)
    L = jpeg.host_lib()
    for n in names:
        assert hasattr(L, n)
    assert ctypes.sizeof(jpeg.Geom) == 4 * (3 + 3 + 3 + 2 + 3 * 5 + 1) + 4 + 8 * 4


def test_randomised_configs_equal_libjpeg():
    """40 seeded random (size, quality, subsampling, restart, optimise) draws."""
    from hkp import jpeg
    from oracle import jpeg_ref
    rng = np.random.default_rng(2024)
    for i in range(40):
        h, w = int(rng.integers(1, 90)), int(rng.integers(1, 90))
        kw = dict(quality=int(rng.integers(5, 101)), subsampling=int(rng.integers(0, 3)),
                  optimize=bool(rng.integers(0, 2)))
        if rng.integers(0, 3) == 0:
            kw["restart_marker_blocks"] = int(rng.integers(1, 9))
        gray = rng.integers(0, 6) == 0
        data = _jpeg(_image(h, w, 100 + i, gray), **kw)
        coefs, qt, g = jpeg.entropy_decode(data)
        got = jpeg_ref.reconstruct(coefs, qt, g.as_dict())
        ref = _pil_bgr(data)
        assert np.array_equal(got, ref), (i, h, w, gray, kw)


def test_device_batches_host_side_items(tmp_path):
    """DeviceBatches(decode="device")'s worker items and collate on the host: a
    batch of one geometry travels as coefficients; a batch holding a progressive
    file or a second geometry is decoded on the host (cv2/PIL) instead."""
    from src.dataset import KeypointsDataset, _CoefView, _collate_coef, transform
    os.makedirs(tmp_path / "images")
    os.makedirs(tmp_path / "labels")
    specs = [(48, 64, {}), (48, 64, {"quality": 55}), (48, 64, {"progressive": True}), (40, 64, {})]
    for i, (h, w, kw) in enumerate(specs):
        (tmp_path / "images" / ("%05d.jpg" % i)).write_bytes(_jpeg(_image(h, w, 40 + i), subsampling=2, **kw))
        np.save(tmp_path / "labels" / ("%05d.npy" % i), np.array([[1.0, 2.0]]))
    ds = KeypointsDataset(str(tmp_path / "images"), str(tmp_path / "labels"), 1, 48, 64, transform, device="cpu")
    view = _CoefView(ds)
    b = _collate_coef([view[0], view[1]])
    assert b[0] == "coef" and b[1].shape[0] == 2 and b[1].dtype.itemsize == 2 and b[2].shape == (2, 3, 64)
    b = _collate_coef([view[0], view[2]])
    assert b[0] == "img"
    for j, i in enumerate([0, 2]):
        assert np.array_equal(b[1][j].numpy(), _pil_bgr(open(ds.imgs[i], "rb").read()))
    # two image sizes cannot form one batch, exactly as on the host-decode path
    with pytest.raises(ValueError):
        _collate_coef([view[0], view[3]])


def test_corrupt_inputs_fail_cleanly():
    """Seeded byte flips, truncations and header garbage: every call either
    decodes or raises JpegError — never a crash or a read outside the buffer
    (the entropy decoder parses untrusted files in the loader workers)."""
    from hkp import jpeg
    rng = np.random.default_rng(9)
    bases = [_jpeg(_image(40, 56, 11), quality=80, subsampling=2),
             _jpeg(_image(33, 47, 12), quality=60, subsampling=0, restart_marker_blocks=2),
             _jpeg(_image(24, 24, 13, gray=True), quality=90, optimize=True)]
    outcomes = {"ok": 0, "error": 0}
    for i in range(600):
        b = bytearray(bases[i % len(bases)])
        kind = i % 3
        if kind == 0:
            for _ in range(int(rng.integers(1, 6))):
                b[int(rng.integers(2, len(b)))] = int(rng.integers(0, 256))
        elif kind == 1:
            b = b[:int(rng.integers(4, len(b)))]
        else:
            j = int(rng.integers(2, min(len(b), 200)))
            b[j:j + 8] = bytes(rng.integers(0, 256, 8).astype(np.uint8))
        try:
            coefs, qt, g = jpeg.entropy_decode(bytes(b))
            assert coefs.shape == (g.nblocks, 64)
            outcomes["ok"] += 1
        except jpeg.JpegError:
            outcomes["error"] += 1
    assert outcomes["ok"] > 0 and outcomes["error"] > 0, outcomes


def _drop_first_rst(data):
    """The JPEG with its first RSTn marker (FF D0..D7 inside the scan) removed."""
    sos = data.index(b"\xff\xda")
    for j in range(sos + 2, len(data) - 1):
        if data[j] == 0xFF and 0xD0 <= data[j + 1] <= 0xD7:
            return data[:j] + data[j + 2:]
    raise AssertionError("no restart marker")


def test_missing_rst_marker_falls_back_to_host_decode(tmp_path):
    """A file with one RST marker missing: the entropy decoder refuses it
    (JpegError: it does not resync), and DeviceBatches(decode="device")'s worker
    item falls back to the host decode — which, like cv2.imread, resyncs and
    still returns an image — instead of killing the loader worker."""
    from hkp import jpeg
    from src.dataset import KeypointsDataset, _CoefView, _collate_coef, transform
    good = _jpeg(_image(48, 64, 71), quality=85, subsampling=2, restart_marker_blocks=2)
    bad = _drop_first_rst(good)
    with pytest.raises(jpeg.JpegError):
        jpeg.entropy_decode(bad)
    ref = _pil_bgr(bad)                                   # libjpeg resyncs: an image comes back
    assert ref.shape == (48, 64, 3)
    os.makedirs(tmp_path / "images")
    os.makedirs(tmp_path / "labels")
    for i, d in enumerate([good, bad]):
        (tmp_path / "images" / ("%05d.jpg" % i)).write_bytes(d)
        np.save(tmp_path / "labels" / ("%05d.npy" % i), np.array([[1.0, 2.0]]))
    ds = KeypointsDataset(str(tmp_path / "images"), str(tmp_path / "labels"), 1, 48, 64, transform, device="cpu")
    view = _CoefView(ds)
    assert view[0][0] == "coef"
    item = view[1]
    assert item[0] == "img" and np.array_equal(item[1], ref)
    b = _collate_coef([view[0], view[1]])                 # the batch decodes on the host
    assert b[0] == "img" and np.array_equal(b[1][1].numpy(), ref)


def test_sos_segment_too_short_is_rejected():
    """An SOS whose length field covers no component bytes, at the very end of the
    buffer: rejected before any byte past the segment is read."""
    from hkp import jpeg
    data = _jpeg(_image(16, 16, 3), quality=80)
    sos = data.index(b"\xff\xda")
    for ln in (2, 3, 5):
        with pytest.raises(jpeg.JpegError, match="SOS"):
            jpeg.entropy_decode(data[:sos] + b"\xff\xda" + bytes([0, ln]) + bytes(max(0, ln - 2)))
