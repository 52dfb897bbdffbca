"""Hybrid JPEG decode for the device data path (replaces the
reference's per-sample ``cv2.imread``, /root/reference/src/dataset.py:71).

The sequential half — marker parsing and Huffman entropy decoding of the
quantised DCT coefficients — runs on the host in ``libhkpjpeg.so`` (plain C,
no GPU runtime, so the loader's forked workers call it); the data-parallel
half — dequantisation, the 8x8 islow IDCT, fancy chroma upsampling and
YCbCr → BGR — runs on the GPU (``hkp_jpeg_reconstruct`` in libhulkkp.so).
The batch that comes out is uint8 [n, H, W, 3] BGR, bit-identical to
libjpeg-turbo's default decode (what cv2.imread and Pillow return).

    coefs, qt, geom = entropy_decode(open(path, "rb").read())       # host, any process
    img = reconstruct(coefs_dev, qt_dev, geom, n)                     # device

Files this decoder does not take (progressive, arithmetic-coded, 12-bit,
CMYK, multi-scan) raise ``JpegUnsupported``; the data loader then decodes
that file on the host instead (an input-format fallback, not a compute one).
"""
import ctypes
import os

import numpy as np
import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
HOST_LIB_PATH = os.path.join(_HERE, "libhkpjpeg.so")

HKPJ_OK, HKPJ_ERR_FORMAT, HKPJ_ERR_UNSUPPORTED, HKPJ_ERR_CORRUPT, HKPJ_ERR_ARG = 0, -1, -2, -3, -4


class JpegError(RuntimeError):
    pass


class JpegUnsupported(JpegError):
    """A valid JPEG outside the hybrid decoder's subset."""


class Geom(ctypes.Structure):
    """hkpj_geom (include/hkp_jpeg.h)."""
    _fields_ = [("width", ctypes.c_int32), ("height", ctypes.c_int32), ("ncomp", ctypes.c_int32),
                ("hs", ctypes.c_int32 * 3), ("vs", ctypes.c_int32 * 3), ("hmax", ctypes.c_int32),
                ("vmax", ctypes.c_int32), ("bw", ctypes.c_int32 * 3), ("bh", ctypes.c_int32 * 3),
                ("dw", ctypes.c_int32 * 3), ("dh", ctypes.c_int32 * 3), ("tq", ctypes.c_int32 * 3),
                ("restart_interval", ctypes.c_int32), ("blk_off", ctypes.c_int64 * 3), ("nblocks", ctypes.c_int64)]

    def key(self):
        """Fields two images must share to be reconstructed in one launch."""
        return (self.width, self.height, self.ncomp, tuple(self.hs), tuple(self.vs), tuple(self.bw),
                tuple(self.bh))

    def as_dict(self):
        return {f: (list(getattr(self, f)) if hasattr(getattr(self, f), "__len__") else getattr(self, f))
                for f, _ in self._fields_}


# name -> (restype, argtypes); every function include/hkp_jpeg.h declares
HOST_SIGNATURES = {
    "hkpj_probe": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int64, ctypes.POINTER(Geom)]),
    "hkpj_decode": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int64, ctypes.POINTER(Geom), ctypes.c_void_p,
                                   ctypes.c_void_p]),
    "hkpj_last_error": (ctypes.c_char_p, []),
}

_host = None


def host_lib():
    """libhkpjpeg.so (loaded once per process; raises if it is not built)."""
    global _host
    if _host is None:
        if not os.path.exists(HOST_LIB_PATH):
            raise RuntimeError("libhkpjpeg.so is not built (%s); run __graft_entry__.build()" % HOST_LIB_PATH)
        L = ctypes.CDLL(HOST_LIB_PATH)
        for name, (res, args) in HOST_SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype, fn.argtypes = res, args
        _host = L
    return _host


def _check(rc, what):
    if rc == HKPJ_OK:
        return
    msg = host_lib().hkpj_last_error().decode(errors="replace")
    if rc == HKPJ_ERR_UNSUPPORTED:
        raise JpegUnsupported("%s: %s" % (what, msg))
    raise JpegError("%s failed (rc=%d): %s" % (what, rc, msg))


def probe(data):
    """Geometry of the JPEG in `data` (bytes)."""
    g = Geom()
    _check(host_lib().hkpj_probe(data, len(data), ctypes.byref(g)), "hkpj_probe")
    return g


def entropy_decode(data):
    """bytes → (coefs int16 [nblocks, 64], qt uint16 [ncomp, 64], Geom) on the host."""
    g = probe(data)
    coefs = np.empty((g.nblocks, 64), np.int16)
    qt = np.empty((g.ncomp, 64), np.uint16)
    _check(host_lib().hkpj_decode(data, len(data), ctypes.byref(g), coefs.ctypes.data, qt.ctypes.data), "hkpj_decode")
    return coefs, qt, g


def planes_bytes(g):
    from ._lib import lib
    n = lib().hkp_jpeg_planes_bytes(ctypes.byref(g))
    if n < 0:
        raise JpegUnsupported("hkp_jpeg_planes_bytes: geometry not taken by the device kernels")
    return n


def reconstruct(coefs, qt, g, n=None, out=None):
    """Device coefficients int16 [n, nblocks, 64] (or [n*nblocks, 64]) and tables
    uint16 [n, ncomp, 64] of n same-geometry images → uint8 [n, H, W, 3] BGR on
    the same device, on the current stream."""
    from ._lib import call
    from .ops import _ptr, _stream
    if not (coefs.is_cuda and qt.is_cuda):
        raise JpegError("reconstruct: coefficients and tables must be on the GPU")
    if coefs.dtype != torch.int16 or qt.dtype != torch.int16 and qt.dtype != torch.uint16:
        raise JpegError("reconstruct: coefs int16, qt uint16 (or int16 bits) expected")
    n = coefs.numel() // (g.nblocks * 64) if n is None else n
    if coefs.numel() != n * g.nblocks * 64 or qt.numel() != n * g.ncomp * 64:
        raise JpegError("reconstruct: %d coefficients / %d table entries for %d images of %d blocks, %d components"
                        % (coefs.numel(), qt.numel(), n, g.nblocks, g.ncomp))
    coefs, qt = coefs.contiguous(), qt.contiguous()
    pb = planes_bytes(g)
    planes = torch.empty(n * pb, dtype=torch.uint8, device=coefs.device)
    if out is None:
        out = torch.empty((n, g.height, g.width, 3), dtype=torch.uint8, device=coefs.device)
    call("hkp_jpeg_reconstruct", n, ctypes.byref(g), _ptr(coefs), _ptr(qt), _ptr(planes), n * pb, _ptr(out),
         _stream())
    return out


def decode_files(paths, device="cuda"):
    """Convenience: files of one geometry → uint8 [n, H, W, 3] BGR on `device`."""
    parts = [entropy_decode(open(p, "rb").read()) for p in paths]
    g = parts[0][2]
    if any(p[2].key() != g.key() for p in parts):
        raise JpegError("decode_files: the images differ in geometry")
    coefs = torch.from_numpy(np.stack([p[0] for p in parts])).to(device)
    qt = torch.from_numpy(np.stack([p[1] for p in parts]).view(np.int16)).to(device)
    return reconstruct(coefs, qt, g, len(parts))
