"""MI355X-native restatement of src/dataset.py's call surface.

  transform         dataset.py:16   ToTensor: HWC uint8 (BGR, as cv2.imread gives) → CHW fp32 / 255
  gauss_2d_batch    dataset.py:36-44  the Gaussian target, computed by the HIP kernel
                    hkp_gauss_target (fp32 arithmetic, fp64 result, on the GPU like the
                    reference's .cuda() meshgrid)
  KeypointsDataset  dataset.py:52-79  same constructor, same (img, gaussians) items; with
                    return_uv=True items are (img, uv) so the fused loss kernel recomputes
                    the target in registers instead of reading a [K,H,W] fp64 tensor.
  DeviceBatches     SURVEY §8(f1): the device data path — images decoded by `workers`
                    DataLoader processes (the reference decodes one image at a time in
                    the training process, dataset.py:71 with num_workers=0,
                    train.py:51), batched as uint8 HWC in pinned host memory, copied
                    asynchronously (3 B/pixel instead of the 12 B/pixel fp32 tensor,
                    one batch ahead on a side stream) and fed to the model as
                    [B,H,W,3] uint8, where the stem's operand pack applies ToTensor;
                    labels travel as (u, v) and the loss kernel makes the target.
"""
import os

import numpy as np
import torch
import torch.nn.functional as F
from torch.utils.data import Dataset

from hkp import ops


def _to_tensor(img):
    """torchvision ToTensor semantics for an HWC uint8 array."""
    a = np.asarray(img)
    if a.ndim == 2:
        a = a[:, :, None]
    t = torch.from_numpy(np.ascontiguousarray(a.transpose(2, 0, 1)))
    return t.to(torch.float32).div_(255.0) if a.dtype == np.uint8 else t.to(torch.float32)


class Compose:
    def __init__(self, transforms):
        self.transforms = transforms

    def __call__(self, x):
        for t in self.transforms:
            x = t(x)
        return x


# No domain randomization (dataset.py:15-16)
transform = Compose([_to_tensor])


def imread_bgr(path):
    """cv2.imread (BGR uint8 HWC) when OpenCV is installed, else PIL converted to BGR."""
    try:
        import cv2  # noqa: F401
        img = cv2.imread(path)
        if img is None:
            raise FileNotFoundError(path)
        return img
    except ImportError:
        from PIL import Image
        with Image.open(path) as im:
            return np.asarray(im.convert("RGB"))[:, :, ::-1].copy()


def normalize(x):
    return F.normalize(x, p=1)


def gauss_2d_batch(width, height, sigma, U, V, normalize_dist=False):
    """[K] U (column) and V (row) → [K, height, width] float64 Gaussians on the GPU.

    Same values as dataset.py:36-44 (exp in fp32, then .double()); unlike the
    reference it does not mutate U/V in place (dataset.py:37-38)."""
    dev = U.device if torch.is_tensor(U) and U.is_cuda else torch.device("cuda")
    u = torch.as_tensor(U).reshape(-1).to(dev, torch.float32)
    v = torch.as_tensor(V).reshape(-1).to(dev, torch.float32)
    uv = torch.stack([u, v], -1).reshape(1, -1, 2).contiguous()
    G = ops.gauss_target(uv, height, width, sigma)[0]
    if normalize_dist:
        return normalize(G.float()).double()
    return G


def vis_gauss(gaussians):
    """dataset.py:46-50: min-max normalised first Gaussian → test.png."""
    g = gaussians[0].detach().cpu().numpy()
    g = (g - g.min()) / max(g.max() - g.min(), 1e-12) * 255.0
    from PIL import Image
    Image.fromarray(g.astype(np.uint8)).save("test.png")


class KeypointsDataset(Dataset):
    def __init__(self, img_folder, labels_folder, num_keypoints, img_height, img_width, transform, gauss_sigma=8,
                 return_uv=False, device="cuda"):
        self.num_keypoints = num_keypoints
        self.img_height = img_height
        self.img_width = img_width
        self.gauss_sigma = gauss_sigma
        self.transform = transform
        self.return_uv = return_uv
        self.imgs = []
        self.labels = []
        self.labels_np = []           # host copies (DataLoader workers never touch the device)
        for i in range(len(os.listdir(labels_folder))):
            label = np.load(os.path.join(labels_folder, "%05d.npy" % i)).reshape(num_keypoints, 2)
            label[:, 0] = np.clip(label[:, 0], 0, self.img_width - 1)      # dataset.py:65
            label[:, 1] = np.clip(label[:, 1], 0, self.img_height - 1)     # dataset.py:66
            self.imgs.append(os.path.join(img_folder, "%05d.jpg" % i))
            self.labels.append(torch.from_numpy(label).to(device))
            self.labels_np.append(label.astype(np.float32))

    def __getitem__(self, index):
        img = self.transform(imread_bgr(self.imgs[index]))
        labels = self.labels[index]
        if self.return_uv:
            return img, labels.float()
        U = labels[:, 0]
        V = labels[:, 1]
        gaussians = gauss_2d_batch(self.img_width, self.img_height, self.gauss_sigma, U, V)
        return img, gaussians

    def raw(self, index):
        """(uint8 [H,W,3] BGR image as cv2.imread gives, fp32 [K,2] (u, v) on the device)."""
        return imread_bgr(self.imgs[index]), self.labels[index].float()

    def __len__(self):
        return len(self.labels)


class _RawView(Dataset):
    """(uint8 [H,W,3] BGR, float32 [K,2]) host items of a KeypointsDataset — what
    DeviceBatches' decode workers produce."""

    def __init__(self, ds):
        self.paths, self.labels = ds.imgs, ds.labels_np

    def __len__(self):
        return len(self.paths)

    def __getitem__(self, i):
        return imread_bgr(self.paths[i]), self.labels[i]


class _CoefView(Dataset):
    """Decode-worker items for DeviceBatches(decode="device"): the host half of the
    hybrid JPEG decode (hkp.jpeg.entropy_decode: quantised DCT coefficients and
    tables), or the host-decoded image for a file outside that decoder's subset."""

    def __init__(self, ds):
        self.paths, self.labels = ds.imgs, ds.labels_np

    def __len__(self):
        return len(self.paths)

    def __getitem__(self, i):
        from hkp import jpeg
        path = self.paths[i]
        try:
            with open(path, "rb") as f:
                coefs, qt, g = jpeg.entropy_decode(f.read())
        except jpeg.JpegError:
            # outside the decoder's subset (JpegUnsupported) or damaged (a missing
            # RST marker, a bad Huffman code): the host decode, which like
            # cv2.imread (dataset.py:71) resyncs / zero-fills and still returns an
            # image, takes this file
            jpeg.host_lib()                  # ... but a missing library is a setup error, not a file's
            return ("img", imread_bgr(path), self.labels[i], path)
        return ("coef", (coefs, qt, bytes(g)), self.labels[i], path)


def _collate_coef(items):
    """One batch of _CoefView items: ("coef", coefs int16 [B,nblocks,64], qt
    [B,ncomp,64], geometry bytes, uv) when every image went through the entropy
    decoder with one geometry, else ("img", uint8 [B,H,W,3], uv) decoded on the host."""
    from hkp import jpeg
    uv = torch.from_numpy(np.stack([it[2] for it in items]))
    if all(it[0] == "coef" for it in items):
        geoms = [jpeg.Geom.from_buffer_copy(it[1][2]) for it in items]
        if all(g.key() == geoms[0].key() for g in geoms):
            coefs = torch.from_numpy(np.stack([it[1][0] for it in items]))
            qt = torch.from_numpy(np.stack([it[1][1] for it in items]).view(np.int16))
            return ("coef", coefs, qt, items[0][1][2], uv)
    imgs = [it[1] if it[0] == "img" else imread_bgr(it[3]) for it in items]
    return ("img", torch.from_numpy(np.stack(imgs)), uv)


class _EpochBatches:
    """Batch sampler of the persistent decode loader: the current epoch's index
    batches (set by DeviceBatches before each epoch; iterated in the main process)."""

    def __init__(self):
        self.batches = []

    def __iter__(self):
        return iter(self.batches)

    def __len__(self):
        return len(self.batches)


def _collate_u8(items):
    imgs = torch.from_numpy(np.stack([it[0] for it in items]))
    uv = torch.from_numpy(np.stack([it[1] for it in items]))
    return imgs, uv


class DeviceBatches:
    """Iterate a KeypointsDataset as device batches (img uint8 [B,H,W,3], uv fp32
    [B,K,2]) for model.forward / Trainer.step(img, uv=uv).

    decode="host": images are decoded on the host (cv2 / PIL, as the reference).
    decode="device": the hybrid JPEG decode (hkp.jpeg) — the host only
    entropy-decodes the quantised DCT coefficients; they are copied (about the
    size of the decoded image) and the IDCT, upsampling and colour conversion run
    on the GPU on the copy stream, bit-identical to the host decode.  Files
    outside that decoder's subset (progressive, CMYK, ...) and batches of mixed
    geometry are decoded on the host instead.

    Host work runs in the calling thread (workers=0), or in `workers` DataLoader
    processes that decode and stack whole batches ahead (`prefetch` batches per
    worker) into pinned memory.  Each batch is copied with non_blocking=True on a
    side stream while the previous batch computes; the consumer's stream waits on
    an event.  `shuffle` uses a seeded permutation per epoch (train.py:61-67
    shuffles); batches come in order for any worker count."""

    def __init__(self, dataset, batch_size, shuffle=False, seed=0, drop_last=False, device="cuda", workers=0,
                 prefetch=4, decode="host"):
        if decode not in ("host", "device"):
            raise ValueError("decode must be 'host' or 'device', got %r" % (decode,))
        self.ds, self.bs, self.shuffle, self.seed, self.drop_last = dataset, batch_size, shuffle, seed, drop_last
        self.device = torch.device(device)
        self.workers, self.prefetch, self.decode = workers, prefetch, decode
        self.epoch = 0
        self._loader = None
        self._sampler = _EpochBatches()

    def __len__(self):
        n = len(self.ds)
        return n // self.bs if self.drop_last else (n + self.bs - 1) // self.bs

    def _host_batches(self, batches):
        """Per index batch, in order: ("img", pinned uint8 [B,H,W,3], float32 [B,K,2])
        or (decode="device") ("coef", pinned coefs, pinned qt, geometry bytes, uv)."""
        view, collate = ((_RawView(self.ds), _collate_u8) if self.decode == "host"
                         else (_CoefView(self.ds), _collate_coef))
        if self.workers <= 0:
            for idx in batches:
                yield self._tag(collate([view[i] for i in idx]))
            return
        if self._loader is None:               # persistent workers: started once, reused every epoch
            from torch.utils.data import DataLoader
            self._loader = DataLoader(view, batch_sampler=self._sampler, num_workers=self.workers,
                                      collate_fn=collate, pin_memory=True, prefetch_factor=self.prefetch,
                                      persistent_workers=True)
        self._sampler.batches = [list(map(int, b)) for b in batches]
        for b in self._loader:
            yield self._tag(b)

    def _tag(self, b):
        """Host batches in one form, tensors pinned (the loader pins them already)."""
        if self.decode == "host":
            imgs, uv = b
            return ("img", imgs if imgs.is_pinned() else imgs.pin_memory(), uv)
        if b[0] == "img":
            return ("img", b[1] if b[1].is_pinned() else b[1].pin_memory(), b[2])
        return tuple(t.pin_memory() if torch.is_tensor(t) and not t.is_pinned() else t for t in b)

    def __iter__(self):
        n = len(self.ds)
        order = (np.random.default_rng(self.seed + self.epoch).permutation(n) if self.shuffle else np.arange(n))
        self.epoch += 1
        batches = [order[i:i + self.bs] for i in range(0, n, self.bs)]
        if self.drop_last and batches and len(batches[-1]) < self.bs:
            batches.pop()
        copy_stream = torch.cuda.Stream(self.device)
        host = self._host_batches(batches)

        def stage():
            b = next(host)
            with torch.cuda.stream(copy_stream):
                if b[0] == "img":
                    buf, uv = b[1], b[2]
                    img = buf.to(self.device, non_blocking=True)
                else:                          # hybrid decode: coefficients up, pixels made on the device
                    from hkp import jpeg
                    _, coefs, qt, gbytes, uv = b
                    buf = (coefs, qt)
                    g = jpeg.Geom.from_buffer_copy(gbytes)
                    img = jpeg.reconstruct(coefs.to(self.device, non_blocking=True),
                                           qt.to(self.device, non_blocking=True), g, coefs.shape[0])
                uvd = uv.to(self.device, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(copy_stream)
            return img, uvd, ev, buf

        nxt = stage() if batches else None
        for bi in range(len(batches)):
            img, uv, ev, buf = nxt
            nxt = stage() if bi + 1 < len(batches) else None
            cur = torch.cuda.current_stream(self.device)
            cur.wait_event(ev)
            img.record_stream(cur)
            uv.record_stream(cur)
            yield img, uv
