"""MI355X-native restatement of src/dataset.py's call surface.

  transform         dataset.py:16   ToTensor: HWC uint8 (BGR, as cv2.imread gives) → CHW fp32 / 255
  gauss_2d_batch    dataset.py:36-44  the Gaussian target, computed by the HIP kernel
                    hkp_gauss_target (fp32 arithmetic, fp64 result, on the GPU like the
                    reference's .cuda() meshgrid)
  KeypointsDataset  dataset.py:52-79  same constructor, same (img, gaussians) items; with
                    return_uv=True items are (img, uv) so the fused loss kernel recomputes
                    the target in registers instead of reading a [K,H,W] fp64 tensor.
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
        for i in range(len(os.listdir(labels_folder))):
            label = np.load(os.path.join(labels_folder, "%05d.npy" % i)).reshape(num_keypoints, 2)
            label[:, 0] = np.clip(label[:, 0], 0, self.img_width - 1)      # dataset.py:65
            label[:, 1] = np.clip(label[:, 1], 0, self.img_height - 1)     # dataset.py:66
            self.imgs.append(os.path.join(img_folder, "%05d.jpg" % i))
            self.labels.append(torch.from_numpy(label).to(device))

    def __getitem__(self, index):
        img = self.transform(imread_bgr(self.imgs[index]))
        labels = self.labels[index]
        if self.return_uv:
            return img, labels.float()
        U = labels[:, 0]
        V = labels[:, 1]
        gaussians = gauss_2d_batch(self.img_width, self.img_height, self.gauss_sigma, U, V)
        return img, gaussians

    def __len__(self):
        return len(self.labels)
