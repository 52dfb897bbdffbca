"""train.py of the reference (train.py:1-82) on the MI355X path.

Same ``forward(sample_batched, model)`` and ``fit(train_data, test_data, model,
epochs, checkpoint_path='')`` surface, same prints and checkpoint names
(model_2_1_<epoch>.pth every 2 epochs, reference state_dict keys).  The loss
is the fused HIP BCE kernel (bit-for-bit the math of nn.BCELoss on
pred.double(), train.py:21,25).

Data parallel: launch with ``torchrun --nproc-per-node N train.py``; each rank
takes a DistributedSampler shard, gradients are all-reduced over RCCL in
buckets overlapped with the backward kernels: the model's grad_ready hook hands
each gradient to hkp.train.GradBucketer as the backward produces it inside
loss.backward(), a full bucket's all-reduce starts right away, and
_reduce_grads only waits for the last ones.  Rank 0 prints and checkpoints.
"""
import os
import sys

import torch
import torch.distributed as dist
from torch.utils.data import DataLoader

from config import *  # noqa: F401,F403
from config import BACKBONE, GAUSS_SIGMA, IMG_HEIGHT, IMG_WIDTH, LOSS, NUM_KEYPOINTS, batch_size, epochs
from hkp import autograd as hkp_autograd
from hkp.train import GradBucketer, broadcast_state
from src.dataset import KeypointsDataset, transform
from src.model import KeypointsGauss

use_cuda = True
optimizer = None
keypoints = None
_bucketer = None


def _rank0():
    return not dist.is_initialized() or dist.get_rank() == 0


def forward(sample_batched, model):
    img, gt = sample_batched
    img = img.cuda(non_blocking=True)
    pred_gauss = model.forward(img)
    if gt.dim() == 3:   # (u, v) labels → the loss kernel recomputes the Gaussian target in registers
        return hkp_autograd.heatmap_loss(pred_gauss, uv=gt.cuda().float().contiguous(), sigma=GAUSS_SIGMA, kind=LOSS)
    return hkp_autograd.heatmap_loss(pred_gauss, target=gt.cuda().double().contiguous(), kind=LOSS)


def _reduce_grads(model):
    """After loss.backward(): wait for the bucket all-reduces the backward already
    launched (model.grad_ready = GradBucketer.ready) and point p.grad at the
    averaged buckets."""
    if _bucketer is None:
        return
    _bucketer.finish()


def setup_data_parallel(model, bucket_mb=32):
    """DP wiring (torchrun): every rank starts from rank 0's parameters and BN
    buffers, and the backward hands each gradient to the bucketer as soon as it
    exists (model.grad_ready), so bucket all-reduces overlap the backward."""
    global _bucketer
    broadcast_state(model)
    _bucketer = GradBucketer(list(model.parameters()), bucket_mb << 20)
    model.grad_ready = _bucketer.ready
    return _bucketer


def fit(train_data, test_data, model, epochs, checkpoint_path=""):
    for epoch in range(epochs):
        if hasattr(getattr(train_data, "sampler", None), "set_epoch"):
            train_data.sampler.set_epoch(epoch)
        train_loss = 0.0
        i_batch = 0
        for i_batch, sample_batched in enumerate(train_data):
            optimizer.zero_grad()
            loss = forward(sample_batched, model)
            loss.backward()
            _reduce_grads(model)
            optimizer.step()
            train_loss += loss.item()
            if _rank0():
                print("[%d, %5d] loss: %.3f" % (epoch + 1, i_batch + 1, loss.item()), end="")
                print("\r", end="")
        if _rank0():
            print("train loss:", train_loss / max(i_batch, 1))   # reference divides by i_batch (train.py:40)
        test_loss = 0.0
        i_batch = 0
        for i_batch, sample_batched in enumerate(test_data):
            loss = forward(sample_batched, model)
            test_loss += loss.item()
        if _rank0():
            print("test loss:", test_loss / max(i_batch, 1))
            if epoch % 2 == 0:
                torch.save(model.state_dict(), checkpoint_path + "/model_2_1_" + str(epoch) + ".pth")


def main(dataset_dir="", output_dir="checkpoints", workers=0):
    global optimizer, keypoints
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    save_dir = os.path.join(output_dir, dataset_dir)
    if _rank0():
        os.makedirs(save_dir, exist_ok=True)
    train_dataset = KeypointsDataset("data/%s/train/images" % dataset_dir, "data/%s/train/keypoints" % dataset_dir,
                                     NUM_KEYPOINTS, IMG_HEIGHT, IMG_WIDTH, transform, gauss_sigma=GAUSS_SIGMA,
                                     return_uv=True)
    test_dataset = KeypointsDataset("data/%s/test/images" % dataset_dir, "data/%s/test/keypoints" % dataset_dir,
                                    NUM_KEYPOINTS, IMG_HEIGHT, IMG_WIDTH, transform, gauss_sigma=GAUSS_SIGMA,
                                    return_uv=True)
    sampler = torch.utils.data.distributed.DistributedSampler(train_dataset) if world > 1 else None
    train_data = DataLoader(train_dataset, batch_size=batch_size, shuffle=sampler is None, sampler=sampler,
                            num_workers=workers)
    test_data = DataLoader(test_dataset, batch_size=batch_size, shuffle=True, num_workers=workers)
    keypoints = KeypointsGauss(NUM_KEYPOINTS, img_height=IMG_HEIGHT, img_width=IMG_WIDTH, backbone=BACKBONE).cuda()
    optimizer = torch.optim.Adam(keypoints.parameters(), lr=1.0e-4, weight_decay=1.0e-4)   # train.py:79
    if world > 1:
        setup_data_parallel(keypoints)
    fit(train_data, test_data, keypoints, epochs=epochs, checkpoint_path=save_dir)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main(*sys.argv[1:2])
