"""analysis.py of the reference (analysis.py:1-43) on the MI355X path:
load a checkpoint (reference state_dict format), run every image of a folder
through Prediction, decode keypoints on the GPU and write the overlay grid.

    python analysis.py <checkpoint name under checkpoints/> <image dir>
    torchrun --nproc-per-node N analysis.py <ckpt> <image dir>      (data parallel)

Data parallel: each rank takes a contiguous slice of the sorted
file list (hkp.parallel.shard_range), writes its own overlays (preds/outNNNN.png,
NNNN = the image's index in the full list, as the single-GPU run names them),
and the int32 (y, x) keypoints of all images are all-gathered; rank 0 saves
them as preds/keypoints.npy ([n_images, K, 2], file order).  Images go through
one at a time (batch 1, train-mode BN — analysis.py:36-42), so results do not
depend on the GPU count.
"""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

from config import BACKBONE, IMG_HEIGHT, IMG_WIDTH, NUM_KEYPOINTS
from hkp import parallel
from src.dataset import imread_bgr, transform
from src.model import KeypointsGauss
from src.prediction import Prediction


def main(model_ckpt="", image_dir="", out_dir="preds", checkpoint_dir="checkpoints"):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    own_group = world > 1 and not dist.is_initialized()
    if world > 1:
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        if own_group:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    keypoints = KeypointsGauss(NUM_KEYPOINTS, img_height=IMG_HEIGHT, img_width=IMG_WIDTH, backbone=BACKBONE,
                               pretrained=False)
    keypoints.load_state_dict(torch.load(os.path.join(checkpoint_dir, model_ckpt), map_location="cpu",
                                         weights_only=True))
    use_cuda = torch.cuda.is_available()
    if use_cuda:
        if world == 1:
            torch.cuda.set_device(0)
        keypoints = keypoints.cuda()
    prediction = Prediction(keypoints, NUM_KEYPOINTS, IMG_HEIGHT, IMG_WIDTH, use_cuda)
    files = sorted(os.listdir(image_dir))
    lo, hi = parallel.shard_range(len(files), parallel.rank(), parallel.world())
    kps = []
    for i in range(lo, hi):
        img = imread_bgr(os.path.join(image_dir, files[i]))
        print(img.shape)
        img_t = transform(img).cuda()
        with torch.no_grad():
            heatmap, kp = keypoints.heatmaps_and_keypoints(img_t.view(-1, *img_t.shape))
        prediction.plot(img, heatmap.cpu().numpy(), image_id=i, keypoints=kp.cpu().numpy(), out_dir=out_dir)
        kps.append(kp[0])
    local_kp = torch.stack(kps) if kps else torch.zeros((0, NUM_KEYPOINTS, 2), dtype=torch.int32, device="cuda")
    all_kp = parallel.gather_keypoints(local_kp).cpu().numpy()
    if parallel.rank() == 0:
        os.makedirs(out_dir, exist_ok=True)
        np.save(os.path.join(out_dir, "keypoints.npy"), all_kp)
    if own_group:
        dist.destroy_process_group()
    return all_kp


if __name__ == "__main__":
    main(*sys.argv[1:3])
