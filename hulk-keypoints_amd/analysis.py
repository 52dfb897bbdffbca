"""analysis.py of the reference (analysis.py:1-43) on the MI355X path:
load a checkpoint (reference state_dict format), run every image of a folder
through Prediction, decode keypoints on the GPU and write the overlay grid.

    python analysis.py <checkpoint name under checkpoints/> <image dir>
"""
import os
import sys

import torch

from config import IMG_HEIGHT, IMG_WIDTH, NUM_KEYPOINTS, BACKBONE
from src.dataset import imread_bgr, transform
from src.model import KeypointsGauss
from src.prediction import Prediction


def main(model_ckpt="", image_dir=""):
    keypoints = KeypointsGauss(NUM_KEYPOINTS, img_height=IMG_HEIGHT, img_width=IMG_WIDTH, backbone=BACKBONE,
                               pretrained=False)
    keypoints.load_state_dict(torch.load("checkpoints/%s" % model_ckpt, map_location="cpu", weights_only=True))
    use_cuda = torch.cuda.is_available()
    if use_cuda:
        torch.cuda.set_device(0)
        keypoints = keypoints.cuda()
    prediction = Prediction(keypoints, NUM_KEYPOINTS, IMG_HEIGHT, IMG_WIDTH, use_cuda)
    for i, f in enumerate(sorted(os.listdir(image_dir))):
        img = imread_bgr(os.path.join(image_dir, f))
        print(img.shape)
        img_t = transform(img).cuda()
        with torch.no_grad():
            heatmap, kp = keypoints.heatmaps_and_keypoints(img_t.view(-1, *img_t.shape))
        prediction.plot(img, heatmap.cpu().numpy(), image_id=i, keypoints=kp.cpu().numpy())


if __name__ == "__main__":
    main(*sys.argv[1:3])
