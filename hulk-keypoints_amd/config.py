"""config.py of the reference (config.py:1-6), same names and defaults.

Additive keys (defaults reproduce the reference): BACKBONE, LOSS
('bce' is what train.py:25 uses; 'mse' is train.py:13's unused MSE).
"""
NUM_KEYPOINTS = 4
IMG_HEIGHT = 480
IMG_WIDTH = 640
GAUSS_SIGMA = 8
epochs = 25
batch_size = 4

BACKBONE = "resnet34"
LOSS = "bce"
