"""Drop-in mirror of the reference's src/ package (model, resnet, resnet_dilated, dataset, prediction)."""
