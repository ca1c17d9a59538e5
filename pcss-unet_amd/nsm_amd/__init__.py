"""nsm_amd — MI355X-native (gfx950) hot path of the PCSS-Unet Neural Shadow
Mapping U-Net: forward, backward, losses and train-step tail on hand-written
HIP kernels (libnsm.so), behind the reference's Python surface.

Importing this package loads libnsm.so and fails loudly if it is missing.
"""
from ._lib import LIB_PATH, NsmError, lib  # noqa: F401  (loads the HIP library)
from .unet import DoubleConv, Unet, reserve_side_stream  # noqa: F401
from .losses import (CustomLoss, EnhancedCustomLoss, L1Loss, PerturbationLoss,  # noqa: F401
                     l1_loss, measure_temporal_instability)
from .optim import FlatAdamW, allreduce_grads, flat_grad  # noqa: F401
from .infer import GraphedUnet  # noqa: F401
from .step import GraphedTrainStep  # noqa: F401
from .vgg import MultiLayerVGGLoss  # noqa: F401

__version__ = "0.1.0"
