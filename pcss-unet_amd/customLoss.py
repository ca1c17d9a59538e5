"""Drop-in replacement for the reference module `customLoss`
(/root/reference/customLoss.py:92-193): CustomLoss(device, alpha) returning
alpha*L1 + (1-alpha)*vgg with the exact reference gradient alpha*sign/N."""
from nsm_amd.losses import CustomLoss  # noqa: F401
