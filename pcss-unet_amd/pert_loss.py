"""Drop-in replacement for the reference module `pert_loss`
(/root/reference/pert_loss.py:7-90): PerturbationLoss()(model, x, out)."""
from nsm_amd.losses import PerturbationLoss  # noqa: F401
