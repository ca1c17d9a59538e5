"""Drop-in replacement for the reference module `pert_loss`
(/root/reference/pert_loss.py): PerturbationLoss()(model, x, out) (:7-90),
EnhancedCustomLoss(device, alpha, perturb_weight) (:92-163, constructible
here: the reference's imports a VGGLoss customLoss.py does not define) and
measure_temporal_instability(frames, motion_vectors, alpha) (:166-199)."""
from nsm_amd.losses import (EnhancedCustomLoss, PerturbationLoss,  # noqa: F401
                            measure_temporal_instability)
