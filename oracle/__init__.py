"""TEST INFRASTRUCTURE ONLY — the CPU oracle for the U-Net hot path.

This package is a PyTorch-CPU fp32 restatement of the reference's algorithm
(SDU-Gary/PCSS-Unet `Unetmodel.py`, `customLoss.py`, `pert_loss.py`,
`setdata.py`). It exists to CHECK the HIP path, never to run it:
only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg
may import it. The product path (`pcss-unet_amd/`) never imports it and fails
loudly when the HIP library is missing.

Pinning: `tests/golden/*.npz` were produced by running the reference's own
`Unetmodel.Unet` / `customLoss.CustomLoss` / `pert_loss.PerturbationLoss`
in the survey container (`tests/golden/make_golden.py`); `tests/test_oracle.py`
checks this restatement against every fixture.
"""
