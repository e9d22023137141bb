"""poor_man_gplvm_amd: MI355X-native engine for the PoissonGPLVMJump1D EM hot path
of poor-man-GPLVM (drop-in for `poor_man_gplvm.PoissonGPLVMJump1D`).

The compute path is libpmg_hip.so (hand-written gfx950 HIP kernels behind the C ABI
in include/pmg.h); PyTorch provides device memory, streams and torch.distributed.
"""
__version__ = "0.1.0"

from .core import (GaussianGPLVM1D, GaussianGPLVMJump1D, PoissonGPLVM1D, PoissonGPLVMJump1D,  # noqa: F401
                   compute_transition_posterior_prob,
                   compute_transition_posterior_prob_latent, fit_em_restarts, run_em,
                   run_em_restarts)
from .engine import AdamConfig, ScanConfig  # noqa: F401
from .gp_kernel import banded_transition, create_transition_prob_1d, generate_basis  # noqa: F401
from . import model_selection_helper, test  # noqa: F401
