"""MI355X-native batched Bayesian-network inference (drop-in for VBN's MCM / IS / LW / RB /
RIS / ancestral path and the gaussian_nn / linear_gaussian / mdn / kde / softmax_nn CPDs).

Importing the package does not touch the GPU; the HIP library is loaded on first use and
the accelerated entry points raise if it is missing (there is no CPU fallback).
"""
from .registry import INFERENCE_REGISTRY, SAMPLING_REGISTRY  # noqa: F401
from .engines import (  # noqa: F401
    AncestralSampler,
    ImportanceSampling,
    LikelihoodWeighting,
    MonteCarloMarginalization,
    Query,
    RaoBlackwellizedMarginalization,
    ResampledImportanceSampling,
)
from .model import BNModel, CPDRecord, model_from_checkpoint, model_from_vbn, random_init_model  # noqa: F401
from .api import VBN, ConfigItem, defaults  # noqa: F401

__version__ = "0.1.0"
