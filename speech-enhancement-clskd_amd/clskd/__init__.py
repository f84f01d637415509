"""clskd — MI355X-native DCCRN + CLSKD (cross-layer similarity KD) hot path.

Drop-in counterparts of the reference modules (KhanhNguyen4999/Speech-Enhancement-CLSKD):
  DCCRN.py                -> clskd.model.DCCRN
  framework.py            -> clskd.framework (MultiResolutionSTFTLoss, SPKDLoss, ABF, ReviewKD,
                             build_review_kd)
  feature_extraction.py   -> clskd.feature_extraction.DCCRN
  tools_for_loss.py       -> clskd.tools_for_loss.si_snr
  distill.py              -> clskd.distill.KnowledgeDistillation (training_step)
  distill_SPKD.py         -> clskd.distill.SPKDDistillation
  config.py               -> clskd.config
A whole step can be captured and replayed as one hipGraph (clskd.graph.StepGraph).
All arithmetic runs in libclskd_hip.so (gfx950); there is no CPU fallback.
"""
from . import config  # noqa: F401
from .weights import recipe_state_dict  # noqa: F401


def __getattr__(name):
    # heavy modules (torch + the HIP library) load lazily
    if name in ("DCCRN",):
        from .model import DCCRN
        return DCCRN
    if name in ("KnowledgeDistillation", "SPKDDistillation", "clskd_step"):
        from . import distill
        return getattr(distill, name)
    if name in ("MultiResolutionSTFTLoss", "SPKDLoss", "build_review_kd", "ReviewKD", "ABF"):
        from . import framework
        return getattr(framework, name)
    if name == "StepGraph":
        from .graph import StepGraph
        return StepGraph
    raise AttributeError(name)
