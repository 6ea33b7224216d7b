"""spine_vision_amd -- MI355X (gfx950) training path for nghiant03/spine-vision.

Drop-in for the reference's training hot path: the timm-style backbone constructor
(``training.models.BackboneFactory``), ``CoordinateRegressor`` / ``Classifier``,
``LocalizationConfig`` / ``ClassificationConfig`` and ``Trainer.train()``, backed by hand-written
HIP kernels (``csrc/``, C ABI in ``include/sv_kernels.h``) and RCCL data parallelism.
"""

from . import native  # noqa: F401

__version__ = "0.1.0"
