"""TEST INFRASTRUCTURE ONLY -- the CPU parity oracle for the spine-vision MI355X training path.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this
package, and only as the checker / the timed CPU baseline.  The product (``spine-vision_amd/``) never
imports, links or executes anything from here; its kernels fail loudly when the HIP library is absent.

What it restates (fp32, PyTorch eager on CPU, NCHW):
  * ``convnext.py``  timm 1.0.22 ``timm/models/convnext.py`` ConvNeXt (num_classes=0) -- the backbone
    behind ``BackboneFactory.create`` (spine_vision/training/models/backbone.py:143-177).  timm is not
    vendored in the reference and not installed here; the restatement is cross-checked against the
    independent HF ``transformers`` ConvNext implementation (tests/golden/make_golden.py).
  * ``resnet.py``    timm ``timm/models/resnet.py`` ResNet-18/50 (BasicBlock / Bottleneck, v1.5).
  * ``heads.py``     CoordinateRegressor head + masked loss (spine_vision/training/models/generic.py:
    340-361, 380-417) and Classifier heads + multi-task loss (generic.py:98-177, core/tasks.py:142-221,
    trainers/classification.py:45-88).
  * ``step.py``      one training step of BaseTrainer/LocalizationTrainer._train_step
    (trainers/base.py:571-599, trainers/localization.py:186-209): zero_grad, forward, loss, backward,
    clip_grad_norm_(1.0), torch.optim.AdamW (base.py:384-390).
  * ``weights.py``   a counter-based deterministic parameter/input generator (splitmix64), so goldens
    can be regenerated bit-identically on the GPU box without shipping weights.

Parity pinning: see DESIGN.md "Oracle" -- head/loss/step pinned against the reference's own Python
(imported with shims in this container, fixtures in tests/golden/), backbone pinned against HF
transformers' ConvNext / ResNet.  The reference itself ships no tests or golden vectors.
"""
