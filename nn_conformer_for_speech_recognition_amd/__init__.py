"""MI355X-native (gfx950 / CDNA4) Conformer encoder hot path.

Host code mirrors the reference's surface (lib.hparams.HParams, lib.standard.asrnn.ASRNN,
lib.standard.runner.Runner, lib.finetuning.finetune.FineTune, torchaudio's Conformer and the
reference's ConvSubSampling / SpecAugment); the hot path runs on hand-written HIP kernels in
libcfm.so behind the C ABI in include/cfm.h.
"""
__version__ = "0.1.0"

from . import library  # noqa: E402,F401  (registers torch.ops.cfm.*)
