"""HParams — the reference's hyper-parameter surface (lib/hparams.py:1-145), plus build knobs.

Same attribute names, defaults and setters as the reference so existing driver code keeps
working; the values are grouped by the subsystem that reads them.  Extra knobs for the
MI355X build (documented in DESIGN.md):

  compute_dtype          'bf16' | 'fp32'   dtype of activations / MFMA operands (fp32 = parity mode)
  frontend_proj          'utterance' | 'frame'   reference whole-utterance Linear (asrnn.py:28)
                                                  or per-subsampled-frame Linear (scalable)
  pos_enc                'none' | 'rel'    torchaudio MHSA or Transformer-XL relative positions
  specaug_ref_noop_masks bool              reproduce the reference's no-op masks (asrnn.py:141,165)
  dp_world_size          int               set by the data-parallel launcher
"""
from __future__ import annotations

import os
from math import inf  # noqa: F401  (the reference module exports it)

import torch

_PATHS = {  # lib/hparams.py:16-26 (relative to base_dir)
    "pretrained_model_path": ("model", "pretrained_weights.pth"),
    "standard_model_path": ("model", "standard_weights.pth"),
    "finetuning_model_path": ("model", "finetuning_weights.pth"),
    "lm_model_path": ("model", "lm_weights.pth"),
}

_OPTIMIZER = dict(beta1=0.9, beta=0.9, ngram=2, scale_parameter=False, relative_step=False, lr=2e-5,
                  pretraining_lr=3e-5)
_DATA = dict(batch_size=32, ntokens=1024, unk_tol=0.3, epochs=15, pretraining_epochs=100, hop_length=512,
             n_mels=40, read_mels=False, max_target_len=None, max_len=None, wpm=False,
             standard_train_type=["train-clean-360", "train-other-500"], librilight_subset="10h")
_FRONTEND = dict(pretraining_insize=1, pretraining_convsub_out_size=256, conv_sub_1_nodes=512, conv_sub_1_kernel=7,
                 conv_sub_1_stride=(2, 2), conv_sub_2_nodes=128, conv_sub_2_kernel=3, conv_sub_2_stride=(2, 2),
                 standard_linear_nodes=512)
_CONFORMER = dict(n_conformers=1, dropout=0.5, conformer_ff1_linear1_nodes=512, conformer_ff2_linear1_nodes=1024,
                  conformer_dropout=0.5, mhsa_num_heads=8, conformer_pointwise_conv1_nodes=1024,
                  conformer_pointwise_conv1_kernel=1, conformer_depthwise_conv_nodes=512,
                  conformer_depthwise_conv_kernel=33, conformer_depthwise_conv_stride=2,
                  conformer_pointwise_conv2_nodes=256, conformer_pointwise_conv2_kernel=1, conformer_size=1024,
                  rel_att=False, pretrained_conformer=False)
_PRETRAIN = dict(mask_probability=0.065, mask_value=0, target_context_vectors_size=320,
                 pretraining_conformer_out_size=64, pretraining_decoder_bidirectional=True,
                 pretraining_decoder_layers=1, encoded_features_out_size=128, mask_change_every_n_steps=10,
                 simplified_pretraining=True, alpha_loss=0.1, temperature_loss=0.1, distractors_K=5,
                 temperature_tau=2, do_pretraining=False, load_pretraining=False)
_DECODER = dict(standard_decoder_layers=1, standard_decoder_bidirectional=True, standard_decoder_nodes=512,
                projection_out_size=256, embedding_dim=64, extra_proj=False)
_SPECAUG = dict(warping_param_W=1, warping_ntimes=1, frequency_mask_param_F=5, frequency_mask_ntimes=2,
                time_multiplicity=2, pm=0.05, ps=0.05, time_mask_param_T=5, adaptive_multiplicity=False,
                adaptive_size=False)
_NST_LM = dict(nst=True, lm=False, train_lm=False, ft_lr=3e-6, ft_epochs=3, ft_train_epochs=1, lm_ntokens=256,
               lm_in_N=4, lm_out_N=4, input_embedding_size=320, lm_in_mhsa_num_heads=8, lm_out_mhsa_num_heads=8,
               lm_masked_out_mhsa_num_heads=8, lm_innner_input_nodes=512, lm_innner_output_nodes=512, lm_epochs=3,
               lm_max_len=20, just_nst=True)
_BUILD = dict(compute_dtype="bf16", frontend_proj="utterance", pos_enc="none", specaug_ref_noop_masks=False,
              dp_world_size=1, layer_norm_eps=1e-5, bn_eps=1e-5, bn_momentum=0.1)


class HParams:
    """Attribute bag with the reference's names (lib/hparams.py:14-145)."""

    def __init__(self, base_dir):
        self.base_dir = base_dir
        if base_dir is not None:
            self.data_dir = os.path.join(base_dir, "data")
            self.model_dir = os.path.join(base_dir, "model")
            self.plots_dir = os.path.join(base_dir, "results")
            for d in (self.model_dir, self.plots_dir):
                os.makedirs(d, exist_ok=True)
            for name, (sub, fn) in _PATHS.items():
                setattr(self, name, os.path.join(base_dir, sub, fn))
        self.device = torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")
        for group in (_OPTIMIZER, _DATA, _FRONTEND, _CONFORMER, _PRETRAIN, _DECODER, _SPECAUG, _NST_LM, _BUILD):
            for k, v in group.items():
                setattr(self, k, list(v) if isinstance(v, list) else v)
        # derived values (hparams.py: pretraining_linear_nodes, decoder_nodes, rel_pos_emb, ...)
        self.pretraining_linear_nodes = self.target_context_vectors_size
        self.decoder_nodes = (self.target_context_vectors_size // 2 if self.pretraining_decoder_bidirectional
                              else self.target_context_vectors_size)
        self.rel_pos_emb = self.rel_att
        self.output_embedding_size = self.input_embedding_size
        self.decoder_fc_nodes = self.projection_out_size

    # setters called by the dataset (speechcommands.py:39-46)
    def set_max_len(self, max_len):
        self.max_len = max_len

    def set_target_max_len(self, max_len):
        self.max_target_len = max_len

    def set_vocab_len(self, n):
        self.ntokens = n

    def set_standard_out_size(self, standard_out_size):
        self.standard_out_size = standard_out_size

    def set_input_dim(self, input_rows, input_cols):
        self.input_rows = input_rows
        self.input_cols = input_cols

    def set_space_index(self, space_idx):
        self.space_idx = space_idx

    def set_blank_index(self, blank_idx):
        self.blank_idx = blank_idx

    def set_ntokens(self, ntokens):
        self.ntokens = ntokens

    def set_max_value(self, max_value):
        self.max_value = int(max_value)
