"""ASRNN — drop-in for the reference's lib/standard/asrnn.py:11-259 with the encoder on libcfm.

Hot path on HIP kernels: SpecAugment (one fused kernel, host draws in
the reference's order), ConvSubSampling (direct conv1 + implicit-GEMM conv2), the front-end
projection, the Conformer layers, the projection block, and the BiLSTM
decoder's recurrence (lstm.LSTM, csrc/lstm.hip).  Kept as torch modules: final_fc, log_softmax.

Front-end projection (hp.frontend_proj):
  'utterance'  the reference's whole-utterance Linear(out_size, d*max_len) (asrnn.py:28,207-209),
               incl. the length crop with its host sync (asrnn.py:211-215) — reference parity mode.
  'frame'      Linear(F'*C2, d) applied to every subsampled frame (features ordered (f', c2)),
               T_enc = T' frames, lengths from the subsampling arithmetic, no host sync — the
               scalable mode used for the Conformer-S/M/L configurations.
"""
from __future__ import annotations

import random
from math import floor  # noqa: F401

import torch
import torch.nn as nn

from ... import specaugment as _sa
from ...conformer import Conformer
from ...ctc import greedy_decode as _greedy_decode
from ...frontend import frame_frontend as _frame_frontend, linear as _linear, projection_block as _projection_block
from ...lstm import LSTM
from ..convsubsampling import ConvSubSampling

_DTYPES = {"bf16": torch.bfloat16, "fp32": torch.float32, torch.bfloat16: torch.bfloat16,
           torch.float32: torch.float32}


def subsampled_lengths(lens, hp):
    """Valid frames after the two strided convs (convsubsampling.py:30-31 arithmetic)."""
    k1, (s1, _) = hp.conv_sub_1_kernel, hp.conv_sub_1_stride
    k2, (s2, _) = hp.conv_sub_2_kernel, hp.conv_sub_2_stride
    return ((lens - k1 + s1) // s1 - k2 + s2) // s2


class ASRNN(nn.Module):
    def __init__(self, hp):
        super().__init__()
        self.hp = hp
        self.compute_dtype = _DTYPES[getattr(hp, "compute_dtype", "bf16")]
        self.frontend_proj = getattr(hp, "frontend_proj", "utterance")
        d = hp.standard_linear_nodes
        self.conv_sub_sampling = ConvSubSampling(hp, hp.pretraining_insize, hp.conv_sub_2_nodes)
        if self.frontend_proj == "utterance":
            self.standard_linear = nn.Linear(self.conv_sub_sampling.out_size, d * hp.max_len)
        elif self.frontend_proj == "frame":
            f2 = ((hp.input_rows - hp.conv_sub_1_kernel + hp.conv_sub_1_stride[0]) // hp.conv_sub_1_stride[0]
                  - hp.conv_sub_2_kernel + hp.conv_sub_2_stride[0]) // hp.conv_sub_2_stride[0]
            self.standard_linear = nn.Linear(f2 * hp.conv_sub_2_nodes, d)
        else:
            raise ValueError(f"frontend_proj must be 'utterance' or 'frame', got {self.frontend_proj!r}")
        self.conformers = Conformer(d, hp.mhsa_num_heads, hp.conformer_ff1_linear1_nodes, hp.n_conformers,
                                    hp.conformer_depthwise_conv_kernel, hp.dropout,
                                    pos_enc=getattr(hp, "pos_enc", "none"), compute_dtype=self.compute_dtype)
        self.projection_fc = nn.Linear(d, hp.projection_out_size)
        self.swish = nn.SiLU()
        self.projection_batch_norm = nn.BatchNorm1d(hp.projection_out_size)
        self.projection_fc_1 = nn.Linear(hp.projection_out_size, hp.projection_out_size)
        dec_layers = hp.standard_decoder_layers
        self.lstm = LSTM(hp.projection_out_size, hp.standard_decoder_nodes,
                            bidirectional=hp.standard_decoder_bidirectional, num_layers=dec_layers,
                            dropout=hp.dropout if dec_layers > 1 else 0.0)
        self.dropout = nn.Dropout(hp.dropout)
        dec_out = hp.standard_decoder_nodes * (2 if hp.standard_decoder_bidirectional else 1)
        self.final_fc = nn.Linear(dec_out, hp.ntokens)
        self.beta = torch.rand(1).to(hp.device)
        self.beta.requires_grad = True
        self.log_softmax = nn.LogSoftmax(-1)

    # ------------------------------------------------------------------ reference surface
    def predict(self, x):
        """Greedy labels (asrnn.py:48-58): argmax over the classes, on the device
        (cfm_ctc_greedy_decode: first maximum wins, exactly torch.argmax's rule)."""
        ids, _, _ = _greedy_decode(x.float() if x.dtype != torch.float32 else x, compact=False)
        return ids

    def conformer_blocks(self, x, lengths=None):
        """asrnn.py:60-71 (kept for API parity): x (B, T, d) through the Conformer layers in turn."""
        if lengths is None:
            lengths = torch.full((x.shape[0],), x.shape[1], dtype=torch.int32, device=x.device)
        return self.conformers(x, lengths)[0]

    def projection_block(self, x, finetuning=False):
        fc = self.projection_fc_1 if finetuning else self.projection_fc
        return _projection_block(x.float().contiguous(), fc, self.projection_batch_norm, self.training,
                                 self.compute_dtype)

    def _augment(self, x, tau, warps=True, freqs=True, times=True):
        hp = self.hp

        class _View:
            pass
        v = _View()
        for k in ("warping_param_W", "frequency_mask_param_F", "pm", "ps", "adaptive_multiplicity",
                  "adaptive_size", "time_mask_param_T"):
            setattr(v, k, getattr(hp, k))
        v.warping_ntimes = hp.warping_ntimes if warps else 0
        v.frequency_mask_ntimes = hp.frequency_mask_ntimes if freqs else 0
        v.time_multiplicity = hp.time_multiplicity if times else 0
        v.adaptive_multiplicity = hp.adaptive_multiplicity if times else False
        v.specaug_ref_noop_masks = getattr(hp, "specaug_ref_noop_masks", False)
        v.mask_value = hp.mask_value
        return _sa.spec_augment(x, tau, v, rng=random)

    def time_warping(self, x, tau):
        """asrnn.py:91-125 (x: (B, F, T))."""
        return self._augment(x.float(), tau, True, False, False)

    def frequency_masking(self, x):
        """asrnn.py:127-144 (draws f, f0; masks applied unless specaug_ref_noop_masks)."""
        tau = [x.shape[-1]] * x.shape[0]
        return self._augment(x.float(), tau, False, True, False)

    def time_masking(self, x, tau):
        """asrnn.py:146-168."""
        return self._augment(x.float(), tau, False, False, True)

    def SpecAugment(self, x, tau):
        """asrnn.py:170-192 — (B, 1, F, T) in, (B, 1, F, T) out; one fused kernel."""
        xs = x.reshape(x.shape[0], x.shape[-2], x.shape[-1])
        return self._augment(xs.float(), tau).unsqueeze(1)

    # ------------------------------------------------------------------ encoder (hot path)
    def encoder(self, x, input_lens, SpecAugment=False, finetuning=False):
        hp = self.hp
        cd = self.compute_dtype
        if SpecAugment:
            x = self.SpecAugment(x, input_lens)
        B = x.shape[0]
        p = hp.dropout if self.training else 0.0
        if self.frontend_proj == "frame":
            # ConvSubSampling -> per-frame Linear -> dropout as ONE folded GEMM (frontend.frame_frontend)
            h = _frame_frontend(self.conv_sub_sampling, self.standard_linear, x, cd, drop_p=p,
                                seed=random.getrandbits(31))
            T2 = h.shape[0] // B
            lens = subsampled_lengths(input_lens.to(h.device).long(), hp)
            lens_i32 = lens.clamp(min=1).to(torch.int32)
            y = self.conformers.forward_tokens(h, lens_i32, B, T2)
            out = self.projection_block(y)
            if finetuning and hp.extra_proj:
                out = self.projection_block(self.dropout(out), True)
            return out, lens
        # 'utterance' (reference-literal) path
        h2 = self.conv_sub_sampling.forward_frames(x, cd)
        feats = h2.permute(0, 3, 2, 1).reshape(B, -1)                          # NCHW flatten order
        h = _linear(feats, self.standard_linear.weight, self.standard_linear.bias, cd=cd, drop_p=p,
                    seed=random.getrandbits(31))
        h = h.view(B, hp.max_len, h.shape[1] // hp.max_len)
        nz = input_lens.gt(0)
        lens = torch.masked_select(input_lens, nz)
        h = h[:lens.shape[0], :int(torch.max(lens).item())]
        y, output_lens = self.conformers(h.contiguous(), lens)
        y = nn.functional.pad(y, (0, 0, 0, hp.max_len - y.shape[1], 0, B - lens.shape[0]))
        y = y.flatten(0, 1)
        out = self.projection_block(y)
        if finetuning and hp.extra_proj:
            out = self.projection_block(self.dropout(out), True)
        return out, output_lens

    def decoder(self, y):
        raise NotImplementedError("ASRNN.decoder is dead code in the reference (asrnn.py:223-236 uses "
                                  "undefined decoder_fc/relu)")

    def forward(self, x, input_lens, SpecAugment=False, lm=None, finetuning=False):
        """asrnn.py:237-259: (B, F, T) mels -> log-probs (B, T_enc, ntokens), output lengths."""
        B = x.shape[0]
        x = x.unsqueeze(1)
        x, output_lens = self.encoder(x, input_lens, SpecAugment, finetuning=finetuning)
        x = self.lstm(x)[0]
        x = self.dropout(x)
        x = self.final_fc(x)
        x = x.view((B, x.shape[0] // B, self.hp.ntokens))
        x = self.log_softmax(x)
        if lm is not None:
            x = x + lm(self.hp.ngram, torch.argmax(x, -1))
        return x, output_lens
