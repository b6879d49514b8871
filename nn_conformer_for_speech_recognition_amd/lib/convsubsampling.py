"""ConvSubSampling — drop-in for the reference's lib/convsubsampling.py:5-45 on libcfm kernels.

Same constructor (hp, in_size, out_nodes), parameter names (conv_sub_1, conv_sub_2), ``out_size``
arithmetic (convsubsampling.py:24-32) and forward contract ((B, in_size, F, T) -> (B, C2, F', T')).
The MI355X path supports the reference's geometry (1 input channel, 7x7/s2 then 3x3/s2) and
raises NotImplementedError for anything else instead of silently falling back.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from ..frontend import conv_subsample


class ConvSubSampling(nn.Module):
    def __init__(self, hp, in_size, out_nodes):
        super().__init__()
        self.hp = hp
        self.conv_sub_1 = nn.Conv2d(in_size, hp.conv_sub_1_nodes, hp.conv_sub_1_kernel, stride=hp.conv_sub_1_stride)
        self.conv_sub_2 = nn.Conv2d(hp.conv_sub_1_nodes, out_nodes, hp.conv_sub_2_kernel,
                                    stride=hp.conv_sub_2_stride)
        geo_ok = (in_size == 1 and hp.conv_sub_1_kernel == 7 and tuple(hp.conv_sub_1_stride) == (2, 2)
                  and hp.conv_sub_2_kernel == 3 and tuple(hp.conv_sub_2_stride) == (2, 2)
                  and hp.conv_sub_1_nodes % 8 == 0 and hp.conv_sub_1_nodes <= 512 and out_nodes % 8 == 0)
        self._geo_ok = geo_ok
        h, w = hp.input_rows, hp.input_cols
        for k, (sh, sw) in ((hp.conv_sub_1_kernel, hp.conv_sub_1_stride), (hp.conv_sub_2_kernel, hp.conv_sub_2_stride)):
            h = (h - k + sh) // sh
            w = (w - k + sw) // sw
        self.out_size = out_nodes * h * w

    def _check(self):
        if not self._geo_ok:
            raise NotImplementedError("libcfm ConvSubSampling supports in_size=1, 7x7/s2 then 3x3/s2, channels % 8 == 0")

    def forward_frames(self, x, compute_dtype=torch.bfloat16):
        """x (B, 1, F, T) or (B, F, T) fp32 -> (B, T', F', C2) in the compute dtype (frame-major)."""
        self._check()
        if x.dim() == 4:
            x = x.reshape(x.shape[0], x.shape[2], x.shape[3])
        return conv_subsample(x.float().contiguous(), self.conv_sub_1.weight, self.conv_sub_1.bias,
                              self.conv_sub_2.weight, self.conv_sub_2.bias, compute_dtype)

    def forward(self, x, compute_dtype=torch.float32):
        """Reference contract (convsubsampling.py:34-45): returns (B, C2, F', T')."""
        return self.forward_frames(x, compute_dtype).permute(0, 3, 2, 1).float()
