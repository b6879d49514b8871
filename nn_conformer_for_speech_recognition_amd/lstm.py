"""BiLSTM decoder on libcfm — drop-in for the reference's `nn.LSTM` decoder.

Reference: /root/reference/lib/standard/asrnn.py:38 builds
`nn.LSTM(projection_out_size, standard_decoder_nodes, bidirectional=..., num_layers=..., dropout=...)` and
:252 calls it on the 2-D encoder output (B*T_enc, 256), which torch treats as ONE unbatched sequence of
L = B*T_enc steps.  This module keeps torch's parameter names (weight_ih_l0,
weight_hh_l0, bias_ih_l0, bias_hh_l0 and the `_reverse` set) so checkpoints load either way, and torch's
`(output, (h_n, c_n))` return.

Per layer: gx = x W_ih^T + b_ih + b_hh for both directions in one fp32 cfm_gemm; the recurrence in one
cooperative launch (cfm_lstm_fwd, csrc/lstm.hip: W_hh held in registers across the whole sequence,
h_t exchanged through HBM as tagged 64-bit words polled directly, both directions concurrently).  Backward: the
reverse-time recurrence (cfm_lstm_bwd) produces the pre-activation gate gradients dG (L, ndir*4H); dx,
dW_ih, dW_hh (time-shifted views of dG and y, no copies) and the bias gradient are cfm_gemm / cfm_colsum.
Everything computes in fp32, like the reference.

Not supported (raise): batched 3-D input, an initial state hx (the reference passes neither).  c_n is
returned without a gradient path (the reference discards the state tuple).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib as L
from . import ops


def _wgrad_strided(a, lda, b, ldb, M, N, K, out):
    """out (M, N) fp32 = sum_k a[k, :M] (x) b[k, :N] over K rows of row-stride lda / ldb (views allowed)."""
    tiles = ((M + 127) // 128) * ((N + 127) // 128)
    split_k = max(1, min(16, 512 // max(tiles, 1), K // 1024))
    ws = torch.empty(split_k * M * N, device=out.device, dtype=torch.float32) if split_k > 1 else None
    return ops.gemm(a, b, out, M, N, K, a_kmajor=False, b_kmajor=False, lda=lda, ldb=ldb, split_k=split_k,
                    workspace=ws)


class _ErrorFlags:
    """Sticky device-side record of the recurrence kernels' wait-limit flags, checked WITHOUT a host sync per
    launch (a per-layer .item() would stall the host queue every pass and cannot run inside a HIP-graph
    capture).  note() folds a launch's flag into a persistent device word (stream-ordered max, capturable);
    poll() copies that word to pinned host memory behind an event and raises once a completed copy shows a
    set flag -- at the next forward, i.e. one step late, never blocking; sync_check() waits and raises now."""

    def __init__(self):
        self.dev = {}
        self.host = {}
        self.event = {}

    def _word(self, device):
        key = str(device)
        if key not in self.dev:
            self.dev[key] = torch.zeros(1, dtype=torch.int32, device=device)
        return self.dev[key]

    def note(self, ws, idx):
        w = self._word(ws.device)
        torch.maximum(w, ws[idx:idx + 1], out=w)

    def poll(self, device):
        """Raise if a finished earlier copy saw a set flag; then (outside capture) start a fresh async copy."""
        key = str(device)
        ev = self.event.get(key)
        if ev is not None and ev.query() and int(self.host[key][0]) != 0:
            self.host[key][0] = 0
            self.dev[key].zero_()
            raise L.CfmError("cfm_lstm_fwd/bwd: a step wait exceeded its limit (workgroups not co-resident?)")
        if torch.cuda.is_current_stream_capturing() or key not in self.dev:
            return
        if key not in self.host:
            self.host[key] = torch.zeros(1, dtype=torch.int32).pin_memory()
        self.host[key].copy_(self.dev[key], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self.event[key] = ev

    def sync_check(self, device):
        key = str(device)
        if key in self.dev and int(self.dev[key].item()) != 0:
            self.dev[key].zero_()
            raise L.CfmError("cfm_lstm_fwd/bwd: a step wait exceeded its limit (workgroups not co-resident?)")


ERRORS = _ErrorFlags()


class _LSTMLayer(torch.autograd.Function):
    """One (bi)directional layer over an unbatched sequence x (L, In) fp32."""

    @staticmethod
    def forward(ctx, x, w_ih, w_hh, bias, H, ndir):
        Lseq = x.shape[0]
        dev = x.device
        gx = ops.linear(x, w_ih, bias=bias)                        # (L, ndir*4H)
        y = torch.empty(Lseq, ndir * H, device=dev, dtype=torch.float32)
        gates = torch.empty(Lseq, ndir * 4 * H, device=dev, dtype=torch.float32)
        c = torch.empty(Lseq, ndir * H, device=dev, dtype=torch.float32)
        ws = torch.empty(L.size_call("cfm_lstm_ws_bytes", H, ndir) // 4, device=dev, dtype=torch.int32)
        L.call("cfm_lstm_fwd", L.ptr(gx), L.ptr(w_hh), L.ptr(y), L.ptr(gates), L.ptr(c), Lseq, H, ndir, L.ptr(ws),
               L.stream())
        ERRORS.note(ws, 0)
        ctx.save_for_backward(x, w_ih, w_hh, y, gates, c)
        ctx.H, ctx.ndir, ctx.ws = H, ndir, ws
        ctx.mark_non_differentiable(c)
        return y, c

    @staticmethod
    def backward(ctx, dy, _dc):
        x, w_ih, w_hh, y, gates, c = ctx.saved_tensors
        H, ndir, ws = ctx.H, ctx.ndir, ctx.ws
        Lseq, In = x.shape
        H4 = 4 * H
        dy = dy.float().contiguous()
        dg = torch.empty(Lseq, ndir * H4, device=x.device, dtype=torch.float32)
        L.call("cfm_lstm_bwd", L.ptr(dy), L.ptr(w_hh), L.ptr(gates), L.ptr(c), L.ptr(dg), Lseq, H, ndir, L.ptr(ws),
               L.stream())
        ERRORS.note(ws, 1)
        dx = ops.linear_dgrad(dg, w_ih) if ctx.needs_input_grad[0] else None
        dw_ih = ops.linear_wgrad(dg, x)
        db = ops.colsum(dg)
        dw_hh = torch.zeros(ndir * H4, H, device=x.device, dtype=torch.float32)
        if Lseq > 1:
            ldg, ldy = ndir * H4, ndir * H
            # forward direction: h_{t-1} = y[t-1] feeds step t; reverse: h_{t+1} = y[t+1] feeds step t
            _wgrad_strided(dg[1:], ldg, y[:-1], ldy, H4, H, Lseq - 1, dw_hh[:H4])
            if ndir == 2:
                _wgrad_strided(dg[:-1, H4:], ldg, y[1:, H:], ldy, H4, H, Lseq - 1, dw_hh[H4:])
        return dx, dw_ih, dw_hh, db, None, None


class LSTM(nn.Module):
    """torch.nn.LSTM surface (unbatched 2-D input, zero initial state) on the libcfm recurrence."""

    def __init__(self, input_size, hidden_size, num_layers=1, bias=True, batch_first=False, dropout=0.0,
                 bidirectional=False, proj_size=0, device=None, dtype=None):
        super().__init__()
        if proj_size:
            raise NotImplementedError("LSTM: proj_size is not supported")
        if hidden_size % 8 or hidden_size > 1024:
            raise ValueError("LSTM: hidden_size must be a multiple of 8 and <= 1024 (cfm_lstm_fwd)")
        self.input_size, self.hidden_size, self.num_layers = input_size, hidden_size, num_layers
        self.bias, self.batch_first, self.dropout = bias, batch_first, float(dropout)
        self.bidirectional = bidirectional
        ndir = 2 if bidirectional else 1
        fk = {"device": device, "dtype": dtype or torch.float32}
        for layer in range(num_layers):
            in_l = input_size if layer == 0 else hidden_size * ndir
            for sfx in ([""] + (["_reverse"] if bidirectional else [])):
                setattr(self, f"weight_ih_l{layer}{sfx}", nn.Parameter(torch.empty(4 * hidden_size, in_l, **fk)))
                setattr(self, f"weight_hh_l{layer}{sfx}", nn.Parameter(torch.empty(4 * hidden_size, hidden_size, **fk)))
                if bias:
                    setattr(self, f"bias_ih_l{layer}{sfx}", nn.Parameter(torch.empty(4 * hidden_size, **fk)))
                    setattr(self, f"bias_hh_l{layer}{sfx}", nn.Parameter(torch.empty(4 * hidden_size, **fk)))
        self.reset_parameters()

    def reset_parameters(self):
        """torch's init: every weight and bias ~ U(-1/sqrt(H), 1/sqrt(H))."""
        k = 1.0 / math.sqrt(self.hidden_size)
        for p in self.parameters():
            nn.init.uniform_(p, -k, k)

    def _sfx(self):
        return [""] + (["_reverse"] if self.bidirectional else [])

    def forward(self, input, hx=None):
        """Wait-limit failures of the recurrence kernels are reported WITHOUT a host sync: this call raises for a
        failure of an earlier pass whose flag copy has completed (typically one forward late), so the failing
        pass's outputs are already consumed.  Call LSTM.check_errors() at the end of a pass (Runner does, after
        every epoch / test / label pass) for a synchronising check of everything launched so far."""
        if hx is not None:
            raise NotImplementedError("LSTM: an initial state hx is not supported (the reference passes none)")
        if input.dim() != 2:
            raise NotImplementedError("LSTM: only the unbatched 2-D (L, input_size) form (asrnn.py:252) is supported")
        H, ndir = self.hidden_size, 2 if self.bidirectional else 1
        ERRORS.poll(input.device)            # earlier passes' wait-limit flags (no host sync)
        x = input.float().contiguous()
        hn, cn = [], []
        for layer in range(self.num_layers):
            sf = self._sfx()
            w_ih = torch.cat([getattr(self, f"weight_ih_l{layer}{s}") for s in sf]).float().contiguous()
            w_hh = torch.cat([getattr(self, f"weight_hh_l{layer}{s}") for s in sf]).float().contiguous()
            if self.bias:
                b = torch.cat([getattr(self, f"bias_ih_l{layer}{s}") + getattr(self, f"bias_hh_l{layer}{s}")
                               for s in sf]).float().contiguous()
            else:
                b = torch.zeros(ndir * 4 * H, device=x.device, dtype=torch.float32)
            y, c = _LSTMLayer.apply(x, w_ih, w_hh, b, H, ndir)
            hn.append(y[-1, :H])
            cn.append(c[-1, :H])
            if ndir == 2:
                hn.append(y[0, H:])
                cn.append(c[0, H:])
            x = y
            if layer < self.num_layers - 1 and self.dropout > 0 and self.training:
                x = F.dropout(x, self.dropout, True)
        out = x.to(input.dtype) if input.dtype != torch.float32 else x
        return out, (torch.stack(hn), torch.stack(cn))

    @staticmethod
    def check_errors(device=None):
        """Synchronising check of every recurrence launched so far on `device` (raises CfmError)."""
        ERRORS.sync_check(device or torch.device("cuda", torch.cuda.current_device()))

    def extra_repr(self):
        return (f"{self.input_size}, {self.hidden_size}, num_layers={self.num_layers}, "
                f"bidirectional={self.bidirectional}, dropout={self.dropout} [libcfm]")
