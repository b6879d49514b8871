"""Adafactor on libcfm — the reference's optimizer (lib/standard/runner.py:36,
``transformers.Adafactor(model.parameters(), lr=hp.lr, beta1=hp.beta1, scale_parameter=False,
relative_step=False)``) as ONE multi-tensor HIP step over all parameters (csrc/optim.hip) instead
of ~10 small PyTorch kernels per tensor.

Same constructor signature and state keys as transformers' Adafactor (exp_avg, exp_avg_sq_row,
exp_avg_sq_col / exp_avg_sq, step).  Supported on the device path: relative_step (host-side
learning-rate schedule), warmup_init; not supported (raise): scale_parameter=True, weight_decay.
"""
from __future__ import annotations

import ctypes
import math

import torch

from . import _lib as L


class Adafactor(torch.optim.Optimizer):
    def __init__(self, params, lr=None, eps=(1e-30, 1e-3), clip_threshold=1.0, decay_rate=-0.8, beta1=None,
                 weight_decay=0.0, scale_parameter=True, relative_step=True, warmup_init=False):
        if lr is not None and relative_step:
            raise ValueError("Cannot combine manual `lr` and `relative_step=True` options")
        if warmup_init and not relative_step:
            raise ValueError("`warmup_init=True` requires `relative_step=True`")
        if scale_parameter:
            raise NotImplementedError("libcfm Adafactor: scale_parameter=True is not on the device path "
                                      "(the reference uses scale_parameter=False, runner.py:36)")
        if weight_decay != 0.0:
            raise NotImplementedError("libcfm Adafactor: weight_decay is not on the device path")
        defaults = dict(lr=lr, eps=eps, clip_threshold=clip_threshold, decay_rate=decay_rate, beta1=beta1,
                        weight_decay=weight_decay, scale_parameter=scale_parameter, relative_step=relative_step,
                        warmup_init=warmup_init)
        super().__init__(params, defaults)
        self._step = 0
        self._dev = {}
        self._tables = {}
        self._fast = {}

    @staticmethod
    def _geom(p):
        if p.dim() >= 2:
            R, C = p.shape[-2], p.shape[-1]
            return True, p.numel() // (R * C), R, C
        return False, 1, 1, p.numel()

    def _ensure_state(self, p, group):
        st = self.state[p]
        if len(st) == 0:
            factored, nb, R, C = self._geom(p)
            st["step"] = 0
            if group["beta1"] is not None:
                st["exp_avg"] = torch.zeros_like(p, dtype=torch.float32)
            if factored:
                st["exp_avg_sq_row"] = torch.zeros(p.shape[:-1], device=p.device, dtype=torch.float32)
                st["exp_avg_sq_col"] = torch.zeros(p.shape[:-2] + p.shape[-1:], device=p.device, dtype=torch.float32)
            else:
                st["exp_avg_sq"] = torch.zeros_like(p, dtype=torch.float32)
            st["RMS"] = 0
        return st

    def _ptrkey(self, ps):
        """Every buffer the cached task table points at: parameter, gradient AND optimizer state
        (exp_avg, exp_avg_sq_row/col or exp_avg_sq).  A state swap (load_state_dict, a reset of
        self.state) changes the key, so the kernel never writes through a stale table."""
        key = []
        for p in ps:
            st = self.state.get(p, {})
            key.append((p.data_ptr(), p.grad.data_ptr(),
                        *(st[k].data_ptr() if torch.is_tensor(st.get(k)) else 0
                          for k in ("exp_avg", "exp_avg_sq_row", "exp_avg_sq_col", "exp_avg_sq"))))
        return tuple(key)

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        for st in self.state.values():     # the device step reads fp32 contiguous state on the param's device
            for k in ("exp_avg", "exp_avg_sq_row", "exp_avg_sq_col", "exp_avg_sq"):
                if torch.is_tensor(st.get(k)):
                    st[k] = st[k].float().contiguous()
        self._fast.clear()
        self._tables.clear()

    def _lr(self, group, step):
        lr = group["lr"]
        if group["relative_step"]:
            min_step = 1e-6 * step if group["warmup_init"] else 1e-2
            lr = min(min_step, 1.0 / math.sqrt(step))
        return lr

    def _build_table(self, group, ps, dev):
        """Host-side task table of one group (one ctypes fill per parameter) -> device copy."""
        lib = L.load()
        n = len(ps)
        host = (ctypes.c_char * L.size_call("cfm_adafactor_table_bytes", n))()
        row_off = col_off = blk_off = rm_off = rm_toff = cp_off = part_off = 0
        steps = []
        for i, p in enumerate(ps):
            st = self._ensure_state(p, group)
            st["step"] += 1
            steps.append(st["step"])
            factored, nb, R, C = self._geom(p)
            m = st.get("exp_avg")
            row = st["exp_avg_sq_row"] if factored else st["exp_avg_sq"]
            col = st["exp_avg_sq_col"] if factored else None
            L.call("cfm_adafactor_fill_table", ctypes.cast(host, ctypes.c_void_p), i, L.ptr(p), L.ptr(p.grad),
                   L.ptr(m), L.ptr(row), L.ptr(col), p.numel(), nb, R, C, row_off, col_off, blk_off, rm_off,
                   rm_toff, cp_off, part_off)
            if factored:
                row_off += lib.cfm_adafactor_row_tasks(nb, R, C)
                cp_off += lib.cfm_adafactor_colpart_tasks(nb, R, C)
                part_off += lib.cfm_adafactor_part_floats(nb, R, C)
                col_off += nb * C
                rm_off += nb
                rm_toff += lib.cfm_adafactor_rowmean_tasks(nb, R)
            blk_off += lib.cfm_adafactor_blocks(p.numel())
        if len(set(steps)) != 1:
            raise L.CfmError("libcfm Adafactor: all parameters of a group must share the step count")
        raw = bytes(host)
        tkey = (id(group), dev)
        cached = self._tables.get(tkey)
        if cached is not None and cached[0] == raw:
            table = cached[1]
        else:
            table = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(dev, non_blocking=False)
            self._tables[tkey] = (raw, table)
        return table, steps[0], (row_off, col_off, blk_off, rm_off, rm_toff, cp_off, part_off)

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        self._step += 1
        for group in self.param_groups:
            ps = [p for p in group["params"] if p.grad is not None]
            if not ps:
                continue
            for p in ps:
                if p.dtype != torch.float32 or p.grad.dtype != torch.float32:
                    raise L.CfmError("libcfm Adafactor expects fp32 parameters and gradients")
                if not p.grad.is_contiguous():
                    p.grad = p.grad.contiguous()
            n = len(ps)
            dev = ps[0].device
            # fast path: same parameter / gradient buffers as the cached table (every step of a
            # training loop whose gradients live in a captured graph's pool, or are re-used in
            # place): no per-parameter ctypes table build on the host, only the step counters
            ptrkey = self._ptrkey(ps)
            fast = self._fast.get((id(group), dev))
            if fast is not None and fast[0] == ptrkey:
                table, offs = fast[1], fast[2]
                steps = set()
                for p in ps:
                    st = self.state[p]
                    st["step"] += 1
                    steps.add(st["step"])
                if len(steps) != 1:
                    raise L.CfmError("libcfm Adafactor: all parameters of a group must share the step count")
                step = steps.pop()
                row_off, col_off, blk_off, rm_off, rm_toff, cp_off, part_off = offs
            else:
                table, step, offs = self._build_table(group, ps, dev)
                row_off, col_off, blk_off, rm_off, rm_toff, cp_off, part_off = offs
                self._fast[(id(group), dev)] = (self._ptrkey(ps), table, offs)   # state now exists
            key = (id(group), dev)
            buf = self._dev.get(key)
            if (buf is None or buf[0].numel() < max(rm_off, 1) or buf[1].numel() < max(part_off, 1)
                    or buf[2].numel() < blk_off):
                buf = (torch.empty(max(rm_off, 1), device=dev), torch.empty(max(part_off, 1), device=dev),
                       torch.empty(max(blk_off, 1), device=dev))
                self._dev[key] = buf
            b2t = 1.0 - math.pow(step, group["decay_rate"])
            beta1 = group["beta1"] if group["beta1"] is not None else 0.0
            L.call("cfm_adafactor_step", L.ptr(table), n, row_off, col_off, blk_off, rm_toff, cp_off, L.ptr(buf[0]),
                   L.ptr(buf[1]), L.ptr(buf[2]),
                   float(self._lr(group, step)), float(beta1), float(b2t), float(group["eps"][0]),
                   float(group["clip_threshold"]), L.stream())
            self._keep = table      # keep the table alive until the stream has consumed it
        return loss
