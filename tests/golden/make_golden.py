"""Generate the golden fixtures under tests/golden/ (run in the build container only).

    python tests/golden/make_golden.py

Sources of truth:
  * the reference's own Python, imported read-only from /root/reference (lib.hparams,
    lib.convsubsampling, lib.standard.asrnn) with stubs for modules absent from this image
    (torchaudio, torchvision, colorama, the missing ``lib.conformer``).  torchaudio's Conformer
    is stubbed with oracle.conformer.ConformerRef (the reference does not vendor it).
  * transformers' Wav2Vec2ConformerEncoderLayer (an independent implementation of the Conformer
    block, incl. Transformer-XL relative positions) for the encoder-layer fixtures.

Outputs are plain .npz / .json data (inputs + expected outputs); no reference source is copied.
Never run on the GPU box (it has no /root/reference).
"""
from __future__ import annotations

import json
import os
import random
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)

from oracle.conformer import ConformerRef  # noqa: E402


def _install_stubs():
    import transformers  # noqa: F401  (must precede the torchvision stub: it probes torchvision)
    ta = types.ModuleType("torchaudio")
    ta_models = types.ModuleType("torchaudio.models")
    ta_models.Conformer = ConformerRef
    ta.models = ta_models
    sys.modules["torchaudio"] = ta
    sys.modules["torchaudio.models"] = ta_models
    tv = types.ModuleType("torchvision")
    tv_models = types.ModuleType("torchvision.models")
    tv_models.convnext_tiny = lambda *a, **k: None
    tv.models = tv_models
    sys.modules["torchvision"] = tv
    sys.modules["torchvision.models"] = tv_models
    lc = types.ModuleType("lib.conformer")
    lc.Conformer = object
    sys.modules["lib.conformer"] = lc
    sys.path.insert(0, REF)


def _hparams(tmp):
    from lib.hparams import HParams
    hp = HParams(tmp)
    hp.device = torch.device("cpu")
    return hp


# ----------------------------------------------------------------------------- SpecAugment
def gen_specaug(tmp):
    from lib.standard.asrnn import ASRNN

    class _SA:
        pass
    for name in ("time_warping", "frequency_masking", "time_masking", "SpecAugment"):
        setattr(_SA, name, getattr(ASRNN, name))

    cases = [
        dict(seed=42, B=4, F=40, T=40, tau=[40, 40, 30, 12], adaptive_multiplicity=False, adaptive_size=False),
        dict(seed=7, B=3, F=16, T=24, tau=[24, 1, 0], adaptive_multiplicity=False, adaptive_size=False),
        dict(seed=123, B=5, F=80, T=101, tau=[101, 77, 50, 3, 1], adaptive_multiplicity=False, adaptive_size=True),
        dict(seed=99, B=2, F=80, T=64, tau=[64, 60], adaptive_multiplicity=True, adaptive_size=True,
             pm=2.7, time_multiplicity=3),
        dict(seed=5, B=6, F=40, T=50, tau=[50, 49, 48, 10, 4, 2], adaptive_multiplicity=False,
             adaptive_size=False, warping_param_W=3, warping_ntimes=2, frequency_mask_ntimes=3),
    ]
    out = []
    orig_randint = random.randint
    for c in cases:
        hp = _hparams(tmp)
        for k in ("adaptive_multiplicity", "adaptive_size", "pm", "time_multiplicity", "warping_param_W",
                  "warping_ntimes", "frequency_mask_ntimes"):
            if k in c:
                setattr(hp, k, c[k])
        sa = _SA()
        sa.hp = hp
        g = torch.Generator().manual_seed(c["seed"])
        x = torch.rand(c["B"], 1, c["F"], c["T"], generator=g)
        tau = torch.LongTensor(c["tau"])
        log = []

        def logged(a, b):
            r = orig_randint(a, b)
            log.append([int(a), int(b), int(r)])
            return r
        random.seed(c["seed"])
        random.randint = logged
        try:
            y = sa.SpecAugment(x.clone(), tau)
        finally:
            random.randint = orig_randint
        # warp table recovered from an index-encoded input (x[b,f,t] = t)
        random.seed(c["seed"])
        xi = torch.arange(c["T"], dtype=torch.float32).repeat(c["B"], 1, c["F"], 1)
        yi = sa.SpecAugment(xi, tau)
        rec = {k: v for k, v in c.items()}
        rec.update(x=x.squeeze(1).numpy().tolist(), y=y.squeeze(1).numpy().tolist(), draws=log,
                   warp_index=yi.squeeze(1)[:, 0, :].numpy().astype(np.int64).tolist(),
                   W=hp.warping_param_W, F_param=hp.frequency_mask_param_F, T_param=hp.time_mask_param_T,
                   ps=hp.ps, pm=hp.pm, warping_ntimes=hp.warping_ntimes,
                   frequency_mask_ntimes=hp.frequency_mask_ntimes, time_multiplicity=hp.time_multiplicity)
        out.append(rec)
    with open(os.path.join(HERE, "specaug.json"), "w") as f:
        json.dump(out, f)
    print("specaug.json", len(out), "cases")


# ------------------------------------------------------------------------- ConvSubSampling
def gen_convsub(tmp):
    from lib.convsubsampling import ConvSubSampling
    arrays = {}
    for ci, (B, Fb, T, C1, C2) in enumerate([(2, 40, 40, 16, 8), (2, 80, 201, 32, 16)]):
        hp = _hparams(tmp)
        hp.conv_sub_1_nodes = C1
        hp.set_input_dim(Fb, T)
        torch.manual_seed(100 + ci)
        m = ConvSubSampling(hp, 1, C2)
        x = torch.rand(B, 1, Fb, T, requires_grad=True)
        y = m(x)
        gy = torch.randn_like(y)
        y.backward(gy)
        p = f"c{ci}_"
        arrays.update({p + "x": x.detach().numpy(), p + "w1": m.conv_sub_1.weight.detach().numpy(),
                       p + "b1": m.conv_sub_1.bias.detach().numpy(), p + "w2": m.conv_sub_2.weight.detach().numpy(),
                       p + "b2": m.conv_sub_2.bias.detach().numpy(), p + "y": y.detach().numpy(),
                       p + "gy": gy.numpy(), p + "gx": x.grad.numpy(),
                       p + "gw1": m.conv_sub_1.weight.grad.numpy(), p + "gb1": m.conv_sub_1.bias.grad.numpy(),
                       p + "gw2": m.conv_sub_2.weight.grad.numpy(), p + "gb2": m.conv_sub_2.bias.grad.numpy(),
                       p + "out_size": np.array(m.out_size)})
    np.savez_compressed(os.path.join(HERE, "convsub.npz"), **arrays)
    print("convsub.npz")


# -------------------------------------------------------------- Conformer layer (transformers)
def _hf_layer_from_ref(ref_layer, d, H, ffn, K, pos):
    from transformers import Wav2Vec2ConformerConfig
    from transformers.models.wav2vec2_conformer.modeling_wav2vec2_conformer import (
        Wav2Vec2ConformerEncoderLayer)
    cfg = Wav2Vec2ConformerConfig(hidden_size=d, num_attention_heads=H, intermediate_size=ffn,
                                  hidden_act="swish", conv_depthwise_kernel_size=K,
                                  position_embeddings_type=pos, attention_dropout=0.0, hidden_dropout=0.0,
                                  activation_dropout=0.0, conformer_conv_dropout=0.0, max_source_positions=512)
    hf = Wav2Vec2ConformerEncoderLayer(cfg)
    r = ref_layer
    with torch.no_grad():
        hf.ffn1_layer_norm.load_state_dict(r.ffn1.sequential[0].state_dict())
        hf.ffn1.intermediate_dense.load_state_dict(r.ffn1.sequential[1].state_dict())
        hf.ffn1.output_dense.load_state_dict(r.ffn1.sequential[4].state_dict())
        hf.ffn2_layer_norm.load_state_dict(r.ffn2.sequential[0].state_dict())
        hf.ffn2.intermediate_dense.load_state_dict(r.ffn2.sequential[1].state_dict())
        hf.ffn2.output_dense.load_state_dict(r.ffn2.sequential[4].state_dict())
        hf.self_attn_layer_norm.load_state_dict(r.self_attn_layer_norm.state_dict())
        W, b = r.self_attn.in_proj_weight, r.self_attn.in_proj_bias
        hf.self_attn.linear_q.weight.copy_(W[:d]); hf.self_attn.linear_q.bias.copy_(b[:d])
        hf.self_attn.linear_k.weight.copy_(W[d:2 * d]); hf.self_attn.linear_k.bias.copy_(b[d:2 * d])
        hf.self_attn.linear_v.weight.copy_(W[2 * d:]); hf.self_attn.linear_v.bias.copy_(b[2 * d:])
        hf.self_attn.linear_out.load_state_dict(r.self_attn.out_proj.state_dict())
        if pos == "relative":
            hf.self_attn.linear_pos.weight.copy_(r.self_attn.linear_pos.weight)
            hf.self_attn.pos_bias_u.copy_(r.self_attn.pos_bias_u)
            hf.self_attn.pos_bias_v.copy_(r.self_attn.pos_bias_v)
        cm = r.conv_module
        hf.conv_module.layer_norm.load_state_dict(cm.layer_norm.state_dict())
        hf.conv_module.pointwise_conv1.weight.copy_(cm.sequential[0].weight)
        hf.conv_module.depthwise_conv.weight.copy_(cm.sequential[2].weight)
        hf.conv_module.batch_norm.load_state_dict(cm.sequential[3].state_dict())
        hf.conv_module.pointwise_conv2.weight.copy_(cm.sequential[5].weight)
        hf.final_layer_norm.load_state_dict(r.final_layer_norm.state_dict())
    return hf


def gen_conformer_layers():
    from transformers.models.wav2vec2_conformer.modeling_wav2vec2_conformer import (
        Wav2Vec2ConformerRelPositionalEmbedding)
    cases = [
        ("s_none", dict(d=144, H=4, ffn=576, K=31, B=3, T=57, lens=[57, 40, 9], pos=None)),
        ("s_rel", dict(d=144, H=4, ffn=576, K=31, B=3, T=57, lens=[57, 40, 9], pos="relative")),
        ("m_rel", dict(d=64, H=2, ffn=256, K=7, B=2, T=33, lens=[33, 20], pos="relative")),
        ("d128_none", dict(d=128, H=2, ffn=512, K=15, B=2, T=70, lens=[70, 64], pos=None)),
    ]
    arrays = {}
    for ci, (name, c) in enumerate(cases):
        torch.manual_seed(1000 + ci)
        d, H, ffn, K, B, T = c["d"], c["H"], c["ffn"], c["K"], c["B"], c["T"]
        pos_enc = "rel" if c["pos"] == "relative" else "none"
        ref = ConformerRef(d, H, ffn, 1, K, 0.0, pos_enc=pos_enc)
        layer = ref.conformer_layers[0]
        with torch.no_grad():      # HF conv-module convs have no bias: zero ours; randomise the rest
            for m in (layer.conv_module.sequential[0], layer.conv_module.sequential[2],
                      layer.conv_module.sequential[5]):
                m.bias.zero_()
            for nm, p in layer.named_parameters():
                if nm.endswith("bias") and "conv_module.sequential" not in nm:
                    p.normal_(0, 0.1)
                if "layer_norm" in nm and nm.endswith("weight"):
                    p.uniform_(0.5, 1.5)
            layer.conv_module.sequential[3].weight.uniform_(0.5, 1.5)
            layer.conv_module.sequential[3].bias.normal_(0, 0.1)
        hf = _hf_layer_from_ref(layer, d, H, ffn, K, c["pos"])
        hf.train()
        x = torch.randn(B, T, d, requires_grad=True)
        lens = torch.tensor(c["lens"])
        valid = torch.arange(T)[None, :] < lens[:, None]
        amask = (1.0 - valid[:, None, None, :].float()) * torch.finfo(torch.float32).min
        rel = None
        if c["pos"] == "relative":
            from transformers import Wav2Vec2ConformerConfig
            cfg = Wav2Vec2ConformerConfig(hidden_size=d, max_source_positions=512)
            rel = Wav2Vec2ConformerRelPositionalEmbedding(cfg)(x)
        y, _ = hf(x, attention_mask=amask, relative_position_embeddings=rel)
        gy = torch.randn_like(y)
        y.backward(gy)
        p = name + "_"
        arrays[p + "cfg"] = np.array([d, H, ffn, K, B, T], dtype=np.int64)
        arrays[p + "lens"] = lens.numpy()
        arrays[p + "x"] = x.detach().numpy()
        arrays[p + "y"] = y.detach().numpy()
        arrays[p + "gy"] = gy.numpy()
        arrays[p + "gx"] = x.grad.numpy()
        for nm, prm in layer.state_dict().items():
            arrays[p + "w." + nm] = prm.detach().numpy()
        # weight grads in torchaudio naming (HF layer holds them)
        arrays[p + "g.ffn1.sequential.1.weight"] = hf.ffn1.intermediate_dense.weight.grad.numpy()
        arrays[p + "g.ffn2.sequential.4.weight"] = hf.ffn2.output_dense.weight.grad.numpy()
        arrays[p + "g.self_attn.in_proj_weight"] = torch.cat(
            [hf.self_attn.linear_q.weight.grad, hf.self_attn.linear_k.weight.grad,
             hf.self_attn.linear_v.weight.grad]).numpy()
        arrays[p + "g.self_attn.out_proj.weight"] = hf.self_attn.linear_out.weight.grad.numpy()
        arrays[p + "g.conv_module.sequential.2.weight"] = hf.conv_module.depthwise_conv.weight.grad.numpy()
        arrays[p + "g.conv_module.sequential.3.weight"] = hf.conv_module.batch_norm.weight.grad.numpy()
        arrays[p + "g.final_layer_norm.weight"] = hf.final_layer_norm.weight.grad.numpy()
        if c["pos"] == "relative":
            arrays[p + "g.self_attn.linear_pos.weight"] = hf.self_attn.linear_pos.weight.grad.numpy()
            arrays[p + "g.self_attn.pos_bias_u"] = hf.self_attn.pos_bias_u.grad.numpy()
            arrays[p + "g.self_attn.pos_bias_v"] = hf.self_attn.pos_bias_v.grad.numpy()
        # BN running stats after one train-mode step
        arrays[p + "bn_running_mean"] = hf.conv_module.batch_norm.running_mean.numpy()
        arrays[p + "bn_running_var"] = hf.conv_module.batch_norm.running_var.numpy()
        print(name, "y", tuple(y.shape))
    np.savez_compressed(os.path.join(HERE, "conformer_layers.npz"), **arrays)
    print("conformer_layers.npz")


# ------------------------------------------------- Conformer-L dims, two layers (seeded weights)
HF_GRAD_NAMES = {   # transformers parameter -> torchaudio name (per layer)
    "ffn1.intermediate_dense.weight": "ffn1.sequential.1.weight",
    "ffn1.output_dense.weight": "ffn1.sequential.4.weight",
    "ffn2.intermediate_dense.weight": "ffn2.sequential.1.weight",
    "ffn2.output_dense.weight": "ffn2.sequential.4.weight",
    "self_attn.linear_out.weight": "self_attn.out_proj.weight",
    "conv_module.pointwise_conv1.weight": "conv_module.sequential.0.weight",
    "conv_module.depthwise_conv.weight": "conv_module.sequential.2.weight",
    "conv_module.pointwise_conv2.weight": "conv_module.sequential.5.weight",
    "conv_module.batch_norm.weight": "conv_module.sequential.3.weight",
    "final_layer_norm.weight": "final_layer_norm.weight",
    "self_attn.linear_pos.weight": "self_attn.linear_pos.weight",
    "self_attn.pos_bias_u": "self_attn.pos_bias_u",
    "self_attn.pos_bias_v": "self_attn.pos_bias_v",
}


def gen_conformer_L():
    """Two Conformer-L layers (d 512, 8 heads, ffn 2048, K 31), ragged lengths, pos none and rel, through
    transformers' encoder layers.  Weights are regenerated from the seed (oracle.conformer.seeded_hf_compatible)
    so the fixture stays small: inputs, outputs, input gradient, BN running stats, and 16 random
    projections of each weight gradient (oracle.conformer.grad_probes)."""
    from oracle.conformer import grad_probes, seeded_hf_compatible
    from transformers import Wav2Vec2ConformerConfig
    from transformers.models.wav2vec2_conformer.modeling_wav2vec2_conformer import (
        Wav2Vec2ConformerRelPositionalEmbedding)
    d, H, ffn, K, L, B, T, lens = 512, 8, 2048, 31, 2, 2, 96, [96, 61]
    arrays = {}
    for ci, (name, pos) in enumerate((("L512_none", None), ("L512_rel", "relative"))):
        seed = 3000 + ci
        ref = seeded_hf_compatible(d, H, ffn, L, K, "rel" if pos else "none", seed)
        hfs = [_hf_layer_from_ref(layer, d, H, ffn, K, pos) for layer in ref.conformer_layers]
        for hf in hfs:
            hf.train()
        g = torch.Generator().manual_seed(seed)
        x = torch.randn(B, T, d, generator=g).requires_grad_()
        ln = torch.tensor(lens)
        valid = torch.arange(T)[None, :] < ln[:, None]
        amask = (1.0 - valid[:, None, None, :].float()) * torch.finfo(torch.float32).min
        rel = None
        if pos:
            rel = Wav2Vec2ConformerRelPositionalEmbedding(Wav2Vec2ConformerConfig(hidden_size=d,
                                                                                  max_source_positions=512))(x)
        y = x
        for hf in hfs:
            y, _ = hf(y, attention_mask=amask, relative_position_embeddings=rel)
        gy = torch.randn(y.shape, generator=g)
        y.backward(gy)
        p = name + "_"
        arrays[p + "cfg"] = np.array([d, H, ffn, K, B, T, L, seed], dtype=np.int64)
        arrays[p + "lens"] = ln.numpy()
        arrays[p + "x"] = x.detach().numpy()
        arrays[p + "y"] = y.detach().numpy()
        arrays[p + "gy"] = gy.numpy()
        arrays[p + "gx"] = x.grad.numpy()
        for li, hf in enumerate(hfs):
            named = dict(hf.named_parameters())
            for hn, tn in HF_GRAD_NAMES.items():
                if hn in named:
                    gr = named[hn].grad
                    key = f"{p}g.conformer_layers.{li}.{tn}"
                    arrays[key] = grad_probes(f"conformer_layers.{li}.{tn}", gr).numpy()
            gin = torch.cat([hf.self_attn.linear_q.weight.grad, hf.self_attn.linear_k.weight.grad,
                             hf.self_attn.linear_v.weight.grad])
            arrays[f"{p}g.conformer_layers.{li}.self_attn.in_proj_weight"] = grad_probes(
                f"conformer_layers.{li}.self_attn.in_proj_weight", gin).numpy()
            arrays[f"{p}bn_running_mean.{li}"] = hf.conv_module.batch_norm.running_mean.numpy()
            arrays[f"{p}bn_running_var.{li}"] = hf.conv_module.batch_norm.running_var.numpy()
        print(name, "y", tuple(y.shape))
    np.savez_compressed(os.path.join(HERE, "conformer_L.npz"), **arrays)
    print("conformer_L.npz")


# ------------------------------------------------------------ ASRNN (reference glue, shrunken)
def gen_asrnn(tmp):
    from lib.standard.asrnn import ASRNN
    hp = _hparams(tmp)
    B, Fb = 4, 16
    hp.batch_size = B
    hp.n_mels = Fb
    hp.set_input_dim(Fb, Fb)
    hp.set_max_len(Fb)          # the reference's tau = n_mels quirk (speechcommands.py:71,75)
    hp.conv_sub_1_nodes = 16
    hp.conv_sub_2_nodes = 8
    hp.standard_linear_nodes = 64
    hp.mhsa_num_heads = 2
    hp.conformer_ff1_linear1_nodes = 64
    hp.conformer_depthwise_conv_kernel = 5
    hp.n_conformers = 2
    hp.dropout = 0.0
    hp.projection_out_size = 32
    hp.standard_decoder_nodes = 32
    hp.set_ntokens(38)
    torch.manual_seed(2024)
    model = ASRNN(hp)
    model.train()
    x = torch.rand(B, Fb, Fb)
    tau = torch.LongTensor([16, 16, 11, 0])     # one empty utterance: exercises the crop/pad glue
    enc, out_lens = model.encoder(x.unsqueeze(1), tau)
    logits, lens2 = model(x, tau)
    arrays = {"x": x.numpy(), "tau": tau.numpy(), "enc": enc.detach().numpy(),
              "out_lens": out_lens.numpy(), "logits": logits.detach().numpy()}
    for k, v in model.state_dict().items():
        arrays["w." + k] = v.detach().numpy()
    arrays["cfg"] = np.array([B, Fb, 16, 8, 64, 2, 64, 5, 2, 32, 32, 38], dtype=np.int64)
    np.savez_compressed(os.path.join(HERE, "asrnn_small.npz"), **arrays)
    print("asrnn_small.npz")


class _TTVocab:
    """torchtext.vocab.Vocab as the reference uses it (torchtext is absent from this image; its published
    semantics): `vocab(ordered_dict, min_freq=1)` keeps the dict's tokens in insertion order, insert_token()
    shifts later ids, lookup by token falls back to the default index once set."""

    def __init__(self, ordered_dict, min_freq=1):
        self.itos = [t for t, f in ordered_dict.items() if f >= min_freq]
        self.default = None

    def insert_token(self, token, index):
        self.itos.insert(index, token)

    def set_default_index(self, i):
        self.default = i

    def __contains__(self, t):
        return t in self.itos

    def __getitem__(self, t):
        if t in self.itos:
            return self.itos.index(t)
        if self.default is None:
            raise RuntimeError(f"token {t!r} not found and default index is not set")
        return self.default

    def __len__(self):
        return len(self.itos)

    def lookup_tokens(self, ids):
        return [self.itos[i] for i in ids]


def _install_runner_stubs(calls):
    """Recording stubs for the Runner / myVocab imports absent from this image (jiwer, torchtext, tqdm,
    colorama) and the plotting module lib.evals (matplotlib): jiwer.wer records the word lists it gets."""
    import importlib.machinery
    import transformers  # noqa: F401  (loads torch's import-time probes of tqdm before the stub replaces it)
    _mod = types.ModuleType

    def mod(name):
        m = _mod(name)
        m.__spec__ = importlib.machinery.ModuleSpec(name, None)
        return m
    tt = mod("torchtext")
    ttv = mod("torchtext.vocab")
    ttv.vocab = lambda od, min_freq=1: _TTVocab(od, min_freq)
    tt.vocab = ttv
    sys.modules["torchtext"] = tt
    sys.modules["torchtext.vocab"] = ttv
    jw = mod("jiwer")

    def wer(t, p):
        calls.append((list(t), list(p)))
        return 0.25
    jw.wer = wer
    sys.modules["jiwer"] = jw

    class _Bar:
        def __init__(self, *a, **k):
            self.postfix = ""
            self.bar_format = ""

        def __enter__(self):
            return self

        def __exit__(self, *a):
            return False

        def set_description(self, *a):
            pass

        def update(self, *a):
            pass
    tq = mod("tqdm")
    tq.tqdm = _Bar
    sys.modules["tqdm"] = tq
    co = mod("colorama")
    co.Fore = types.SimpleNamespace(MAGENTA="", RESET="", CYAN="", GREEN="", RED="", BLUE="", YELLOW="")
    sys.modules["colorama"] = co
    ev = mod("lib.evals")

    class Evals:
        def __init__(self, *a, **k):
            pass

        def plot(self, *a, **k):
            pass

        def heatmap(self, *a, **k):
            pass
    ev.Evals = Evals
    sys.modules["lib.evals"] = ev


def gen_runner_vocab(tmp):
    """The Runner / vocabulary surface around the hot path: the reference's own
    myVocab (reading its shipped vocabs/myvocab.txt, and building from sentences), myVocab.decode on fixed
    id rows (myvocab.py:211-231), and Runner.train / test / generate_labels (runner.py:102-281) driven by a
    stub model that returns fixed logits -- the word lists the reference hands to jiwer.wer are recorded."""
    calls = []
    _install_runner_stubs(calls)
    from lib.standard.myvocab import myVocab
    from lib.standard.runner import Runner
    vocab_file = os.path.join(REF, "vocabs", "myvocab.txt")
    voc = myVocab(tmp, vocab_path=vocab_file)
    itos = voc.vocab.lookup_tokens(list(range(len(voc))))
    sents = ["yes no yes", "up down", "left yes", "no no no go", "stop"]
    data = [(None, None, s) for s in sents]
    built = myVocab(tmp, data=data, vocab_path=os.path.join(tmp, "built.txt"))
    built_itos = built.vocab.lookup_tokens(list(range(len(built))))
    parsed = [voc.parse(s) for s in ["yes no", "up unknownword down"]]
    g = torch.Generator().manual_seed(11)
    V = len(itos)
    rows = torch.randint(0, V, (6, 9), generator=g)
    rows[0, :] = 1                              # all <pad>
    rows[1, :] = torch.tensor([0, 0, 5, 5, 0, 1, 7, 7, 2])   # blanks, repeats (not collapsed), <unk>
    decoded = voc.decode(rows)

    hp = _hparams(tmp)
    hp.batch_size = 4
    hp.set_blank_index(voc.vocab[voc.blank_token])
    hp.plots_dir = tmp
    hp.standard_model_path = os.path.join(tmp, "std.pth")
    hp.finetuning_model_path = os.path.join(tmp, "ft.pth")
    B, T = 4, 12
    logits = torch.randn(5, B, T, V, generator=g) * 3.0      # train x2, validation x1, pretrain x2
    logits[0, 2] = -10.0
    logits[0, 2, :, 0] = 10.0                   # an all-blank prediction -> '_' in the word lists
    out_lens = torch.tensor([T, T, T - 3, T])
    tgts = torch.randint(3, V, (3, B, 2), generator=g)
    tgt_lens = torch.tensor([[1, 2, 1, 0], [2, 1, 1, 1], [1, 1, 0, 2]])
    for j in range(3):
        for b in range(B):
            tgts[j, b, tgt_lens[j, b]:] = voc.vocab[voc.pad_token]    # padded with <pad>, as get_batch does

    class StubModel(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.w = torch.nn.Parameter(torch.zeros(1))
            self.i = 0

        def forward(self, x, input_lens, SpecAugment=False, lm=None, finetuning=False):
            k = int(x.reshape(-1)[0].item())
            return torch.log_softmax(logits[k] + self.w, -1), out_lens.clone()

        def predict(self, lg):
            return torch.argmax(lg, dim=-1)

    class StubData:
        idxes = {"train": list(range(8)), "validation": list(range(4)), "pretrain": list(range(8))}
        vocab = voc

        def shuffle(self, kind):
            pass

        def get_batch(self, i, kind):
            k = {"train": i, "validation": 2, "pretrain": 3 + i}[kind]
            x = torch.full((B, 1, 4, 4), float(k))
            j = min(k, 2)
            return {"input": {"mels": x, "tau": torch.full((B,), T)},
                    "target": {"transcripts": tgts[j].clone(), "lens": tgt_lens[j].clone()}, "unpadded_len": B}

    model = StubModel()
    runner = Runner(model, hp)
    runner.train(StubData(), 1)
    train_calls = [list(c) for c in calls]
    labels = runner.generate_labels(StubData())
    rec = {"itos": itos, "built_from": sents, "built_itos": built_itos, "parsed": parsed,
           "decode_rows": rows.tolist(), "decoded": decoded, "batch": B, "T": T,
           "logits": logits.tolist(), "out_lens": out_lens.tolist(), "targets": tgts.tolist(),
           "target_lens": tgt_lens.tolist(), "wer_calls": train_calls, "labels": labels,
           "note": "wer_calls: (target words, predicted words) the reference's Runner.train passes to jiwer.wer: "
                   "2 train batches then 1 validation batch; labels: Runner.generate_labels over 2 pretrain batches"}
    with open(os.path.join(HERE, "runner_vocab.json"), "w") as f:
        json.dump(rec, f)
    print("runner_vocab.json", len(train_calls), "wer calls,", len(labels), "labels")


def main():
    import tempfile
    _install_stubs()
    with tempfile.TemporaryDirectory() as tmp:
        gen_specaug(tmp)
        gen_convsub(tmp)
        gen_conformer_layers()
        gen_conformer_L()
        gen_asrnn(tmp)
        gen_runner_vocab(tmp)


if __name__ == "__main__":
    main()
