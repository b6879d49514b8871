"""Pin the CPU oracle against the golden fixtures (CPU only).

Fixtures come from tests/golden/make_golden.py: the reference's own Python (SpecAugment,
ConvSubSampling, ASRNN glue) and transformers' Wav2Vec2Conformer layer (Conformer block).
"""
import json
import os
import random
from types import SimpleNamespace

import numpy as np
import pytest
import torch

from oracle import conformer as oc
from oracle import frontend as of
from oracle import specaug as osa


def _hp(c):
    return SimpleNamespace(warping_param_W=c["W"], warping_ntimes=c["warping_ntimes"],
                           frequency_mask_param_F=c["F_param"], frequency_mask_ntimes=c["frequency_mask_ntimes"],
                           time_multiplicity=c["time_multiplicity"], adaptive_multiplicity=c["adaptive_multiplicity"],
                           pm=c["pm"], ps=c["ps"], adaptive_size=c["adaptive_size"], time_mask_param_T=c["T_param"])


def _flatten_draws(d, tau, W):
    seq = []
    for ws in d.warps:
        for u, (w, w0) in enumerate(ws):
            seq.append(w)
            if tau[u] >= 2 * W:
                seq.append(w0)
    for f, f0 in d.freq:
        seq += [f, f0]
    for ts in d.time:
        for t, t0 in ts:
            seq += [t, t0]
    return seq


@pytest.fixture(scope="module")
def specaug_cases(golden_dir):
    with open(os.path.join(golden_dir, "specaug.json")) as f:
        return json.load(f)


def test_specaug_draw_trace_bit_exact(specaug_cases):
    for c in specaug_cases:
        random.seed(c["seed"])
        d = osa.draw(c["B"], c["F"], c["tau"], _hp(c))
        assert _flatten_draws(d, c["tau"], c["W"]) == [r for (_, _, r) in c["draws"]], c["seed"]


def test_specaug_warp_table_and_output(specaug_cases):
    for c in specaug_cases:
        random.seed(c["seed"])
        d = osa.draw(c["B"], c["F"], c["tau"], _hp(c))
        if len(d.warps) == 1:
            Wt = [osa.warp_table(w, w0, c["tau"][u], c["T"]) for u, (w, w0) in enumerate(d.warps[0])]
            assert Wt == c["warp_index"]
        y = osa.apply(np.array(c["x"], np.float32), c["tau"], d, mode="reference")
        np.testing.assert_array_equal(y, np.array(c["y"], np.float32))


def test_specaug_intended_masks_touch_drawn_ranges(specaug_cases):
    c = specaug_cases[0]
    random.seed(c["seed"])
    d = osa.draw(c["B"], c["F"], c["tau"], _hp(c))
    x = np.ones((c["B"], c["F"], c["T"]), np.float32)
    y = osa.apply(x, c["tau"], d, mode="intended")
    for f, f0 in d.freq:
        assert np.all(y[:, f0:f0 + f, :] == 0)
    for ts in d.time:
        for u, (t, t0) in enumerate(ts):
            assert np.all(y[u, :, t0:t0 + t] == 0)


def test_convsub_matches_reference(golden_dir):
    z = np.load(os.path.join(golden_dir, "convsub.npz"))
    for ci in range(2):
        p = f"c{ci}_"
        x = torch.tensor(z[p + "x"], requires_grad=True)
        ws = [torch.tensor(z[p + k], requires_grad=True) for k in ("w1", "b1", "w2", "b2")]
        y = of.convsub_forward(x, *ws)
        np.testing.assert_allclose(y.detach().numpy(), z[p + "y"], rtol=1e-5, atol=1e-5)
        y.backward(torch.tensor(z[p + "gy"]))
        for t, k in zip(ws, ("gw1", "gb1", "gw2", "gb2")):
            np.testing.assert_allclose(t.grad.numpy(), z[p + k], rtol=1e-4, atol=1e-4)
        B, C2, Fp, Tp = z[p + "y"].shape
        assert int(z[p + "out_size"]) == C2 * Fp * Tp
        Fb, T = z[p + "x"].shape[2:]
        assert of.stage_len(of.stage_len(Fb, 7, 2), 3, 2) == Fp
        assert of.stage_len(of.stage_len(T, 7, 2), 3, 2) == Tp


LAYER_CASES = ["s_none", "s_rel", "m_rel", "d128_none"]


def load_layer_case(z, name):
    p = name + "_"
    d, H, ffn, K, B, T = [int(v) for v in z[p + "cfg"]]
    pos = "rel" if name.endswith("rel") else "none"
    ref = oc.ConformerRef(d, H, ffn, 1, K, 0.0, pos_enc=pos)
    sd = {k[len(p) + 2:]: torch.tensor(z[k]) for k in z.files if k.startswith(p + "w.")}
    ref.conformer_layers[0].load_state_dict(sd)
    return ref, dict(d=d, H=H, ffn=ffn, K=K, B=B, T=T, pos=pos)


@pytest.mark.parametrize("name", LAYER_CASES)
def test_conformer_layer_matches_transformers(golden_dir, name):
    z = np.load(os.path.join(golden_dir, "conformer_layers.npz"))
    p = name + "_"
    ref, cfg = load_layer_case(z, name)
    ref.train()
    x = torch.tensor(z[p + "x"], requires_grad=True)
    lens = torch.tensor(z[p + "lens"])
    y, _ = ref(x, lens)
    # transformers' layer sees padded queries too; compare every row (keys are masked only)
    np.testing.assert_allclose(y.detach().numpy(), z[p + "y"], rtol=1e-4, atol=2e-5)
    y.backward(torch.tensor(z[p + "gy"]))
    np.testing.assert_allclose(x.grad.numpy(), z[p + "gx"], rtol=1e-3, atol=1e-4)
    named = dict(ref.conformer_layers[0].named_parameters())
    for k in z.files:
        if k.startswith(p + "g."):
            nm = k[len(p) + 2:]
            np.testing.assert_allclose(named[nm].grad.numpy(), z[k], rtol=1e-3, atol=2e-4, err_msg=nm)
    bn = ref.conformer_layers[0].conv_module.sequential[3]
    np.testing.assert_allclose(bn.running_mean.numpy(), z[p + "bn_running_mean"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(bn.running_var.numpy(), z[p + "bn_running_var"], rtol=1e-5, atol=1e-6)


def test_rel_pos_table_matches_transformers():
    from transformers import Wav2Vec2ConformerConfig
    from transformers.models.wav2vec2_conformer.modeling_wav2vec2_conformer import (
        Wav2Vec2ConformerRelPositionalEmbedding)
    T, d = 37, 64
    cfg = Wav2Vec2ConformerConfig(hidden_size=d, max_source_positions=128)
    hf = Wav2Vec2ConformerRelPositionalEmbedding(cfg)(torch.zeros(1, T, d))[0]
    np.testing.assert_allclose(oc.rel_pos_table(T, d).numpy(), hf.numpy(), rtol=0, atol=1e-6)


def test_asrnn_encoder_glue_matches_reference(golden_dir):
    """oracle frontend + ConformerRef composed as asrnn.py:193-221 reproduce the reference's encoder."""
    z = np.load(os.path.join(golden_dir, "asrnn_small.npz"))
    B, Fb, C1, C2, d, H, ffn, K, L, proj, dec, V = [int(v) for v in z["cfg"]]
    w = {k[2:]: torch.tensor(z[k]) for k in z.files if k.startswith("w.")}
    x = torch.tensor(z["x"]).unsqueeze(1)
    tau = torch.tensor(z["tau"])
    y = of.convsub_forward(x, w["conv_sub_sampling.conv_sub_1.weight"], w["conv_sub_sampling.conv_sub_1.bias"],
                           w["conv_sub_sampling.conv_sub_2.weight"], w["conv_sub_sampling.conv_sub_2.bias"])
    h = of.utterance_projection(y, w["standard_linear.weight"], w["standard_linear.bias"], Fb)
    keep = tau > 0
    lens = tau[keep]
    h = h[:lens.shape[0], :int(lens.max())]
    conf = oc.ConformerRef(d, H, ffn, L, K, 0.0)
    conf.load_state_dict({k[len("conformers."):]: v for k, v in w.items() if k.startswith("conformers.")})
    conf.train()
    h, out_lens = conf(h, lens)
    h = torch.nn.functional.pad(h, (0, 0, 0, Fb - h.shape[1], 0, B - lens.shape[0])).flatten(0, 1)
    h = torch.nn.functional.linear(h, w["projection_fc.weight"], w["projection_fc.bias"])
    h = torch.nn.functional.silu(h)
    h = torch.nn.functional.batch_norm(h, None, None, w["projection_batch_norm.weight"],
                                       w["projection_batch_norm.bias"], training=True)
    np.testing.assert_allclose(h.detach().numpy(), z["enc"], rtol=1e-4, atol=1e-5)
    np.testing.assert_array_equal(out_lens.numpy(), z["out_lens"])


@pytest.mark.parametrize("name", ["L512_none", "L512_rel"])
def test_conformer_L_two_layers_match_transformers(golden_dir, name):
    """Conformer-L dims (d 512, 8 heads, ffn 2048, K 31), two layers, ragged lengths: the oracle with the
    seeded weights (oracle.conformer.seeded_hf_compatible) vs transformers' encoder layers (fixture):
    outputs, input gradient, 16 random projections of every compared weight gradient, BN running stats."""
    z = np.load(os.path.join(golden_dir, "conformer_L.npz"))
    p = name + "_"
    d, H, ffn, K, B, T, L, seed = [int(v) for v in z[p + "cfg"]]
    pos = "rel" if name.endswith("rel") else "none"
    ref = oc.seeded_hf_compatible(d, H, ffn, L, K, pos, seed).train()
    x = torch.tensor(z[p + "x"], requires_grad=True)
    y, _ = ref(x, torch.tensor(z[p + "lens"]))
    np.testing.assert_allclose(y.detach().numpy(), z[p + "y"], rtol=1e-4, atol=5e-5)
    y.backward(torch.tensor(z[p + "gy"]))
    np.testing.assert_allclose(x.grad.numpy(), z[p + "gx"], rtol=1e-3, atol=2e-4)
    named = dict(ref.named_parameters())
    for k in z.files:
        if k.startswith(p + "g."):
            nm = k[len(p) + 2:]
            got = oc.grad_probes(nm, named[nm].grad).numpy()
            np.testing.assert_allclose(got, z[k], rtol=2e-3, atol=2e-3 * np.abs(z[k]).max(), err_msg=nm)
    for li in range(L):
        bn = ref.conformer_layers[li].conv_module.sequential[3]
        np.testing.assert_allclose(bn.running_mean.numpy(), z[f"{p}bn_running_mean.{li}"], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(bn.running_var.numpy(), z[f"{p}bn_running_var.{li}"], rtol=1e-5, atol=1e-6)
