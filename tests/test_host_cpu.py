"""Host-side logic on the CPU: library exports, module surfaces, state-dict compatibility,
SpecAugment draws (bit-exact vs the oracle / reference fixtures), error behaviour."""
import ctypes
import json
import os
import random
import re
from types import SimpleNamespace

import numpy as np
import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_symbols():
    src = open(os.path.join(REPO, "include", "cfm.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(cfm_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    from nn_conformer_for_speech_recognition_amd import _lib
    lib = ctypes.CDLL(_lib.LIB_PATH)
    syms = _header_symbols()
    assert len(syms) >= 20
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    assert set(syms) == set(_lib.EXPORTED), set(syms) ^ set(_lib.EXPORTED)
    _lib.load()
    assert lib.cfm_version() >= 1


def test_error_path_sets_message():
    from nn_conformer_for_speech_recognition_amd import _lib
    lib = _lib.load()
    rc = lib.cfm_layernorm_fwd(None, 0, None, None, None, 0, None, None, 4, 4, 1e-5, None)
    assert rc == -1
    assert b"null" in lib.cfm_get_last_error()
    rc = lib.cfm_glu_dwconv_fwd(ctypes.c_void_p(16), 0, ctypes.c_void_p(16), ctypes.c_void_p(16),
                                ctypes.c_void_p(16), 1, 1, 1, 4, ctypes.c_void_p(16), None)
    assert rc == -5    # even kernel rejected before any launch


def test_conformer_state_dict_matches_torchaudio_names():
    from nn_conformer_for_speech_recognition_amd.conformer import Conformer
    from oracle.conformer import ConformerRef
    for pos in ("none", "rel"):
        a = Conformer(64, 4, 128, 2, 7, 0.1, pos_enc=pos)
        b = ConformerRef(64, 4, 128, 2, 7, 0.1, pos_enc=pos)
        ka, kb = set(a.state_dict()), set(b.state_dict())
        assert ka == kb, ka ^ kb
        for k in ka:
            assert a.state_dict()[k].shape == b.state_dict()[k].shape, k
        a.load_state_dict(b.state_dict())


def test_conformer_rejects_even_kernel_and_cpu_tensors():
    from nn_conformer_for_speech_recognition_amd.conformer import Conformer
    with pytest.raises(ValueError):
        Conformer(64, 4, 128, 1, 6)
    m = Conformer(64, 4, 128, 1, 7)
    with pytest.raises(RuntimeError):
        m(torch.zeros(1, 8, 64), torch.tensor([8]))


def _hp_from_case(c):
    return SimpleNamespace(warping_param_W=c["W"], warping_ntimes=c["warping_ntimes"],
                           frequency_mask_param_F=c["F_param"], frequency_mask_ntimes=c["frequency_mask_ntimes"],
                           time_multiplicity=c["time_multiplicity"], adaptive_multiplicity=c["adaptive_multiplicity"],
                           pm=c["pm"], ps=c["ps"], adaptive_size=c["adaptive_size"], time_mask_param_T=c["T_param"])


def test_product_specaug_draws_match_reference_trace(golden_dir):
    from nn_conformer_for_speech_recognition_amd import specaugment as psa
    with open(os.path.join(golden_dir, "specaug.json")) as f:
        cases = json.load(f)
    for c in cases:
        random.seed(c["seed"])
        warps, freqs, times = psa.draw(c["B"], c["F"], c["tau"], _hp_from_case(c))
        seq = []
        for per in warps:
            for u, (w, w0) in enumerate(per):
                seq.append(w)
                if c["tau"][u] >= 2 * c["W"]:
                    seq.append(w0)
        for f, f0 in freqs:
            seq += [f, f0]
        for per in times:
            for t, t0 in per:
                seq += [t, t0]
        assert seq == [r for (_, _, r) in c["draws"]]


def test_specaug_pack_layout_and_rank_slices():
    from nn_conformer_for_speech_recognition_amd import specaugment as psa
    from nn_conformer_for_speech_recognition_amd.lib.hparams import HParams
    hp = HParams(None)
    tau = [40, 38, 20, 5]
    random.seed(1)
    d = psa.draw(4, 40, tau, hp)
    full = psa.pack(d, tau).tolist()
    assert full[:4] == [1, 2, 2, 0]
    halves = [psa.pack(d, tau, 0, 2).tolist(), psa.pack(d, tau, 2, 4).tolist()]
    # freq masks are shared; warp/time entries split by utterance
    assert full[4:4 + 6] == halves[0][4:4 + 6] and full[4 + 6:4 + 12] == halves[1][4:4 + 6]


def test_specaug_reference_raises_where_reference_raises():
    from nn_conformer_for_speech_recognition_amd import specaugment as psa
    from nn_conformer_for_speech_recognition_amd.lib.hparams import HParams
    hp = HParams(None)
    with pytest.raises(ValueError):       # tau = 2W: randint(W, tau-W-1) is an empty range (asrnn.py:108)
        psa.draw(1, 40, [2], hp)


def test_hparams_surface():
    from nn_conformer_for_speech_recognition_amd.lib.hparams import HParams
    hp = HParams(None)
    for k, v in dict(batch_size=32, n_mels=40, conv_sub_1_nodes=512, conv_sub_1_kernel=7, conv_sub_2_nodes=128,
                     mhsa_num_heads=8, conformer_depthwise_conv_kernel=33, standard_linear_nodes=512,
                     conformer_ff1_linear1_nodes=512, warping_param_W=1, frequency_mask_param_F=5,
                     time_mask_param_T=5, time_multiplicity=2, projection_out_size=256, lr=2e-5).items():
        assert getattr(hp, k) == v, k
    hp.set_input_dim(40, 40)
    hp.set_max_len(40)
    hp.set_blank_index(0)
    assert (hp.input_rows, hp.input_cols, hp.max_len, hp.blank_idx) == (40, 40, 40, 0)


def _plan(tiles, nxcd=8, cus=32):
    from nn_conformer_for_speech_recognition_amd import _lib
    lib = _lib.load()
    t = np.array(tiles, dtype=np.int64)
    cap = int(t.sum()) * 16 + 64 * nxcd
    sched = np.empty(cap, dtype=np.uint32)
    split = np.zeros(len(tiles), dtype=np.int32)
    grid = lib.cfm_wgrad_group_plan(t.ctypes.data, len(tiles), nxcd, cus, sched.ctypes.data, cap, split.ctypes.data)
    assert grid > 0
    return sched[:grid], split


def _check_plan(tiles, sched, split, nxcd):
    """every (task, tile) covered exactly once per K slice of its task; padding only at the end of an XCD list"""
    EMPTY = 0xFFFFFFFF
    seen = {}
    for w in sched.tolist():
        if w == EMPTY:
            continue
        task, ks, tile = w >> 20, (w >> 16) & 15, w & 0xFFFF
        assert tile < tiles[task] and ks < split[task]
        seen[(task, tile, ks)] = seen.get((task, tile, ks), 0) + 1
    want = {(i, t, s) for i, n in enumerate(tiles) for t in range(n) for s in range(split[i])}
    assert set(seen) == want and all(v == 1 for v in seen.values())
    lists = sched.reshape(-1, nxcd).T                  # XCD x: workgroups x, x + nxcd, ...
    for l in lists:
        nz = np.nonzero(l != EMPTY)[0]
        assert len(nz) == 0 or nz[-1] == len(nz) - 1      # no padding before real work


def test_wgrad_plan_l15_layout():
    """The L15 backward (17 layers x [FFN2 down/up, pw2, pw1, out, QKV, FFN1 down/up] = 16,16,4,8,4,12,16,16 tiles):
    6 full rounds of 32 tiles per XCD made of whole tasks, and the 28 leftover tiles (seven 4-tile tasks) split
    over 8 K slices, one slice per XCD."""
    layer = [16, 16, 4, 8, 4, 12, 16, 16]
    tiles = layer * 17
    sched, split = _plan(tiles)
    _check_plan(tiles, sched, split, 8)
    assert sorted(set(split.tolist())) == [1, 8] and sum(tiles[i] for i in range(len(tiles)) if split[i] > 1) == 28
    assert len(sched) == 8 * (6 * 32 + 28)
    lists = sched.reshape(-1, 8).T
    for x, l in enumerate(lists):
        rounds = l[: 6 * 32].reshape(6, 32)
        for r in rounds:                                  # each round: whole tasks only
            tasks = r >> 20
            for t in set(tasks.tolist()):
                assert (tasks == t).sum() == tiles[t]
        assert set(((l[6 * 32:] >> 16) & 15).tolist()) == {x}   # the tail: K slice x on XCD x


@pytest.mark.parametrize("tiles,nxcd,cus", [([3, 70, 1, 5], 8, 32), ([40] * 9, 8, 32), ([1], 8, 32),
                                            ([7, 9, 33, 2, 64, 5], 2, 4), ([32] * 16, 8, 32)])
def test_wgrad_plan_covers_every_tile(tiles, nxcd, cus):
    sched, split = _plan(tiles, nxcd, cus)
    _check_plan(tiles, sched, split, nxcd)
