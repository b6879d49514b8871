"""CPU oracle for the Conformer encoder hot path — TEST INFRASTRUCTURE ONLY.

This package restates, on the CPU, the reference's algorithm for the hot path
(SpecAugment → ConvSubSampling → frame projection → Conformer blocks) so that the
HIP kernels in ``nn_conformer_for_speech_recognition_amd`` can be checked against it.

Rules:
  * Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
    leg may import anything from here, and only as the checker / the timed CPU baseline.
  * The product path never imports this package; it fails loudly when its HIP
    library is missing.

Pinning: ``tests/golden/make_golden.py`` produced the fixtures under ``tests/golden/``
by (a) importing the reference's own Python (``/root/reference/lib``) with stubs for
absent third-party modules, and (b) running ``transformers``' Wav2Vec2Conformer encoder
layer (an independent implementation of the same block, incl. relative positions).
``tests/test_oracle_golden.py`` checks this package against those fixtures.

Modules:
  specaug   — draw-order-exact SpecAugment (python ``random`` + numpy), asrnn.py:91-192
  conformer — torchaudio Conformer semantics + Transformer-XL rel-pos MHSA (torch CPU fp32)
  frontend  — ConvSubSampling (convsubsampling.py:16-45), standard/frame projection,
              ASRNN.encoder composition (asrnn.py:193-221)
"""
