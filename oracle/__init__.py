"""CPU oracle for the CMX RGB-X training step — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import this package, and only as the checker / CPU baseline.  The product path
(``rgbx_semantic_segmentation_amd``) never imports it and has no CPU fallback.

Contents
--------
``cmx_ref``        module-form fp32/fp64 restatement of the reference model; the module
                   tree and ``state_dict`` keys are those of the reference
                   (``models/builder.py``, ``models/encoders/dual_segformer.py``,
                   ``models/net_utils.py``, ``models/decoders/MLPDecoder.py``).
``cmx_functional`` an independent functional/einsum restatement (fp64) of the same
                   forward, driven by a ``state_dict`` — used to cross-check
                   ``cmx_ref`` (two restatements must agree to ~1e-6).
``train_ref``      the reference ``train.py`` step semantics on CPU (AdamW param
                   groups of ``utils/init_func.py:group_weight``, ``WarmUpPolyLR``
                   applied after ``optimizer.step()``), used as the CPU baseline.

Parity status: the reference publishes no fixtures and importing/running it was
denied, so this oracle is pinned by hand-derived known-answer tests
(tests/test_oracle_kats.py) and the two-restatement cross-check, not by reference
outputs — "parity unpinned" with respect to reference-generated vectors.
"""
