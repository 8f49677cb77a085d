"""TEST INFRASTRUCTURE ONLY — the CPU oracle for the ViT-detector forward path.

Nothing in the product (`vision_transformer_detector_amd`) imports this package.
Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg use
it, and only as the checker / the timed CPU restatement.

* `vtd_numpy`     — float64 NumPy restatement of the Keras graph
                    (`/root/reference/vision_transformer_detector.py:119-206, 239-583, 586-647`).
* `vtd_torch_cpu` — independent float32 torch-CPU restatement of the same graph
                    (second implementation for cross-checking, and the CPU baseline).

PARITY STATUS: **parity unpinned** against executed reference output.  The reference
is TensorFlow 2.9.1 / Keras 2.9 / tensorflow-addons (none importable here, no network),
and its own tests (`testcases_vision_transformer_detector.py`) contain no forward-pass
vectors.  What pins the restatement instead:
  1. the layer-shape fixture transcribed from the notebook's `plot_model` diagram
     (`vision_transformer_detector.ipynb` cell 10) -> `tests/golden/plot_model_shapes.json`;
  2. hand-derived known-answer tests of every upstream op semantic the graph relies on
      -> `tests/test_oracle_kat.py`;
  3. agreement of two independent implementations (fp64 NumPy vs fp32 torch).
"""
