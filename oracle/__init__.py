"""CPU oracle for the depth+uncertainty training step -- TEST INFRASTRUCTURE.

This package is a plain-PyTorch (CPU, op-for-op) *restatement* of the
reference's algorithm for the hot path named in BASELINE.json:north_star:
model forward (random-DAG encoder + multi-scale decoder), the Monodepth loss
stack, and one Adam training step.  Every function cites the reference
``file:line`` it restates.

Rules (see DESIGN.md "Oracle"):
  * Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
    ``cpu_baseline`` leg may import this package -- as the *checker* / the CPU
    baseline, never as the thing measured or shipped.  The product path
    (``uncertainty-model_amd/``) never imports it and fails loudly without its
    HIP library.
  * The oracle is pinned against golden fixtures produced by running the
    reference itself in the build container (``tests/golden/make_goldens.py``);
    ``tests/test_oracle_goldens.py`` checks it.
"""
