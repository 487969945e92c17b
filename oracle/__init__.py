"""Oracle — TEST INFRASTRUCTURE ONLY.

A CPU restatement (torch-CPU, float64 by default) of the reference's Keras 2.13 semantics for the
head-pose regression hot path.  It is the checker that the HIP path
is compared against; it is never the thing measured or shipped.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it.

Parity status: the reference's arithmetic lives in TensorFlow/Keras 2.13,
which is absent from this image and from ``/root/reference``; the reference ships no tests and no
TF-produced outputs.  The oracle is pinned by the reference's own TF-trained weights (145
checkpoint exemplars covering every graph signature of the 684 ``.h5`` files, converted by
``tests/golden/make_fixtures.py``) and datasets, and cross-checked against the survey's independent
restatement (BASELINE.md §2 MAEs) — forward-vs-TF is therefore "parity partially pinned".
"""
