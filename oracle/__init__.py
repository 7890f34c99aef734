"""CPU oracle for the ExPecto Beluga hot path -- TEST INFRASTRUCTURE ONLY.

This package restates, on the CPU, the reference algorithm of every row of
SURVEY.md section 8(a):

* ``beluga_np``   -- the Beluga forward (``Beluga.py:18-51``) in numpy fp32, plus a
                     torch-CPU functional twin used as the timed CPU baseline.
* ``encode_np``   -- ``encodeSeqs`` (``chromatin.py:138-172``) and the
                     ``fetchSeqs`` window geometry (``chromatin.py:175-209``).
* ``reduce_np``   -- the TSS spatial-transform reduction
                     (``compute_expecto_features.py:88-124``) and the variant-side
                     reduction (``predict.py:87-147,183-194``).
* ``gblinear_np`` -- the xgboost gblinear expression scoring of ``predict.py:150-166``.
* ``weights``     -- the seeded synthetic Beluga weights the golden vectors use.

Pinning: the restatement is checked against golden vectors produced by running
the reference itself in the build container (``tests/golden/make_golden.py``;
the reference Beluga, encodeSeqs, chromatin.py, compute/replicate TSS scripts and
predict.py's feature math run there with stubbed I/O dependencies).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this package, and only as the checker.  The product
(``expecto_amd``) never imports it.
"""
