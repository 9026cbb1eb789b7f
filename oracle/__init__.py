"""CPU oracle for the Kompressor encode/decode hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import anything under ``oracle/``; the product package ``kompressor_amd`` never does.

What this is
------------
``oracle.common`` / ``oracle.volume`` / ``oracle.image`` are an op-for-op numpy
restatement of the reference's hot path (``src/kompressor/utils.py``,
``src/kompressor/volume/*.py``, ``src/kompressor/image/*.py`` of
rosalindfranklininstitute/kompressor @ v1), keeping its materialised intermediates
(padded highres, ``features``, 19-/5-way ``predictions``, float32 scatter-add maps) so that
it is also the "reference CPU path" timed by ``bench.py``.  ``oracle.loops`` is a second,
independent per-element pure-Python restatement used to cross-check the first on small cases.
``oracle.predictors`` restates the reference tests' predictor doubles.

Parity status
-------------
The reference runs on JAX (``jaxlib==0.1.76``, Dockerfile:39), which is not installed in
this image and cannot be fetched (an ordinary ``ModuleNotFoundError``, not a denial).  The
reference ships **no golden vectors**: its tests pin only shapes, dtypes, lossless round
trips, chunk invariance and validator errors.  The oracle is therefore
pinned by
  (i)  every one of those reference assertions, re-expressed in ``tests/test_oracle_reference_spec.py``,
  (ii) closed-form known-answer tests derived from the reference arithmetic
       (``tests/test_oracle_kat.py``), and
  (iii) agreement of two independent restatements (numpy op-for-op vs per-element loops).
**Value-level parity is unpinned** by reference-produced outputs (none exist and the
reference cannot run here).  The golden fixtures under ``tests/golden/`` are produced by this
oracle (``tests/golden/make_golden.py``) and pin the HIP path to it.

XLA semantics restated: float->int casts truncate toward zero (out-of-range
values saturate -- the build's choice, unpinned for jaxlib 0.1.76); ``jnp.pad`` modes equal
numpy's; ``%`` is floor-mod; ``jnp.mean`` is an f32 sum divided by N (exact for uint16 with
N <= 216, i.e. padding <= 2, and for uint8 with padding <= 4); ``jnp.argsort`` is stable;
x64 is disabled so integer coders work in int32.
"""

from . import common, volume, image, predictors, loops  # noqa: F401

VERSION = 'v1.0a'  # src/kompressor/__init__.py:26
