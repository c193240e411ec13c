"""ORACLE — CPU restatement of FedSim's server aggregation arithmetic.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import this package, and only as the
checker (or the timed CPU baseline) — never as the thing measured or shipped.
The product path (``fedsim_amd``) never imports it and has no CPU fallback.

Contents
  fedagg_ref.c / libfedagg_ref.so   C restatement (bit-exact, pinned by goldens)
  ref.py                            ctypes binding of the C oracle + numpy twin
  reference_loop.py                 torch-CPU restatement of the reference's own
                                    per-client loop (the timed cpu_baseline)
  vectors.py                        deterministic platform-independent inputs

Parity is PINNED: tests/golden was produced by importing the reference's own
modules (tools/gen_golden.py) and every oracle function must reproduce it
bit for bit (tests/test_oracle_golden.py).
"""
