"""CPU oracle for the speechbrain_amd hot path — TEST INFRASTRUCTURE ONLY.

This package is a from-scratch, functional CPU restatement (PyTorch CPU ops,
fp32; float64 for the RNN-T lattice) of the reference algorithms that
speechbrain_amd replaces with HIP kernels.  Every function cites the reference
file:line it restates (paths relative to Sinica-SLAM/speechbrain @ 0.5.13).

Who may use it (and nothing else may):
  * tests/                 — as the parity checker for the HIP path;
  * __graft_entry__.smoke  — to check one small HIP invocation;
  * bench.py cpu_baseline  — timed as the host-CPU "port" baseline.
The product package `speechbrain_amd` never imports it; the HIP path fails
loudly when its extension is missing instead of falling back here.

Pinning: each restatement is checked against golden vectors produced by the
real reference (tests/golden/gen_golden.py, fixtures tests/golden/*.npz) and,
for the RNN-T loss, against the reference's own known-answer test
(tests/unittests/test_losses.py:109-152) plus brute-force path enumeration.
"""
