"""CPU oracle for the per-frame radar chain -- TEST INFRASTRUCTURE ONLY.

This package is a line-by-line numpy/scipy restatement of the MATLAB reference
(XuZerui2023/Radar-Signal-Simulation-and-Target-Detection):

* ``oracle.precompute`` follows ``main_simulate_echoes_with_array_v8.m:79-155``.
* ``oracle.chain`` follows ``fun_process_single_frame.m:45-407``.
* ``oracle.philox`` is the documented counter-based noise generator that replaces
  MATLAB ``randn`` (``fun_process_single_frame.m:84-85``), which cannot be
  reproduced outside MATLAB.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this package, and only as the checker / the timed CPU baseline.
The product (``radar-signal-simulation-and-target-detection_amd/``) never
imports it.

Parity status: the reference is MATLAB and cannot be run in this container or on
the GPU box (no MATLAB/Octave).  The reference holds no golden vectors or tests.
The restatement is pinned by the known-answer tests derivable from the
reference's own files (integer geometry,
FIR group delay, beam-peak angles of the reference DBF CSV, and the noiseless
range/Doppler peak position), see ``tests/test_oracle_kat.py``.  Beyond those
pins the MATLAB built-in equivalences (fft, filter, circshift, fftshift, kaiser,
interp1 'spline' = not-a-knot) are documented, not measured against MATLAB:
"parity partially pinned (KATs only)".
"""
