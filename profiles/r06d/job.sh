#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r06d: the capped unit-sphere loop (crt_renderer_set_sphere_cap).  The loop counts of r06c put the two rejection loops
# at 6.5 VALU per ray (16 % of the kernel's 41.2) at 20 % / 11 % lane fill: a pass runs max over ~47 lanes of a
# geometric(0.52) = 6.2 sphere iterations while a lane needs 1.7.  With a cap of K candidates per pass a lane that has
# not accepted keeps its hit parked and goes on at the next pass.  Compile at occupancy 7: 72 VGPRs, 3 VGPR spills (as
# before), 18 SGPR spills (+1), scratch 32 B/lane (16 before).
# Prediction, config C main kernel: cap 3 -3 .. -5 % (the loop at <= 3 iterations saves ~3.2 x 41 VALU per pass, 2.7
# VALU per ray; ~4.4 deferred lanes per pass cost ~10 % more passes per ray, +0.7 VALU per ray), cap 2 about the same,
# cap 4 -2 .. -3 %; E and the N = 8 share like C; B (latency-bound) 0 .. +5 % (a deferred lane's chain waits a pass).
# Frames, RNG state, ray / path counts and work counters identical at every cap.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r06d; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_sphere_cap.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_cap.log 2>&1
timeout -k 10 600 python3 -u tools/cap_ab.py --configs C,B,E,N8 --caps 0,2,3,4 --reps 3 > $OUT/cap_ab.log 2>&1
echo job done
