#!/bin/bash
# Per-wave timeline of the headline step with 2 / 4 env groups (stamps build), then one default bench line.
set -o pipefail
mkdir -p gpurun_out
export SWARM_STAMPS_LIB=build/stx/libswarm_stamps.so
timeout -k 10 120 python -u tools/stamps_groups.py 2 200 > gpurun_out/sg2.txt 2>&1 &&
timeout -k 10 120 python -u tools/stamps_groups.py 4 200 > gpurun_out/sg4.txt 2>&1 &&
timeout -k 10 120 python -u tools/stamps_groups.py 1 200 > gpurun_out/sg1.txt 2>&1 &&
timeout -k 10 180 python -u bench.py --steps 20 --warmup 5 > gpurun_out/b20.txt 2>&1 &&
timeout -k 10 180 python -u bench.py > gpurun_out/bdef.txt 2>&1
