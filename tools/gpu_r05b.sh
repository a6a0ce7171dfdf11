#!/bin/bash
# round 5: GPU tests of the new ABI paths, then the chain critical-path split of the C3 1/8 shard
step() { tools/gpu_step.sh "$@" || exit 1; }
step r05b_pytest 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "multi or dist or volume_queue"
NART_HIP_LIB=abbuild/wprof/libnart_hip.so step r05b_chain_c3_r2 300 python -u tools/chain_breakdown.py --config c3 --n 8 --rank 2
NART_HIP_LIB=abbuild/wprof/libnart_hip.so step r05b_chain_c3_r0 300 python -u tools/chain_breakdown.py --config c3 --n 8 --rank 0 --alone 1
echo all-done
