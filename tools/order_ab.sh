#!/bin/bash
# Wave-group refill order: parity tests, then full-frame C3 times per order (GPU box).
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "group_refill_order" -x -v --timeout 200 --timeout-method thread > gpurun_out/order_pytest.log 2>&1 || { tail -30 gpurun_out/order_pytest.log; exit 1; }
tail -2 gpurun_out/order_pytest.log
bash tools/env_ab.sh "NART_RQ_ORDER=0" "NART_RQ_ORDER=1" "NART_RQ_ORDER=2 NART_RQ_TOPF=10" "NART_RQ_ORDER=2 NART_RQ_TOPF=20" "NART_RQ_ORDER=2 NART_RQ_TOPF=35" "NART_RQ_ORDER=0"
