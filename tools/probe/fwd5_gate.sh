set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "relgate or wavlm" > /tmp/g1.log 2>&1 || { tail -30 /tmp/g1.log; exit 1; }
tail -1 /tmp/g1.log
timeout -k 10 200 python -u tools/probe/fwd5_gate.py
