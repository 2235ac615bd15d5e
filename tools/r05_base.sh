set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py > gpurun_out/r05a_bench_default.json 2> gpurun_out/r05a_bench_default.err && \
timeout -k 10 300 python -u bench.py --config c4 --no-cpu-baseline > gpurun_out/r05a_bench_c4.json 2> gpurun_out/r05a_bench_c4.err && \
timeout -k 10 180 python -u tools/attn6_bench.py > gpurun_out/r05a_attn6.txt 2>&1
